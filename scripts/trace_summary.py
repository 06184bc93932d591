"""Per-kernel, per-grid-size count / average / total duration from a rocprofv3 output directory
(rocpd .db or *kernel_trace.csv).  Launches of one kernel with different grids (e.g. the split
rollout's half-size ensemble launches beside the full ones) are separate rows, so a per-launch figure
is never an average over different launch sizes.

usage: python scripts/trace_summary.py <dir> [name-filter] [--json OUT.json] [--top N]
"""
import argparse
import collections
import csv
import glob
import json
import os
import sqlite3


def from_csv(paths):
    agg = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            grid = int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])
            wg = int(r['Workgroup_Size_X']) * int(r['Workgroup_Size_Y']) * int(r['Workgroup_Size_Z'])
            agg[(r['Kernel_Name'], grid, wg)].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    return agg


def from_db(paths):
    agg = collections.defaultdict(list)
    for db in paths:
        c = sqlite3.connect(db)
        cols = [x[1] for x in c.execute('pragma table_info(kernels)').fetchall()]
        gx = [g for g in ('grid_size_x', 'grid_x', 'grid_size') if g in cols]
        q = 'select name, %s, "end" - start from kernels' % (gx[0] if gx else '0')
        for name, grid, dur in c.execute(q).fetchall():
            agg[(name, int(grid or 0), 0)].append(dur)
    return agg


def summarize(d):
    csvs = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    agg = from_csv(csvs) if csvs else from_db(glob.glob(os.path.join(d, '**', '*.db'), recursive=True))
    rows = []
    for (name, grid, wg), durs in agg.items():
        durs = sorted(durs)
        rows.append({'kernel': name, 'grid_threads': grid, 'workgroup': wg, 'count': len(durs),
                     'avg_us': sum(durs) / len(durs) / 1e3, 'median_us': durs[len(durs) // 2] / 1e3,
                     'min_us': durs[0] / 1e3, 'max_us': durs[-1] / 1e3, 'total_us': sum(durs) / 1e3})
    rows.sort(key=lambda r: -r['total_us'])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('filter', nargs='?', default='')
    ap.add_argument('--json', default=None)
    ap.add_argument('--top', type=int, default=30)
    a = ap.parse_args()
    rows = [r for r in summarize(a.dir) if a.filter in r['kernel']]
    print('%10s %10s %6s %10s %12s  %s' % ('avg_us', 'median_us', 'count', 'grid', 'total_us', 'kernel'))
    for r in rows[:a.top]:
        print('%10.2f %10.2f %6d %10d %12.1f  %s' % (r['avg_us'], r['median_us'], r['count'], r['grid_threads'],
                                                    r['total_us'], r['kernel'][:140]))
    if a.json:
        json.dump(rows, open(a.json, 'w'), indent=1)


if __name__ == '__main__':
    main()
