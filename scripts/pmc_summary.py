"""Reduce the rocprofv3 --pmc passes written by scripts/pmc.sh (gpurun_out/pmc1..5) to one JSON.

Per kernel: mean FETCH_SIZE / WRITE_SIZE per dispatch (rocprofv3 reports KiB; converted to bytes),
the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md §HBM (wide 16-B/lane reads are tallied at
half their bytes -> x2), MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/XCDs x CUs
x 4 SIMDs) and the wave-cycle wait share, the L2 hit rate and the instruction mix (pass 5).  Usage: python scripts/pmc_summary.py OUT.json [pmc_dir]
"""
import collections
import csv
import json
import os
import sys

XCDS, CUS = 8, 256


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for i in range(1, 6):
        f = os.path.join(d, 'pmc%d' % i, 'run_counter_collection.csv')
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')
            agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
            agg[n]['_grid'].append(float(r['Grid_Size']))
    return agg


def summarize(agg):
    out = {}
    for n, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items() if c != '_grid'}
        e = {'dispatches': max(len(v) for c, v in d.items() if c != '_grid'),
             'grid_threads': sorted(set(int(g) for g in d['_grid']))}
        if 'FETCH_SIZE' in m:
            e['fetch_bytes_raw'] = m['FETCH_SIZE'] * 1024
            e['fetch_bytes_corrected'] = 2 * m['FETCH_SIZE'] * 1024
        if 'WRITE_SIZE' in m:
            e['write_bytes'] = m['WRITE_SIZE'] * 1024
        if 'fetch_bytes_corrected' in e and 'write_bytes' in e:
            e['hbm_bytes'] = e['fetch_bytes_corrected'] + e['write_bytes']
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in m and m.get('GRBM_GUI_ACTIVE'):
            e['mfma_busy_frac'] = m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / XCDS * CUS * 4)
            e['gui_active_cycles_per_xcd'] = m['GRBM_GUI_ACTIVE'] / XCDS
        if 'SQ_WAVES' in m:
            e['waves'] = m['SQ_WAVES']
        if m.get('SQ_WAVE_CYCLES'):
            e['wait_inst_any_frac'] = m.get('SQ_WAIT_INST_ANY', 0) / m['SQ_WAVE_CYCLES']
        if m.get('TCC_HIT_sum', 0) + m.get('TCC_MISS_sum', 0) > 0:
            e['l2_hit_frac'] = m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum'])
        for c in ('SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT'):
            if c in m:
                e[c.lower()] = m[c]
        out[n] = e
    return out


if __name__ == '__main__':
    # usage: pmc_summary.py OUT.json PMC_DIR WORKLOAD -- merges this workload's kernels into OUT.json
    # ({"workloads": {workload_key: {...}}}); bench.py reports a kernel's traffic only for the workload
    # its passes ran (bench.py workload_key)
    dst = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else 'gpurun_out'
    workload = sys.argv[3] if len(sys.argv) > 3 else 'unknown'
    s = summarize(load(src))
    s = {k: v for k, v in s.items() if 'mopo::' in k}
    d = json.load(open(dst)) if os.path.exists(dst) else {}
    d.setdefault('source', 'rocprofv3 --pmc passes of scripts/pmc.sh (bench.py --steps 3 --warmup 1 --sac-steps 50 '
                           '--config/--ensemble-dtype of the workload), one counter group per pass')
    d.setdefault('workloads', {})[workload] = {'kernels': s}
    json.dump(d, open(dst, 'w'), indent=1)
    for k, v in s.items():
        print(workload, k, {a: round(b, 4) if isinstance(b, float) else b for a, b in v.items()})
