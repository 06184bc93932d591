"""Timeline of the split rollout from a rocprofv3 kernel trace (scripts/gpu_r04_trace.sh): for the last
N rollouts (rollout_start_kernel marks each), per-kernel busy time, the union of busy intervals (GPU busy),
and the wall span per rollout.  usage: python scripts/rollout_timeline.py run_kernel_trace.csv [N]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    ks = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows))
    starts = [i for i, k in enumerate(ks) if 'rollout_start_kernel' in k[2]]
    sel = starts[-(n + 1):]          # the last n complete rollouts (each from its start kernel to the next)
    short = lambda s: s.split('(')[0].replace('void ', '').replace('mopo::', '')[:40]
    for a, b in zip(sel[:-1], sel[1:]):
        seg = ks[a:b]
        t0 = seg[0][0]
        t1 = max(e for _, e, nm in seg if 'sac' not in nm and 'gemm' not in nm)
        busy = defaultdict(float)
        iv = []
        for s, e, nm in seg:
            if e > t1:
                continue
            busy[short(nm)] += (e - s) / 1e3
            iv.append((s, e))
        iv.sort()
        union, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    union += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        union += ce - cs
        print('rollout span %.1f us, GPU busy (union) %.1f us, sum of kernels %.1f us' % ((t1 - t0) / 1e3, union / 1e3,
                                                                                     sum(busy.values())))
        print('   ' + ', '.join('%s %.1f' % kv for kv in sorted(busy.items(), key=lambda x: -x[1])))


if __name__ == '__main__':
    main()
