"""SAC kernel durations from a rocprofv3 kernel trace: mean duration per kernel name (and calls per
step), the step period as the mean interval between consecutive starts of the step's anchor launch
(the critic dh1 launch: the grouped-GEMM launch with the largest grid), and per-position durations.
Usage: python scripts/sac_trace.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
sac = [r for r in rows if any(k in r['Kernel_Name'] for k in ('gemm_group', 'mlp12', 'sac_', 'pi_head'))]
grid = lambda r: int(r.get('Grid_Size_X') or r.get('Grid_Size') or 0)
# anchor: the largest-grid grouped-GEMM launch (critic dh1 + loss tail: 1025 blocks at batch 256)
gmax = max(grid(r) for r in sac if 'gemm_group' in r['Kernel_Name'])
anchor = [int(r['Start_Timestamp']) for r in sac if 'gemm_group' in r['Kernel_Name'] and grid(r) == gmax]
skip = len(anchor) // 4
t0, t1 = anchor[skip], anchor[-1]
steps = len(anchor) - 1 - skip
dur = collections.defaultdict(list)
busy = 0
for r in sac:
    st = int(r['Start_Timestamp'])
    if t0 <= st < t1:
        d = (int(r['End_Timestamp']) - st) / 1e3
        dur[r['Kernel_Name'].split('(')[0]].append(d)
        busy += d
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print('%-34s %5.1f calls/step  %6.2f us avg  %6.1f us/step' % (n, len(v) / steps, sum(v) / len(v), sum(v) / steps))
print('step period %.1f us (anchor-to-anchor, %d steps); kernel-busy %.1f us/step'
      % ((t1 - t0) / 1e3 / steps, steps, busy / steps))

# per position within the period (dispatch order after an anchor launch)
pos = collections.defaultdict(list)
cur = -1
for r in sac:
    st = int(r['Start_Timestamp'])
    if 'gemm_group' in r['Kernel_Name'] and grid(r) == gmax:
        cur = 0
    if cur < 0 or not (t0 <= st < t1):
        continue
    pos[(cur, r['Kernel_Name'].split('(')[0], r.get('Grid_Size_X', ''))].append((int(r['End_Timestamp']) - st) / 1e3)
    cur += 1
for (i, n, gx), v in sorted(pos.items()):
    print('  %2d %-30s grid %7s  %6.2f us' % (i, n, gx, sum(v) / len(v)))
