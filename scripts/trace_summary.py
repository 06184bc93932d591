"""Per-kernel count / average / total duration from a rocprofv3 output directory (rocpd .db or
kernel_stats.csv):  python scripts/trace_summary.py <dir> [name-filter]"""
import glob
import os
import sqlite3
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
dbs = glob.glob(os.path.join(d, '**', '*.db'), recursive=True)
rows = []
for db in dbs:
    c = sqlite3.connect(db)
    rows += c.execute('select name, count(*), avg("end" - start), sum("end" - start) from kernels group by name').fetchall()
rows.sort(key=lambda r: -r[3])
print('%10s %6s %12s  %s' % ('avg_us', 'count', 'total_us', 'kernel'))
for name, n, avg, tot in rows[:25]:
    if flt in name:
        print('%10.2f %6d %12.1f  %s' % (avg / 1e3, n, tot / 1e3, name[:150]))
