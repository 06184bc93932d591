"""Mean of every counter per kernel over the pmc* passes of a rocprofv3 --pmc directory:
python scripts/pmc_counters.py <dir> [kernel-name filter]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, 'pmc*', '*counter_collection.csv'))):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')
        if flt in n:
            agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n, cs in agg.items():
    print(n)
    for c, v in sorted(cs.items()):
        print('   %-28s %14.1f  (n=%d)' % (c, sum(v) / len(v), len(v)))
