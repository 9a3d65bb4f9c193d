"""Mean per-dispatch PMC values per kernel from rocprofv3 counter_collection
CSVs under a directory.  Usage: python pmc_sum.py <dir> [kernel substring]"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][:50]
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
sub = sys.argv[2] if len(sys.argv) > 2 else ''
for k, d in acc.items():
    if sub not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f'   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})')
