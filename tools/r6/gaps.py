"""Kernel timeline of a rocprofv3 --kernel-trace CSV: per kernel name the
count / mean duration, and the sequence of the last `n` dispatches with the
idle gap before each (us).  Usage: python gaps.py <kernel_trace.csv> [n]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r['Start_Timestamp']))
agg = defaultdict(list)
for r in rows:
    agg[r['Kernel_Name'].split('(')[0][:60]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f'{k:60s} n={len(v):5d} mean={sum(v)/len(v):9.2f} us  total={sum(v)/1e3:8.3f} ms')
print('--- last', n)
prev = None
for r in rows[-n:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f'{gap:8.2f} gap  {(e - s) / 1e3:9.2f} us  {r["Kernel_Name"].split("(")[0][:70]}  grid={r.get("Grid_Size", "")}')
    prev = e
