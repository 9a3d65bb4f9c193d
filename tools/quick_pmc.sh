#!/bin/bash
# One rocprofv3 PMC pass (SQ counters) over a short bench run; prints the
# per-dispatch averages per engine kernel (diagnostic, not the product).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/qpmc
rm -rf $OUT; mkdir -p $OUT
CNT=${CNT:-"SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU"}
timeout -s KILL 120 rocprofv3 --pmc $CNT -d $OUT -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS} > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
python3 - <<'PY'
import csv, glob, re, collections
f = glob.glob('gpurun_out/qpmc/**/run_counter_collection.csv', recursive=True)[0]
per = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    m = re.search(r'lde::(k_\w+)', r['Kernel_Name'])
    if m:
        per[(m.group(1), r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for (k, d, c), v in per.items():
    agg[k][c].append(v)
for k, cs in sorted(agg.items()):
    print(k, {c: '%.4g' % (sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
