#!/bin/bash
# One rocprofv3 kernel-trace pass over a short bench run; prints per-kernel
# average durations (diagnostic, not the product).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/qp
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS} > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
grep '^{' $OUT/log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g step %.4f dom %.4f' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']), d['roofline']['kernel_ms'])"
python3 - <<'PY'
import csv, glob, re
f = glob.glob('gpurun_out/qp/**/run_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:16]:
    m = re.search(r'lde::(k_\w+)', r['Name'])
    print('%-28s calls %5s avg %9.2f us' % ((m.group(1) if m else r['Name'][:28]), r['Calls'], float(r['AverageNs']) / 1e3))
PY
