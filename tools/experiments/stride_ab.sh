#!/bin/bash
# Interleaved runs of bench.py with the dominant kernel stamped on every step
# (--timing-stride 1) vs every 5th step vs never (LDE_BENCH_UNTIMED=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq ${REPS:-3}); do
  for cfg in "1 0" "5 0" "5 1"; do
    set -- $cfg
    LDE_BENCH_UNTIMED=$2 timeout -k 10 150 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --e2e-steps 0 --timing-stride $1 > gpurun_out/sab_one.log 2>&1 || { tail -5 gpurun_out/sab_one.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/sab_one.log') if l.startswith('{')][0]);r=d['roofline'];print('stride $1 untimed $2 step %.4f dom %.4f launches %d' % (d['ms_per_step'], r['avg_launch_ms'], r['launches']))"
  done
done
