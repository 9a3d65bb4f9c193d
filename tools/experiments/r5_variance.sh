#!/bin/bash
# round 5: run-to-run spread of the DREAM bench on one box (N runs)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq ${N:-6}); do
  timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 ${BENCH_ARGS} > gpurun_out/var_$r.log 2>&1 || { tail -5 gpurun_out/var_$r.log; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/var_$r.log') if l.startswith('{')][0]);r=d['roofline'];print('run $r', 'step %.4f' % d['ms_per_step'], ' '.join('%s=%.4f' % kv for kv in r['kernel_ms'].items()))"
done
