#!/bin/bash
# A/B of two engine builds on one box: tools/ab/libbase.so (baseline) vs the
# in-tree library, alternating, ${REPS:-3} bench runs each (diagnostic).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq ${REPS:-3}); do
  for v in base new; do
    if [ $v = base ]; then export LDE_LIBRARY=tools/ab/libbase.so; else unset LDE_LIBRARY; fi
    timeout -k 10 150 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS} > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][0]);r=d['roofline'];print('$v', 'step %.4f' % d['ms_per_step'], 'value %.4g' % d['value'], ' '.join('%s=%.4f' % kv for kv in r['kernel_ms'].items()))"
  done
done
