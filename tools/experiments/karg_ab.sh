#!/bin/bash
# A/B of the kernel-argument descriptor table (LDE_KARG_SEGS) on the default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2 3; do
for p in 0 1; do
  LDE_KARG_SEGS=$p timeout -k 10 200 python bench.py --no-cpu-baseline --e2e-steps 0 --steps 40 > gpurun_out/karg_$p.log 2>&1 || { echo "bench karg=$p failed"; tail -5 gpurun_out/karg_$p.log; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/karg_$p.log') if l.startswith('{')][0]);print('karg $p', round(d['ms_per_step'],4), '%.4g'%d['value'], round(d['roofline']['kernel_ms']['binning'],4))"
done
done
