#!/bin/bash
# A/B of k_cold_sort blocks per cold region (LDE_SORT_HALVES) on the default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2 3; do
for p in 1 2; do
  LDE_SORT_HALVES=$p timeout -k 10 200 python bench.py --no-cpu-baseline --e2e-steps 0 --steps 40 > gpurun_out/halves_$p.log 2>&1 || { echo "bench karg=$p failed"; tail -5 gpurun_out/halves_$p.log; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/halves_$p.log') if l.startswith('{')][0]);print('halves $p', round(d['ms_per_step'],4), '%.4g'%d['value'], round(d['roofline']['kernel_ms']['binning'],4))"
done
done
