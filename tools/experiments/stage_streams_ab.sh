#!/bin/bash
# A/B of one vs two H2D copy streams for host staging (end_to_end leg).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
for p in 1 2; do
  LDE_STAGE_STREAMS=$p timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 5 > gpurun_out/sstream_$p.log 2>&1 || { echo "bench streams=$p failed"; tail -5 gpurun_out/sstream_$p.log; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/sstream_$p.log') if l.startswith('{')][0]);print('streams $p', round(d['end_to_end']['ms_per_step'],3), '%.4g'%d['end_to_end']['value'])"
done
done
