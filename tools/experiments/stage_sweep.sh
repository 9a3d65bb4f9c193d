#!/bin/bash
# Host-staging thread sweep: end_to_end leg of bench.py per LDE_STAGE_THREADS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for t in ${THREADS:-1 4 8 16}; do
  LDE_STAGE_THREADS=$t timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 4 > gpurun_out/stage_t$t.log 2>&1 || { echo "bench t=$t failed"; tail -5 gpurun_out/stage_t$t.log; exit 1; }
  python -c "import json,sys;d=json.loads([l for l in open('gpurun_out/stage_t$t.log') if l.startswith('{')][0]);print('threads $t', d['end_to_end']['ms_per_step'], d['end_to_end']['value'])"
done
