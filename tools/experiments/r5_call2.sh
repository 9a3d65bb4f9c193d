#!/bin/bash
# round 5: the whole GPU suite after pruning the +-0 variants, then the
# default bench and the LOKI / BIFROST lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests -m gpu --durations=25 > gpurun_out/r5c2_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -45 gpurun_out/r5c2_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r5c2_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --workload loki > gpurun_out/r5c2_loki.log 2>&1 && \
timeout -k 10 300 python bench.py --workload bifrost > gpurun_out/r5c2_bifrost.log 2>&1
brc=$?
echo "bench rc=$brc"; tail -c 2500 gpurun_out/r5c2_bench.log; tail -c 1500 gpurun_out/r5c2_loki.log; tail -c 1200 gpurun_out/r5c2_bifrost.log
exit $brc
