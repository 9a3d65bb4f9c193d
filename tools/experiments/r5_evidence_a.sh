#!/bin/bash
# round 5 evidence, call A: the whole GPU suite, then the DREAM profile
# (kernel trace + PMC passes) and its untraced bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest --maxfail=10 -v --timeout 300 --timeout-method thread \
  tests -m gpu --durations=15 > gpurun_out/r5_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_gpu_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
TAG=r5 NAMES="dream" bash tools/evidence.sh
