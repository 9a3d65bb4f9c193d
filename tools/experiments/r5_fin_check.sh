#!/bin/bash
# round 5: sparse finalize -- the whole GPU suite, then an interleaved A/B of
# the DREAM bench against the previous build (tools/ab/libbase.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest --maxfail=10 -v --timeout 300 --timeout-method thread \
  tests -m gpu > gpurun_out/r5f_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5f_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
REPS=3 BENCH_ARGS="--bank-steps 0" bash tools/ab.sh
