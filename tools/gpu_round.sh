#!/bin/bash
# One GPU call: parity tests, then (unless the GPU faulted) a short bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "GPU step failed hard (rc=$rc); stopping"; exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -20 gpurun_out/bench.log
exit $brc
