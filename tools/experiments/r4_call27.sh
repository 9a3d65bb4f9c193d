#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_logical_views.py -x -q --timeout 300 --timeout-method thread -k "dream or split or view" > gpurun_out/r4_call27_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call27_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=4 timeout -k 10 500 bash tools/ab.sh > gpurun_out/r4_call27_ab.txt 2>&1; rc=$?; cat gpurun_out/r4_call27_ab.txt; exit $rc
