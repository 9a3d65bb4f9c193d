#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_concurrent.py -x -v -s --timeout 180 --timeout-method thread > gpurun_out/r4_call30_conc.log 2>&1; rc=$?; grep -h "five jobs\|passed\|failed" gpurun_out/r4_call30_conc.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r4_smoke.log; exit $rc
