#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wavelength.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r4_call26_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call26_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 BENCH_ARGS="--coordinate wavelength" timeout -k 10 400 bash tools/ab.sh > gpurun_out/r4_call26_ab.txt 2>&1; rc=$?; cat gpurun_out/r4_call26_ab.txt; exit $rc
