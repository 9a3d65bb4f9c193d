#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavelength.py tests/test_gpu_finalize_split.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r4_call19_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call19_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 BENCH_ARGS="--coordinate wavelength" timeout -k 10 400 bash tools/ab.sh > gpurun_out/r4_call19_ab.txt 2>&1; rc=$?; cat gpurun_out/r4_call19_ab.txt; [ $rc -eq 0 ] || exit $rc
REPS=2 BENCH_ARGS="--coordinate wavelength" timeout -k 10 300 bash tools/knob_ab.sh tools/experiments/knobs_r4_w24.txt > gpurun_out/r4_call19_fb.txt 2>&1; rc=$?; tail -2 gpurun_out/r4_call19_fb.txt; exit $rc
