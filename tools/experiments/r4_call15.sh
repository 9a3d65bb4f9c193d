#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_finalize_split.py tests/test_gpu_headline.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_call15_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_call15_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 timeout -k 10 300 bash tools/knob_ab.sh tools/experiments/knobs_r4_finsplit.txt > gpurun_out/r4_call15_fin.txt 2>&1; rc=$?; tail -3 gpurun_out/r4_call15_fin.txt; [ $rc -eq 0 ] || exit $rc
REPS=2 BENCH_ARGS="--coordinate wavelength" timeout -k 10 500 bash tools/knob_ab.sh tools/experiments/knobs_r4_keyabl.txt > gpurun_out/r4_call15_key.txt 2>&1; rc=$?; tail -7 gpurun_out/r4_call15_key.txt; exit $rc
