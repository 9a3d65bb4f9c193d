#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread -k "dream or split or headline" > gpurun_out/r4_call23_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call23_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 timeout -k 10 400 bash tools/ab.sh > gpurun_out/r4_call23_ab.txt 2>&1; rc=$?; cat gpurun_out/r4_call23_ab.txt; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 300 bash tools/knob_ab.sh tools/experiments/knobs_r4_sortkpt.txt > gpurun_out/r4_call23_kpt.txt 2>&1; rc=$?; tail -2 gpurun_out/r4_call23_kpt.txt; exit $rc
