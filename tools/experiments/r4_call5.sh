#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "pixel_variants or predicted_slots" > gpurun_out/r4_call5_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call5_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=4 timeout -k 10 700 bash tools/knob_ab.sh tools/experiments/knobs_r4_nt.txt
