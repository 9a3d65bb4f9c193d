#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "pixel_variants" > gpurun_out/r4_call7_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call7_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=4 BENCH_ARGS="--workload loki" timeout -k 10 600 bash tools/knob_ab.sh tools/experiments/knobs_r4_pf2.txt
