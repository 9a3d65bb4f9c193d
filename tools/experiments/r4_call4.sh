#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_wavelength.py -x -q --timeout 250 --timeout-method thread -k "pixel or loki or headline or bench_workload" > gpurun_out/r4_call4_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_call4_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 BENCH_ARGS="--workload loki" timeout -k 10 400 bash tools/knob_ab.sh tools/experiments/knobs_r4_ranges.txt || exit 1
cp gpurun_out/knob_ab.log gpurun_out/knob_ab_ranges.log
REPS=2 timeout -k 10 600 bash tools/knob_ab.sh tools/experiments/knobs_r4_ablate.txt
