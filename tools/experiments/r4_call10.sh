#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LDE_VERBOSE=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > gpurun_out/r4_win_verbose.log 2>&1; rc=$?; grep "lde split" gpurun_out/r4_win_verbose.log | head -5; [ $rc -eq 0 ] || { tail -5 gpurun_out/r4_win_verbose.log; exit $rc; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_logical_views.py tests/test_gpu_wavelength.py -x -q --timeout 250 --timeout-method thread -k "split or skewed or headline or bench_workload or view or pixel or loki" > gpurun_out/r4_call10_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call10_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=3 timeout -k 10 300 bash tools/knob_ab.sh tools/experiments/knobs_r4_window.txt || exit 1
cp gpurun_out/knob_ab.log gpurun_out/knob_ab_window.log
REPS=3 BENCH_ARGS="--workload loki" timeout -k 10 300 bash tools/ab.sh
