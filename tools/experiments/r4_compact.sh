#!/bin/bash
# r4: lane-compact sieve variant: parity (split, variants 20/21) then interleaved A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "skewed and split and (20 or 21 or 0-)" > gpurun_out/r4_compact_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_compact_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=${REPS:-4} timeout -k 10 900 bash tools/knob_ab.sh tools/experiments/knobs_r4_compact.txt
