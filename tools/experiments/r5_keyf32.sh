#!/bin/bash
# round 5: the keyed pass's float32 first pass -- wavelength parity (incl.
# the near-edge test and the f64-only variant), then rocprofv3 kernel
# averages against the previous build (tools/ab/libbase.so), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_wavelength.py -m gpu > gpurun_out/r5kf_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5kf_tests.log | tail -6
[ $rc -ne 0 ] && exit $rc
REPS=2 BENCH_ARGS="--coordinate wavelength" KGREP="event_key\|k_sieve" bash tools/experiments/r5_kprof_ab.sh
