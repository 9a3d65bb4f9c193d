#!/bin/bash
# round 5: kernel prologues with every table load issued before its LDS
# stores (lds_fill) -- parity of the touched kernels, then interleaved A/B
# against the previous build (tools/ab/libbase.so) on DREAM, LOKI, wavelength
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_wavelength.py tests/test_gpu_headline.py -m gpu > gpurun_out/r5p_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5p_tests.log | tail -6
[ $rc -ne 0 ] && exit $rc
echo "== dream"; REPS=3 BENCH_ARGS="--bank-steps 0" bash tools/ab.sh || exit 1
echo "== loki"; REPS=2 BENCH_ARGS="--workload loki --bank-steps 0" bash tools/ab.sh || exit 1
echo "== wavelength"; REPS=2 BENCH_ARGS="--coordinate wavelength --bank-steps 0" bash tools/ab.sh
