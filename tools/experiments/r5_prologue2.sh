#!/bin/bash
# round 5: prologues II -- the cold sort's first key round requested before
# its scans, pass-B items read with their count (cold accumulate, PIXEL pass
# B), plus lds_fill: parity, block timeline, interleaved A/B against HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_wavelength.py -m gpu > gpurun_out/r5p2_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5p2_tests.log | tail -6
[ $rc -ne 0 ] && exit $rc
LDE_LIBRARY=$PWD/esslivedata_amd/libesslivedata_amd_diag.so LDE_SIEVE_TRACE=1 timeout -k 10 200 python bench.py --steps 10 \
  --warmup 2 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 > gpurun_out/r5p2_trace.log 2>&1 || exit 1
grep "sieve trace" gpurun_out/r5p2_trace.log
echo "== dream"; REPS=3 BENCH_ARGS="--bank-steps 0" bash tools/ab.sh || exit 1
echo "== loki"; REPS=3 BENCH_ARGS="--workload loki --bank-steps 0" bash tools/ab.sh
