#!/bin/bash
# round 5, first GPU call: the new tests (time-coord KATs, f32 fused finalize,
# many-message ATOMIC, bench cadences / bank leg), then the default bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_kats.py tests/test_outputs.py \
  "tests/test_gpu_parity.py::test_bifrost_float32_fused_finalize_cadences" \
  "tests/test_gpu_parity.py::test_atomic_many_large_messages_proportional_blocks" \
  "tests/test_gpu_parity.py::test_atomic_many_messages" \
  "tests/test_gpu_parity.py::test_bifrost_float32_accumulation" \
  "tests/test_gpu_parity.py::test_bifrost_float32_partials_match_finalize" \
  tests/test_bench_contract.py -m gpu > gpurun_out/r5c1_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/r5c1_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r5c1_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --workload bifrost > gpurun_out/r5c1_bifrost.log 2>&1
brc=$?
echo "bench rc=$brc"; tail -c 3000 gpurun_out/r5c1_bench.log; tail -c 1500 gpurun_out/r5c1_bifrost.log
exit $brc
