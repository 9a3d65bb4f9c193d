#!/bin/bash
# round 5: tile-major cold counts, XCD-aware sort rows -- SPLIT parity first, then
# the DREAM bench and its kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail=5 -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_wavelength.py -m gpu > gpurun_out/r5c9_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5c9_tests.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --bank-steps 0 > gpurun_out/r5c9_bench.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_r5c9 -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 > gpurun_out/r5c9_prof.log 2>&1
brc=$?
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"bit_exact_vs_oracle": [a-z]*\|"frac": [0-9.]*' gpurun_out/r5c9_bench.log | head -5 | tr '\n' ' '; echo
python tools/kstats_db.py $(find /tmp/prof_r5c9 -name "*results.db" | head -1) 40 | grep "_ZN3lde"
[ $brc -ne 0 ] && exit $brc
LDE_LIBRARY=$PWD/esslivedata_amd/libesslivedata_amd_diag.so LDE_SIEVE_TRACE=2 timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 > gpurun_out/r5c9_trace.log 2>&1; echo trace rc=$?
