#!/bin/bash
# round 5: sieve dynamic tail -- parity (tail tests + SPLIT suite), then
# DREAM bench, kernel A/B of LDE_SIEVE_TAIL_PCT (diagnostics build) and the
# per-block trace of both settings
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5t}
timeout -k 10 600 python -u -m pytest --maxfail=5 -v --timeout 200 --timeout-method thread \
  -k "tail or split or sieve or keyed or headline or dream" \
  tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_wavelength.py -m gpu > gpurun_out/${T}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${T}_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --bank-steps 0 > gpurun_out/${T}_bench.log 2>&1 || exit 1
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"bit_exact_vs_oracle": [a-z]*\|"frac": [0-9.]*' gpurun_out/${T}_bench.log | head -5 | tr '\n' ' '; echo
TAG=${T}k CFGS="LDE_SIEVE_TAIL_PCT=0 LDE_SIEVE_TAIL_PCT=8 LDE_SIEVE_TAIL_PCT=0 LDE_SIEVE_TAIL_PCT=8 LDE_SIEVE_TAIL_PCT=5" bash tools/experiments/r5_kernel_ab.sh || exit 1
for pct in 0 8; do
  LDE_LIBRARY=$PWD/esslivedata_amd/libesslivedata_amd_diag.so LDE_SIEVE_TAIL_PCT=$pct LDE_SIEVE_TRACE=2 timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 > gpurun_out/${T}_trace$pct.log 2>&1 || exit 1
done
echo done
