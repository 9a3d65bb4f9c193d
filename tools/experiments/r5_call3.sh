#!/bin/bash
# round 5: GPU suite (pruned variants, direct cold sort, per-wave PIXEL
# counters as a diagnostics knob), DREAM bench + kernel trace, LOKI A/B of
# LDE_PIX_PW (diagnostics build, interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest --maxfail=10 -v --timeout 300 --timeout-method thread \
  tests -m gpu --durations=25 > gpurun_out/r5c3_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/r5c3_tests.log
[ $rc -ne 0 ] && exit $rc
DIAG=$PWD/esslivedata_amd/libesslivedata_amd_diag.so
timeout -k 10 400 python bench.py > gpurun_out/r5c3_bench.log 2>&1 && \
LDE_VERBOSE=1 timeout -k 10 300 python bench.py --workload loki --steps 20 > gpurun_out/r5c3_loki.log 2>&1 && \
LDE_LIBRARY=$DIAG LDE_PIX_PW=1 timeout -k 10 300 python bench.py --workload loki --steps 20 > gpurun_out/r5c3_loki_pw1a.log 2>&1 && \
LDE_LIBRARY=$DIAG LDE_PIX_PW=0 timeout -k 10 300 python bench.py --workload loki --steps 20 > gpurun_out/r5c3_loki_pw0a.log 2>&1 && \
LDE_LIBRARY=$DIAG LDE_PIX_PW=1 timeout -k 10 300 python bench.py --workload loki --steps 20 > gpurun_out/r5c3_loki_pw1b.log 2>&1 && \
LDE_LIBRARY=$DIAG LDE_PIX_PW=0 timeout -k 10 300 python bench.py --workload loki --steps 20 > gpurun_out/r5c3_loki_pw0b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5c3 -o dream -- python bench.py --steps 20 > gpurun_out/r5c3_prof.log 2>&1
brc=$?
echo "bench rc=$brc"
for f in gpurun_out/r5c3_bench.log gpurun_out/r5c3_loki*.log; do echo "== $f"; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"bit_exact_vs_oracle": [a-z]*\|"frac": [0-9.]*' $f | head -4 | tr '\n' ' '; echo; done
grep "lde pixel" gpurun_out/r5c3_loki.log | head -2
find gpurun_out/prof_r5c3 -name "*kernel_stats.csv" -exec head -14 {} \;
exit $brc
