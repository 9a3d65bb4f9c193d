#!/bin/bash
# round 5: block timelines -- tools/ubench_sgather.hip's plain stream and
# the sieve (default and stream skeleton, LDE_SIEVE_TRACE, diagnostics build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 tools/ubench_sgather.hip -o /tmp/ubsg 2>/dev/null || exit 1
timeout -k 10 60 /tmp/ubsg 116 | head -6 || exit 1
export LDE_LIBRARY=$PWD/esslivedata_amd/libesslivedata_amd_diag.so
for abl in 0 4096; do
  LDE_SIEVE_TRACE=1 LDE_SIEVE_ABLATE=$abl timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline \
    --e2e-steps 0 --bank-steps 0 > gpurun_out/r5trace_$abl.log 2>&1 || { tail -5 gpurun_out/r5trace_$abl.log; exit 1; }
  echo "== ablate $abl"; grep "sieve trace" gpurun_out/r5trace_$abl.log
done
