#!/bin/bash
# round 5: the sieve's stream skeleton (LDE_SIEVE_ABLATE=4096, diagnostics
# build) against tools/ubench_sgather.hip's plain stream on the same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 tools/ubench_sgather.hip -o /tmp/ubsg 2>/dev/null || exit 1
timeout -k 10 60 /tmp/ubsg 116 | head -6 || exit 1
TAG=r5skel CFGS="X=0 LDE_SIEVE_ABLATE=4096 LDE_SIEVE_ABLATE=16384 LDE_SIEVE_ABLATE=49152" bash tools/experiments/r5_kernel_ab.sh
