#!/bin/bash
# round 5: finalize images into non-coherent (coarse-grained) host blocks
# (diagnostics knob LDE_HOST_NC=1): image parity first, then the kernel A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LDE_HOST_NC=1 LDE_LIBRARY=$PWD/esslivedata_amd/libesslivedata_amd_diag.so \
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_workflows.py tests/test_gpu_kats.py -m gpu > gpurun_out/r5nc_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5nc_tests.log | tail -6
[ $rc -ne 0 ] && exit $rc
TAG=r5nc CFGS="X=0 LDE_HOST_NC=1 X=0 LDE_HOST_NC=1" bash tools/experiments/r5_kernel_ab.sh
