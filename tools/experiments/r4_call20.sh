#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_wavelength.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_call20_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call20_tests.log; [ $rc -eq 0 ] || exit $rc
NAMES="loki wavelength" timeout -k 10 700 bash tools/evidence.sh > gpurun_out/evidence_b.log 2>&1; rc=$?; tail -4 gpurun_out/evidence_b.log; exit $rc
