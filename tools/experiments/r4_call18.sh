#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wavelength.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r4_call18_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_call18_tests.log; [ $rc -eq 0 ] || exit $rc
NAMES="dream loki wavelength" timeout -k 10 1000 bash tools/evidence.sh > gpurun_out/evidence_a.log 2>&1; rc=$?; tail -8 gpurun_out/evidence_a.log; exit $rc
