#!/bin/bash
# One GPU call for the round's closing evidence: tools/evidence.sh (profiles +
# bench lines), then the whole -m gpu suite and smoke().
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 500 bash tools/evidence.sh > gpurun_out/evidence.log 2>&1 || { tail -5 gpurun_out/evidence.log; exit 1; }
echo evidence ok
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; exit $rc
