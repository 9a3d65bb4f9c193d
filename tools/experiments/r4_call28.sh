#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
NAMES="dream strip_view" timeout -k 10 1100 bash tools/evidence.sh > gpurun_out/evidence_f.log 2>&1; rc=$?; tail -4 gpurun_out/evidence_f.log; exit $rc
