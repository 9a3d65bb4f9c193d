#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
NAMES="loki monitor bifrost" timeout -k 10 1100 bash tools/evidence.sh > gpurun_out/evidence_d.log 2>&1; rc=$?; tail -4 gpurun_out/evidence_d.log; exit $rc
