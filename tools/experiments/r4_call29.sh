#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
NAMES="wire_view mantle_front_layer" timeout -k 10 1100 bash tools/evidence.sh > gpurun_out/evidence_g.log 2>&1; rc=$?; tail -4 gpurun_out/evidence_g.log; exit $rc
