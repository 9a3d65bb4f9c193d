#!/bin/bash
# One rocprofv3 PMC pass per counter set over a short bench command.
# Usage: bash tools/r6/pmc.sh <tag> "<bench args>" "<counters>" ["<counters>" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=$1; args=$2; shift 2
i=0
for pmc in "$@"; do
  out=gpurun_out/$tag/pmc$i
  mkdir -p $out
  timeout -s KILL 150 rocprofv3 --pmc $pmc -d $out -o run --output-format csv -- python3 bench.py $args > $out.log 2>&1
  rc=$?
  echo "pmc $pmc rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out.log; exit $rc; fi
  i=$((i+1))
done
