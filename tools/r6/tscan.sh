#!/bin/bash
# Round 6: the engine at the reference's reachable TOA configurations
# (EdgesModel num_bins 1..10000, linear/log, parameter_models.py:82-105).
# Usage (GPU box): bash tools/r6/tscan.sh <tag> [extra bench args]
set -o pipefail
tag=${1:-tscan}; shift
out=gpurun_out/$tag; mkdir -p $out
run() {  # name, bench args...
  local name=$1; shift
  echo "== $name: $*"
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --e2e-steps 0 --bank-steps 0 \
      --cpu-baseline-seconds 1 "$@" > $out/$name.json 2> $out/$name.err
  local rc=$?
  tail -c 600 $out/$name.json; echo " rc=$rc"
  return $rc
}
for spec in ${SPECS:-"dream:164:log" "dream:1000:log" "dream:10000:log" "loki:164:linear" "loki:1000:linear" "loki:10000:linear"}; do
  IFS=: read w nb sc st <<< "$spec"
  run ${w}_${nb}_${sc}${st:+_$st} --workload $w --num-bins $nb --toa-scale $sc ${st:+--toa-start $st} "$@" || exit $?
done
