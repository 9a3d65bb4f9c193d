#!/bin/bash
# A/B of diagnostics knobs on one box: bench lines per setting (exact results).
# Usage: bash tools/r6/knobab.sh <tag> "<VAR=v,VAR2=w> <...>" [bench args]
set -o pipefail
tag=$1; sets=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
i=0
for kv in $sets; do
  env_args=$(echo $kv | tr ',' ' ')
  [ "$kv" = "-" ] && env_args=""
  env LDE_LIBRARY=esslivedata_amd/libesslivedata_amd_diag.so $env_args timeout -k 10 200 python -u bench.py \
    --steps 8 --warmup 2 --e2e-steps 0 --bank-steps 0 --no-cpu-baseline "$@" > $out/ab_$i.json 2> $out/ab_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('$out/ab_$i.json').read().strip().splitlines()[-1])
print('$kv'.ljust(40), 'ms/step %.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['roofline']['kernel_ms'].items() if k in ('wide', 'wide_accumulate', 'finalize', 'split', 'paged', 'pixel')})"
  i=$((i+1))
done
