#!/bin/bash
# First-pass timing ablations of WIDE (diagnostics build), one bench per mode.
# Usage: bash tools/r6/abl.sh <tag> "<modes>" [bench args]
set -o pipefail
tag=$1; modes=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for m in $modes; do
  LDE_LIBRARY=esslivedata_amd/libesslivedata_amd_diag.so LDE_WIDE_ABLATE=$m timeout -k 10 200 python -u bench.py \
    --steps 5 --warmup 2 --e2e-steps 0 --bank-steps 0 --no-cpu-baseline "$@" > $out/abl_$m.json 2> $out/abl_$m.err || exit $?
  python3 -c "
import json; d=json.loads(open('$out/abl_$m.json').read().strip().splitlines()[-1])
print('ablate $m', 'ms/step %.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['roofline']['kernel_ms'].items()})"
done
