#!/bin/bash
# A/B of the product library (one build) against the diagnostics library
# (another build of the same sources), interleaved on one box.
# Usage: bash tools/r6/libab.sh <tag> <rounds> [bench args]
set -o pipefail
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for lib in product diag; do
    if [ $lib = diag ]; then L=esslivedata_amd/libesslivedata_amd_diag.so; else L=esslivedata_amd/libesslivedata_amd.so; fi
    env LDE_LIBRARY=$L timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --e2e-steps 0 --bank-steps 0 \
      --no-cpu-baseline "$@" > $out/${lib}_$r.json 2> $out/${lib}_$r.err || exit $?
    python3 -c "
import json; d=json.loads(open('$out/${lib}_$r.json').read().strip().splitlines()[-1])
print('$lib'.ljust(10), 'ms/step %.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['roofline']['kernel_ms'].items() if k in ('wide', 'wide_accumulate', 'finalize', 'split', 'pixel')})"
  done
done
