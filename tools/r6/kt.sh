#!/bin/bash
# Kernel trace of one bench configuration + the per-kernel timeline summary.
# Usage: bash tools/r6/kt.sh <tag> [bench args]   (LDE_LIBRARY etc. from env)
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/kt_$tag; rm -rf $out; mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv -- python3 bench.py \
  --steps 8 --warmup 2 --timing-stride 1 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 "$@" > $out/kt.log 2>&1 || { tail -20 $out/kt.log; exit 1; }
python3 tools/r6/gaps.py $out/kt/run_kernel_trace.csv 12 > $out/gaps.txt && head -14 $out/gaps.txt
grep -h '^{' $out/kt.log | tail -1 | cut -c1-200
