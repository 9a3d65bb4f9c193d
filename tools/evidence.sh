#!/bin/bash
# Round evidence in one GPU call: rocprofv3 summaries of the DREAM and LOKI
# bench commands (tools/prof_round.sh) and the bench lines that read them.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-r2}
for wl in dream loki; do
  TAG=$TAG WL=$wl bash tools/prof_round.sh > gpurun_out/prof_$wl.log 2>&1 || { echo "prof $wl failed"; tail -20 gpurun_out/prof_$wl.log; exit 1; }
  mkdir -p gpurun_out/profiles
  cp gpurun_out/prof_${TAG}_${wl}/${TAG}_${wl}_bench.json gpurun_out/prof_${TAG}_${wl}/${TAG}_${wl}_bench_kernel_stats.csv gpurun_out/profiles/ || exit 1
  cp gpurun_out/profiles/${TAG}_${wl}_bench.json gpurun_out/profiles/${TAG}_${wl}_bench_kernel_stats.csv profiles/ || exit 1
done
timeout -k 10 400 python bench.py > gpurun_out/bench_dream.log 2>&1 || { tail -20 gpurun_out/bench_dream.log; exit 1; }
timeout -k 10 300 python bench.py --workload loki --no-cpu-baseline > gpurun_out/bench_loki.log 2>&1 || { tail -20 gpurun_out/bench_loki.log; exit 1; }
timeout -k 10 300 python bench.py --coordinate wavelength --no-cpu-baseline --e2e-steps 0 > gpurun_out/bench_wl.log 2>&1 || { tail -20 gpurun_out/bench_wl.log; exit 1; }
grep -h '^{' gpurun_out/bench_dream.log gpurun_out/bench_loki.log gpurun_out/bench_wl.log | cut -c1-400
