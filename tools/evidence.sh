#!/bin/bash
# Round evidence in one GPU call: rocprofv3 summaries (tools/prof_round.sh) of
# the DREAM, LOKI and wavelength bench commands, then the bench lines that
# read them, then the DREAM logical-view lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/profiles
TAG=${TAG:-r3}
prof() {  # name workload bench-args
  TAG=$TAG NAME=$1 WL=$2 BENCH_ARGS="$3" bash tools/prof_round.sh > gpurun_out/prof_$1.log 2>&1 || { echo "prof $1 failed"; tail -20 gpurun_out/prof_$1.log; exit 1; }
  cp gpurun_out/prof_${TAG}_$1/${TAG}_$1_bench.json gpurun_out/prof_${TAG}_$1/${TAG}_$1_bench_kernel_stats.csv gpurun_out/prof_${TAG}_$1/${TAG}_$1_traced_bench_line.json gpurun_out/profiles/ || exit 1
  cp gpurun_out/profiles/${TAG}_$1_bench.json gpurun_out/profiles/${TAG}_$1_bench_kernel_stats.csv gpurun_out/profiles/${TAG}_$1_traced_bench_line.json profiles/ || exit 1
}
if [ -z "$SKIP_PROF" ]; then
  prof dream dream ""
  prof loki loki ""
  prof wavelength dream "--coordinate wavelength"
  prof monitor monitor ""
  prof bifrost bifrost ""
fi
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 400 python bench.py > gpurun_out/bench_dream.log 2>&1 || { tail -20 gpurun_out/bench_dream.log; exit 1; }
timeout -k 10 300 python bench.py --workload loki --e2e-steps 0 --cpu-baseline-seconds 3 > gpurun_out/bench_loki.log 2>&1 || { tail -20 gpurun_out/bench_loki.log; exit 1; }
timeout -k 10 300 python bench.py --coordinate wavelength --no-cpu-baseline --e2e-steps 0 > gpurun_out/bench_wl.log 2>&1 || { tail -20 gpurun_out/bench_wl.log; exit 1; }
timeout -k 10 300 python bench.py --workload monitor --cpu-baseline-seconds 3 > gpurun_out/bench_monitor.log 2>&1 || { tail -20 gpurun_out/bench_monitor.log; exit 1; }
timeout -k 10 300 python bench.py --workload bifrost > gpurun_out/bench_bifrost.log 2>&1 || { tail -20 gpurun_out/bench_bifrost.log; exit 1; }
for v in strip_view wire_view mantle_front_layer; do
  timeout -k 10 300 python bench.py --view $v --e2e-steps 0 --cpu-baseline-seconds 3 > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
done
# the bench lines beside the profiles they cite
grep -h '^{' gpurun_out/bench_dream.log | tail -1 > gpurun_out/profiles/${TAG}_bench_line.json
grep -h '^{' gpurun_out/bench_loki.log | tail -1 > gpurun_out/profiles/${TAG}_loki_bench_line.json
grep -h '^{' gpurun_out/bench_wl.log | tail -1 > gpurun_out/profiles/${TAG}_wavelength_bench_line.json
grep -h '^{' gpurun_out/bench_monitor.log | tail -1 > gpurun_out/profiles/${TAG}_monitor_bench_line.json
grep -h '^{' gpurun_out/bench_bifrost.log | tail -1 > gpurun_out/profiles/${TAG}_bifrost_bench_line.json
for v in strip_view wire_view mantle_front_layer; do
  grep -h '^{' gpurun_out/bench_$v.log | tail -1 > gpurun_out/profiles/${TAG}_${v}_bench_line.json
done
grep -h '^{' gpurun_out/bench_*.log | cut -c1-300
