#!/bin/bash
# Round evidence: rocprofv3 summaries (tools/prof_round.sh) of the bench
# commands, each with the bench line of its own traced run, then the untraced
# bench lines that cite them.  NAMES selects the profiles (default: all, in
# two GPU calls: NAMES="dream loki wavelength" and NAMES="monitor bifrost
# strip_view wire_view mantle_front_layer"); SET=main|views kept as shorthands.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/profiles
TAG=${TAG:-r6}
case "${SET:-}" in
  main) NAMES=${NAMES:-"dream loki wavelength monitor bifrost"} ;;
  views) NAMES=${NAMES:-"strip_view wire_view mantle_front_layer"} ;;
esac
NAMES=${NAMES:-"dream loki wavelength monitor bifrost strip_view wire_view mantle_front_layer"}
prof_args() {  # name -> workload and bench args of the profile
  case $1 in
    dream) echo "dream|" ;;
    loki) echo "loki|" ;;
    wavelength) echo "dream|--coordinate wavelength" ;;
    monitor) echo "monitor|" ;;
    bifrost) echo "bifrost|" ;;
    dream_t1000log) echo "dream|--num-bins 1000 --toa-scale log" ;;
    dream_t10000log) echo "dream|--num-bins 10000 --toa-scale log" ;;
    loki_t1000linear) echo "loki|--num-bins 1000 --toa-scale linear" ;;
    *) echo "dream|--view $1" ;;
  esac
}
line_args() {  # name -> args of the untraced bench line
  case $1 in
    dream) echo "" ;;
    loki) echo "--workload loki --e2e-steps 0 --cpu-baseline-seconds 3" ;;
    wavelength) echo "--coordinate wavelength --e2e-steps 0" ;;
    monitor) echo "--workload monitor --cpu-baseline-seconds 3" ;;
    bifrost) echo "--workload bifrost" ;;
    dream_t1000log) echo "--num-bins 1000 --toa-scale log --e2e-steps 0 --cpu-baseline-seconds 3" ;;
    dream_t10000log) echo "--num-bins 10000 --toa-scale log --e2e-steps 0 --cpu-baseline-seconds 3" ;;
    loki_t1000linear) echo "--workload loki --num-bins 1000 --toa-scale linear --e2e-steps 0 --cpu-baseline-seconds 3" ;;
    *) echo "--view $1 --e2e-steps 0 --cpu-baseline-seconds 3" ;;
  esac
}
prof() {  # name
  local a; a=$(prof_args $1)
  TAG=$TAG NAME=$1 WL=${a%%|*} BENCH_ARGS="${a#*|}" bash tools/prof_round.sh > gpurun_out/prof_$1.log 2>&1 || { echo "prof $1 failed"; tail -20 gpurun_out/prof_$1.log; exit 1; }
  for f in ${TAG}_$1_bench.json ${TAG}_$1_bench_kernel_stats.csv ${TAG}_$1_traced_bench_line.json; do
    cp gpurun_out/prof_${TAG}_$1/$f gpurun_out/profiles/ && cp gpurun_out/prof_${TAG}_$1/$f profiles/ || exit 1
  done
  echo "prof $1 done"
}
line() {  # name: the untraced bench line beside the profile
  timeout -k 10 400 python bench.py $(line_args $1) > gpurun_out/bench_$1.log 2>&1 || { tail -20 gpurun_out/bench_$1.log; exit 1; }
  grep -h '^{' gpurun_out/bench_$1.log | tail -1 > gpurun_out/profiles/${TAG}_$1_bench_line.json
  cut -c1-300 gpurun_out/profiles/${TAG}_$1_bench_line.json
}
if [ -z "$SKIP_PROF" ]; then
  for n in $NAMES; do prof $n; done
fi
[ -n "$SKIP_BENCH" ] && exit 0
for n in $NAMES; do line $n; done
exit 0
