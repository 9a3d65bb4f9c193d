#!/bin/bash
# Round evidence: rocprofv3 summaries (tools/prof_round.sh) of the bench
# commands, each with the bench line of its own traced run, then the untraced
# bench lines that cite them.  SET=main (DREAM, LOKI, wavelength, monitor,
# BIFROST) or SET=views (the DREAM logical views); one GPU call each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/profiles
TAG=${TAG:-r4}
SET=${SET:-main}
prof() {  # name workload bench-args
  TAG=$TAG NAME=$1 WL=$2 BENCH_ARGS="$3" bash tools/prof_round.sh > gpurun_out/prof_$1.log 2>&1 || { echo "prof $1 failed"; tail -20 gpurun_out/prof_$1.log; exit 1; }
  for f in ${TAG}_$1_bench.json ${TAG}_$1_bench_kernel_stats.csv ${TAG}_$1_traced_bench_line.json; do
    cp gpurun_out/prof_${TAG}_$1/$f gpurun_out/profiles/ && cp gpurun_out/prof_${TAG}_$1/$f profiles/ || exit 1
  done
}
line() {  # name bench-args: the untraced bench line beside the profile
  timeout -k 10 400 python bench.py $2 > gpurun_out/bench_$1.log 2>&1 || { tail -20 gpurun_out/bench_$1.log; exit 1; }
  grep -h '^{' gpurun_out/bench_$1.log | tail -1 > gpurun_out/profiles/${TAG}_$1_bench_line.json
  cut -c1-300 gpurun_out/profiles/${TAG}_$1_bench_line.json
}
if [ "$SET" = main ]; then
  if [ -z "$SKIP_PROF" ]; then
    prof dream dream ""
    prof loki loki ""
    prof wavelength dream "--coordinate wavelength"
    prof monitor monitor ""
    prof bifrost bifrost ""
  fi
  [ -n "$SKIP_BENCH" ] && exit 0
  line dream ""
  line loki "--workload loki --e2e-steps 0 --cpu-baseline-seconds 3"
  line wavelength "--coordinate wavelength --e2e-steps 0"
  line monitor "--workload monitor --cpu-baseline-seconds 3"
  line bifrost "--workload bifrost"
else
  if [ -z "$SKIP_PROF" ]; then
    for v in strip_view wire_view mantle_front_layer; do
      prof $v dream "--view $v"
    done
  fi
  [ -n "$SKIP_BENCH" ] && exit 0
  for v in strip_view wire_view mantle_front_layer; do
    line $v "--view $v --e2e-steps 0 --cpu-baseline-seconds 3"
  done
fi
exit 0
