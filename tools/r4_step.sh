#!/bin/bash
# Round-4 working call: selected GPU tests, then the DREAM and LOKI bench lines.
# TESTS="<pytest -k expr or paths>" BENCHES="dream loki ..." bash tools/r4_step.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r4_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for b in $BENCHES; do
  case $b in
    dream) args="";;
    loki) args="--workload loki --cpu-baseline-seconds 3";;
    wl) args="--coordinate wavelength";;
    monitor) args="--workload monitor --cpu-baseline-seconds 3";;
    bifrost) args="--workload bifrost";;
    *) args="--view $b --cpu-baseline-seconds 3";;
  esac
  timeout -k 10 300 python bench.py $args --e2e-steps 0 $BENCH_EXTRA > gpurun_out/r4_bench_$b.log 2>&1 || { tail -20 gpurun_out/r4_bench_$b.log; exit 1; }
  grep -h '^{' gpurun_out/r4_bench_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$b', d['config']['strategy'], 'ms/step %.4f'%d['ms_per_step'], 'val %.3e'%d['value'], r['kernel'], 'kms %.4f'%r['avg_launch_ms'], 'frac %.3f'%r['frac'], 'step_frac %.3f'%r['step_frac'], 'hostcpu %.3f'%d.get('host_cpu_ms_per_step',-1), 'exact', d.get('check',{}).get('bit_exact_vs_oracle'))"
done
