#!/bin/bash
# Bench the DREAM workload under several engine knob settings (one process each).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/knob_sweep.log
: > $out
while read -r line; do
  [ -z "$line" ] && continue
  echo "== $line" >> $out
  env $line timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS} > gpurun_out/ks_one.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc" >> $out; tail -5 gpurun_out/ks_one.log >> $out; exit $rc; fi
  python - gpurun_out/ks_one.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); r = d['roofline']
        print(f"value {d['value']:.4g} step {d['ms_per_step']:.4f} dom {r['avg_launch_ms']:.4f} frac {r['frac']:.3f} " +
              ' '.join(f"{k}={v:.4f}" for k, v in r['kernel_ms'].items()))
PY
done < "${1:-tools/knobs.txt}"
cat $out
