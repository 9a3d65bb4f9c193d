#!/bin/bash
# Interleaved A/B of engine knob settings (one bench process per run, REPS
# rounds over the settings in the file), then the per-setting means.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/knob_ab.log
: > $out
for r in $(seq ${REPS:-3}); do
  while read -r line; do
    [ -z "$line" ] && continue
    env $line timeout -k 10 120 python bench.py --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --e2e-steps 0 ${BENCH_ARGS} > gpurun_out/kab_one.log 2>&1 || { echo "rc fail: $line"; tail -5 gpurun_out/kab_one.log; exit 1; }
    python3 - "$line" gpurun_out/kab_one.log >> $out <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith('{'):
        d = json.loads(l); r = d['roofline']; k = r['kernel_ms']
        print(json.dumps({'cfg': sys.argv[1], 'step': d['ms_per_step'], 'dom': r['avg_launch_ms'], **k}))
PY
  done < "$1"
done
python3 - $out <<'PY'
import json, sys, collections
acc = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); acc[d.pop('cfg')].append(d)
for cfg, rows in acc.items():
    keys = rows[0].keys()
    print(f'{cfg:40s} n={len(rows)} ' + ' '.join(f'{k}={sum(r[k] for r in rows)/len(rows):.4f}' for k in keys))
PY
