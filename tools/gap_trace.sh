#!/bin/bash
# Kernel-trace gaps between consecutive kernels of the bench (one rocprofv3
# kernel-trace pass per knob setting given as arguments, e.g. LDE_TAIL_RELEASE=0).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "$@"; do
  d=gpurun_out/gap_$(echo $cfg | tr '=' '_')
  rm -rf $d
  export $cfg
  timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $d.log 2>&1 || { echo "fail $cfg"; tail -5 $d.log; exit 1; }
  python3 - $d "$cfg" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
gaps = {}
prev = None
for r in rows:
    name = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('lde::', '')
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if prev is not None and name.startswith('k_') and not name.startswith('k_sieve<'):
        gaps.setdefault(prev[0] + ' -> ' + name, []).append((s - prev[1]) / 1e3)
    prev = (name, e)
for k, v in gaps.items():
    if len(v) >= 5:
        v = sorted(v)[:8]
        print(sys.argv[2], k, 'gap us median %.1f' % v[len(v) // 2])
PY
  unset ${cfg%%=*}
done
