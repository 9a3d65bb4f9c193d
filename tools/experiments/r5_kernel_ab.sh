#!/bin/bash
# round 5: per-kernel durations (rocprofv3 --kernel-trace) of the DREAM bench
# under engine settings CFGS (space-separated VAR=value items, diagnostics
# build; ablations give wrong counts by design).  TAG names the output.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export LDE_LIBRARY=$PWD/esslivedata_amd/libesslivedata_amd_diag.so
tag=${TAG:-ab}
i=0
for cfg in ${CFGS:-X=0}; do
  i=$((i+1))
  export ${cfg//,/ }
  timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_$tag/$i -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 ${BENCH_ARGS} > gpurun_out/${tag}_$i.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/${tag}_$i.log; exit 1; }
  for kv in ${cfg//,/ }; do unset ${kv%%=*}; done
  echo "== $cfg"
  python tools/kstats_db.py $(find /tmp/prof_$tag/$i -name "*results.db" | head -1) 40 | grep "_ZN3lde" | grep "${KGREP:-finalize\|k_sieve\|cold}"
  grep -o "\"ms_per_step\": [0-9.]*\|\"bit_exact_vs_oracle\": [a-z]*" gpurun_out/${tag}_$i.log | head -2 | tr "\n" " "; echo
done
