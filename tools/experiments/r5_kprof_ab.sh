#!/bin/bash
# round 5: rocprofv3 kernel averages of two engine builds on one box,
# interleaved: tools/ab/libbase.so (base) and the in-tree library (new)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for r in $(seq ${REPS:-2}); do
  for v in base new; do
    i=$((i+1))
    if [ $v = base ]; then export LDE_LIBRARY=$PWD/tools/ab/libbase.so; else unset LDE_LIBRARY; fi
    timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/kab/$i -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 ${BENCH_ARGS} > gpurun_out/kab_$i.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/kab_$i.log; exit 1; }
    echo "== $v"
    python tools/kstats_db.py $(find /tmp/kab/$i -name "*results.db" | head -1) 40 | grep "_ZN3lde" | grep "${KGREP:-k_sieve\|cold\|pix_acc\|pix_scat\|finalize}"
  done
done
