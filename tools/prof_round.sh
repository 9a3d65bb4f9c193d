#!/bin/bash
# rocprofv3 on the bench command itself: one kernel-trace/--stats pass, then
# separate PMC passes (no tracing domains combined with --pmc), then the
# summary into profiles/${TAG}_${WL}_bench{.json,_kernel_stats.csv}.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
WL=${WL:-dream}
TAG=${TAG:-r3}
NAME=${NAME:-$WL}  # profile name (e.g. wavelength with BENCH_ARGS="--coordinate wavelength")
OUT=gpurun_out/prof_${TAG}_${NAME}
ARGS="bench.py --workload $WL --steps ${STEPS:-10} --warmup 2 --timing-stride 1 --no-cpu-baseline --e2e-steps 0 --bank-steps 0 ${BENCH_ARGS}"
rm -rf $OUT
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $ARGS > $OUT/kt.log 2>&1
rc=$?
echo "kernel trace rc=$rc"
if [ $rc -ne 0 ]; then tail -20 $OUT/kt.log; exit $rc; fi
# the bench line of the traced run itself: its HIP-event kernel average and
# the rocprofv3 average come from the same dispatches
grep -h '^{' $OUT/kt.log | tail -1 > $OUT/${TAG}_${NAME}_traced_bench_line.json
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_$name -o run --output-format csv -- python3 $ARGS > $OUT/pmc_$name.log 2>&1
  rc=$?
  echo "pmc $pmc rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$name.log; exit $rc; fi
done
python3 tools/prof_summary.py $OUT $OUT/${TAG}_${NAME}_bench > $OUT/summary.log 2>&1 || { cat $OUT/summary.log; exit 1; }
echo done
