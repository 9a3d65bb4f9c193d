#!/bin/bash
# rocprofv3: kernel trace + separate PMC passes for one workload (diagnostic)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
WL=${WL:-dream}
OUT=gpurun_out/prof_${TAG:-r1}_${WL}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/kbench.py prof $WL > $OUT/kt.log 2>&1 || { echo "kt failed $?"; exit 1; }
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $pmc -d $OUT/pmc_$name -o run --output-format csv -- python3 tools/kbench.py prof $WL > $OUT/pmc_$name.log 2>&1
  rc=$?
  echo "pmc $pmc rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$name.log; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
echo done
