cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { # tag env...
  tag=$1; shift
  for pmc in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $pmc | cut -c1-12 | tr ' ' '_')
    env "$@" timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/pp_$tag/$n -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --strategy split > gpurun_out/pp_${tag}_$n.log 2>&1 || { tail -5 gpurun_out/pp_${tag}_$n.log; return 1; }
  done
}
run real LDE_PIXEL_CACHE_BITS=14 && run nocache LDE_PIXEL_CACHE_BITS=0 && run abl1 LDE_ABLATE=1
