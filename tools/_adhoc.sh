cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "dream or split or tie or empty or device" > gpurun_out/t_sieve.log 2>&1 || { tail -50 gpurun_out/t_sieve.log; exit 1; }
tail -2 gpurun_out/t_sieve.log
rm -rf gpurun_out/kt1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/kt1.log 2>&1 || { tail -20 gpurun_out/kt1.log; exit 1; }
f=$(find gpurun_out/kt1 -name '*kernel_stats.csv' | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'lde' in r['Name']: print('%-40s %6s %10.2f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))
"
tail -1 gpurun_out/kt1.log | cut -c1-200
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES TA_BUSY_avr TA_BUSY_max" "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $pmc | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $pmc -d gpurun_out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -3 gpurun_out/pmc_$name.log; }
done
python3 - <<'PY'
import csv,glob,collections
for f in glob.glob('gpurun_out/pmc_*/**/*counter_collection.csv', recursive=True):
    agg=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'k_sieve' in r['Kernel_Name'] or 'k_cold' in r['Kernel_Name']:
            agg[(r['Kernel_Name'][:24],r['Counter_Name'])].append(float(r['Counter_Value']))
    for k,v in sorted(agg.items()): print(k, '%.4g' % (sum(v)/len(v)))
PY
