cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_sieve.log 2>&1 || { tail -50 gpurun_out/t_sieve.log; exit 1; }
tail -2 gpurun_out/t_sieve.log
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "${BA[@]}" > gpurun_out/k_$tag.json 2>gpurun_out/k.err || { tail gpurun_out/k.err; exit 1; }
python3 -c "import json;D=json.load(open('gpurun_out/k_$tag.json'));d=D['roofline']['kernel_ms'];print('$tag', '%.4g'%D['value'], D['config']['strategy'], ' '.join('%s=%.4f'%(k,v) for k,v in d.items() if v))"; }
BA=()
run default LDE_X=0
BA=(--strategy split)
run s_abl2 LDE_SIEVE_ABLATE=2
run s_abl4 LDE_SIEVE_ABLATE=4
run s_nosieve LDE_SIEVE=0
