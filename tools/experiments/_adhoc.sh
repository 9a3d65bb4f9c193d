cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -50 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "${BA[@]}" > gpurun_out/k_$tag.json 2>gpurun_out/k.err || { tail gpurun_out/k.err; exit 1; }
python3 -c "import json;D=json.load(open('gpurun_out/k_$tag.json'));r=D['roofline'];d=r['kernel_ms'];print('$tag', '%.4g'%D['value'], '%.4f'%D['ms_per_step'], 'frac %.3f pipe %.3f'%(r['frac'],r['pipeline_frac']), ' '.join('%s=%.4f'%(k,v) for k,v in d.items() if v))"; }
BA=()
run default LDE_X=0
run default2 LDE_X=0
