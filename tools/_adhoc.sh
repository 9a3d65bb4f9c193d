cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --workload loki --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_loki.json 2>gpurun_out/b_loki.err || { tail gpurun_out/b_loki.err; exit 1; }
python3 -c "import json;D=json.load(open('gpurun_out/b_loki.json'));r=D['roofline'];d=r['kernel_ms'];print('loki', '%.4g'%D['value'], '%.4f'%D['ms_per_step'], D['config']['strategy'], 'frac %.3f pipe %.3f'%(r['frac'],r['pipeline_frac']), ' '.join('%s=%.4f'%(k,v) for k,v in d.items() if v))"
