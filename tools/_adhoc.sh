cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "split or dream or tie" --timeout 120 --timeout-method thread > gpurun_out/t_split.log 2>&1 || { tail -50 gpurun_out/t_split.log; exit 1; }
tail -2 gpurun_out/t_split.log
LDE_VERBOSE=1 timeout -k 10 120 python bench.py --steps 10 --warmup 5 --no-cpu-baseline --strategy split > gpurun_out/b_split.json 2>gpurun_out/b_split.err || { tail gpurun_out/b_split.err; exit 1; }
head -5 gpurun_out/b_split.err
for cb in 12 14; do LDE_PIXEL_CACHE_BITS=$cb timeout -k 10 120 python bench.py --steps 10 --warmup 5 --no-cpu-baseline --strategy split > gpurun_out/b_c$cb.json 2>gpurun_out/b_c.err || { tail gpurun_out/b_c.err; exit 1; }; done
