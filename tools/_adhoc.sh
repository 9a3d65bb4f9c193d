cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/host_probe.py > gpurun_out/host_probe.log 2>&1 || { tail gpurun_out/host_probe.log; exit 1; }
cat gpurun_out/host_probe.log
