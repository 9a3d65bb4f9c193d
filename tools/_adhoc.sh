cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench_gather3 > gpurun_out/gather3.txt 2>&1 || { cat gpurun_out/gather3.txt; exit 1; }
cat gpurun_out/gather3.txt
