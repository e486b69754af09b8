cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4f.sh; echo "r4f rc=$?" > gpurun_out/r4fg_status.txt
bash scripts/gpu_r4g.sh; echo "r4g rc=$?" >> gpurun_out/r4fg_status.txt
cat gpurun_out/r4fg_status.txt
