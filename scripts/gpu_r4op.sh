cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4p.sh && bash scripts/gpu_r4o.sh
