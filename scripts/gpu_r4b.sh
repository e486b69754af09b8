# round-4 profiling: per-kernel timeline of the GBM step at 11M and 1.375M rows,
# and the routing / precision-pin probe at 11M
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b
bash scripts/gpu_prof.sh r4b_11m --instrument-steps 0 --fit-trees 0 &&
bash scripts/gpu_prof.sh r4b_1375k --rows 1375000 --instrument-steps 0 --fit-trees 0 &&
timeout -k 10 400 python3 -u scripts/route_check.py --rows 11000000 --trees 50 --out gpurun_out/r4b/route > gpurun_out/r4b/route.log 2>&1
