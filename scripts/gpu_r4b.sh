# round-4 profiling: per-kernel timeline of the GBM step at 11M and 1.375M rows,
# and the routing / precision-pin probe at 11M
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/prof11m -o run -- python3 bench.py --steps 10 --warmup 3 --instrument-steps 0 --fit-trees 0 --no-auc > gpurun_out/r4b/bench11m.json 2> gpurun_out/r4b/bench11m.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/prof1375k -o run -- python3 bench.py --steps 10 --warmup 3 --rows 1375000 --instrument-steps 0 --fit-trees 0 --no-auc > gpurun_out/r4b/bench1375k.json 2> gpurun_out/r4b/bench1375k.err &&
timeout -k 10 400 python3 -u scripts/route_check.py --rows 11000000 --trees 50 --out gpurun_out/r4b/route > gpurun_out/r4b/route.log 2>&1
