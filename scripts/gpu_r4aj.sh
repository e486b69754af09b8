# round 4 final validation: smoke(), full GPU suite, default bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4aj
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4aj/smoke.log 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4aj/pytest_full.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r4aj/bench.json 2> gpurun_out/r4aj/bench.err
tail -3 gpurun_out/r4aj/pytest_full.log
