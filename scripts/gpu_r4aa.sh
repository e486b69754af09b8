# round 4: DL estimator-default step timeline (hipBLASLt small GEMMs, 8-step graph replays)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4aa
export TMPDIR=/tmp
OUT=gpurun_out/r4aa/dlprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > gpurun_out/r4aa/dlest.json 2> gpurun_out/r4aa/dlest.err &&
python3 scripts/prof_summary.py $OUT adadelta > gpurun_out/r4aa/dl_summary.txt 2>&1
