# round 4: DL estimator defaults, gemm_dact (fused dgrad + activation backward) for the
# 256-row mini-batch layers (H2OMX_DACT_MIN_BLOCKS=16) vs hipBLASLt + act_backward_bias
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ag
export TMPDIR=/tmp
for mb in 128 16; do
  H2OMX_DACT_MIN_BLOCKS=$mb timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4ag/dlest_mb$mb.json 2> gpurun_out/r4ag/dlest_mb$mb.err || exit 1
done &&
H2OMX_DACT_MIN_BLOCKS=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ag/dlprof -o run -- python3 bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > /dev/null 2> gpurun_out/r4ag/dlprof.err &&
python3 scripts/prof_summary.py gpurun_out/r4ag/dlprof adadelta > gpurun_out/r4ag/dl_summary.txt 2>&1
