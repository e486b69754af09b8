# round 4: chained step graph (tree_begin in the leaf finalisation, archive in
# boost_update) + 8-deep slab loads in reduce_split: tests, A/B, timelines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_bench_contract.py tests/test_categorical_splits.py tests/test_monotone.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4d/pytest.log 2>&1 &&
for ch in 1 0; do
  H2OMX_CHAIN_BEGIN=$ch timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > gpurun_out/r4d/b11m_ch$ch.json 2> gpurun_out/r4d/b11m_ch$ch.err || exit 1
  H2OMX_CHAIN_BEGIN=$ch timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --rows 1375000 > gpurun_out/r4d/b1375k_ch$ch.json 2> gpurun_out/r4d/b1375k_ch$ch.err || exit 1
done &&
bash scripts/gpu_prof.sh r4d_1375k --rows 1375000 --instrument-steps 0 --fit-trees 0 &&
bash scripts/gpu_prof.sh r4d_11m --instrument-steps 0 --fit-trees 0
