# round 4: fused slab reduction + split scan (reduce_split) - tree GPU tests,
# A/B bench at 11M and 1.375M rows, kernel timeline at 1.375M
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_tree_gpu.py tests/test_categorical_splits.py tests/test_monotone.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4c/pytest.log 2>&1 &&
for rs in 1 0; do
  H2OMX_FUSE_RS=$rs timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 > gpurun_out/r4c/b11m_rs$rs.json 2> gpurun_out/r4c/b11m_rs$rs.err || exit 1
  H2OMX_FUSE_RS=$rs timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --rows 1375000 > gpurun_out/r4c/b1375k_rs$rs.json 2> gpurun_out/r4c/b1375k_rs$rs.err || exit 1
done &&
bash scripts/gpu_prof.sh r4c_1375k --rows 1375000 --instrument-steps 0 --fit-trees 0 &&
bash scripts/gpu_prof.sh r4c_11m --instrument-steps 0 --fit-trees 0
