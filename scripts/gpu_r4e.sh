# round 4: multi-tree step graphs (H2OMX_GRAPH_TREES) - tests + A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_bench_contract.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4e/pytest.log 2>&1 &&
for g in 4 1 8; do
  H2OMX_GRAPH_TREES=$g timeout -k 10 200 python3 bench.py --steps 40 --warmup 4 > gpurun_out/r4e/b11m_g$g.json 2> gpurun_out/r4e/b11m_g$g.err || exit 1
  H2OMX_GRAPH_TREES=$g timeout -k 10 200 python3 bench.py --steps 40 --warmup 4 --rows 1375000 > gpurun_out/r4e/b1375k_g$g.json 2> gpurun_out/r4e/b1375k_g$g.err || exit 1
done
[ $? -eq 0 ] && bash scripts/gpu_drf10m.sh > gpurun_out/r4e/drf10m.log 2>&1
