# round 4: K-Means host-side centroid tables (one upload per pass): tests + timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ak
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py tests/test_estimators_gpu.py -x -q -k "kmeans or KMeans or no_reference" --timeout 120 --timeout-method thread > gpurun_out/r4ak/pytest.log 2>&1 &&
timeout -k 10 120 python3 scripts/dense_pmc_run.py 5 na_free > gpurun_out/r4ak/dense.json 2> gpurun_out/r4ak/dense.err
