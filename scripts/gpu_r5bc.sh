#!/bin/bash
# GLM IRLS pass 10M x 100: one slab per workgroup (new) vs one per wave (ab_old = the previous commit's package)
set -o pipefail
O=gpurun_out/r5bc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dense_gpu.py -k "glm" tests/test_glm_solvers.py > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python scripts/dense_pmc_run.py 20 na_free glm > $O/new_$rep.json 2> $O/new_$rep.err || exit 1
  (cd ab_old && timeout -k 10 200 python ../scripts/dense_pmc_run.py 20 na_free glm > ../$O/old_$rep.json 2> ../$O/old_$rep.err) || exit 1
done
