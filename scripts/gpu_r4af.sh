# round 4: cProfile of the AutoML GLM fit (lambda search, 3-fold CV) at 10M x 100
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4af
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/glm_automl_prof.py > gpurun_out/r4af/glm_prof.txt 2>&1
