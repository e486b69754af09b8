# round 4: DRF depth 20 (10M x 100): host node-count syncs per deep level (SYNC_NODE_CAP) A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ai
export TMPDIR=/tmp
for cap in 4096 65536 1048576 4096; do
  H2OMX_SYNC_NODE_CAP=$cap timeout -k 10 200 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4ai/drf_$cap.txt 2>&1 || { tail -5 gpurun_out/r4ai/drf_$cap.txt; exit 1; }
  echo "cap=$cap $(grep 'DRF' gpurun_out/r4ai/drf_$cap.txt | tail -1)" | tee -a gpurun_out/r4ai/sweep.txt
done
