# round 4: DRF depth-20 (10M x 100) direct-level knob sweep, 10-tree train time each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4z
export TMPDIR=/tmp
i=0
for E in "H2OMX_X=0" "H2OMX_DIRECT_MIN_NODES=512" "H2OMX_DIRECT_MIN_NODES=2048" "H2OMX_DIRECT_WAVE_ROWS=128" "H2OMX_DIRECT_WAVE_ROWS=512" "H2OMX_PART_WAVE_NODES=1024" "H2OMX_PART_WAVE_NODES=4096" "H2OMX_X=0"; do
  i=$((i+1))
  env $E timeout -k 10 200 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4z/drf_$i.txt 2>&1 || { echo "FAIL $E"; tail -5 gpurun_out/r4z/drf_$i.txt; exit 1; }
  echo "$E $(grep 'DRF' gpurun_out/r4z/drf_$i.txt | tail -1)" | tee -a gpurun_out/r4z/sweep.txt
done
