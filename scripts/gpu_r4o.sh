# 11M GBM histogram knob sweep with the round-4 pipeline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SWEEP_TAG=r4o_11m BENCH_ARGS="" bash scripts/sweep_env2.sh base l0c4:H2OMX_HIST_L0_COPIES=4 l0c1:H2OMX_HIST_L0_COPIES=1 fmp8:H2OMX_FUSE_MAX_PREV=8 lds96:H2OMX_HIST_LDS_KB=96 deep96:H2OMX_HIST_DEEP_LDS_KB=96 wgs768:H2OMX_HIST_WGS=768 base2
