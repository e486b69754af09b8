#!/bin/bash
# A/B the headline bench over tree-kernel variants and env settings.
# Usage: gpu_variants.sh "LABEL|VARIANT_DIR_OR_-|ENV=V ENV2=V" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  IFS='|' read -r label vdir envs <<< "$spec"
  libdir=""; [ "$vdir" != "-" ] && libdir="H2OMX_LIB_DIR=h2omx/lib/variants/$vdir"
  env $libdir $envs timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-auc > gpurun_out/var_$label.json 2> gpurun_out/var_$label.err \
    || { echo "$label FAILED"; tail -5 gpurun_out/var_$label.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var_$label.json')); print('$label', round(d['ms_per_step'],4), 'ms/step')"
done
