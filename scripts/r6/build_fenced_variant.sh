#!/bin/bash
# Timing-only diagnostic (not a product build): the r6 write-through P2P
# protocol with round 5's cache maintenance put back - a system-scope release
# fence (L2 write-back) before every flag post and a system-scope acquire
# (L2 + L1 invalidate) after every poll.  Output:
# h2omx/lib/variants/fenced/libh2omx_tree.so (H2OMX_LIB_DIR=h2omx/lib/variants/fenced).
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
cp h2omx/csrc/*.h h2omx/csrc/tree_kernels.hip h2omx/csrc/sketch_kernels.hip $T/
python3 - "$T/p2p_device.h" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
a = "  if (threadIdx.x < kWave) {\n    const int lane = threadIdx.x;\n    if (lane < d.world) {"
assert a in s
s = s.replace(a, "  if (threadIdx.x < kWave) {\n    const int lane = threadIdx.x;\n    __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"\");\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    if (lane < d.world) {", 1)
b = "  if (threadIdx.x < kWave) wave_wait(d, d.flags[d.rank] + slot * kMaxRanks, e);\n  __syncthreads();"
assert b in s
s = s.replace(b, "  if (threadIdx.x < kWave) {\n    wave_wait(d, d.flags[d.rank] + slot * kMaxRanks, e);\n    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"\");\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n  }\n  __syncthreads();", 1)
open(p, "w").write(s)
PY
mkdir -p h2omx/lib/variants/fenced
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -munsafe-fp-atomics -I $T \
  -o h2omx/lib/variants/fenced/libh2omx_tree.so $T/tree_kernels.hip $T/sketch_kernels.hip
rm -rf $T
ls -la h2omx/lib/variants/fenced/libh2omx_tree.so
