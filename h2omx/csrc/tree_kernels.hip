// Histogram tree engine kernels (GBM / XGBoost-hist / DRF) for gfx950.
//
// Design (see docs/ARCHITECTURE.md "Tree engine"):
//   * Features are pre-binned once into uint8 codes stored FEATURE-MAJOR
//     ([F][npad]) so that a workgroup that owns a group of features streams
//     exactly those columns, 16 rows per lane per 16-byte load.
//   * Trees grow level-wise.  Every level streams all rows once; rows are
//     routed by a per-row node id (nid).  Only the smaller child of every
//     split is histogrammed ("built"); the sibling is parent - built
//     (subtraction trick), so LDS atomics are spent on <= half the rows.
//   * Per-workgroup private histograms live in LDS as packed fixed-point
//     integers: one ds_add_u64 per (row, feature) carries (int32 G_q << 32 |
//     uint32 S_q) (see K3 below).  Each workgroup flushes its histogram with
//     plain coalesced stores into a partial slab and hist_reduce sums the
//     slabs in exact int64; split scans decode to fp64.  No global atomics
//     on the hot path (see MI355X_MICROARCH.md "Global float atomics").
//   * Deep levels of the segmented engine (DRF / XGBoost depth 10-20) run
//     in direct mode: rows live in per-node segments and seg_direct_kernel
//     builds each node's eligible features and scans them in LDS.
//   * The level bookkeeping (which nodes split, which child gets built,
//     node numbering) runs on the device, so a whole tree is a fixed
//     sequence of launches with NO host synchronisation: the host only
//     enqueues work, the GPU decides the tree.  Between the reduce and the
//     split scan the caller may insert an all-reduce of the built
//     histograms (RCCL over xGMI) - that is the only communication.
//
// Reference parity: the reference repository (isgasho/h2o-kubernetes)
// deploys the H2O-3 Java image whose GBM/DRF/XGBoost implement these
// algorithms (src/k8s/templates.rs:28-30 launches h2o.jar); this file is the
// MI355X-native replacement of that compute path.
#include "common.h"
#include "p2p_device.h"
#include <math.h>

#include <algorithm>
#include <cstdlib>

namespace {

struct SplitParams {
  int mode;          // 0: H2O squared-error gain on (G, W); 1: XGBoost 2nd-order gain on (G, H)
  int leaf_mode;     // 0: Newton step -G/(H+lambda); 1: mean -G/W (DRF)
  int F;
  int is_last_level;
  double min_rows;            // min sum of weights per child (mode 0 and 1)
  double min_child_weight;    // min hessian sum per child (mode 1)
  double lambda_;             // L2 on leaf weights (mode 1 / leaf)
  double alpha;               // L1 on leaf weights
  double gamma;               // min loss reduction (mode 1)
  double min_split_improvement;  // relative (mode 0)
  double learn_rate;          // multiplies leaf values
  double max_abs_leaf;        // |leaf| clip (0 = none)
  uint32_t seed;
  int tree_index;
  int depth;
  float col_rate;             // per-node column sampling rate (1 = all)
  int mtries;                 // exact per-node feature count (0 = off)
  int children_leaves;        // children of splits at this level are final leaves
  int pad2;
  // monotone constraints (nullptr = none): mono[F] in {-1, 0, +1}; gbound
  // [capacity][2] = [lo, hi] interval of every node's value, set by its parent
  const signed char* mono;
  double* gbound;
  // interaction constraints (nullptr = none): ifsets[F] = bit mask of the
  // user's interaction sets holding feature f (0: unlisted, interacts only
  // with itself); istate[capacity][2] = (compatible-set mask, solo feature)
  // of every node, written by its parent's split (root: all sets, -2 = no
  // feature on the path yet)
  const unsigned long long* ifsets;
  long long* istate;
  // categorical group splits (nullptr = no categorical features): catf[F] = 1
  // for an identity-binned enum column (bin = level code); a split of such a
  // feature sends a SET of levels left (levels sorted by G / S inside the node,
  // best prefix of that order).  fbcat [max_nodes][F][8] holds each (node,
  // feature) winner's left-set bitset (256 bits); the finalisation copies the
  // chosen one into treecat [capacity][8] (the tree's bitsets, by node id)
  const uint8_t* catf;
  uint32_t* fbcat;
  uint32_t* treecat;
  // per-node histogram rule (adaptive_candidates): hist_mode 0 = every fine bin,
  // 1 UniformAdaptive, 2 Random, 3 RoundRobin; edges [F][NBT] fine cut points,
  // frange [F][4] = (min, max, exact, integer)
  const float* edges;
  const float* frange;
  int hist_mode;
  int hist_top;      // nbins_top_level
  int hist_nbins;    // nbins (per-node floor)
  int pad3;
};

struct NodeSplit {  // best split of one node at the current level (64 B)
  double gain;
  double G, H, W;      // node totals
  double GL, HL, WL;   // left-child totals of the chosen split
  int feat;            // -1 = no valid split
  int bin;             // rows with bin <= this go left
  int na_left;
  int pad;
};

struct NodeLink {  // per node of a level: where its histogram comes from
  int slot;       // >= 0: histogram built this level in that slot
  int sib_slot;   // if slot < 0: sibling's slot (hist = parent - sibling)
  int parent;     // local index of the parent in the previous level
  int pad;
};

struct PartInfo {  // per node of a level: routing decision for partition
  int feat;
  int bin;       // threshold bin; categorical split: low 32 bits of its bitset pointer
  int na_left;   // bit 0: NA goes left; bit 1: categorical split; bits 8..31: bitset pointer >> 32
  int child;  // local id of left child at next level, -1 = node is a leaf
  int gid;    // global node id inside the tree
  int leaf_children;  // 1: children are leaves, rows retire into them now
  int child_gid;      // global id of the left child
  int pad;            // split nodes: build slots of the children, int16 left | int16 right << 16
};

struct TreeNode {  // model representation (32 B)
  int feat;      // -1 = leaf
  int bin;
  int left;      // global id of left child (right = left + 1)
  int na_left;   // bit 0: NA goes left; bit 1: categorical split (left set = the tree's bitset of this node)
  float thr;     // raw-value threshold: x <= thr goes left (NaN -> na_left)
  float value;   // leaf value (already scaled by the learning rate)
  float gain;
  float weight;  // sum of weights in the node
};

// Routing of a row with bin code b through a split record: 1 = right.
// Categorical splits test the left-set bitset the record points to (bits of
// the tree's bitset table, see SplitParams::treecat); numeric ones the bin.
__device__ __forceinline__ int part_right(const PartInfo& pi, int b, int nbt) {
  if (b == nbt - 1) return !(pi.na_left & 1);
  if (pi.na_left & 2) {
    const uint32_t* bits = reinterpret_cast<const uint32_t*>(
        (uint64_t)(uint32_t)pi.bin | ((uint64_t)((uint32_t)pi.na_left >> 8) << 32));
    return !((bits[b >> 5] >> (b & 31)) & 1u);
  }
  return b > pi.bin;
}

// the record fields of a categorical split whose left set is `bits`
__device__ __forceinline__ void part_set_cat(PartInfo& pi, const uint32_t* bits, int na_left) {
  const uint64_t a = reinterpret_cast<uint64_t>(bits);
  pi.bin = (int)(uint32_t)a;
  pi.na_left = (na_left & 1) | 2 | (int)((uint32_t)(a >> 32) << 8);
}

// ctl layout (int32 device array, one per level buffer):
//   [0] n_nodes at this level, [1] n_slots built at this level,
//   [2] base = global id of local node 0, [3] total nodes in tree so far
constexpr int CTL_N = 0, CTL_SLOTS = 1, CTL_BASE = 2, CTL_TOTAL = 3;

__device__ __forceinline__ double leaf_value(double G, double H, double W, const SplitParams& p) {
  double v;
  if (p.leaf_mode == 1) {
    v = (W > 0.0) ? -G / W : 0.0;
  } else {
    double g = G;
    if (p.alpha > 0.0) {
      if (g > p.alpha) g -= p.alpha;
      else if (g < -p.alpha) g += p.alpha;
      else g = 0.0;
    }
    double den = H + p.lambda_;
    v = (den > 1e-12) ? -g / den : 0.0;
  }
  v *= p.learn_rate;
  if (p.max_abs_leaf > 0.0) v = fmin(fmax(v, -p.max_abs_leaf), p.max_abs_leaf);
  return v;
}

__device__ __forceinline__ double l1_thresh(double g, double a) {
  if (a <= 0.0) return g;
  if (g > a) return g - a;
  if (g < -a) return g + a;
  return 0.0;
}

// Gain of splitting a node with totals (G, S) into L = (GL, SL) and R = total
// - L.  S is the weight/count (mode 0, H2O squared error) or the hessian
// (mode 1, XGBoost).  Returns -inf if the split violates a constraint.
// the parent's term of the gain (G^2 / S, or t(G)^2 / (S + lambda)): the same
// for every candidate of a node, so scans that see many features of one node
// compute it once (split_gain_pt; identical bits to split_gain)
__device__ __forceinline__ double parent_term(double G, double S, const SplitParams& p) {
  if (p.mode == 0) return G * G / S;
  const double tt = l1_thresh(G, p.alpha);
  return tt * tt / (S + p.lambda_);
}

__device__ __forceinline__ double split_gain_pt(double GL, double SL, double G, double S, double pt,
                                                const SplitParams& p) {
  const double GR = G - GL, SR = S - SL;
  if (p.mode == 0) {
    if (SL < p.min_rows || SR < p.min_rows || SL <= 0.0 || SR <= 0.0) return -INFINITY;
    return GL * GL / SL + GR * GR / SR - pt;
  }
  if (SL < p.min_child_weight || SR < p.min_child_weight || SL <= 0.0 || SR <= 0.0) return -INFINITY;
  const double lam = p.lambda_;
  const double tl = l1_thresh(GL, p.alpha), tr = l1_thresh(GR, p.alpha);
  return 0.5 * (tl * tl / (SL + lam) + tr * tr / (SR + lam) - pt) - p.gamma;
}

__device__ __forceinline__ double split_gain(double GL, double SL, double G, double S, const SplitParams& p) {
  return split_gain_pt(GL, SL, G, S, parent_term(G, S, p), p);
}

// ---------------------------------------------------------------------------
// DPP wave primitives for the split scans.  The row_shr 1 / 2 / 4 / 8 steps,
// then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3), run on the VALU
// data path; the __shfl_* forms they replace go through ds_bpermute (an LDS
// round trip per step), and a scan is a chain of six dependent steps.  Lanes
// without a source (or outside the row mask) take the operation's identity.
// ---------------------------------------------------------------------------
template <int CTRL, int RM>
__device__ __forceinline__ long long dpp_i64(long long v) {
  const unsigned long long u = (unsigned long long)v;
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, RM, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, RM, 0xf, false);
  return (long long)(((unsigned long long)hi << 32) | lo);
}

// inclusive prefix sum over the 64 lanes (exact int64: the same values as the
// shfl_up scan)
__device__ __forceinline__ long long wave_incl_scan_i64(long long x) {
  x += dpp_i64<0x111, 0xf>(x);
  x += dpp_i64<0x112, 0xf>(x);
  x += dpp_i64<0x114, 0xf>(x);
  x += dpp_i64<0x118, 0xf>(x);
  x += dpp_i64<0x142, 0xa>(x);
  x += dpp_i64<0x143, 0xc>(x);
  return x;
}

__device__ __forceinline__ long long readlane_i64(long long v, int l);

// wave sum (exact int64), every lane returns it
__device__ __forceinline__ long long wave_sum_i64(long long x) { return readlane_i64(wave_incl_scan_i64(x), 63); }

__device__ __forceinline__ int wave_sum_i32(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return __builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ long long readlane_i64(long long v, int l) {
  const unsigned long long u = (unsigned long long)v;
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return (long long)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __longlong_as_double(readlane_i64(__double_as_longlong(v), l));
}

// one step of the (larger gain, then smaller code) arg-max; identity (-inf, INT_MAX)
template <int CTRL, int RM>
__device__ __forceinline__ void argmax_step(double& g, int& c) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(g);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, RM, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)0xFFF00000u, (int)(unsigned)(u >> 32), CTRL, RM, 0xf,
                                                            false);
  const int oc = __builtin_amdgcn_update_dpp(0x7fffffff, c, CTRL, RM, 0xf, false);
  const double og = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
  if (og > g || (og == g && oc < c)) { g = og; c = oc; }
}

// wave arg-max of (g, c) (a total order: the result is the xor-butterfly's);
// every lane returns it
__device__ __forceinline__ void wave_argmax(double& g, int& c) {
  argmax_step<0x111, 0xf>(g, c);
  argmax_step<0x112, 0xf>(g, c);
  argmax_step<0x114, 0xf>(g, c);
  argmax_step<0x118, 0xf>(g, c);
  argmax_step<0x142, 0xa>(g, c);
  argmax_step<0x143, 0xc>(g, c);
  g = readlane_f64(g, 63);
  c = __builtin_amdgcn_readlane(c, 63);
}

// the same for (gain, 64-bit key) pairs; identity (-inf, LLONG_MAX)
template <int CTRL, int RM>
__device__ __forceinline__ void argmax_key_step(double& g, long long& k) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(g);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, RM, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)0xFFF00000u, (int)(unsigned)(u >> 32), CTRL, RM, 0xf,
                                                            false);
  const unsigned long long uk = (unsigned long long)k;
  const unsigned klo = (unsigned)__builtin_amdgcn_update_dpp((int)0xFFFFFFFFu, (int)(unsigned)uk, CTRL, RM, 0xf, false);
  const unsigned khi = (unsigned)__builtin_amdgcn_update_dpp(0x7fffffff, (int)(unsigned)(uk >> 32), CTRL, RM, 0xf,
                                                             false);
  const double og = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
  const long long ok = (long long)(((unsigned long long)khi << 32) | klo);
  if (og > g || (og == g && ok < k)) { g = og; k = ok; }
}

__device__ __forceinline__ void wave_argmax_key(double& g, long long& k) {
  argmax_key_step<0x111, 0xf>(g, k);
  argmax_key_step<0x112, 0xf>(g, k);
  argmax_key_step<0x114, 0xf>(g, k);
  argmax_key_step<0x118, 0xf>(g, k);
  argmax_key_step<0x142, 0xa>(g, k);
  argmax_key_step<0x143, 0xc>(g, k);
  g = readlane_f64(g, 63);
  k = readlane_i64(k, 63);
}

// wave min (MAX = false) / max (MAX = true) of an int; every lane returns it
template <bool MAX, int CTRL, int RM>
__device__ __forceinline__ int minmax_step(int v) {
  const int o = __builtin_amdgcn_update_dpp(MAX ? (int)0x80000000 : 0x7fffffff, v, CTRL, RM, 0xf, false);
  return MAX ? max(v, o) : min(v, o);
}
template <bool MAX>
__device__ __forceinline__ int wave_minmax_i32(int v) {
  v = minmax_step<MAX, 0x111, 0xf>(v);
  v = minmax_step<MAX, 0x112, 0xf>(v);
  v = minmax_step<MAX, 0x114, 0xf>(v);
  v = minmax_step<MAX, 0x118, 0xf>(v);
  v = minmax_step<MAX, 0x142, 0xa>(v);
  v = minmax_step<MAX, 0x143, 0xc>(v);
  return __builtin_amdgcn_readlane(v, 63);
}

// Monotone constraint of the candidate split's feature (H2O / XGBoost
// monotone_constraints): +1 needs value(left) <= value(right), -1 the
// reverse; child values from the split's (G, S) totals (S = W or H by mode).
// The node-value interval [lo, hi] (SplitParams::gbound) then keeps every
// descendant on its side of the split's midpoint (see lf_write_node).
__device__ __forceinline__ bool mono_ok(int mf, double GL, double SL, double G, double S, const SplitParams& p) {
  if (mf == 0) return true;
  const double wl = leaf_value(GL, SL, SL, p), wr = leaf_value(G - GL, S - SL, S - SL, p);
  return mf > 0 ? wl <= wr : wl >= wr;
}

// H2O / XGBoost interaction_constraints: may node gid split on feature f?
// (every feature on the root path and f must share one interaction set;
// an unlisted feature only combines with itself)
__device__ __forceinline__ bool inter_ok(const SplitParams& p, int gid, int f) {
  if (p.istate == nullptr) return true;
  const long long solo = p.istate[2 * gid + 1];
  if (solo == -2) return true;            // nothing on the path yet
  if (solo >= 0) return f == (int)solo;   // path used an unlisted feature
  return (p.ifsets[f] & (unsigned long long)p.istate[2 * gid]) != 0ull;
}

// the state a split of node gid on feature f hands to both children
__device__ __forceinline__ void inter_children(const SplitParams& p, int gid, int f, int cg) {
  const long long solo = p.istate[2 * gid + 1];
  const unsigned long long fs = p.ifsets[f];
  long long c_mask = 0, c_solo = f;
  if (fs != 0ull) {
    const unsigned long long comp = (solo == -2) ? ~0ull : (unsigned long long)p.istate[2 * gid];
    c_mask = (long long)(comp & fs);
    c_solo = -1;
  }
  p.istate[2 * cg] = c_mask; p.istate[2 * cg + 1] = c_solo;
  p.istate[2 * cg + 2] = c_mask; p.istate[2 * cg + 3] = c_solo;
}

__device__ __forceinline__ double clamp_bound(double v, const SplitParams& p, int gid, int cap) {
  if (p.gbound == nullptr || gid <= 0 || gid >= cap) return v;
  return fmin(fmax(v, p.gbound[2 * gid]), p.gbound[2 * gid + 1]);
}

}  // namespace

// ---------------------------------------------------------------------------
// K1: feature binning.  X is feature-major fp32 [F][ld]; edges is [F][NBT]
// (edges[f][j] for j < nvb[f]-1 are the sorted bin upper edges).  A value v
// maps to lower_bound(edges, v); NaN maps to the NA bin NBT-1.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bin_features_kernel(const float* __restrict__ X, int64_t ld, int64_t n,
                                                           const float* __restrict__ edges,
                                                           const int* __restrict__ nvb, int nbt,
                                                           uint8_t* __restrict__ codes, int64_t npad) {
  __shared__ float e[256];
  const int f = blockIdx.y;
  const int m = nvb[f] - 1;  // number of edges
  for (int j = threadIdx.x; j < 256; j += blockDim.x) e[j] = (j < m) ? edges[(int64_t)f * nbt + j] : INFINITY;
  __syncthreads();
  const float* x = X + (int64_t)f * ld;
  uint8_t* c = codes + (int64_t)f * npad;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < npad; r += (int64_t)gridDim.x * blockDim.x) {
    uint8_t code = 0;
    if (r < n) {
      const float v = x[r];
      if (v != v) {
        code = (uint8_t)(nbt - 1);
      } else {
        int lo = 0, hi = m;  // first index with e[idx] >= v
        while (lo < hi) {
          int mid = (lo + hi) >> 1;
          if (e[mid] < v) lo = mid + 1; else hi = mid;
        }
        code = (uint8_t)lo;
      }
    }
    c[r] = code;
  }
}

// ---------------------------------------------------------------------------
// K3: LDS-privatised histogram build with packed fixed-point integer atomics.
//
// Measured on MI355X (bench_micro/lds_atomics.hip): ds_add_f32 retires only
// ~0.33 lanes/CU/cycle whatever the address pattern, while ds_add_u64 on
// random bins retires ~4.5 lanes/CU/cycle.  So every (row, feature) does ONE
// 64-bit integer LDS atomic carrying both statistics:
//     packed = (int32 G_q) << 32 | (uint32 S_q)
// G_q / S_q are the row's gradient and second statistic (weight/count for
// H2O squared-error mode, hessian for XGBoost mode) stochastically rounded to
// fixed point with per-tree scales (QG / max|g|, QS / max s).  A workgroup
// accumulates at most ROWS_CAP rows, which bounds |sum G_q| < 2^31 and
// sum S_q < 2^32, so the low half never carries into the high half and the
// packed 64-bit add is exact.  The reduction over workgroups is exact int64
// arithmetic: histograms are bitwise deterministic regardless of atomic order.
// Low-cardinality features (e.g. 3-valued b-tags) are replicated R = NBT /
// (nvb+1) times inside their own NBT-wide LDS slice, lane l using copy l % R,
// which removes the same-address serialisation (measured 4x slower) at no LDS
// cost.  Grid = n_groups * wgpg (wgpg % 8 == 0); blockIdx -> (chunk, group)
// keeps the groups of one row chunk on one XCD (L2 reuse of g/h/nid; speed
// only, never correctness).
// ---------------------------------------------------------------------------
constexpr int ROWS_CAP = 2097152;        // max rows per workgroup chunk (host picks <= this; the scales adapt)
constexpr float QG = 32768.0f;           // |G_q| per row <= QG  -> |sum| <= 2^30
constexpr float QS = 65536.0f;           // S_q per row <= QS    -> sum <= 2^31

// qscale (double[8]): [0] QG/gmax [1] QS/smax [2] 1/[0] [3] 1/[1]
//                     [4] leaf g scale [5] leaf h scale [6] leaf w scale
// stat_max (uint32[4] float bits): max|g|, max h, max w (atomicMax targets)

__device__ __forceinline__ uint32_t row_hash(int64_t r, uint32_t salt) {
  return mix32((uint32_t)r * 0x9E3779B1u ^ mix32(salt + (uint32_t)(r >> 32)));
}

// LDS written by some lanes of a wave, read by other lanes of the same wave
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// PKM (per-row inputs):
//   0  node id -> NodeLink slot, (g, s2) quantised here (segmented engine)
//   1  as 0, and feature group 0 stores the packed quantised row pk[r]
//      (level 0 of the scan engine: the quantisation is fixed for the tree)
//   2  slot16[r] written by the previous partition + stored pk[r]: no link
//      gathers and no dither hashing on deeper levels, where several
//      feature groups / slot passes would otherwise redo that per-row work
//   3  as 1, pk stored as 32 bits (int16 G_q << 16 | uint16 S_q)
//   4  as 2, reading those 32-bit rows: halves the per-row stream that every
//      feature group of a deep level re-reads.  The host picks 3/4 only when
//      the per-row magnitudes fit 16 bits (rows per workgroup >= 2^16 puts
//      |G_q| <= 2^14 and S_q <= 2^15), so histograms stay bit-identical.
// ROUTE (deeper levels, PKM 2/4): the previous level's partition is fused in.
// Instead of slot16, every row's previous-level node id (nid) is routed
// through that level's PartInfo table (split feature code gathered per row)
// to its node at this level and its build slot; feature group 0 of the
// writer pass stores the new node ids into nid_out (double-buffered: every
// group and slot pass reads the previous ids).  Rows of nodes that stopped
// splitting retire as ~gid; their exact leaf sums are added by the tree's
// final partition (all-rows mode).  Saves one streaming pass per level.
// CMP (deeper levels, PKM 2/4, ROWS 16): LDS-staged wave compaction.  A
// ds_add_u64 wave-instruction costs ~14 CU-cycles whatever its lane mask
// (bench_micro/lds_mask.hip: 14.3 cycles with 12 % of lanes active, 17.3 with
// all), so issuing one atomic per (row position, feature) wastes most of the
// LDS pipe on levels where only the smaller children (<= 50 % of the rows)
// are built.  Here each wave (1024 consecutive rows) ranks its live rows with
// five bit-plane ballots, writes them as 16-bit entries (row offset | slot <<
// 10) into a per-wave 2 KB LDS area and reads them back transposed (lane j:
// entries j, j + 64, ...).  Per feature the 1 KB code tile is stored to that
// area with one ds_write_b128 per lane (the same coalesced column load as the
// plain path) and every atomic then carries 64 live rows: ceil(live / 64)
// full-mask atomics instead of 16 mostly-empty ones.  Same adds, same
// integer histograms (bit-identical).
struct GradParams {
  int dist;
  int apply_tree;      // add the leaf values of `tree` to F first
  float sample_rate;   // row bagging (1 = off)
  uint32_t seed;
  int tree_index;      // index of the NEXT tree (bag seed)
  float tweedie_power;
  float quantile_alpha;
  float huber_delta;
  long long row_base;   // global index of this rank's first row (bagging hash)
  int skip_nid;         // 1: leave nid alone (the scan engine treats level 0 / 1 as an implicit root)
  int pad;
};

__device__ __forceinline__ void dist_grad(int dist, float f, float y, const GradParams& gp, float& g, float& h) {
  switch (dist) {
    case 0: g = f - y; h = 1.0f; break;
    case 1: {
      const float pr = 1.0f / (1.0f + __expf(-f));
      g = pr - y;
      h = fmaxf(pr * (1.0f - pr), 1e-16f);
      break;
    }
    case 2: { const float mu = __expf(f); g = mu - y; h = fmaxf(mu, 1e-16f); break; }
    case 3: { const float e = y * __expf(-f); g = 1.0f - e; h = fmaxf(e, 1e-16f); break; }
    case 4: {
      const float rho = gp.tweedie_power;
      const float a = y * __expf((1.0f - rho) * f), b = __expf((2.0f - rho) * f);
      g = -a + b;
      h = fmaxf(-(1.0f - rho) * a + (2.0f - rho) * b, 1e-16f);
      break;
    }
    case 5: g = (f > y) ? 1.0f : ((f < y) ? -1.0f : 0.0f); h = 1.0f; break;
    case 6: g = (y > f) ? -gp.quantile_alpha : (1.0f - gp.quantile_alpha); h = 1.0f; break;
    case 7: { const float r = f - y; g = fabsf(r) <= gp.huber_delta ? r : copysignf(gp.huber_delta, r); h = 1.0f; break; }
    default: g = -y; h = 1.0f; break;  // DRF: fit the response directly
  }
}

// PKM 5: level 0 with the gradient pass fused in (K2 + K7 + K3).  The tree
// begins from the PREVIOUS tree's leaves: F += value[~nid] (apply), (g, h)
// from (F, y) by dist_grad, quantised with scales fixed by the distribution's
// gradient bounds (|g| <= 1, h <= 1/4 for bernoulli, ...: the host writes the
// bounds into stat_max instead of reducing per-tree maxima), so the separate
// boost_update pass and the max reduction disappear.  Group 0 stores F, g, h
// (exact leaf sums of the final partition) and the 32-bit packed rows.
constexpr int GF_LDS_NODES = 1024;
struct GradFuse {
  float* F;
  const float* y;
  const int* nid;          // previous tree's leaf per row (~gid), read when apply
  const TreeNode* tree;    // previous tree
  float* g;
  float* h;
  int apply;
  int s_is_h;              // second statistic: h (mode 1) or w = 1 (mode 0)
  int pk64;                // store 64-bit packed rows (PKM 1 layout) instead of 32-bit (PKM 3)
  int cap;                 // tree capacity (nodes): <= GF_LDS_NODES values are staged in LDS
  GradParams gp;
};

constexpr int CMP_STAGE_BYTES = 2048;   // per wave
constexpr int HB_PF = 1;     // feature code loads kept in flight per lane

// COP > 1 (level 0, PKM 1 / 3): every (slot, feature, bin) entry is COP
// interleaved u64 copies, [bin][copy], lane l adding into copy l % COP: the
// 16 lanes of a ds_add_u64 group then hit at most two addresses per bank pair
// (bench_micro/lds_atomics.hip: random bins 14.4 CU-cycles per wave-atomic,
// conflict-free 7.3), at COP x the LDS per feature (fewer features per group)
// NID16 (fused-routing levels): the previous / next node ids are int16 streams
// (2 bytes a row each way instead of 4; padding rows hold INT16_MIN)
template <int NBT, int ROWS, int PKM, bool ROUTE, bool CMP, int COP = 1, bool NID16 = false>
__global__ __launch_bounds__(1024) void hist_build_kernel(
    const uint8_t* __restrict__ codes, int64_t npad, const float* __restrict__ g, const float* __restrict__ s2,
    const int* __restrict__ nid, const NodeLink* __restrict__ link, const int* __restrict__ ctl,
    const int* __restrict__ nvb, const double* __restrict__ qscale, uint32_t salt, int F, int fg, int n_groups,
    int wgpg, int slot_lo, int slot_cnt, const short* __restrict__ slot16, unsigned long long* __restrict__ pk_buf,
    unsigned long long* __restrict__ partials, const PartInfo* __restrict__ part_prev,
    const int* __restrict__ ctl_prev, int* __restrict__ nid_out, int writer, GradFuse gf) {
  salt = (uint32_t)qscale[9];  // per-tree dither salt, written by tree_begin (graph-replay safe)
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds64[];
  __shared__ int width_s[256], rep_s[256];
  __shared__ float rcp_s[256];
  const int n_slots = ctl[CTL_SLOTS];
  const int b = blockIdx.x;
  const int xcd = b & 7, i = b >> 3;
  const int group = i % n_groups;
  const int chunk = xcd + 8 * (i / n_groups);
  // uniform: nothing to build in this pass (a routing writer still moves the rows)
  const bool route_w = ROUTE && writer && group == 0 && ctl_prev[CTL_N] > 0;
  const bool build = slot_lo < n_slots;
  if (!build && !route_w) return;
  const int f0 = group * fg;
  const int nf = min(fg, F - f0);
  static_assert(COP == 1 || ((PKM == 1 || PKM == 3 || PKM == 6) && !ROUTE && !CMP), "copies: level-0 kernel only");
  const int hist_elems = slot_cnt * fg * NBT;
  const int lane = threadIdx.x & 63;

  for (int j = threadIdx.x; j < hist_elems * COP; j += blockDim.x) lds64[j] = 0ull;
  if (threadIdx.x < fg) {
    const int fi = threadIdx.x;
    const int w = (fi < nf) ? nvb[f0 + fi] + 1 : NBT;
    width_s[fi] = w;
    int r = NBT / w;
    r = r < 1 ? 1 : (r > 64 ? 64 : r);
    // the copies already spread the lanes (slicing low-cardinality features
    // inside the copies' space measured slower: profiles/r6/l0_sliced_ab_r6m.txt)
    if (COP > 1) r = 1;
    rep_s[fi] = r;
    rcp_s[fi] = 1.0f / (float)r;   // lane % rep without an integer division (lane < 64: exact)
  }
  __shared__ float tval_s[PKM == 5 ? GF_LDS_NODES : 1];
  if constexpr (PKM == 5) {   // previous tree's node values (leaf gathers from LDS)
    if (gf.apply && gf.cap <= GF_LDS_NODES)
      for (int j = threadIdx.x; j < gf.cap; j += blockDim.x) tval_s[j] = gf.tree[j].value;
  }
  const float sg = (float)qscale[0], ss = (float)qscale[1];
  const int64_t rb = (int64_t)qscale[7];  // global row offset of this rank (dither)
  const int64_t n_rows = (int64_t)qscale[8];  // this rank's live rows (implicit-root levels)
  __syncthreads();

  const int64_t units = npad / ROWS;
  const int64_t u0 = units * chunk / wgpg, u1 = units * (chunk + 1) / wgpg;
  // CMP: waves step through the chunk together (64 consecutive units per wave
  // step) so the ballots below see converged waves; tail lanes re-read the
  // chunk's last unit and contribute no rows
  const int64_t ustart = CMP ? u0 + (threadIdx.x & ~63) : u0 + threadIdx.x;
  for (int64_t uu = ustart; uu < u1; uu += blockDim.x) {
    const bool inb = !CMP || uu + lane < u1;
    const int64_t u = CMP ? (inb ? uu + lane : u1 - 1) : uu;
    const int64_t r0 = u * ROWS;
    int s[ROWS];
    bool any = false;
    if constexpr (ROUTE) {
      int nn[ROWS], nx[ROWS];
      if (nid == nullptr) {
        // implicit root (previous level = the root): every live row is in node 0,
        // no node-id stream to read (boost_update no longer resets it)
#pragma unroll
        for (int k = 0; k < ROWS; ++k) nn[k] = (r0 + k < n_rows) ? 0 : INT32_MIN;
      } else if constexpr (NID16) {
        const short* n16 = reinterpret_cast<const short*>(nid);
#pragma unroll
        for (int q = 0; q < ROWS / 8; ++q) {
          const uint4 v = *reinterpret_cast<const uint4*>(n16 + r0 + 8 * q);
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 8; ++k) nn[8 * q + k] = (int)(short)(w4[k >> 1] >> (16 * (k & 1)));
        }
      } else {
#pragma unroll
        for (int q = 0; q < ROWS / 4; ++q) {
          const int4 n4 = *reinterpret_cast<const int4*>(nid + r0 + 4 * q);
          nn[4 * q] = n4.x; nn[4 * q + 1] = n4.y; nn[4 * q + 2] = n4.z; nn[4 * q + 3] = n4.w;
        }
      }
#pragma unroll
      for (int k = 0; k < ROWS; ++k) { nx[k] = nn[k]; s[k] = -1; }
      // one wave-uniform pass per previous-level node: its split feature's codes
      // for the lane's ROWS rows come in ONE coalesced load (no per-row byte
      // gathers); the host fuses only levels whose previous level has few nodes
      const int n_prev = ctl_prev[CTL_N];
      for (int j = 0; j < n_prev; ++j) {
        bool mine = false;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) mine |= (nn[k] == j);
        if (!mine) continue;
        const PartInfo pj = part_prev[j];
        if (pj.child < 0) {
#pragma unroll
          for (int k = 0; k < ROWS; ++k)
            if (nn[k] == j) nx[k] = ~pj.gid;
          continue;
        }
        uint32_t cw[ROWS / 4];
        const uint8_t* cp = codes + (int64_t)pj.feat * npad + r0;
        if constexpr (ROWS == 16) {
          const uint4 c4 = *reinterpret_cast<const uint4*>(cp);
          cw[0] = c4.x; cw[1] = c4.y; cw[2] = c4.z; cw[3] = c4.w;
        } else {
          const uint2 c2 = *reinterpret_cast<const uint2*>(cp);
          cw[0] = c2.x; cw[1] = c2.y;
        }
        const int sl_l = (int)(short)(pj.pad & 0xFFFF), sl_r = pj.pad >> 16;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
          if (nn[k] == j) {
            const int bc = (cw[k >> 2] >> (8 * (k & 3))) & 0xff;
            const int right = part_right(pj, bc, NBT);
            nx[k] = pj.child + right;
            s[k] = right ? sl_r : sl_l;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < ROWS; ++k) {
        int sl = s[k] - slot_lo;
        if (sl < 0 || sl >= slot_cnt || !build) sl = -1;
        s[k] = sl;
        any |= (sl >= 0);
      }
      if (route_w) {
        if constexpr (NID16) {
          short* o16 = reinterpret_cast<short*>(nid_out);
#pragma unroll
          for (int q = 0; q < ROWS / 8; ++q) {
            uint32_t w4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
              w4[k] = ((uint32_t)(uint16_t)max(nx[8 * q + 2 * k], -32768)) |
                      ((uint32_t)(uint16_t)max(nx[8 * q + 2 * k + 1], -32768) << 16);
            *reinterpret_cast<uint4*>(o16 + r0 + 8 * q) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
          }
        } else {
#pragma unroll
          for (int q = 0; q < ROWS / 4; ++q)
            *reinterpret_cast<int4*>(nid_out + r0 + 4 * q) = make_int4(nx[4 * q], nx[4 * q + 1], nx[4 * q + 2], nx[4 * q + 3]);
        }
      }
    } else if constexpr (PKM == 2 || PKM == 4) {
#pragma unroll
      for (int q = 0; q < ROWS / 8; ++q) {
        const int4 v4 = *reinterpret_cast<const int4*>(slot16 + r0 + 8 * q);
        const int vw[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          int sl = (int)(short)(vw[k >> 1] >> (16 * (k & 1))) - slot_lo;
          if (sl < 0 || sl >= slot_cnt) sl = -1;
          s[8 * q + k] = sl;
          any |= (sl >= 0);
        }
      }
    } else if (nid == nullptr) {
      // implicit root (level 0 of the scan engine): live rows are node 0, slot 0
#pragma unroll
      for (int k = 0; k < ROWS; ++k) {
        int sl = (r0 + k < n_rows) ? 0 - slot_lo : -1;
        if (sl >= slot_cnt) sl = -1;
        s[k] = sl;
        any |= (sl >= 0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < ROWS / 4; ++q) {
        const int4 n4 = *reinterpret_cast<const int4*>(nid + r0 + 4 * q);
        const int nn[4] = {n4.x, n4.y, n4.z, n4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          int sl = -1;
          if (nn[k] >= 0) {
            sl = link[nn[k]].slot - slot_lo;
            if (sl >= slot_cnt) sl = -1;
          }
          s[4 * q + k] = sl;
          any |= (sl >= 0);
        }
      }
    }
    if constexpr (CMP) {
      if (__ballot(any && inb) == 0ull) continue;   // wave-uniform
    } else {
      if (!any) continue;
    }
    // codes of the next HB_PF features are in flight while this feature's
    // atomics issue (one load per wave in flight starved HBM: ~3 TB/s); the
    // first ones are issued before the per-row inputs below, so their latency
    // overlaps the (g, s) loads / gradient chain instead of following it
    uint32_t pf[HB_PF][ROWS / 4];
    auto load_codes = [&](int fi, uint32_t* cw) {
      const uint8_t* cp = codes + (int64_t)(f0 + fi) * npad + r0;
      if constexpr (ROWS == 16) {
        const uint4 c4 = *reinterpret_cast<const uint4*>(cp);
        cw[0] = c4.x; cw[1] = c4.y; cw[2] = c4.z; cw[3] = c4.w;
      } else {
        const uint2 c2 = *reinterpret_cast<const uint2*>(cp);
        cw[0] = c2.x; cw[1] = c2.y;
      }
    };
    if constexpr (!CMP) {
#pragma unroll
      for (int q = 0; q < HB_PF; ++q)
        if (q < nf) load_codes(q, pf[q]);
    }
    unsigned long long pk[ROWS];
    if constexpr (PKM == 2) {
#pragma unroll
      for (int q = 0; q < ROWS / 2; ++q) {
        const ulonglong2 p2 = *reinterpret_cast<const ulonglong2*>(pk_buf + r0 + 2 * q);
        pk[2 * q] = p2.x;
        pk[2 * q + 1] = p2.y;
      }
    } else if constexpr (PKM == 4 || PKM == 6) {
      // PKM 6 (level 0): the 16-bit packed rows boost_update quantised for this tree
      const uint32_t* pk32 = reinterpret_cast<const uint32_t*>(pk_buf);
#pragma unroll
      for (int q = 0; q < ROWS / 4; ++q) {
        const uint4 p4 = *reinterpret_cast<const uint4*>(pk32 + r0 + 4 * q);
        const uint32_t pw[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          pk[4 * q + k] = ((unsigned long long)(uint32_t)(int)(short)(pw[k] >> 16) << 32) |
                          (unsigned long long)(pw[k] & 0xFFFFu);
      }
    } else if constexpr (PKM == 5) {
#pragma unroll
      for (int q = 0; q < ROWS / 4; ++q) {
        const float4 f4 = *reinterpret_cast<const float4*>(gf.F + r0 + 4 * q);
        const float4 y4 = *reinterpret_cast<const float4*>(gf.y + r0 + 4 * q);
        int4 n4 = make_int4(-1, -1, -1, -1);
        if (gf.apply) n4 = *reinterpret_cast<const int4*>(gf.nid + r0 + 4 * q);
        float fv[4] = {f4.x, f4.y, f4.z, f4.w};
        const float yv[4] = {y4.x, y4.y, y4.z, y4.w};
        const int nv[4] = {n4.x, n4.y, n4.z, n4.w};
        float gv[4], hv[4];
        uint32_t pw[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t r = r0 + 4 * q + k;
          gv[k] = 0.f; hv[k] = 0.f; pw[k] = 0u;
          pk[4 * q + k] = 0ull;
          if (r >= n_rows) continue;
          if (gf.apply) fv[k] += (gf.cap <= GF_LDS_NODES) ? tval_s[~nv[k]] : gf.tree[~nv[k]].value;
          dist_grad(gf.gp.dist, fv[k], yv[k], gf.gp, gv[k], hv[k]);
          const uint32_t hsh = row_hash(rb + r, salt);
          const float d1 = (hsh & 0xFFFF) * (1.0f / 65536.0f), d2 = (hsh >> 16) * (1.0f / 65536.0f);
          const int gq = (int)floorf(fmaf(gv[k], sg, d1));
          const uint32_t sq = (uint32_t)floorf(fmaf(gf.s_is_h ? hv[k] : 1.0f, ss, d2));
          pk[4 * q + k] = ((unsigned long long)(uint32_t)gq << 32) | (unsigned long long)sq;
          pw[k] = ((uint32_t)gq << 16) | (sq & 0xFFFFu);
        }
        if (group == 0) {
          if (gf.apply) *reinterpret_cast<float4*>(gf.F + r0 + 4 * q) = make_float4(fv[0], fv[1], fv[2], fv[3]);
          *reinterpret_cast<float4*>(gf.g + r0 + 4 * q) = make_float4(gv[0], gv[1], gv[2], gv[3]);
          *reinterpret_cast<float4*>(gf.h + r0 + 4 * q) = make_float4(hv[0], hv[1], hv[2], hv[3]);
          if (gf.pk64) {   // deeper levels read PKM 2 rows
            *reinterpret_cast<ulonglong2*>(pk_buf + r0 + 4 * q) = make_ulonglong2(pk[4 * q], pk[4 * q + 1]);
            *reinterpret_cast<ulonglong2*>(pk_buf + r0 + 4 * q + 2) = make_ulonglong2(pk[4 * q + 2], pk[4 * q + 3]);
          } else {         // PKM 4 rows (16-bit fields: the host picked pk32)
            *reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(pk_buf) + r0 + 4 * q) =
                make_uint4(pw[0], pw[1], pw[2], pw[3]);
          }
        }
      }
    } else {
#pragma unroll
    for (int q = 0; q < ROWS / 4; ++q) {
      const float4 g4 = *reinterpret_cast<const float4*>(g + r0 + 4 * q);
      float4 s4 = make_float4(1.f, 1.f, 1.f, 1.f);
      if (s2) s4 = *reinterpret_cast<const float4*>(s2 + r0 + 4 * q);
      const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
      const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t hsh = row_hash(rb + r0 + 4 * q + k, salt);
        const float d1 = (hsh & 0xFFFF) * (1.0f / 65536.0f), d2 = (hsh >> 16) * (1.0f / 65536.0f);
        const int gq = (int)floorf(fmaf(gv[k], sg, d1));
        const uint32_t sq = (uint32_t)floorf(fmaf(sv[k], ss, d2));
        pk[4 * q + k] = ((unsigned long long)(uint32_t)gq << 32) | (unsigned long long)sq;
      }
    }
    if (PKM == 1 && group == 0) {
#pragma unroll
      for (int q = 0; q < ROWS / 2; ++q)
        *reinterpret_cast<ulonglong2*>(pk_buf + r0 + 2 * q) = make_ulonglong2(pk[2 * q], pk[2 * q + 1]);
    }
    if (PKM == 3 && group == 0) {
      uint32_t* pk32 = reinterpret_cast<uint32_t*>(pk_buf);
#pragma unroll
      for (int q = 0; q < ROWS / 4; ++q) {
        uint32_t pw[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const unsigned long long v = pk[4 * q + k];
          pw[k] = ((uint32_t)(v >> 32) << 16) | ((uint32_t)v & 0xFFFFu);
        }
        *reinterpret_cast<uint4*>(pk32 + r0 + 4 * q) = make_uint4(pw[0], pw[1], pw[2], pw[3]);
      }
    }
    }
    if constexpr (CMP) {
      static_assert(ROWS == 16 && (PKM == 2 || PKM == 4), "compaction: 16-row units reading stored rows");
      uint32_t m = 0;
#pragma unroll
      for (int r = 0; r < ROWS; ++r)
        if (inb && s[r] >= 0 && pk[r] != 0ull) m |= 1u << r;
      // exclusive rank of this lane's first live row in the wave, from the
      // bit planes of the per-lane counts (0..16): five ballots, no LDS
      const uint32_t cnt = __popc(m);
      const unsigned long long lt = (1ull << lane) - 1ull;
      int excl = 0, total = 0;
#pragma unroll
      for (int bit = 0; bit < 5; ++bit) {
        const unsigned long long bm = __ballot((cnt >> bit) & 1u);
        excl += __popcll(bm & lt) << bit;
        total += __popcll(bm) << bit;
      }
      if (total == 0) continue;
      uint16_t* st16 = reinterpret_cast<uint16_t*>(lds64 + hist_elems) + (threadIdx.x >> 6) * (CMP_STAGE_BYTES / 2);
      int j = excl;
#pragma unroll
      for (int r = 0; r < ROWS; ++r)
        if ((m >> r) & 1u) st16[j++] = (uint16_t)((lane * ROWS + r) | (s[r] << 10));
      const int niter = (total + 63) >> 6;
      const int64_t tile0 = (uu)*ROWS;   // first row of this wave's tile
      // entry i of this lane is live iff i * 64 + lane < total (every 16-bit
      // pattern is a valid entry: offset 1023 in slot 63 is 0xFFFF)
      uint32_t ent[ROWS];
      unsigned long long pkc[ROWS];
#pragma unroll
      for (int i = 0; i < ROWS; ++i) {
        ent[i] = 0u;
        if (i * 64 + lane < total) ent[i] = st16[i * 64 + lane];
      }
#pragma unroll
      for (int i = 0; i < ROWS; ++i) {
        pkc[i] = 0ull;
        if (i * 64 + lane < total) {
          const int64_t row = tile0 + (ent[i] & 1023u);
          if constexpr (PKM == 2) {
            pkc[i] = pk_buf[row];
          } else {
            const uint32_t pw = reinterpret_cast<const uint32_t*>(pk_buf)[row];
            pkc[i] = ((unsigned long long)(uint32_t)(int)(short)(pw >> 16) << 32) | (unsigned long long)(pw & 0xFFFFu);
          }
        }
      }
      // the entries are in registers before the code tiles overwrite the area
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint8_t* stc = reinterpret_cast<uint8_t*>(st16);
      uint4 pf[HB_PF];
#pragma unroll
      for (int q = 0; q < HB_PF; ++q)
        if (q < nf) pf[q] = *reinterpret_cast<const uint4*>(codes + (int64_t)(f0 + q) * npad + r0);
      for (int fb = 0; fb < nf; fb += HB_PF) {
#pragma unroll
        for (int q = 0; q < HB_PF; ++q) {
          const int fi = fb + q;
          if (fi < nf) {
            *reinterpret_cast<uint4*>(stc + lane * ROWS) = pf[q];
            if (fi + HB_PF < nf) pf[q] = *reinterpret_cast<const uint4*>(codes + (int64_t)(f0 + fi + HB_PF) * npad + r0);
            const int width = width_s[fi], rep = rep_s[fi];
            const int copy_off = (rep > 1) ? (lane % rep) * width : 0;
            const int na_slot = (rep > 1) ? width - 1 : NBT - 1;   // see the fold below
            unsigned long long* hb = lds64 + fi * NBT + copy_off;
#pragma unroll
            for (int i = 0; i < ROWS; ++i) {
              if (i < niter && i * 64 + lane < total) {
                int bin = stc[ent[i] & 1023u];
                if (bin == NBT - 1) bin = na_slot;
                atomicAdd(hb + (int)(ent[i] >> 10) * fg * NBT + bin, pkc[i]);
              }
            }
          }
        }
      }
      continue;
    }
    // per-row slot offset into the histogram (-1: nothing to add), once per unit
    int so[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) so[r] = (s[r] >= 0 && pk[r] != 0ull) ? s[r] * fg * NBT : -1;
    for (int fb = 0; fb < nf; fb += HB_PF) {
#pragma unroll
      for (int q = 0; q < HB_PF; ++q) {
        const int fi = fb + q;
        if (fi < nf) {
          uint32_t cw[ROWS / 4];
#pragma unroll
          for (int k = 0; k < ROWS / 4; ++k) cw[k] = pf[q][k];
          if (fi + HB_PF < nf) load_codes(fi + HB_PF, pf[q]);
          const int rep = rep_s[fi];
          if (rep > 1) {
            // replicated low-cardinality slice: copy lane % rep, NA at the
            // slice's last slot (wave-uniform branch: rep is per feature)
            const int width = width_s[fi];
            const int copy = lane - rep * (int)(((float)lane + 0.5f) * rcp_s[fi]);
            unsigned long long* hb = lds64 + fi * NBT + copy * width;
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
              if (so[r] >= 0) {
                int bin = (cw[r >> 2] >> (8 * (r & 3))) & 0xff;
                if (bin == NBT - 1) bin = width - 1;
                atomicAdd(hb + so[r] + bin, pk[r]);
              }
            }
          } else if (COP > 1) {
            // interleaved copies: entry (slot, fi, bin) at ((slot * fg + fi) * NBT + bin) * COP + copy
            unsigned long long* hb = lds64 + fi * NBT * COP + (lane & (COP - 1));
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
              if (so[r] >= 0) atomicAdd(hb + (so[r] + ((cw[r >> 2] >> (8 * (r & 3))) & 0xff)) * COP, pk[r]);
            }
          } else {
            // one NBT-wide slice: the NA code NBT - 1 is its own slot (no remap)
            unsigned long long* hb = lds64 + fi * NBT;
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
              if (so[r] >= 0) atomicAdd(hb + so[r] + ((cw[r >> 2] >> (8 * (r & 3))) & 0xff), pk[r]);
            }
          }
        }
      }
    }
  }
  __syncthreads();
  // fold the lane copies and write this workgroup's slab (plain stores)
  unsigned long long* out = partials + (int64_t)(group * wgpg + chunk) * hist_elems;
  if constexpr (COP > 1) {
    // fold the copies (rotated start: the threads of a lane group read different banks)
    for (int j = threadIdx.x; j < hist_elems; j += blockDim.x) {
      unsigned long long acc = 0ull;
#pragma unroll
      for (int c = 0; c < COP; ++c) acc += lds64[j * COP + ((c + j) & (COP - 1))];
      out[j] = acc;
    }
    return;
  }
  for (int j = threadIdx.x; j < hist_elems; j += blockDim.x) {
    const int bin = j % NBT;
    const int fi = (j / NBT) % fg;
    const int sl = j / (NBT * fg);
    const int width = width_s[fi], rep = rep_s[fi];
    const unsigned long long* hb = lds64 + (sl * fg + fi) * NBT;
    unsigned long long acc = 0ull;
    if (rep == 1) {
      acc = hb[bin];   // one slice, NA kept in its own slot NBT - 1
    } else {
      const int src = (bin == NBT - 1) ? width - 1 : bin;
      if (src < width - 1 || bin == NBT - 1)
        for (int c = 0; c < rep; ++c) acc += hb[c * width + src];
    }
    out[j] = acc;
  }
}

// Sum the per-workgroup slabs of one pass into exact int64 histograms
// built[slot][F][2][NBT] (plane 0: G_q, plane 1: S_q).
// Each 256-thread block owns 32 consecutive output bins and splits the
// workgroup-slab dimension over 8 lane groups (4 loads in flight per lane),
// then folds the 8 partial sums through LDS: latency is hidden by parallel
// slabs instead of a long dependent chain per output element.
__global__ __launch_bounds__(256) void hist_reduce_kernel(const unsigned long long* __restrict__ partials,
                                                          int n_groups, int wgpg, int fg, int F, int nbt, int slot_lo,
                                                          int slot_cnt, const int* __restrict__ ctl,
                                                          long long* __restrict__ built) {
  __shared__ long long rg[8][33], rs[8][33];
  const int n_slots = ctl[CTL_SLOTS];
  const int64_t hist_elems = (int64_t)slot_cnt * fg * nbt;
  const int e = threadIdx.x & 31, c0 = threadIdx.x >> 5;
  const int64_t idx = (int64_t)blockIdx.x * 32 + e;  // output element (s, f, bin)
  const int bin = idx % nbt;
  const int f = (idx / nbt) % F;
  const int s = idx / ((int64_t)nbt * F);
  const bool live = (s < slot_cnt) && (slot_lo + s < n_slots);
  long long ag = 0, as = 0;
  if (live) {
    const int group = f / fg, fi = f % fg;
    const unsigned long long* p =
        partials + (int64_t)group * wgpg * hist_elems + ((int64_t)s * fg + fi) * nbt + bin;
    int c = c0;
    for (; c + 24 < wgpg; c += 32) {
      const unsigned long long v0 = p[(int64_t)c * hist_elems], v1 = p[(int64_t)(c + 8) * hist_elems];
      const unsigned long long v2 = p[(int64_t)(c + 16) * hist_elems], v3 = p[(int64_t)(c + 24) * hist_elems];
      ag += (long long)(int32_t)(uint32_t)(v0 >> 32) + (long long)(int32_t)(uint32_t)(v1 >> 32) +
            (long long)(int32_t)(uint32_t)(v2 >> 32) + (long long)(int32_t)(uint32_t)(v3 >> 32);
      as += (long long)(uint32_t)v0 + (long long)(uint32_t)v1 + (long long)(uint32_t)v2 + (long long)(uint32_t)v3;
    }
    for (; c < wgpg; c += 8) {
      const unsigned long long v = p[(int64_t)c * hist_elems];
      ag += (long long)(int32_t)(uint32_t)(v >> 32);
      as += (long long)(uint32_t)v;
    }
  }
  rg[c0][e] = ag;
  rs[c0][e] = as;
  __syncthreads();
  if (c0 == 0 && live) {
    long long tg = 0, ts = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) { tg += rg[k][e]; ts += rs[k][e]; }
    long long* o = built + (((int64_t)(slot_lo + s) * F + f) * 2) * nbt + bin;
    o[0] = tg;
    o[nbt] = ts;
  }
}

// ---------------------------------------------------------------------------
// K4 + K5: complete the level's histograms (built or parent - sibling, exact
// int64), keep them as parents for the next level, and scan for the best
// threshold of one (node, feature) pair per 256-thread workgroup (thread t
// owns bin t; grid = max_nodes x F so even a 16-node level fills the chip).
// The per-node arg-max over features happens in level_finalize.
// ---------------------------------------------------------------------------
struct FeatBest {  // 64 B
  double gain;
  double GL, SL;   // left-child totals of the chosen threshold
  double G, S;     // node totals (as seen from this feature's histogram)
  double pad0;
  int code;        // (bin * 2 + na_left), INT_MAX = none
  int pad1;
  double pad2;
};

// Best threshold of (node, f) computed by one wave; every lane returns the
// same result (gain -inf / code INT_MAX = none).  Also stores the completed
// histogram row into `full` (parent of the next level) when given.
struct WaveBest {
  double gain, GL, SL, G, S;
  int code;
};

// Categorical (node, feature): H2O / LightGBM group split.  The non-empty
// level bins are ordered by G / S (S = W or H by mode; ties by level code,
// empty bins last), and every prefix of that order is a candidate left set,
// scored for both NA directions like a threshold.  One wave, no LDS: each
// lane's inclusive prefix in sorted order comes from an all-pairs pass over
// the NBT bins (256 shuffled (key, G, S) triples - categorical features are
// few and this runs per node only for them).  The winner's left set is
// written as a 256-bit bitset to p.fbcat[node][f].
template <int NBT>
__device__ __forceinline__ WaveBest feat_best_cat_wave(const long long* gi, const long long* si, long long ng_i,
                                                    long long ns_i, int node, int f, int m, double ig, double is,
                                                    const SplitParams& p) {
  constexpr int B = NBT <= 64 ? 1 : NBT / 64;
  const int lane = threadIdx.x & 63;
  double key[B];
  bool ne[B];
  long long tg_l = 0, ts_l = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int bin = lane * B + k;
    ne[k] = bin < m && bin < NBT - 1 && si[k] > 0;
    key[k] = ne[k] ? (double)gi[k] / (double)si[k] : INFINITY;
    tg_l += gi[k];
    ts_l += si[k];
  }
  tg_l = wave_sum_i64(tg_l);
  ts_l = wave_sum_i64(ts_l);
  const double tg = (double)(tg_l + ng_i) * ig, ts = (double)(ts_l + ns_i) * is;
  const double ng = (double)ng_i * ig, ns = (double)ns_i * is;
  long long cg[B], cs[B];
#pragma unroll
  for (int k = 0; k < B; ++k) { cg[k] = 0; cs[k] = 0; }
  const int lanes = NBT < 64 ? NBT : 64;
  for (int jl = 0; jl < lanes; ++jl) {
#pragma unroll
    for (int jk = 0; jk < B; ++jk) {
      const double kj = __shfl(key[jk], jl, kWave);
      const long long gj = __shfl(gi[jk], jl, kWave), sj = __shfl(si[jk], jl, kWave);
      const int j = jl * B + jk;
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int bin = lane * B + k;
        if (ne[k] && (kj < key[k] || (kj == key[k] && j <= bin))) { cg[k] += gj; cs[k] += sj; }
      }
    }
  }
  double best_gain = -INFINITY;
  int best_code = 0x7fffffff;
  double bGL = 0, bSL = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int t = lane * B + k;
    if (!ne[k]) continue;
    const double sg = (double)cg[k] * ig, ssum = (double)cs[k] * is;
    const double gA = split_gain(sg, ssum, tg, ts, p);
    const double gB = ns > 0.0 ? split_gain(sg + ng, ssum + ns, tg, ts, p) : -INFINITY;
    if (gA > -INFINITY && (gA > best_gain || (gA == best_gain && 2 * t < best_code))) {
      best_gain = gA; best_code = 2 * t; bGL = sg; bSL = ssum;
    }
    if (gB > -INFINITY && (gB > best_gain || (gB == best_gain && 2 * t + 1 < best_code))) {
      best_gain = gB; best_code = 2 * t + 1; bGL = sg + ng; bSL = ssum + ns;
    }
  }
  double bg = best_gain;
  int bc = best_code;
  wave_argmax(bg, bc);
  WaveBest r;
  r.G = tg; r.S = ts;
  r.gain = (bc == 0x7fffffff) ? -INFINITY : bg;
  r.code = bc;
  r.GL = r.SL = 0.0;
  uint32_t word = 0;
  if (bc != 0x7fffffff) {
    const unsigned long long own = __ballot(best_code == bc);
    const int src = __builtin_amdgcn_readfirstlane(__ffsll((long long)own) - 1);
    r.GL = readlane_f64(bGL, src);
    r.SL = readlane_f64(bSL, src);
    // left set: every non-empty bin at or before the winner in (key, level) order
    const int wb = bc >> 1;
    double kown = key[0];
#pragma unroll
    for (int k = 1; k < B; ++k)
      if (k == wb % B) kown = key[k];
    const double kw = __shfl(kown, wb / B, kWave);
    uint32_t nib = 0;
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int bin = lane * B + k;
      if (ne[k] && (key[k] < kw || (key[k] == kw && bin <= wb))) nib |= 1u << k;
    }
    constexpr int LPW = 32 / B;   // lanes per 32-bit bitset word
    word = nib << (B * (lane % LPW));
#pragma unroll
    for (int o = 1; o < LPW; o <<= 1) word |= __shfl_xor(word, o, kWave);
  }
  // lanes 0..7 store the 8 words (word w lives in lane w * LPW; words past the
  // last lane's bins are zero)
  {
    constexpr int LPW = 32 / B;
    const int srcl = lane * LPW;
    const uint32_t wv = __shfl(word, srcl < 64 ? srcl : 63, kWave);
    if (lane < 8) p.fbcat[((int64_t)node * p.F + f) * 8 + lane] = (srcl < 64) ? wv : 0u;
  }
  return r;
}

// Feature eligibility of (node, f), wave-uniform: a feature outside the node's
// mtries / column sample only needs its histogram row completed for the next
// level and the node totals - no prefix scan, no gains (DRF looks at sqrt(F)
// of F features, so this skips most of the per-node work)
__device__ __forceinline__ bool feat_allowed(const uint8_t* __restrict__ tree_fmask, const SplitParams& p, int node,
                                             int f, int gid) {
  const int F = p.F;
  const int lane = threadIdx.x & 63;
  bool allowed = (tree_fmask == nullptr) || tree_fmask[f];
  if (allowed && (p.mtries > 0 || p.col_rate < 1.0f)) {
    const uint32_t key = (uint32_t)p.tree_index * 131u + (uint32_t)p.depth;
    const uint32_t hf = hash4(p.seed, key, (uint32_t)node, (uint32_t)f);
    if (p.mtries > 0) {
      int rank = 0;
      for (int j0 = 0; j0 < F; j0 += 64) {
        const int j = j0 + lane;
        bool below = false;
        if (j < F) {
          const uint32_t hj = hash4(p.seed, key, (uint32_t)node, (uint32_t)j);
          below = (hj < hf) || (hj == hf && j < f);
        }
        rank += __popcll(__ballot(below));
      }
      allowed = rank < p.mtries;
    } else {
      allowed = u01(hf) < p.col_rate;
    }
  }
  return allowed && inter_ok(p, gid, f);
}

// H2O's adaptive histograms (hex/tree/DHistogram; histogram_type AUTO =
// UniformAdaptive) re-bin every node's own [min, max] of a numeric column into
// nb = max(nbins_top_level >> depth, nbins) equal-width bins (Random: nb - 1
// uniform random cut points in that range, drawn per node; RoundRobin: one of
// UniformAdaptive, UniformAdaptive, Random, QuantilesGlobal by tree index, the
// AUTO entry of H2O's cycle being UniformAdaptive).  Here the histogram stays
// the fine one (<= 255 quantile or one-per-value bins) and the node's candidate
// thresholds are restricted instead: fine edge e[t] stays a candidate iff some
// cut falls in its cell (midpoint to the previous interior edge, midpoint to
// the next], i.e. it is the interior edge nearest to that cut (ties: the lower
// one).  The node's range comes from its first / last non-empty fine bin
// (their lower / upper boundaries; exact bins: their values, the true node
// min / max).  An integer column spanning <= nb values keeps every threshold
// (H2O: one bin per integer).  Returns bit k = bin lane * B + k is a candidate;
// thresholds outside [lo, hi) (NA-only partitions) always are.
// CPU mirror: reference/tree.py adaptive_mask (same double arithmetic,
// contraction off, same hashes).
__device__ __forceinline__ double ua_cut(double lo, double span, int k, int nb) {
#pragma clang fp contract(off)
  return lo + (span * (double)k) / (double)nb;
}

// number of uniform cuts c_1 .. c_{nb-1} at or below x
__device__ __forceinline__ int ua_count(double x, double lo, double span, int nb) {
#pragma clang fp contract(off)
  if (x == -INFINITY) return 0;
  if (x == INFINITY) return nb - 1;
  const double r = (x - lo) * (double)nb / span;
  int k = r < 0.0 ? 0 : (r >= (double)(nb - 1) ? nb - 1 : (int)r);
  while (k < nb - 1 && ua_cut(lo, span, k + 1, nb) <= x) ++k;
  while (k > 0 && ua_cut(lo, span, k, nb) > x) --k;
  return k;
}

// ua_count against a table of the exact cuts (cut[k] = ua_cut(lo, span, k, nb),
// k < nb): the estimate comes from a multiply by nb / span instead of a
// division and is then corrected against the exact cuts.  The cuts are
// non-decreasing in k, so the two correction loops end on the unique count
// whatever the start: the same k as ua_count, without its three divisions.
__device__ __forceinline__ int ua_count_tab(double x, double lo, double rs, int nb, const double* __restrict__ cut) {
#pragma clang fp contract(off)
  if (x == -INFINITY) return 0;
  if (x == INFINITY) return nb - 1;
  const double r = (x - lo) * rs;
  int k = r < 0.0 ? 0 : (r >= (double)(nb - 1) ? nb - 1 : (int)r);
  while (k < nb - 1 && cut[k + 1] <= x) ++k;
  while (k > 0 && cut[k] > x) --k;
  return k;
}

// cut_tab: 64 doubles of per-wave LDS (nullptr: the division form)
template <int NBT, int B>
__device__ uint32_t adaptive_candidates(const long long* si, int m, int node, int f, const SplitParams& p,
                                        double* cut_tab = nullptr) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  int mode = p.hist_mode;
  if (mode == 3) mode = (0x0211 >> (4 * (p.tree_index & 3))) & 15;   // UA, UA, Random, QuantilesGlobal
  if (mode == 0) return 0xffffffffu;
  // the node's occupied fine bins: weight plane > 0, i.e. its rows of
  // POSITIVE weight (zero-weight rows widen no node range, as H2O's
  // histograms skip them; tests/test_hist_adaptive.py zero-weight parity)
  int lo = 0x7fffffff, hi = -1;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int t = lane * B + k;
    if (t < m && t < NBT - 1 && si[k] > 0) { lo = min(lo, t); hi = max(hi, t); }
  }
  lo = wave_minmax_i32<false>(lo);
  hi = wave_minmax_i32<true>(hi);
  if (hi - lo < 1) return 0xffffffffu;   // no interior threshold
  const float* e = p.edges + (int64_t)f * NBT;
  const float* fr = p.frange + (int64_t)f * 4;
  const bool exact = fr[2] != 0.0f;
  double lo_v, hi_v;
  if (exact) {
    lo_v = (double)(lo < m - 1 ? e[lo] : fr[1]);
    hi_v = (double)(hi < m - 1 ? e[hi] : fr[1]);
  } else {
    lo_v = (double)(lo == 0 ? fr[0] : e[lo - 1]);
    hi_v = (double)(hi == m - 1 ? fr[1] : e[hi]);
  }
  const double span = hi_v - lo_v;
  if (!(span > 0.0) || !(span < INFINITY)) return 0xffffffffu;
  const int top = p.depth < 31 ? (p.hist_top >> p.depth) : 0;
  const int nb = max(max(top, p.hist_nbins), 2);
  if (fr[3] != 0.0f && span + 1.0 <= (double)nb) return 0xffffffffu;
  double mL[B], mR[B];
  uint32_t inner = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int t = lane * B + k;
    mL[k] = -INFINITY; mR[k] = INFINITY;
    if (t >= lo && t < hi) {
      inner |= 1u << k;
      const double x = (double)e[t];
      if (t > lo) mL[k] = 0.5 * ((double)e[t - 1] + x);
      if (t < hi - 1) mR[k] = 0.5 * (x + (double)e[t + 1]);
    }
  }
  uint32_t hit = 0;
  if (mode == 1 && cut_tab != nullptr && nb <= 64) {
    // UniformAdaptive with <= 64 cuts (every level from depth 4 on with H2O's
    // defaults): the cuts once per feature (one division per lane), and each
    // interior boundary counted once - bin t's upper midpoint is bin t + 1's
    // lower one (same operands, same bits), so the lower count is the
    // neighbour's upper count.  Same candidate bits as the branch below.
    if (lane < nb) cut_tab[lane] = ua_cut(lo_v, span, lane, nb);
    wave_lds_sync();
    const double rs = (double)nb / span;
    int cR[B];
#pragma unroll
    for (int k = 0; k < B; ++k) cR[k] = ((inner >> k) & 1u) ? ua_count_tab(mR[k], lo_v, rs, nb, cut_tab) : 0;
    const int prev = __shfl_up(cR[B - 1], 1, kWave);
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int t = lane * B + k;
      const int cL = t > lo ? (k > 0 ? cR[k - (k > 0)] : prev) : 0;
      if (((inner >> k) & 1u) && cR[k] > cL) hit |= 1u << k;
    }
    wave_lds_sync();   // the table is rewritten by the wave's next feature
  } else if (mode == 1) {
#pragma unroll
    for (int k = 0; k < B; ++k)
      if (((inner >> k) & 1u) && ua_count(mR[k], lo_v, span, nb) > ua_count(mL[k], lo_v, span, nb)) hit |= 1u << k;
  } else if (inner) {
    const uint32_t key = ((uint32_t)p.tree_index * 131u + (uint32_t)p.depth) ^ ((uint32_t)f * 0x9E3779B1u);
    const uint32_t s2 = p.seed ^ 0x52414E44u;
    for (int j = 1; j < nb; ++j) {
      const double c = lo_v + span * (double)u01(hash4(s2, key, (uint32_t)node, (uint32_t)j));
#pragma unroll
      for (int k = 0; k < B; ++k)
        if (mL[k] < c && c <= mR[k]) hit |= 1u << k;
    }
    hit &= inner;
  }
  return (~inner) | hit;
}

__device__ __forceinline__ WaveBest wave_best_none() {
  WaveBest r;
  r.G = r.S = 0.0;
  r.gain = -INFINITY; r.code = 0x7fffffff; r.GL = r.SL = 0.0;
  return r;
}

// Best threshold of (node, f) from the completed histogram row held in
// registers (lane owns bins lane * B .. lane * B + B - 1; B = NBT / 64).
template <int NBT, bool CAT>
__device__ __forceinline__ WaveBest feat_scan_wave(long long* gi, long long* si, bool allowed, int node, int f,
                                                   const int* __restrict__ nvb, double ig, double is,
                                                   const SplitParams& p) {
  constexpr int B = NBT <= 64 ? 1 : NBT / 64;  // bins per lane
  const int lane = threadIdx.x & 63;
  if (!allowed) {
    long long tg_i = 0, ts_i = 0;
#pragma unroll
    for (int k = 0; k < B; ++k) { tg_i += gi[k]; ts_i += si[k]; }
    tg_i = wave_sum_i64(tg_i);
    ts_i = wave_sum_i64(ts_i);
    WaveBest r;
    r.G = (double)tg_i * ig; r.S = (double)ts_i * is;
    r.gain = -INFINITY; r.code = 0x7fffffff; r.GL = r.SL = 0.0;
    return r;
  }
  // NA bin (NBT - 1) excluded from the running sums
  constexpr int NA_LANE = (NBT - 1) / B, NA_K = (NBT - 1) % B;
  const long long ng_i = readlane_i64(gi[NA_K], NA_LANE), ns_i = readlane_i64(si[NA_K], NA_LANE);
  if (lane == NA_LANE) { gi[NA_K] = 0; si[NA_K] = 0; }
  if constexpr (CAT) {   // instantiated only for data with categorical features
    if (p.catf != nullptr && p.catf[f])
      return feat_best_cat_wave<NBT>(gi, si, ng_i, ns_i, node, f, nvb[f], ig, is, p);
  }
  long long lg = 0, ls = 0;  // inclusive local prefix
  long long pg[B], ps[B];
#pragma unroll
  for (int k = 0; k < B; ++k) { lg += gi[k]; ls += si[k]; pg[k] = lg; ps[k] = ls; }
  const long long xg = wave_incl_scan_i64(lg), xs = wave_incl_scan_i64(ls);  // wave inclusive scan of lane totals
  const long long tg_i = readlane_i64(xg, 63) + ng_i, ts_i = readlane_i64(xs, 63) + ns_i;
  const long long eg = xg - lg, es = xs - ls;  // exclusive lane offset
  const double ng = (double)ng_i * ig, ns = (double)ns_i * is;
  const double tg = (double)tg_i * ig, ts = (double)ts_i * is;

  double best_gain = -INFINITY;
  int best_code = 0x7fffffff;
  double bGL = 0, bSL = 0;
  const int m = nvb[f];
  const int mf = p.mono ? (int)p.mono[f] : 0;
  const uint32_t cand = p.hist_mode ? adaptive_candidates<NBT, B>(si, m, node, f, p) : 0xffffffffu;
  if (allowed) {
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int t = lane * B + k;
      if (t < m && t < NBT - 1 && ((cand >> k) & 1u)) {
        const double sg = (double)(eg + pg[k]) * ig, ssum = (double)(es + ps[k]) * is;
        const double gA = mono_ok(mf, sg, ssum, tg, ts, p) ? split_gain(sg, ssum, tg, ts, p) : -INFINITY;
        const double gB = (ns > 0.0 && mono_ok(mf, sg + ng, ssum + ns, tg, ts, p))
                              ? split_gain(sg + ng, ssum + ns, tg, ts, p) : -INFINITY;
        if (gA > -INFINITY && (gA > best_gain || (gA == best_gain && 2 * t < best_code))) {
          best_gain = gA; best_code = 2 * t; bGL = sg; bSL = ssum;
        }
        if (gB > -INFINITY && (gB > best_gain || (gB == best_gain && 2 * t + 1 < best_code))) {
          best_gain = gB; best_code = 2 * t + 1; bGL = sg + ng; bSL = ssum + ns;
        }
      }
    }
  }
  double bg = best_gain;
  int bc = best_code;
  wave_argmax(bg, bc);
  WaveBest r;
  r.G = tg; r.S = ts;
  r.gain = (bc == 0x7fffffff) ? -INFINITY : bg;
  r.code = bc;
  r.GL = r.SL = 0.0;
  if (bc != 0x7fffffff) {
    // unique owner of the winning threshold broadcasts its left totals
    const unsigned long long own = __ballot(best_code == bc);
    const int src = __builtin_amdgcn_readfirstlane(__ffsll((long long)own) - 1);
    r.GL = readlane_f64(bGL, src);
    r.SL = readlane_f64(bSL, src);
  }
  return r;
}

// Best threshold of (node, f) computed by one wave from the level's built
// histograms (slot, or parent - built sibling); also stores the completed row
// into `full` (parent of the next level) when given.
template <int NBT, bool CAT = false>
__device__ __forceinline__ WaveBest feat_best_wave(const long long* __restrict__ built,
                                                   const long long* __restrict__ parent_full,
                                                   long long* __restrict__ full, const NodeLink& lk, int node, int f,
                                                   const int* __restrict__ nvb,
                                                   const uint8_t* __restrict__ tree_fmask, double ig, double is,
                                                   const SplitParams& p, int gid) {
  constexpr int B = NBT <= 64 ? 1 : NBT / 64;  // bins per lane
  const int lane = threadIdx.x & 63;
  const int64_t per = (int64_t)p.F * 2 * NBT;
  const int64_t off = ((int64_t)f * 2) * NBT;
  const bool allowed = feat_allowed(tree_fmask, p, node, f, gid);
  // last level: no histogram row to keep and the node totals come from
  // feature 0 (node_best reads fbest[node][0]) - nothing to load at all
  if (!allowed && full == nullptr && f != 0) return wave_best_none();
  long long gi[B], si[B];
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int bin = lane * B + k;
    gi[k] = 0; si[k] = 0;
    if (bin < NBT) {
      if (lk.slot >= 0) {
        const long long* bp = built + lk.slot * per + off + bin;
        gi[k] = bp[0]; si[k] = bp[NBT];
      } else {
        const long long* pp = parent_full + lk.parent * per + off + bin;
        const long long* sp = built + lk.sib_slot * per + off + bin;
        gi[k] = pp[0] - sp[0]; si[k] = pp[NBT] - sp[NBT];
      }
      if (full) {
        long long* fp = full + node * per + off + bin;
        fp[0] = gi[k]; fp[NBT] = si[k];
      }
    }
  }
  return feat_scan_wave<NBT, CAT>(gi, si, allowed, node, f, nvb, ig, is, p);
}

__device__ __forceinline__ void store_feat_best(FeatBest* __restrict__ out, int64_t i, const WaveBest& w) {
  FeatBest r{};
  r.gain = w.gain; r.GL = w.GL; r.SL = w.SL;
  r.G = w.G; r.S = w.S;
  r.code = w.code;
  out[i] = r;
}

// K3 tail + K5 fused: one 1024-thread workgroup per (built slot, feature)
// sums that histogram row's workgroup slabs (16-byte loads: LANES slab lanes
// x NBT / 2 bin pairs, 8 loads of a lane in flight), keeps the exact int64
// row in LDS and scans the slot's two nodes right away (wave 0: node 2s,
// wave 1: node 2s + 1 - the children of the s-th splitting node; the unbuilt
// one is parent - built).  The built rows never round-trip through global
// memory and the level drops the split_find launch (hist_reduce + split_find
// were 4.7 + 7.5 us a level at 1.375M rows, mostly fixed cost).
// N ranks run the same single launch with the row exchange inside it
// (reduce_split_p2p_kernel below).

// slab partials of built slot s (pass-local), feature f -> row[2][NBT] (LDS)
template <int NBT>
__device__ __forceinline__ void rs_reduce_row(const unsigned long long* __restrict__ partials, int wgpg, int fg,
                                              int slot_cnt, int s, int f, long long (*red)[NBT / 2][4],
                                              long long (*row)[NBT]) {
  constexpr int PAIRS = NBT / 2, LANES = 1024 / PAIRS;
  const int group = f / fg, fi = f % fg;
  const int64_t hist_elems = (int64_t)slot_cnt * fg * NBT;
  const unsigned long long* src = partials + (int64_t)group * wgpg * hist_elems + ((int64_t)s * fg + fi) * NBT;
  const int t = threadIdx.x, bp = t % PAIRS, c0 = t / PAIRS;
  long long g0 = 0, s0 = 0, g1 = 0, s1 = 0;
  {
    const uint4* q = reinterpret_cast<const uint4*>(src) + bp;
    const int64_t stride = hist_elems / 2;   // uint4 per slab
    int c = c0;
    // 8 slab loads in flight per lane (wgpg is typically 64-256: one or two
    // batches; 16 deep measured slower: 10.4-14.8 vs 8-13 us a level)
    for (; c + 7 * LANES < wgpg; c += 8 * LANES) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = q[(int64_t)(c + k * LANES) * stride];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g0 += (long long)(int32_t)v[k].y; s0 += (long long)v[k].x;
        g1 += (long long)(int32_t)v[k].w; s1 += (long long)v[k].z;
      }
    }
    for (; c < wgpg; c += LANES) {
      const uint4 v = q[(int64_t)c * stride];
      g0 += (long long)(int32_t)v.y; s0 += (long long)v.x;
      g1 += (long long)(int32_t)v.w; s1 += (long long)v.z;
    }
  }
  red[c0][bp][0] = g0; red[c0][bp][1] = s0; red[c0][bp][2] = g1; red[c0][bp][3] = s1;
  __syncthreads();
  if (t < NBT) {
    const int pr = t >> 1, h = (t & 1) * 2;
    long long tg = 0, ts = 0;
#pragma unroll 8
    for (int k = 0; k < LANES; ++k) { tg += red[k][pr][h]; ts += red[k][pr][h + 1]; }
    row[0][t] = tg;
    row[1][t] = ts;
  }
  __syncthreads();
}

// waves 0 / 1 of the block: split scan of the two children of `slot` for
// feature f from the completed built row in LDS.  Returns false for a wave
// without a node (waves >= 2, or a child beyond the level); otherwise `node`
// and its best threshold `w` (every lane holds it).
template <int NBT, bool CAT>
__device__ __forceinline__ bool rs_scan_node(const long long (*row)[NBT], int slot, int f,
                                             const long long* __restrict__ parent_full, long long* __restrict__ full,
                                             const int* __restrict__ ctl, const NodeLink* __restrict__ link,
                                             const int* __restrict__ nvb, const uint8_t* __restrict__ tree_fmask,
                                             const double* __restrict__ qscale, const SplitParams& p, int& node,
                                             WaveBest& w) {
  const int t = threadIdx.x;
  const int wid = t >> 6, lane = t & 63;
  if (wid >= 2) return false;
  const int F = p.F;
  const int n = ctl[CTL_N];
  node = 2 * slot + wid;   // level 0: slot 0 = the root, n = 1
  if (node >= n) return false;
  const NodeLink lk = link[node];
  if (lk.slot != slot && lk.sib_slot != slot) return false;   // (not a child pair: cannot happen)
  const int gid = ctl[CTL_BASE] + node;
  const bool allowed = feat_allowed(tree_fmask, p, node, f, gid);
  if (!allowed && full == nullptr && f != 0) {
    w = wave_best_none();
  } else {
    constexpr int B = NBT <= 64 ? 1 : NBT / 64;
    const int64_t per = (int64_t)F * 2 * NBT;
    const int64_t off = ((int64_t)f * 2) * NBT;
    long long gi[B], si[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
      const int bin = lane * B + k;
      gi[k] = 0; si[k] = 0;
      if (bin < NBT) {
        gi[k] = row[0][bin]; si[k] = row[1][bin];
        if (lk.slot != slot) {
          const long long* pp = parent_full + lk.parent * per + off + bin;
          gi[k] = pp[0] - gi[k]; si[k] = pp[NBT] - si[k];
        }
        if (full) {
          long long* fp = full + node * per + off + bin;
          fp[0] = gi[k]; fp[NBT] = si[k];
        }
      }
    }
    w = feat_scan_wave<NBT, CAT>(gi, si, allowed, node, f, nvb, qscale[2], qscale[3], p);
  }
  return true;
}

// The level finalisation folded into the LAST workgroup of a level's reduce +
// split-scan launch (one launch and one kernel boundary less per level): every
// split record is stored write-through (agent scope, `sc1`), every wave drains
// its stores before the workgroup's ticket (agent-scope atomic), and the
// workgroup whose ticket comes last reads the records with `sc1` loads and runs
// node_best + level_finalize_body - no release / acquire fences (round 5's
// fenced version cost more than the launch it saved,
// profiles/r5/fused_finalize_ab.txt).
struct LevelFin {
  int* ctl_next;
  const float* edges;
  PartInfo* part;
  NodeLink* next_link;
  TreeNode* tree;
  NodeSplit* nsplit;
  int* ticket;          // zeroed once; the last workgroup resets it
  int max_next_nodes;
  int tree_capacity;
};

__device__ __forceinline__ void store_feat_best_wt(FeatBest* __restrict__ out, int64_t i, const WaveBest& w) {
  FeatBest* d = out + i;
  __hip_atomic_store(&d->gain, w.gain, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&d->GL, w.GL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&d->SL, w.SL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&d->G, w.G, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&d->S, w.S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(reinterpret_cast<long long*>(&d->code), (long long)(uint32_t)w.code, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// true (to every thread) in the workgroup whose ticket came last; every wave
// has drained its stores before the ticket
__device__ __forceinline__ bool lf_last_block(int* ticket, int nblocks) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == nblocks - 1;
    if (s_last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last != 0;
}

// (defined after level_finalize_body) MODE 1: records written by this launch's
// workgroups (agent-scope loads); 2: pushed by peer ranks (system-scope loads)
template <int MODE>
__device__ void level_fin_records(const FeatBest* __restrict__ fbest, const int* __restrict__ ctl, const SplitParams& p,
                                  const int* __restrict__ nvb, int nbt, const LevelFin& fin);

template <int NBT, bool CAT, bool FIN = false>
__global__ __launch_bounds__(1024) void reduce_split_kernel(
    const unsigned long long* __restrict__ partials, int wgpg, int fg, int slot_lo, int slot_cnt,
    const long long* __restrict__ parent_full, long long* __restrict__ full, const int* __restrict__ ctl,
    const NodeLink* __restrict__ link, const int* __restrict__ nvb, const uint8_t* __restrict__ tree_fmask,
    const double* __restrict__ qscale, SplitParams p, FeatBest* __restrict__ out, LevelFin fin) {
  __shared__ long long red[1024 / (NBT / 2)][NBT / 2][4];   // 32 KB
  __shared__ long long row[2][NBT];                         // exact (G_q, S_q) of the built slot
  const int s = blockIdx.x, f = blockIdx.y;
  const int slot = slot_lo + s;
  const bool active = slot < ctl[CTL_SLOTS];   // whole workgroup
  if (!FIN && !active) return;
  if (active) {
    rs_reduce_row<NBT>(partials, wgpg, fg, slot_cnt, s, f, red, row);
    int node;
    WaveBest w;
    if (rs_scan_node<NBT, CAT>(row, slot, f, parent_full, full, ctl, link, nvb, tree_fmask, qscale, p, node, w) &&
        (threadIdx.x & 63) == 0) {
      if constexpr (FIN) store_feat_best_wt(out, (int64_t)node * p.F + f, w);
      else store_feat_best(out, (int64_t)node * p.F + f, w);
    }
  }
  if constexpr (FIN) {
    if (lf_last_block(fin.ticket, (int)(gridDim.x * gridDim.y))) level_fin_records<1>(out, ctl, p, nvb, NBT, fin);
  }
}

// ---- N ranks: reduce-scatter by feature + all-gather of the split records ----
// Symmetric-buffer layout of the fused N-rank level (parallel/p2p.py sizes it):
//   [parity 0 | parity 1] (cap bytes each): the histogram rows PUSHED to this
//     rank - rows[slot][f / N][src] of ROW = 2 * NBT int64 for the features
//     f = rank (mod N) this rank owns (the same features at every level, so
//     the parent rows of the next level's sibling subtraction stay local);
//   [split records: parity 0 | parity 1] (cap / 2 bytes each, from 2 * cap):
//     FeatBest[node][F] of the level, all-gathered (every owner pushes its
//     features' records to every rank).
__device__ __forceinline__ FeatBest* p2p_fbest_table(const p2pdev::P2PDesc& d, int r, uint32_t e) {
  return reinterpret_cast<FeatBest*>(static_cast<char*>(d.sym[r]) + 2 * d.cap + (int64_t)(e & 1u) * (d.cap / 2));
}

// lanes 0 .. N-1 each push the record into one rank's table (loopback: lane 0
// into its own); 6 write-through 8-byte words, the pads are never read
__device__ __forceinline__ void p2p_push_feat_best(const p2pdev::P2PDesc& d, uint32_t e, int64_t i, const WaveBest& w,
                                                   int lane) {
  const int nr = d.loopback ? 1 : d.world;
  if (lane >= nr) return;
  FeatBest* dst = p2p_fbest_table(d, d.loopback ? d.rank : lane, e) + i;
  p2pdev::st_sys(&dst->gain, w.gain);
  p2pdev::st_sys(&dst->GL, w.GL);
  p2pdev::st_sys(&dst->SL, w.SL);
  p2pdev::st_sys(&dst->G, w.G);
  p2pdev::st_sys(&dst->S, w.S);
  p2pdev::st_sys(reinterpret_cast<long long*>(&dst->code), (long long)(uint32_t)w.code);
}

// N-rank level in ONE launch (one pass: slot_lo = 0, slot_cnt = the level's
// built slots).  Persistent blocks walk the (slot, feature) items:
//   A. every rank reduces its slabs of EVERY item (its own rows only) and
//      pushes the exact int64 row to the item's owner, rank f % N (write-
//      through stores into the owner's symmetric buffer), then posts;
//   B. the owner waits for block b's posts of every rank, sums the N rows in
//      rank order (local loads: every byte it reads was pushed to it) and
//      runs the split scan of its items only, pushing each record to every
//      rank's split table;
//   C. the launch's last block posts this rank's done word; the level
//      finalisation (node_best_finalize_p2p) waits for every rank's, then
//      reads the all-gathered records.
// So each rank scans 1/N of the level's items, reads no peer memory (the
// cross-rank traffic is posted writes: its rows to their owners, its records
// to every rank), and an N-rank level is hist_build -> reduce_split_p2p ->
// level finalisation, the same three launches as one rank.  Items map to
// blocks identically on every rank (same grid).
// Loopback (one GPU standing in for N ranks; bench.py --loopback-ranks): the
// rows of this rank's features go to source slot 0 and are read N times, the
// other rows to the slots no one reads (the pushes' write traffic); records of the
// features this rank does not own are written as "none" (the same number of
// record writes as a real rank's pushes), so loopback trees split on the
// owned features only - the timing proxy of one rank's share.
template <int NBT, bool CAT, bool FIN = false>
__global__ __launch_bounds__(1024) void reduce_split_p2p_kernel(
    p2pdev::P2PDesc d, const unsigned long long* __restrict__ partials, int wgpg, int fg, int slot_cnt,
    const long long* __restrict__ parent_full, long long* __restrict__ full, const int* __restrict__ ctl,
    const NodeLink* __restrict__ link, const int* __restrict__ nvb, const uint8_t* __restrict__ tree_fmask,
    const double* __restrict__ qscale, SplitParams p, LevelFin fin) {
  __shared__ long long red[1024 / (NBT / 2)][NBT / 2][4];
  __shared__ long long row[2][NBT];
  __shared__ uint32_t s_epoch;
  constexpr int64_t ROW = 2 * NBT;
  const int F = p.F, t = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
  const int N = d.world, FL = (F + N - 1) / N;   // owned-feature slots per rank
  const int items = slot_cnt * F;
  const uint32_t e = p2pdev::begin_epoch(d, &s_epoch);
  const int n_slots = ctl[CTL_SLOTS];
  // A: reduce + push every item's row to its owner
  for (int it = b; it < items; it += nb) {
    const int s = it / F, f = it % F;
    if (s >= n_slots) continue;   // block-uniform
    rs_reduce_row<NBT>(partials, wgpg, fg, slot_cnt, s, f, red, row);
    const int owner = f % N;
    // loopback: every row lands in this rank's own buffer - its own features'
    // rows in source slot 0 (read N times below), the others in slots 1 .. N - 1
    // (never read: the stand-in for the pushes to the other owners)
    const int src = d.loopback ? owner : d.rank;
    long long* dst = reinterpret_cast<long long*>(p2pdev::parity_base(d, d.loopback ? d.rank : owner, e)) +
                     (((int64_t)s * FL + f / N) * N + src) * ROW;
    if (t < NBT) {
      p2pdev::st_sys(dst + t, row[0][t]);
      p2pdev::st_sys(dst + NBT + t, row[1][t]);
    }
    __syncthreads();
  }
  p2pdev::post(d, b, e);
  // B: the owned items of this block
  bool waited = false;
  const long long* mine = reinterpret_cast<const long long*>(p2pdev::parity_base(d, d.rank, e));
  for (int it = b; it < items; it += nb) {
    const int s = it / F, f = it % F;
    if (s >= n_slots) continue;
    if (f % N != d.rank) {
      if (d.loopback && t < 2 * kWave) {   // stand-in for the owners' pushes: "none" records
        const int node = 2 * s + (t >> 6);
        if (node < ctl[CTL_N]) p2p_push_feat_best(d, e, (int64_t)node * F + f, wave_best_none(), t & 63);
      }
      continue;
    }
    if (!waited) {
      p2pdev::wait(d, b, e);
      waited = true;
    }
    if (t < 2 * NBT) {
      // thread t owns (plane t / NBT, bin t % NBT): every rank's value loaded
      // before the rank-order sum
      const long long* base = mine + ((int64_t)s * FL + f / N) * N * ROW + t;
      long long v[p2pdev::kMaxRanks];
#pragma unroll
      for (int r = 0; r < p2pdev::kMaxRanks; ++r) v[r] = r < N ? p2pdev::ld_sys(base + (d.loopback ? 0 : r) * ROW) : 0ll;
      long long acc = v[0];
#pragma unroll
      for (int r = 1; r < p2pdev::kMaxRanks; ++r) acc += v[r];
      row[t / NBT][t % NBT] = acc;
    }
    __syncthreads();
    int node;
    WaveBest w;
    if (rs_scan_node<NBT, CAT>(row, s, f, parent_full, full, ctl, link, nvb, tree_fmask, qscale, p, node, w))
      p2p_push_feat_best(d, e, (int64_t)node * F + f, w, t & 63);
    __syncthreads();
  }
  // C: this rank's records all pushed -> done word to every rank
  const bool last = p2pdev::finish(d, nb, e, true);
  if constexpr (FIN) {
    // the last workgroup waits for every rank's done word, then finalises the
    // level from the all-gathered table (node_best_finalize_p2p in this launch)
    if (last) {
      if (threadIdx.x < kWave) p2pdev::wave_wait(d, d.flags[d.rank] + p2pdev::kDoneBase, e);
      __syncthreads();
      level_fin_records<2>(p2p_fbest_table(d, d.rank, e), ctl, p, nvb, NBT, fin);
    }
  }
}

// K5: best threshold of every (node, feature).  One wave per (node, feature)
// (4 features per 256-thread block, grid = nodes x ceil(F / 4)), each lane
// owning NBT / 64 consecutive bins: the histogram row (built slot, or
// parent - built sibling) is loaded as exact int64, scanned with wave
// shuffles only (no LDS, no block barriers - deep trees run 10^5 nodes per
// level, so per-block latency dominates), converted to fp64 exactly and
// scored for both NA directions.  mtries / column sampling ranks the
// feature's hash among all features with one ballot per 64 features.
template <int NBT, bool CAT>
__global__ __launch_bounds__(256) void split_find_kernel(const long long* __restrict__ built,
                                                         const long long* __restrict__ parent_full,
                                                         long long* __restrict__ full, const int* __restrict__ ctl,
                                                         const NodeLink* __restrict__ link,
                                                         const int* __restrict__ nvb,
                                                         const uint8_t* __restrict__ tree_fmask,
                                                         const double* __restrict__ qscale, SplitParams p,
                                                         FeatBest* __restrict__ out) {
  const int node = blockIdx.x;
  if (node >= ctl[CTL_N]) return;
  const int f = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (f >= p.F) return;  // whole wave
  const NodeLink lk = link[node];
  const WaveBest w = feat_best_wave<NBT, CAT>(built, parent_full, full, lk, node, f, nvb, tree_fmask, qscale[2],
                                              qscale[3], p, ctl[CTL_BASE] + node);
  if ((threadIdx.x & 63) == 0) {
    FeatBest r{};
    r.gain = w.gain; r.GL = w.GL; r.SL = w.SL;
    r.G = w.G; r.S = w.S;
    r.code = w.code;
    out[(int64_t)node * p.F + f] = r;
  }
}

// Per-node arg-max over the features' best thresholds (gain desc, then
// feature / bin / NA-direction asc): one wave per node, lane = feature.
// MODE 0: plain loads (records of an earlier launch); 1: written by other
// workgroups of this launch (agent-scope `sc1` loads); 2: pushed by peer ranks
// (N-rank split table, system-scope loads; p2p_device.h)
template <int MODE>
__device__ __forceinline__ double fb_ld(const double* p) {
  if constexpr (MODE == 2) return p2pdev::ld_sys(p);
  else if constexpr (MODE == 1) return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <int MODE>
__device__ __forceinline__ int fb_code(const FeatBest* r) {
  const uint32_t* c = reinterpret_cast<const uint32_t*>(&r->code);
  if constexpr (MODE == 2) return (int)p2pdev::ld_sys(c);
  else if constexpr (MODE == 1) return (int)__hip_atomic_load(const_cast<uint32_t*>(c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return r->code;
}

template <int SYS = 0>
__device__ __forceinline__ void node_best_wave(const FeatBest* __restrict__ fbest, int F, int node, int lane,
                                               NodeSplit* __restrict__ out) {
  const FeatBest* fb = fbest + (int64_t)node * F;
  double bg = -INFINITY;
  long long key = 0x7fffffffffffffffLL;  // (feature, code) order for ties
  int bf = -1;
  for (int f = lane; f < F; f += 64) {
    const double gn = fb_ld<SYS>(&fb[f].gain);
    const int code = fb_code<SYS>(&fb[f]);
    if (code == 0x7fffffff || !(gn > -INFINITY)) continue;
    const long long k = ((long long)f << 32) | (unsigned)code;
    if (bf < 0 || gn > bg || (gn == bg && k < key)) { bg = gn; key = k; bf = f; }
  }
  wave_argmax_key(bg, key);
  if (lane == 0) {
    NodeSplit s;
    // S is W (mode 0) or H (mode 1); exact leaf (G, H, W) sums come from the
    // partition kernels, these only steer the split decisions
    s.G = fb_ld<SYS>(&fb[0].G); s.H = fb_ld<SYS>(&fb[0].S); s.W = s.H;
    s.pad = 0;
    if (key != 0x7fffffffffffffffLL) {
      const int f = (int)(key >> 32), code = (int)(key & 0xffffffff);
      const FeatBest& c = fb[f];
      s.gain = fb_ld<SYS>(&c.gain); s.GL = fb_ld<SYS>(&c.GL); s.HL = fb_ld<SYS>(&c.SL); s.WL = s.HL;
      s.feat = f; s.bin = code >> 1; s.na_left = code & 1;
    } else {
      s.gain = -INFINITY; s.GL = s.HL = s.WL = 0.0;
      s.feat = -1; s.bin = 0; s.na_left = 0;
    }
    out[node] = s;
  }
}

__global__ __launch_bounds__(64) void node_best_kernel(const FeatBest* __restrict__ fbest,
                                                       const int* __restrict__ ctl, int F,
                                                       NodeSplit* __restrict__ out) {
  const int node = blockIdx.x;
  if (node >= ctl[CTL_N]) return;
  node_best_wave(fbest, F, node, threadIdx.x, out);
}

// ---------------------------------------------------------------------------
// Level finalisation (single workgroup): decide split/leaf per node, number
// the children, pick the smaller child to build, write tree records and the
// partition table.  ctl_next receives the next level's counts.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool lf_decide(const NodeSplit& s, const SplitParams& p) {
  bool do_split = !p.is_last_level && s.feat >= 0 && isfinite(s.gain) && s.gain > 0.0;
  if (do_split && p.mode == 0 && p.min_split_improvement > 0.0) {
    // relative improvement over the node's explained sum of squares
    const double base_term = (s.W > 0.0) ? s.G * s.G / s.W : 0.0;
    do_split = s.gain > p.min_split_improvement * fmax(base_term, 1e-12);
  }
  return do_split;
}

// node i of the level: tree record, partition entry and (split nodes) the
// children's links; k_idx = rank of i among the level's splitting nodes
__device__ __forceinline__ void lf_write_node(int i, const NodeSplit& s, bool do_split, int k_idx, int base,
                                              int next_base, int max_next_nodes, const SplitParams& p,
                                              const float* __restrict__ edges, const int* __restrict__ nvb, int nbt,
                                              PartInfo* __restrict__ part, NodeLink* __restrict__ next_link,
                                              TreeNode* __restrict__ tree, int tree_capacity) {
  if (do_split && 2 * (k_idx + 1) > max_next_nodes) do_split = false;  // capacity guard
  const int gid = base + i;
  const double v = clamp_bound(leaf_value(s.G, s.H, s.W, p), p, gid, tree_capacity);
  PartInfo pi;
  pi.gid = gid;
  pi.leaf_children = 0;
  pi.child_gid = -1;
  pi.pad = 0;
  TreeNode tn;
  tn.value = (float)v;
  tn.weight = (float)s.W;
  tn.gain = do_split ? (float)s.gain : 0.0f;
  if (do_split) {
    pi.feat = s.feat; pi.bin = s.bin; pi.na_left = s.na_left; pi.child = 2 * k_idx;
    tn.feat = s.feat; tn.bin = s.bin; tn.na_left = s.na_left; tn.left = next_base + 2 * k_idx;
    const int m = nvb[s.feat];
    tn.thr = (s.bin < m - 1) ? edges[(int64_t)s.feat * nbt + s.bin] : INFINITY;
    if (p.catf != nullptr && p.catf[s.feat] && gid < tree_capacity) {
      // categorical group split: the (node, feature) scan's left-set bitset
      // becomes the tree's bitset of this node, and the partition record points at it
      const uint32_t* src = p.fbcat + ((int64_t)i * p.F + s.feat) * 8;
      uint32_t* dst = p.treecat + (int64_t)gid * 8;
#pragma unroll
      for (int w = 0; w < 8; ++w) dst[w] = src[w];
      part_set_cat(pi, dst, s.na_left);
      tn.na_left = (s.na_left & 1) | 2;
      tn.thr = __int_as_float(0x7fc00000);   // NaN: not a threshold split
    }
    const bool build_left = s.WL <= (s.W - s.WL);
    NodeLink L, R;
    L.parent = R.parent = i;
    L.pad = R.pad = 0;
    L.slot = build_left ? k_idx : -1;
    L.sib_slot = build_left ? -1 : k_idx;
    R.slot = build_left ? -1 : k_idx;
    R.sib_slot = build_left ? k_idx : -1;
    if (next_link) {
      next_link[2 * k_idx] = L;
      next_link[2 * k_idx + 1] = R;
    }
    pi.pad = (L.slot & 0xFFFF) | (R.slot << 16);  // children's build slots (partition -> slot16)
    pi.child_gid = next_base + 2 * k_idx;
    const int cg = next_base + 2 * k_idx;
    if (p.gbound != nullptr && cg + 1 < tree_capacity) {
      // monotone constraints: children inherit this node's interval; a split on a
      // constrained feature cuts it at the midpoint of the (clipped) child values
      double lo = -INFINITY, hi = INFINITY;
      if (gid > 0 && gid < tree_capacity) { lo = p.gbound[2 * gid]; hi = p.gbound[2 * gid + 1]; }
      double llo = lo, lhi = hi, rlo = lo, rhi = hi;
      const int mf = (int)p.mono[s.feat];
      if (mf != 0) {
        const double wl = fmin(fmax(leaf_value(s.GL, s.HL, s.WL, p), lo), hi);
        const double wr = fmin(fmax(leaf_value(s.G - s.GL, s.H - s.HL, s.W - s.WL, p), lo), hi);
        const double mid = 0.5 * (wl + wr);
        if (mf > 0) { lhi = mid; rlo = mid; } else { llo = mid; rhi = mid; }
      }
      p.gbound[2 * cg] = llo; p.gbound[2 * cg + 1] = lhi;
      p.gbound[2 * cg + 2] = rlo; p.gbound[2 * cg + 3] = rhi;
    }
    if (p.istate != nullptr && cg + 1 < tree_capacity && gid < tree_capacity) inter_children(p, gid, s.feat, cg);
    if (p.children_leaves) {
      // children are final: their totals come from this split's left stats
      pi.leaf_children = 1;
      const double GR = s.G - s.GL, HR = s.H - s.HL, WR = s.W - s.WL;
      TreeNode lc, rc;
      lc.feat = rc.feat = -1;
      lc.bin = rc.bin = 0;
      lc.left = rc.left = -1;
      lc.na_left = rc.na_left = 0;
      lc.thr = rc.thr = 0.0f;
      lc.gain = rc.gain = 0.0f;
      lc.value = (float)clamp_bound(leaf_value(s.GL, s.HL, s.WL, p), p, cg, tree_capacity);
      rc.value = (float)clamp_bound(leaf_value(GR, HR, WR, p), p, cg + 1, tree_capacity);
      lc.weight = (float)s.WL;
      rc.weight = (float)WR;
      if (next_base + 2 * k_idx + 1 < tree_capacity) {
        tree[next_base + 2 * k_idx] = lc;
        tree[next_base + 2 * k_idx + 1] = rc;
      }
    }
  } else {
    pi.feat = -1; pi.bin = 0; pi.na_left = 0; pi.child = -1;
    tn.feat = -1; tn.bin = 0; tn.na_left = 0; tn.left = -1; tn.thr = 0.0f;
  }
  part[i] = pi;
  if (gid < tree_capacity) tree[gid] = tn;
}

__device__ __forceinline__ void lf_write_ctl(int* __restrict__ ctl_next, int ks, int next_base, int max_next_nodes) {
  if (2 * ks > max_next_nodes) ks = max_next_nodes / 2;
  ctl_next[CTL_N] = 2 * ks;
  ctl_next[CTL_SLOTS] = ks;
  ctl_next[CTL_BASE] = next_base;
  ctl_next[CTL_TOTAL] = next_base + 2 * ks;
}

__device__ void level_finalize_body(const NodeSplit* __restrict__ nsplit, const int* __restrict__ ctl,
                                    int* __restrict__ ctl_next, const SplitParams& p, const float* __restrict__ edges,
                                    const int* __restrict__ nvb, int nbt, int max_next_nodes,
                                    PartInfo* __restrict__ part, NodeLink* __restrict__ next_link,
                                    TreeNode* __restrict__ tree, int tree_capacity) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int n = ctl[CTL_N];
  const int base = ctl[CTL_BASE];
  const int next_base = base + n;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += blockDim.x) {
    const int i = c0 + t;
    bool do_split = false;
    NodeSplit s;
    if (i < n) {
      s = nsplit[i];
      do_split = lf_decide(s, p);
    }
    // block exclusive scan of do_split
    const unsigned long long bal = __ballot(do_split);
    const int within = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wid] = __popcll(bal);
    __syncthreads();
    int before = carry;
    for (int k = 0; k < wid; ++k) before += wsum[k];
    if (i < n)
      lf_write_node(i, s, do_split, before + within, base, next_base, max_next_nodes, p, edges, nvb, nbt, part,
                    next_link, tree, tree_capacity);
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) tot += wsum[k];
      carry += tot;
    }
    __syncthreads();
  }
  if (t == 0) lf_write_ctl(ctl_next, carry, next_base, max_next_nodes);
}

// Multi-block level finalisation (levels with tens of thousands of nodes,
// where one workgroup walking the level took ~0.9 ms at depth 19): count the
// splitting nodes per 1024-node tile, scan the tile counts in one small
// workgroup, then every tile numbers its nodes from its prefix.  Same
// decisions and numbering as level_finalize_body.
constexpr int LF_TILE = 1024;
__global__ __launch_bounds__(LF_TILE) void lf_count_kernel(const NodeSplit* __restrict__ nsplit,
                                                           const int* __restrict__ ctl, SplitParams p,
                                                           int* __restrict__ tiles) {
  __shared__ int wsum[16];
  const int n = ctl[CTL_N];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int i = blockIdx.x * LF_TILE + t;
  if (blockIdx.x * LF_TILE >= n) {
    if (t == 0) tiles[blockIdx.x] = 0;
    return;
  }
  const bool do_split = i < n && lf_decide(nsplit[i], p);
  const unsigned long long bal = __ballot(do_split);
  if (lane == 0) wsum[wid] = __popcll(bal);
  __syncthreads();
  if (t == 0) {
    int tot = 0;
    for (int k = 0; k < LF_TILE / 64; ++k) tot += wsum[k];
    tiles[blockIdx.x] = tot;
  }
}

__global__ __launch_bounds__(1024) void lf_scan_kernel(int* __restrict__ tiles, int ntiles, const int* __restrict__ ctl,
                                                       int* __restrict__ ctl_next, int max_next_nodes) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int c0 = 0; c0 < ntiles; c0 += 1024) {
    const int i = c0 + t;
    const int v = i < ntiles ? tiles[i] : 0;
    int x = v;   // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, kWave);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int before = carry;
    for (int k = 0; k < wid; ++k) before += wsum[k];
    if (i < ntiles) tiles[i] = before + x - v;   // exclusive
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int k = 0; k < 16; ++k) tot += wsum[k];
      carry += tot;
    }
    __syncthreads();
  }
  if (t == 0) lf_write_ctl(ctl_next, carry, ctl[CTL_BASE] + ctl[CTL_N], max_next_nodes);
}

__global__ __launch_bounds__(LF_TILE) void lf_write_kernel(const NodeSplit* __restrict__ nsplit,
                                                           const int* __restrict__ ctl, SplitParams p,
                                                           const float* __restrict__ edges,
                                                           const int* __restrict__ nvb, int nbt, int max_next_nodes,
                                                           PartInfo* __restrict__ part,
                                                           NodeLink* __restrict__ next_link,
                                                           TreeNode* __restrict__ tree, int tree_capacity,
                                                           const int* __restrict__ tiles) {
  __shared__ int wsum[16];
  const int n = ctl[CTL_N];
  if (blockIdx.x * LF_TILE >= n) return;
  const int base = ctl[CTL_BASE];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int i = blockIdx.x * LF_TILE + t;
  NodeSplit s;
  bool do_split = false;
  if (i < n) {
    s = nsplit[i];
    do_split = lf_decide(s, p);
  }
  const unsigned long long bal = __ballot(do_split);
  if (lane == 0) wsum[wid] = __popcll(bal);
  __syncthreads();
  int before = tiles[blockIdx.x];
  for (int k = 0; k < wid; ++k) before += wsum[k];
  if (i < n)
    lf_write_node(i, s, do_split, before + __popcll(bal & ((1ull << lane) - 1ull)), base, base + n, max_next_nodes,
                  p, edges, nvb, nbt, part, next_link, tree, tree_capacity);
}

__global__ __launch_bounds__(1024) void level_finalize_kernel(const NodeSplit* __restrict__ nsplit,
                                                              const int* __restrict__ ctl, int* __restrict__ ctl_next,
                                                              SplitParams p, const float* __restrict__ edges,
                                                              const int* __restrict__ nvb, int nbt,
                                                              int max_next_nodes, PartInfo* __restrict__ part,
                                                              NodeLink* __restrict__ next_link,
                                                              TreeNode* __restrict__ tree, int tree_capacity) {
  level_finalize_body(nsplit, ctl, ctl_next, p, edges, nvb, nbt, max_next_nodes, part, next_link, tree,
                      tree_capacity);
}

// Per-node arg-max and level finalisation in ONE single-workgroup launch (the
// 16 waves take the nodes round-robin, then the workgroup finalises): saves a
// dependent launch per level on the scan engine, whose levels hold few nodes.
// The NodeSplit records go through global memory; the workgroup barrier
// (workgroup-scope fence + s_barrier) orders them for the finalising threads.
__global__ __launch_bounds__(1024) void node_best_finalize_kernel(
    const FeatBest* __restrict__ fbest, const int* __restrict__ ctl, int* __restrict__ ctl_next, SplitParams p,
    const float* __restrict__ edges, const int* __restrict__ nvb, int nbt, int max_next_nodes,
    PartInfo* __restrict__ part, NodeLink* __restrict__ next_link, TreeNode* __restrict__ tree, int tree_capacity,
    NodeSplit* __restrict__ nsplit) {
  const int n = ctl[CTL_N];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int node = wid; node < n; node += nw) node_best_wave(fbest, p.F, node, lane, nsplit);
  __syncthreads();
  level_finalize_body(nsplit, ctl, ctl_next, p, edges, nvb, nbt, max_next_nodes, part, next_link, tree,
                      tree_capacity);
}

// N ranks (after reduce_split_p2p): wait for every rank's done word, then the
// same per-node arg-max over the all-gathered split table + finalisation.
// Identical records on every rank -> identical trees.
__global__ __launch_bounds__(1024) void node_best_finalize_p2p_kernel(
    p2pdev::P2PDesc d, const int* __restrict__ ctl, int* __restrict__ ctl_next, SplitParams p,
    const float* __restrict__ edges, const int* __restrict__ nvb, int nbt, int max_next_nodes,
    PartInfo* __restrict__ part, NodeLink* __restrict__ next_link, TreeNode* __restrict__ tree, int tree_capacity,
    NodeSplit* __restrict__ nsplit) {
  __shared__ uint32_t s_epoch;
  const uint32_t e = p2pdev::wait_done(d, &s_epoch);
  const FeatBest* fbest = p2p_fbest_table(d, d.rank, e);
  const int n = ctl[CTL_N];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int node = wid; node < n; node += nw) node_best_wave<2>(fbest, p.F, node, lane, nsplit);
  __syncthreads();
  level_finalize_body(nsplit, ctl, ctl_next, p, edges, nvb, nbt, max_next_nodes, part, next_link, tree,
                      tree_capacity);
}


// K6: route every row to its child, or retire it into its leaf (nid = ~gid).
// Rows retiring at this level add their (g, h, w) to the exact int64 leaf
// sums (every row retires exactly once per tree, so after the last level the
// sums are complete) - this replaces a separate pass over the rows.
// The leaves that can appear at this level have gids in the window
// [base, base + n + n_next) (nodes that stop here, and at the last level the
// children of its splits); their sums are privatised in LDS as R = 8 lane
// copies laid out [slot][copy] (lane l adds into copy l % R: consecutive
// lanes hit consecutive u64; the [copy][slot] layout measured 4.3M LDS
// bank-conflict cycles per last-level dispatch, and 32 conflict-free copies
// cost more occupancy than they saved, profiles/r5/partition_ab.txt).  Each
// workgroup folds its copies and adds the window with integer global atomics
// (order-independent: deterministic).
constexpr int PART_LDS_NODES = 256;   // levels up to this many nodes read their split records from LDS

// Leaf-sum replicas (scan engine): each partition workgroup adds its folded
// leaf window into slice (workgroup mod reps) of leaf_acc = [reps][3 * cap]
// instead of all 1024 workgroups adding into the same ~3 x 63 words (the
// same-address device atomics cost ~15 us of the 65 us final partition at 11M
// rows, profiles/r6/partition_atomics_r6g.txt); the leaf finalisations read the
// sum of the slices.  reps = qs[10] (the host sets it; 1 = one slice).
__device__ __forceinline__ int leaf_reps(const double* __restrict__ qs) {
  const int r = (int)qs[10];
  return r < 1 ? 1 : r;
}
// the slices' loads are issued together (a runtime-count loop waited on each
// load before the next add: 16 serial L2 round trips per sum, ~15 us of the
// one-workgroup leaf_finalize_begin at 16 slices)
constexpr int LEAF_REPS_MAX = 16;
__device__ __forceinline__ long long leaf_sum(const unsigned long long* __restrict__ acc, int64_t i, int reps,
                                              int64_t stride) {
  unsigned long long x[LEAF_REPS_MAX];
#pragma unroll
  for (int r = 0; r < LEAF_REPS_MAX; ++r) x[r] = r < reps ? acc[i + r * stride] : 0ull;
  long long v = 0;
#pragma unroll
  for (int r = 0; r < LEAF_REPS_MAX; ++r) v += (long long)x[r];
  for (int r = LEAF_REPS_MAX; r < reps; ++r) v += (long long)acc[i + r * stride];
  return v;
}
__device__ __forceinline__ void leaf_zero(unsigned long long* __restrict__ acc, int64_t i, int reps, int64_t stride) {
  for (int r = 0; r < reps; ++r) acc[i + r * stride] = 0ull;
}

// NIDM bit 0: nid (input) is an int16 stream, bit 1: nid_out is int16 (fused pipeline)
template <bool PREF, int RPL, int NIDM = 0>
__global__ __launch_bounds__(256) void partition_kernel(const uint8_t* __restrict__ codes, int64_t npad,
                                                        int* nid, const PartInfo* __restrict__ part,
                                                        int nbt, const float* __restrict__ g,
                                                        const float* __restrict__ h, const float* __restrict__ w,
                                                        const double* __restrict__ qs, int cap,
                                                        unsigned long long* __restrict__ leaf_acc,
                                                        const int* __restrict__ ctl_cur,
                                                        const int* __restrict__ ctl_next, int win_max, int R,
                                                        short* __restrict__ slot16, int* nid_out, int all_rows,
                                                        const float* __restrict__ Fm, const float* __restrict__ yv,
                                                        GradParams gp, const uint8_t* __restrict__ y8) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lacc[];
  __shared__ PartInfo ps[PART_LDS_NODES];
  const bool use_lds = leaf_acc != nullptr && win_max > 0;
  // all_rows (final level of the fused-routing pipeline): rows that retired at
  // earlier levels (nid = ~gid) add their sums here too; the LDS window is the
  // whole tree [0, win_max)
  const int base = all_rows ? 0 : ctl_cur[CTL_BASE];
  const int win = use_lds ? (all_rows ? win_max : min(win_max, ctl_cur[CTL_N] + ctl_next[CTL_N])) : 0;
  // the level's split records: LDS-staged when they fit (the node id -> split
  // record -> split code chain then has one dependent global load, not two)
  const int n_cur = ctl_cur[CTL_N];
  const bool rec_lds = n_cur <= PART_LDS_NODES;   // split records staged in LDS
  if (rec_lds)
    for (int j = threadIdx.x; j < n_cur; j += blockDim.x) ps[j] = part[j];
  if (use_lds)
    for (int j = threadIdx.x; j < 3 * win * R; j += blockDim.x) lacc[j] = 0ull;
  __syncthreads();
  const int copy = (threadIdx.x & 63) % R;
  float lg = 0, lh = 0, lw = 0;
  if (leaf_acc) { lg = (float)qs[4]; lh = (float)qs[5]; lw = (float)qs[6]; }
  // RPL rows per lane per step.  All loads of a step are issued before any
  // row is decided: node ids (+ g / h / w on the last level), then - after the
  // split records - the RPL split-code gathers together (unconditionally, at
  // a clamped address), so a step pays the nid -> code chain once, not once
  // per row behind each row's branches
  const int64_t nq = npad / RPL;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r0 = q * RPL;
    int nn[RPL];
    if constexpr (NIDM & 1) {
      static_assert(RPL % 8 == 0, "int16 node ids: 8-row vectors");
#pragma unroll
      for (int v = 0; v < RPL / 8; ++v) {
        const uint4 q4 = *reinterpret_cast<const uint4*>(reinterpret_cast<const short*>(nid) + r0 + 8 * v);
        const uint32_t w4[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) nn[8 * v + k] = (int)(short)(w4[k >> 1] >> (16 * (k & 1)));
      }
    } else {
#pragma unroll
      for (int v = 0; v < RPL / 4; ++v) {
        const int4 na = *reinterpret_cast<int4*>(nid + r0 + 4 * v);
        nn[4 * v] = na.x; nn[4 * v + 1] = na.y; nn[4 * v + 2] = na.z; nn[4 * v + 3] = na.w;
      }
    }
    float gv[RPL], hv[RPL], wv8[RPL];
    if (PREF) {
#pragma unroll
      for (int v = 0; v < RPL / 4; ++v) {
        if (Fm != nullptr) {
          // chained graph steps: boost_update no longer stores (g, h); re-derive
          // them from the margins / labels exactly as it did (unweighted rows)
          const float4 f0 = *reinterpret_cast<const float4*>(Fm + r0 + 4 * v);
          float4 y0;
          if (y8 != nullptr) {
            const uint32_t b4 = *reinterpret_cast<const uint32_t*>(y8 + r0 + 4 * v);
            y0 = make_float4((float)(b4 & 0xff), (float)((b4 >> 8) & 0xff), (float)((b4 >> 16) & 0xff),
                             (float)(b4 >> 24));
          } else {
            y0 = *reinterpret_cast<const float4*>(yv + r0 + 4 * v);
          }
          const float fa[4] = {f0.x, f0.y, f0.z, f0.w}, ya[4] = {y0.x, y0.y, y0.z, y0.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) dist_grad(gp.dist, fa[k], ya[k], gp, gv[4 * v + k], hv[4 * v + k]);
        } else {
          const float4 g0 = *reinterpret_cast<const float4*>(g + r0 + 4 * v);
          const float4 h0 = *reinterpret_cast<const float4*>(h + r0 + 4 * v);
          gv[4 * v] = g0.x; gv[4 * v + 1] = g0.y; gv[4 * v + 2] = g0.z; gv[4 * v + 3] = g0.w;
          hv[4 * v] = h0.x; hv[4 * v + 1] = h0.y; hv[4 * v + 2] = h0.z; hv[4 * v + 3] = h0.w;
        }
        if (w) {
          const float4 w0 = *reinterpret_cast<const float4*>(w + r0 + 4 * v);
          wv8[4 * v] = w0.x; wv8[4 * v + 1] = w0.y; wv8[4 * v + 2] = w0.z; wv8[4 * v + 3] = w0.w;
        } else {
          wv8[4 * v] = wv8[4 * v + 1] = wv8[4 * v + 2] = wv8[4 * v + 3] = 1.0f;
        }
      }
    }
    bool changed = false;
    int sv[RPL];  // next level's build slot per row (-1: retired, or histogram derived from the sibling)
    {
      // every level (the final one too): the RPL split-code gathers are issued
      // together at clamped addresses before any row is decided (the per-row
      // node -> split -> code chain on the final level measured 0.813 vs 0.778
      // ms/tree, profiles/r5/partition_ab.txt)
      PartInfo pi[RPL];
      int bc[RPL];
#pragma unroll
      for (int k = 0; k < RPL; ++k) {
        const int n = nn[k] >= 0 ? nn[k] : 0;   // retired rows / padding: any record, unused
        pi[k] = rec_lds ? ps[n] : part[n];
      }
#pragma unroll
      for (int k = 0; k < RPL; ++k) {
        const int f = (nn[k] >= 0 && pi[k].child >= 0) ? pi[k].feat : 0;
        bc[k] = codes[(int64_t)f * npad + r0 + k];
      }
#pragma unroll
      for (int k = 0; k < RPL; ++k) {
        sv[k] = -1;
        const int n = nn[k];
        int leaf = -1;
        if (n < 0) {
          if (!all_rows) continue;
          leaf = ~n;  // retired earlier (padding: INT_MIN -> beyond cap, no sums)
        } else {
          changed = true;
          const PartInfo& p = pi[k];
          if (p.child < 0) {
            leaf = p.gid;
          } else {
            const int b = bc[k];
            const int right = part_right(p, b, nbt);
            if (p.leaf_children) {
              leaf = p.child_gid + right;
            } else {
              nn[k] = p.child + right;
              sv[k] = right ? (p.pad >> 16) : (int)(short)(p.pad & 0xFFFF);
            }
          }
          if (leaf >= 0) nn[k] = ~leaf;
        }
        if (leaf >= 0 && leaf_acc && leaf < cap) {
          const float wv = PREF ? wv8[k] : (w ? w[r0 + k] : 1.0f);
          if (wv != 0.0f) {
            const float gk = PREF ? gv[k] : g[r0 + k], hk = PREF ? hv[k] : h[r0 + k];
            const unsigned long long a = (unsigned long long)(long long)__float2int_rn(gk * lg);
            const unsigned long long b = (unsigned long long)(long long)__float2int_rn(hk * lh);
            const unsigned long long c = (unsigned long long)(long long)__float2int_rn(wv * lw);
            const int li = leaf - base;
            // separate call sites keep LDS atomics as ds_add_u64 (a pointer
            // selected between LDS and global memory would become FLAT)
            if (li >= 0 && li < win) {
              unsigned long long* d = lacc + (3 * li) * R + copy;
              atomicAdd(d, a);
              atomicAdd(d + R, b);
              atomicAdd(d + 2 * R, c);
            } else {
              atomicAdd(leaf_acc + 3 * leaf + 0, a);
              atomicAdd(leaf_acc + 3 * leaf + 1, b);
              atomicAdd(leaf_acc + 3 * leaf + 2, c);
            }
          }
        }
      }
    }
    if (changed || nid_out != nid) {
      if constexpr (NIDM & 2) {
#pragma unroll
        for (int v = 0; v < RPL / 8; ++v) {
          uint32_t w4[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            w4[k] = ((uint32_t)(uint16_t)max(nn[8 * v + 2 * k], -32768)) |
                    ((uint32_t)(uint16_t)max(nn[8 * v + 2 * k + 1], -32768) << 16);
          *reinterpret_cast<uint4*>(reinterpret_cast<short*>(nid_out) + r0 + 8 * v) =
              make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
      } else {
#pragma unroll
        for (int v = 0; v < RPL / 4; ++v)
          *reinterpret_cast<int4*>(nid_out + r0 + 4 * v) =
              make_int4(nn[4 * v], nn[4 * v + 1], nn[4 * v + 2], nn[4 * v + 3]);
      }
    }
    if (slot16) {  // every row, so rows outside the tree read -1 on the next level
#pragma unroll
      for (int v = 0; v < RPL / 8; ++v)
        *reinterpret_cast<int4*>(slot16 + r0 + 8 * v) =
            make_int4((sv[8 * v] & 0xFFFF) | (sv[8 * v + 1] << 16), (sv[8 * v + 2] & 0xFFFF) | (sv[8 * v + 3] << 16),
                      (sv[8 * v + 4] & 0xFFFF) | (sv[8 * v + 5] << 16), (sv[8 * v + 6] & 0xFFFF) | (sv[8 * v + 7] << 16));
    }
  }
  if (use_lds) {
    // this workgroup's replica slice of the leaf sums
    const int64_t rep_off = (int64_t)(blockIdx.x % leaf_reps(qs)) * 3 * cap;
    __syncthreads();
    // fold the R copies: thread t sums slot t's copies starting at copy t mod R
    // (rotated so the threads of a lane group hit different banks; a shuffle
    // butterfly over consecutive copies measured 168 vs 100 us per final level)
    {
      for (int t = threadIdx.x; t < 3 * win; t += blockDim.x) {
        unsigned long long v = 0ull;
        for (int c = 0; c < R; ++c) v += lacc[t * R + ((c + t) & (R - 1))];
        if (v && base + t / 3 < cap) atomicAdd(leaf_acc + rep_off + 3 * base + t, v);
      }
    }
  }
}

// leaf_acc[j] += sum over the partition slabs (one 256-thread block per j).
__global__ __launch_bounds__(256) void leaf_reduce_kernel(const unsigned long long* __restrict__ slab, int n_slabs,
                                                          int width, unsigned long long* __restrict__ leaf_acc) {
  __shared__ unsigned long long red[256];
  const int j = blockIdx.x;
  unsigned long long v = 0ull;
  for (int s = threadIdx.x; s < n_slabs; s += blockDim.x) v += slab[(int64_t)s * width + j];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0 && red[0]) leaf_acc[j] += red[0];
}

// ---------------------------------------------------------------------------
// K2 + K7: apply the finished tree to the margins and compute the next
// tree's gradients, bagging weights and reset the row->node ids, fused in
// one pass over the rows.
// dist: 0 gaussian, 1 bernoulli, 2 poisson, 3 gamma, 4 tweedie, 5 laplace,
//       6 quantile, 7 huber, 8 drf (g = -y, h = 1)
// ---------------------------------------------------------------------------



// Block-level max of three non-negative statistics, written (no atomics) to
// this block's slot of a fixed-size slab; stat_reduce folds the slab.
constexpr int STAT_BLOCKS = 4096;

__device__ __forceinline__ void block_max3(float a, float b, float c, unsigned int* __restrict__ stat_slab) {
  __shared__ float red[3][16];
  a = wave_max(a); b = wave_max(b); c = wave_max(c);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = a; red[1][wid] = b; red[2][wid] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    float m0 = 0.f, m1 = 0.f, m2 = 0.f;
    for (int k = 0; k < nw; ++k) { m0 = fmaxf(m0, red[0][k]); m1 = fmaxf(m1, red[1][k]); m2 = fmaxf(m2, red[2][k]); }
    unsigned int* o = stat_slab + 4 * blockIdx.x;
    o[0] = __float_as_uint(m0); o[1] = __float_as_uint(m1); o[2] = __float_as_uint(m2); o[3] = 0u;
  }
}

__global__ __launch_bounds__(256) void boost_update_kernel(float* __restrict__ F, const float* __restrict__ y,
                                                           const float* __restrict__ wobs, int64_t n, int64_t npad,
                                                           int* __restrict__ nid, const TreeNode* __restrict__ tree,
                                                           GradParams gp, float* __restrict__ g, float* __restrict__ h,
                                                           float* __restrict__ wout, unsigned int* __restrict__ stat_max,
                                                           const uint4* __restrict__ arch_src, int arch_n16,
                                                           uint4* __restrict__ ring, int ring_n,
                                                           const int* __restrict__ tree_ctr, int ctr_off,
                                                           uint32_t* __restrict__ pk32_out,
                                                           const double* __restrict__ qs, int s_is_h, int store_gh,
                                                           const uint8_t* __restrict__ y8,
                                                           const short* __restrict__ nid16) {
  if (ring != nullptr) {
    // graph replay: the applied tree also goes to ring slot (tree_ctr - ctr_off)
    // mod ring_n (tree_archive folded into this launch)
    const int slot = (int)(((unsigned)(tree_ctr[0] - ctr_off)) % (unsigned)ring_n);
    uint4* dst = ring + (int64_t)slot * arch_n16;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < arch_n16; i += gridDim.x * blockDim.x) dst[i] = arch_src[i];
  }
  float mg = 0.f, mh = 0.f, mw = 0.f;
  const int64_t nq = npad / 4;  // 4 rows per lane, 16-byte accesses
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r0 = 4 * q;
    float4 f4 = *reinterpret_cast<const float4*>(F + r0);
    float4 y4;
    if (y8 != nullptr) {   // 0 / 1 labels as bytes (a quarter of the label traffic)
      const uint32_t b4 = *reinterpret_cast<const uint32_t*>(y8 + r0);
      y4 = make_float4((float)(b4 & 0xff), (float)((b4 >> 8) & 0xff), (float)((b4 >> 16) & 0xff), (float)(b4 >> 24));
    } else {
      y4 = *reinterpret_cast<const float4*>(y + r0);
    }
    float4 w4 = make_float4(1.f, 1.f, 1.f, 1.f);
    if (wobs) w4 = *reinterpret_cast<const float4*>(wobs + r0);
    int4 n4 = make_int4(0, 0, 0, 0);
    if (gp.apply_tree) {
      if (nid16 != nullptr) {   // int16 leaf ids (fused pipeline graph steps)
        const uint2 v = *reinterpret_cast<const uint2*>(nid16 + r0);
        n4 = make_int4((int)(short)(v.x & 0xffff), (int)(short)(v.x >> 16), (int)(short)(v.y & 0xffff),
                       (int)(short)(v.y >> 16));
      } else {
        n4 = *reinterpret_cast<const int4*>(nid + r0);
      }
    }
    float fv[4] = {f4.x, f4.y, f4.z, f4.w}, yv[4] = {y4.x, y4.y, y4.z, y4.w}, wv[4] = {w4.x, w4.y, w4.z, w4.w};
    const int nv[4] = {n4.x, n4.y, n4.z, n4.w};
    float gv[4], hv[4];
    int nn[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t r = r0 + k;
      if (r >= n) {
        nn[k] = INT32_MIN; gv[k] = 0.f; hv[k] = 0.f; wv[k] = 0.f;
        continue;
      }
      if (gp.apply_tree) fv[k] += tree[~nv[k]].value;
      dist_grad(gp.dist, fv[k], yv[k], gp, gv[k], hv[k]);
      if (gp.sample_rate < 1.0f) {
        const float u = u01(hash4(gp.seed, (uint32_t)gp.tree_index, (uint32_t)(r + gp.row_base), 0x5bd1e995u));
        if (u >= gp.sample_rate) wv[k] = 0.0f;
      }
      gv[k] *= wv[k];
      hv[k] *= wv[k];
      nn[k] = 0;
      mg = fmaxf(mg, fabsf(gv[k])); mh = fmaxf(mh, hv[k]); mw = fmaxf(mw, wv[k]);
    }
    if (pk32_out != nullptr) {
      // the next tree's level-0 rows, quantised exactly as hist_build does it
      // (scales and dither salt of that tree: its begin already ran)
      const float sg = (float)qs[0], ss = (float)qs[1];
      const uint32_t salt = (uint32_t)qs[9];
      const int64_t rb = (int64_t)qs[7];
      uint32_t pw[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t hsh = row_hash(rb + r0 + k, salt);
        const float d1 = (hsh & 0xFFFF) * (1.0f / 65536.0f), d2 = (hsh >> 16) * (1.0f / 65536.0f);
        const float sv = s_is_h ? hv[k] : wv[k];
        const int gq = (int)floorf(fmaf(gv[k], sg, d1));
        const uint32_t sq = (uint32_t)floorf(fmaf(sv, ss, d2));
        pw[k] = ((uint32_t)gq << 16) | (sq & 0xFFFFu);
      }
      *reinterpret_cast<uint4*>(pk32_out + r0) = make_uint4(pw[0], pw[1], pw[2], pw[3]);
    }
    if (gp.apply_tree) *reinterpret_cast<float4*>(F + r0) = make_float4(fv[0], fv[1], fv[2], fv[3]);
    if (store_gh) {   // (chained graph steps: the final partition re-derives them)
      *reinterpret_cast<float4*>(g + r0) = make_float4(gv[0], gv[1], gv[2], gv[3]);
      *reinterpret_cast<float4*>(h + r0) = make_float4(hv[0], hv[1], hv[2], hv[3]);
    }
    if (wout) *reinterpret_cast<float4*>(wout + r0) = make_float4(wv[0], wv[1], wv[2], wv[3]);
    if (!gp.skip_nid) *reinterpret_cast<int4*>(nid + r0) = make_int4(nn[0], nn[1], nn[2], nn[3]);
  }
  if (stat_max) block_max3(mg, mh, mw, stat_max);
}

// Apply a finished tree only (multi-class path): F[k][r] += value[leaf].
__global__ __launch_bounds__(256) void apply_tree_kernel(float* __restrict__ F, int64_t n,
                                                         const int* __restrict__ nid,
                                                         const TreeNode* __restrict__ tree) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  F[r] += tree[~nid[r]].value;
}

// DRF out-of-bag accumulation: after tree t (class k) is built, every row
// that tree t's bag left out (same hash as boost_update's bagging) adds the
// value of the leaf it fell into (nid = ~leaf gid) to oob_sum and, for the
// first class, counts the tree in oob_cnt.  H2O DRF reports its training
// metrics on these out-of-bag predictions.
__global__ __launch_bounds__(256) void oob_accumulate_kernel(float* __restrict__ oob_sum,
                                                             float* __restrict__ oob_cnt, int64_t n,
                                                             const int* __restrict__ nid,
                                                             const TreeNode* __restrict__ tree,
                                                             const float* __restrict__ wobs, uint32_t seed,
                                                             uint32_t tree_index, float sample_rate,
                                                             int64_t row_base, int count) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const float u = u01(hash4(seed, tree_index, (uint32_t)(r + row_base), 0x5bd1e995u));
    if (u < sample_rate) continue;                       // in the bag of this tree
    if (wobs && wobs[r] == 0.0f) continue;
    const int leaf = ~nid[r];
    if (leaf < 0) continue;
    oob_sum[r] += tree[leaf].value;
    if (count) oob_cnt[r] += 1.0f;
  }
}

// Multinomial softmax gradients for class k plus bagging / nid reset.
__global__ __launch_bounds__(256) void softmax_grad_kernel(const float* __restrict__ F, int K, int64_t ldF,
                                                           const int* __restrict__ yk, const float* __restrict__ wobs,
                                                           int64_t n, int64_t npad, int cls, GradParams gp,
                                                           int* __restrict__ nid, float* __restrict__ g,
                                                           float* __restrict__ h, float* __restrict__ wout,
                                                           unsigned int* __restrict__ stat_max) {
  float mg = 0.f, mh = 0.f, mw = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < npad; r += (int64_t)gridDim.x * blockDim.x) {
    if (r >= n) {
      nid[r] = INT32_MIN; g[r] = 0.f; h[r] = 0.f;
      if (wout) wout[r] = 0.f;
      continue;
    }
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, F[k * ldF + r]);
    float den = 0.f, fk = 0.f;
    for (int k = 0; k < K; ++k) {
      const float e = __expf(F[k * ldF + r] - mx);
      den += e;
      if (k == cls) fk = e;
    }
    const float pk = fk / den;
    const float yv = (yk[r] == cls) ? 1.0f : 0.0f;
    float wv = wobs ? wobs[r] : 1.0f;
    if (gp.sample_rate < 1.0f) {
      const float u = u01(hash4(gp.seed, (uint32_t)gp.tree_index, (uint32_t)(r + gp.row_base), 0x5bd1e995u));
      if (u >= gp.sample_rate) wv = 0.0f;
    }
    const float gv = (pk - yv) * wv, hv = fmaxf(pk * (1.0f - pk), 1e-16f) * wv;
    g[r] = gv;
    h[r] = hv;
    if (wout) wout[r] = wv;
    nid[r] = 0;
    mg = fmaxf(mg, fabsf(gv)); mh = fmaxf(mh, hv); mw = fmaxf(mw, wv);
  }
  if (stat_max) block_max3(mg, mh, mw, stat_max);
}

// Turn the (all-reduced) per-tree maxima into quantisation scales.
// Fold the per-block maxima slab into stat_max (uint32 float bits).
__global__ __launch_bounds__(1024) void stat_reduce_kernel(const unsigned int* __restrict__ slab, int n,
                                                          unsigned int* __restrict__ stat_max) {
  __shared__ unsigned int red[3][16];
  unsigned int m0 = 0, m1 = 0, m2 = 0;  // non-negative float bits order like the floats
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    m0 = max(m0, slab[4 * i]); m1 = max(m1, slab[4 * i + 1]); m2 = max(m2, slab[4 * i + 2]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    m0 = max(m0, (unsigned)__shfl_xor((int)m0, off, kWave));
    m1 = max(m1, (unsigned)__shfl_xor((int)m1, off, kWave));
    m2 = max(m2, (unsigned)__shfl_xor((int)m2, off, kWave));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = m0; red[1][wid] = m1; red[2][wid] = m2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      m0 = max(m0, red[0][k]); m1 = max(m1, red[1][k]); m2 = max(m2, red[2][k]);
    }
    m0 = max(m0, red[0][0]); m1 = max(m1, red[1][0]); m2 = max(m2, red[2][0]);
    stat_max[0] = m0; stat_max[1] = m1; stat_max[2] = m2; stat_max[3] = 0u;
  }
}

// Start of a tree: quantisation scales from the (all-reduced) maxima, level-0
// control block / link, and zeroed leaf sums - one launch instead of five.
// qg / qsr: per-row fixed-point ranges chosen by the host from the largest
// workgroup chunk of the tree's level plans (<= QG / QS): smaller chunks give
// proportionally finer quantisation.
__device__ void tree_begin_scales(const unsigned int* __restrict__ stat_max, int mode, double qg, double qsr,
                                  double* __restrict__ qs, int* __restrict__ ctl0, NodeLink* __restrict__ link0,
                                  long long row_base, int tree_index, int* __restrict__ tree_ctr) {
  // dither salt of this tree: the host's tree index, or (captured / replayed
  // trees) a device counter that advances once per tree
  int ti = tree_index;
  if (tree_ctr != nullptr) { ti = tree_ctr[0]; tree_ctr[0] = ti + 1; }
  qs[9] = (double)(ti & 0x7FFFFFFF);
  const double gmax = fmax((double)__uint_as_float(stat_max[0]), 1e-30);
  const double hmax = fmax((double)__uint_as_float(stat_max[1]), 1e-30);
  const double wmax = fmax((double)__uint_as_float(stat_max[2]), 1e-30);
  const double smax = (mode == 0) ? wmax : hmax;
  // power-of-two scales keep the double conversions exact
  const double sg = exp2(floor(log2(fmin(qg, (double)QG) / gmax)));
  const double ss = exp2(floor(log2(fmin(qsr, (double)QS) / smax)));
  qs[0] = sg; qs[1] = ss; qs[2] = 1.0 / sg; qs[3] = 1.0 / ss;
  // leaf sums: |per-row value| < 2^30 so int32 conversions suffice
  qs[4] = exp2(floor(log2(1073741823.0 / gmax)));
  qs[5] = exp2(floor(log2(1073741823.0 / hmax)));
  qs[6] = exp2(floor(log2(1073741823.0 / wmax)));
  qs[7] = (double)row_base;  // exact below 2^53
  ctl0[CTL_N] = 1; ctl0[CTL_SLOTS] = 1; ctl0[CTL_BASE] = 0; ctl0[CTL_TOTAL] = 1;
  NodeLink root;
  root.slot = 0; root.sib_slot = -1; root.parent = -1; root.pad = 0;
  link0[0] = root;
}

__global__ __launch_bounds__(256) void tree_begin_kernel(const unsigned int* __restrict__ stat_max, int mode,
                                                         double qg, double qsr, double* __restrict__ qs,
                                                         int* __restrict__ ctl0, NodeLink* __restrict__ link0,
                                                         unsigned long long* __restrict__ leaf_acc, int leaf_n,
                                                         long long row_base, int tree_index, int* __restrict__ tree_ctr) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < leaf_n; i += gridDim.x * blockDim.x) leaf_acc[i] = 0ull;
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  tree_begin_scales(stat_max, mode, qg, qsr, qs, ctl0, link0, row_base, tree_index, tree_ctr);
}

// Exact per-leaf (G, H, W) sums after the last partition: every row carries
// nid = ~leaf_gid.  int64 fixed point -> deterministic; LDS-privatised when
// the tree capacity fits (depth <= 10), global atomics otherwise.
__global__ __launch_bounds__(256) void leaf_stats_kernel(const int* __restrict__ nid, const float* __restrict__ g,
                                                         const float* __restrict__ h, const float* __restrict__ w,
                                                         int64_t n, const double* __restrict__ qs, int cap,
                                                         unsigned long long* __restrict__ acc) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lacc[];
  const bool use_lds = cap <= 2048;
  if (use_lds) {
    for (int j = threadIdx.x; j < 3 * cap; j += blockDim.x) lacc[j] = 0ull;
    __syncthreads();
  }
  const double lg = qs[4], lh = qs[5], lw = qs[6];
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int leaf = ~nid[r];
    if (leaf < 0 || leaf >= cap) continue;
    const float wv = w ? w[r] : 1.0f;
    if (wv == 0.0f) continue;
    const long long gq = __float2int_rn(g[r] * (float)lg), hq = __float2int_rn(h[r] * (float)lh),
                    wq = __float2int_rn(wv * (float)lw);
    if (use_lds) {  // separate call sites keep ds_add_u64 (see partition_kernel)
      atomicAdd(lacc + 3 * leaf + 0, (unsigned long long)gq);
      atomicAdd(lacc + 3 * leaf + 1, (unsigned long long)hq);
      atomicAdd(lacc + 3 * leaf + 2, (unsigned long long)wq);
    } else {
      atomicAdd(acc + 3 * leaf + 0, (unsigned long long)gq);
      atomicAdd(acc + 3 * leaf + 1, (unsigned long long)hq);
      atomicAdd(acc + 3 * leaf + 2, (unsigned long long)wq);
    }
  }
  if (use_lds) {
    __syncthreads();
    for (int j = threadIdx.x; j < 3 * cap; j += blockDim.x)
      if (lacc[j]) atomicAdd(acc + j, lacc[j]);
  }
}

// Overwrite every leaf's value with the Newton / mean step from the exact
// leaf sums (and record its weight).
__global__ __launch_bounds__(256) void leaf_finalize_kernel(const unsigned long long* __restrict__ acc,
                                                            const int* __restrict__ ctl_final,
                                                            const double* __restrict__ qs, SplitParams p,
                                                            TreeNode* __restrict__ tree, int cap) {
  const int total = min(ctl_final[CTL_TOTAL], cap);
  const int reps = leaf_reps(qs);
  const int64_t st = 3 * (int64_t)cap;
  for (int gid = blockIdx.x * blockDim.x + threadIdx.x; gid < total; gid += gridDim.x * blockDim.x) {
    TreeNode nd = tree[gid];
    const double G = (double)leaf_sum(acc, 3 * gid, reps, st) / qs[4];
    const double H = (double)leaf_sum(acc, 3 * gid + 1, reps, st) / qs[5];
    const double W = (double)leaf_sum(acc, 3 * gid + 2, reps, st) / qs[6];
    if (nd.feat < 0) {
      nd.value = (float)clamp_bound(leaf_value(G, H, W, p), p, gid, cap);
      nd.weight = (float)W;
      tree[gid] = nd;
    }
  }
}

// Graph replay with fixed gradient bounds: leaf_finalize, then (same
// workgroup, after every leaf sum was read) the NEXT tree's tree_begin - the
// leaf sums it read are zeroed (only [0, 3 * total) was written this tree,
// so the whole buffer is zero again), scales / level-0 control / root link
// set and the tree counter advanced.  Saves the tree_begin launch per tree.
__global__ __launch_bounds__(1024) void leaf_finalize_begin_kernel(
    unsigned long long* __restrict__ acc, const int* __restrict__ ctl_final, double* __restrict__ qs, SplitParams p,
    TreeNode* __restrict__ tree, int cap, const unsigned int* __restrict__ stat_max, int mode, double qg, double qsr,
    int* __restrict__ ctl0, NodeLink* __restrict__ link0, long long row_base, int* __restrict__ tree_ctr) {
  const int total = min(ctl_final[CTL_TOTAL], cap);
  const double s4 = qs[4], s5 = qs[5], s6 = qs[6];
  const int reps = leaf_reps(qs);
  const int64_t st = 3 * (int64_t)cap;
  for (int gid = threadIdx.x; gid < total; gid += blockDim.x) {
    const long long ag = leaf_sum(acc, 3 * gid, reps, st), ah = leaf_sum(acc, 3 * gid + 1, reps, st),
                    aw = leaf_sum(acc, 3 * gid + 2, reps, st);
#pragma unroll
    for (int k = 0; k < 3; ++k) leaf_zero(acc, 3 * gid + k, reps, st);
    TreeNode nd = tree[gid];
    if (nd.feat < 0) {
      const double G = (double)ag / s4, H = (double)ah / s5, W = (double)aw / s6;
      nd.value = (float)clamp_bound(leaf_value(G, H, W, p), p, gid, cap);
      nd.weight = (float)W;
      tree[gid] = nd;
    }
  }
  __syncthreads();   // ctl_final may be ctl0 (even depth); qs read above
  if (threadIdx.x == 0) tree_begin_scales(stat_max, mode, qg, qsr, qs, ctl0, link0, row_base, 0, tree_ctr);
}

// N ranks: the exact leaf sums exchanged inside the leaf finalisation.  Block
// b owns the leaves gid = 256 * (b + k * nb) + [0, 256): it pushes this rank's
// (G, H, W) sums of those leaves into slot `rank` of every rank's symmetric
// buffer (write-through; loopback: its own slot 0 only), posts, waits for
// every rank's block b, sums the N copies in rank order (local loads, exact
// int64) and writes the leaf values - so no rank reads peer memory and the
// exchange is spread over the grid.  With `begin` the sums are zeroed after
// the read and the launch's last block (finish ticket: every block has read
// qs and ctl_final) runs the chained next tree's tree_begin exactly as
// leaf_finalize_begin_kernel.  The tree's leaf all-reduce is no separate launch.
constexpr int LEAF_P2P_THREADS = 256;
__global__ __launch_bounds__(LEAF_P2P_THREADS) void leaf_finalize_p2p_kernel(
    p2pdev::P2PDesc d, unsigned long long* __restrict__ acc, const int* __restrict__ ctl_final,
    double* __restrict__ qs, SplitParams p, TreeNode* __restrict__ tree, int cap, int begin,
    const unsigned int* __restrict__ stat_max, int mode, double qg, double qsr, int* __restrict__ ctl0,
    NodeLink* __restrict__ link0, long long row_base, int* __restrict__ tree_ctr) {
  __shared__ uint32_t s_epoch;
  const uint32_t e = p2pdev::begin_epoch(d, &s_epoch);
  const int total = min(ctl_final[CTL_TOTAL], cap);
  const int b = blockIdx.x, nb = gridDim.x, t = threadIdx.x;
  const int64_t per_src = 3 * (int64_t)cap;   // one rank's sums in the receiving buffer
  const int src = d.loopback ? 0 : d.rank;
  const int nr = d.loopback ? 1 : d.world;
  const int reps = leaf_reps(qs);
  const int64_t st = 3 * (int64_t)cap;
  for (int c = b; c * LEAF_P2P_THREADS < total; c += nb) {
    const int gid = c * LEAF_P2P_THREADS + t;
    if (gid < total)
      for (int r = 0; r < nr; ++r) {
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(
                                      p2pdev::parity_base(d, d.loopback ? d.rank : r, e)) + src * per_src + 3 * gid;
#pragma unroll
        for (int k = 0; k < 3; ++k) p2pdev::st_sys(dst + k, (unsigned long long)leaf_sum(acc, 3 * gid + k, reps, st));
      }
  }
  p2pdev::post_wait(d, b, e);
  const double s4 = qs[4], s5 = qs[5], s6 = qs[6];
  const unsigned long long* mine = reinterpret_cast<const unsigned long long*>(p2pdev::parity_base(d, d.rank, e));
  for (int c = b; c * LEAF_P2P_THREADS < total; c += nb) {
    const int gid = c * LEAF_P2P_THREADS + t;
    if (gid >= total) continue;
    long long a3[3] = {0, 0, 0};
    for (int r = 0; r < d.world; ++r) {
      const unsigned long long* sr = mine + (d.loopback ? 0 : r) * per_src + 3 * gid;
#pragma unroll
      for (int k = 0; k < 3; ++k) a3[k] += (long long)p2pdev::ld_sys(sr + k);
    }
    // chained: the sums are zeroed for the next tree; otherwise they keep the
    // GLOBAL sums, as after the all-reduce path (a later reader of leaf_acc sees
    // the same values on every rank)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      leaf_zero(acc, 3 * gid + k, reps, st);
      if (!begin) acc[3 * gid + k] = (unsigned long long)a3[k];
    }
    TreeNode nd = tree[gid];
    if (nd.feat < 0) {
      const double G = (double)a3[0] / s4, H = (double)a3[1] / s5, W = (double)a3[2] / s6;
      nd.value = (float)clamp_bound(leaf_value(G, H, W, p), p, gid, cap);
      nd.weight = (float)W;
      tree[gid] = nd;
    }
  }
  // (drains and block barrier first: qs and ctl_final read above)
  const bool last = p2pdev::finish(d, nb, e);
  if (begin && last && threadIdx.x == 0)
    tree_begin_scales(stat_max, mode, qg, qsr, qs, ctl0, link0, row_base, 0, tree_ctr);
}

// Monotone constraints with H2O's squared-error splits (mode 0) and Newton
// leaves (leaf_mode 0): the histograms carry (G, W), so the node intervals the
// level finalisation cut at W-scale midpoints (-G/W) are on the wrong scale for
// Newton leaf values (-G/H; bernoulli H <= W / 4).  After the leaf sums are
// exact this one-workgroup pass re-derives every interval on the leaf scale,
// as H2O's gamma-based bounds do: depth of each reachable node (top-down),
// subtree (G, H) sums (bottom-up), then [lo, hi] cut at the midpoint of the
// clipped Newton child values (top-down), and every leaf is clamped into its
// interval.  scratch: int dep[cap] | double SG[cap], SH[cap], LO[cap], HI[cap].
__global__ __launch_bounds__(1024) void mono_newton_kernel(const unsigned long long* __restrict__ acc,
                                                           const int* __restrict__ ctl_final,
                                                           const double* __restrict__ qs, SplitParams p,
                                                           TreeNode* __restrict__ tree, int cap, char* scratch) {
  const int total = min(ctl_final[CTL_TOTAL], cap);
  int* dep = reinterpret_cast<int*>(scratch);
  double* SG = reinterpret_cast<double*>(scratch + (((int64_t)cap * 4 + 15) / 16) * 16);
  double* SH = SG + cap;
  double* LO = SH + cap;
  double* HI = LO + cap;
  __shared__ int s_any;
  for (int i = threadIdx.x; i < total; i += blockDim.x) dep[i] = (i == 0) ? 0 : -1;
  __syncthreads();
  int maxd = 0;
  for (int d = 0;; ++d) {
    if (threadIdx.x == 0) s_any = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      if (dep[i] != d) continue;
      const TreeNode nd = tree[i];
      if (nd.feat >= 0 && nd.left > 0 && nd.left + 1 < total) {
        dep[nd.left] = d + 1;
        dep[nd.left + 1] = d + 1;
        s_any = 1;
      }
    }
    __syncthreads();
    const int any = s_any;
    __syncthreads();
    if (!any) { maxd = d; break; }
  }
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    if (dep[i] >= 0 && tree[i].feat < 0) {
      SG[i] = (double)leaf_sum(acc, 3 * i, leaf_reps(qs), 3 * (int64_t)cap) / qs[4];
      SH[i] = (double)leaf_sum(acc, 3 * i + 1, leaf_reps(qs), 3 * (int64_t)cap) / qs[5];
    }
  }
  __syncthreads();
  for (int d = maxd - 1; d >= 0; --d) {
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      if (dep[i] != d) continue;
      const TreeNode nd = tree[i];
      if (nd.feat >= 0) {
        SG[i] = SG[nd.left] + SG[nd.left + 1];
        SH[i] = SH[nd.left] + SH[nd.left + 1];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { LO[0] = -INFINITY; HI[0] = INFINITY; }
  __syncthreads();
  for (int d = 0; d <= maxd; ++d) {
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      if (dep[i] != d) continue;
      TreeNode nd = tree[i];
      const double lo = LO[i], hi = HI[i];
      if (nd.feat < 0) {
        const double W = (double)leaf_sum(acc, 3 * i + 2, leaf_reps(qs), 3 * (int64_t)cap) / qs[6];
        nd.value = (float)fmin(fmax(leaf_value(SG[i], SH[i], W, p), lo), hi);
        tree[i] = nd;
        continue;
      }
      const int l = nd.left;
      double llo = lo, lhi = hi, rlo = lo, rhi = hi;
      const int mf = (int)p.mono[nd.feat];
      if (mf != 0) {
        const double wl = fmin(fmax(leaf_value(SG[l], SH[l], SH[l], p), lo), hi);
        const double wr = fmin(fmax(leaf_value(SG[l + 1], SH[l + 1], SH[l + 1], p), lo), hi);
        const double mid = 0.5 * (wl + wr);
        if (mf > 0) { lhi = mid; rlo = mid; } else { llo = mid; rhi = mid; }
      }
      LO[l] = llo; HI[l] = lhi; LO[l + 1] = rlo; HI[l + 1] = rhi;
    }
    __syncthreads();
  }
}

H2OMX_API int64_t h2omx_mono_scratch_bytes(int cap) { return (((int64_t)cap * 4 + 15) / 16) * 16 + (int64_t)cap * 32; }

// ---------------------------------------------------------------------------
// K8: score raw (unbinned) feature-major data with a tree ensemble.
// nodes: all trees concatenated; roots[t] = offset of tree t; out[cls][r] +=
// sum of leaf values of the trees of class cls (tree t belongs to class t % K).
// ---------------------------------------------------------------------------
// categorical split of a tree node: is level / bin code b in its left set?
// (codes outside 0..255 - unseen levels - follow the NA direction)
__device__ __forceinline__ bool cat_left(const uint32_t* __restrict__ bits, int b, int na_left) {
  if (b < 0 || b > 255) return (na_left & 1) != 0;
  return ((bits[b >> 5] >> (b & 31)) & 1u) != 0;
}

__global__ __launch_bounds__(256) void predict_raw_kernel(const float* __restrict__ X, int64_t ld, int64_t n,
                                                          const TreeNode* __restrict__ nodes,
                                                          const int* __restrict__ roots, int ntrees, int K,
                                                          float* __restrict__ out, int64_t ldo,
                                                          const uint32_t* __restrict__ catbits) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  for (int t = 0; t < ntrees; ++t) {
    const TreeNode* tr = nodes + roots[t];
    int id = 0;
    for (int guard = 0; guard < 64; ++guard) {
      const TreeNode nd = tr[id];
      if (nd.feat < 0) break;
      const float v = X[(int64_t)nd.feat * ld + r];
      bool left;
      if (v != v) left = (nd.na_left & 1) != 0;
      else if (nd.na_left & 2) left = cat_left(catbits + 8 * ((int64_t)roots[t] + id), (int)v, nd.na_left);
      else left = v <= nd.thr;
      id = left ? nd.left : nd.left + 1;
    }
    out[(int64_t)(t % K) * ldo + r] += tr[id].value;
  }
}

// Same on binned codes (training frame), avoids re-binning.
__global__ __launch_bounds__(256) void predict_binned_kernel(const uint8_t* __restrict__ codes, int64_t npad,
                                                             int64_t n, const TreeNode* __restrict__ nodes,
                                                             const int* __restrict__ roots, int ntrees, int K,
                                                             int nbt, float* __restrict__ out, int64_t ldo,
                                                             const uint32_t* __restrict__ catbits) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  for (int t = 0; t < ntrees; ++t) {
    const TreeNode* tr = nodes + roots[t];
    int id = 0;
    for (int guard = 0; guard < 64; ++guard) {
      const TreeNode nd = tr[id];
      if (nd.feat < 0) break;
      const int b = codes[(int64_t)nd.feat * npad + r];
      bool left;
      if (b == nbt - 1) left = (nd.na_left & 1) != 0;
      else if (nd.na_left & 2) left = cat_left(catbits + 8 * ((int64_t)roots[t] + id), b, nd.na_left);
      else left = b <= nd.bin;
      id = left ? nd.left : nd.left + 1;
    }
    out[(int64_t)(t % K) * ldo + r] += tr[id].value;
  }
}

// ===========================================================================
// C ABI
// ===========================================================================
static inline int grid_for(int64_t n, int block, int cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

H2OMX_API int h2omx_tree_sizes(int* out) {
  out[0] = sizeof(SplitParams);
  out[1] = sizeof(FeatBest);
  out[2] = sizeof(NodeLink);
  out[3] = sizeof(PartInfo);
  out[4] = sizeof(TreeNode);
  out[5] = sizeof(GradParams);
  return kOk;
}

H2OMX_API int h2omx_bin_features(const float* X, int64_t ld, int64_t n, int F, const float* edges, const int* nvb,
                                 int nbt, uint8_t* codes, int64_t npad, hipStream_t stream) {
  if (nbt > 256 || nbt < 2 || npad < n) return kBadArg;
  dim3 grid(grid_for(npad, 256, 4096), F);
  hipLaunchKernelGGL(bin_features_kernel, grid, dim3(256), 0, stream, X, ld, n, edges, nvb, nbt, codes, npad);
  return launch_status();
}

static int hist_build_launch(const uint8_t* codes, int64_t npad, const float* g, const float* s2, const int* nid,
                             const void* link, const int* ctl, const int* nvb, const double* qscale, int salt,
                             int F, int nbt, int fg, int n_groups, int wgpg, int slot_lo, int slot_cnt,
                             int rows_per_lane, int threads, const short* slot16, unsigned long long* pk_buf,
                             int pkm, unsigned long long* partials, const void* part_prev, const int* ctl_prev,
                             int* nid_out, int writer, hipStream_t stream, const GradFuse* gfp = nullptr) {
  const bool route = part_prev != nullptr;
  GradFuse gfz{};
  if (gfp) gfz = *gfp;
  // pkm bit 3: wave-compacted atomics (CMP; stored rows, 16-row units, <= 64 slots per pass)
  const bool cmp = (pkm & 8) != 0;
  // pkm bit 4 / 5: level-0 histograms in 8 / 4 interleaved lane copies (PKM 1 / 3 only)
  const int cop = (pkm & 16) ? 8 : ((pkm & 32) ? 4 : 1);
  // pkm bit 6: int16 node-id streams (routed levels only)
  const bool nid16 = (pkm & 64) != 0;
  pkm &= 7;
  if (nid16 && (!route || cmp || rows_per_lane != 16)) return kBadArg;
  if (cop > 1 && ((pkm != 1 && pkm != 3 && pkm != 6) || route || cmp)) return kBadArg;
  // pkm 6: level 0 reading the packed rows boost_update wrote (implicit root)
  if (pkm == 6 && (nid != nullptr || route || cmp || pk_buf == nullptr)) return kBadArg;
  if (cmp && ((pkm != 2 && pkm != 4) || rows_per_lane != 16 || slot_cnt > 64)) return kBadArg;
  if (route && (ctl_prev == nullptr || nid_out == nullptr || nid_out == nid || (pkm != 2 && pkm != 4)))
    return kBadArg;
  const PartInfo* pp = reinterpret_cast<const PartInfo*>(part_prev);
  if (wgpg % 8 != 0 || npad % 16 != 0 || fg > 256 || threads % 64 != 0 || threads > 1024 || threads < fg)
    return kBadArg;
  if (pkm < 0 || pkm > 6 || (pkm > 0 && pk_buf == nullptr) || ((pkm == 2 || pkm == 4) && !route && slot16 == nullptr))
    return kBadArg;
  // fused gradient level: implicit root (no node ids), 32-bit packed rows, no compaction / routing
  if ((pkm == 5) != (gfp != nullptr) || (pkm == 5 && (nid != nullptr || route || cmp || gfz.F == nullptr ||
                                                      gfz.y == nullptr || gfz.g == nullptr || gfz.h == nullptr ||
                                                      (gfz.apply && (gfz.nid == nullptr || gfz.tree == nullptr)))))
    return kBadArg;
  const int64_t units = npad / rows_per_lane;
  if ((units + wgpg - 1) / wgpg * rows_per_lane > ROWS_CAP) return kBadArg;  // fixed-point headroom
  const size_t lds = (size_t)slot_cnt * fg * nbt * cop * sizeof(unsigned long long) +
                     (cmp ? (size_t)(threads / 64) * CMP_STAGE_BYTES : 0);
  if (lds > 156 * 1024) return kBadArg;
  const int grid = n_groups * wgpg;
  const NodeLink* lk = reinterpret_cast<const NodeLink*>(link);
#define LAUNCH_HBK(NB, R, M, RT, C)                                                                           \
  hipLaunchKernelGGL((hist_build_kernel<NB, R, M, RT, C>), dim3(grid), dim3(threads), lds, stream, codes, npad, \
                     g, s2, nid, lk, ctl, nvb, qscale, (uint32_t)salt, F, fg, n_groups, wgpg, slot_lo, slot_cnt,  \
                     slot16, pk_buf, partials, pp, ctl_prev, nid_out, writer, gfz)
#define LAUNCH_HBKC(NB, R, M, CP)                                                                                \
  hipLaunchKernelGGL((hist_build_kernel<NB, R, M, false, false, CP>), dim3(grid), dim3(threads), lds, stream, codes, \
                     npad, g, s2, nid, lk, ctl, nvb, qscale, (uint32_t)salt, F, fg, n_groups, wgpg, slot_lo,        \
                     slot_cnt, slot16, pk_buf, partials, pp, ctl_prev, nid_out, writer, gfz)
#define LAUNCH_HBK16(NB, M)                                                                                      \
  hipLaunchKernelGGL((hist_build_kernel<NB, 16, M, true, false, 1, true>), dim3(grid), dim3(threads), lds, stream, \
                     codes, npad, g, s2, nid, lk, ctl, nvb, qscale, (uint32_t)salt, F, fg, n_groups, wgpg, slot_lo,    \
                     slot_cnt, slot16, pk_buf, partials, pp, ctl_prev, nid_out, writer, gfz)
#define LAUNCH_HB(NB, R)                                            \
  do {                                                             \
    if (pkm == 0) LAUNCH_HBK(NB, R, 0, false, false);               \
    else if (pkm == 1 && cop == 8) LAUNCH_HBKC(NB, R, 1, 8);        \
    else if (pkm == 3 && cop == 8) LAUNCH_HBKC(NB, R, 3, 8);        \
    else if (pkm == 1 && cop == 4) LAUNCH_HBKC(NB, R, 1, 4);        \
    else if (pkm == 3 && cop == 4) LAUNCH_HBKC(NB, R, 3, 4);        \
    else if (pkm == 6 && cop == 8) LAUNCH_HBKC(NB, R, 6, 8);        \
    else if (pkm == 6 && cop == 4) LAUNCH_HBKC(NB, R, 6, 4);        \
    else if (pkm == 6) LAUNCH_HBK(NB, R, 6, false, false);          \
    else if (pkm == 1) LAUNCH_HBK(NB, R, 1, false, false);          \
    else if (pkm == 2 && route) LAUNCH_HBK(NB, R, 2, true, false);  \
    else if (pkm == 2) LAUNCH_HBK(NB, R, 2, false, false);          \
    else if (pkm == 3) LAUNCH_HBK(NB, R, 3, false, false);          \
    else if (pkm == 5) LAUNCH_HBK(NB, R, 5, false, false);          \
    else if (route) LAUNCH_HBK(NB, R, 4, true, false);              \
    else LAUNCH_HBK(NB, R, 4, false, false);                        \
  } while (0)
#define LAUNCH_HBCMP(NB)                                             \
  do {                                                              \
    if (pkm == 2 && route) LAUNCH_HBK(NB, 16, 2, true, true);        \
    else if (pkm == 2) LAUNCH_HBK(NB, 16, 2, false, true);           \
    else if (route) LAUNCH_HBK(NB, 16, 4, true, true);               \
    else LAUNCH_HBK(NB, 16, 4, false, true);                         \
  } while (0)
  if (cmp) {
    switch (nbt) {
      case 32: LAUNCH_HBCMP(32); break;
      case 64: LAUNCH_HBCMP(64); break;
      case 128: LAUNCH_HBCMP(128); break;
      case 256: LAUNCH_HBCMP(256); break;
      default: return kBadArg;
    }
  } else if (nid16) {
    switch (nbt) {
      case 32: if (pkm == 2) LAUNCH_HBK16(32, 2); else LAUNCH_HBK16(32, 4); break;
      case 64: if (pkm == 2) LAUNCH_HBK16(64, 2); else LAUNCH_HBK16(64, 4); break;
      case 128: if (pkm == 2) LAUNCH_HBK16(128, 2); else LAUNCH_HBK16(128, 4); break;
      case 256: if (pkm == 2) LAUNCH_HBK16(256, 2); else LAUNCH_HBK16(256, 4); break;
      default: return kBadArg;
    }
  } else if (rows_per_lane == 16) {
    switch (nbt) {
      case 32: LAUNCH_HB(32, 16); break;
      case 64: LAUNCH_HB(64, 16); break;
      case 128: LAUNCH_HB(128, 16); break;
      case 256: LAUNCH_HB(256, 16); break;
      default: return kBadArg;
    }
  } else if (rows_per_lane == 8) {
    switch (nbt) {
      case 32: LAUNCH_HB(32, 8); break;
      case 64: LAUNCH_HB(64, 8); break;
      case 128: LAUNCH_HB(128, 8); break;
      case 256: LAUNCH_HB(256, 8); break;
      default: return kBadArg;
    }
  } else {
    return kBadArg;
  }
#undef LAUNCH_HB
#undef LAUNCH_HBK16
#undef LAUNCH_HBCMP
#undef LAUNCH_HBK
#undef LAUNCH_HBKC
  return launch_status();
}

H2OMX_API int h2omx_hist_build(const uint8_t* codes, int64_t npad, const float* g, const float* s2, const int* nid,
                               const void* link, const int* ctl, const int* nvb, const double* qscale, int salt,
                               int F, int nbt, int fg, int n_groups, int wgpg, int slot_lo, int slot_cnt,
                               int rows_per_lane, int threads, const short* slot16, unsigned long long* pk_buf,
                               int pkm, unsigned long long* partials, hipStream_t stream) {
  return hist_build_launch(codes, npad, g, s2, nid, link, ctl, nvb, qscale, salt, F, nbt, fg, n_groups, wgpg, slot_lo,
                           slot_cnt, rows_per_lane, threads, slot16, pk_buf, pkm, partials, nullptr, nullptr, nullptr,
                           0, stream);
}

// Level 0 with the gradient pass fused in (PKM 5, see GradFuse): F / y / the
// previous tree's leaves -> F, g, h and the 32-bit packed rows.
H2OMX_API int h2omx_hist_build_grad(const uint8_t* codes, int64_t npad, const int* ctl, const int* nvb,
                                    const double* qscale, int salt, int F, int nbt, int fg, int n_groups, int wgpg,
                                    int slot_cnt, int rows_per_lane, int threads, unsigned long long* pk_buf,
                                    unsigned long long* partials, float* Fm, const float* y, const int* nid_leaf,
                                    const void* tree, int cap, float* g, float* h, int apply, int s_is_h,
                                    int pk64, const void* gparams, hipStream_t stream) {
  if (gparams == nullptr) return kBadArg;
  GradFuse gf{};
  gf.F = Fm; gf.y = y; gf.nid = nid_leaf; gf.tree = reinterpret_cast<const TreeNode*>(tree);
  gf.g = g; gf.h = h; gf.apply = apply; gf.s_is_h = s_is_h; gf.pk64 = pk64; gf.cap = cap;
  gf.gp = *reinterpret_cast<const GradParams*>(gparams);
  return hist_build_launch(codes, npad, nullptr, nullptr, nullptr, nullptr, ctl, nvb, qscale, salt, F, nbt, fg,
                           n_groups, wgpg, 0, slot_cnt, rows_per_lane, threads, nullptr, pk_buf, 5, partials, nullptr,
                           nullptr, nullptr, 0, stream, &gf);
}

// Deeper level with the previous level's partition fused in (see ROUTE):
// nid_prev -> nid_out (writer pass only), part_prev / ctl_prev = that level.
H2OMX_API int h2omx_hist_build_route(const uint8_t* codes, int64_t npad, const int* nid_prev, const void* part_prev,
                                     const int* ctl_prev, int* nid_out, int writer, const int* ctl, const int* nvb,
                                     const double* qscale, int F, int nbt, int fg, int n_groups, int wgpg,
                                     int slot_lo, int slot_cnt, int rows_per_lane, int threads,
                                     unsigned long long* pk_buf, int pkm, unsigned long long* partials,
                                     hipStream_t stream) {
  if (part_prev == nullptr) return kBadArg;
  return hist_build_launch(codes, npad, nullptr, nullptr, nid_prev, nullptr, ctl, nvb, qscale, 0, F, nbt, fg, n_groups,
                           wgpg, slot_lo, slot_cnt, rows_per_lane, threads, nullptr, pk_buf, pkm, partials, part_prev,
                           ctl_prev, nid_out, writer, stream);
}

H2OMX_API int h2omx_hist_reduce(const unsigned long long* partials, int n_groups, int wgpg, int fg, int F, int nbt,
                                int slot_lo, int slot_cnt, const int* ctl, long long* built, hipStream_t stream) {
  const int64_t total = (int64_t)slot_cnt * F * nbt;  // nbt is a multiple of 32
  hipLaunchKernelGGL(hist_reduce_kernel, dim3((unsigned)(total / 32)), dim3(256), 0, stream, partials,
                     n_groups, wgpg, fg, F, nbt, slot_lo, slot_cnt, ctl, built);
  return launch_status();
}

H2OMX_API int h2omx_split_find(const long long* built, const long long* parent_full, long long* full, const int* ctl,
                               const void* link, const int* nvb, const uint8_t* tree_fmask, const double* qscale,
                               const void* params, int max_nodes, int nbt, void* out, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  const NodeLink* lk = reinterpret_cast<const NodeLink*>(link);
  FeatBest* o = reinterpret_cast<FeatBest*>(out);
  const dim3 grid(max_nodes, (p.F + 3) / 4);
#define LAUNCH_SF(NB)                                                                                          \
  if (p.catf != nullptr)                                                                                      \
    hipLaunchKernelGGL((split_find_kernel<NB, true>), grid, dim3(256), 0, stream, built, parent_full, full, ctl, \
                       lk, nvb, tree_fmask, qscale, p, o);                                                    \
  else                                                                                                        \
    hipLaunchKernelGGL((split_find_kernel<NB, false>), grid, dim3(256), 0, stream, built, parent_full, full,    \
                       ctl, lk, nvb, tree_fmask, qscale, p, o)
  switch (nbt) {
    case 32: LAUNCH_SF(32); break;
    case 64: LAUNCH_SF(64); break;
    case 128: LAUNCH_SF(128); break;
    case 256: LAUNCH_SF(256); break;
    default: return kBadArg;
  }
#undef LAUNCH_SF
  return launch_status();
}

H2OMX_API int h2omx_reduce_split(const unsigned long long* partials, int wgpg, int fg, int slot_lo, int slot_cnt,
                                 const long long* parent_full, long long* full, const int* ctl, const void* link,
                                 const int* nvb, const uint8_t* tree_fmask, const double* qscale, const void* params,
                                 int nbt, void* out, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (slot_cnt < 1 || wgpg < 1 || fg < 1 || p.F < 1) return kBadArg;
  const NodeLink* lk = reinterpret_cast<const NodeLink*>(link);
  FeatBest* o = reinterpret_cast<FeatBest*>(out);
  const dim3 grid(slot_cnt, p.F);
  const LevelFin nofin{};
#define LAUNCH_RS(NB)                                                                                              \
  if (p.catf != nullptr)                                                                                          \
    hipLaunchKernelGGL((reduce_split_kernel<NB, true>), grid, dim3(1024), 0, stream, partials, wgpg, fg, slot_lo, \
                       slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, o, nofin);               \
  else                                                                                                            \
    hipLaunchKernelGGL((reduce_split_kernel<NB, false>), grid, dim3(1024), 0, stream, partials, wgpg, fg,         \
                       slot_lo, slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, o, nofin)
  switch (nbt) {
    case 32: LAUNCH_RS(32); break;
    case 64: LAUNCH_RS(64); break;
    case 128: LAUNCH_RS(128); break;
    case 256: LAUNCH_RS(256); break;
    default: return kBadArg;
  }
#undef LAUNCH_RS
  return launch_status();
}

// One-pass level (slot_lo = 0, slot_cnt = the level's slots) with the level
// finalisation in its last workgroup (LevelFin): replaces reduce_split +
// level_finalize (node_best_finalize) for levels of <= 64 nodes.  ticket: an
// int zeroed once (each launch leaves it zero).
static LevelFin make_fin(int* ctl_next, const float* edges, int max_next_nodes, void* part, void* next_link,
                         void* tree, int tree_capacity, void* nsplit, int* ticket) {
  LevelFin f;
  f.ctl_next = ctl_next; f.edges = edges; f.part = reinterpret_cast<PartInfo*>(part);
  f.next_link = reinterpret_cast<NodeLink*>(next_link); f.tree = reinterpret_cast<TreeNode*>(tree);
  f.nsplit = reinterpret_cast<NodeSplit*>(nsplit); f.ticket = ticket;
  f.max_next_nodes = max_next_nodes; f.tree_capacity = tree_capacity;
  return f;
}

H2OMX_API int h2omx_reduce_split_fin(const unsigned long long* partials, int wgpg, int fg, int slot_cnt,
                                     const long long* parent_full, long long* full, const int* ctl, const void* link,
                                     const int* nvb, const uint8_t* tree_fmask, const double* qscale,
                                     const void* params, int nbt, void* out, int* ctl_next, const float* edges,
                                     int max_next_nodes, void* part, void* next_link, void* tree, int tree_capacity,
                                     void* nsplit, int* ticket, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (slot_cnt < 1 || wgpg < 1 || fg < 1 || p.F < 1 || ticket == nullptr || nsplit == nullptr) return kBadArg;
  const NodeLink* lk = reinterpret_cast<const NodeLink*>(link);
  FeatBest* o = reinterpret_cast<FeatBest*>(out);
  const dim3 grid(slot_cnt, p.F);
  const LevelFin fin = make_fin(ctl_next, edges, max_next_nodes, part, next_link, tree, tree_capacity, nsplit, ticket);
#define LAUNCH_RSF(NB)                                                                                             \
  if (p.catf != nullptr)                                                                                          \
    hipLaunchKernelGGL((reduce_split_kernel<NB, true, true>), grid, dim3(1024), 0, stream, partials, wgpg, fg, 0,  \
                       slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, o, fin);                 \
  else                                                                                                            \
    hipLaunchKernelGGL((reduce_split_kernel<NB, false, true>), grid, dim3(1024), 0, stream, partials, wgpg, fg, 0, \
                       slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, o, fin)
  switch (nbt) {
    case 32: LAUNCH_RSF(32); break;
    case 64: LAUNCH_RSF(64); break;
    case 128: LAUNCH_RSF(128); break;
    case 256: LAUNCH_RSF(256); break;
    default: return kBadArg;
  }
#undef LAUNCH_RSF
  return launch_status();
}

// N-rank fused level (reduce_split_p2p_kernel); desc = host P2PDesc image.
// One pass only (slot_cnt = the level's slots): the host routes multi-pass
// levels through hist_reduce + all-reduce + split_find.  The split records
// land in the symmetric buffer's split table (h2omx_node_best_finalize_p2p
// reads them); capacity: the pushed rows fit a parity, the records half of one.
// With a ticket (non-null), the launch's last workgroup also waits for every
// rank's done word and finalises the level (node_best_finalize_p2p folded in:
// the ticket is unused beyond selecting that mode - the P2P finish ticket
// picks the workgroup).
H2OMX_API int h2omx_reduce_split_p2p(const void* desc, const unsigned long long* partials, int wgpg, int fg,
                                     int slot_cnt, const long long* parent_full, long long* full, const int* ctl,
                                     const void* link, const int* nvb, const uint8_t* tree_fmask,
                                     const double* qscale, const void* params, int nbt, int max_blocks,
                                     int* ctl_next, const float* edges, int max_next_nodes, void* part,
                                     void* next_link, void* tree, int tree_capacity, void* nsplit, int* ticket,
                                     hipStream_t stream) {
  if (desc == nullptr) return kBadArg;
  const p2pdev::P2PDesc d = *reinterpret_cast<const p2pdev::P2PDesc*>(desc);
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (slot_cnt < 1 || wgpg < 1 || fg < 1 || p.F < 1) return kBadArg;
  if (d.world < 2 || d.world > p2pdev::kMaxRanks || d.rank < 0 || d.rank >= d.world) return kBadArg;
  const int64_t items = (int64_t)slot_cnt * p.F;
  const int64_t fl = (p.F + d.world - 1) / d.world;
  if ((int64_t)slot_cnt * fl * d.world * 2 * nbt * 8 > d.cap) return kBadArg;
  if ((int64_t)2 * slot_cnt * p.F * (int64_t)sizeof(FeatBest) > d.cap / 2) return kBadArg;
  const int nb = (int)std::min<int64_t>(items, std::min(std::max(max_blocks, 1), p2pdev::kMaxBlocks));
  const NodeLink* lk = reinterpret_cast<const NodeLink*>(link);
  const LevelFin fin = make_fin(ctl_next, edges, max_next_nodes, part, next_link, tree, tree_capacity, nsplit, ticket);
  const bool with_fin = ticket != nullptr;
  if (with_fin && nsplit == nullptr) return kBadArg;
#define LAUNCH_RSP(NB)                                                                                             \
  if (p.catf != nullptr && with_fin)                                                                              \
    hipLaunchKernelGGL((reduce_split_p2p_kernel<NB, true, true>), dim3(nb), dim3(1024), 0, stream, d, partials,   \
                       wgpg, fg, slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, fin);          \
  else if (p.catf != nullptr)                                                                                     \
    hipLaunchKernelGGL((reduce_split_p2p_kernel<NB, true>), dim3(nb), dim3(1024), 0, stream, d, partials, wgpg,   \
                       fg, slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, fin);                \
  else if (with_fin)                                                                                              \
    hipLaunchKernelGGL((reduce_split_p2p_kernel<NB, false, true>), dim3(nb), dim3(1024), 0, stream, d, partials,  \
                       wgpg, fg, slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, fin);          \
  else                                                                                                            \
    hipLaunchKernelGGL((reduce_split_p2p_kernel<NB, false>), dim3(nb), dim3(1024), 0, stream, d, partials, wgpg,  \
                       fg, slot_cnt, parent_full, full, ctl, lk, nvb, tree_fmask, qscale, p, fin)
  switch (nbt) {
    case 32: LAUNCH_RSP(32); break;
    case 64: LAUNCH_RSP(64); break;
    case 128: LAUNCH_RSP(128); break;
    case 256: LAUNCH_RSP(256); break;
    default: return kBadArg;
  }
#undef LAUNCH_RSP
  return launch_status();
}

// level finalisation from per-node splits: one workgroup for small levels,
// count / scan / write tiles (lf_*_kernel) when the level can hold more than
// LF_MB_NODES nodes and the caller passed a tile scratch (>= max_nodes / 1024 + 1 ints)
constexpr int LF_MB_NODES = 8192;
static void level_finalize_launch(const NodeSplit* ns, const int* ctl, int* ctl_next, const SplitParams& p,
                                  const float* edges, const int* nvb, int nbt, int max_next_nodes, void* part,
                                  void* next_link, void* tree, int tree_capacity, int max_nodes, int* tiles,
                                  hipStream_t stream) {
  PartInfo* pi = reinterpret_cast<PartInfo*>(part);
  NodeLink* nl = reinterpret_cast<NodeLink*>(next_link);
  TreeNode* tr = reinterpret_cast<TreeNode*>(tree);
  if (tiles == nullptr || max_nodes <= LF_MB_NODES) {
    hipLaunchKernelGGL(level_finalize_kernel, dim3(1), dim3(1024), 0, stream, ns, ctl, ctl_next, p, edges, nvb, nbt,
                       max_next_nodes, pi, nl, tr, tree_capacity);
    return;
  }
  const int nt = (max_nodes + LF_TILE - 1) / LF_TILE;
  hipLaunchKernelGGL(lf_count_kernel, dim3(nt), dim3(LF_TILE), 0, stream, ns, ctl, p, tiles);
  hipLaunchKernelGGL(lf_scan_kernel, dim3(1), dim3(1024), 0, stream, tiles, nt, ctl, ctl_next, max_next_nodes);
  hipLaunchKernelGGL(lf_write_kernel, dim3(nt), dim3(LF_TILE), 0, stream, ns, ctl, p, edges, nvb, nbt, max_next_nodes,
                     pi, nl, tr, tree_capacity, tiles);
}

H2OMX_API int h2omx_level_finalize(const void* fbest, const int* ctl, int* ctl_next, const void* params,
                                   const float* edges, const int* nvb, int nbt, int max_next_nodes, void* part,
                                   void* next_link, void* tree, int tree_capacity, void* nsplit,
                                   int max_nodes, int* tiles, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  NodeSplit* ns = reinterpret_cast<NodeSplit*>(nsplit);
  if (max_nodes <= 64) {   // one launch: the per-node arg-max inside the finalisation
    hipLaunchKernelGGL(node_best_finalize_kernel, dim3(1), dim3(1024), 0, stream,
                       reinterpret_cast<const FeatBest*>(fbest), ctl, ctl_next, p, edges, nvb, nbt, max_next_nodes,
                       reinterpret_cast<PartInfo*>(part), reinterpret_cast<NodeLink*>(next_link),
                       reinterpret_cast<TreeNode*>(tree), tree_capacity, ns);
    return launch_status();
  }
  hipLaunchKernelGGL(node_best_kernel, dim3(max_nodes), dim3(64), 0, stream, reinterpret_cast<const FeatBest*>(fbest),
                     ctl, p.F, ns);
  level_finalize_launch(ns, ctl, ctl_next, p, edges, nvb, nbt, max_next_nodes, part, next_link, tree, tree_capacity,
                        max_nodes, tiles, stream);
  return launch_status();
}

template <int MODE>
__device__ void level_fin_records(const FeatBest* __restrict__ fbest, const int* __restrict__ ctl, const SplitParams& p,
                                  const int* __restrict__ nvb, int nbt, const LevelFin& fin) {
  const int n = ctl[CTL_N];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int node = wid; node < n; node += nw) node_best_wave<MODE>(fbest, p.F, node, lane, fin.nsplit);
  __syncthreads();
  level_finalize_body(fin.nsplit, ctl, fin.ctl_next, p, fin.edges, nvb, nbt, fin.max_next_nodes, fin.part,
                      fin.next_link, fin.tree, fin.tree_capacity);
}

// N-rank level finalisation (after h2omx_reduce_split_p2p, same desc)
H2OMX_API int h2omx_node_best_finalize_p2p(const void* desc, const int* ctl, int* ctl_next, const void* params,
                                           const float* edges, const int* nvb, int nbt, int max_next_nodes,
                                           void* part, void* next_link, void* tree, int tree_capacity,
                                           void* nsplit, hipStream_t stream) {
  if (desc == nullptr) return kBadArg;
  const p2pdev::P2PDesc d = *reinterpret_cast<const p2pdev::P2PDesc*>(desc);
  if (d.world < 2 || d.world > p2pdev::kMaxRanks || d.rank < 0 || d.rank >= d.world) return kBadArg;
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  hipLaunchKernelGGL(node_best_finalize_p2p_kernel, dim3(1), dim3(1024), 0, stream, d, ctl, ctl_next, p, edges, nvb,
                     nbt, max_next_nodes, reinterpret_cast<PartInfo*>(part), reinterpret_cast<NodeLink*>(next_link),
                     reinterpret_cast<TreeNode*>(tree), tree_capacity, reinterpret_cast<NodeSplit*>(nsplit));
  return launch_status();
}

constexpr int PARTITION_BLOCKS = 8192;
constexpr int PART_RPL = 8;    // rows per lane per step (16: 1.52 vs 1.47 ms/tree on HIGGS)

static int partition_launch(const uint8_t* codes, int64_t npad, int* nid, const void* part, int nbt, const float* g,
                            const float* h, const float* w, const double* qscale, int cap,
                            unsigned long long* leaf_acc, const int* ctl_cur, const int* ctl_next, int win_max,
                            int blocks, int prefetch, short* slot16, int* nid_out, int all_rows, hipStream_t stream,
                            const float* Fm = nullptr, const float* yv = nullptr, const GradParams* gpp = nullptr,
                            int nidm = 0, const uint8_t* y8 = nullptr) {
  // nidm bit 0: nid is an int16 stream, bit 1: nid_out is (fused pipeline; distinct buffers)
  if (nidm != 0 && nid_out == nid) return kBadArg;
  GradParams gp{};
  if (gpp) gp = *gpp;
  if ((Fm != nullptr) != (gpp != nullptr) || (Fm != nullptr && (yv == nullptr || w != nullptr || !prefetch)))
    return kBadArg;
  if (slot16 && prefetch) return kBadArg;
  if (npad % PART_RPL != 0 || blocks < 1 || blocks > PARTITION_BLOCKS || win_max < 0) return kBadArg;
  if (all_rows && (leaf_acc == nullptr || win_max > cap)) return kBadArg;
  // 8 lane copies of the leaf window (12 KB for a depth-5 tree): occupancy
  // hides the split-code gathers better than conflict-free 32 copies (48 KB;
  // 0.778 vs 0.796 ms/tree, profiles/r5/partition_ab.txt)
  constexpr size_t kWinLds = 64 * 1024;
  int R = 8;
  while (R > 1 && (size_t)3 * win_max * R * sizeof(unsigned long long) > kWinLds) R >>= 1;
  if ((size_t)3 * win_max * R * sizeof(unsigned long long) > kWinLds) {
    if (all_rows) return kBadArg;  // the whole-tree window must fit
    win_max = 0;
  }
  const size_t lds = (leaf_acc && win_max > 0) ? (size_t)3 * win_max * R * sizeof(unsigned long long) : 0;
#define LAUNCH_PK(PF, NM, WIN)                                                                                  \
  hipLaunchKernelGGL((partition_kernel<PF, PART_RPL, NM>), dim3(blocks), dim3(256), lds, stream, codes, npad, nid, \
                     reinterpret_cast<const PartInfo*>(part), nbt, g, h, w, qscale, cap, leaf_acc, ctl_cur,        \
                     ctl_next, WIN, R, slot16, nid_out, all_rows, Fm, yv, gp, y8)
  if (prefetch && leaf_acc) {
    if (nidm == 3) LAUNCH_PK(true, 3, win_max);
    else if (nidm & 1) LAUNCH_PK(true, 1, win_max);
    else LAUNCH_PK(true, 0, win_max);
  } else {
    if (nidm == 3) LAUNCH_PK(false, 3, leaf_acc ? win_max : 0);
    else if (nidm == 1) LAUNCH_PK(false, 1, leaf_acc ? win_max : 0);
    else if (nidm == 2) LAUNCH_PK(false, 2, leaf_acc ? win_max : 0);
    else LAUNCH_PK(false, 0, leaf_acc ? win_max : 0);
  }
#undef LAUNCH_PK
  return launch_status();
}

H2OMX_API int h2omx_partition(const uint8_t* codes, int64_t npad, int* nid, const void* part, int nbt, const float* g,
                              const float* h, const float* w, const double* qscale, int cap,
                              unsigned long long* leaf_acc, const int* ctl_cur, const int* ctl_next, int win_max,
                              int blocks, int prefetch, short* slot16, hipStream_t stream) {
  return partition_launch(codes, npad, nid, part, nbt, g, h, w, qscale, cap, leaf_acc, ctl_cur, ctl_next, win_max,
                          blocks, prefetch, slot16, nid, 0, stream);
}

// Intermediate level of the fused-routing pipeline that is not fused into the
// next histogram (previous level too wide for per-node code loads): routes
// nid_in -> nid_out and writes slot16; no leaf sums (the final level adds them).
H2OMX_API int h2omx_partition_route(const uint8_t* codes, int64_t npad, const int* nid_in, int* nid_out,
                                    const void* part, int nbt, const int* ctl_cur, const int* ctl_next, int blocks,
                                    short* slot16, int nidm, hipStream_t stream) {
  if (slot16 == nullptr) return kBadArg;
  return partition_launch(codes, npad, const_cast<int*>(nid_in), part, nbt, nullptr, nullptr, nullptr, nullptr, 0,
                          nullptr, ctl_cur, ctl_next, 0, blocks, 0, slot16, nid_out, 0, stream, nullptr, nullptr,
                          nullptr, nidm);
}

// Final level of the fused-routing pipeline: nid_in (this level's node ids,
// earlier leaves as ~gid) -> nid_out leaves, exact sums of EVERY row into the
// whole-tree LDS window [0, cap).
H2OMX_API int h2omx_partition_final(const uint8_t* codes, int64_t npad, const int* nid_in, int* nid_out,
                                    const void* part, int nbt, const float* g, const float* h, const float* w,
                                    const double* qscale, int cap, unsigned long long* leaf_acc, const int* ctl_cur,
                                    const int* ctl_next, int blocks, const float* Fm, const float* y,
                                    const void* gparams, int nidm, const uint8_t* y8, hipStream_t stream) {
  // Fm / y / gparams (optional): the rows' (g, h) are re-derived from the margins;
  // nidm 1: nid_in is an int16 stream (nid_out stays int32: boost_update reads it)
  return partition_launch(codes, npad, const_cast<int*>(nid_in), part, nbt, g, h, w, qscale, cap, leaf_acc, ctl_cur,
                          ctl_next, cap, blocks, 1, nullptr, nid_out, 1, stream, Fm, y,
                          reinterpret_cast<const GradParams*>(gparams), nidm, y8);
}

static inline int stream_grid(int64_t) { return STAT_BLOCKS; }

// ring != nullptr: also copy `tree` (tree_bytes) into ring slot
// (tree_ctr - ctr_off) mod ring_n (graph replay's tree archive)
H2OMX_API int h2omx_boost_update(float* F, const float* y, const float* wobs, int64_t n, int64_t npad, int* nid,
                                 const void* tree, const void* gparams, float* g, float* h, float* wout,
                                 unsigned int* stat_max, int64_t tree_bytes, void* ring, int ring_n,
                                 const int* tree_ctr, int ctr_off, void* pk32_out, const double* qscale,
                                 int s_is_h, int store_gh, const uint8_t* y8, const void* nid16, hipStream_t stream) {
  const GradParams gp = *reinterpret_cast<const GradParams*>(gparams);
  if (ring != nullptr && (tree_bytes % 16 != 0 || ring_n < 1 || tree_ctr == nullptr)) return kBadArg;
  if (pk32_out != nullptr && qscale == nullptr) return kBadArg;
  hipLaunchKernelGGL(boost_update_kernel, dim3(stream_grid(npad)), dim3(256), 0, stream, F, y, wobs, n, npad, nid,
                     reinterpret_cast<const TreeNode*>(tree), gp, g, h, wout, stat_max,
                     reinterpret_cast<const uint4*>(tree), (int)(tree_bytes / 16), reinterpret_cast<uint4*>(ring),
                     ring_n, tree_ctr, ctr_off, reinterpret_cast<uint32_t*>(pk32_out), qscale, s_is_h, store_gh, y8,
                     reinterpret_cast<const short*>(nid16));
  return launch_status();
}

// Graph replay: the finished tree -> slot (tree_ctr - 1) mod R of a ring of R
// tree heaps (tree_begin advanced the counter), so a replayed step needs no
// host-side snapshot copy per tree (boost.TreeGraph freezes the ring every R trees)
__global__ __launch_bounds__(256) void tree_archive_kernel(const uint4* __restrict__ src, int n16,
                                                           uint4* __restrict__ ring, int R,
                                                           const int* __restrict__ tree_ctr) {
  const int slot = (int)(((unsigned)(tree_ctr[0] - 1)) % (unsigned)R);
  uint4* dst = ring + (int64_t)slot * n16;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

H2OMX_API int h2omx_tree_archive(const void* tree, int64_t bytes, void* ring, int R, const int* tree_ctr,
                                 hipStream_t stream) {
  if (bytes % 16 != 0 || R < 1 || tree_ctr == nullptr) return kBadArg;
  const int n16 = (int)(bytes / 16);
  hipLaunchKernelGGL(tree_archive_kernel, dim3(grid_for(n16, 256, 64)), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(tree), n16, reinterpret_cast<uint4*>(ring), R, tree_ctr);
  return launch_status();
}

H2OMX_API int h2omx_apply_tree(float* F, int64_t n, const int* nid, const void* tree, hipStream_t stream) {
  hipLaunchKernelGGL(apply_tree_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, F, n, nid,
                     reinterpret_cast<const TreeNode*>(tree));
  return launch_status();
}

H2OMX_API int h2omx_oob_accumulate(float* oob_sum, float* oob_cnt, int64_t n, const int* nid, const void* tree,
                                   const float* wobs, uint32_t seed, int tree_index, float sample_rate,
                                   int64_t row_base, int count, hipStream_t stream) {
  hipLaunchKernelGGL(oob_accumulate_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, stream, oob_sum, oob_cnt, n,
                     nid, reinterpret_cast<const TreeNode*>(tree), wobs, seed, (uint32_t)tree_index, sample_rate,
                     row_base, count);
  return launch_status();
}

H2OMX_API int h2omx_softmax_grad(const float* F, int K, int64_t ldF, const int* yk, const float* wobs, int64_t n,
                                 int64_t npad, int cls, const void* gparams, int* nid, float* g, float* h,
                                 float* wout, unsigned int* stat_max, hipStream_t stream) {
  const GradParams gp = *reinterpret_cast<const GradParams*>(gparams);
  hipLaunchKernelGGL(softmax_grad_kernel, dim3(stream_grid(npad)), dim3(256), 0, stream, F, K, ldF, yk, wobs, n,
                     npad, cls, gp, nid, g, h, wout, stat_max);
  return launch_status();
}

H2OMX_API int h2omx_stat_blocks() { return STAT_BLOCKS; }

H2OMX_API int h2omx_stat_reduce(const unsigned int* slab, unsigned int* stat_max, hipStream_t stream) {
  hipLaunchKernelGGL(stat_reduce_kernel, dim3(1), dim3(1024), 0, stream, slab, STAT_BLOCKS, stat_max);
  return launch_status();
}

H2OMX_API int h2omx_tree_begin(const unsigned int* stat_max, int mode, int max_rows_per_wg, double* qscale,
                               int* ctl0, void* link0, unsigned long long* leaf_acc, int leaf_n,
                               long long row_base, int tree_index, int* tree_ctr, hipStream_t stream) {
  if (max_rows_per_wg < 1 || max_rows_per_wg > ROWS_CAP) return kBadArg;
  const double qg = exp2(floor(log2(1073741824.0 / max_rows_per_wg)));   // |sum| <= 2^30
  const double qsr = exp2(floor(log2(2147483648.0 / max_rows_per_wg)));  // sum <= 2^31
  hipLaunchKernelGGL(tree_begin_kernel, dim3(grid_for(leaf_n, 256, 1024)), dim3(256), 0, stream, stat_max, mode, qg,
                     qsr, qscale, ctl0, reinterpret_cast<NodeLink*>(link0), leaf_acc, leaf_n, row_base, tree_index,
                     tree_ctr);
  return launch_status();
}

H2OMX_API int h2omx_leaf_stats(const int* nid, const float* g, const float* h, const float* w, int64_t n,
                               const double* qscale, int cap, unsigned long long* acc, hipStream_t stream) {
  const size_t lds = cap <= 2048 ? (size_t)cap * 3 * sizeof(unsigned long long) : 0;
  hipLaunchKernelGGL(leaf_stats_kernel, dim3(grid_for(n, 256, 1024)), dim3(256), lds, stream, nid, g, h, w, n, qscale,
                     cap, acc);
  return launch_status();
}

H2OMX_API int h2omx_partition_blocks() { return PARTITION_BLOCKS; }

H2OMX_API int h2omx_leaf_reduce(const unsigned long long* slab, int n_slabs, int cap, unsigned long long* leaf_acc,
                                hipStream_t stream) {
  if (n_slabs <= 0) return kOk;
  hipLaunchKernelGGL(leaf_reduce_kernel, dim3(3 * cap), dim3(256), 0, stream, slab, n_slabs, 3 * cap, leaf_acc);
  return launch_status();
}

H2OMX_API int h2omx_leaf_finalize(const unsigned long long* acc, const int* ctl_final, const double* qscale,
                                  const void* params, void* tree, int cap, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  hipLaunchKernelGGL(leaf_finalize_kernel, dim3(grid_for(cap, 256, 1024)), dim3(256), 0, stream, acc, ctl_final,
                     qscale, p, reinterpret_cast<TreeNode*>(tree), cap);
  return launch_status();
}

H2OMX_API int h2omx_leaf_finalize_begin(unsigned long long* acc, const int* ctl_final, double* qscale,
                                        const void* params, void* tree, int cap, const unsigned int* stat_max,
                                        int mode, int max_rows_per_wg, int* ctl0, void* link0, long long row_base,
                                        int* tree_ctr, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (max_rows_per_wg < 1 || max_rows_per_wg > ROWS_CAP || tree_ctr == nullptr || p.gbound != nullptr) return kBadArg;
  const double qg = exp2(floor(log2(1073741824.0 / max_rows_per_wg)));
  const double qsr = exp2(floor(log2(2147483648.0 / max_rows_per_wg)));
  hipLaunchKernelGGL(leaf_finalize_begin_kernel, dim3(1), dim3(1024), 0, stream, acc, ctl_final, qscale, p,
                     reinterpret_cast<TreeNode*>(tree), cap, stat_max, mode, qg, qsr, ctl0,
                     reinterpret_cast<NodeLink*>(link0), row_base, tree_ctr);
  return launch_status();
}

// N-rank leaf finalisation with the leaf-sum exchange inside (one launch);
// begin = 1: also the chained next tree's tree_begin (as leaf_finalize_begin)
H2OMX_API int h2omx_leaf_finalize_p2p(const void* desc, unsigned long long* acc, const int* ctl_final, double* qscale,
                                      const void* params, void* tree, int cap, int begin,
                                      const unsigned int* stat_max, int mode, int max_rows_per_wg, int* ctl0,
                                      void* link0, long long row_base, int* tree_ctr, hipStream_t stream) {
  if (desc == nullptr) return kBadArg;
  const p2pdev::P2PDesc d = *reinterpret_cast<const p2pdev::P2PDesc*>(desc);
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (d.world < 2 || d.world > p2pdev::kMaxRanks || d.rank < 0 || d.rank >= d.world) return kBadArg;
  if ((int64_t)cap * 3 * 8 * (d.loopback ? 1 : d.world) > d.cap || p.gbound != nullptr) return kBadArg;
  double qg = 0.0, qsr = 0.0;
  if (begin) {
    if (max_rows_per_wg < 1 || max_rows_per_wg > ROWS_CAP || tree_ctr == nullptr) return kBadArg;
    qg = exp2(floor(log2(1073741824.0 / max_rows_per_wg)));
    qsr = exp2(floor(log2(2147483648.0 / max_rows_per_wg)));
  }
  const int nb = std::min(p2pdev::kMaxBlocks, (cap + LEAF_P2P_THREADS - 1) / LEAF_P2P_THREADS);
  hipLaunchKernelGGL(leaf_finalize_p2p_kernel, dim3(nb), dim3(LEAF_P2P_THREADS), 0, stream, d, acc, ctl_final, qscale, p,
                     reinterpret_cast<TreeNode*>(tree), cap, begin ? 1 : 0, stat_max, mode, qg, qsr, ctl0,
                     reinterpret_cast<NodeLink*>(link0), row_base, tree_ctr);
  return launch_status();
}

// leaf_finalize + (mode 0, Newton leaves, monotone constraints) the leaf-scale
// interval pass; scratch of h2omx_mono_scratch_bytes(cap) bytes
H2OMX_API int h2omx_leaf_finalize_mono(const unsigned long long* acc, const int* ctl_final, const double* qscale,
                                       const void* params, void* tree, int cap, void* scratch, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (p.mono == nullptr || scratch == nullptr) return kBadArg;
  hipLaunchKernelGGL(leaf_finalize_kernel, dim3(grid_for(cap, 256, 1024)), dim3(256), 0, stream, acc, ctl_final,
                     qscale, p, reinterpret_cast<TreeNode*>(tree), cap);
  hipLaunchKernelGGL(mono_newton_kernel, dim3(1), dim3(1024), 0, stream, acc, ctl_final, qscale, p,
                     reinterpret_cast<TreeNode*>(tree), cap, static_cast<char*>(scratch));
  return launch_status();
}

// catbits: [total nodes][8] left-set bitsets aligned with `nodes` (nullptr:
// no categorical splits)
H2OMX_API int h2omx_predict_raw(const float* X, int64_t ld, int64_t n, const void* nodes, const int* roots,
                                int ntrees, int K, float* out, int64_t ldo, const uint32_t* catbits,
                                hipStream_t stream) {
  hipLaunchKernelGGL(predict_raw_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, X, ld, n,
                     reinterpret_cast<const TreeNode*>(nodes), roots, ntrees, K, out, ldo, catbits);
  return launch_status();
}

H2OMX_API int h2omx_predict_binned(const uint8_t* codes, int64_t npad, int64_t n, const void* nodes,
                                   const int* roots, int ntrees, int K, int nbt, float* out, int64_t ldo,
                                   const uint32_t* catbits, hipStream_t stream) {
  hipLaunchKernelGGL(predict_binned_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, codes, npad, n,
                     reinterpret_cast<const TreeNode*>(nodes), roots, ntrees, K, nbt, out, ldo, catbits);
  return launch_status();
}

// ===========================================================================
// Row-partitioned level pipeline ("segmented" engine).
//
// The scan engine above re-reads every row's node id, gradient and codes
// once per feature group at every level; at depth >= 3 that is ~1 GB of HBM
// traffic per level.  Here the rows of every node live in one contiguous
// segment of a row-index permutation (idx), kept stably partitioned level
// by level (XGBoost-hist / LightGBM style), so a level touches only the rows
// of the nodes it actually builds:
//
//   tree_begin_seg  scales, root segment [0, n), chunk prefixes, zero built
//   hist_build_seg  one workgroup per (row chunk of a built node, feature
//                   group): gathers row-major codes (28 B/row) + g/s by idx,
//                   packed fixed-point u64 LDS atomics, per-chunk slab
//   hist_reduce_seg slabs of each slot -> exact int64 histograms (integer
//                   atomics split over chunk subsets: deterministic)
//   (split_find / level_finalize unchanged)
//   part_count      left-row count per partition chunk
//   level_close     one block: in-node chunk offsets, children segments,
//                   next level's chunk prefixes, zero next built histograms
//   part_scatter    stable in-chunk ranks (wave ballots) -> idx_out, node
//                   ids, and exact leaf sums of retiring rows (block
//                   reduction + 3 integer atomics per chunk: no LDS atomics)
//
// Chunk tables are implicit: per node an exclusive prefix of its chunk
// count (hc_first / pc_first, length n+1); a workgroup finds its node by
// binary search.  Chunk sizes: hist C_h rows (<= ROWS_CAP, fixed-point
// headroom), partition C_p = 4096 rows.
// ===========================================================================
constexpr int PC_ROWS = 4096;

// largest i in [0, n) with first[i] <= c < first[i + 1] (empty nodes sharing
// a prefix value resolve to the last of them), by one wave: a 64-ary search
// (64 parallel probes a round, ~3 dependent loads instead of a binary
// search's ~log2(n)); every lane of the wave must call it
__device__ __forceinline__ int chunk_node_wave(const int* __restrict__ first, int n, int c, int lane) {
  int lo = 0, hi = n - 1;   // answer: the largest i with first[i] <= c (first[0] = 0 <= c)
  while (hi > lo) {
    const int span = hi - lo + 1;
    const int st = (span + 63) >> 6;
    const int i = lo + lane * st;
    const bool ok = i <= hi && first[i] <= c;
    const unsigned long long b = __ballot(ok);
    const int k = 63 - __clzll((long long)b);   // last probe at or below c (lane 0 always is)
    lo = lo + k * st;
    hi = min(hi, lo + st - 1);
    if (st == 1) break;
  }
  return lo;
}

__global__ __launch_bounds__(256) void tree_begin_seg_kernel(
    const unsigned int* __restrict__ stat_max, int mode, double qg, double qsr, double* __restrict__ qs,
    int* __restrict__ ctl0, NodeLink* __restrict__ link0, unsigned long long* __restrict__ leaf_acc, int leaf_n,
    long long* __restrict__ built, int built_n, int n_rows, int hc_rows, int* __restrict__ seg_start,
    int* __restrict__ seg_cnt, int* __restrict__ hc_first, int* __restrict__ pc_first, int* __restrict__ slot_node,
    long long row_base, int tree_index, int* __restrict__ tree_ctr) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < leaf_n; i += gridDim.x * blockDim.x) leaf_acc[i] = 0ull;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < built_n; i += gridDim.x * blockDim.x) built[i] = 0ll;
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  tree_begin_scales(stat_max, mode, qg, qsr, qs, ctl0, link0, row_base, tree_index, tree_ctr);
  seg_start[0] = 0;
  seg_cnt[0] = n_rows;
  hc_first[0] = 0;
  hc_first[1] = (n_rows + hc_rows - 1) / hc_rows;
  pc_first[0] = 0;
  pc_first[1] = (n_rows + PC_ROWS - 1) / PC_ROWS;
  slot_node[0] = 0;
}

// In-bag root segment (HipTreeBuilder.BAG_COMPACT, bagged deep trees): the
// rows of weight 0 - out of this tree's bag (DRF: 37 %) - carry g = s = 0 and
// change no histogram, split or leaf sum, yet every level would read,
// partition and scan them.  The root segment instead holds only rows of
// nonzero weight, ascending (per-chunk counts -> one-workgroup scan ->
// ballot-ordered scatter, deterministic), with their (g, s2) gathered into
// segment order; the dropped rows get their leaf by walking the finished tree
// (bag_route_out_kernel).
constexpr int BAG_CHUNK = 4096;
__global__ __launch_bounds__(256) void bag_count_kernel(const float* __restrict__ w, int64_t n, int* __restrict__ cnt) {
  __shared__ int red[4];
  const int64_t c0 = (int64_t)blockIdx.x * BAG_CHUNK;
  int k = 0;
  for (int i = threadIdx.x; i < BAG_CHUNK; i += 256) {
    const int64_t r = c0 + i;
    k += (r < n && w[r] != 0.0f) ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) k += __shfl_down(k, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = k;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(1024) void bag_scan_kernel(int* __restrict__ cnt, int nch, int* __restrict__ seg_cnt,
                                                        int* __restrict__ hc_first, int* __restrict__ pc_first,
                                                        int hc_rows) {
  __shared__ int sc[1024];
  const int t = threadIdx.x;
  int carry = 0;
  for (int b0 = 0; b0 < nch; b0 += 1024) {
    const int v = b0 + t < nch ? cnt[b0 + t] : 0;
    sc[t] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int x = t >= o ? sc[t - o] : 0;
      __syncthreads();
      sc[t] += x;
      __syncthreads();
    }
    if (b0 + t < nch) cnt[b0 + t] = carry + sc[t] - v;   // exclusive offsets
    carry += sc[1023];
    __syncthreads();
  }
  if (t == 0) {
    seg_cnt[0] = carry;
    hc_first[1] = (carry + hc_rows - 1) / hc_rows;
    pc_first[1] = (carry + PC_ROWS - 1) / PC_ROWS;
  }
}

__global__ __launch_bounds__(256) void bag_scatter_kernel(const float* __restrict__ w, int64_t n,
                                                          const int* __restrict__ off, const float* __restrict__ g,
                                                          const float* __restrict__ s2, int* __restrict__ idx,
                                                          float* __restrict__ gout, float* __restrict__ sout) {
  __shared__ int wc[4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * BAG_CHUNK;
  int base = off[blockIdx.x];
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int i0 = 0; i0 < BAG_CHUNK; i0 += 256) {
    const int64_t r = c0 + i0 + t;
    const bool in = r < n && w[r] != 0.0f;
    const unsigned long long bl = __ballot(in);
    if (lane == 0) wc[wid] = __popcll(bl);
    __syncthreads();
    int before = 0, tot = 0;
    for (int k = 0; k < 4; ++k) {
      if (k < wid) before += wc[k];
      tot += wc[k];
    }
    if (in) {
      const int pos = base + before + __popcll(bl & lt);
      idx[pos] = (int)r;
      gout[pos] = g[r];
      sout[pos] = s2[r];
    }
    base += tot;
    __syncthreads();
  }
}

// the leaf of every row of weight 0 (not in the root segment): walk the
// finished tree on the row-major codes - a row's ~20 code reads hit one line
// (numeric splits; NA code nbt - 1 follows na_left), nid = ~leaf as the
// partitions write it
__global__ __launch_bounds__(256) void bag_route_out_kernel(const float* __restrict__ w, int64_t n,
                                                            const uint8_t* __restrict__ codes_rm, int fp,
                                                            const TreeNode* __restrict__ tree, int nbt,
                                                            int* __restrict__ nid) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (w[r] != 0.0f) continue;
    int node = 0;
    for (int it = 0; it < 64; ++it) {
      const TreeNode nd = tree[node];
      if (nd.feat < 0) break;
      const int b = codes_rm[r * fp + nd.feat];
      const int right = b == nbt - 1 ? !(nd.na_left & 1) : (b > nd.bin ? 1 : 0);
      node = nd.left + right;
    }
    nid[r] = ~node;
  }
}

template <int NBT>
__global__ __launch_bounds__(512) void hist_build_seg_kernel(
    const uint8_t* __restrict__ codes_rm, int fp, const int* __restrict__ idx, const float* __restrict__ g,
    const float* __restrict__ s2, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ hc_first, const int* __restrict__ ctl, const int* __restrict__ nvb,
    const double* __restrict__ qscale, uint32_t salt, int F, int fg, int n_groups, int hc_rows,
    unsigned long long* __restrict__ slab, int gpos, const uint8_t* __restrict__ crow,
    const int* __restrict__ cpos) {
  salt = (uint32_t)qscale[9];  // per-tree dither salt, written by tree_begin (graph-replay safe)
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds64[];
  __shared__ int width_s[256], rep_s[256];
  __shared__ int range_s[2];
  const int n = ctl[CTL_N];
  const int total = hc_first[n];
  const int b = blockIdx.x;
  const int xcd = b & 7, i = b >> 3;
  const int grp = i % n_groups;
  const int c = xcd + 8 * (i / n_groups);
  if (c >= total) return;
  const int f0 = grp * fg;
  const int nf = min(fg, F - f0);
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    const int node = chunk_node_wave(hc_first, n, c, lane);
    if (lane == 0) {
      const int k = c - hc_first[node];
      const int lo = seg_start[node] + k * hc_rows;
      range_s[0] = lo;
      range_s[1] = min(lo + hc_rows, seg_start[node] + seg_cnt[node]);
    }
  }
  for (int j = threadIdx.x; j < fg * NBT; j += blockDim.x) lds64[j] = 0ull;
  bool sliced = false;
  if (threadIdx.x < fg) {
    const int fi = threadIdx.x;
    const int w = (fi < nf) ? nvb[f0 + fi] + 1 : NBT;
    width_s[fi] = w;
    const int r = NBT / w;
    rep_s[fi] = r < 1 ? 1 : (r > 64 ? 64 : r);
    sliced = r > 1;
  }
  const float sg = (float)qscale[0], ss = (float)qscale[1];
  const int64_t rb = (int64_t)qscale[7];  // global row offset of this rank (dither)
  // plain: no feature of the group is replicated - every feature is one
  // NBT-wide slice with NA in its own slot NBT - 1, so the row loop needs no
  // per-feature width / copy lookups (two LDS reads, a wait and a branch per
  // code byte) and loads the row's code words 8 at a time
  const bool plain = !__syncthreads_or(sliced);
  const int lo = range_s[0], hi = range_s[1];
  const int nw = (nf + 3) >> 2;
  for (int j = lo + threadIdx.x; j < hi; j += blockDim.x) {
    const int r = idx ? idx[j] : j;
    const uint32_t hsh = row_hash(rb + r, salt);   // global row id: multi-rank == one rank
    const float d1 = (hsh & 0xFFFF) * (1.0f / 65536.0f), d2 = (hsh >> 16) * (1.0f / 65536.0f);
    const int gi = gpos ? j : r;   // g / s2 stored in segment order (part_scatter) or by row
    const float sv = s2 ? s2[gi] : 1.0f;
    const int gq = (int)floorf(fmaf(g[gi], sg, d1));
    const uint32_t sq = (uint32_t)floorf(fmaf(sv, ss, d2));
    const unsigned long long pk = ((unsigned long long)(uint32_t)gq << 32) | (unsigned long long)sq;
    if (pk == 0ull) continue;
    const uint32_t* row = reinterpret_cast<const uint32_t*>(
        (crow ? crow + (int64_t)(cpos ? cpos[j] : j) * fp : codes_rm + (int64_t)r * fp) + f0);
    if (plain) {
      for (int w0 = 0; w0 < nw; w0 += 8) {
        uint32_t c8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c8[u] = (w0 + u < nw) ? row[w0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int fi = 4 * (w0 + u) + k;
            if (fi < nf) atomicAdd(lds64 + fi * NBT + ((c8[u] >> (8 * k)) & 0xff), pk);
          }
        }
      }
      continue;
    }
    for (int wq = 0; wq < nw; ++wq) {
      const uint32_t cw = row[wq];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int fi = 4 * wq + k;
        if (fi < nf) {
          const int width = width_s[fi];
          int bin = (cw >> (8 * k)) & 0xff;
          if (bin == NBT - 1) bin = width - 1;  // NA -> last slot of the feature slice
          const int copy_off = (rep_s[fi] > 1) ? (lane % rep_s[fi]) * width : 0;
          atomicAdd(lds64 + fi * NBT + copy_off + bin, pk);
        }
      }
    }
  }
  __syncthreads();
  unsigned long long* out = slab + ((int64_t)c * n_groups + grp) * fg * NBT;
  for (int j = threadIdx.x; j < fg * NBT; j += blockDim.x) {
    if (plain) {   // one slice per feature, NA in its own slot
      out[j] = lds64[j];
      continue;
    }
    const int bin = j % NBT, fi = j / NBT;
    const int width = width_s[fi], rep = rep_s[fi];
    const int src = (bin == NBT - 1) ? width - 1 : bin;
    unsigned long long acc = 0ull;
    if (src < width - 1 || bin == NBT - 1) {
      const unsigned long long* hb = lds64 + fi * NBT;
      for (int cc = 0; cc < rep; ++cc) acc += hb[cc * width + src];
    }
    out[j] = acc;
  }
}

// built[s][F][2][NBT] += sum over the slot's chunks (subset blockIdx.z of K)
__global__ __launch_bounds__(256) void hist_reduce_seg_kernel(const unsigned long long* __restrict__ slab,
                                                              const int* __restrict__ hc_first,
                                                              const int* __restrict__ slot_node,
                                                              const int* __restrict__ ctl, int F, int nbt, int fg,
                                                              int n_groups, long long* __restrict__ built) {
  const int s = blockIdx.y;
  if (s >= ctl[CTL_SLOTS]) return;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= F * nbt) return;
  const int f = e / nbt, bin = e % nbt;
  const int grp = f / fg, fi = f % fg;
  const int node = slot_node[s];
  const int c0 = hc_first[node], c1 = hc_first[node + 1];
  const int K = gridDim.z;
  long long ag = 0, as = 0;
  const int64_t stride = (int64_t)n_groups * fg * nbt;
  const unsigned long long* p = slab + (int64_t)grp * fg * nbt + (int64_t)fi * nbt + bin;
  for (int c = c0 + (int)blockIdx.z; c < c1; c += K) {
    const unsigned long long v = p[(int64_t)c * stride];
    ag += (long long)(int32_t)(uint32_t)(v >> 32);
    as += (long long)(uint32_t)v;
  }
  long long* o = built + (((int64_t)s * F + f) * 2) * nbt + bin;
  if (ag) atomicAdd(reinterpret_cast<unsigned long long*>(o), (unsigned long long)ag);
  if (as) atomicAdd(reinterpret_cast<unsigned long long*>(o + nbt), (unsigned long long)as);
}

__device__ __forceinline__ int split_dir(const uint8_t* __restrict__ codes, int64_t npad, const PartInfo& pi,
                                         int nbt, int r) {
  const int b = codes[(int64_t)pi.feat * npad + r];
  return part_right(pi, b, nbt);
}

// Row-major code rows kept in segment order (segmented engine):
// in = this level's rows by segment position j (nullptr: gather codes_rm by row
// id), out = the next level's (part_scatter moves every inner row's fp bytes
// with it), so deep levels read their nodes' rows contiguously instead of one
// random cache line per row
struct SegRows {
  const uint8_t* in;
  uint8_t* out;
  int fp;
  const int* cpos_in;   // row j's position in `in` (nullptr = j)
  int* cpos_out;        // rows stay put: the next level's positions (moved like idx)
};

// The wave's rows (lane i: row r / segment position j -> segment position dst,
// dst < 0 = nothing to move) copied cooperatively: consecutive lanes move
// consecutive 4-byte words of one row, so the reads (rows j contiguous) and
// the writes (left / right children are two order-preserving runs) coalesce.
// Called by every lane of the wave.
__device__ __forceinline__ void seg_move_rows_wave(const SegRows& sr, const uint8_t* __restrict__ codes_rm, int r,
                                                   int j, int dst) {
  const int lane = threadIdx.x & 63;
  const unsigned long long act = __ballot(dst >= 0);
  if (act == 0ull) return;
  const int nr = 64 - __clzll((long long)act);   // rows of lanes [0, nr)
  const int W = sr.fp >> 2;
  for (int base = 0; base < nr * W; base += 64) {
    const int q = base + lane;
    const int i = min(q / W, 63), k = q - (q / W) * W;
    const int di = __shfl(dst, i, kWave), ri = __shfl(r, i, kWave), ji = __shfl(j, i, kWave);
    if (q < nr * W && di >= 0) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(sr.in ? sr.in + (int64_t)ji * sr.fp
                                                                    : codes_rm + (int64_t)ri * sr.fp);
      reinterpret_cast<uint32_t*>(sr.out + (int64_t)di * sr.fp)[k] = src[k];
    }
  }
}

__device__ __forceinline__ int seg_split_dir(const uint8_t* __restrict__ codes, int64_t npad, const PartInfo& pi,
                                             int nbt, int r, int j, const SegRows& sr) {
  if (sr.in != nullptr)
    return part_right(pi, sr.in[(int64_t)(sr.cpos_in ? sr.cpos_in[j] : j) * sr.fp + pi.feat], nbt);
  return split_dir(codes, npad, pi, nbt, r);
}

// number of rows of chunk c going left (nodes that split into inner nodes);
// dirb (optional, indexed like idx): every split node's row directions, so
// part_scatter moves rows without gathering their split codes again
__global__ __launch_bounds__(256) void part_count_kernel(const uint8_t* __restrict__ codes, int64_t npad,
                                                         const int* __restrict__ idx, const int* __restrict__ seg_start,
                                                         const int* __restrict__ seg_cnt,
                                                         const int* __restrict__ pc_first, const int* __restrict__ ctl,
                                                         const PartInfo* __restrict__ part, int nbt,
                                                         int* __restrict__ pc_left, SegRows sr,
                                                         int8_t* __restrict__ dirb) {
  __shared__ int red[4];
  const int n = ctl[CTL_N];
  const int c = blockIdx.x;
  if (c >= pc_first[n]) return;
  const int node = chunk_node_wave(pc_first, n, c, threadIdx.x & 63);   // every wave (uniform answer)
  const PartInfo pi = part[node];
  int cnt = 0;
  if (pi.child >= 0 && (dirb != nullptr || !pi.leaf_children)) {
    const int lo = seg_start[node] + (c - pc_first[node]) * PC_ROWS;
    const int hi = min(lo + PC_ROWS, seg_start[node] + seg_cnt[node]);
    // four rows per thread in flight: their row ids, then their code gathers
    const int bs = blockDim.x;
    int j = lo + threadIdx.x;
    for (; j + 3 * bs < hi; j += 4 * bs) {
      int r4[4], d4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) r4[u] = idx ? idx[j + u * bs] : j + u * bs;
#pragma unroll
      for (int u = 0; u < 4; ++u) d4[u] = seg_split_dir(codes, npad, pi, nbt, r4[u], j + u * bs, sr);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (dirb) dirb[j + u * bs] = (int8_t)d4[u];
        cnt += 1 - d4[u];
      }
    }
    for (; j < hi; j += bs) {
      const int r = idx ? idx[j] : j;
      const int d = seg_split_dir(codes, npad, pi, nbt, r, j, sr);
      if (dirb) dirb[j] = (int8_t)d;
      cnt += 1 - d;
    }
    if (pi.leaf_children) cnt = 0;   // only inner splits count
  }
  cnt = (int)wave_sum((float)cnt);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) pc_left[c] = red[0] + red[1] + red[2] + red[3];
}

// Single block: offsets of every chunk's left rows inside its node, node
// left totals, children segments, the next level's chunk prefixes and slot
// map, and zeroed next-level histograms.
__global__ __launch_bounds__(1024) void level_close_kernel(
    const int* __restrict__ ctl, const int* __restrict__ ctl_next, const PartInfo* __restrict__ part,
    const NodeLink* __restrict__ link_next, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ pc_first, int* __restrict__ pc_left /* in: counts, out: in-node offsets */,
    int* __restrict__ node_nl, int* __restrict__ nseg_start, int* __restrict__ nseg_cnt,
    int* __restrict__ nhc_first, int* __restrict__ npc_first, int* __restrict__ nslot_node, int hc_rows,
    long long* __restrict__ nbuilt, int per_slot) {
  __shared__ int wsum[16];
  __shared__ int carry_s[2];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int n = ctl[CTL_N];
  const int total = pc_first[n];
  // (a) global exclusive scan of left counts
  if (t == 0) carry_s[0] = 0;
  __syncthreads();
  for (int c0 = 0; c0 < total; c0 += blockDim.x) {
    const int c = c0 + t;
    const int v = c < total ? pc_left[c] : 0;
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    int before = carry_s[0];
    for (int k = 0; k < wid; ++k) before += wsum[k];
    if (c < total) pc_left[c] = before + x - v;
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) tot += wsum[k];
      carry_s[0] += tot;
    }
    __syncthreads();
  }
  const int grand = carry_s[0];
  // (b) node left totals (node_nl) and node bases (kept in nseg_cnt temporarily is unsafe: use node_nl[n + i])
  for (int i = t; i < n; i += blockDim.x) {
    const int a = pc_first[i], z = pc_first[i + 1];
    const int base = a < total ? pc_left[a] : grand;
    const int end = z < total ? pc_left[z] : grand;
    node_nl[i] = end - base;
    node_nl[n + i] = base;
  }
  __syncthreads();
  // chunks of node i are [pc_first[i], pc_first[i+1]): node-parallel rebase
  // (a binary search per chunk costs ~17 dependent loads at 10^5 nodes); few
  // nodes own thousands of chunks each (10M rows at the root: 2441 chunks, one
  // thread walking them took 157 us), so they rebase with the whole block
  if (n <= 64) {
    for (int i = 0; i < n; ++i) {
      const int base = node_nl[n + i];
      for (int c = pc_first[i] + t; c < pc_first[i + 1]; c += blockDim.x) pc_left[c] -= base;
    }
  } else {
    for (int i = t; i < n; i += blockDim.x) {
      const int base = node_nl[n + i];
      for (int c = pc_first[i]; c < pc_first[i + 1]; ++c) pc_left[c] -= base;
    }
  }
  // (c) children segments
  for (int i = t; i < n; i += blockDim.x) {
    const PartInfo pi = part[i];
    if (pi.child >= 0 && !pi.leaf_children) {
      const int nl = node_nl[i];
      nseg_start[pi.child] = seg_start[i];
      nseg_cnt[pi.child] = nl;
      nseg_start[pi.child + 1] = seg_start[i] + nl;
      nseg_cnt[pi.child + 1] = seg_cnt[i] - nl;
    }
  }
  __syncthreads();
  // (d) next level chunk prefixes + slot map
  const int nn = ctl_next[CTL_N];
  if (t == 0) { carry_s[0] = 0; carry_s[1] = 0; }
  __syncthreads();
  for (int j0 = 0; j0 < nn; j0 += blockDim.x) {
    const int j = j0 + t;
    int hcv = 0, pcv = 0;
    if (j < nn) {
      const int cnt = nseg_cnt[j];
      const NodeLink L = link_next[j];
      hcv = (L.slot >= 0) ? (cnt + hc_rows - 1) / hc_rows : 0;
      pcv = (cnt + PC_ROWS - 1) / PC_ROWS;
      if (L.slot >= 0) nslot_node[L.slot] = j;
    }
    // pack both counts in one 32-bit scan (each < 2^16 per block pass is not
    // guaranteed) -> two scans
    int xh = hcv, xp = pcv;
    for (int o = 1; o < 64; o <<= 1) {
      const int yh = __shfl_up(xh, o, 64), yp = __shfl_up(xp, o, 64);
      if (lane >= o) { xh += yh; xp += yp; }
    }
    __shared__ int wh[16], wp[16];
    if (lane == 63) { wh[wid] = xh; wp[wid] = xp; }
    __syncthreads();
    int bh = carry_s[0], bp = carry_s[1];
    for (int k = 0; k < wid; ++k) { bh += wh[k]; bp += wp[k]; }
    if (j < nn) { nhc_first[j] = bh + xh - hcv; npc_first[j] = bp + xp - pcv; }
    __syncthreads();
    if (t == 0) {
      int th = 0, tp = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { th += wh[k]; tp += wp[k]; }
      carry_s[0] += th; carry_s[1] += tp;
    }
    __syncthreads();
  }
  if (t == 0) { nhc_first[nn] = carry_s[0]; npc_first[nn] = carry_s[1]; }
  // (e) the next level's built histograms are zeroed by zero_slots_kernel over
  // the whole chip (13-26 MB at DRF levels 8-9: 186 / 356 us in this one block)
}

// --- multi-block level close (levels with thousands of nodes) --------------
// A single-block level_close scans ~10^5 chunks / nodes with block barriers
// per 1024 entries (2.6 ms per deep DRF level); here the same work is a
// device-wide 3-phase exclusive scan plus node-parallel kernels.
constexpr int SCAN_TILE = 1024;

// aux[0] = partition chunks of this level, aux[1] = next-level nodes
__global__ void close_prep_kernel(const int* __restrict__ ctl, const int* __restrict__ ctl_next,
                                  const int* __restrict__ pc_first, int* __restrict__ aux) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    aux[0] = pc_first[ctl[CTL_N]];
    aux[1] = ctl_next[CTL_N];
  }
}

__device__ __forceinline__ int block_excl_scan_1024(int v, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  int before = 0;
  total = 0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
    if (k < wid) before += wsum[k];
    total += wsum[k];
  }
  return before + x - v;
}

// phase 1: per-tile exclusive scan of in[0 .. aux[k]) -> out, tile totals -> tiles
__global__ __launch_bounds__(SCAN_TILE) void scan_tiles_kernel(const int* __restrict__ in, int* __restrict__ out,
                                                               int* __restrict__ tiles, const int* __restrict__ aux,
                                                               int k) {
  __shared__ int wsum[16];
  const int count = aux[k];
  const int i = blockIdx.x * SCAN_TILE + threadIdx.x;
  if (blockIdx.x * SCAN_TILE >= count) return;  // uniform per block
  const int v = i < count ? in[i] : 0;
  int total;
  const int e = block_excl_scan_1024(v, wsum, total);
  if (i < count) out[i] = e;
  if (threadIdx.x == 0) tiles[blockIdx.x] = total;
}

// phase 2 (one block): exclusive scan of the tile totals; grand total -> out[count] and total_out
__global__ __launch_bounds__(SCAN_TILE) void scan_tile_sums_kernel(int* __restrict__ tiles, int* __restrict__ out,
                                                                   const int* __restrict__ aux, int k,
                                                                   int* __restrict__ total_out) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int count = aux[k];
  const int nt = (count + SCAN_TILE - 1) / SCAN_TILE;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int t0 = 0; t0 < nt; t0 += SCAN_TILE) {
    const int t = t0 + threadIdx.x;
    const int v = t < nt ? tiles[t] : 0;
    int total;
    const int e = block_excl_scan_1024(v, wsum, total);
    if (t < nt) tiles[t] = carry + e;
    __syncthreads();
    if (threadIdx.x == 0) carry += total;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (out) out[count] = carry;
    if (total_out) *total_out = carry;
  }
}

// phase 3: add tile offsets
__global__ __launch_bounds__(SCAN_TILE) void scan_add_kernel(int* __restrict__ out, const int* __restrict__ tiles,
                                                             const int* __restrict__ aux, int k) {
  const int count = aux[k];
  const int i = blockIdx.x * SCAN_TILE + threadIdx.x;
  if (i < count) out[i] += tiles[blockIdx.x];
}

// node-parallel part of level_close: left totals, in-node chunk offsets,
// children segments, next-level chunk counts and slot map
__global__ __launch_bounds__(256) void node_close_kernel(
    const int* __restrict__ ctl, const PartInfo* __restrict__ part, const NodeLink* __restrict__ link_next,
    const int* __restrict__ seg_start, const int* __restrict__ seg_cnt, const int* __restrict__ pc_first,
    const int* __restrict__ pc_excl, const int* __restrict__ aux, int* __restrict__ pc_off,
    int* __restrict__ node_nl, int* __restrict__ nseg_start, int* __restrict__ nseg_cnt, int* __restrict__ cnt_h,
    int* __restrict__ cnt_p, int* __restrict__ nslot_node, int hc_rows) {
  const int n = ctl[CTL_N];
  const int total = aux[0], grand = aux[2];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int a = pc_first[i], z = pc_first[i + 1];
    const int base = a < total ? pc_excl[a] : grand;
    const int end = z < total ? pc_excl[z] : grand;
    const int nl = end - base;
    node_nl[i] = nl;
    for (int c = a; c < z; ++c) pc_off[c] = pc_excl[c] - base;
    const PartInfo pi = part[i];
    if (pi.child >= 0 && !pi.leaf_children) {
      const int cl = pi.child, cr = pi.child + 1;
      const int cntl = nl, cntr = seg_cnt[i] - nl;
      nseg_start[cl] = seg_start[i];
      nseg_cnt[cl] = cntl;
      nseg_start[cr] = seg_start[i] + nl;
      nseg_cnt[cr] = cntr;
      const NodeLink L = link_next[cl], R = link_next[cr];
      cnt_h[cl] = L.slot >= 0 ? (cntl + hc_rows - 1) / hc_rows : 0;
      cnt_h[cr] = R.slot >= 0 ? (cntr + hc_rows - 1) / hc_rows : 0;
      cnt_p[cl] = (cntl + PC_ROWS - 1) / PC_ROWS;
      cnt_p[cr] = (cntr + PC_ROWS - 1) / PC_ROWS;
      if (L.slot >= 0) nslot_node[L.slot] = cl;
      if (R.slot >= 0) nslot_node[R.slot] = cr;
    }
  }
}

// ---------------------------------------------------------------------------
// Deep levels, direct mode (segmented engine): one workgroup per node builds
// the histograms of the node's ELIGIBLE features only (mtries / column
// sampling / per-tree mask, the same hash ranks as split_find) straight from
// the node's rows and scans them in LDS - no parent histograms, no sibling
// subtraction, no histogram ever written to global memory.  At depth 10-20
// the subtraction machinery moved nodes x F x bins int64 rows per level
// (split_find copying parents, hist_reduce, zero_slots: ~15 ms at level 18 of
// DRF 10M x 100, profiles/drf_depth20_level_breakdown.txt) while the rows of
// all nodes are only n x (eligible F) bytes.  Exact int64 sums of the same
// quantised rows: bit-identical splits to the subtraction path.  Writes the
// node's NodeSplit directly (level_finalize_ns follows).
// ---------------------------------------------------------------------------
constexpr int DIRECT_LDS_BYTES = 96 * 1024;   // histogram batch (G and S int64 planes)
constexpr int DIRECT_WAVES = 4;   // waves per node workgroup (<= 4)
// Nodes with fewer rows than this accumulate ONE packed 64-bit LDS atomic per
// (row, feature) - (int32 G_q << 32) + uint32 S_q, as hist_build_kernel - instead
// of a G and an S plane: per-row |G_q| <= 2^15 and S_q <= 2^16 keep |sum G_q| <
// 2^31 and sum S_q < 2^32, so the halves never carry into each other.
constexpr int DIRECT_PACK_ROWS = 65536;

struct DirectBest {
  double gain, GL, SL;
  long long key;   // (feature << 32 | code), smallest wins ties; LLONG_MAX = none
};

// Per-lane running best over every feature a wave scans: one wave arg-max per
// node (lane_best_reduce) instead of one per feature.  key = f * 1024 + code
// (code = 2 * bin + na_left < 1024, f < 1024): ordered like DirectBest::key, so
// (max gain, smallest key) over lanes is the sequential per-feature result.
struct LaneBest {
  double gain, GL, SL;
  int key;   // INT_MAX = none
};

__device__ __forceinline__ void lane_best_init(LaneBest& b) {
  b.gain = -INFINITY; b.GL = b.SL = 0.0; b.key = 0x7fffffff;
}

// every lane of the wave returns the wave's best (called by all 64 lanes)
__device__ __forceinline__ DirectBest lane_best_reduce(const LaneBest& lb) {
  double g = lb.gain;
  int k = lb.key;
  wave_argmax(g, k);
  DirectBest r;
  r.gain = -INFINITY; r.GL = r.SL = 0.0; r.key = 0x7fffffffffffffffLL;
  if (k != 0x7fffffff) {
    const unsigned long long own = __ballot(lb.key == k);   // keys are unique per lane
    const int src = __builtin_amdgcn_readfirstlane(__ffsll((long long)own) - 1);
    r.gain = g;
    r.GL = readlane_f64(lb.GL, src);
    r.SL = readlane_f64(lb.SL, src);
    r.key = ((long long)(k >> 10) << 32) | (unsigned)(k & 1023);
  }
  return r;
}

// the split scan of one feature's LDS histogram by one wave (split_find's
// feat_best_wave on exact int64 rows) into the lanes' running bests; PACKED:
// one packed u64 per bin, scanned as ONE int64 prefix sum ((int32 G_q << 32) +
// uint32 S_q: the node's S_q sum stays below 2^32 - the packed-atomics bound -
// so the halves never carry and both prefix sums are exact)
template <int NBT, bool PACKED>
__device__ __forceinline__ void direct_scan_feature(const long long* __restrict__ h, int node, int f, int m,
                                                    double ig, double is, const SplitParams& p, int lane,
                                                    LaneBest& lb, double& ptc, double* cut_tab) {
  constexpr int B = NBT <= 64 ? 1 : NBT / 64;
  constexpr int NA_LANE = (NBT - 1) / B, NA_K = (NBT - 1) % B;
  long long gi[B], si[B];
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int bin = lane * B + k;
    gi[k] = 0; si[k] = 0;
    if (bin < NBT) {
      if constexpr (PACKED) {
        const unsigned long long v = (unsigned long long)h[bin];
        gi[k] = (long long)(int)(uint32_t)(v >> 32);
        si[k] = (long long)(uint32_t)v;
      } else {
        gi[k] = h[bin];
        si[k] = h[NBT + bin];
      }
    }
  }
  const long long ng_i = readlane_i64(gi[NA_K], NA_LANE), ns_i = readlane_i64(si[NA_K], NA_LANE);
  if (lane == NA_LANE) { gi[NA_K] = 0; si[NA_K] = 0; }
  long long lg = 0, ls = 0;
  long long pg[B], ps[B];
#pragma unroll
  for (int k = 0; k < B; ++k) { lg += gi[k]; ls += si[k]; pg[k] = lg; ps[k] = ls; }
  long long xg, xs;
  if constexpr (PACKED) {
    const long long xp = wave_incl_scan_i64((long long)(((unsigned long long)(uint32_t)(int)lg << 32) +
                                                        (unsigned long long)(uint32_t)ls));
    xg = (long long)(int)(uint32_t)((unsigned long long)xp >> 32);
    xs = (long long)(uint32_t)(unsigned long long)xp;
  } else {
    xg = wave_incl_scan_i64(lg);
    xs = wave_incl_scan_i64(ls);
  }
  const long long tg_i = readlane_i64(xg, 63) + ng_i, ts_i = readlane_i64(xs, 63) + ns_i;
  const long long eg = xg - lg, es = xs - ls;
  const double ng = (double)ng_i * ig, ns = (double)ns_i * is;
  const double tg = (double)tg_i * ig, ts = (double)ts_i * is;
  double fbg = -INFINITY;
  int fbc = 0x7fffffff;
  double fGL = 0, fSL = 0;
  const int mf = p.mono ? (int)p.mono[f] : 0;
  const uint32_t cand = p.hist_mode ? adaptive_candidates<NBT, B>(si, m, node, f, p, cut_tab) : 0xffffffffu;
  // (tg, ts) are the node's exact totals, the same for every feature of the node:
  // its parent term is computed by the first feature scanned (ptc NaN before)
  if (ptc != ptc) ptc = parent_term(tg, ts, p);
  const double pt = ptc;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int tt = lane * B + k;
    if (tt < m && tt < NBT - 1 && ((cand >> k) & 1u)) {
      const double sgd = (double)(eg + pg[k]) * ig, ssum = (double)(es + ps[k]) * is;
      const double gA = mono_ok(mf, sgd, ssum, tg, ts, p) ? split_gain_pt(sgd, ssum, tg, ts, pt, p) : -INFINITY;
      const double gB = (ns > 0.0 && mono_ok(mf, sgd + ng, ssum + ns, tg, ts, p))
                            ? split_gain_pt(sgd + ng, ssum + ns, tg, ts, pt, p) : -INFINITY;
      if (gA > -INFINITY && (gA > fbg || (gA == fbg && 2 * tt < fbc))) { fbg = gA; fbc = 2 * tt; fGL = sgd; fSL = ssum; }
      if (gB > -INFINITY && (gB > fbg || (gB == fbg && 2 * tt + 1 < fbc))) {
        fbg = gB; fbc = 2 * tt + 1; fGL = sgd + ng; fSL = ssum + ns;
      }
    }
  }
  if (fbc != 0x7fffffff) {
    const int key = f * 1024 + fbc;
    if (fbg > lb.gain || (fbg == lb.gain && key < lb.key)) { lb.gain = fbg; lb.key = key; lb.GL = fGL; lb.SL = fSL; }
  }
}

__device__ __forceinline__ NodeSplit direct_node_split(const DirectBest& b, long long tgq, long long tsq, double ig,
                                                       double is) {
  NodeSplit sp;
  sp.G = (double)tgq * ig; sp.H = (double)tsq * is; sp.W = sp.H;
  sp.pad = 0;
  if (b.key != 0x7fffffffffffffffLL) {
    sp.gain = b.gain; sp.GL = b.GL; sp.HL = b.SL; sp.WL = b.SL;
    sp.feat = (int)(b.key >> 32); const int code = (int)(b.key & 0xffffffff);
    sp.bin = code >> 1; sp.na_left = code & 1;
  } else {
    sp.gain = -INFINITY; sp.GL = sp.HL = sp.WL = 0.0; sp.feat = -1; sp.bin = 0; sp.na_left = 0;
  }
  return sp;
}

// per-row quantised statistics, the same dither as every histogram path
// (gi: index of the row's g / s2 - its segment position when part_scatter
// keeps them in segment order, else the row id)
__device__ __forceinline__ void direct_row_q(int r, int gi, int64_t rb, uint32_t salt, const float* __restrict__ g,
                                             const float* __restrict__ s2, float sg, float ss, long long& gq,
                                             long long& sq) {
  const uint32_t hsh = row_hash(rb + r, salt);
  const float d1 = (hsh & 0xFFFF) * (1.0f / 65536.0f), d2 = (hsh >> 16) * (1.0f / 65536.0f);
  const float sv = s2 ? s2[gi] : 1.0f;
  gq = (long long)(int)floorf(fmaf(g[gi], sg, d1));
  sq = (long long)(uint32_t)floorf(fmaf(sv, ss, d2));
}

// one row's atomics for features flist[0, nb) of the batch: the code bytes of
// DIRECT_FB features are loaded together (independent loads in flight) before
// their atomics - a load -> atomic chain per feature left each node's rows
// waiting on nb serial HBM round trips.  c0: codes of the first chunk,
// already loaded by the caller (issued before the gradient loads resolve).
// Eligible-feature codes kept for the partition (nodes of few eligible
// features, e.g. DRF mtries): the direct pass already loads every row's codes
// of the node's eligible features, so it also stores them in segment order
// (codes[j * stride + q], q = index in the node's feature list) and the index
// of the chosen feature per node (nodeq); part_count / part_scatter then read
// one byte at the row's segment position instead of gathering a byte from
// the 10M-row feature column at a random row.
struct ECodes {
  uint8_t* codes;   // nullptr = off; the host enables it only when the node's features fit one batch
  int stride;       // 8 or 16 bytes per row
  int* nodeq;
  const uint8_t* crow;   // code rows in segment order (SegRows::in), nullptr = gather codes_rm by row id
  const int* cpos;       // row j's position in crow (rows moved once, then only positions), nullptr = j
  // crow layout: row-major rows (rs = fp, fs = 1) or column-major feature
  // planes (rs = 1, fs = plane positions; seg_colmajor_kernel): the code of
  // feature f at position q is crow[q * rs + f * fs]
  int rs;
  int64_t fs;
};

// XCD-aware block order: dispatch puts block b on XCD b % 8; renumber so XCD x
// takes the contiguous range [x * g / 8, (x + 1) * g / 8) - neighbouring
// nodes (descendants of one ancestor, whose code rows sit together once the
// rows were moved) then share an L2.  g must be a multiple of 8 (the host pads).
__device__ __forceinline__ int xcd_block(int b, int g) {
  return ((g & 7) == 0) ? (b & 7) * (g >> 3) + (b >> 3) : b;
}

template <typename FL>
__device__ __forceinline__ int direct_feat_pos(const FL* flist, int nfl, long long key) {
  if (key == 0x7fffffffffffffffLL) return -1;
  const int f = (int)(key >> 32);
  for (int q = 0; q < nfl; ++q)
    if ((int)flist[q] == f) return q;
  return -1;
}

constexpr int DIRECT_FB = 8;
template <int NBT>
__device__ __forceinline__ void direct_chunk_atomics(int q0, int nb, bool packed, int per_f, long long* hist,
                                                     unsigned long long pk, long long gq, long long sq,
                                                     const uint32_t* c) {
  if (packed) {
#pragma unroll
    for (int u = 0; u < DIRECT_FB; ++u)
      if (q0 + u < nb) atomicAdd(reinterpret_cast<unsigned long long*>(hist + (q0 + u) * NBT + c[u]), pk);
  } else {
#pragma unroll
    for (int u = 0; u < DIRECT_FB; ++u) {
      if (q0 + u < nb) {
        unsigned long long* hb = reinterpret_cast<unsigned long long*>(hist + (q0 + u) * per_f + c[u]);
        atomicAdd(hb, (unsigned long long)gq);
        atomicAdd(hb + NBT, (unsigned long long)sq);
      }
    }
  }
}

// erow (ECodes, nb <= 16): the row's codes of the node's features stored as
// ONE 8- or 16-byte vector (estride) at its segment position
template <int NBT, typename FL>
__device__ __forceinline__ void direct_row_atomics(const uint8_t* __restrict__ row, int64_t fs, const FL* flist, int nb,
                                                   bool packed, int per_f, long long* hist, long long gq, long long sq,
                                                   const uint32_t* c0, uint8_t* erow, int estride) {
  const bool live = gq != 0 || sq != 0;
  if (!live && erow == nullptr) return;
  const unsigned long long pk = ((unsigned long long)(uint32_t)(int)gq << 32) | (unsigned long long)sq;
  uint32_t c1[DIRECT_FB];
#pragma unroll
  for (int u = 0; u < DIRECT_FB; ++u) c1[u] = (DIRECT_FB + u < nb) ? row[flist[DIRECT_FB + u] * fs] : 0u;
  if (erow) {
    const uint32_t w0 = c0[0] | (c0[1] << 8) | (c0[2] << 16) | (c0[3] << 24);
    const uint32_t w1 = c0[4] | (c0[5] << 8) | (c0[6] << 16) | (c0[7] << 24);
    if (estride == 16) {
      const uint32_t w2 = c1[0] | (c1[1] << 8) | (c1[2] << 16) | (c1[3] << 24);
      const uint32_t w3 = c1[4] | (c1[5] << 8) | (c1[6] << 16) | (c1[7] << 24);
      *reinterpret_cast<uint4*>(erow) = make_uint4(w0, w1, w2, w3);
    } else {
      *reinterpret_cast<uint2*>(erow) = make_uint2(w0, w1);
    }
  }
  if (!live) return;
  direct_chunk_atomics<NBT>(0, nb, packed, per_f, hist, pk, gq, sq, c0);
  if (nb > DIRECT_FB) direct_chunk_atomics<NBT>(DIRECT_FB, nb, packed, per_f, hist, pk, gq, sq, c1);
  uint32_t c[DIRECT_FB];
  for (int q0 = 2 * DIRECT_FB; q0 < nb; q0 += DIRECT_FB) {
#pragma unroll
    for (int u = 0; u < DIRECT_FB; ++u) c[u] = (q0 + u < nb) ? row[flist[q0 + u] * fs] : 0u;
    direct_chunk_atomics<NBT>(q0, nb, packed, per_f, hist, pk, gq, sq, c);
  }
}

template <typename FL>
__device__ __forceinline__ int direct_eligible(int node, int gid_i, const SplitParams& p,
                                              const uint8_t* __restrict__ tree_fmask, FL* flist, uint32_t* hsh_s,
                                              int lane);

template <int NBT>
__global__ __launch_bounds__(256) void seg_direct_kernel(
    const uint8_t* __restrict__ codes_rm, int fp, const int* __restrict__ idx, const float* __restrict__ g,
    const float* __restrict__ s2, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ ctl, const int* __restrict__ nvb, const uint8_t* __restrict__ tree_fmask,
    const double* __restrict__ qscale, uint32_t salt, SplitParams p, int batch, NodeSplit* __restrict__ out,
    int gpos, ECodes ec) {
  salt = (uint32_t)qscale[9];  // per-tree dither salt, written by tree_begin (graph-replay safe)
  extern __shared__ __attribute__((aligned(16))) long long hist[];   // [batch][2][NBT] (packed: [batch][NBT])
  __shared__ int flist[1024];
  __shared__ uint32_t hsh_s[1024];
  __shared__ int nfl_s;
  __shared__ long long tot_s[2][4];
  __shared__ double wb_gain[4], wb_GL[4], wb_SL[4];
  __shared__ long long wb_key[4];
  __shared__ double cut_s[4][64];   // per-wave UniformAdaptive cut tables
  const int node = ec.crow ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  if (node >= ctl[CTL_N]) return;
  const int F = p.F;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int lo = seg_start[node], cnt = seg_cnt[node];
  const int gid_i = ctl[CTL_BASE] + node;   // interaction-constraint state
  // eligible features of this node (wave 0), in ascending order: the mtries
  // smallest (hash, index) keys, as split_find
  if (wid == 0) {
    const int c = direct_eligible(node, gid_i, p, tree_fmask, flist, hsh_s, lane);
    if (lane == 0) nfl_s = c < 1024 ? c : 1024;
  }
  if (t < 8) tot_s[t >> 2][t & 3] = 0;
  __syncthreads();
  const int nfl = nfl_s;
  const float sg = (float)qscale[0], ss = (float)qscale[1];
  const double ig = qscale[2], is = qscale[3];
  const int64_t rb = (int64_t)qscale[7];
  const bool packed = cnt < DIRECT_PACK_ROWS;                 // block-uniform
  const int per_f = packed ? NBT : 2 * NBT;                   // int64 entries per feature
  const int bat = packed ? 2 * batch : batch;                 // same LDS bytes
  LaneBest lb;
  lane_best_init(lb);
  double ptc = NAN;   // the node's parent gain term (direct_scan_feature)
  long long tg_row = 0, ts_row = 0;   // node totals (G_q, S_q), accumulated in the first batch
  // eligible-code rows only for nodes scanned in ONE batch (the partition falls
  // back to the code rows for the others: nodeq -1)
  uint8_t* const ecw = (ec.codes && nfl <= bat) ? ec.codes : nullptr;
  for (int b0 = 0; b0 < nfl; b0 += bat) {
    const int nb = min(bat, nfl - b0);
    for (int j = t; j < nb * per_f; j += blockDim.x) hist[j] = 0;
    __syncthreads();
    for (int j = lo + t; j < lo + cnt; j += blockDim.x) {
      const int r = idx ? idx[j] : j;
      const uint8_t* row = ec.crow ? ec.crow + (int64_t)(ec.cpos ? ec.cpos[j] : j) * ec.rs : codes_rm + (int64_t)r * fp;
      const int64_t fs = ec.crow ? ec.fs : 1;
      uint32_t c0[DIRECT_FB];
#pragma unroll
      for (int u = 0; u < DIRECT_FB; ++u) c0[u] = (u < nb) ? row[flist[b0 + u] * fs] : 0u;
      long long gq, sq;
      direct_row_q(r, gpos ? j : r, rb, salt, g, s2, sg, ss, gq, sq);
      if (b0 == 0) { tg_row += gq; ts_row += sq; }
      direct_row_atomics<NBT>(row, fs, flist + b0, nb, packed, per_f, hist, gq, sq, c0,
                              ecw ? ecw + (int64_t)j * ec.stride : nullptr, ec.stride);
    }
    __syncthreads();
    if (b0 == 0) {
      tg_row = wave_sum_i64(tg_row);
      ts_row = wave_sum_i64(ts_row);
      if (lane == 0) { tot_s[0][wid] = tg_row; tot_s[1][wid] = ts_row; }
    }
    // one wave per feature of the batch
    for (int q = wid; q < nb; q += DIRECT_WAVES) {
      const int f = flist[b0 + q];
      if (packed) direct_scan_feature<NBT, true>(hist + q * per_f, node, f, nvb[f], ig, is, p, lane, lb, ptc, cut_s[wid]);
      else direct_scan_feature<NBT, false>(hist + q * per_f, node, f, nvb[f], ig, is, p, lane, lb, ptc, cut_s[wid]);
    }
    __syncthreads();
  }
  {
    const DirectBest best = lane_best_reduce(lb);
    if (lane == 0) { wb_gain[wid] = best.gain; wb_key[wid] = best.key; wb_GL[wid] = best.GL; wb_SL[wid] = best.SL; }
  }
  __syncthreads();
  if (t == 0) {
    DirectBest b;
    b.gain = -INFINITY; b.GL = b.SL = 0.0; b.key = 0x7fffffffffffffffLL;
    for (int w = 0; w < DIRECT_WAVES; ++w)
      if (wb_key[w] != 0x7fffffffffffffffLL && (wb_gain[w] > b.gain || (wb_gain[w] == b.gain && wb_key[w] < b.key))) {
        b.gain = wb_gain[w]; b.key = wb_key[w]; b.GL = wb_GL[w]; b.SL = wb_SL[w];
      }
    const long long tgq = tot_s[0][0] + tot_s[0][1] + tot_s[0][2] + tot_s[0][3];
    const long long tsq = tot_s[1][0] + tot_s[1][1] + tot_s[1][2] + tot_s[1][3];
    out[node] = direct_node_split(b, tgq, tsq, ig, is);
    if (ec.nodeq) ec.nodeq[node] = ecw ? direct_feat_pos(flist, nfl, b.key) : -1;
  }
}

// Column-major segment codes (row-chunk direct levels, HipTreeBuilder.COLMAJOR_EVERY):
// the code rows of this level's positions [0, n) (row idx[j] of the row-major
// codes) transposed into F feature planes of `plane` positions, so a direct
// pass reads each eligible feature of a node's rows as a contiguous byte run
// instead of one random code row per row (DRF 10M x 100, level 10: 1121 ->
// 521 us, profiles/r6/drf_colmajor_r6j.txt).  Later levels keep the planes and
// move only positions (part_scatter cpos); the one-wave-per-node levels are
// bound by the split scan's instruction issue, not by their code loads, and
// read the row-major codes.  One workgroup per CM_ROWS positions: rows staged
// in LDS (consecutive lanes load consecutive words of one row), then 4 x 4
// byte blocks leave as one dword per feature and 4 positions.
// Positions of retired segments hold stale row ids: rows outside [0, nrows)
// are read as zeros (their plane bytes are never read).
constexpr int CM_ROWS = 256;
__global__ __launch_bounds__(256) void seg_colmajor_kernel(const uint8_t* __restrict__ codes_rm, int fp, int F,
                                                           const int* __restrict__ idx, int n, int64_t nrows,
                                                           uint8_t* __restrict__ ccol, int64_t plane) {
  extern __shared__ uint32_t cm_tile[];   // [CM_ROWS][WP] dwords
  __shared__ int rows[CM_ROWS];
  const int t = threadIdx.x;
  const int j0 = blockIdx.x * CM_ROWS;
  // the words holding the F codes (not the row's pad), at an odd LDS row
  // pitch: the 4 x 4 block reads below step 4 rows per lane
  const int W = (F + 3) >> 2;
  {
    const int j = j0 + t;
    const int r = j < n ? (idx ? idx[j] : j) : -1;
    rows[t] = (r >= 0 && (int64_t)r < nrows) ? r : -1;
  }
  __syncthreads();
  // 16-byte rows (fp % 16 == 0 on an aligned base, so the W16 chunks holding
  // the F codes stay inside the row): LPR lanes per row, 8 chunk loads per lane
  // in flight (and no per-word index division, as in the dword loop below),
  // stored with ds_write_b128 at a pitch of an odd number of chunks.  Row i's
  // chunks are rotated by i / 4 so that the 4-row block reads below stay
  // 4-way, like the dword layout's odd pitch.
  const bool vec = (fp & 15) == 0 && (reinterpret_cast<uintptr_t>(codes_rm) & 15) == 0;
  const int W16 = (F + 15) >> 4;
  const int WP4 = vec ? (W16 | 1) : 0;   // pitch in 16-byte chunks
  const int WP = vec ? 4 * WP4 : (W | 1);
  if (vec) {
    const int LPR = W16 <= 4 ? 4 : (W16 <= 8 ? 8 : (W16 <= 16 ? 16 : 32));   // W16 <= 24 (fp <= 384)
    const int RPI = 256 / LPR;
    const int k = t & (LPR - 1), tr = t / LPR;
    for (int i0 = tr; i0 < CM_ROWS; i0 += 8 * RPI) {
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * RPI;
        const int r = (i < CM_ROWS && k < W16) ? rows[i] : -1;
        v[u] = r >= 0 ? reinterpret_cast<const uint4*>(codes_rm + (int64_t)r * fp)[k] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * RPI;
        if (i < CM_ROWS && k < W16) {
          int c = k + ((i >> 2) % WP4);
          c = c >= WP4 ? c - WP4 : c;
          reinterpret_cast<uint4*>(cm_tile + i * WP)[c] = v[u];
        }
      }
    }
  } else {
    for (int q = t; q < CM_ROWS * W; q += 256) {
      const int i = q / W, k = q - i * W;
      const int r = rows[i];
      cm_tile[i * WP + k] = r >= 0 ? reinterpret_cast<const uint32_t*>(codes_rm + (int64_t)r * fp)[k] : 0u;
    }
  }
  __syncthreads();
  // 4 x 4 byte blocks: 4 rows' dword f4 (features 4 f4 .. 4 f4 + 3) in, each
  // feature's dword of those 4 positions out (one LDS dword read per output
  // dword instead of four byte reads)
  constexpr int R4 = CM_ROWS / 4;
  const int F4 = (F + 3) >> 2;
  for (int q = t; q < F4 * R4; q += 256) {
    const int f4 = q / R4, r4 = q - f4 * R4;
    int col = f4;
    if (vec) {   // the chunk rotation of the rows 4 r4 .. 4 r4 + 3
      int c = (f4 >> 2) + r4 % WP4;
      c = c >= WP4 ? c - WP4 : c;
      col = 4 * c + (f4 & 3);
    }
    const uint32_t* src = cm_tile + 4 * r4 * WP + col;
    const uint32_t a0 = src[0], a1 = src[WP], a2 = src[2 * WP], a3 = src[3 * WP];
    uint32_t o[4];
    o[0] = (a0 & 0xffu) | ((a1 & 0xffu) << 8) | ((a2 & 0xffu) << 16) | (a3 << 24);
    o[1] = ((a0 >> 8) & 0xffu) | (a1 & 0xff00u) | ((a2 & 0xff00u) << 8) | ((a3 & 0xff00u) << 16);
    o[2] = ((a0 >> 16) & 0xffu) | ((a1 >> 8) & 0xff00u) | (a2 & 0xff0000u) | ((a3 & 0xff0000u) << 8);
    o[3] = (a0 >> 24) | ((a1 >> 16) & 0xff00u) | ((a2 >> 8) & 0xff0000u) | (a3 & 0xff000000u);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int f = 4 * f4 + b;
      if (f < F) reinterpret_cast<uint32_t*>(ccol + (int64_t)f * plane + j0)[r4] = o[b];
    }
  }
}



// Row-major code rows from the feature-major codes (BinnedMatrix.codes_rm, built
// once per matrix for the segmented engine): [F][npad] -> [n][fp], pad bytes
// zero.  One workgroup per 256 rows and 128 features at a time: each feature's
// 256 bytes come in as one wave-wide dword load, and every thread leaves with
// its own row in 16-byte stores (replaces a strided torch copy: 10M x 100,
// 3.7 ms).
constexpr int RM_ROWS = 256, RM_FC = 128;
__global__ __launch_bounds__(256) void codes_rowmajor_kernel(const uint8_t* __restrict__ codes, int64_t npad, int F,
                                                             int64_t n, uint8_t* __restrict__ rm, int fp) {
  __shared__ uint32_t tile[RM_FC * RM_ROWS / 4];   // [feature][256 rows] bytes
  const uint8_t* tb = reinterpret_cast<const uint8_t*>(tile);
  const int t = threadIdx.x;
  const int64_t j0 = (int64_t)blockIdx.x * RM_ROWS;
  const int64_t j = j0 + t;
  for (int fc0 = 0; fc0 < fp; fc0 += RM_FC) {
    const int fcnt = min(RM_FC, F - fc0);   // may be <= 0: pad-only chunk
    for (int q = t; q < max(fcnt, 0) * (RM_ROWS / 4); q += 256) {
      const int f = q / (RM_ROWS / 4), w = q - f * (RM_ROWS / 4);
      const int64_t p0 = j0 + 4 * w;
      tile[q] = p0 < npad ? reinterpret_cast<const uint32_t*>(codes + (int64_t)(fc0 + f) * npad + j0)[w] : 0u;
    }
    __syncthreads();
    if (j < n) {
      uint8_t* dst = rm + j * fp + fc0;
      const int nb = min(RM_FC, fp - fc0);   // bytes of this chunk in the row (a multiple of 4)
      for (int b0 = 0; b0 < nb; b0 += 16) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t x = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int f = b0 + 4 * k + e;
            if (f < fcnt) x |= (uint32_t)tb[f * RM_ROWS + t] << (8 * e);
          }
          v[k] = x;
        }
        if ((fp & 15) == 0 && b0 + 16 <= nb) {
          *reinterpret_cast<uint4*>(dst + b0) = make_uint4(v[0], v[1], v[2], v[3]);
        } else {
          for (int k = 0; 4 * k < nb - b0; ++k) reinterpret_cast<uint32_t*>(dst + b0)[k] = v[k];
        }
      }
    }
    __syncthreads();
  }
}

// mtries selection of a wave's features (lane + 64 k, k < 4, F <= 256, hashes
// hv): feature f is eligible iff fewer than m features have a smaller
// (hash, index) key - the m smallest keys.  Instead of ranking every pair (F
// readlane steps x 4 compares per lane), a 32-step ballot bisection finds v,
// the m-th smallest hash; every feature below v is in, and of the features
// hashing to v the first m - #below by index.  The same set as the pairwise
// rank (rank < m), so every engine agrees.
__device__ __forceinline__ void mtries_select(const uint32_t (&hv)[4], int F, int m, int lane, bool (&sel)[4]) {
  bool valid[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) valid[k] = lane + 64 * k < F;
  if (m >= F) {
#pragma unroll
    for (int k = 0; k < 4; ++k) sel[k] = valid[k];
    return;
  }
  const int kn = (F + 63) >> 6;   // wave-uniform
  uint32_t lo = 0u, hi = 0xffffffffu;
  while (lo < hi) {   // smallest v with #{hash <= v} >= m
    const uint32_t mid = lo + ((hi - lo) >> 1);
    int c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < kn) c += __popcll(__ballot(valid[k] && hv[k] <= mid));
    if (c >= m) hi = mid;
    else lo = mid + 1u;
  }
  int below = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < kn) below += __popcll(__ballot(valid[k] && hv[k] < lo));
  const int need = m - below;
  int eq_before = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool eq = valid[k] && hv[k] == lo;
    const unsigned long long be = __ballot(eq);
    const int pos = eq_before + __popcll(be & ((1ull << lane) - 1ull));
    sel[k] = valid[k] && (hv[k] < lo || (eq && pos < need));
    eq_before += __popcll(be);
  }
}

// Eligible features of a node (mtries / column sample / tree mask), ascending,
// computed by ONE wave into flist; returns the count (wave-uniform).  F <=
// 256: per-lane hashes in registers ranked with scalar lane reads; wider: the
// hashes go through LDS (hsh_s, F entries).
template <typename FL>
__device__ __forceinline__ int direct_eligible(int node, int gid_i, const SplitParams& p,
                                              const uint8_t* __restrict__ tree_fmask,
                                              FL* flist, uint32_t* hsh_s, int lane) {
  const int F = p.F;
  const uint32_t key = (uint32_t)p.tree_index * 131u + (uint32_t)p.depth;
  const bool sampled = p.mtries > 0 || p.col_rate < 1.0f;
  int nfl = 0;
  if (F <= 256) {
    uint32_t hv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int f = lane + 64 * k;
      hv[k] = (sampled && f < F) ? hash4(p.seed, key, (uint32_t)node, (uint32_t)f) : 0xffffffffu;
    }
    bool msel[4] = {true, true, true, true};
    if (p.mtries > 0) mtries_select(hv, F, p.mtries, lane, msel);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int f = lane + 64 * k;
      bool ok = f < F && (tree_fmask == nullptr || tree_fmask[f]) && inter_ok(p, gid_i, f);
      if (ok && sampled) ok = p.mtries > 0 ? msel[k] : u01(hv[k]) < p.col_rate;
      const unsigned long long bal = __ballot(ok);
      if (ok) flist[nfl + __popcll(bal & ((1ull << lane) - 1ull))] = (FL)f;
      nfl += __popcll(bal);
    }
    return nfl;
  }
  if (sampled)
    for (int f = lane; f < F; f += 64) hsh_s[f] = hash4(p.seed, key, (uint32_t)node, (uint32_t)f);
  wave_lds_sync();
  for (int f0 = 0; f0 < F; f0 += 64) {
    const int f = f0 + lane;
    bool ok = f < F && (tree_fmask == nullptr || tree_fmask[f]) && inter_ok(p, gid_i, f);
    if (ok && sampled) {
      const uint32_t hf = hsh_s[f];
      if (p.mtries > 0) {
        int rank = 0;
        for (int j = 0; j < F; ++j) {
          const uint32_t hj = hsh_s[j];
          rank += (hj < hf) || (hj == hf && j < f);
        }
        ok = rank < p.mtries;
      } else {
        ok = u01(hf) < p.col_rate;
      }
    }
    const unsigned long long bal = __ballot(ok);
    const int pos = nfl + __popcll(bal & ((1ull << lane) - 1ull));
    if (ok && pos < 1024) flist[pos] = (FL)f;
    nfl += __popcll(bal);
  }
  return nfl < 1024 ? nfl : 1024;
}

// Data-parallel direct levels (N ranks, row shards): the direct engine split
// at its reduction point.  direct_dp_hist_kernel builds, per node of the
// chunk [node0, node0 + gridDim.x), the exact int64 histograms of the node's
// eligible features (G and S planes) from this rank's rows and writes them
// with the node totals to dh[slot] = [G_q, S_q, (q, plane, bin)...] (stride
// 2 + max_elig * 2 * NBT; every slot written, zeros past the node's list), so
// the caller all-reduces the chunk; direct_dp_scan_kernel then scans the
// summed histograms exactly like seg_direct (same eligible list, same
// tie-breaks), so N ranks grow the 1-rank trees bit for bit.
template <int NBT>
__global__ __launch_bounds__(256) void direct_dp_hist_kernel(
    const uint8_t* __restrict__ codes_rm, int fp, const int* __restrict__ idx, const float* __restrict__ g,
    const float* __restrict__ s2, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ ctl, const uint8_t* __restrict__ tree_fmask, const double* __restrict__ qscale,
    SplitParams p, int batch, int node0, int max_elig, long long* __restrict__ dh, int gpos,
    const uint8_t* __restrict__ crow) {
  extern __shared__ __attribute__((aligned(16))) long long hist[];   // [batch][2][NBT]
  const ECodes ec{nullptr, 0, nullptr, crow, nullptr, fp, 1};
  __shared__ int flist[1024];
  __shared__ uint32_t hsh_s[1024];
  __shared__ int nfl_s;
  __shared__ long long tot_s[2][4];
  const uint32_t salt = (uint32_t)qscale[9];
  const int node = node0 + blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t stride = 2 + (int64_t)max_elig * 2 * NBT;
  long long* out = dh + (int64_t)blockIdx.x * stride;
  const bool live = node < ctl[CTL_N];
  if (wid == 0) {
    const int nfl = live ? direct_eligible(node, ctl[CTL_BASE] + node, p, tree_fmask, flist, hsh_s, lane) : 0;
    if (lane == 0) nfl_s = min(nfl, max_elig);
  }
  if (t < 8) tot_s[t >> 2][t & 3] = 0;
  __syncthreads();
  const int nfl = nfl_s;
  for (int64_t j = 2 + (int64_t)nfl * 2 * NBT + t; j < stride; j += blockDim.x) out[j] = 0;   // unused tail
  const int lo = live ? seg_start[node] : 0, cnt = live ? seg_cnt[node] : 0;
  const float sg = (float)qscale[0], ss = (float)qscale[1];
  const int64_t rb = (int64_t)qscale[7];
  long long tg_row = 0, ts_row = 0;
  for (int b0 = 0; b0 < nfl; b0 += batch) {   // (no eligible feature: zero totals, as seg_direct)
    const int nb = min(batch, nfl - b0);
    for (int j = t; j < nb * 2 * NBT; j += blockDim.x) hist[j] = 0;
    __syncthreads();
    for (int j = lo + t; j < lo + cnt; j += blockDim.x) {
      const int r = idx ? idx[j] : j;
      const uint8_t* row = ec.crow ? ec.crow + (int64_t)(ec.cpos ? ec.cpos[j] : j) * ec.rs : codes_rm + (int64_t)r * fp;
      const int64_t fs = ec.crow ? ec.fs : 1;
      uint32_t c0[DIRECT_FB];
#pragma unroll
      for (int u = 0; u < DIRECT_FB; ++u) c0[u] = (u < nb) ? row[flist[b0 + u] * fs] : 0u;
      long long gq, sq;
      direct_row_q(r, gpos ? j : r, rb, salt, g, s2, sg, ss, gq, sq);
      if (b0 == 0) { tg_row += gq; ts_row += sq; }
      direct_row_atomics<NBT>(row, fs, flist + b0, nb, false, 2 * NBT, hist, gq, sq, c0, nullptr, 0);
    }
    __syncthreads();
    for (int j = t; j < nb * 2 * NBT; j += blockDim.x) out[2 + (int64_t)b0 * 2 * NBT + j] = hist[j];
    __syncthreads();
  }
  tg_row = wave_sum_i64(tg_row);
  ts_row = wave_sum_i64(ts_row);
  if (lane == 0) { tot_s[0][wid] = tg_row; tot_s[1][wid] = ts_row; }
  __syncthreads();
  if (t == 0) {
    out[0] = tot_s[0][0] + tot_s[0][1] + tot_s[0][2] + tot_s[0][3];
    out[1] = tot_s[1][0] + tot_s[1][1] + tot_s[1][2] + tot_s[1][3];
  }
}

template <int NBT>
__global__ __launch_bounds__(256) void direct_dp_scan_kernel(
    const int* __restrict__ ctl, const int* __restrict__ nvb, const uint8_t* __restrict__ tree_fmask,
    const double* __restrict__ qscale, SplitParams p, int node0, int max_elig, const long long* __restrict__ dh,
    NodeSplit* __restrict__ ns) {
  __shared__ int flist[1024];
  __shared__ uint32_t hsh_s[1024];
  __shared__ int nfl_s;
  __shared__ double wb_gain[4], wb_GL[4], wb_SL[4];
  __shared__ long long wb_key[4];
  __shared__ double cut_s[4][64];   // per-wave UniformAdaptive cut tables
  const int node = node0 + blockIdx.x;
  if (node >= ctl[CTL_N]) return;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t stride = 2 + (int64_t)max_elig * 2 * NBT;
  const long long* h = dh + (int64_t)blockIdx.x * stride;
  if (wid == 0) {
    const int nfl = direct_eligible(node, ctl[CTL_BASE] + node, p, tree_fmask, flist, hsh_s, lane);
    if (lane == 0) nfl_s = min(nfl, max_elig);
  }
  __syncthreads();
  const int nfl = nfl_s;
  const double ig = qscale[2], is = qscale[3];
  LaneBest lb;
  lane_best_init(lb);
  double ptc = NAN;   // the node's parent gain term (direct_scan_feature)
  for (int q = wid; q < nfl; q += 4) {
    const int f = flist[q];
    direct_scan_feature<NBT, false>(h + 2 + (int64_t)q * 2 * NBT, node, f, nvb[f], ig, is, p, lane, lb, ptc, cut_s[wid]);
  }
  {
    const DirectBest best = lane_best_reduce(lb);
    if (lane == 0) { wb_gain[wid] = best.gain; wb_key[wid] = best.key; wb_GL[wid] = best.GL; wb_SL[wid] = best.SL; }
  }
  __syncthreads();
  if (t == 0) {
    DirectBest b;
    b.gain = -INFINITY; b.GL = b.SL = 0.0; b.key = 0x7fffffffffffffffLL;
    for (int w = 0; w < 4; ++w)
      if (wb_key[w] != 0x7fffffffffffffffLL && (wb_gain[w] > b.gain || (wb_gain[w] == b.gain && wb_key[w] < b.key))) {
        b.gain = wb_gain[w]; b.key = wb_key[w]; b.GL = wb_GL[w]; b.SL = wb_SL[w];
      }
    ns[node] = direct_node_split(b, h[0], h[1], ig, is);
  }
}

// Direct levels whose nodes still hold thousands of rows (the first direct
// levels): one workgroup per PC_ROWS row chunk, not per node, so a large node
// is spread over many workgroups instead of being the kernel's tail.  Each
// chunk (<= 4096 rows: packed 64-bit atomics are always exact) builds the
// node's eligible features in LDS; a single-chunk node scans them at once,
// otherwise the chunk stores its packed histogram and totals in a slab and
// the node's last chunk to arrive (agent-scope release / ticket / acquire)
// sums the slabs exactly into G and S planes and scans.
constexpr int DIRECT_CHUNK_LDS = 64 * 1024;   // two-plane histograms of every eligible feature
__global__ __launch_bounds__(256) void direct_empty_kernel(const int* __restrict__ seg_cnt,
                                                           const int* __restrict__ ctl, NodeSplit* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ctl[CTL_N] || seg_cnt[i] != 0) return;
  DirectBest b;
  b.gain = -INFINITY; b.GL = b.SL = 0.0; b.key = 0x7fffffffffffffffLL;
  out[i] = direct_node_split(b, 0, 0, 0.0, 0.0);
}

template <int NBT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void seg_direct_chunk_kernel(
    const uint8_t* __restrict__ codes_rm, int fp, const int* __restrict__ idx, const float* __restrict__ g,
    const float* __restrict__ s2, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ pc_first, const int* __restrict__ ctl, const int* __restrict__ nvb,
    const uint8_t* __restrict__ tree_fmask, const double* __restrict__ qscale, uint32_t salt, SplitParams p,
    int nfl_max, unsigned long long* __restrict__ slab, long long* __restrict__ tot_slab, int* __restrict__ ticket,
    NodeSplit* __restrict__ out, int gpos, ECodes ec) {
  salt = (uint32_t)qscale[9];  // per-tree dither salt, written by tree_begin (graph-replay safe)
  extern __shared__ __attribute__((aligned(16))) long long hist[];   // packed [nfl][NBT]; reduce: [nfl][2][NBT]
  __shared__ int flist[1024];
  __shared__ uint32_t hsh_s[1024];
  __shared__ int node_s, nfl_s, last_s;
  __shared__ long long tot_s[2][4];
  __shared__ double wb_gain[4], wb_GL[4], wb_SL[4];
  __shared__ long long wb_key[4];
  __shared__ double cut_s[4][64];   // per-wave UniformAdaptive cut tables
  const int n = ctl[CTL_N];
  const int c = ec.crow ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  if (c >= pc_first[n]) return;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  if (wid == 0) {
    const int node = chunk_node_wave(pc_first, n, c, lane);
    const int nfl = direct_eligible(node, ctl[CTL_BASE] + node, p, tree_fmask, flist, hsh_s, lane);
    if (lane == 0) { node_s = node; nfl_s = min(nfl, nfl_max); }
  }
  __syncthreads();
  const int node = node_s, nfl = nfl_s;
  const int c0 = pc_first[node], nch = pc_first[node + 1] - c0;
  const int start = seg_start[node];
  const int lo = start + (c - c0) * PC_ROWS;
  const int hi = min(lo + PC_ROWS, start + seg_cnt[node]);
  const float sg = (float)qscale[0], ss = (float)qscale[1];
  const double ig = qscale[2], is = qscale[3];
  const int64_t rb = (int64_t)qscale[7];
  for (int j = t; j < nfl * NBT; j += blockDim.x) hist[j] = 0;
  __syncthreads();
  long long tg_row = 0, ts_row = 0;
  const int64_t fs = ec.crow ? ec.fs : 1;
  if (nfl <= 2 * DIRECT_FB) {
    // <= 16 eligible features (DRF mtries): the features' code offsets are
    // wave-uniform (scalar registers, no LDS read per code byte) and each
    // row's id / plane position is loaded one iteration ahead, so a row's
    // chain is its code loads -> atomics instead of id -> codes -> atomics
    int64_t fo[2 * DIRECT_FB];
#pragma unroll
    for (int u = 0; u < 2 * DIRECT_FB; ++u)
      fo[u] = u < nfl ? (int64_t)__builtin_amdgcn_readfirstlane(flist[u]) * fs : 0;
    auto row_of = [&](int j, int r) -> const uint8_t* {
      return ec.crow ? ec.crow + (int64_t)(ec.cpos ? ec.cpos[j] : j) * ec.rs : codes_rm + (int64_t)r * fp;
    };
    int j = lo + t;
    int r = (j < hi) ? (idx ? idx[j] : j) : 0;
    const uint8_t* row = (j < hi) ? row_of(j, r) : codes_rm;
    for (; j < hi; j += blockDim.x) {
      uint32_t cc[2 * DIRECT_FB];
#pragma unroll
      for (int u = 0; u < 2 * DIRECT_FB; ++u) cc[u] = (u < nfl) ? row[fo[u]] : 0u;
      long long gq, sq;
      direct_row_q(r, gpos ? j : r, rb, salt, g, s2, sg, ss, gq, sq);
      // next row's id and code row (independent of this row's atomics)
      const int jn = j + blockDim.x;
      const int rn = (jn < hi) ? (idx ? idx[jn] : jn) : 0;
      const uint8_t* rown = (jn < hi) ? row_of(jn, rn) : codes_rm;
      tg_row += gq; ts_row += sq;
      const bool live = gq != 0 || sq != 0;
      if (ec.codes) {
        uint8_t* erow = ec.codes + (int64_t)j * ec.stride;
        const uint32_t w0 = cc[0] | (cc[1] << 8) | (cc[2] << 16) | (cc[3] << 24);
        const uint32_t w1 = cc[4] | (cc[5] << 8) | (cc[6] << 16) | (cc[7] << 24);
        if (ec.stride == 16) {
          const uint32_t w2 = cc[8] | (cc[9] << 8) | (cc[10] << 16) | (cc[11] << 24);
          const uint32_t w3 = cc[12] | (cc[13] << 8) | (cc[14] << 16) | (cc[15] << 24);
          *reinterpret_cast<uint4*>(erow) = make_uint4(w0, w1, w2, w3);
        } else {
          *reinterpret_cast<uint2*>(erow) = make_uint2(w0, w1);
        }
      }
      if (live) {
        const unsigned long long pk = ((unsigned long long)(uint32_t)(int)gq << 32) | (unsigned long long)sq;
#pragma unroll
        for (int u = 0; u < 2 * DIRECT_FB; ++u)
          if (u < nfl) atomicAdd(reinterpret_cast<unsigned long long*>(hist + u * NBT + cc[u]), pk);
      }
      r = rn;
      row = rown;
    }
  } else {
    for (int j = lo + t; j < hi; j += blockDim.x) {
      const int r = idx ? idx[j] : j;
      const uint8_t* row = ec.crow ? ec.crow + (int64_t)(ec.cpos ? ec.cpos[j] : j) * ec.rs : codes_rm + (int64_t)r * fp;
      uint32_t cc[DIRECT_FB];
#pragma unroll
      for (int u = 0; u < DIRECT_FB; ++u) cc[u] = (u < nfl) ? row[flist[u] * fs] : 0u;
      long long gq, sq;
      direct_row_q(r, gpos ? j : r, rb, salt, g, s2, sg, ss, gq, sq);
      tg_row += gq; ts_row += sq;
      direct_row_atomics<NBT>(row, fs, flist, nfl, true, NBT, hist, gq, sq, cc,
                              ec.codes ? ec.codes + (int64_t)j * ec.stride : nullptr, ec.stride);
    }
  }
  tg_row = wave_sum_i64(tg_row);
  ts_row = wave_sum_i64(ts_row);
  if (lane == 0) { tot_s[0][wid] = tg_row; tot_s[1][wid] = ts_row; }
  __syncthreads();
  long long tgq = tot_s[0][0] + tot_s[0][1] + tot_s[0][2] + tot_s[0][3];
  long long tsq = tot_s[1][0] + tot_s[1][1] + tot_s[1][2] + tot_s[1][3];
  bool packed = true;
  if (nch > 1) {
    // publish this chunk, then the node's last chunk reduces every chunk
    unsigned long long* my = slab + (int64_t)c * nfl_max * NBT;
    for (int j = t; j < nfl * NBT; j += blockDim.x) my[j] = (unsigned long long)hist[j];
    if (t == 0) { tot_slab[2 * c] = tgq; tot_slab[2 * c + 1] = tsq; }
    __syncthreads();
    if (t == 0) {
      __atomic_thread_fence(__ATOMIC_RELEASE);
      const int prev = __hip_atomic_fetch_add(ticket + node, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      last_s = prev == nch - 1;
      if (last_s) ticket[node] = 0;   // ready for the next level
    }
    __syncthreads();
    if (!last_s) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    packed = false;
    for (int e = t; e < nfl * NBT; e += blockDim.x) {
      long long G = 0, S = 0;
      for (int k = 0; k < nch; ++k) {
        const unsigned long long v = __hip_atomic_load(slab + (int64_t)(c0 + k) * nfl_max * NBT + e, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        G += (long long)(int)(uint32_t)(v >> 32);
        S += (long long)(uint32_t)v;
      }
      const int q = e / NBT, b = e - q * NBT;
      hist[q * 2 * NBT + b] = G;
      hist[q * 2 * NBT + NBT + b] = S;
    }
    if (t == 0) {
      long long a = 0, b = 0;
      for (int k = 0; k < nch; ++k) {
        a += __hip_atomic_load(tot_slab + 2 * (c0 + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b += __hip_atomic_load(tot_slab + 2 * (c0 + k) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      tot_s[0][0] = a; tot_s[1][0] = b;
    }
    __syncthreads();
    tgq = tot_s[0][0]; tsq = tot_s[1][0];
  }
  LaneBest lb;
  lane_best_init(lb);
  double ptc = NAN;   // the node's parent gain term (direct_scan_feature)
  for (int q = wid; q < nfl; q += 4) {
    const int f = flist[q];
    if (packed) direct_scan_feature<NBT, true>(hist + q * NBT, node, f, nvb[f], ig, is, p, lane, lb, ptc, cut_s[wid]);
    else direct_scan_feature<NBT, false>(hist + q * 2 * NBT, node, f, nvb[f], ig, is, p, lane, lb, ptc, cut_s[wid]);
  }
  {
    const DirectBest best = lane_best_reduce(lb);
    if (lane == 0) { wb_gain[wid] = best.gain; wb_key[wid] = best.key; wb_GL[wid] = best.GL; wb_SL[wid] = best.SL; }
  }
  __syncthreads();
  if (t == 0) {
    DirectBest b;
    b.gain = -INFINITY; b.GL = b.SL = 0.0; b.key = 0x7fffffffffffffffLL;
    for (int w = 0; w < 4; ++w)
      if (wb_key[w] != 0x7fffffffffffffffLL && (wb_gain[w] > b.gain || (wb_gain[w] == b.gain && wb_key[w] < b.key))) {
        b.gain = wb_gain[w]; b.key = wb_key[w]; b.GL = wb_GL[w]; b.SL = wb_SL[w];
      }
    out[node] = direct_node_split(b, tgq, tsq, ig, is);
    if (ec.nodeq) ec.nodeq[node] = direct_feat_pos(flist, nfl, b.key);
  }
}

// Deepest levels (nodes of a few hundred rows): one WAVE per node, four
// nodes per 256-thread workgroup, every wave on its own LDS area - no
// workgroup barriers, so a node's short latency chain (segment -> rows ->
// codes -> atomics -> scan) overlaps with three others per workgroup and
// many more per CU.  Eligible features from per-lane hashes in registers
// (F <= 256) ranked with scalar lane reads (no LDS round trips).
constexpr int DIRECT_WAVE_F = 256;
constexpr int DIRECT_WAVE_LDS = 8 * 1024;   // max histogram bytes per wave (8 / 10 / 16 KB measured alike, profiles/r5/drf_deep_ab.txt)

template <int NBT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void seg_direct_wave_kernel(
    const uint8_t* __restrict__ codes_rm, int fp, const int* __restrict__ idx, const float* __restrict__ g,
    const float* __restrict__ s2, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ ctl, const int* __restrict__ nvb, const uint8_t* __restrict__ tree_fmask,
    const double* __restrict__ qscale, uint32_t salt, SplitParams p, int batch, NodeSplit* __restrict__ out,
    int gpos, ECodes ec) {
  salt = (uint32_t)qscale[9];  // per-tree dither salt, written by tree_begin (graph-replay safe)
  extern __shared__ __attribute__((aligned(16))) long long hist_all[];   // [4][batch * 2 * NBT]
  __shared__ short flist_all[4][DIRECT_WAVE_F];
  __shared__ double cut_s[4][64];   // per-wave UniformAdaptive cut tables
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int node = (ec.crow ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x) * 4 + wid;
  if (node >= ctl[CTL_N]) return;   // whole wave: no workgroup barrier below
  long long* hist = hist_all + wid * batch * 2 * NBT;
  short* flist = flist_all[wid];
  const int F = p.F;
  const int lo = seg_start[node], cnt = seg_cnt[node];
  const int gid_i = ctl[CTL_BASE] + node;   // interaction-constraint state
  // eligible features, ascending
  const uint32_t key = (uint32_t)p.tree_index * 131u + (uint32_t)p.depth;
  const bool sampled = p.mtries > 0 || p.col_rate < 1.0f;
  uint32_t hv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int f = lane + 64 * k;
    hv[k] = (sampled && f < F) ? hash4(p.seed, key, (uint32_t)node, (uint32_t)f) : 0xffffffffu;
  }
  bool msel[4] = {true, true, true, true};
  if (p.mtries > 0) mtries_select(hv, F, p.mtries, lane, msel);
  int nfl = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int f = lane + 64 * k;
    bool ok = f < F && (tree_fmask == nullptr || tree_fmask[f]) && inter_ok(p, gid_i, f);
    if (ok && sampled) ok = p.mtries > 0 ? msel[k] : u01(hv[k]) < p.col_rate;
    const unsigned long long bal = __ballot(ok);
    if (ok) flist[nfl + __popcll(bal & ((1ull << lane) - 1ull))] = (short)f;
    nfl += __popcll(bal);
  }
  const float sg = (float)qscale[0], ss = (float)qscale[1];
  const double ig = qscale[2], is = qscale[3];
  const int64_t rb = (int64_t)qscale[7];
  const bool packed = cnt < DIRECT_PACK_ROWS;
  const int per_f = packed ? NBT : 2 * NBT;
  const int bat = packed ? 2 * batch : batch;
  LaneBest lb;
  lane_best_init(lb);
  double ptc = NAN;   // the node's parent gain term (direct_scan_feature)
  long long tg_row = 0, ts_row = 0;
  // eligible-code rows only for nodes scanned in ONE batch (see seg_direct_kernel)
  uint8_t* const ecw = (ec.codes && nfl <= bat) ? ec.codes : nullptr;
  wave_lds_sync();
  for (int b0 = 0; b0 < max(nfl, 1); b0 += bat) {
    const int nb = min(bat, nfl - b0);
    for (int j = lane; j < nb * per_f; j += 64) hist[j] = 0;
    wave_lds_sync();
    for (int j = lo + lane; j < lo + cnt; j += 64) {
      const int r = idx ? idx[j] : j;
      const uint8_t* row = ec.crow ? ec.crow + (int64_t)(ec.cpos ? ec.cpos[j] : j) * ec.rs : codes_rm + (int64_t)r * fp;
      const int64_t fs = ec.crow ? ec.fs : 1;
      uint32_t c0[DIRECT_FB];
#pragma unroll
      for (int u = 0; u < DIRECT_FB; ++u) c0[u] = (u < nb) ? row[flist[b0 + u] * fs] : 0u;
      long long gq, sq;
      direct_row_q(r, gpos ? j : r, rb, salt, g, s2, sg, ss, gq, sq);
      if (b0 == 0) { tg_row += gq; ts_row += sq; }
      if (nb <= 0) continue;
      direct_row_atomics<NBT>(row, fs, flist + b0, nb, packed, per_f, hist, gq, sq, c0,
                              ecw ? ecw + (int64_t)j * ec.stride : nullptr, ec.stride);
    }
    if (b0 == 0) {
      // a node whose weight (mode 0) / hessian (mode 1) total is below twice the
      // child minimum (or not positive) has no split any scan could accept -
      // every candidate's gain is -inf - so its feature scans are skipped
      // (same NodeSplit: no split); deep DRF levels hold many such nodes
      const double S = (double)wave_sum_i64(ts_row) * is;
      const double cmin = p.mode == 0 ? p.min_rows : p.min_child_weight;
      if (!(S > 0.0) || S < 2.0 * cmin) break;
    }
    wave_lds_sync();
    for (int q = 0; q < nb; ++q) {
      const int f = flist[b0 + q];
      if (packed) direct_scan_feature<NBT, true>(hist + q * per_f, node, f, nvb[f], ig, is, p, lane, lb, ptc, cut_s[wid]);
      else direct_scan_feature<NBT, false>(hist + q * per_f, node, f, nvb[f], ig, is, p, lane, lb, ptc, cut_s[wid]);
    }
    wave_lds_sync();
  }
  tg_row = wave_sum_i64(tg_row);
  ts_row = wave_sum_i64(ts_row);
  const DirectBest best = lane_best_reduce(lb);
  if (lane == 0) {
    out[node] = direct_node_split(best, tg_row, ts_row, ig, is);
    if (ec.nodeq) ec.nodeq[node] = ecw ? direct_feat_pos(flist, nfl, best.key) : -1;
  }
}

__global__ __launch_bounds__(256) void zero_slots_kernel(long long* __restrict__ built,
                                                         const int* __restrict__ ctl_next, int per_slot) {
  const int64_t m = (int64_t)ctl_next[CTL_SLOTS] * per_slot;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x)
    built[k] = 0ll;
}

__device__ __forceinline__ long long block_sum_ll(long long v, long long* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  long long s = 0;
  if (threadIdx.x == 0)
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += red[k];
  return s;  // valid in thread 0
}

// Stable partition of each chunk into idx_out + node ids + leaf sums.
__global__ __launch_bounds__(256) void part_scatter_kernel(
    const uint8_t* __restrict__ codes, int64_t npad, const int* __restrict__ idx, int* __restrict__ idx_out,
    int* __restrict__ nid, int write_nid, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ pc_first, const int* __restrict__ pc_off, const int* __restrict__ node_nl,
    const int* __restrict__ ctl, const PartInfo* __restrict__ part, int nbt, const float* __restrict__ g,
    const float* __restrict__ h, const float* __restrict__ w, const double* __restrict__ qs, int cap,
    unsigned long long* __restrict__ leaf_acc, const float* __restrict__ gin, const float* __restrict__ sin,
    float* __restrict__ gout, float* __restrict__ sout, SegRows sr, const uint8_t* __restrict__ codes_rm,
    const int8_t* __restrict__ dirb) {
  __shared__ int wl[4];
  __shared__ long long red[4];
  const int n = ctl[CTL_N];
  const int c = blockIdx.x;
  if (c >= pc_first[n]) return;
  const int node = chunk_node_wave(pc_first, n, c, threadIdx.x & 63);   // every wave (uniform answer)
  const PartInfo pi = part[node];
  const int start = seg_start[node];
  const int lo = start + (c - pc_first[node]) * PC_ROWS;
  const int hi = min(lo + PC_ROWS, start + seg_cnt[node]);
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const bool inner = pi.child >= 0 && !pi.leaf_children;
  const bool retire = !inner;  // leaf here (no split) or children are leaves
  long long sg[2] = {0, 0}, sh[2] = {0, 0}, sw[2] = {0, 0};
  const float lg = leaf_acc ? (float)qs[4] : 0.f, lh = leaf_acc ? (float)qs[5] : 0.f,
              lw = leaf_acc ? (float)qs[6] : 0.f;
  int base_l = inner ? pc_off[c] : 0;
  int base_r = inner ? (lo - start) - base_l : 0;
  const int nl = inner ? node_nl[node] : 0;
  // the row's id, direction and moved (g, s2) are loaded one iteration ahead
  // (independent of the two barriers per iteration), so the loop's critical
  // path no longer starts with their load latency
  auto fetch = [&](int j, int& r, int& dir, float& gv, float& sv) {
    r = 0; dir = 0; gv = 0.f; sv = 0.f;
    if (j < hi) {
      r = idx ? idx[j] : j;
      if (pi.child >= 0 && dirb) dir = (int)dirb[j];
      if (inner && gout) {
        gv = gin[j];
        if (sout) sv = sin[j];
      }
    }
  };
  int r_n, dir_n;
  float gv_n, sv_n;
  fetch(lo + t, r_n, dir_n, gv_n, sv_n);
  for (int j0 = lo; j0 < hi; j0 += blockDim.x) {
    const int j = j0 + t;
    const bool valid = j < hi;
    int r = r_n, dir = dir_n;
    const float gv = gv_n, sv = sv_n;
    fetch(j + blockDim.x, r_n, dir_n, gv_n, sv_n);
    if (valid && pi.child >= 0 && !dirb) dir = seg_split_dir(codes, npad, pi, nbt, r, j, sr);
    if (inner) {
      const bool goes_left = valid && dir == 0;
      const unsigned long long bl = __ballot(goes_left);
      const unsigned long long bv = __ballot(valid);
      if (lane == 0) wl[wid] = __popcll(bl) | (__popcll(bv) << 16);
      __syncthreads();
      int before_l = 0, before_v = 0, tot_l = 0, tot_v = 0;
      for (int k = 0; k < 4; ++k) {
        const int a = wl[k] & 0xFFFF, v = wl[k] >> 16;
        if (k < wid) { before_l += a; before_v += v; }
        tot_l += a; tot_v += v;
      }
      const unsigned long long lt = (1ull << lane) - 1ull;
      const int my_l = before_l + __popcll(bl & lt);
      const int my_v = before_v + __popcll(bv & lt);
      if (valid) {
        const int pos = goes_left ? base_l + my_l : nl + base_r + (my_v - my_l);
        idx_out[start + pos] = r;
        if (sr.cpos_out) sr.cpos_out[start + pos] = sr.cpos_in ? sr.cpos_in[j] : j;
        if (write_nid) nid[r] = pi.child + dir;
        if (gout) {   // the (g, s2) the next level reads, moved with the row into segment order
          gout[start + pos] = gv;
          if (sout) sout[start + pos] = sv;
        }
      }
      if (sr.out) {
        int dst = -1;
        if (valid) dst = start + (goes_left ? base_l + my_l : nl + base_r + (my_v - my_l));
        seg_move_rows_wave(sr, codes_rm, r, j, dst);
      }
      base_l += tot_l;
      base_r += tot_v - tot_l;
      __syncthreads();
    } else if (valid) {
      const int leaf = (pi.child >= 0) ? pi.child_gid + dir : pi.gid;
      nid[r] = ~leaf;
      if (leaf_acc && leaf < cap) {
        const float wv = w ? w[r] : 1.0f;
        if (wv != 0.0f) {
          sg[dir] += __float2int_rn(g[r] * lg);
          if (h) sh[dir] += __float2int_rn(h[r] * lh);   // (no h: mean leaves, H unused)
          sw[dir] += __float2int_rn(wv * lw);
        }
      }
    }
  }
  if (retire && leaf_acc) {
    const int nleaf = (pi.child >= 0) ? 2 : 1;
    for (int d = 0; d < nleaf; ++d) {
      const int leaf = (pi.child >= 0) ? pi.child_gid + d : pi.gid;
      const long long a = block_sum_ll(sg[d], red);
      const long long b = block_sum_ll(sh[d], red);
      const long long e = block_sum_ll(sw[d], red);
      if (t == 0 && leaf < cap) {
        if (a) atomicAdd(leaf_acc + 3 * leaf, (unsigned long long)a);
        if (b) atomicAdd(leaf_acc + 3 * leaf + 1, (unsigned long long)b);
        if (e) atomicAdd(leaf_acc + 3 * leaf + 2, (unsigned long long)e);
      }
    }
  }
}

// Wave-granular partition for levels with thousands of nodes: one WAVE per
// PC_ROWS chunk (four chunks per workgroup) and the chunk's node found by a
// 64-ary search (three rounds of 64 parallel probes instead of ~18 dependent
// binary-search loads), so a level of 10^5 single-chunk nodes launches 4x
// fewer workgroups whose latency chains overlap.  part_count_wave also stores
// each row's direction byte (dirb, indexed like idx) for every node with a
// split, so part_scatter_wave moves rows without re-gathering split codes.
// Same counts, offsets and row order as part_count / part_scatter.

__global__ __launch_bounds__(256) void part_count_wave_kernel(const uint8_t* __restrict__ codes, int64_t npad,
                                                              const int* __restrict__ idx,
                                                              const int* __restrict__ seg_start,
                                                              const int* __restrict__ seg_cnt,
                                                              const int* __restrict__ pc_first,
                                                              const int* __restrict__ ctl,
                                                              const PartInfo* __restrict__ part, int nbt,
                                                              int* __restrict__ pc_left, int8_t* __restrict__ dirb,
                                                              const uint8_t* __restrict__ ecodes, int ecs,
                                                              const int* __restrict__ nodeq, SegRows sr) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = ctl[CTL_N];
  if (c >= pc_first[n]) return;
  const int node = chunk_node_wave(pc_first, n, c, lane);
  const PartInfo pi = part[node];
  int cnt = 0;
  if (pi.child >= 0) {
    const int lo = seg_start[node] + (c - pc_first[node]) * PC_ROWS;
    const int hi = min(lo + PC_ROWS, seg_start[node] + seg_cnt[node]);
    const int eq = ecodes ? nodeq[node] : -1;   // -1: the node's codes were not stored
    for (int j = lo + lane; j < hi; j += 64) {
      int d;
      if (eq >= 0) {
        const int b = ecodes[(int64_t)j * ecs + eq];
        d = part_right(pi, b, nbt);
      } else {
        d = seg_split_dir(codes, npad, pi, nbt, idx ? idx[j] : j, j, sr);
      }
      if (dirb) dirb[j] = (int8_t)d;
      cnt += 1 - d;
    }
    if (pi.leaf_children) cnt = 0;   // only inner splits count (as part_count)
  }
  cnt = wave_sum_i32(cnt);
  if (lane == 0) pc_left[c] = cnt;
}

__global__ __launch_bounds__(256) void part_scatter_wave_kernel(
    const uint8_t* __restrict__ codes, int64_t npad, const int* __restrict__ idx, int* __restrict__ idx_out,
    int* __restrict__ nid, int write_nid, const int* __restrict__ seg_start, const int* __restrict__ seg_cnt,
    const int* __restrict__ pc_first, const int* __restrict__ pc_off, const int* __restrict__ node_nl,
    const int* __restrict__ ctl, const PartInfo* __restrict__ part, int nbt, const float* __restrict__ g,
    const float* __restrict__ h, const float* __restrict__ w, const double* __restrict__ qs, int cap,
    unsigned long long* __restrict__ leaf_acc, const int8_t* __restrict__ dirb, const float* __restrict__ gin,
    const float* __restrict__ sin, float* __restrict__ gout, float* __restrict__ sout,
    const uint8_t* __restrict__ ecodes, int ecs, const int* __restrict__ nodeq, int segf, SegRows sr,
    const uint8_t* __restrict__ codes_rm) {
  // segf (last level): bit 0 - gin / sin hold g and s2 in segment order (read
  // them at j instead of gathering g[r] / s2[r] by row: one random 4-byte
  // gather per row left instead of three); bit 1 - s2 is h (else w)
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = ctl[CTL_N];
  if (c >= pc_first[n]) return;
  const int node = chunk_node_wave(pc_first, n, c, lane);
  const PartInfo pi = part[node];
  const int start = seg_start[node];
  const int lo = start + (c - pc_first[node]) * PC_ROWS;
  const int hi = min(lo + PC_ROWS, start + seg_cnt[node]);
  const bool inner = pi.child >= 0 && !pi.leaf_children;
  long long sg[2] = {0, 0}, sh[2] = {0, 0}, sw[2] = {0, 0};
  const float lg = leaf_acc ? (float)qs[4] : 0.f, lh = leaf_acc ? (float)qs[5] : 0.f,
              lw = leaf_acc ? (float)qs[6] : 0.f;
  int base_l = inner ? pc_off[c] : 0;
  int base_r = inner ? (lo - start) - base_l : 0;
  const int nl = inner ? node_nl[node] : 0;
  const unsigned long long lt = (1ull << lane) - 1ull;
  // inner nodes with stored directions: a row's id, direction, plane position
  // and moved (g, s2) are loaded one iteration ahead (independent loads off
  // the iteration's critical path)
  const bool ahead = inner && dirb != nullptr;
  int r_n = 0, d_n = 0, cp_n = 0;
  float gv_n = 0.f, sv_n = 0.f;
  auto fetch = [&](int j) {
    if (j < hi) {
      r_n = idx ? idx[j] : j;
      d_n = dirb[j];
      if (sr.cpos_out) cp_n = sr.cpos_in ? sr.cpos_in[j] : j;
      if (gout) {
        gv_n = gin[j];
        if (sout) sv_n = sin[j];
      }
    }
  };
  if (ahead) fetch(lo + lane);
  for (int j0 = lo; j0 < hi; j0 += 64) {
    const int j = j0 + lane;
    const bool valid = j < hi;
    int r = 0, dir = 0, cp = 0;
    float gv = 0.f, sv = 0.f;
    if (ahead) {
      r = r_n; dir = d_n; cp = cp_n; gv = gv_n; sv = sv_n;
      fetch(j + 64);
    } else if (valid) {
      r = idx ? idx[j] : j;
      if (pi.child >= 0) {
        if (dirb) {
          dir = dirb[j];
        } else if (ecodes && nodeq[node] >= 0) {
          const int b = ecodes[(int64_t)j * ecs + nodeq[node]];
          dir = part_right(pi, b, nbt);
        } else {
          dir = seg_split_dir(codes, npad, pi, nbt, r, j, sr);
        }
      }
      if (inner) {
        if (sr.cpos_out) cp = sr.cpos_in ? sr.cpos_in[j] : j;
        if (gout) {
          gv = gin[j];
          if (sout) sv = sin[j];
        }
      }
    }
    if (inner) {
      const unsigned long long bl = __ballot(valid && dir == 0);
      const unsigned long long bv = __ballot(valid);
      if (valid) {
        const int my_l = __popcll(bl & lt), my_v = __popcll(bv & lt);
        const int pos = dir == 0 ? base_l + my_l : nl + base_r + (my_v - my_l);
        idx_out[start + pos] = r;
        if (sr.cpos_out) sr.cpos_out[start + pos] = cp;
        if (write_nid) nid[r] = pi.child + dir;
        if (gout) {
          gout[start + pos] = gv;
          if (sout) sout[start + pos] = sv;
        }
      }
      if (sr.out) {
        int dst = -1;
        if (valid) {
          const int my_l = __popcll(bl & lt), my_v = __popcll(bv & lt);
          dst = start + (dir == 0 ? base_l + my_l : nl + base_r + (my_v - my_l));
        }
        seg_move_rows_wave(sr, codes_rm, r, j, dst);
      }
      base_l += __popcll(bl);
      base_r += __popcll(bv) - __popcll(bl);
    } else if (valid) {
      const int leaf = (pi.child >= 0) ? pi.child_gid + dir : pi.gid;
      nid[r] = ~leaf;
      if (leaf_acc && leaf < cap) {
        const bool sg_seg = segf & 1, s_is_h = segf & 2;
        const float wv = (sg_seg && !s_is_h) ? (sin ? sin[j] : 1.0f) : (w ? w[r] : 1.0f);
        if (wv != 0.0f) {
          const float gk = sg_seg ? gin[j] : g[r];
          const float hk = (sg_seg && s_is_h) ? sin[j] : (h ? h[r] : 0.f);   // (no h: mean leaves)
          sg[dir] += __float2int_rn(gk * lg);
          sh[dir] += __float2int_rn(hk * lh);
          sw[dir] += __float2int_rn(wv * lw);
        }
      }
    }
  }
  if (!inner && leaf_acc) {
    const int nleaf = (pi.child >= 0) ? 2 : 1;
    for (int d = 0; d < nleaf; ++d) {
      long long a = sg[d], b = sh[d], e = sw[d];
      a = wave_sum_i64(a);
      b = wave_sum_i64(b);
      e = wave_sum_i64(e);
      const int leaf = (pi.child >= 0) ? pi.child_gid + d : pi.gid;
      if (lane == 0 && leaf < cap) {
        if (a) atomicAdd(leaf_acc + 3 * leaf, (unsigned long long)a);
        if (b) atomicAdd(leaf_acc + 3 * leaf + 1, (unsigned long long)b);
        if (e) atomicAdd(leaf_acc + 3 * leaf + 2, (unsigned long long)e);
      }
    }
  }
}

// --- C ABI of the segmented pipeline -----------------------------------------
H2OMX_API int h2omx_pc_rows() { return PC_ROWS; }

// in-bag root segment (bag_*_kernel): idx / gout / sout hold >= n entries, cnt
// >= ceil(n / BAG_CHUNK) ints; the root's seg_cnt / hc_first / pc_first are rewritten
H2OMX_API int h2omx_bag_compact(const float* w, long long n, const float* g, const float* s2, int* cnt, int* idx,
                                float* gout, float* sout, int* seg_cnt, int* hc_first, int* pc_first, int hc_rows,
                                hipStream_t stream) {
  if (!w || !g || !s2 || !cnt || !idx || !gout || !sout || !seg_cnt || !hc_first || !pc_first || n < 1 || hc_rows < 1)
    return kBadArg;
  const int nch = (int)((n + BAG_CHUNK - 1) / BAG_CHUNK);
  hipLaunchKernelGGL(bag_count_kernel, dim3(nch), dim3(256), 0, stream, w, (int64_t)n, cnt);
  hipLaunchKernelGGL(bag_scan_kernel, dim3(1), dim3(1024), 0, stream, cnt, nch, seg_cnt, hc_first, pc_first, hc_rows);
  hipLaunchKernelGGL(bag_scatter_kernel, dim3(nch), dim3(256), 0, stream, w, (int64_t)n, cnt, g, s2, idx, gout, sout);
  return launch_status();
}

H2OMX_API int h2omx_bag_route_out(const float* w, long long n, const uint8_t* codes_rm, int fp, const void* tree,
                                  int nbt, int* nid, hipStream_t stream) {
  if (!w || !codes_rm || !tree || !nid || n < 1 || fp < 1) return kBadArg;
  hipLaunchKernelGGL(bag_route_out_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, stream, w, (int64_t)n, codes_rm,
                     fp, reinterpret_cast<const TreeNode*>(tree), nbt, nid);
  return launch_status();
}

H2OMX_API int h2omx_tree_begin_seg(const unsigned int* stat_max, int mode, int max_rows_per_wg, double* qscale,
                                   int* ctl0, void* link0, unsigned long long* leaf_acc, int leaf_n,
                                   long long* built, int built_n, int n_rows, int hc_rows, int* seg_start,
                                   int* seg_cnt, int* hc_first, int* pc_first, int* slot_node, long long row_base,
                                   int tree_index, int* tree_ctr, hipStream_t stream) {
  if (max_rows_per_wg < 1 || max_rows_per_wg > ROWS_CAP || hc_rows > max_rows_per_wg) return kBadArg;
  const double qg = exp2(floor(log2(1073741824.0 / max_rows_per_wg)));
  const double qsr = exp2(floor(log2(2147483648.0 / max_rows_per_wg)));
  const int m = leaf_n > built_n ? leaf_n : built_n;
  hipLaunchKernelGGL(tree_begin_seg_kernel, dim3(grid_for(m, 256, 1024)), dim3(256), 0, stream, stat_max, mode, qg,
                     qsr, qscale, ctl0, reinterpret_cast<NodeLink*>(link0), leaf_acc, leaf_n, built, built_n, n_rows,
                     hc_rows, seg_start, seg_cnt, hc_first, pc_first, slot_node, row_base, tree_index, tree_ctr);
  return launch_status();
}

H2OMX_API int h2omx_hist_build_seg(const uint8_t* codes_rm, int fp, const int* idx, const float* g, const float* s2,
                                   const int* seg_start, const int* seg_cnt, const int* hc_first, const int* ctl,
                                   const int* nvb, const double* qscale, int salt, int F, int nbt, int fg,
                                   int n_groups, int hc_rows, int max_chunks, int threads,
                                   unsigned long long* slab, int gpos, const uint8_t* crow, const int* cpos,
                                   hipStream_t stream) {
  if (fg > 256 || threads > 512 || threads % 64 || threads < fg || fp % 4 || (n_groups > 1 && fg % 4) ||
      hc_rows > ROWS_CAP)
    return kBadArg;
  const size_t lds = (size_t)fg * nbt * sizeof(unsigned long long);
  if (lds > 156 * 1024) return kBadArg;
  const int grid = ((max_chunks + 7) / 8) * 8 * n_groups;
#define LAUNCH_HBS(NB)                                                                                        \
  hipLaunchKernelGGL(hist_build_seg_kernel<NB>, dim3(grid), dim3(threads), lds, stream, codes_rm, fp, idx, g, s2, \
                     seg_start, seg_cnt, hc_first, ctl, nvb, qscale, (uint32_t)salt, F, fg, n_groups, hc_rows, slab, \
                     gpos, crow, cpos)
  switch (nbt) {
    case 32: LAUNCH_HBS(32); break;
    case 64: LAUNCH_HBS(64); break;
    case 128: LAUNCH_HBS(128); break;
    case 256: LAUNCH_HBS(256); break;
    default: return kBadArg;
  }
#undef LAUNCH_HBS
  return launch_status();
}

H2OMX_API int h2omx_hist_reduce_seg(const unsigned long long* slab, const int* hc_first, const int* slot_node,
                                    const int* ctl, int F, int nbt, int fg, int n_groups, int max_slots, int ksplit,
                                    long long* built, hipStream_t stream) {
  if (ksplit < 1 || max_slots < 1) return kBadArg;
  dim3 grid((F * nbt + 255) / 256, max_slots, ksplit);
  hipLaunchKernelGGL(hist_reduce_seg_kernel, grid, dim3(256), 0, stream, slab, hc_first, slot_node, ctl, F, nbt, fg,
                     n_groups, built);
  return launch_status();
}

H2OMX_API int h2omx_part_count(const uint8_t* codes, int64_t npad, const int* idx, const int* seg_start,
                               const int* seg_cnt, const int* pc_first, const int* ctl, const void* part, int nbt,
                               int max_chunks, int* pc_left, int wave, int8_t* dirb, const uint8_t* ecodes,
                               int ecs, const int* nodeq, const uint8_t* crow, int fp, const int* cpos,
                               hipStream_t stream) {
  if (ecodes && !wave) return kBadArg;
  const SegRows sr{crow, nullptr, fp, cpos, nullptr};
  if (wave) {
    hipLaunchKernelGGL(part_count_wave_kernel, dim3((max_chunks + 3) / 4), dim3(256), 0, stream, codes, npad, idx,
                       seg_start, seg_cnt, pc_first, ctl, reinterpret_cast<const PartInfo*>(part), nbt, pc_left, dirb,
                       ecodes, ecs, nodeq, sr);
    return launch_status();
  }
  hipLaunchKernelGGL(part_count_kernel, dim3(max_chunks), dim3(256), 0, stream, codes, npad, idx, seg_start, seg_cnt,
                     pc_first, ctl, reinterpret_cast<const PartInfo*>(part), nbt, pc_left, sr, dirb);
  return launch_status();
}

H2OMX_API int h2omx_seg_direct(const uint8_t* codes_rm, int fp, const int* idx, const float* g, const float* s2,
                               const int* seg_start, const int* seg_cnt, const int* ctl, const int* nvb,
                               const uint8_t* tree_fmask, const double* qscale, int salt, const void* params, int nbt,
                               int max_nodes, int mode, const int* pc_first, int max_pc, unsigned long long* slab,
                               long long* tot_slab, int* ticket, void* nsplit, int gpos, uint8_t* ecodes, int ecs,
                               int* nodeq, const uint8_t* crow, const int* cpos, long long plane, hipStream_t stream) {
  if (ecodes && ecs != 8 && ecs != 16) return kBadArg;
  const ECodes ec{ecodes, ecs, nodeq, crow, cpos, plane > 0 ? 1 : fp, plane > 0 ? (int64_t)plane : 1};
  // moved code rows: XCD-aware block order over grids padded to a multiple of 8
  auto pad8 = [&](int g) { return crow ? (g + 7) / 8 * 8 : g; };
  // mode 0: one workgroup per node, 1: one wave per node (F <= 256),
  // 2: one workgroup per PC_ROWS chunk (slab / tot_slab: max_pc x max_elig x
  //    nbt and max_pc x 2 int64, ticket: max_nodes zeroed ints)
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (max_nodes < 1 || p.F > 1024 || p.F > fp || nbt < 2) return kBadArg;
  NodeSplit* ns = reinterpret_cast<NodeSplit*>(nsplit);
  // LDS sized to the features a node can have (mtries, else F): small
  // allocations keep many node workgroups resident per CU
  const int per_f_bytes = 2 * nbt * 8;
  const int max_elig = p.mtries > 0 ? std::min(p.mtries, p.F) : p.F;
  if (mode == 2) {
    if (max_elig * per_f_bytes > DIRECT_CHUNK_LDS || !pc_first || !slab || !tot_slab || !ticket) return kBadArg;
    hipLaunchKernelGGL(direct_empty_kernel, dim3((max_nodes + 255) / 256), dim3(256), 0, stream, seg_cnt, ctl, ns);
    const size_t lds = (size_t)max_elig * per_f_bytes;
#define LAUNCH_SDC(NB)                                                                                            \
  hipLaunchKernelGGL(seg_direct_chunk_kernel<NB>, dim3(pad8(max_pc)), dim3(256), lds, stream, codes_rm, fp, idx, g, s2, \
                     seg_start, seg_cnt, pc_first, ctl, nvb, tree_fmask, qscale, (uint32_t)salt, p, max_elig, slab, \
                     tot_slab, ticket, ns, gpos, ec)
    switch (nbt) {
      case 32: LAUNCH_SDC(32); break;
      case 64: LAUNCH_SDC(64); break;
      case 128: LAUNCH_SDC(128); break;
      case 256: LAUNCH_SDC(256); break;
      default: return kBadArg;
    }
#undef LAUNCH_SDC
    return launch_status();
  }
  if (mode == 1 && p.F <= DIRECT_WAVE_F) {
    const int batch = std::max(1, std::min(max_elig, DIRECT_WAVE_LDS / per_f_bytes));
    const size_t lds = (size_t)4 * batch * per_f_bytes;
#define LAUNCH_SDW(NB)                                                                                              \
  hipLaunchKernelGGL(seg_direct_wave_kernel<NB>, dim3(pad8((max_nodes + 3) / 4)), dim3(256), lds, stream, codes_rm, fp, \
                     idx, g, s2, seg_start, seg_cnt, ctl, nvb, tree_fmask, qscale, (uint32_t)salt, p, batch, ns, gpos, ec)
    switch (nbt) {
      case 32: LAUNCH_SDW(32); break;
      case 64: LAUNCH_SDW(64); break;
      case 128: LAUNCH_SDW(128); break;
      case 256: LAUNCH_SDW(256); break;
      default: return kBadArg;
    }
#undef LAUNCH_SDW
    return launch_status();
  }
  const int batch = std::max(1, std::min(max_elig, DIRECT_LDS_BYTES / per_f_bytes));
  const size_t lds = (size_t)batch * per_f_bytes;
#define LAUNCH_SD(NB)                                                                                             \
  hipLaunchKernelGGL(seg_direct_kernel<NB>, dim3(pad8(max_nodes)), dim3(64 * DIRECT_WAVES), lds, stream, codes_rm, fp, \
                     idx, g, s2,                                                                                 \
                     seg_start, seg_cnt, ctl, nvb, tree_fmask, qscale, (uint32_t)salt, p, batch, ns, gpos, ec)
  switch (nbt) {
    case 32: LAUNCH_SD(32); break;
    case 64: LAUNCH_SD(64); break;
    case 128: LAUNCH_SD(128); break;
    case 256: LAUNCH_SD(256); break;
    default: return kBadArg;
  }
#undef LAUNCH_SD
  return launch_status();
}

// column-major planes of this level's positions (seg_colmajor_kernel); plane:
// positions per feature plane (>= n rounded up to CM_ROWS, a multiple of 4)
// BinnedMatrix.codes_rm: rm [n][fp] (fp % 4 == 0, fp >= F, rm 16-byte aligned;
// 16-byte stores when fp % 16 == 0) from codes [F][npad] (npad % 64 == 0)
H2OMX_API int h2omx_codes_rowmajor(const uint8_t* codes, long long npad, int F, long long n, uint8_t* rm, int fp,
                                   hipStream_t stream) {
  if (!codes || !rm || n < 1 || F < 1 || fp < F || fp % 4 || npad % 64 || npad < n ||
      (reinterpret_cast<uintptr_t>(rm) & 15) || (reinterpret_cast<uintptr_t>(codes) & 3))
    return kBadArg;
  const int64_t nb = (n + RM_ROWS - 1) / RM_ROWS;
  hipLaunchKernelGGL(codes_rowmajor_kernel, dim3((unsigned)nb), dim3(256), 0, stream, codes, (int64_t)npad, F,
                     (int64_t)n, rm, fp);
  return launch_status();
}

H2OMX_API int h2omx_seg_colmajor(const uint8_t* codes_rm, int fp, int F, const int* idx, int n, long long nrows,
                                 uint8_t* ccol, long long plane, hipStream_t stream) {
  const int nb = (n + CM_ROWS - 1) / CM_ROWS;
  // dword layout: an odd pitch of W <= fp / 4 words; 16-byte layout (fp % 16 == 0):
  // an odd pitch of W16 = ceil(F / 16) chunks (seg_colmajor_kernel)
  const bool vec = (fp & 15) == 0 && (reinterpret_cast<uintptr_t>(codes_rm) & 15) == 0;
  const size_t lds = (size_t)CM_ROWS * (vec ? 16 * (((F + 15) >> 4) | 1) : fp + 4);
  if (n < 1 || fp % 4 || F < 1 || F > fp || lds > 128 * 1024 || plane % 4 || plane < (long long)nb * CM_ROWS ||
      !codes_rm || !ccol)
    return kBadArg;
  hipLaunchKernelGGL(seg_colmajor_kernel, dim3(nb), dim3(256), lds, stream, codes_rm, fp, F, idx, n,
                     (int64_t)nrows, ccol, (int64_t)plane);
  return launch_status();
}

// int64 entries per node of the data-parallel direct histogram buffer
H2OMX_API long long h2omx_direct_dp_stride(const void* params, int nbt) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  const int max_elig = p.mtries > 0 ? std::min(p.mtries, p.F) : p.F;
  return 2 + (long long)max_elig * 2 * nbt;
}

// phase 0: histograms of nodes [node0, node0 + n_chunk) into dh; phase 1: scan them
H2OMX_API int h2omx_direct_dp(int phase, const uint8_t* codes_rm, int fp, const int* idx, const float* g,
                              const float* s2, const int* seg_start, const int* seg_cnt, const int* ctl,
                              const int* nvb, const uint8_t* tree_fmask, const double* qscale, const void* params,
                              int nbt, int node0, int n_chunk, long long* dh, void* nsplit, int gpos,
                              const uint8_t* crow, hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  if (n_chunk < 1 || p.F > 1024 || p.F > fp || nbt < 2 || dh == nullptr) return kBadArg;
  const int max_elig = p.mtries > 0 ? std::min(p.mtries, p.F) : p.F;
  const int per_f_bytes = 2 * nbt * 8;
  const int batch = std::max(1, std::min(max_elig, DIRECT_LDS_BYTES / per_f_bytes));
  const size_t lds = (size_t)batch * per_f_bytes;
  NodeSplit* ns = reinterpret_cast<NodeSplit*>(nsplit);
#define LAUNCH_DDP(NB)                                                                                        \
  if (phase == 0)                                                                                            \
    hipLaunchKernelGGL(direct_dp_hist_kernel<NB>, dim3(n_chunk), dim3(256), lds, stream, codes_rm, fp, idx,  \
                       g, s2, seg_start, seg_cnt, ctl, tree_fmask, qscale, p, batch, node0, max_elig, dh,   \
                       gpos, crow);                                                                          \
  else                                                                                                       \
    hipLaunchKernelGGL(direct_dp_scan_kernel<NB>, dim3(n_chunk), dim3(256), 0, stream, ctl, nvb, tree_fmask,  \
                       qscale, p, node0, max_elig, dh, ns)
  switch (nbt) {
    case 32: LAUNCH_DDP(32); break;
    case 64: LAUNCH_DDP(64); break;
    case 128: LAUNCH_DDP(128); break;
    case 256: LAUNCH_DDP(256); break;
    default: return kBadArg;
  }
#undef LAUNCH_DDP
  return launch_status();
}

// level_finalize from per-node splits already in nsplit (direct mode)
H2OMX_API int h2omx_level_finalize_ns(const void* nsplit, const int* ctl, int* ctl_next, const void* params,
                                      const float* edges, const int* nvb, int nbt, int max_next_nodes, void* part,
                                      void* next_link, void* tree, int tree_capacity, int max_nodes, int* tiles,
                                      hipStream_t stream) {
  const SplitParams p = *reinterpret_cast<const SplitParams*>(params);
  level_finalize_launch(reinterpret_cast<const NodeSplit*>(nsplit), ctl, ctl_next, p, edges, nvb, nbt, max_next_nodes,
                        part, next_link, tree, tree_capacity, max_nodes, tiles, stream);
  return launch_status();
}

H2OMX_API int h2omx_level_close(const int* ctl, const int* ctl_next, const void* part, const void* link_next,
                                const int* seg_start, const int* seg_cnt, const int* pc_first, int* pc_left,
                                int* node_nl, int* nseg_start, int* nseg_cnt, int* nhc_first, int* npc_first,
                                int* nslot_node, int hc_rows, long long* nbuilt, int per_slot, hipStream_t stream) {
  hipLaunchKernelGGL(level_close_kernel, dim3(1), dim3(1024), 0, stream, ctl, ctl_next,
                     reinterpret_cast<const PartInfo*>(part), reinterpret_cast<const NodeLink*>(link_next), seg_start,
                     seg_cnt, pc_first, pc_left, node_nl, nseg_start, nseg_cnt, nhc_first, npc_first, nslot_node,
                     hc_rows, nbuilt, per_slot);
  if (nbuilt)
    hipLaunchKernelGGL(zero_slots_kernel, dim3(1024), dim3(256), 0, stream, nbuilt, ctl_next, per_slot);
  return launch_status();
}

static int device_scan(const int* in, int* out, int* tiles, const int* aux, int k, int max_count, int* total_out,
                       bool write_end, hipStream_t stream) {
  const int nt = (max_count + SCAN_TILE - 1) / SCAN_TILE;
  if (nt < 1) return kOk;
  hipLaunchKernelGGL(scan_tiles_kernel, dim3(nt), dim3(SCAN_TILE), 0, stream, in, out, tiles, aux, k);
  hipLaunchKernelGGL(scan_tile_sums_kernel, dim3(1), dim3(SCAN_TILE), 0, stream, tiles, write_end ? out : nullptr,
                     aux, k, total_out);
  hipLaunchKernelGGL(scan_add_kernel, dim3(nt), dim3(SCAN_TILE), 0, stream, out, tiles, aux, k);
  return launch_status();
}

// Multi-block level close; scratch: pc_excl[max_pc], tiles[max(max_pc, next_nodes)/1024 + 1],
// cnt_h / cnt_p[next_nodes], aux[4]
H2OMX_API int h2omx_level_close_mb(const int* ctl, const int* ctl_next, const void* part, const void* link_next,
                                   const int* seg_start, const int* seg_cnt, const int* pc_first, int* pc_left,
                                   int* node_nl, int* nseg_start, int* nseg_cnt, int* nhc_first, int* npc_first,
                                   int* nslot_node, int hc_rows, long long* nbuilt, int per_slot, int max_nodes,
                                   int max_pc, int* pc_excl, int* tiles, int* cnt_h, int* cnt_p, int* aux,
                                   hipStream_t stream) {
  hipLaunchKernelGGL(close_prep_kernel, dim3(1), dim3(64), 0, stream, ctl, ctl_next, pc_first, aux);
  int rc = device_scan(pc_left, pc_excl, tiles, aux, 0, max_pc, aux + 2, false, stream);
  if (rc) return rc;
  const int nb = std::max(1, std::min(4096, (max_nodes + 255) / 256));
  hipLaunchKernelGGL(node_close_kernel, dim3(nb), dim3(256), 0, stream, ctl, reinterpret_cast<const PartInfo*>(part),
                     reinterpret_cast<const NodeLink*>(link_next), seg_start, seg_cnt, pc_first, pc_excl, aux,
                     pc_left, node_nl, nseg_start, nseg_cnt, cnt_h, cnt_p, nslot_node, hc_rows);
  rc = device_scan(cnt_h, nhc_first, tiles, aux, 1, 2 * max_nodes, nullptr, true, stream);
  if (rc) return rc;
  rc = device_scan(cnt_p, npc_first, tiles, aux, 1, 2 * max_nodes, nullptr, true, stream);
  if (rc) return rc;
  if (nbuilt) hipLaunchKernelGGL(zero_slots_kernel, dim3(1024), dim3(256), 0, stream, nbuilt, ctl_next, per_slot);
  return launch_status();
}

H2OMX_API int h2omx_part_scatter(const uint8_t* codes, int64_t npad, const int* idx, int* idx_out, int* nid,
                                 int write_nid, const int* seg_start, const int* seg_cnt, const int* pc_first,
                                 const int* pc_off, const int* node_nl, const int* ctl, const void* part, int nbt,
                                 const float* g, const float* h, const float* w, const double* qscale, int cap,
                                 unsigned long long* leaf_acc, int max_chunks, int wave, const int8_t* dirb,
                                 const float* gin, const float* sin, float* gout, float* sout,
                                 const uint8_t* ecodes, int ecs, const int* nodeq, const uint8_t* codes_rm,
                                 const uint8_t* crow_in, uint8_t* crow_out, int fp, const int* cpos_in, int* cpos_out,
                                 hipStream_t stream) {
  // crow_out: move every inner row's code row into the next level's segment order
  // (source crow_in by position, or codes_rm by row id when crow_in is nullptr);
  // cpos_out: the rows stay where they are in crow_in, their positions move
  const SegRows sr{crow_in, crow_out, fp, cpos_in, cpos_out};
  if (crow_out != nullptr && ((crow_in == nullptr && codes_rm == nullptr) || fp % 4 != 0 || cpos_in || cpos_out))
    return kBadArg;
  // (cpos without crow_in: column-major planes outside SegRows, the split codes
  // are gathered from the feature-major codes by row id)
  // wave: bit 0 wave-granular kernel; bits 1-2 its segf flags (last level)
  const int segf = wave >> 1;
  wave &= 1;
  if ((ecodes || segf) && !wave) return kBadArg;
  if ((segf & 1) && (!gin || ((segf & 2) && !sin))) return kBadArg;
  if (wave) {
    hipLaunchKernelGGL(part_scatter_wave_kernel, dim3((max_chunks + 3) / 4), dim3(256), 0, stream, codes, npad, idx,
                       idx_out, nid, write_nid, seg_start, seg_cnt, pc_first, pc_off, node_nl, ctl,
                       reinterpret_cast<const PartInfo*>(part), nbt, g, h, w, qscale, cap, leaf_acc, dirb, gin, sin,
                       gout, sout, ecodes, ecs, nodeq, segf, sr, codes_rm);
    return launch_status();
  }
  hipLaunchKernelGGL(part_scatter_kernel, dim3(max_chunks), dim3(256), 0, stream, codes, npad, idx, idx_out, nid,
                     write_nid, seg_start, seg_cnt, pc_first, pc_off, node_nl, ctl,
                     reinterpret_cast<const PartInfo*>(part), nbt, g, h, w, qscale, cap, leaf_acc, gin, sin, gout,
                     sout, sr, codes_rm, dirb);
  return launch_status();
}
