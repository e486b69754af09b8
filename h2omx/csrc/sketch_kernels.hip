// K1 quantile sketch: exact per-feature order statistics
// of the binning sample without sorting it.  Part of libh2omx_tree.
//
// The reference's H2O-3 image computes GBM / DRF / XGBoost cut points from
// quantiles of the data (hex/tree/DHistogram, QuantilesGlobal; deployed by
// isgasho/h2o-kubernetes templates.rs:28-30).  h2omx takes the numpy 'lower'
// quantiles of a row sample (binning.py _edges_from_sorted); this file finds
// exactly those order statistics with a two-level radix select:
//
//   1. sketch_hist: every sample's order-preserving 32-bit key goes into a
//      65536-bin histogram of its top 16 bits (per feature; 16-bit LDS
//      counters per 65535-sample chunk, flushed to global; NaN keys =
//      0xFFFFFFFF land in the last bin alone).
//   2. sketch_plan (one workgroup per feature): prefix sums of the bins, the
//      non-NaN count, the target ranks floor((cnt - 1) q_j) in fp64 (numpy's
//      expression), each target's bin and its rank inside it; those bins are
//      marked.  A feature with <= max_value_bins non-empty bins is a
//      low-cardinality candidate instead: all its non-empty bins are marked.
//   3. sketch_gather: the keys of marked bins (<= 256 slots per feature) into
//      per-bin segments, one global range claim per (chunk, slot).
//   4. sketch_select (one workgroup per target): bitonic sort of the bin's
//      segment in LDS (<= SK_MAX_BIN keys) and the key at the in-bin rank; a
//      larger bin must hold one distinct key.  sketch_distinct: the single
//      key of every non-empty bin of a low-cardinality candidate.
//      Anything else (a big mixed bin, two values in one bin of a
//      low-cardinality candidate) flags the feature for the sort path.
// The answers are the keys a full sort would put at those ranks (exact,
// deterministic).
#include "common.h"

namespace {

constexpr int SK_BINS = 65536;
constexpr int SK_MAX_BIN = 8192;     // largest bin refined in LDS (32 KB of keys)

__device__ __forceinline__ uint32_t sk_key(float v) {
  if (v != v) return 0xFFFFFFFFu;    // NaN: sorts last, alone in the last bin
  if (v == 0.0f) return 0x80000000u;  // -0 == +0 (one value, as numpy's unique / sort compare)
  const uint32_t b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

}  // namespace

// one 1024-thread workgroup per (chunk of <= SK_CHUNK samples, feature): the
// 65536 counts as 16-bit halves of 32768 LDS words (a chunk cannot overflow a
// half), then the non-zero bins are added to the global histogram
constexpr int SK_CHUNK = 65535;
__global__ __launch_bounds__(1024) void sketch_hist_kernel(const float* __restrict__ S, int64_t ld, int m,
                                                           unsigned int* __restrict__ H) {
  __shared__ unsigned int cw[SK_BINS / 2];
  const int f = blockIdx.y;
  for (int i = threadIdx.x; i < SK_BINS / 2; i += blockDim.x) cw[i] = 0u;
  __syncthreads();
  const float* col = S + (int64_t)f * ld;
  const int i0 = blockIdx.x * SK_CHUNK, i1 = min(m, i0 + SK_CHUNK);
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint32_t b = sk_key(col[i]) >> 16;
    atomicAdd(&cw[b >> 1], 1u << (16 * (b & 1)));
  }
  __syncthreads();
  unsigned int* h = H + (int64_t)f * SK_BINS;
  for (int i = threadIdx.x; i < SK_BINS / 2; i += blockDim.x) {
    const unsigned int v = cw[i];
    if (v & 0xFFFFu) atomicAdd(h + 2 * i, v & 0xFFFFu);
    if (v >> 16) atomicAdd(h + 2 * i + 1, v >> 16);
  }
}

// per feature f (one 1024-thread workgroup):
//   P[f][b] exclusive prefix of H; tbin / trank of the T quantile ranks and the
//   maximum; mark[f][b] (bin to gather), off[f][b] (its segment start);
//   low-cardinality candidates (<= max_value_bins non-empty bins) gather every
//   non-empty bin instead and list them ascending in lcbin[f][*];
//   info[f] = cnt, non-empty bins, low-cardinality candidate, fallback (0 here)
__device__ __forceinline__ unsigned int sk_block_excl_scan(unsigned int local, unsigned int* wsum,
                                                           unsigned int* total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned int incl = local;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  __syncthreads();
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  if (t == 0) {
    unsigned int a = 0;
    for (int i = 0; i < 16; ++i) { const unsigned int v = wsum[i]; wsum[i] = a; a += v; }
    wsum[16] = a;
  }
  __syncthreads();
  if (total) *total = wsum[16];
  return wsum[w] + incl - local;
}

__global__ __launch_bounds__(1024) void sketch_plan_kernel(const unsigned int* __restrict__ H, int T,
                                                           const double* __restrict__ qv, int max_value_bins,
                                                           unsigned int* __restrict__ P, int* __restrict__ tbin,
                                                           int* __restrict__ trank, int* __restrict__ mark,
                                                           unsigned int* __restrict__ off, int* __restrict__ lcbin,
                                                           int* __restrict__ info) {
  const int f = blockIdx.x;
  const int t = threadIdx.x;
  constexpr int PER = SK_BINS / 1024;
  const unsigned int* h = H + (int64_t)f * SK_BINS;
  unsigned int* p = P + (int64_t)f * SK_BINS;
  int* mk = mark + (int64_t)f * SK_BINS;
  unsigned int* of = off + (int64_t)f * SK_BINS;
  __shared__ unsigned int wsum[17];
  // 1. prefix sums of the counts (64 consecutive bins per thread) + non-empty bins
  unsigned int local = 0, ne = 0;
  for (int i = 0; i < PER; ++i) {
    const int b = t * PER + i;
    const unsigned int c = h[b];
    local += c;
    ne += (c != 0u && b != SK_BINS - 1) ? 1u : 0u;
  }
  unsigned int total, nonempty;
  unsigned int run = sk_block_excl_scan(local, wsum, &total);
  sk_block_excl_scan(ne, wsum, &nonempty);
  const bool lowcand = (int)nonempty <= max_value_bins;
  for (int i = 0; i < PER; ++i) {
    const int b = t * PER + i;
    const unsigned int c = h[b];
    p[b] = run;
    run += c;
    const bool used = c != 0u && b != SK_BINS - 1;
    mk[b] = (lowcand && used) ? 1 : 0;
  }
  __syncthreads();
  const int cnt = (int)(total - h[SK_BINS - 1]);   // non-NaN samples
  // 2. quantile targets (high-cardinality features): T ranks + the maximum
  if (!lowcand) {
    for (int j = t; j <= T; j += blockDim.x) {
      int r;
      if (j < T) r = (int)floor((double)((cnt > 1 ? cnt : 1) - 1) * qv[j]);
      else r = cnt > 0 ? cnt - 1 : 0;
      int lo = 0, hi = SK_BINS - 2;      // last bin with P[b] <= r (the bin holding rank r)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (p[mid] <= (unsigned)r) lo = mid; else hi = mid - 1;
      }
      tbin[f * (T + 1) + j] = lo;
      trank[f * (T + 1) + j] = r - (int)p[lo];
      mk[lo] = 1;
    }
  }
  __syncthreads();
  // 3. segment offsets of the marked bins, and their slot ids (ascending bin
  //    order, <= 256 per feature): mark[b] = slot + 1, lcbin[f][slot] = b
  local = 0;
  unsigned int nm = 0;
  for (int i = 0; i < PER; ++i) {
    const int b = t * PER + i;
    if (mk[b]) { local += h[b]; ++nm; }
  }
  run = sk_block_excl_scan(local, wsum, nullptr);
  unsigned int srun = sk_block_excl_scan(nm, wsum, nullptr);
  for (int i = 0; i < PER; ++i) {
    const int b = t * PER + i;
    of[b] = run;
    if (mk[b]) {
      run += h[b];
      mk[b] = (int)srun + 1;
      lcbin[f * 256 + (int)srun] = b;
      ++srun;
    }
  }
  if (t == 0) {
    info[4 * f + 0] = cnt;
    info[4 * f + 1] = (int)nonempty;
    info[4 * f + 2] = lowcand ? 1 : 0;
    info[4 * f + 3] = 0;
  }
}

// one 1024-thread workgroup per (chunk of SK_CHUNK samples, feature): marked
// samples counted per slot in LDS, one global claim per (chunk, slot), then a
// second pass writes each sample into its claimed range (LDS slot cursors)
__global__ __launch_bounds__(1024) void sketch_gather_kernel(const float* __restrict__ S, int64_t ld, int m,
                                                             const int* __restrict__ mark,
                                                             const unsigned int* __restrict__ off,
                                                             const int* __restrict__ lcbin,
                                                             unsigned int* __restrict__ fill,
                                                             unsigned int* __restrict__ buf) {
  __shared__ unsigned int cnt[256], base[256];
  const int f = blockIdx.y;
  const int* mk = mark + (int64_t)f * SK_BINS;
  unsigned int* out = buf + (int64_t)f * m;
  const float* col = S + (int64_t)f * ld;
  const int i0 = blockIdx.x * SK_CHUNK, i1 = min(m, i0 + SK_CHUNK);
  if (threadIdx.x < 256) cnt[threadIdx.x] = 0u;
  __syncthreads();
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int sl = mk[sk_key(col[i]) >> 16] - 1;
    if (sl >= 0) atomicAdd(&cnt[sl], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 256) {
    const unsigned int c = cnt[threadIdx.x];
    if (c) {
      const int b = lcbin[f * 256 + threadIdx.x];
      base[threadIdx.x] = off[(int64_t)f * SK_BINS + b] + atomicAdd(fill + (int64_t)f * SK_BINS + b, c);
    }
    cnt[threadIdx.x] = 0u;
  }
  __syncthreads();
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint32_t k = sk_key(col[i]);
    const int sl = mk[k >> 16] - 1;
    if (sl >= 0) out[base[sl] + atomicAdd(&cnt[sl], 1u)] = k;
  }
}

// min / max of a segment by the whole workgroup
__device__ __forceinline__ void sk_minmax(const unsigned int* __restrict__ src, int n, unsigned int* smin,
                                          unsigned int* smax, unsigned int& lo, unsigned int& hi) {
  unsigned int a = 0xFFFFFFFFu, c = 0u;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const unsigned int v = src[i];
    a = min(a, v);
    c = max(c, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    a = min(a, (unsigned int)__shfl_xor((int)a, o, 64));
    c = max(c, (unsigned int)__shfl_xor((int)c, o, 64));
  }
  if (threadIdx.x == 0) { *smin = 0xFFFFFFFFu; *smax = 0u; }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) { atomicMin(smin, a); atomicMax(smax, c); }
  __syncthreads();
  lo = *smin;
  hi = *smax;
}

// grid (T + 1, F): the key at quantile target j of a high-cardinality feature.
// Bins up to SK_MAX_BIN keys are bitonic-sorted in LDS; a larger bin is
// answered only when it holds one distinct key, otherwise the feature takes
// the sort path (info[f][3] = 1).
__global__ __launch_bounds__(1024) void sketch_select_kernel(const unsigned int* __restrict__ H, int m, int T,
                                                             const int* __restrict__ tbin,
                                                             const int* __restrict__ trank,
                                                             const unsigned int* __restrict__ off,
                                                             int* __restrict__ info,
                                                             const unsigned int* __restrict__ buf,
                                                             unsigned int* __restrict__ out_key) {
  const int f = blockIdx.y, j = blockIdx.x;
  if (info[4 * f + 2] || info[4 * f + 0] == 0) return;   // low-cardinality / empty feature (uniform)
  const int tj = f * (T + 1) + j;
  __shared__ unsigned int keys[SK_MAX_BIN];
  __shared__ unsigned int smin, smax;
  const int b = tbin[tj];
  const int n = (int)H[(int64_t)f * SK_BINS + b];
  const unsigned int* src = buf + (int64_t)f * m + off[(int64_t)f * SK_BINS + b];
  if (n > SK_MAX_BIN) {
    unsigned int lo, hi;
    sk_minmax(src, n, &smin, &smax, lo, hi);
    if (threadIdx.x == 0) {
      out_key[tj] = lo;
      if (lo != hi) atomicOr(info + 4 * f + 3, 1);
    }
    return;
  }
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += blockDim.x) keys[i] = (i < n) ? src[i] : 0xFFFFFFFFu;
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int st = k >> 1; st > 0; st >>= 1) {
      for (int i = threadIdx.x; i < np2; i += blockDim.x) {
        const int l = i ^ st;
        if (l > i) {
          const unsigned int a = keys[i], c = keys[l];
          if ((a > c) == ((i & k) == 0)) { keys[i] = c; keys[l] = a; }
        }
      }
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) out_key[tj] = keys[trank[tj]];
}

// grid (256, F): the single key of non-empty bin s of a low-cardinality
// candidate; a bin holding two distinct keys sends the feature to the sort path
__global__ __launch_bounds__(1024) void sketch_distinct_kernel(const unsigned int* __restrict__ H, int m,
                                                               const int* __restrict__ lcbin,
                                                               const unsigned int* __restrict__ off,
                                                               int* __restrict__ info,
                                                               const unsigned int* __restrict__ buf,
                                                               unsigned int* __restrict__ lckey) {
  const int f = blockIdx.y, sidx = blockIdx.x;
  if (!info[4 * f + 2] || sidx >= info[4 * f + 1]) return;   // uniform
  __shared__ unsigned int smin, smax;
  const int b = lcbin[f * 256 + sidx];
  const int n = (int)H[(int64_t)f * SK_BINS + b];
  unsigned int lo, hi;
  sk_minmax(buf + (int64_t)f * m + off[(int64_t)f * SK_BINS + b], n, &smin, &smax, lo, hi);
  if (threadIdx.x == 0) {
    lckey[f * 256 + sidx] = lo;
    if (lo != hi) atomicOr(info + 4 * f + 3, 1);
  }
}

H2OMX_API int h2omx_sketch_bins() { return SK_BINS; }

// S [F][ld] float32 sample; T quantile levels qv (fp64); work buffers sized by
// the caller: H / MN / MX / P / mark / off / fill [F][SK_BINS], tbin / trank /
// out_key / out_open [F][T + 1], info [F][4], buf [F][m].
// S [F][ld] float32 sample; T quantile levels qv (fp64, T <= 1023); work
// buffers of the caller: H / P / mark / off / fill [F][SK_BINS], tbin / trank /
// out_key [F][T + 1], lcbin / lckey [F][256], info [F][4], buf [F][m].
H2OMX_API int h2omx_sketch(const float* S, int64_t ld, int m, int F, int T, const double* qv, int max_value_bins,
                           unsigned int* H, unsigned int* P, int* mark, unsigned int* off, unsigned int* fill,
                           int* tbin, int* trank, unsigned int* out_key, int* lcbin, unsigned int* lckey, int* info,
                           unsigned int* buf, hipStream_t stream) {
  if (m < 1 || F < 1 || T < 0 || T > 1023 || ld < m || max_value_bins > 255) return kBadArg;
  const size_t nb = (size_t)F * SK_BINS * sizeof(unsigned int);
  if (hipMemsetAsync(H, 0, nb, stream) != hipSuccess || hipMemsetAsync(fill, 0, nb, stream) != hipSuccess)
    return kLaunchFailed;
  const int chunks = (m + SK_CHUNK - 1) / SK_CHUNK;
  hipLaunchKernelGGL(sketch_hist_kernel, dim3(chunks, F), dim3(1024), 0, stream, S, ld, m, H);
  hipLaunchKernelGGL(sketch_plan_kernel, dim3(F), dim3(1024), 0, stream, H, T, qv, max_value_bins, P, tbin, trank,
                     mark, off, lcbin, info);
  hipLaunchKernelGGL(sketch_gather_kernel, dim3(chunks, F), dim3(1024), 0, stream, S, ld, m, mark, off, lcbin, fill,
                     buf);
  hipLaunchKernelGGL(sketch_select_kernel, dim3(T + 1, F), dim3(1024), 0, stream, H, m, T, tbin, trank, off, info,
                     buf, out_key);
  hipLaunchKernelGGL(sketch_distinct_kernel, dim3(256, F), dim3(1024), 0, stream, H, m, lcbin, off, info, buf,
                     lckey);
  return launch_status();
}
