// Model explanation kernels: path-dependent TreeSHAP contributions for tree
// ensembles (H2O predict_contributions for GBM / DRF / XGBoost).
//
// The host flattens every root-to-leaf path of the ensemble into a leaf
// record {first element, unique features m, leaf value} and m path elements
// {feature | na_ok << 30 | categorical << 29, zero fraction z, lo, hi}: a row
// "follows" the path on feature f (one fraction o = 1) when lo < x <= hi (NA:
// na_ok; categorical: level x in the path's level set sets[lo]), and z is
// the product of the cover ratios of the path's edges on f.  For the path
// polynomial P(t) = prod_j (z_j + o_j t) the Shapley contribution of
// element i is
//     phi_i += v (o_i - z_i) sum_k w(m, k) [t^k] P(t) / (z_i + o_i t),
// w(m, k) = k! (m - 1 - k)! / m!   (Lundberg et al. 2020, path form used by
// GPUTreeShap).  One thread per row walks the same leaf list, so leaf and
// element loads are wave-uniform (scalar / broadcast) and the per-feature
// accumulators are written coalesced: in LDS ([F][256] per workgroup) when
// they fit, else straight to the feature-major output.
#include "common.h"

namespace {

template <int MAXM, bool LDS>
__global__ __launch_bounds__(256) void tree_shap_kernel(const float* __restrict__ X, int64_t ld, int64_t n, int F,
                                                        const int4* __restrict__ leaves, int nleaves,
                                                        const float4* __restrict__ elems,
                                                        const float* __restrict__ wtab, float* __restrict__ out,
                                                        const uint32_t* __restrict__ sets) {
  extern __shared__ float acc[];
  __shared__ float w_s[(MAXM + 1) * (MAXM + 1)];
  const int tid = threadIdx.x;
  const int64_t r = (int64_t)blockIdx.x * 256 + tid;
  const bool live = r < n;
  const int64_t rr = live ? r : 0;
  for (int j = tid; j < (MAXM + 1) * (MAXM + 1); j += 256) w_s[j] = wtab[j];
  if (LDS)
    for (int j = tid; j < F * 256; j += 256) acc[j] = 0.0f;
  __syncthreads();
  for (int L = 0; L < nleaves; ++L) {
    const int4 hd = leaves[L];
    const int m = hd.y;
    const float v = __int_as_float(hd.z);
    float z[MAXM], o[MAXM];
    int fe[MAXM];
    float P[MAXM + 1];
    P[0] = 1.0f;
#pragma unroll
    for (int k = 1; k <= MAXM; ++k) P[k] = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      z[j] = 1.0f; o[j] = 1.0f; fe[j] = 0;
      if (j < m) {
        const float4 e = elems[hd.x + j];
        const int fi = __float_as_int(e.x);
        const int f = fi & 0x1FFFFFFF;
        const float x = X[(int64_t)f * ld + rr];
        float oj;
        if (x != x) {
          oj = (float)((fi >> 30) & 1);
        } else if ((fi >> 29) & 1) {
          // categorical feature: the path's allowed level set (unseen levels: NA direction)
          const int b = (int)x;
          const uint32_t* st = sets + 8 * (int64_t)e.z;
          oj = (b < 0 || b > 255) ? (float)((fi >> 30) & 1) : (float)((st[b >> 5] >> (b & 31)) & 1u);
        } else {
          oj = (x > e.z && x <= e.w) ? 1.0f : 0.0f;
        }
        z[j] = e.y; o[j] = oj; fe[j] = f;
#pragma unroll
        for (int k = MAXM; k >= 1; --k)
          if (k <= j + 1) P[k] = e.y * P[k] + oj * P[k - 1];
        P[0] *= e.y;
      }
    }
    const float* wm = w_s + m * (MAXM + 1);
#pragma unroll
    for (int i = 0; i < MAXM; ++i) {
      if (i < m) {
        const float zi = z[i], oi = o[i];
        float s = 0.0f;
        if (oi != 0.0f) {
          // P / (z_i + t) by synthetic division from the top coefficient
          float carry = 0.0f;
#pragma unroll
          for (int k = MAXM; k >= 1; --k) {
            if (k <= m) {
              const float q = P[k] - zi * carry;
              s += q * wm[k - 1];
              carry = q;
            }
          }
        } else if (zi > 0.0f) {
          const float inv = 1.0f / zi;
#pragma unroll
          for (int k = 0; k < MAXM; ++k)
            if (k < m) s += P[k] * inv * wm[k];
        }
        const float phi = v * (oi - zi) * s;
        if (LDS) acc[fe[i] * 256 + tid] += phi;
        else if (live) out[(int64_t)fe[i] * n + r] += phi;
      }
    }
  }
  if (LDS) {
    __syncthreads();
    if (live)
      for (int f = 0; f < F; ++f) out[(int64_t)f * n + r] = acc[f * 256 + tid];
  }
}

}  // namespace

H2OMX_API int h2omx_tree_shap(const float* X, int64_t ld, int64_t n, int F, const void* leaves, int nleaves,
                              const void* elems, const float* wtab, int maxm, float* out, const uint32_t* sets,
                              hipStream_t stream) {
  if (n <= 0) return kOk;
  if (F <= 0 || maxm < 1 || maxm > 32) return kBadArg;
  const int grid = (int)((n + 255) / 256);
  const bool lds = (size_t)F * 256 * sizeof(float) <= 64 * 1024;
  const size_t shm = lds ? (size_t)F * 256 * sizeof(float) : 0;
  const int4* lv = reinterpret_cast<const int4*>(leaves);
  const float4* el = reinterpret_cast<const float4*>(elems);
#define LAUNCH_SHAP(M)                                                                                           \
  do {                                                                                                          \
    if (lds)                                                                                                    \
      hipLaunchKernelGGL((tree_shap_kernel<M, true>), dim3(grid), dim3(256), shm, stream, X, ld, n, F, lv,      \
                         nleaves, el, wtab, out, sets);                                                         \
    else                                                                                                        \
      hipLaunchKernelGGL((tree_shap_kernel<M, false>), dim3(grid), dim3(256), 0, stream, X, ld, n, F, lv,       \
                         nleaves, el, wtab, out, sets);                                                         \
  } while (0)
  if (maxm <= 8) LAUNCH_SHAP(8);
  else if (maxm <= 16) LAUNCH_SHAP(16);
  else LAUNCH_SHAP(32);
#undef LAUNCH_SHAP
  return launch_status();
}
