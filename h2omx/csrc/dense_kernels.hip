// Dense (matrix-shaped) hot paths on fp32 MFMA for gfx950:
//   * GLM IRLS: one fused pass per iteration computes eta = X beta, the IRLS
//     weights / working response, and the weighted Gram [X 1 z]^T W [X 1 z]
//     (X^T W X, X^T W z, z^T W z) with v_mfma_f32_32x32x2_f32 from an
//     LDS-staged row chunk; per-workgroup fp32 slabs are reduced in fp64.
//   * K-Means: LDS-staged row chunk, centroid distances by MFMA
//     (D = C . X^T so every lane owns one row's distances), in-register
//     arg-min, and atomic-free per-workgroup cluster sums.
//   * MLP: a tiled fp32-MFMA GEMM (NN / NT / TN) with a fused bias +
//     activation epilogue, plus the small elementwise kernels of the
//     backward pass and the ADADELTA / momentum optimizers.
// fp32-input MFMA is exact fp32 (a k-ordered fmaf chain; see
// cdna_hip_programming.md §3), so results match an fp32 reference.
//
// Reference parity: the reference deploys H2O-3 (templates.rs:28-30 of
// isgasho/h2o-kubernetes) whose GLM / K-Means / DeepLearning these replace
// (SURVEY.md §2.5 K10-K16).
#include "common.h"

#include <math.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ===========================================================================
// GLM IRLS pass
// ===========================================================================
struct GlmParams {
  int family;  // 0 gaussian 1 binomial 2 poisson 3 gamma 4 tweedie 5 multinomial 6 quasibinomial
  int link;    // 0 identity 1 logit 2 log 3 inverse 4 tweedie-power
  int p;       // features (without intercept)
  int K;       // classes for multinomial, else 1
  int cls;     // class being updated (multinomial)
  int pad;
  double var_power;   // tweedie variance power
  double link_power;  // tweedie link power
};

__device__ __forceinline__ void glm_link(const GlmParams& P, double eta, double& mu, double& dmu) {
  switch (P.link) {
    case 1: {
      const double e = exp(-fabs(eta));
      const double s = eta >= 0 ? 1.0 / (1.0 + e) : e / (1.0 + e);
      mu = s;
      dmu = fmax(s * (1.0 - s), 1e-10);
      break;
    }
    case 2: mu = exp(fmin(eta, 700.0)); dmu = fmax(mu, 1e-10); break;
    case 3: {
      const double e = (fabs(eta) < 1e-10) ? copysign(1e-10, eta) : eta;
      mu = 1.0 / e;
      dmu = -mu * mu;
      break;
    }
    case 4: {
      const double q = P.link_power;
      if (q == 0.0) { mu = exp(fmin(eta, 700.0)); dmu = fmax(mu, 1e-10); }
      else { const double e = fmax(eta, 1e-10); mu = pow(e, 1.0 / q); dmu = mu / (q * e); }
      break;
    }
    default: mu = eta; dmu = 1.0;
  }
}

__device__ __forceinline__ double glm_var(const GlmParams& P, double mu) {
  switch (P.family) {
    case 1: case 6: return fmax(mu * (1.0 - mu), 1e-10);
    case 2: return fmax(mu, 1e-10);
    case 3: return fmax(mu * mu, 1e-20);
    case 4: return fmax(pow(fmax(mu, 1e-10), P.var_power), 1e-20);
    default: return 1.0;
  }
}

__device__ __forceinline__ double glm_dev(const GlmParams& P, double y, double mu) {
  switch (P.family) {
    case 1: case 6: {
      const double m = fmin(fmax(mu, 1e-15), 1.0 - 1e-15);
      return -2.0 * (y * log(m) + (1.0 - y) * log(1.0 - m));
    }
    case 2: {
      const double m = fmax(mu, 1e-15);
      return 2.0 * ((y > 0 ? y * log(y / m) : 0.0) - (y - m));
    }
    case 3: {
      const double m = fmax(mu, 1e-15), yy = fmax(y, 1e-15);
      return 2.0 * (-log(yy / m) + (y - m) / m);
    }
    case 4: {
      const double r = P.var_power, m = fmax(mu, 1e-15);
      const double a = (y > 0) ? pow(y, 2 - r) / ((1 - r) * (2 - r)) : 0.0;
      return 2.0 * (a - y * pow(m, 1 - r) / (1 - r) + pow(m, 2 - r) / (2 - r));
    }
    default: return (y - mu) * (y - mu);
  }
}

constexpr int GLM_RB = 64;  // rows per LDS chunk

template <int TP>
__global__ __launch_bounds__(256) void glm_irls_kernel(const float* __restrict__ X, int64_t ld, int64_t n,
                                                       const float* __restrict__ y, const float* __restrict__ wprior,
                                                       const float* __restrict__ offset,
                                                       const float* __restrict__ means,
                                                       const float* __restrict__ beta, GlmParams P,
                                                       int64_t rows_per_wg, float* __restrict__ slab,
                                                       double* __restrict__ dev_out) {
  constexpr int PP = 32 * TP;            // padded augmented width [X | 1 | z | 0...]
  constexpr int LDR = GLM_RB + 1;        // +1 float row pad: conflict-free column reads
  constexpr int T = TP * (TP + 1) / 2;   // upper-triangular 32x32 tiles
  constexpr int NT = (T + 3) / 4;        // tiles per wave
  __shared__ float A[PP * LDR];
  __shared__ float sw[GLM_RB], sz[GLM_RB];
  __shared__ double part[4][GLM_RB];
  __shared__ double devred[4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int p = P.p;
  const int64_t r_begin = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r_end = min(n, r_begin + rows_per_wg);

  for (int j = t; j < PP * LDR; j += 256) A[j] = 0.0f;  // padding columns stay zero
  f32x16 acc[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[u][e] = 0.0f;
  int ti_[NT], tj_[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    int id = wid + 4 * u, ti = 0;
    while (id >= TP - ti && ti < TP) { id -= TP - ti; ++ti; }
    ti_[u] = ti;
    tj_[u] = ti + id;
  }
  double dev_acc = 0.0;
  const float* bk = beta + (int64_t)P.cls * (p + 1);
  __syncthreads();

  for (int64_t r0 = r_begin; r0 < r_end; r0 += GLM_RB) {
    // 1. stage X (mean-imputed) column-major into LDS
    for (int j = t; j < p * GLM_RB; j += 256) {
      const int c = j >> 6, r = j & 63;
      float v = 0.0f;
      if (r0 + r < r_end) {
        v = X[(int64_t)c * ld + r0 + r];
        if (v != v) v = means[c];
      }
      A[c * LDR + r] = v;
    }
    __syncthreads();
    // 2. linear predictors: 4 partial dot products per row
    {
      const int r = t & 63, q = t >> 6;
      if (P.family == 5) {
        // multinomial: need every class' eta for the softmax
        double mx = -1e300, den = 0.0, ek = 0.0;
        for (int k = 0; k < P.K; ++k) {
          const float* bb = beta + (int64_t)k * (p + 1);
          double e = 0.0;
          for (int c = q; c < p; c += 4) e += (double)A[c * LDR + r] * bb[c];
          part[q][r] = e;
          __syncthreads();
          if (q == 0) {
            const double etak = part[0][r] + part[1][r] + part[2][r] + part[3][r] + bb[p];
            // online softmax over classes
            if (etak > mx) { den = den * exp(mx - etak) + 1.0; ek = (k == P.cls) ? 1.0 : ek * exp(mx - etak); mx = etak; }
            else { den += exp(etak - mx); if (k == P.cls) ek = exp(etak - mx); }
            if (k == P.cls) sz[r] = (float)etak;
          }
          __syncthreads();
        }
        if (q == 0) {
          const int64_t row = r0 + r;
          float wv = 0.0f, zv = 0.0f;
          if (row < r_end) {
            const double pk = fmin(fmax(ek / den, 1e-10), 1.0 - 1e-10);
            const double yk = ((int)y[row] == P.cls) ? 1.0 : 0.0;
            const double wpv = wprior ? wprior[row] : 1.0;
            const double wi = pk * (1.0 - pk);
            zv = (float)(sz[r] + (yk - pk) / wi);
            wv = (float)sqrt(fmax(wpv * wi, 0.0));
            dev_acc += wpv * (yk > 0 ? -2.0 * log(pk) : 0.0);
          }
          sw[r] = wv;
          sz[r] = zv;
        }
      } else {
        double e = 0.0;
        for (int c = q; c < p; c += 4) e += (double)A[c * LDR + r] * bk[c];
        part[q][r] = e;
        __syncthreads();
        if (q == 0) {
          const int64_t row = r0 + r;
          float wv = 0.0f, zv = 0.0f;
          if (row < r_end) {
            const double off = offset ? offset[row] : 0.0;
            const double eta = part[0][r] + part[1][r] + part[2][r] + part[3][r] + bk[p] + off;
            double mu, dmu;
            glm_link(P, eta, mu, dmu);
            const double yv = y[row];
            const double wpv = wprior ? wprior[row] : 1.0;
            const double wi = wpv * dmu * dmu / glm_var(P, mu);
            zv = (float)(eta - off + (yv - mu) / dmu);
            wv = (float)sqrt(fmax(wi, 0.0));
            dev_acc += wpv * glm_dev(P, yv, mu);
          }
          sw[r] = wv;
          sz[r] = zv;
        }
      }
    }
    __syncthreads();
    // 3. scale by sqrt(w), append the intercept and working-response columns
    for (int j = t; j < (p + 2) * GLM_RB; j += 256) {
      const int c = j >> 6, r = j & 63;
      const float s = sw[r];
      if (c < p) A[c * LDR + r] *= s;
      else if (c == p) A[c * LDR + r] = s;
      else A[c * LDR + r] = sz[r] * s;
    }
    __syncthreads();
    // 4. Gram tiles on the matrix cores: G[i][j] += sum_r a_i(r) a_j(r)
    const int li = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      if (wid + 4 * u < T) {
        const float* ca = A + (ti_[u] * 32 + li) * LDR + lh;
        const float* cb = A + (tj_[u] * 32 + li) * LDR + lh;
#pragma unroll 8
        for (int s = 0; s < GLM_RB / 2; ++s) acc[u] = mfma32(ca[2 * s], cb[2 * s], acc[u]);
      }
    }
    __syncthreads();
  }
  // write this workgroup's upper tiles
  float* out = slab + (int64_t)blockIdx.x * PP * PP;
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    if (wid + 4 * u < T) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int i = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int j = lane & 31;
        out[(ti_[u] * 32 + i) * PP + tj_[u] * 32 + j] = acc[u][e];
      }
    }
  }
  // deviance of this workgroup (only q==0 threads accumulated)
  double d = wave_sum(dev_acc);
  if (lane == 0) devred[wid] = d;
  __syncthreads();
  if (t == 0) dev_out[blockIdx.x] = devred[0] + devred[1] + devred[2] + devred[3];
}

// fp64 reduction of the per-workgroup slabs (upper tiles only are written;
// lower-tile entries of the slab are never read)
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, int n_slabs, int width,
                                                          double* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= width) return;
  const int PP = (int)sqrtf((float)width);
  const int i = j / PP, k = j % PP;
  if ((i >> 5) > (k >> 5)) {  // strictly-lower tile: mirror later
    out[j] = 0.0;
    return;
  }
  double acc = 0.0;
  for (int s = 0; s < n_slabs; ++s) acc += slab[(int64_t)s * width + j];
  out[j] = acc;
}

// ===========================================================================
// K-Means: assign + per-workgroup cluster sums
// ===========================================================================
constexpr int KM_RB = 64;

// X [d][ld] (already standardized by the caller), C [k][d], cn[k] = ||c||^2.
// Outputs: assign[n], per-workgroup slab of [k][d] sums + k counts + k SSE.
template <int DP, int KP>
__global__ __launch_bounds__(256) void kmeans_kernel(const float* __restrict__ X, int64_t ld, int64_t n, int d,
                                                     const float* __restrict__ C, const float* __restrict__ cn, int k,
                                                     int64_t rows_per_wg, int* __restrict__ assign,
                                                     float* __restrict__ slab) {
  constexpr int LDR = KM_RB + 1;
  __shared__ float Xs[DP * LDR];    // staged chunk [feature][row]
  __shared__ float Cs[KP * (DP + 1)];  // centroids [cluster][feature]
  __shared__ float S[KP * DP];      // cluster sums
  __shared__ float cnt[KP], sse[KP], cns[KP];
  __shared__ int asg[KM_RB];
  __shared__ float bestd[KM_RB];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int j = t; j < KP * (DP + 1); j += 256) {
    const int c = j / (DP + 1), f = j % (DP + 1);
    Cs[j] = (c < k && f < d) ? C[(int64_t)c * d + f] : 0.0f;
  }
  for (int j = t; j < KP * DP; j += 256) S[j] = 0.0f;
  for (int j = t; j < KP; j += 256) {
    cnt[j] = 0.0f; sse[j] = 0.0f;
    cns[j] = (j < k) ? cn[j] : INFINITY;
  }
  for (int j = t; j < DP * LDR; j += 256) Xs[j] = 0.0f;
  __syncthreads();
  const int64_t r_begin = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r_end = min(n, r_begin + rows_per_wg);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += KM_RB) {
    for (int j = t; j < d * KM_RB; j += 256) {
      const int f = j >> 6, r = j & 63;
      float v = 0.0f;
      if (r0 + r < r_end) {
        v = X[(int64_t)f * ld + r0 + r];
        if (v != v) v = 0.0f;  // NA -> mean (0 in standardized space)
      }
      Xs[f * LDR + r] = v;
    }
    __syncthreads();
    // waves 0,1 each own 32 rows; D[c][row] = sum_f C[c][f] X[f][row]
    if (wid < 2) {
      const int li = lane & 31, lh = lane >> 5;
      const int rloc = wid * 32 + li;
      float best = INFINITY;
      int bi = 0;
      for (int ct = 0; ct < KP / 32; ++ct) {
        f32x16 acc;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
        const float* ca = Cs + (ct * 32 + li) * (DP + 1) + lh;
        const float* xb = Xs + lh * LDR + wid * 32 + li;
        for (int s = 0; s < DP / 2; ++s) acc = mfma32(ca[2 * s], xb[2 * s * LDR], acc);
        // lane holds clusters c = ct*32 + (e&3) + 8(e>>2) + 4*lh for row rloc
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int c = ct * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          const float dist = cns[c] - 2.0f * acc[e];
          if (dist < best || (dist == best && c < bi)) { best = dist; bi = c; }
        }
      }
      // combine the two half-waves holding the same row
      const float ob = __shfl_xor(best, 32, kWave);
      const int oi = __shfl_xor(bi, 32, kWave);
      if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      if (lh == 0) { asg[rloc] = bi; bestd[rloc] = best; }
    }
    __syncthreads();
    // cluster sums: thread f owns feature column f of S (no atomics)
    for (int f = t; f < d; f += 256) {
      for (int r = 0; r < KM_RB; ++r) {
        if (r0 + r >= r_end) break;
        S[asg[r] * DP + f] += Xs[f * LDR + r];
      }
    }
    if (t < KM_RB && r0 + t < r_end) {
      float x2 = 0.0f;
      for (int f = 0; f < d; ++f) x2 += Xs[f * LDR + t] * Xs[f * LDR + t];
      assign[r0 + t] = asg[t];
      // counts / SSE through LDS atomics (64 per chunk, negligible)
      atomicAdd(&cnt[asg[t]], 1.0f);
      atomicAdd(&sse[asg[t]], fmaxf(bestd[t] + x2, 0.0f));
    }
    __syncthreads();
  }
  // slab layout: [k][d] sums | k counts | k sse
  float* out = slab + (int64_t)blockIdx.x * (k * d + 2 * k);
  for (int j = t; j < k * d; j += 256) out[j] = S[(j / d) * DP + (j % d)];
  for (int j = t; j < k; j += 256) {
    out[k * d + j] = cnt[j];
    out[k * d + k + j] = sse[j];
  }
}

__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slab, int n_slabs, int width,
                                                       double* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= width) return;
  double acc = 0.0;
  for (int s = 0; s < n_slabs; ++s) acc += slab[(int64_t)s * width + j];
  out[j] = acc;
}

// ===========================================================================
// MLP: tiled fp32-MFMA GEMM with fused bias + activation
// C[M][N] = act(op(A)[M][K] op(B)[K][N] + bias[N]);  row-major storage.
//   TA: A stored [K][M] (use A^T), TB: B stored [N][K] (use B^T).
// 256 threads, 128x128 block tile, each wave a 64x64 quadrant = 2x2 MFMA
// tiles of 32x32, K staged 16 at a time through LDS as [k][m] / [k][n].
// ===========================================================================
constexpr int GB = 128, GK = 32, GPAD = 4;

// One K-step of a 128 x 32 operand tile: global -> registers (float4 along
// the contiguous dimension when the leading dimension allows it).
// "MK" layout: element (m, k) at P[m * ld + k] (contiguous along k);
// "KM" layout: element (m, k) at P[k * ld + m] (contiguous along m).
constexpr int GTHREADS = 512;   // 8 waves per 128 x 128 tile
constexpr int GLD = GB * GK / 4 / GTHREADS;  // float4 per thread per operand tile

struct TileRegs {
  float v[4 * GLD];
};

template <bool KM>
__device__ __forceinline__ void load_tile(const float* __restrict__ P, int ld, int rows, int k_lim, int r0, int k0,
                                          bool vec, TileRegs& t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < GLD; ++q) {
    const int f = tid + GTHREADS * q;  // float4 index in the 128 x 32 tile
    int r, k;
    if (KM) { k = f >> 5; r = (f & 31) * 4; }   // 32 float4 per k-row of 128
    else { r = f >> 3; k = (f & 7) * 4; }       // 8 float4 per m-row of 32
    const int gr = r0 + r, gk = k0 + k;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f;
    if (KM) {
      if (gk < k_lim) {
        const float* src = P + (int64_t)gk * ld + gr;
        if (vec && gr + 3 < rows) {
          const float4 v4 = *reinterpret_cast<const float4*>(src);
          x0 = v4.x; x1 = v4.y; x2 = v4.z; x3 = v4.w;
        } else {
          if (gr < rows) x0 = src[0];
          if (gr + 1 < rows) x1 = src[1];
          if (gr + 2 < rows) x2 = src[2];
          if (gr + 3 < rows) x3 = src[3];
        }
      }
    } else {
      if (gr < rows) {
        const float* src = P + (int64_t)gr * ld + gk;
        if (vec && gk + 3 < k_lim) {
          const float4 v4 = *reinterpret_cast<const float4*>(src);
          x0 = v4.x; x1 = v4.y; x2 = v4.z; x3 = v4.w;
        } else {
          if (gk < k_lim) x0 = src[0];
          if (gk + 1 < k_lim) x1 = src[1];
          if (gk + 2 < k_lim) x2 = src[2];
          if (gk + 3 < k_lim) x3 = src[3];
        }
      }
    }
    t.v[4 * q] = x0; t.v[4 * q + 1] = x1; t.v[4 * q + 2] = x2; t.v[4 * q + 3] = x3;
  }
}

// registers -> LDS tile S[k][r] (r contiguous: MFMA operand reads are conflict free)
template <bool KM>
__device__ __forceinline__ void store_tile(float (*S)[GB + GPAD], const TileRegs& t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < GLD; ++q) {
    const int f = tid + GTHREADS * q;
    if (KM) {
      const int k = f >> 5, r = (f & 31) * 4;
      *reinterpret_cast<float4*>(&S[k][r]) = make_float4(t.v[4 * q], t.v[4 * q + 1], t.v[4 * q + 2], t.v[4 * q + 3]);
    } else {
      const int r = f >> 3, k = (f & 7) * 4;
      S[k][r] = t.v[4 * q];
      S[k + 1][r] = t.v[4 * q + 1];
      S[k + 2][r] = t.v[4 * q + 2];
      S[k + 3][r] = t.v[4 * q + 3];
    }
  }
}

// MLP GEMM on the fp32 matrix cores:
//   C[M][N] = act(op(A)[M][K] op(B)[K][N] + bias[N] (+ beta_c C)), row-major.
//   TA: A stored [K][M]; TB: B stored [N][K].
// 512 threads, 128 x 128 block tile, 8 waves of 32 x 64 (2 MFMA 32x32x2
// accumulators each; 8 waves per CU even when the grid has only one tile
// per CU).  K advances 32 per step through double-
// buffered LDS; the next step's global loads are issued into registers
// before the current step's 64 MFMAs per wave, so HBM latency hides behind
// matrix-core work.  blockIdx.z splits K (split-K partials, see
// gemm_splitk_reduce_kernel).
template <bool TA, bool TB>
__global__ __launch_bounds__(512, 1) void gemm_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                      float* __restrict__ Cm, const float* __restrict__ bias, int M,
                                                      int N, int K, int act, float beta_c) {
  __shared__ __attribute__((aligned(16))) float As[2][GK][GB + GPAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][GK][GB + GPAD];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int m0 = blockIdx.y * GB, n0 = blockIdx.x * GB;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 64;
  const int S = gridDim.z;
  const int kchunk = ((K + S - 1) / S + GK - 1) / GK * GK;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  if (S > 1) Cm += (int64_t)blockIdx.z * M * N;
  // A as (m, k): TA -> KM layout (ld = M), else MK (ld = K); B as (n, k): TB -> MK (ld = K), else KM (ld = N)
  const bool va = (TA ? (M % 4 == 0) : (K % 4 == 0)) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool vb = (TB ? (K % 4 == 0) : (N % 4 == 0)) && ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
  f32x16 acc[2];
#pragma unroll
  for (int y = 0; y < 2; ++y)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[y][e] = 0.0f;
  const int li = lane & 31, lh = lane >> 5;
  TileRegs ra, rb;
  int buf = 0;
  if (kb < ke) {
    load_tile<TA>(A, TA ? M : K, M, ke, m0, kb, va, ra);
    load_tile<!TB>(B, TB ? K : N, N, ke, n0, kb, vb, rb);
    store_tile<TA>(As[0], ra);
    store_tile<!TB>(Bs[0], rb);
  }
  __syncthreads();
  for (int k0 = kb; k0 < ke; k0 += GK) {
    const bool more = k0 + GK < ke;
    if (more) {
      load_tile<TA>(A, TA ? M : K, M, ke, m0, k0 + GK, va, ra);
      load_tile<!TB>(B, TB ? K : N, N, ke, n0, k0 + GK, vb, rb);
    }
#pragma unroll
    for (int s2 = 0; s2 < GK / 2; ++s2) {
      const int kk = 2 * s2 + lh;
      const float a0 = As[buf][kk][wm + li];
      const float b0 = Bs[buf][kk][wn + li], b1 = Bs[buf][kk][wn + 32 + li];
      acc[0] = mfma32(a0, b0, acc[0]);
      acc[1] = mfma32(a0, b1, acc[1]);
    }
    if (more) {
      store_tile<TA>(As[buf ^ 1], ra);
      store_tile<!TB>(Bs[buf ^ 1], rb);
    }
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int i = m0 + wm + (e & 3) + 8 * (e >> 2) + 4 * lh;
        const int j = n0 + wn + 32 * y + li;
        if (i < M && j < N) {
          float v = acc[y][e];
          if (S > 1) {
            Cm[(int64_t)i * N + j] = v;
            continue;
          }
          if (beta_c != 0.0f) v += beta_c * Cm[(int64_t)i * N + j];
          if (bias) v += bias[j];
          if (act == 1) v = fmaxf(v, 0.0f);
          else if (act == 2) v = tanhf(v);
          Cm[(int64_t)i * N + j] = v;
        }
      }
}

// C = act(sum_z W[z] + beta_c * C + bias): split-K epilogue (fixed order: deterministic)
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const float* __restrict__ W, int S, int M, int N,
                                                                 float* __restrict__ C, const float* __restrict__ bias,
                                                                 int act, float beta_c) {
  const int64_t MN = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < MN; i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.0f;
    for (int z = 0; z < S; ++z) v += W[z * MN + i];
    if (beta_c != 0.0f) v += beta_c * C[i];
    if (bias) v += bias[i % N];
    if (act == 1) v = fmaxf(v, 0.0f);
    else if (act == 2) v = tanhf(v);
    C[i] = v;
  }
}

// column sums of dY [M][N] (bias gradients), stage 1: block (64 columns x
// 4 row phases) sums one row slice, folds the phases in LDS -> ws[slice][col]
__global__ __launch_bounds__(256) void bias_grad_split_kernel(const float* __restrict__ dY, float* __restrict__ ws,
                                                              int M, int N) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  const int S = gridDim.y;
  const int rows = (M + S - 1) / S;
  const int r0 = blockIdx.y * rows, r1 = min(M, r0 + rows);
  float s0 = 0.f, s1 = 0.f;
  if (j < N) {
    int i = r0 + ph;
    for (; i + 4 < r1; i += 8) {
      s0 += dY[(int64_t)i * N + j];
      s1 += dY[(int64_t)(i + 4) * N + j];
    }
    for (; i < r1; i += 4) s0 += dY[(int64_t)i * N + j];
  }
  red[ph][c] = s0 + s1;
  __syncthreads();
  if (ph == 0 && j < N) ws[(int64_t)blockIdx.y * N + j] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// dZ = dY * act'(Y)  (act: 0 none, 1 relu, 2 tanh), in place allowed
__global__ __launch_bounds__(256) void act_backward_kernel(const float* __restrict__ Y, float* __restrict__ dY,
                                                           int64_t n, int act) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float g = dY[i];
  if (act == 1) g = Y[i] > 0.0f ? g : 0.0f;
  else if (act == 2) g = g * (1.0f - Y[i] * Y[i]);
  dY[i] = g;
}

// db[j] = sum_i dY[i][j]
__global__ __launch_bounds__(256) void bias_grad_kernel(const float* __restrict__ dY, float* __restrict__ db, int M,
                                                        int N) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  float s = 0.0f;
  for (int i = 0; i < M; ++i) s += dY[(int64_t)i * N + j];
  db[j] = s;
}

// softmax cross-entropy over logits Z [M][K]: writes dZ = (softmax - onehot) * w / norm
// and accumulates the loss into loss[0].
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ Z, const int* __restrict__ y,
                                                           float* __restrict__ dZ, float* __restrict__ loss, int M,
                                                           int K) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float l = 0.0f;
  if (i < M) {
    const float* z = Z + (int64_t)i * K;
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, z[k]);
    float den = 0.0f;
    for (int k = 0; k < K; ++k) den += __expf(z[k] - mx);
    const int yi = y[i];
    for (int k = 0; k < K; ++k) {
      const float pk = __expf(z[k] - mx) / den;
      dZ[(int64_t)i * K + k] = (pk - (k == yi ? 1.0f : 0.0f)) / (float)M;
      if (k == yi) l = -logf(fmaxf(pk, 1e-30f));
    }
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) atomicAdd(loss, l / (float)M);
}

// ADADELTA (H2O DeepLearning default: rho 0.99, epsilon 1e-8) with L1/L2
__global__ __launch_bounds__(256) void adadelta_kernel(float* __restrict__ W, const float* __restrict__ G,
                                                       float* __restrict__ Eg2, float* __restrict__ Edx2, int64_t n,
                                                       float rho, float eps, float l2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = G[i] + l2 * W[i];
  const float eg = rho * Eg2[i] + (1.0f - rho) * g * g;
  const float dx = -sqrtf(Edx2[i] + eps) / sqrtf(eg + eps) * g;
  Eg2[i] = eg;
  Edx2[i] = rho * Edx2[i] + (1.0f - rho) * dx * dx;
  W[i] += dx;
}

__global__ __launch_bounds__(256) void sgd_momentum_kernel(float* __restrict__ W, const float* __restrict__ G,
                                                           float* __restrict__ V, int64_t n, float lr, float mom,
                                                           float l2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = mom * V[i] - lr * (G[i] + l2 * W[i]);
  V[i] = v;
  W[i] += v;
}

// ===========================================================================
// C ABI
// ===========================================================================
static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

H2OMX_API int h2omx_dense_sizes(int* out) {
  out[0] = sizeof(GlmParams);
  return kOk;
}

H2OMX_API int h2omx_glm_irls(const float* X, int64_t ld, int64_t n, const float* y, const float* wprior,
                             const float* offset, const float* means, const float* beta, const void* params,
                             int n_wg, int tp, float* slab, double* dev_out, hipStream_t stream) {
  const GlmParams P = *reinterpret_cast<const GlmParams*>(params);
  if (P.p + 2 > 32 * tp || n_wg < 1) return kBadArg;
  const int64_t rows_per_wg = ((n + n_wg - 1) / n_wg + GLM_RB - 1) / GLM_RB * GLM_RB;
#define GLM_L(TP)                                                                                      \
  hipLaunchKernelGGL(glm_irls_kernel<TP>, dim3(n_wg), dim3(256), 0, stream, X, ld, n, y, wprior, offset, \
                     means, beta, P, rows_per_wg, slab, dev_out)
  switch (tp) {
    case 1: GLM_L(1); break;
    case 2: GLM_L(2); break;
    case 4: GLM_L(4); break;
    case 8: GLM_L(8); break;
    default: return kBadArg;
  }
#undef GLM_L
  return launch_status();
}

H2OMX_API int h2omx_slab_reduce_upper(const float* slab, int n_slabs, int width, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(cdiv(width, 256)), dim3(256), 0, stream, slab, n_slabs, width, out);
  return launch_status();
}

H2OMX_API int h2omx_slab_sum(const float* slab, int n_slabs, int width, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(slab_sum_kernel, dim3(cdiv(width, 256)), dim3(256), 0, stream, slab, n_slabs, width, out);
  return launch_status();
}

H2OMX_API int h2omx_kmeans(const float* X, int64_t ld, int64_t n, int d, const float* C, const float* cn, int k,
                           int n_wg, int* assign, float* slab, hipStream_t stream) {
  if (n_wg < 1) return kBadArg;
  const int64_t rows_per_wg = ((n + n_wg - 1) / n_wg + KM_RB - 1) / KM_RB * KM_RB;
#define KM_L(DP, KP)                                                                                         \
  hipLaunchKernelGGL((kmeans_kernel<DP, KP>), dim3(n_wg), dim3(256), 0, stream, X, ld, n, d, C, cn, k, rows_per_wg, \
                     assign, slab)
  const int dp = d <= 32 ? 32 : (d <= 64 ? 64 : (d <= 128 ? 128 : (d <= 256 ? 256 : 0)));
  const int kp = k <= 32 ? 32 : (k <= 64 ? 64 : (k <= 128 ? 128 : 0));
  if (!dp || !kp || (size_t)dp * 65 * 4 + (size_t)kp * (dp + 1) * 4 + (size_t)kp * dp * 4 > 150 * 1024)
    return kBadArg;
  if (dp == 32 && kp == 32) KM_L(32, 32);
  else if (dp == 32 && kp == 64) KM_L(32, 64);
  else if (dp == 32 && kp == 128) KM_L(32, 128);
  else if (dp == 64 && kp == 32) KM_L(64, 32);
  else if (dp == 64 && kp == 64) KM_L(64, 64);
  else if (dp == 64 && kp == 128) KM_L(64, 128);
  else if (dp == 128 && kp == 32) KM_L(128, 32);
  else if (dp == 128 && kp == 64) KM_L(128, 64);
  else if (dp == 256 && kp == 32) KM_L(256, 32);
  else return kBadArg;
#undef KM_L
  return launch_status();
}

H2OMX_API int h2omx_gemm(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int ta,
                         int tb, int act, float beta_c, int splitk, float* ws, hipStream_t stream) {
  if (splitk < 1 || (splitk > 1 && !ws)) return kBadArg;
  const dim3 grid(cdiv(N, GB), cdiv(M, GB), splitk);
  float* out = splitk > 1 ? ws : C;
  const dim3 blk(GTHREADS);
  if (!ta && !tb) hipLaunchKernelGGL((gemm_kernel<false, false>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
  else if (!ta && tb) hipLaunchKernelGGL((gemm_kernel<false, true>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
  else if (ta && !tb) hipLaunchKernelGGL((gemm_kernel<true, false>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
  else hipLaunchKernelGGL((gemm_kernel<true, true>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
  if (splitk > 1)
    hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(cdiv((int64_t)M * N, 256) < 4096 ? cdiv((int64_t)M * N, 256) : 4096),
                       dim3(256), 0, stream, ws, splitk, M, N, C, bias, act, beta_c);
  return launch_status();
}

H2OMX_API int h2omx_act_backward(const float* Y, float* dY, int64_t n, int act, hipStream_t stream) {
  hipLaunchKernelGGL(act_backward_kernel, dim3(cdiv(n, 256)), dim3(256), 0, stream, Y, dY, n, act);
  return launch_status();
}

H2OMX_API int h2omx_bias_grad(const float* dY, float* db, int M, int N, float* ws, int splits, hipStream_t stream) {
  if (splits < 1 || !ws) return kBadArg;
  hipLaunchKernelGGL(bias_grad_split_kernel, dim3(cdiv(N, 64), splits), dim3(256), 0, stream, dY, ws, M, N);
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(cdiv(N, 256)), dim3(256), 0, stream, ws, splits, 1, N, db,
                     nullptr, 0, 0.0f);
  return launch_status();
}

H2OMX_API int h2omx_softmax_xent(const float* Z, const int* y, float* dZ, float* loss, int M, int K,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(cdiv(M, 256)), dim3(256), 0, stream, Z, y, dZ, loss, M, K);
  return launch_status();
}

H2OMX_API int h2omx_adadelta(float* W, const float* G, float* Eg2, float* Edx2, int64_t n, float rho, float eps,
                             float l2, hipStream_t stream) {
  hipLaunchKernelGGL(adadelta_kernel, dim3(cdiv(n, 256)), dim3(256), 0, stream, W, G, Eg2, Edx2, n, rho, eps, l2);
  return launch_status();
}

H2OMX_API int h2omx_sgd_momentum(float* W, const float* G, float* V, int64_t n, float lr, float mom, float l2,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3(cdiv(n, 256)), dim3(256), 0, stream, W, G, V, n, lr, mom, l2);
  return launch_status();
}
