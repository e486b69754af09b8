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
               // (also fractionalbinomial) 7 negativebinomial
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
    case 7: return fmax(mu + P.var_power * mu * mu, 1e-10);   // negative binomial, var_power = theta
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
    case 7: {  // negative binomial (theta = var_power)
      const double th = P.var_power, m = fmax(mu, 1e-15);
      const double a = (y > 0) ? y * log(y / m) : 0.0;
      return 2.0 * (a - (y + 1.0 / th) * log((1.0 + th * y) / (1.0 + th * m)));
    }
    default: return (y - mu) * (y - mu);
  }
}

// ---------------------------------------------------------------------------
// GLM with more predictors than the fused Gram kernel's 254-column tile
// (one-hot categoricals with hundreds of levels): per row chunk the linear
// predictors come from the MFMA GEMM E = B [K][p] x Xc [p][m] (gemm_kernel),
// glm_wz_kernel turns them into IRLS weights / working responses (same
// per-row math as glm_irls_kernel), glm_aug_kernel writes the scaled augmented
// design sqrt(w) [x | 1 | z] [(p+2)][m], and the Gram is the GEMM A x A^T
// (fp32 per chunk, summed in fp64 by slab_sum_kernel).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void glm_wz_kernel(const float* __restrict__ E, int64_t m,
                                                     const float* __restrict__ y, const float* __restrict__ wprior,
                                                     const float* __restrict__ offset,
                                                     const float* __restrict__ beta, GlmParams P,
                                                     float* __restrict__ sw, float* __restrict__ z,
                                                     double* __restrict__ dev_part) {
  __shared__ double red[256];
  const int p = P.p;
  double dacc = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256) {
    const double wpv = wprior ? wprior[r] : 1.0;
    double wi, zv;
    if (P.family == 5) {
      double mx = -1e300;
      for (int k = 0; k < P.K; ++k) mx = fmax(mx, (double)E[(int64_t)k * m + r] + beta[(int64_t)k * (p + 1) + p]);
      double den = 0.0, ek = 0.0, etak = 0.0;
      for (int k = 0; k < P.K; ++k) {
        const double e = (double)E[(int64_t)k * m + r] + beta[(int64_t)k * (p + 1) + p];
        const double x = exp(e - mx);
        den += x;
        if (k == P.cls) { ek = x; etak = e; }
      }
      const double pk = fmin(fmax(ek / den, 1e-10), 1.0 - 1e-10);
      const double yk = ((int)y[r] == P.cls) ? 1.0 : 0.0;
      const double w0 = pk * (1.0 - pk);
      zv = etak + (yk - pk) / w0;
      wi = wpv * w0;
      dacc += wpv * (yk > 0 ? -2.0 * log(pk) : 0.0);
    } else {
      const double off = offset ? offset[r] : 0.0;
      const double eta = (double)E[(int64_t)P.cls * m + r] + beta[(int64_t)P.cls * (p + 1) + p] + off;
      double mu, dmu;
      glm_link(P, eta, mu, dmu);
      const double yv = y[r];
      wi = wpv * dmu * dmu / glm_var(P, mu);
      zv = eta - off + (yv - mu) / dmu;
      dacc += wpv * glm_dev(P, yv, mu);
    }
    sw[r] = (float)sqrt(fmax(wi, 0.0));
    z[r] = (float)zv;
  }
  red[threadIdx.x] = dacc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dev_part[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------
// GLM gradient pass (solver L_BFGS): two streaming kernels over the
// feature-major design, no Gram.  glm_resid_kernel: one thread per row, the
// K linear predictors eta = B x + b0 (+ offset) from coalesced feature rows,
// then the row's gradient weight r_k = w (mu - y) mu'(eta) / V(mu)
// (multinomial: w (p_k - [y == k])) and its deviance.  glm_xtr_kernel:
// grad[k][j] = sum_i x_ji r_ki, one workgroup per (feature, row split) doing
// contiguous dot products (the intercept row j = p sums r).  fp64 throughout
// the accumulation; per-split partials are summed on the host in fixed order.
// ---------------------------------------------------------------------------
constexpr int kGradMaxK = 16;

__global__ __launch_bounds__(256) void glm_resid_kernel(const float* __restrict__ X, int64_t ld, int64_t n,
                                                        const double* __restrict__ beta, const float* __restrict__ y,
                                                        const float* __restrict__ wprior,
                                                        const float* __restrict__ offset, GlmParams P,
                                                        float* __restrict__ R, double* __restrict__ dev_part) {
  extern __shared__ double sb[];   // beta [K][p + 1]
  __shared__ double red[256];
  const int p = P.p, K = P.K;
  for (int i = threadIdx.x; i < K * (p + 1); i += 256) sb[i] = beta[i];
  __syncthreads();
  double dacc = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    double eta[kGradMaxK];
#pragma unroll
    for (int k = 0; k < kGradMaxK; ++k) eta[k] = (k < K) ? sb[k * (p + 1) + p] : 0.0;
    for (int j = 0; j < p; ++j) {
      const double x = X[(int64_t)j * ld + r];
#pragma unroll
      for (int k = 0; k < kGradMaxK; ++k)
        if (k < K) eta[k] += sb[k * (p + 1) + j] * x;
    }
    const double wpv = wprior ? wprior[r] : 1.0;
    if (P.family == 5) {
      double mx = -1e300;
#pragma unroll
      for (int k = 0; k < kGradMaxK; ++k)
        if (k < K) mx = fmax(mx, eta[k]);
      double den = 0.0;
#pragma unroll
      for (int k = 0; k < kGradMaxK; ++k)
        if (k < K) den += exp(eta[k] - mx);
      const int yc = (int)y[r];
#pragma unroll
      for (int k = 0; k < kGradMaxK; ++k) {
        if (k < K) {
          const double pk = exp(eta[k] - mx) / den;
          R[(int64_t)k * n + r] = (float)(wpv * (pk - (k == yc ? 1.0 : 0.0)));
          if (k == yc) dacc += wpv * -2.0 * log(fmax(pk, 1e-300));
        }
      }
    } else {
      const double e = eta[0] + (offset ? offset[r] : 0.0);
      double mu, dmu;
      glm_link(P, e, mu, dmu);
      const double yv = y[r];
      R[r] = (float)(wpv * (mu - yv) * dmu / glm_var(P, mu));
      dacc += wpv * glm_dev(P, yv, mu);
    }
  }
  red[threadIdx.x] = dacc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dev_part[blockIdx.x] = red[0];
}

// grid (p + 1, splits): out[split][k][j] = sum over the split's rows of x_ji r_ki
__global__ __launch_bounds__(256) void glm_xtr_kernel(const float* __restrict__ X, int64_t ld, int64_t n, int p,
                                                      int K, const float* __restrict__ R, double* __restrict__ out) {
  __shared__ double red[kGradMaxK][4];
  const int j = blockIdx.x, sp = blockIdx.y, ns = gridDim.y;
  const int64_t per = (n + ns - 1) / ns;
  const int64_t r0 = (int64_t)sp * per, r1 = min(n, r0 + per);
  double acc[kGradMaxK];
#pragma unroll
  for (int k = 0; k < kGradMaxK; ++k) acc[k] = 0.0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    const double x = (j < p) ? (double)X[(int64_t)j * ld + r] : 1.0;
#pragma unroll
    for (int k = 0; k < kGradMaxK; ++k)
      if (k < K) acc[k] += x * (double)R[(int64_t)k * n + r];
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < kGradMaxK; ++k) {
    if (k < K) {
      const double v = wave_sum(acc[k]);
      if (lane == 0) red[k][wv] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < K)
    out[((int64_t)sp * K + threadIdx.x) * (p + 1) + j] =
        red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
}

// A [(p+2)][m] = sqrt(w) * [x (NaN -> column mean) | 1 | z]; Xc [p][m] is the
// staged chunk (NaN kept), grid.y = augmented row
__global__ __launch_bounds__(256) void glm_aug_kernel(const float* __restrict__ Xc, int p, int64_t m,
                                                      const float* __restrict__ means,
                                                      const float* __restrict__ sw, const float* __restrict__ z,
                                                      float* __restrict__ A) {
  const int c = blockIdx.y;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256) {
    float v;
    if (c < p) {
      v = Xc[(int64_t)c * m + r];
      if (v != v) v = means[c];
    } else {
      v = (c == p) ? 1.0f : z[r];
    }
    A[(int64_t)c * m + r] = sw[r] * v;
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

// ---------------------------------------------------------------------------
// GLM IRLS pass, wave-private row chunks (glm_irls_wave_kernel): the default
// for p + 2 <= 128 and every family but multinomial.
//
// glm_irls_kernel above runs each 64-row chunk as a workgroup-wide chain
// (stage -> barrier -> dot products -> barrier -> link math on ONE wave ->
// barrier -> scale -> barrier -> MFMA), ~7 ms per pass at 10M x 100 with the
// waves parked on barriers ~75 % of the time (profiles/r2/dense_pmc).  Here
// every wave is an independent unit over its own row range:
//   * the augmented design [x | 1 | z] of a 64-row chunk lives in REGISTERS:
//     lane l = (h = l / 16, c = l % 16) holds column blk * 16 + c of rows
//     h * 16 .. h * 16 + 15 for every 16-column block blk (64 contiguous bytes
//     per lane and block), which is exactly the operand layout of
//     v_mfma_f32_16x16x4f32 (A: i = l % 16, k = l / 16; step s = row h*16+s);
//   * the next chunk's columns / y / weights / offsets are loaded while the
//     current chunk is computed (register double buffer, one wait per chunk);
//   * linear predictors: per lane 16 partial dot products (its columns) in
//     fp64, reduce-scattered over the 16 lanes of the row group (15 shuffles)
//     so that every lane owns ONE row: the link / weight / deviance math runs
//     on all 64 lanes;
//   * sqrt(w) and z come back to the column lanes with 16 + 16 shuffles; the
//     scaled chunk feeds 16 MFMA steps per upper 16x16 Gram tile (16-column
//     granularity: 28 tiles at p = 100 instead of 10 32x32 tiles padded to 128);
//   * no LDS, no barriers.  Each unit accumulates at most a few thousand rows
//     in fp32 before the fp64 slab reduction (slab_reduce16_kernel).
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GW_S = 8;            // rows per lane group and chunk = MFMA k-steps of 4 rows
constexpr int GW_RB = 4 * GW_S;    // rows per chunk

template <int NB, bool VEC>
__global__ __launch_bounds__(256) void glm_irls_wave_kernel(const float* __restrict__ X, int64_t ld, int64_t n,
                                                            const float* __restrict__ y,
                                                            const float* __restrict__ wprior,
                                                            const float* __restrict__ offset,
                                                            const float* __restrict__ means,
                                                            const float* __restrict__ beta, GlmParams P,
                                                            int64_t rows_per_unit, int n_units,
                                                            float* __restrict__ slab, double* __restrict__ dev_out) {
  constexpr int PW = NB * 16;                 // padded augmented width
  constexpr int T = NB * (NB + 1) / 2;        // upper 16x16 tiles
  // coefficients / imputation means in LDS: read per chunk through the LDS
  // counter, so they never wait behind the next chunk's in-flight global loads
  __shared__ double bsh[PW];
  __shared__ float msh[PW];
  const int p = P.p;
  for (int c = threadIdx.x; c < PW; c += blockDim.x) {
    bsh[c] = (c < p) ? (double)beta[c] : 0.0;
    msh[c] = (c < p) ? means[c] : 0.0f;
  }
  __syncthreads();   // the only barrier: before any wave can leave
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (unit >= n_units) return;
  const int h = lane >> 4, cl = lane & 15;
  const int64_t r_begin = (int64_t)unit * rows_per_unit;
  const int64_t r_end = min(n, r_begin + rows_per_unit);

  f32x4 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const double b0 = (double)beta[p];
  double dev_acc = 0.0;

  float xc[NB][GW_S], xn[NB][GW_S];
  float yc = 0.f, wc = 1.f, oc = 0.f, yn = 0.f, wn = 1.f, on = 0.f;
  auto load = [&](int64_t r0, float (&xb)[NB][GW_S], float& yv, float& wv, float& ov) {
    const int64_t rr = r0 + h * GW_S;         // first row of this lane's group
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int c = b * 16 + cl;
      if (c < p) {
        const float* src = X + (int64_t)c * ld + rr;
        if (VEC && rr + GW_S <= r_end) {
#pragma unroll
          for (int q = 0; q < GW_S / 4; ++q) {
            const float4 v = *reinterpret_cast<const float4*>(src + 4 * q);
            xb[b][4 * q] = v.x; xb[b][4 * q + 1] = v.y; xb[b][4 * q + 2] = v.z; xb[b][4 * q + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int s = 0; s < GW_S; ++s) xb[b][s] = (rr + s < r_end) ? src[s] : 0.0f;
        }
      } else {
#pragma unroll
        for (int s = 0; s < GW_S; ++s) xb[b][s] = 0.0f;
      }
    }
    const int64_t row = r0 + h * GW_S + (cl & (GW_S - 1));   // the row this lane owns in the link step
    if (row < r_end) {
      yv = y[row];
      wv = wprior ? wprior[row] : 1.0f;
      ov = offset ? offset[row] : 0.0f;
    } else {
      yv = 0.f; wv = 0.f; ov = 0.f;
    }
  };
  auto compute = [&](int64_t r0, float (&xb)[NB][GW_S], float yv, float wv, float ov) {
    // 1. mean-impute NaNs, partial linear predictors of the lane's rows
    double part[GW_S];
#pragma unroll
    for (int s = 0; s < GW_S; ++s) part[s] = 0.0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int c = b * 16 + cl;
      const double bc = bsh[c];
      const float mc = msh[c];
#pragma unroll
      for (int s = 0; s < GW_S; ++s) {
        float v = xb[b][s];
        if (v != v) v = mc;
        xb[b][s] = v;
        part[s] = fma((double)v, bc, part[s]);
      }
    }
    // 2. sum over the 16 column lanes of the group: a butterfly over lane bit 3,
    //    then a reduce-scatter over bits 2..0 -> lane c owns row c % 8
#pragma unroll
    for (int s = 0; s < GW_S; ++s) part[s] += __shfl_xor(part[s], 8, kWave);
#pragma unroll
    for (int off = GW_S / 2; off >= 1; off >>= 1) {
      const bool hi = (cl & off) != 0;
#pragma unroll
      for (int j = 0; j < off; ++j) {
        const double send = hi ? part[j] : part[j + off];
        const double recv = __shfl_xor(send, off, kWave);
        part[j] = (hi ? part[j + off] : part[j]) + recv;
      }
    }
    // 3. link / IRLS weight / working response / deviance of this lane's row
    const int64_t row = r0 + h * GW_S + (cl & (GW_S - 1));
    float sw = 0.f, zz = 0.f;
    if (row < r_end) {
      const double eta = part[0] + b0 + (double)ov;
      double mu, dmu;
      glm_link(P, eta, mu, dmu);
      const double wi = (double)wv * dmu * dmu / glm_var(P, mu);
      zz = (float)(eta - (double)ov + ((double)yv - mu) / dmu);
      sw = (float)sqrt(fmax(wi, 0.0));
      if (cl < GW_S) dev_acc += (double)wv * glm_dev(P, (double)yv, mu);   // lanes c and c + 8 share a row
    }
    // 4. scale the columns by sqrt(w) of their rows; intercept and z columns
    const int base = lane & 48;
#pragma unroll
    for (int s = 0; s < GW_S; ++s) {
      const float sws = __shfl(sw, base + s, kWave);
      const float zs = __shfl(zz, base + s, kWave);
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int c = b * 16 + cl;
        const float v = xb[b][s] * sws;
        xb[b][s] = (c == p) ? sws : ((c == p + 1) ? zs * sws : v);
      }
    }
    // 5. upper Gram tiles on the matrix cores (A: i = lane % 16, k = lane / 16)
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = bi; bj < NB; ++bj, ++t)
#pragma unroll
        for (int s = 0; s < GW_S; ++s)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[bi][s], xb[bj][s], acc[t], 0, 0, 0);
  };

  int64_t r0 = r_begin;
  if (r0 < r_end) load(r0, xc, yc, wc, oc);
  for (; r0 < r_end; r0 += GW_RB) {
    // the next chunk's loads are in flight while this one computes; one copy of
    // compute() (a two-chunk unroll doubles the inlined link math and spills)
    if (r0 + GW_RB < r_end) load(r0 + GW_RB, xn, yn, wn, on);
    compute(r0, xc, yc, wc, oc);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int s = 0; s < GW_S; ++s) xc[b][s] = xn[b][s];
    yc = yn; wc = wn; oc = on;
  }
  // this unit's upper tiles -> slab [unit][PW][PW] (16x16 tile layout: lane
  // holds D[4 * (l / 16) + v][l % 16]); strictly-lower tiles are never read
  float* out = slab + (int64_t)unit * PW * PW;
  int t = 0;
#pragma unroll
  for (int bi = 0; bi < NB; ++bi)
#pragma unroll
    for (int bj = bi; bj < NB; ++bj, ++t)
#pragma unroll
      for (int v = 0; v < 4; ++v) out[(bi * 16 + 4 * h + v) * PW + bj * 16 + cl] = acc[t][v];
  const double d = wave_sum(dev_acc);
  if (lane == 0) dev_out[unit] = d;
}

// ---------------------------------------------------------------------------
// GLM IRLS pass with the Gram on the bf16 matrix cores (glm_irls_split_kernel,
// the default for the wave path).
//
// glm_irls_wave_kernel above is bound by its fp32 MFMAs: 28 upper tiles x 8
// v_mfma_f32_16x16x4_f32 per 32-row chunk at 32 cycles each = 7.2k cycles,
// 1.1 ms of a 2.5 ms pass at 10M x 100 (SQ_VALU_MFMA_BUSY_CYCLES,
// profiles/r3/dense_pmc).  bf16 MFMA runs 16x the fp32 rate, and every fp32
// value splits EXACTLY into three bf16 pieces by truncation:
//   hi = x with the low 16 bits cleared (sign, exponent, 7 mantissa bits),
//   r = x - hi (exact: the low 16 mantissa bits, <= 16 significant bits),
//   mid = r with the low 16 bits cleared (the top 8 significant bits of r),
//   lo = r - mid (exact, <= 8 significant bits, so a bf16 exactly),
// x = hi + mid + lo with no rounding.  A product a * b then sums 9 partial
// products; the 6 with weight >= 2^-16 (hh, hm, mh, hl, lh, mm) are kept, the
// dropped ml + lm + ll are below ~2^-23 |a b|: fp32-product accuracy (each
// bf16 x bf16 product is exact in the fp32 accumulator).  6 x
// v_mfma_f32_16x16x32_bf16 (16 cycles) per tile and chunk = 96 cycles vs 256.
//
// The register layout is glm_irls_wave_kernel's (lane (h, c) holds column
// blk * 16 + c of rows h * 8 .. h * 8 + 7), which is exactly the A / B operand
// layout of the 16x16x32 bf16 MFMA (i = lane % 16, k = 8 (lane / 16) + 0..7),
// so a tile (bi, bj) is 6 MFMAs on the packed pieces of blocks bi and bj.
// Also cut from the VALU stream: the design has no NA (the GLM imputes
// before the pass, `means` is unused here), the intercept column is loaded
// as the constant 1 (then scaled like any column), the working response
// column is always in the last block (p + 1 >= 16 (NB - 1)), and the
// per-lane partial linear predictors run in fp32 (x and beta are fp32, each
// lane sums <= NB products; the 16-lane reduction stays fp64).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8_g __attribute__((ext_vector_type(8)));
typedef unsigned u32x4_g __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8_g as_bf16x8(u32x4_g v) { return __builtin_bit_cast(bf16x8_g, v); }

// exact three-way bf16 split of 8 fp32 values (see above), packed 2 per dword
__device__ __forceinline__ void split3_bf16(const float (&x)[GW_S], u32x4_g& H, u32x4_g& M, u32x4_g& L) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned u0 = __float_as_uint(x[2 * q]), u1 = __float_as_uint(x[2 * q + 1]);
    const float r0 = x[2 * q] - __uint_as_float(u0 & 0xffff0000u);
    const float r1 = x[2 * q + 1] - __uint_as_float(u1 & 0xffff0000u);
    const unsigned v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
    const float l0 = r0 - __uint_as_float(v0 & 0xffff0000u);
    const float l1 = r1 - __uint_as_float(v1 & 0xffff0000u);
    // high halves of (first, second) -> (low, high) half of the packed dword
    H[q] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
    M[q] = __builtin_amdgcn_perm(v1, v0, 0x07060302u);
    L[q] = __builtin_amdgcn_perm(__float_as_uint(l1), __float_as_uint(l0), 0x07060302u);
  }
}

// binomial / logit per-row IRLS quantities without branches: mu = sigmoid(eta)
// from e = exp(-|eta|), var(mu) = mu' (so w = prior * mu'), and the deviance
// from one log1p: log mu = min(eta, 0) - log1p(e), log(1 - mu) = -max(eta, 0)
// - log1p(e), each floored at log(1e-15) like glm_dev's clamp of mu.
__device__ __forceinline__ void glm_row_binomial(double eta, double ov, double yv, double wv, float& sw, float& zz,
                                                 double& dev) {
  const double e = exp(-fabs(eta));
  const double r1 = 1.0 / (1.0 + e);
  const double mu = eta >= 0 ? r1 : e * r1;
  const double dmu = fmax(mu * (1.0 - mu), 1e-10);
  zz = (float)(eta - ov + (yv - mu) / dmu);
  sw = (float)sqrt(wv * dmu);
  const double l1p = log1p(e);
  const double lfloor = -34.538776394910684;   // log(1e-15)
  const double lm = fmax(fmin(eta, 0.0) - l1p, lfloor), l1m = fmax(-fmax(eta, 0.0) - l1p, lfloor);
  dev = -2.0 * wv * (yv * lm + (1.0 - yv) * l1m);
}

// (an fp32 variant of the binomial row math measured no faster: profiles/r4/dense)

// FAM 1: binomial family with the logit link (branch-free row math, so the
// previous chunk's MFMAs and this chunk's link math share one basic block and
// the scheduler overlaps them); FAM 0: any family / link (glm_link / glm_var /
// glm_dev switches).  Software pipeline: iteration i issues chunk i + 1's
// loads, the MFMAs of chunk i - 1's bf16 pieces, and chunk i's linear
// predictors, link math, scaling and split (one wave per SIMD: 4 chunks' worth
// of registers - accumulators, pieces, current and next chunk).
// G: full chunks staged global -> LDS by LDS-DMA (global_load_lds_dwordx4), two
// chunks in flight per wave in two LDS slots, read back lane-linear (each
// lane its own 16-byte pieces) - no prefetch registers, no register copies.
// !G: one chunk ahead in registers (unaligned designs).
template <int NB, bool VEC, int FAM, bool G>
__global__ __launch_bounds__(256) void glm_irls_split_kernel(const float* __restrict__ X, int64_t ld, int64_t n,
                                                             const float* __restrict__ y,
                                                             const float* __restrict__ wprior,
                                                             const float* __restrict__ offset,
                                                             const float* __restrict__ beta, GlmParams P,
                                                             int64_t rows_per_unit, int n_units,
                                                             float* __restrict__ slab, double* __restrict__ dev_out) {
  constexpr int PW = NB * 16;
  constexpr int T = NB * (NB + 1) / 2;
  // ONE shared array (per-slot staging of every wave, then the coefficients):
  // the compiler's LDS-DMA wait tracking then needs no extra vmcnt(0)
  constexpr int SLOTF = NB * 512 + 192;      // floats: NB x 2 x 64 lanes x 16 B, then y / w / offset
  constexpr int GLDS = G ? 4 * 2 * SLOTF : 0;
  __shared__ __attribute__((aligned(16))) float lds_all[GLDS + PW];
  float* bsh = lds_all + GLDS;
  const int p = P.p;
  for (int c = threadIdx.x; c < PW; c += blockDim.x) bsh[c] = (c < p) ? beta[c] : 0.0f;
  __syncthreads();   // the only barrier: before any wave can leave
  const int lane = threadIdx.x & 63;
  // wave-uniform unit: the row loop, the full-chunk test and the row bases are scalar
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (unit >= n_units) return;
  const int h = lane >> 4, cl = lane & 15;
  const int64_t r_begin = (int64_t)unit * rows_per_unit;
  const int64_t r_end = min(n, r_begin + rows_per_unit);
  const bool zlane = (NB - 1) * 16 + cl == p + 1;   // this lane's last-block column is z
  float bl[NB];                                      // this lane's coefficients, one per block
#pragma unroll
  for (int b = 0; b < NB; ++b) bl[b] = bsh[b * 16 + cl];

  f32x4 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const double b0 = (double)beta[p];
  double dev_acc = 0.0;
  u32x4_g H[NB], M[NB], L[NB];   // the previous chunk's pieces (zero before the first)
#pragma unroll
  for (int b = 0; b < NB; ++b) H[b] = M[b] = L[b] = u32x4_g{0u, 0u, 0u, 0u};

  float xc[NB][GW_S], xn[NB][GW_S];
  float yc = 0.f, wc = 1.f, oc = 0.f, yn = 0.f, wn = 1.f, on = 0.f;
  // Blocks 0 .. NB-3 are all data columns (p >= 16 NB - 17); the last two read
  // a clamped column and select data / 1 (intercept) / 0.  Rows past r_end
  // (the last unit's tail chunk) load as 0 and get a zero sqrt(w).
  auto load = [&](int64_t r0, float (&xb)[NB][GW_S], float& yv, float& wv, float& ov) {
    const int64_t rr = r0 + h * GW_S;
    const bool full = VEC && r0 + GW_RB <= r_end;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int c = b * 16 + cl;
      const float* src = X + (int64_t)(b >= NB - 2 ? min(c, p - 1) : c) * ld;
      if (full) {
#pragma unroll
        for (int q = 0; q < GW_S / 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(src + rr + 4 * q);
          xb[b][4 * q] = v.x; xb[b][4 * q + 1] = v.y; xb[b][4 * q + 2] = v.z; xb[b][4 * q + 3] = v.w;
        }
      } else {   // (guarded loads: a form the 16-byte path above is not merged with)
#pragma unroll
        for (int s = 0; s < GW_S; ++s) xb[b][s] = (rr + s < r_end) ? src[rr + s] : 0.0f;
      }
      if (b >= NB - 2) {
        const float k = (c == p) ? 1.0f : 0.0f;   // intercept column
#pragma unroll
        for (int s = 0; s < GW_S; ++s) xb[b][s] = (c < p) ? xb[b][s] : k;
      }
    }
    const int64_t row = min(r0 + h * GW_S + (cl & (GW_S - 1)), r_end - 1);
    yv = y[row];
    wv = wprior ? wprior[row] : 1.0f;
    ov = offset ? offset[row] : 0.0f;
  };
  // upper Gram tiles of the pieces in H / M / L: 6 significant products per tile
  auto gram = [&]() {
    int t = 0;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = bi; bj < NB; ++bj, ++t) {
        f32x4 a = acc[t];
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(M[bi]), as_bf16x8(M[bj]), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(L[bi]), as_bf16x8(H[bj]), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(H[bi]), as_bf16x8(L[bj]), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(M[bi]), as_bf16x8(H[bj]), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(H[bi]), as_bf16x8(M[bj]), a, 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(H[bi]), as_bf16x8(H[bj]), a, 0, 0, 0);
      }
  };
  auto prepare = [&](int64_t r0, float (&xb)[NB][GW_S], float yv, float wv, float ov) {
    // 1. partial linear predictors of the lane's 8 rows over its NB columns
    float pf[GW_S];
#pragma unroll
    for (int s = 0; s < GW_S; ++s) pf[s] = 0.f;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int s = 0; s < GW_S; ++s) pf[s] = fmaf(xb[b][s], bl[b], pf[s]);
    // 2. fp64 sum over the 16 column lanes: butterfly over lane bit 3, then a
    //    reduce-scatter over bits 2..0 -> lane c owns row c % 8
    double part[GW_S];
#pragma unroll
    for (int s = 0; s < GW_S; ++s) {
      part[s] = (double)pf[s];
      part[s] += __shfl_xor(part[s], 8, kWave);
    }
#pragma unroll
    for (int off = GW_S / 2; off >= 1; off >>= 1) {
      const bool hi = (cl & off) != 0;
#pragma unroll
      for (int j = 0; j < off; ++j) {
        const double send = hi ? part[j] : part[j + off];
        const double recv = __shfl_xor(send, off, kWave);
        part[j] = (hi ? part[j + off] : part[j]) + recv;
      }
    }
    // 3. IRLS weight / working response / deviance of this lane's row
    const int64_t row = r0 + h * GW_S + (cl & (GW_S - 1));
    const bool live = row < r_end;
    const double eta = part[0] + b0 + (double)ov;
    float sw, zz;
    double dv;
    if (FAM == 1) {
      glm_row_binomial(eta, (double)ov, (double)yv, (double)wv, sw, zz, dv);
    } else {
      double mu, dmu;
      glm_link(P, eta, mu, dmu);
      const double wi = (double)wv * dmu * dmu / glm_var(P, mu);
      zz = (float)(eta - (double)ov + ((double)yv - mu) / dmu);
      sw = (float)sqrt(fmax(wi, 0.0));
      dv = (double)wv * glm_dev(P, (double)yv, mu);
    }
    sw = live ? sw : 0.f;
    zz = live ? zz : 0.f;
    dev_acc += (live && cl < GW_S) ? dv : 0.0;   // lanes c and c + 8 share a row
    // 4. scale by sqrt(w) of the rows (the intercept column becomes sqrt(w)),
    //    z column, then the exact bf16 pieces of every block
    const int base = lane & 48;
#pragma unroll
    for (int s = 0; s < GW_S; ++s) {
      const float sws = __shfl(sw, base + s, kWave);
      const float zs = __shfl(zz, base + s, kWave);
#pragma unroll
      for (int b = 0; b < NB; ++b) xb[b][s] *= sws;
      xb[NB - 1][s] = zlane ? zs * sws : xb[NB - 1][s];
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) split3_bf16(xb[b], H[b], M[b], L[b]);
  };

  if (G) {
    const int wid = threadIdx.x >> 6;
    // chunk r (full) -> slot: per block two 1 KB lane-linear pieces, then y / w / offset
    auto issue = [&](int64_t r, int slot) {
      float* sb = lds_all + (wid * 2 + slot) * SLOTF;
      const int64_t rr = r + h * GW_S;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int c = b * 16 + cl;
        const float* src = X + (int64_t)(b >= NB - 2 ? min(c, p - 1) : c) * ld + rr;
#pragma unroll
        for (int q = 0; q < GW_S / 4; ++q)
          __builtin_amdgcn_global_load_lds(src + 4 * q, sb + (b * 2 + q) * 256, 16, 0, 0);
      }
      const int64_t row = r + h * GW_S + (cl & (GW_S - 1));
      __builtin_amdgcn_global_load_lds(y + row, sb + NB * 512, 4, 0, 0);
      __builtin_amdgcn_global_load_lds((wprior ? wprior : y) + row, sb + NB * 512 + 64, 4, 0, 0);
      __builtin_amdgcn_global_load_lds((offset ? offset : y) + row, sb + NB * 512 + 128, 4, 0, 0);
    };
    // s_waitcnt immediates (gfx9 encoding; expcnt / lgkmcnt left at their maxima)
    constexpr int NI = 2 * NB + 3;                                   // LDS-DMAs per chunk
    constexpr int W_ONE = (NI & 15) | (7 << 4) | (15 << 8) | ((NI >> 4) << 14);   // vmcnt <= NI
    constexpr int W_ALL = (7 << 4) | (15 << 8);                      // vmcnt 0
    const int64_t nfull = (r_end - r_begin) / GW_RB;
    if (nfull > 0) issue(r_begin, 0);
    if (nfull > 1) issue(r_begin + GW_RB, 1);
    for (int64_t i = 0; i < nfull; ++i) {
      const int64_t r = r_begin + i * GW_RB;
      const int slot = (int)(i & 1);
      if (i + 1 < nfull) __builtin_amdgcn_s_waitcnt(W_ONE);          // chunk i landed, i + 1 in flight
      else __builtin_amdgcn_s_waitcnt(W_ALL);
      // the slot's reads in inline asm: hipcc cannot see that they only touch
      // the landed chunk and would drain every LDS-DMA (vmcnt(0)) before a
      // compiler-visible ds_read; one lgkmcnt(0) wait, then register fences
      // order every use after it (and the slot's refill after the reads)
      const uint32_t la = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)(
                              lds_all + (wid * 2 + slot) * SLOTF) + (uint32_t)lane * 16u;
      const uint32_t lb = la - (uint32_t)lane * 12u;   // + lane * 4: the y / w / offset rows
      f32x4 t[NB][2];
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(t[b][q]) : "v"(la), "i"((b * 2 + q) * 1024));
      float ty, tw, to;
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(ty) : "v"(lb), "i"(NB * 2048));
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(tw) : "v"(lb), "i"(NB * 2048 + 256));
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(to) : "v"(lb), "i"(NB * 2048 + 512));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < 2; ++q) asm volatile("" : "+v"(t[b][q]));
      asm volatile("" : "+v"(ty), "+v"(tw), "+v"(to));
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int c = b * 16 + cl;
#pragma unroll
        for (int q = 0; q < GW_S / 4; ++q) {
          const f32x4 v = t[b][q];
          xc[b][4 * q] = v[0]; xc[b][4 * q + 1] = v[1]; xc[b][4 * q + 2] = v[2]; xc[b][4 * q + 3] = v[3];
        }
        if (b >= NB - 2) {
          const float kk = (c == p) ? 1.0f : 0.0f;   // intercept column
#pragma unroll
          for (int s = 0; s < GW_S; ++s) xc[b][s] = (c < p) ? xc[b][s] : kk;
        }
      }
      yc = ty;
      wc = wprior ? tw : 1.0f;
      oc = offset ? to : 0.0f;
      if (i + 2 < nfull) issue(r + 2 * GW_RB, slot);
      gram();                        // previous chunk (zero pieces on the first pass)
      prepare(r, xc, yc, wc, oc);    // this chunk -> H / M / L
    }
    const int64_t rt = r_begin + nfull * GW_RB;   // partial tail chunk: ordinary guarded loads
    if (rt < r_end) {
      load(rt, xc, yc, wc, oc);
      gram();
      prepare(rt, xc, yc, wc, oc);
    }
  } else {
    int64_t r0 = r_begin;
    if (r0 < r_end) load(r0, xc, yc, wc, oc);
    for (; r0 < r_end; r0 += GW_RB) {
      if (r0 + GW_RB < r_end) load(r0 + GW_RB, xn, yn, wn, on);
      gram();                        // previous chunk (zero pieces on the first pass)
      prepare(r0, xc, yc, wc, oc);   // this chunk -> H / M / L
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int s = 0; s < GW_S; ++s) xc[b][s] = xn[b][s];
      yc = yn; wc = wn; oc = on;
    }
  }
  gram();                          // the last chunk
  float* out = slab + (int64_t)unit * PW * PW;
  int t = 0;
#pragma unroll
  for (int bi = 0; bi < NB; ++bi)
#pragma unroll
    for (int bj = bi; bj < NB; ++bj, ++t)
#pragma unroll
      for (int v = 0; v < 4; ++v) out[(bi * 16 + 4 * h + v) * PW + bj * 16 + cl] = acc[t][v];
  const double d = wave_sum(dev_acc);
  if (lane == 0) dev_out[unit] = d;
}

// fp64 sum of the per-unit slabs of glm_irls_wave_kernel (upper 16x16 tiles;
// strictly-lower tile entries come out 0 and are mirrored on the host).
// Pass 1 (grid.y = SLAB_SPLIT): each thread sums every SLAB_SPLIT-th slab of
// one element into part[y][j] (enough independent loads in flight to stream
// the slabs at HBM rate); pass 2 folds the SLAB_SPLIT partials in fixed order.
constexpr int SLAB_SPLIT = 32;
__global__ __launch_bounds__(256) void slab_reduce16_kernel(const float* __restrict__ slab, int n_slabs, int pw,
                                                            double* __restrict__ part) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t w = (int64_t)pw * pw;
  if (j >= w) return;
  const int i = j / pw, k = j % pw;
  double a0 = 0.0, a1 = 0.0;
  if ((i >> 4) <= (k >> 4)) {
    int s = blockIdx.y;
    for (; s + SLAB_SPLIT < n_slabs; s += 2 * SLAB_SPLIT) {
      a0 += slab[(int64_t)s * w + j];
      a1 += slab[(int64_t)(s + SLAB_SPLIT) * w + j];
    }
    if (s < n_slabs) a0 += slab[(int64_t)s * w + j];
  }
  part[(int64_t)blockIdx.y * w + j] = a0 + a1;
}

__global__ __launch_bounds__(256) void slab_fold_kernel(const double* __restrict__ part, int64_t w,
                                                        double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= w) return;
  double a = 0.0;
#pragma unroll
  for (int y = 0; y < SLAB_SPLIT; ++y) a += part[(int64_t)y * w + j];
  out[j] = a;
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

// ---------------------------------------------------------------------------
// K-Means beyond the fused kernel's LDS tiles (d > 256 or k > 128): per row
// chunk [row0, row0 + m) the distances come from the MFMA GEMM
// G = C [k][d] x Xc [d][m] (gemm_kernel), then
//   kmeans_stage_kernel   X chunk -> dense Xc [d][m] (NaN -> 0, standardized space)
//   kmeans_argmin_kernel  best cluster per row from cn - 2 G, ||x||^2, per-block
//                         count / SSE slab (LDS atomics, one slab per block)
//   kmeans_onehot_kernel  OH [k][m] indicator of the assignment
// and the cluster sums are the GEMM OH x Xc^T (per-chunk fp32 slabs, reduced in
// fp64 by slab_sum_kernel): every FLOP on the matrix cores, no vendor library.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void kmeans_stage_kernel(const float* __restrict__ X, int64_t ldx, int d,
                                                           int64_t row0, int64_t m, float* __restrict__ Xc) {
  const int f = blockIdx.y;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256) {
    float v = X[(int64_t)f * ldx + row0 + r];
    Xc[(int64_t)f * m + r] = (v != v) ? 0.0f : v;
  }
}

__global__ __launch_bounds__(256) void kmeans_argmin_kernel(const float* __restrict__ G, int k, int64_t m,
                                                            const float* __restrict__ cn,
                                                            const float* __restrict__ Xc, int d,
                                                            int* __restrict__ assign, float* __restrict__ stat) {
  extern __shared__ float kst[];   // [k] counts | [k] sse
  for (int c = threadIdx.x; c < 2 * k; c += 256) kst[c] = 0.0f;
  __syncthreads();
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256) {
    float best = INFINITY;
    int bi = 0;
    for (int c = 0; c < k; ++c) {
      const float dist = cn[c] - 2.0f * G[(int64_t)c * m + r];
      if (dist < best) { best = dist; bi = c; }   // ascending c: ties keep the smaller id
    }
    float x2 = 0.0f;
    for (int f = 0; f < d; ++f) {
      const float v = Xc[(int64_t)f * m + r];
      x2 = fmaf(v, v, x2);
    }
    assign[r] = bi;
    atomicAdd(&kst[bi], 1.0f);
    atomicAdd(&kst[k + bi], fmaxf(best + x2, 0.0f));
  }
  __syncthreads();
  float* out = stat + (int64_t)blockIdx.x * 2 * k;
  for (int c = threadIdx.x; c < 2 * k; c += 256) out[c] = kst[c];
}

__global__ __launch_bounds__(256) void kmeans_onehot_kernel(const int* __restrict__ assign, int k, int64_t m,
                                                            float* __restrict__ OH) {
  const int c = blockIdx.y;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256)
    OH[(int64_t)c * m + r] = (assign[r] == c) ? 1.0f : 0.0f;
}

// OutT float: the fp64 sum rounded once into an fp32 destination (a bias
// gradient written in place: no separate fp64 -> fp32 copy launch)
template <typename OutT = double>
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slab, int n_slabs, int width,
                                                       OutT* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= width) return;
  double acc = 0.0;
  for (int s = 0; s < n_slabs; ++s) acc += slab[(int64_t)s * width + j];
  out[j] = (OutT)acc;
}

// Many slabs of a narrow width (per-wave K-Means slabs: ~1000 x 1020): one
// 1024-thread block per 32 columns, 32 slab groups of strided slabs with 4
// loads in flight per thread, folded through LDS in fixed order (deterministic)
__global__ __launch_bounds__(1024) void slab_sum_wide_kernel(const float* __restrict__ slab, int n_slabs, int width,
                                                             double* __restrict__ out) {
  __shared__ double red[32][33];
  const int c = threadIdx.x & 31, grp = threadIdx.x >> 5;
  const int j = blockIdx.x * 32 + c;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (j < width) {
    int s = grp;
    for (; s + 96 < n_slabs; s += 128) {
      a0 += slab[(int64_t)s * width + j];
      a1 += slab[(int64_t)(s + 32) * width + j];
      a2 += slab[(int64_t)(s + 64) * width + j];
      a3 += slab[(int64_t)(s + 96) * width + j];
    }
    for (; s < n_slabs; s += 32) a0 += slab[(int64_t)s * width + j];
  }
  red[grp][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (grp == 0 && j < width) {
    double acc = 0.0;
    for (int g = 0; g < 32; ++g) acc += red[g][c];
    out[j] = acc;
  }
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
    if (KM) { k = f >> 5; r = (f & 31) * 4; }                  // 32 float4 per k-row of 128
    else { r = f / (GK / 4); k = (f % (GK / 4)) * 4; }         // GK / 4 float4 per m-row of GK
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
      const int r = f / (GK / 4), k = (f % (GK / 4)) * 4;
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

// Same GEMM on 64 x 64 tiles: 256 threads, each wave one 32 x 32 MFMA
// accumulator.  The MLP's GEMMs (8192 x 512 x 512, weight gradients split-K)
// give only one 128 x 128 tile per CU - 8 waves whose load / barrier latency
// nothing else covers; quarter-size tiles put 4 workgroups (16 waves) on every
// CU.  Same K order per output element as gemm_kernel (k ascending in fmaf
// steps): bit-identical results.
constexpr int G64 = 64, G64T = 256;
struct Tile64 {
  float v[8];
};
template <bool KM>
__device__ __forceinline__ void load_tile64(const float* __restrict__ P, int ld, int rows, int k_lim, int r0, int k0,
                                            bool vec, Tile64& t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int f = tid + G64T * q;   // float4 index in the 64 x 32 tile
    int r, k;
    if (KM) { k = f >> 4; r = (f & 15) * 4; }   // 16 float4 per k-row of 64
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

template <bool KM>
__device__ __forceinline__ void store_tile64(float (*S)[G64 + GPAD], const Tile64& t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int f = tid + G64T * q;
    if (KM) {
      const int k = f >> 4, r = (f & 15) * 4;
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

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm64_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                     float* __restrict__ Cm, const float* __restrict__ bias, int M,
                                                     int N, int K, int act, float beta_c) {
  __shared__ __attribute__((aligned(16))) float As[2][32][G64 + GPAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][32][G64 + GPAD];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int m0 = blockIdx.y * G64, n0 = blockIdx.x * G64;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  const int S = gridDim.z;
  const int kchunk = ((K + S - 1) / S + 31) / 32 * 32;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  if (S > 1) Cm += (int64_t)blockIdx.z * M * N;
  const bool va = (TA ? (M % 4 == 0) : (K % 4 == 0)) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool vb = (TB ? (K % 4 == 0) : (N % 4 == 0)) && ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
  const int li = lane & 31, lh = lane >> 5;
  Tile64 ra, rb;
  int buf = 0;
  if (kb < ke) {
    load_tile64<TA>(A, TA ? M : K, M, ke, m0, kb, va, ra);
    load_tile64<!TB>(B, TB ? K : N, N, ke, n0, kb, vb, rb);
    store_tile64<TA>(As[0], ra);
    store_tile64<!TB>(Bs[0], rb);
  }
  __syncthreads();
  for (int k0 = kb; k0 < ke; k0 += 32) {
    const bool more = k0 + 32 < ke;
    if (more) {
      load_tile64<TA>(A, TA ? M : K, M, ke, m0, k0 + 32, va, ra);
      load_tile64<!TB>(B, TB ? K : N, N, ke, n0, k0 + 32, vb, rb);
    }
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) {
      const int kk = 2 * s2 + lh;
      acc = mfma32(As[buf][kk][wm + li], Bs[buf][kk][wn + li], acc);
    }
    if (more) {
      store_tile64<TA>(As[buf ^ 1], ra);
      store_tile64<!TB>(Bs[buf ^ 1], rb);
    }
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int i = m0 + wm + (e & 3) + 8 * (e >> 2) + 4 * lh;
    const int j = n0 + wn + li;
    if (i < M && j < N) {
      float v = acc[e];
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

// ---------------------------------------------------------------------------
// fp32 GEMM with 64 x 64 wave tiles (the MLP's 8192 x 512 x 512 layers).
// gemm64_kernel gives each wave one 32 x 32 accumulator: two LDS reads per
// 32x32x2 MFMA and a barrier every 16 MFMAs, ~50 % of the fp32 MFMA peak.
// Here 4 waves (2 x 2) share a BM x BN block tile and each wave owns a
// (BM/2) x (BN/2) tile of (BM/64) x (BN/64) 32x32 accumulators: per k pair a
// lane reads BM/64 + BN/64 operands for (BM/64)(BN/64) MFMAs, and a K-step of
// 32 is 16 x that many MFMAs between barriers (64 per wave at 128 x 128), long
// enough to hide the register-staged global loads of the next K-step.
// LDS images are [k][row]: row-major (MK) operands are transposed by scalar
// ds_write_b32 into rows of 129 floats (bank (k + r) % 32: the 32 lanes of a
// half-wave write 32 distinct banks), column-major (KM) ones by ds_write_b128
// into rows of 132 floats.
// EPI 0: C = act(acc + bias + beta_c C), or the raw split-K partial (gridDim.z > 1).
// EPI 1 (back-propagation through an activation): C = acc * act'(Y) with Y the
//   layer's output [M][N], plus the column sums of C over this block's BM rows
//   -> bws[blockIdx.y][N] (the bias-gradient partials gemm_wgrad_bias folds).
// ---------------------------------------------------------------------------
constexpr int GW_T = 256;
constexpr int GW_SPLIT = 4;   // k pairs (of 16 per K-step) before the FULL pipeline's LDS write / next loads
// dY * act'(Y) given the activation's output Y (Rectifier / Tanh)
__device__ __forceinline__ float act_grad(float g, float y, int act) {
  if (act == 1) return y > 0.0f ? g : 0.0f;
  if (act == 2) return g * (1.0f - y * y);
  return g;
}

template <bool KM> struct GwPad { static constexpr int v = KM ? 4 : 1; };

template <int R, bool KM, bool FULL>
__device__ __forceinline__ void gw_load(const float* __restrict__ P, int ld, int rows, int k_lim, int r0, int k0,
                                        bool vec, float (&t)[R / 8]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < R / 32; ++q) {
    const int f = tid + GW_T * q;   // float4 index in the R x 32 tile
    int r, k;
    if (KM) { k = f / (R / 4); r = (f % (R / 4)) * 4; }
    else { r = f >> 3; k = (f & 7) * 4; }
    const int gr = r0 + r, gk = k0 + k;
    if (FULL) {
      // 16-byte aligned rows, K and the KM operands' row counts % 4 == 0: one dwordx4
      // per float4, masked by one compare per edge (partial K-step / partial tile)
      float4 v4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gk < k_lim && gr < rows)
        v4 = *reinterpret_cast<const float4*>(KM ? P + (int64_t)gk * ld + gr : P + (int64_t)gr * ld + gk);
      t[4 * q] = v4.x; t[4 * q + 1] = v4.y; t[4 * q + 2] = v4.z; t[4 * q + 3] = v4.w;
      continue;
    }
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
    t[4 * q] = x0; t[4 * q + 1] = x1; t[4 * q + 2] = x2; t[4 * q + 3] = x3;
  }
}

template <int R, bool KM>
__device__ __forceinline__ void gw_store(float* __restrict__ S, const float (&t)[R / 8]) {
  constexpr int LD = R + GwPad<KM>::v;
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < R / 32; ++q) {
    const int f = tid + GW_T * q;
    if (KM) {
      const int k = f / (R / 4), r = (f % (R / 4)) * 4;
      *reinterpret_cast<float4*>(S + k * LD + r) = make_float4(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
    } else {
      const int r = f >> 3, k = (f & 7) * 4;
      S[k * LD + r] = t[4 * q];
      S[(k + 1) * LD + r] = t[4 * q + 1];
      S[(k + 2) * LD + r] = t[4 * q + 2];
      S[(k + 3) * LD + r] = t[4 * q + 3];
    }
  }
}

// FULL: M, N, K % 4 == 0, 16-byte aligned operands: dwordx4 loads masked by one
// compare per edge, the XCD-aware tile order (consecutive tiles of one
// XCD share A row blocks in its L2) and the next K-step's LDS image written
// between the two halves of the current step's MFMAs.
template <bool TA, bool TB, int BM, int BN, int EPI, bool FULL>
__global__ __launch_bounds__(GW_T) void gemm_w64_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                       float* __restrict__ Cm, const float* __restrict__ bias,
                                                       const float* __restrict__ Y, float* __restrict__ bws, int M,
                                                       int N, int K, int act, float beta_c) {
  constexpr int FM = BM / 64, FN = BN / 64;
  constexpr int LDA = BM + GwPad<TA>::v, LDB = BN + GwPad<!TB>::v;
  __shared__ __attribute__((aligned(16))) float As[2][32 * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[2][32 * LDB];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  int tile_x = blockIdx.x, tile_y = blockIdx.y;
  if (FULL) {
    // dispatch puts linear block b on XCD b % 8: renumber so that XCD x owns the
    // contiguous tile range [x * nb / 8, (x + 1) * nb / 8) (row-major over tiles)
    const int gx = gridDim.x, nb = gx * gridDim.y;
    if ((nb & 7) == 0) {
      const int b = blockIdx.y * gx + blockIdx.x;
      const int r = (b & 7) * (nb >> 3) + (b >> 3);
      tile_x = r % gx;
      tile_y = r / gx;
    }
  }
  const int m0 = tile_y * BM, n0 = tile_x * BN;
  const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
  const int S = gridDim.z;
  const int kchunk = ((K + S - 1) / S + 31) / 32 * 32;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  if (S > 1) Cm += (int64_t)blockIdx.z * M * N;
  const bool va = (TA ? (M % 4 == 0) : (K % 4 == 0)) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool vb = (TB ? (K % 4 == 0) : (N % 4 == 0)) && ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
  f32x16 acc[FM][FN];
#pragma unroll
  for (int x = 0; x < FM; ++x)
#pragma unroll
    for (int y = 0; y < FN; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.0f;
  const int li = lane & 31, lh = lane >> 5;
  float ra[BM / 8], rb[BN / 8];
  int buf = 0;
  if (kb < ke) {
    gw_load<BM, TA, FULL>(A, TA ? M : K, M, ke, m0, kb, va, ra);
    gw_load<BN, !TB, FULL>(B, TB ? K : N, N, ke, n0, kb, vb, rb);
    gw_store<BM, TA>(As[0], ra);
    gw_store<BN, !TB>(Bs[0], rb);
    if (FULL && kb + 32 < ke) {
      // FULL pipeline: the registers always hold the NEXT K-step's tile
      gw_load<BM, TA, FULL>(A, TA ? M : K, M, ke, m0, kb + 32, va, ra);
      gw_load<BN, !TB, FULL>(B, TB ? K : N, N, ke, n0, kb + 32, vb, rb);
    }
  }
  __syncthreads();
  // operands of k pair s2 + 1 are read from LDS before the MFMAs of pair s2
  // issue (register double buffer): the LDS latency hides behind the matrix
  // pipe instead of stalling every pair at an lgkmcnt(0)
  auto mfma_steps = [&](const float* as, const float* bs, int s_lo, int s_hi) {
    float a[2][FM], b[2][FN];
#pragma unroll
    for (int x = 0; x < FM; ++x) a[0][x] = as[(2 * s_lo + lh) * LDA + wm + 32 * x + li];
#pragma unroll
    for (int y = 0; y < FN; ++y) b[0][y] = bs[(2 * s_lo + lh) * LDB + wn + 32 * y + li];
#pragma unroll
    for (int s2 = s_lo; s2 < s_hi; ++s2) {
      const int c = (s2 - s_lo) & 1;
      if (s2 + 1 < s_hi) {
        const int kn = 2 * (s2 + 1) + lh;
#pragma unroll
        for (int x = 0; x < FM; ++x) a[c ^ 1][x] = as[kn * LDA + wm + 32 * x + li];
#pragma unroll
        for (int y = 0; y < FN; ++y) b[c ^ 1][y] = bs[kn * LDB + wn + 32 * y + li];
      }
      // keep the scheduler from sinking the prefetch below the MFMAs
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y) acc[x][y] = mfma32(a[c][x], b[c][y], acc[x][y]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int k0 = kb; k0 < ke; k0 += 32) {
    const bool more = k0 + 32 < ke;
    if (FULL) {
      // registers hold step k+1 (loaded one whole K-step ago): after the first
      // GW_SPLIT k pairs, write them to the other LDS buffer (last read before the
      // previous barrier) and issue step k+2's loads into the same registers, so
      // every global load has a full K-step of MFMAs to arrive.  (Spreading the
      // stores / loads one float4 per k pair between the MFMA groups measured
      // slower: 51.5 vs 50.0 us at 8192 x 512 x 512, 57 vs 50 us for the weight
      // gradient.)
      mfma_steps(As[buf], Bs[buf], 0, GW_SPLIT);
      if (more) {
        gw_store<BM, TA>(As[buf ^ 1], ra);
        gw_store<BN, !TB>(Bs[buf ^ 1], rb);
        if (k0 + 64 < ke) {
          gw_load<BM, TA, FULL>(A, TA ? M : K, M, ke, m0, k0 + 64, va, ra);
          gw_load<BN, !TB, FULL>(B, TB ? K : N, N, ke, n0, k0 + 64, vb, rb);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_steps(As[buf], Bs[buf], GW_SPLIT, 16);
    } else {
      if (more) {
        gw_load<BM, TA, FULL>(A, TA ? M : K, M, ke, m0, k0 + 32, va, ra);
        gw_load<BN, !TB, FULL>(B, TB ? K : N, N, ke, n0, k0 + 32, vb, rb);
      }
      mfma_steps(As[buf], Bs[buf], 0, 16);
      if (more) {
        gw_store<BM, TA>(As[buf ^ 1], ra);
        gw_store<BN, !TB>(Bs[buf ^ 1], rb);
      }
    }
    __syncthreads();
    buf ^= 1;
  }
  if (EPI == 1) {
    // C = acc * act'(Y); per-column partial sums of C over the block's rows
    float* red = As[0];   // [2 row-waves][BN] (the K loop ended on a barrier)
#pragma unroll
    for (int y = 0; y < FN; ++y) {
      const int j = n0 + wn + 32 * y + li;
      float cs = 0.0f;
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int i = m0 + wm + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * lh;
          if (i < M && j < N) {
            const int64_t o = (int64_t)i * N + j;
            const float v = act_grad(acc[x][y][e], Y[o], act);
            Cm[o] = v;
            cs += v;
          }
        }
      cs += __shfl_xor(cs, 32);
      if (lh == 0) red[(wid >> 1) * BN + wn + 32 * y + li] = cs;
    }
    __syncthreads();
    for (int c = t; c < BN; c += GW_T) {
      const int j = n0 + c;
      if (j < N) bws[(int64_t)tile_y * N + j] = red[c] + red[BN + c];
    }
    return;
  }
#pragma unroll
  for (int x = 0; x < FM; ++x)
#pragma unroll
    for (int y = 0; y < FN; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int i = m0 + wm + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * lh;
        const int j = n0 + wn + 32 * y + li;
        if (i < M && j < N) {
          float v = acc[x][y][e];
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

// Skinny outputs (N <= 8, e.g. the MLP's 2-class output layer): C[M][N] =
// act(A[M][K] B[N][K]^T + bias).  A 128 x 128 MFMA tile would compute 64x
// more zeros than results (45 us for 8192 x 2 x 512); here one wave per row
// streams its A row with float4 loads (B rows stay in L1/L2) and reduces
// the N dot products with wave shuffles.
constexpr int SKINNY_N = 8;
// (y != nullptr: softmax cross-entropy epilogue - the row's N logits are in
// every lane after the wave reduction, so dZ = (softmax - onehot(y)) / M is
// written beside them with softmax_xent_kernel's exact arithmetic)
__global__ __launch_bounds__(256) void gemm_skinny_nt_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                             float* __restrict__ C, const float* __restrict__ bias,
                                                             int M, int N, int K, int act,
                                                             const int* __restrict__ y = nullptr,
                                                             float* __restrict__ dZ = nullptr) {
  const int lane = threadIdx.x & 63;
  const int waves = gridDim.x * (blockDim.x >> 6);
  const bool vec = (K % 4 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(B) & 15) == 0);
  for (int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < M; i += waves) {
    const float* a = A + (int64_t)i * K;
    float acc[SKINNY_N];
#pragma unroll
    for (int n = 0; n < SKINNY_N; ++n) acc[n] = 0.0f;
    if (vec) {
      for (int k = 4 * lane; k < K; k += 256) {
        const float4 x = *reinterpret_cast<const float4*>(a + k);
#pragma unroll
        for (int n = 0; n < SKINNY_N; ++n) {
          if (n < N) {
            const float4 w = *reinterpret_cast<const float4*>(B + (int64_t)n * K + k);
            acc[n] += x.x * w.x + x.y * w.y + x.z * w.z + x.w * w.w;
          }
        }
      }
    } else {
      for (int k = lane; k < K; k += 64) {
        const float x = a[k];
#pragma unroll
        for (int n = 0; n < SKINNY_N; ++n)
          if (n < N) acc[n] += x * B[(int64_t)n * K + k];
      }
    }
#pragma unroll
    for (int n = 0; n < SKINNY_N; ++n) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc[n] += __shfl_xor(acc[n], o, 64);
    }
    if (lane < N) {
      float v = 0.0f;
#pragma unroll
      for (int n = 0; n < SKINNY_N; ++n)
        if (n == lane) v = acc[n];
      if (bias) v += bias[lane];
      if (act == 1) v = fmaxf(v, 0.0f);
      else if (act == 2) v = tanhf(v);
      C[(int64_t)i * N + lane] = v;
    }
    if (y != nullptr) {
      float z[SKINNY_N];
#pragma unroll
      for (int n = 0; n < SKINNY_N; ++n) z[n] = (n < N) ? acc[n] + (bias ? bias[n] : 0.0f) : 0.0f;
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < SKINNY_N; ++n)
        if (n < N) mx = fmaxf(mx, z[n]);
      float den = 0.0f;
#pragma unroll
      for (int n = 0; n < SKINNY_N; ++n)
        if (n < N) den += __expf(z[n] - mx);
      const int yi = y[i];
      if (lane < N) {
        float zl = 0.0f;
#pragma unroll
        for (int n = 0; n < SKINNY_N; ++n)
          if (n == lane) zl = z[n];
        const float pk = __expf(zl - mx) / den;
        dZ[(int64_t)i * N + lane] = (pk - (lane == yi ? 1.0f : 0.0f)) / (float)M;
      }
    }
  }
}

// Tiny inner dimension (K <= 8, e.g. dH = dZ W through the 2-class output
// layer): C[M][N] = A[M][K] B[K][N] as a streaming outer-product sum, fused
// with the activation derivative of the layer below (act_y: Y of that layer,
// act: 1 relu, 2 tanh) so dZ comes out in one pass.
__global__ __launch_bounds__(256) void gemm_thin_k_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                          float* __restrict__ C, int64_t M, int N, int K,
                                                          const float* __restrict__ act_y, int act) {
  const int64_t total = M * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / N;
    const int j = (int)(e - i * N);
    float v = 0.0f;
    for (int k = 0; k < K; ++k) v += A[i * K + k] * B[(int64_t)k * N + j];
    if (act_y) {
      const float y = act_y[e];
      if (act == 1) v = y > 0.0f ? v : 0.0f;
      else if (act == 2) v *= 1.0f - y * y;
    }
    C[e] = v;
  }
}

// dZ = dY * act'(Y) and the column partial sums of dZ (the bias gradient of
// that layer) in ONE pass over dY: block = 256 columns (float4 per lane) x 4
// row phases over one row slice -> ws[slice][col]; the slices are summed
// later in a fixed order (deterministic), e.g. by the weight gradient's
// split-K reduce (gemm_splitk_reduce_kernel second job).  N % 4 == 0.
__global__ __launch_bounds__(256) void act_backward_bias_kernel(const float* __restrict__ Y, float* __restrict__ dY,
                                                                float* __restrict__ ws, int M, int N, int act) {
  __shared__ float4 red[4][64];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = (blockIdx.x * 64 + c) * 4;
  const int S = gridDim.y;
  const int rows = (M + S - 1) / S;
  const int r0 = blockIdx.y * rows, r1 = min(M, r0 + rows);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < N) {
    int i = r0 + ph;
    for (; i + 4 < r1; i += 8) {   // two rows' loads in flight per lane
      const int64_t e0 = (int64_t)i * N + j, e1 = e0 + 4 * (int64_t)N;
      float4 g0 = *reinterpret_cast<const float4*>(dY + e0), g1 = *reinterpret_cast<const float4*>(dY + e1);
      const float4 y0 = *reinterpret_cast<const float4*>(Y + e0), y1 = *reinterpret_cast<const float4*>(Y + e1);
      g0 = make_float4(act_grad(g0.x, y0.x, act), act_grad(g0.y, y0.y, act), act_grad(g0.z, y0.z, act),
                       act_grad(g0.w, y0.w, act));
      g1 = make_float4(act_grad(g1.x, y1.x, act), act_grad(g1.y, y1.y, act), act_grad(g1.z, y1.z, act),
                       act_grad(g1.w, y1.w, act));
      *reinterpret_cast<float4*>(dY + e0) = g0;
      *reinterpret_cast<float4*>(dY + e1) = g1;
      s.x += g0.x + g1.x; s.y += g0.y + g1.y; s.z += g0.z + g1.z; s.w += g0.w + g1.w;
    }
    for (; i < r1; i += 4) {
      const int64_t e0 = (int64_t)i * N + j;
      float4 g0 = *reinterpret_cast<const float4*>(dY + e0);
      const float4 y0 = *reinterpret_cast<const float4*>(Y + e0);
      g0 = make_float4(act_grad(g0.x, y0.x, act), act_grad(g0.y, y0.y, act), act_grad(g0.z, y0.z, act),
                       act_grad(g0.w, y0.w, act));
      *reinterpret_cast<float4*>(dY + e0) = g0;
      s.x += g0.x; s.y += g0.y; s.z += g0.z; s.w += g0.w;
    }
  }
  red[ph][c] = s;
  __syncthreads();
  if (ph == 0 && j < N) {
    const float4 a = red[0][c], b = red[1][c], d = red[2][c], e = red[3][c];
    *reinterpret_cast<float4*>(ws + (int64_t)blockIdx.y * N + j) =
        make_float4((a.x + b.x) + (d.x + e.x), (a.y + b.y) + (d.y + e.y), (a.z + b.z) + (d.z + e.z),
                    (a.w + b.w) + (d.w + e.w));
  }
}

// C = act(sum_z W[z] + beta_c * C + bias): split-K epilogue (fixed order: deterministic)
// Optional second job (W2 != nullptr): blocks >= main_blocks sum the S2
// slices of a [S2][N2] workspace into C2 (a bias gradient folded into the
// weight gradient's reduce launch).
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const float* __restrict__ W, int S, int M, int N,
                                                                 float* __restrict__ C, const float* __restrict__ bias,
                                                                 int act, float beta_c, int main_blocks = 0,
                                                                 const float* __restrict__ W2 = nullptr, int S2 = 0,
                                                                 int N2 = 0, float* __restrict__ C2 = nullptr) {
  if (W2 != nullptr && (int)blockIdx.x >= main_blocks) {
    // 64 columns per block, the 4 waves take every 4th slice (loads in flight), fixed-order fold
    __shared__ float red2[4][64];
    const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int j = (blockIdx.x - main_blocks) * 64 + c;
    float a = 0.0f, b = 0.0f;
    if (j < N2) {
      int z = ph;
      // 8 (a, b) pairs of loads in flight, then the adds in the same order
      for (; z + 60 < S2; z += 64) {
        float la[8], lb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          la[u] = W2[(int64_t)(z + 8 * u) * N2 + j];
          lb[u] = W2[(int64_t)(z + 8 * u + 4) * N2 + j];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          a += la[u];
          b += lb[u];
        }
      }
      for (; z + 4 < S2; z += 8) {
        a += W2[(int64_t)z * N2 + j];
        b += W2[(int64_t)(z + 4) * N2 + j];
      }
      for (; z < S2; z += 4) a += W2[(int64_t)z * N2 + j];
    }
    red2[ph][c] = a + b;
    __syncthreads();
    if (ph == 0 && j < N2) C2[j] = (red2[0][c] + red2[1][c]) + (red2[2][c] + red2[3][c]);
    return;
  }
  const int64_t MN = (int64_t)M * N;
  const int64_t gstride = (int64_t)(W2 != nullptr ? main_blocks : gridDim.x) * blockDim.x;
  if (bias == nullptr && act == 0 && beta_c == 0.0f && (MN & 3) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(C) & 15) == 0) {
    // plain sum (weight gradients): 4 columns per thread, 8 slices' loads in
    // flight, the adds in slice order (the same bits as the scalar loop below)
    const int64_t MN4 = MN >> 2;
    const float4* W4 = reinterpret_cast<const float4*>(W);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < MN4; i += gstride) {
      float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      int z = 0;
      for (; z + 8 <= S; z += 8) {
        float4 t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = W4[(int64_t)(z + u) * MN4 + i];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          v.x += t[u].x; v.y += t[u].y; v.z += t[u].z; v.w += t[u].w;
        }
      }
      for (; z < S; ++z) {
        const float4 t = W4[(int64_t)z * MN4 + i];
        v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
      }
      reinterpret_cast<float4*>(C)[i] = v;
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < MN; i += gstride) {
    float v = 0.0f;
    for (int z = 0; z < S; ++z) v += W[z * MN + i];
    if (beta_c != 0.0f) v += beta_c * C[i];
    if (bias) v += bias[i % N];
    if (act == 1) v = fmaxf(v, 0.0f);
    else if (act == 2) v = tanhf(v);
    C[i] = v;
  }
}

// ---------------------------------------------------------------------------
// MLP output layer with few classes (C <= 8, e.g. the 2-class softmax): the
// weight gradient dW[C][N] = dZ^T H and dZ_prev = (dZ W) * act'(H) are
// bandwidth work over H [M][N] (16 MB at 8192 x 512), not GEMMs: split-K MFMA
// tiles of a 2-row output (19.6 us + reduce) and a thin-K GEMM followed by the
// activation backward (9.5 + 9.8 us) become one streaming pass each.
// Block = 64 float4 columns (256 columns) x 4 row phases over one row slice.
// ---------------------------------------------------------------------------
constexpr int OUT_C = 8;

// stage 1: row z of ws[slice][C * N + C] = partial dZ^T H ([C][N]) followed by the
// partial column sums of dZ ([C]); the fold sums the slices of both in one pass
template <int C>
__global__ __launch_bounds__(256) void out_wgrad_kernel(const float* __restrict__ dZ, const float* __restrict__ H,
                                                        float* __restrict__ ws, int M, int N) {
  const int64_t T = (int64_t)C * N + C;
  __shared__ float4 red[4][64][C];
  const int c4 = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = (blockIdx.x * 64 + c4) * 4;
  const int S = gridDim.y;
  const int rows = (M + S - 1) / S;
  const int r0 = blockIdx.y * rows, r1 = min(M, r0 + rows);
  float4 acc[C];
  float bs[C];
#pragma unroll
  for (int c = 0; c < C; ++c) { acc[c] = make_float4(0.f, 0.f, 0.f, 0.f); bs[c] = 0.f; }
  if (j < N) {
    for (int i = r0 + ph; i < r1; i += 4) {
      const float4 h = *reinterpret_cast<const float4*>(H + (int64_t)i * N + j);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float z = dZ[(int64_t)i * C + c];
        acc[c].x += z * h.x; acc[c].y += z * h.y; acc[c].z += z * h.z; acc[c].w += z * h.w;
        bs[c] += z;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) red[ph][c4][c] = acc[c];
  __syncthreads();
  if (ph == 0 && j < N) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float4 a = red[0][c4][c], b = red[1][c4][c], d = red[2][c4][c], e = red[3][c4][c];
      float* o = ws + blockIdx.y * T + (int64_t)c * N + j;      // T may be odd: scalar stores
      o[0] = (a.x + b.x) + (d.x + e.x);
      o[1] = (a.y + b.y) + (d.y + e.y);
      o[2] = (a.z + b.z) + (d.z + e.z);
      o[3] = (a.w + b.w) + (d.w + e.w);
    }
  }
  if (blockIdx.x == 0) {
    // column sums of dZ over the slice (every column block computes them; block 0 writes)
    __syncthreads();
    float* rb = reinterpret_cast<float*>(red);     // [4 phases][64 lanes][C]
#pragma unroll
    for (int c = 0; c < C; ++c) rb[(ph * 64 + c4) * C + c] = (c4 == 0) ? bs[c] : 0.0f;
    __syncthreads();
    if (threadIdx.x < C) {
      const int c = threadIdx.x;
      ws[blockIdx.y * T + (int64_t)C * N + c] = (rb[(0 * 64) * C + c] + rb[(1 * 64) * C + c]) +
                                                (rb[(2 * 64) * C + c] + rb[(3 * 64) * C + c]);
    }
  }
}

// dZ_prev [M][N] = (dZ [M][C] W [C][N]) * act'(Y [M][N]) plus its column partial sums ws[slice][N]
template <int C>
__global__ __launch_bounds__(256) void thin_dact_kernel(const float* __restrict__ dZ, const float* __restrict__ W,
                                                        const float* __restrict__ Y, float* __restrict__ out,
                                                        float* __restrict__ ws, int M, int N, int act) {
  __shared__ float4 red[4][64];
  const int c4 = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = (blockIdx.x * 64 + c4) * 4;
  const int S = gridDim.y;
  const int rows = (M + S - 1) / S;
  const int r0 = blockIdx.y * rows, r1 = min(M, r0 + rows);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < N) {
    float4 w[C];
#pragma unroll
    for (int c = 0; c < C; ++c) w[c] = *reinterpret_cast<const float4*>(W + (int64_t)c * N + j);
    for (int i = r0 + ph; i < r1; i += 4) {
      const int64_t e = (int64_t)i * N + j;
      const float4 y = *reinterpret_cast<const float4*>(Y + e);
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float z = dZ[(int64_t)i * C + c];
        g.x += z * w[c].x; g.y += z * w[c].y; g.z += z * w[c].z; g.w += z * w[c].w;
      }
      g = make_float4(act_grad(g.x, y.x, act), act_grad(g.y, y.y, act), act_grad(g.z, y.z, act),
                      act_grad(g.w, y.w, act));
      *reinterpret_cast<float4*>(out + e) = g;
      s.x += g.x; s.y += g.y; s.z += g.z; s.w += g.w;
    }
  }
  red[ph][c4] = s;
  __syncthreads();
  if (ph == 0 && j < N) {
    const float4 a = red[0][c4], b = red[1][c4], d = red[2][c4], e = red[3][c4];
    *reinterpret_cast<float4*>(ws + (int64_t)blockIdx.y * N + j) =
        make_float4((a.x + b.x) + (d.x + e.x), (a.y + b.y) + (d.y + e.y), (a.z + b.z) + (d.z + e.z),
                    (a.w + b.w) + (d.w + e.w));
  }
}

// The output layer's whole backward in one pass over its input H [M][N]
// (out_wgrad_kernel + thin_dact_kernel fused: both stream the same H and dZ
// with the same (column block, row slice) grid): the weight / bias gradient
// partial rows -> wsw[slice][C * N + C], dZ_prev = (dZ W) * act'(H) -> out and
// its column partial sums -> wsb[slice][N].  Same arithmetic, same order.
template <int C>
__global__ __launch_bounds__(256) void out_backward_kernel(const float* __restrict__ dZ, const float* __restrict__ H,
                                                           const float* __restrict__ W, float* __restrict__ out,
                                                           float* __restrict__ wsw, float* __restrict__ wsb, int M,
                                                           int N, int act) {
  const int64_t T = (int64_t)C * N + C;
  __shared__ float4 red[4][64][C];
  __shared__ float4 redb[4][64];
  const int c4 = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = (blockIdx.x * 64 + c4) * 4;
  const int S = gridDim.y;
  const int rows = (M + S - 1) / S;
  const int r0 = blockIdx.y * rows, r1 = min(M, r0 + rows);
  float4 acc[C];
  float bs[C];
#pragma unroll
  for (int c = 0; c < C; ++c) { acc[c] = make_float4(0.f, 0.f, 0.f, 0.f); bs[c] = 0.f; }
  float4 sb = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < N) {
    float4 w[C];
#pragma unroll
    for (int c = 0; c < C; ++c) w[c] = *reinterpret_cast<const float4*>(W + (int64_t)c * N + j);
    for (int i = r0 + ph; i < r1; i += 4) {
      const int64_t e = (int64_t)i * N + j;
      const float4 h = *reinterpret_cast<const float4*>(H + e);
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float z = dZ[(int64_t)i * C + c];
        acc[c].x += z * h.x; acc[c].y += z * h.y; acc[c].z += z * h.z; acc[c].w += z * h.w;
        bs[c] += z;
        g.x += z * w[c].x; g.y += z * w[c].y; g.z += z * w[c].z; g.w += z * w[c].w;
      }
      g = make_float4(act_grad(g.x, h.x, act), act_grad(g.y, h.y, act), act_grad(g.z, h.z, act),
                      act_grad(g.w, h.w, act));
      *reinterpret_cast<float4*>(out + e) = g;
      sb.x += g.x; sb.y += g.y; sb.z += g.z; sb.w += g.w;
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c) red[ph][c4][c] = acc[c];
  redb[ph][c4] = sb;
  __syncthreads();
  if (ph == 0 && j < N) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float4 a = red[0][c4][c], b = red[1][c4][c], d = red[2][c4][c], e = red[3][c4][c];
      float* o = wsw + blockIdx.y * T + (int64_t)c * N + j;      // T may be odd: scalar stores
      o[0] = (a.x + b.x) + (d.x + e.x);
      o[1] = (a.y + b.y) + (d.y + e.y);
      o[2] = (a.z + b.z) + (d.z + e.z);
      o[3] = (a.w + b.w) + (d.w + e.w);
    }
    const float4 a = redb[0][c4], b = redb[1][c4], d = redb[2][c4], e = redb[3][c4];
    *reinterpret_cast<float4*>(wsb + (int64_t)blockIdx.y * N + j) =
        make_float4((a.x + b.x) + (d.x + e.x), (a.y + b.y) + (d.y + e.y), (a.z + b.z) + (d.z + e.z),
                    (a.w + b.w) + (d.w + e.w));
  }
  if (blockIdx.x == 0) {
    __syncthreads();
    float* rb = reinterpret_cast<float*>(red);     // [4 phases][64 lanes][C]
#pragma unroll
    for (int c = 0; c < C; ++c) rb[(ph * 64 + c4) * C + c] = (c4 == 0) ? bs[c] : 0.0f;
    __syncthreads();
    if (threadIdx.x < C) {
      const int c = threadIdx.x;
      wsw[blockIdx.y * T + (int64_t)C * N + c] = (rb[(0 * 64) * C + c] + rb[(1 * 64) * C + c]) +
                                                 (rb[(2 * 64) * C + c] + rb[(3 * 64) * C + c]);
    }
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
  if (loss == nullptr) return;      // training steps that do not report the loss
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

// ADADELTA with the last reductions of the backward folded in: gradient
// entries [off, off + len) are the fp64 sum of `splits` fp32 partial rows
// (stride floats apart) - the bias gradients' act-backward slices and the
// output layer's split weight gradient - written back to G and used at once
// (saves one small launch per layer on launch-bound mini-batch steps)
struct GradFix {
  int64_t off;
  const float* ws;
  int len, splits, stride, pad;
};
constexpr int MAX_GRAD_FIX = 8;
struct GradFixes {
  int n, pad;
  GradFix f[MAX_GRAD_FIX];
};

__device__ __forceinline__ float grad_fixed(const GradFixes& fx, int64_t i, float gi, bool& fixed) {
  for (int e = 0; e < fx.n; ++e) {
    const int64_t j = i - fx.f[e].off;
    if (j >= 0 && j < fx.f[e].len) {
      double a = 0.0;
      for (int s = 0; s < fx.f[e].splits; ++s) a += fx.f[e].ws[(int64_t)s * fx.f[e].stride + j];
      fixed = true;
      return (float)a;
    }
  }
  return gi;
}

__device__ __forceinline__ void adadelta_one(float& w, float g, float& eg2, float& edx2, float rho, float eps,
                                             float l2) {
  g += l2 * w;
  const float eg = rho * eg2 + (1.0f - rho) * g * g;
  const float dx = -sqrtf(edx2 + eps) / sqrtf(eg + eps) * g;
  eg2 = eg;
  edx2 = rho * edx2 + (1.0f - rho) * dx * dx;
  w += dx;
}

// one parameter per thread: the few fold entries spread over many threads
// (a 4-per-thread float4 version measured slower: its fold blocks straggle)
__global__ __launch_bounds__(256) void adadelta_fix_kernel(float* __restrict__ W, float* __restrict__ G,
                                                           float* __restrict__ Eg2, float* __restrict__ Edx2, int64_t n,
                                                           float rho, float eps, float l2, GradFixes fx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // block-uniform test first: most blocks touch no fold range and skip the per-element search
  const int64_t blo = (int64_t)blockIdx.x * blockDim.x, bhi = blo + blockDim.x;
  bool touch = false;
  for (int e = 0; e < fx.n; ++e) touch |= fx.f[e].off < bhi && fx.f[e].off + fx.f[e].len > blo;
  bool fixed = false;
  const float gi = touch ? grad_fixed(fx, i, G[i], fixed) : G[i];
  if (fixed) G[i] = gi;
  float w = W[i], eg2 = Eg2[i], edx2 = Edx2[i];
  adadelta_one(w, gi, eg2, edx2, rho, eps, l2);
  W[i] = w;
  Eg2[i] = eg2;
  Edx2[i] = edx2;
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
// bf16 MLP path: bf16 operands on the matrix cores (v_mfma_f32_32x32x16_bf16,
// 16x the fp32-MFMA rate), fp32 accumulation, fp32 master weights / optimizer.
//
// One GEMM form, "NT": C[m][n] = sum_k A[m*lda + k] * B[n*ldb + k], both
// operands K-contiguous, so every MFMA fragment (8 consecutive k of one row)
// is ONE 16-byte LDS read.  The MLP's three products map onto it by keeping
// the transposed copies the backward pass needs (written by the producing
// epilogue, never by a separate transpose):
//   forward   H_l     = act(H_{l-1} . W_l^T + b)   A = H_{l-1}, B = W_l
//   weights   dW_l    = dZ_l^T . H_{l-1}            A = dZ_l^T,  B = H_{l-1}^T
//   inputs    dZ_{l-1}= (dZ_l . W_l) * act'(H)      A = dZ_l,    B = W_l^T
// K (and lda / ldb) must be multiples of 8 (16-byte rows; callers zero-pad).
// 128 x 128 block tile, 8 waves of 32 x 64 (2 accumulators), BK = 64 per
// double-buffered LDS stage (rows padded to 144 B: the 16 lanes of a
// ds_read_b128 group hit 16 distinct 16-byte bank slots).
// ===========================================================================
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int HB = 128, HK = 64, HPAD = 8, HROW = HK + HPAD;   // bf16 elements
static int g_bf16_variant = -1;  // tile-variant override for A/B runs (h2omx_gemm_bf16_variant)

struct BfEpi {
  const float* bias;        // [N] or null
  const uint16_t* ymask;    // act' source Y (bf16 [M][ldy]) or null
  float* cf;                // fp32 out [M][ldc] or null
  uint16_t* cb;             // bf16 out [M][ldc] or null
  uint16_t* cbt;            // bf16 transposed out [N][ldt] or null
  float* c_last;            // column N-1 -> c_last[m] instead of cf (bias gradients via a ones row)
  int ldy, ldc, ldt;
  int act;                  // 0 none, 1 relu, 2 tanh (applied to the output)
  int mask_act;             // act' of ymask multiplied in (1 relu, 2 tanh), 0 none
  float beta_c;             // cf += beta_c * old cf
};

__device__ __forceinline__ uint16_t f2bf(float v) {
  __bf16 b = (__bf16)v;
  return *reinterpret_cast<uint16_t*>(&b);
}
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }

// global -> registers: a ROWS x 64 bf16 tile in 16-byte chunks, 8 chunks per row
template <int ROWS, int THREADS>
struct BfTile {
  static constexpr int NQ = ROWS * 8 / THREADS;
  uint4 v[NQ];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ P, int ld, int rows, int K, int r0, int k0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = threadIdx.x + THREADS * q;
      const int r = r0 + (c >> 3), kk = k0 + (c & 7) * 8;
      v[q] = (r < rows && kk < K) ? *reinterpret_cast<const uint4*>(P + (int64_t)r * ld + kk) : make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(uint16_t* S) const {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = threadIdx.x + THREADS * q;
      *reinterpret_cast<uint4*>(S + (c >> 3) * HROW + (c & 7) * 8) = v[q];
    }
  }
};

// Block tile BM x BN, wave tile WTM x WTN ((WTM / 32) x (WTN / 32) MFMA
// accumulators of 32 x 32), (BM / WTM) x (BN / WTN) waves.  Instances:
//   <128, 128, 64, 64>  4 waves, one 128 x 128 block per CU: 2 + 2 fragment
//                       reads per 4 MFMAs (the wide products)
//   <128,  64, 32, 64>  4 waves, two blocks per CU (narrow outputs)
template <int BM, int BN, int WTM, int WTN>
__global__ __launch_bounds__(64 * (BM / WTM) * (BN / WTN))
void gemm_bf16_nt_kernel(const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ B, int ldb, int M,
                         int N, int K, float* __restrict__ ws, BfEpi ep) {
  constexpr int WR = BM / WTM, WC = BN / WTN, THREADS = 64 * WR * WC;
  constexpr int AM = WTM / 32, AN = WTN / 32;
  __shared__ __attribute__((aligned(16))) uint16_t As[2][BM * HROW];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN * HROW];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int wm = (wid / WC) * WTM, wn = (wid % WC) * WTN;
  const int S = gridDim.z;
  const int kchunk = ((K + S - 1) / S + HK - 1) / HK * HK;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  f32x16 acc[AM][AN];
#pragma unroll
  for (int a = 0; a < AM; ++a)
#pragma unroll
    for (int b = 0; b < AN; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;
  const int li = lane & 31, lh = lane >> 5;
  // register prefetch PD stages deep: at step s the tiles of stage s + 1 (loaded
  // PD steps earlier) go to LDS and their registers immediately start loading
  // stage s + 1 + PD, so several global-load latencies overlap
  constexpr int PD = 3;
  BfTile<BM, THREADS> ra[PD];
  BfTile<BN, THREADS> rb[PD];
  const int nsteps = kb < ke ? (ke - kb + HK - 1) / HK : 0;
#pragma unroll
  for (int d = 0; d < PD; ++d) {
    if (d < nsteps) {
      ra[d].load(A, lda, M, ke, m0, kb + d * HK);
      rb[d].load(B, ldb, N, ke, n0, kb + d * HK);
    }
  }
  if (nsteps > 0) {
    ra[0].store(As[0]);
    rb[0].store(Bs[0]);
    if (PD < nsteps) {
      ra[0].load(A, lda, M, ke, m0, kb + PD * HK);
      rb[0].load(B, ldb, N, ke, n0, kb + PD * HK);
    }
  }
  __syncthreads();
  for (int s0 = 0; s0 < nsteps; s0 += PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int st = s0 + u;
      if (st < nsteps) {
        const int buf = st & 1;
        const uint16_t* as = As[buf] + (wm + li) * HROW + 8 * lh;
        const uint16_t* bs = Bs[buf] + (wn + li) * HROW + 8 * lh;
#pragma unroll
        for (int s2 = 0; s2 < HK / 16; ++s2) {
          bf16x8 af[AM], bfr[AN];
#pragma unroll
          for (int a = 0; a < AM; ++a) af[a] = *reinterpret_cast<const bf16x8*>(as + a * 32 * HROW + 16 * s2);
#pragma unroll
          for (int b = 0; b < AN; ++b) bfr[b] = *reinterpret_cast<const bf16x8*>(bs + b * 32 * HROW + 16 * s2);
#pragma unroll
          for (int a = 0; a < AM; ++a)
#pragma unroll
            for (int b = 0; b < AN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
        }
        if (st + 1 < nsteps) {
          const int nr = (u + 1) % PD;  // static once the u loop is unrolled
          ra[nr].store(As[buf ^ 1]);
          rb[nr].store(Bs[buf ^ 1]);
          if (st + 1 + PD < nsteps) {
            ra[nr].load(A, lda, M, ke, m0, kb + (st + 1 + PD) * HK);
            rb[nr].load(B, ldb, N, ke, n0, kb + (st + 1 + PD) * HK);
          }
        }
        __syncthreads();
      }
    }
  }
  // epilogue: lane owns column j, registers e are rows (e&3) + 8(e>>2) + 4h
#pragma unroll
  for (int a = 0; a < AM; ++a) {
#pragma unroll
    for (int y = 0; y < AN; ++y) {
      const int j = n0 + wn + 32 * y + li;
      if (j >= N) continue;
      const int mrow = m0 + wm + 32 * a;
      if (S > 1) {
        float* w = ws + (int64_t)blockIdx.z * M * N;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int i = mrow + (e & 3) + 8 * (e >> 2) + 4 * lh;
          if (i < M) w[(int64_t)i * N + j] = acc[a][y][e];
        }
        continue;
      }
      const float bj = ep.bias ? ep.bias[j] : 0.0f;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int i0 = mrow + 8 * g4 + 4 * lh;
        float v4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = i0 + q;
          float v = acc[a][y][4 * g4 + q] + bj;
          if (i < M) {
            if (ep.cf && ep.beta_c != 0.0f) v += ep.beta_c * ep.cf[(int64_t)i * ep.ldc + j];
            if (ep.act == 1) v = fmaxf(v, 0.0f);
            else if (ep.act == 2) v = tanhf(v);
            if (ep.mask_act) {
              const float yv = bf2f(ep.ymask[(int64_t)i * ep.ldy + j]);
              v = (ep.mask_act == 1) ? (yv > 0.0f ? v : 0.0f) : v * (1.0f - yv * yv);
            }
            if (ep.c_last && j == N - 1) ep.c_last[i] = v;
            else if (ep.cf) ep.cf[(int64_t)i * ep.ldc + j] = v;
            if (ep.cb) ep.cb[(int64_t)i * ep.ldc + j] = f2bf(v);
          }
          v4[q] = v;
        }
        if (ep.cbt) {
          uint16_t* d = ep.cbt + (int64_t)j * ep.ldt + i0;
          if (i0 + 3 < M) {
            const uint32_t lo = (uint32_t)f2bf(v4[0]) | ((uint32_t)f2bf(v4[1]) << 16);
            const uint32_t hi = (uint32_t)f2bf(v4[2]) | ((uint32_t)f2bf(v4[3]) << 16);
            *reinterpret_cast<uint2*>(d) = make_uint2(lo, hi);
          } else {
            for (int q = 0; q < 4 && i0 + q < M; ++q) d[q] = f2bf(v4[q]);
          }
        }
      }
    }
  }
}

// split-K partials [S][M][N] -> cf[m][n] (ld ldc) for n < N - 1 (or all n
// when c_last is null) and c_last[m] for n = N - 1; fixed summation order
__global__ __launch_bounds__(256) void splitk_reduce_cols_kernel(const float* __restrict__ W, int S, int M, int N,
                                                                 float* __restrict__ C, int ldc,
                                                                 float* __restrict__ c_last) {
  const int64_t MN = (int64_t)M * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < MN; e += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.0f;
    for (int z = 0; z < S; ++z) v += W[z * MN + e];
    const int i = (int)(e / N), j = (int)(e % N);
    if (c_last && j == N - 1) c_last[i] = v;
    else C[(int64_t)i * ldc + j] = v;
  }
}

// fp32 [R][C] (ld ldx) -> bf16 [R][ldo] (columns >= C zero up to ldo) and/or
// bf16 transposed [C][ldot] (rows >= C untouched, columns >= R untouched).
// 64 x 64 tiles through LDS so both outputs are written row-contiguous.
__global__ __launch_bounds__(256) void cvt_bf16_kernel(const float* __restrict__ X, int ldx, int R, int C,
                                                       uint16_t* __restrict__ out, int ldo,
                                                       uint16_t* __restrict__ outT, int ldot) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int rr = ty; rr < 64; rr += 4) {
    const int r = r0 + rr, c = c0 + tx;
    const float v = (r < R && c < C) ? X[(int64_t)r * ldx + c] : 0.0f;
    tile[rr][tx] = v;
    if (out && r < R && c < ldo) out[(int64_t)r * ldo + c] = f2bf(v);
  }
  if (!outT) return;
  __syncthreads();
  for (int cc = ty; cc < 64; cc += 4) {
    const int c = c0 + cc, r = r0 + tx;
    if (c < C && r < R) outT[(int64_t)c * ldot + r] = f2bf(tile[tx][cc]);
  }
}

// out[n] = sum_b X[n][b] for bf16 rows (bias gradients from dZ^T): one wave per row
__global__ __launch_bounds__(256) void rowsum_bf16_kernel(const uint16_t* __restrict__ X, int ld, int R, int C,
                                                          float* __restrict__ out) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= R) return;
  const uint16_t* x = X + (int64_t)r * ld;
  float s = 0.0f;
  for (int c = lane * 8; c < C; c += 512) {
    if (c + 8 <= C) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + c);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) s += bf2f((uint16_t)(w[q] & 0xFFFF)) + bf2f((uint16_t)(w[q] >> 16));
    } else {
      for (int q = c; q < C; ++q) s += bf2f(x[q]);
    }
  }
  s = wave_sum(s);
  if (lane == 0) out[r] = s;
}

struct CvtJob {
  const float* X;
  uint16_t* out;
  uint16_t* outT;
  int ldx, R, C, ldo, ldot, pad[3];
};
struct CvtJobs {
  CvtJob j[8];
};

// several fp32 -> bf16 (+ transposed) conversions in one launch (blockIdx.z = job):
// the MLP's per-layer weight refresh after every optimizer step
__global__ __launch_bounds__(256) void cvt_bf16_multi_kernel(CvtJobs jobs) {
  const CvtJob& jb = jobs.j[blockIdx.z];
  const int cols = jb.out ? (jb.ldo > jb.C ? jb.ldo : jb.C) : jb.C;
  if ((int)blockIdx.x * 64 >= cols || (int)blockIdx.y * 64 >= jb.R) return;
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int rr = ty; rr < 64; rr += 4) {
    const int r = r0 + rr, c = c0 + tx;
    const float v = (r < jb.R && c < jb.C) ? jb.X[(int64_t)r * jb.ldx + c] : 0.0f;
    tile[rr][tx] = v;
    if (jb.out && r < jb.R && c < jb.ldo) jb.out[(int64_t)r * jb.ldo + c] = f2bf(v);
  }
  if (!jb.outT) return;
  __syncthreads();
  for (int cc = ty; cc < 64; cc += 4) {
    const int c = c0 + cc, r = r0 + tx;
    if (c < jb.C && r < jb.R) jb.outT[(int64_t)c * jb.ldot + r] = f2bf(tile[tx][cc]);
  }
}

// softmax cross-entropy of fp32 logits Z [M][K] -> bf16 dZ [M][ldd] (k < K) and
// bf16 dZ^T [K][ldt]; mean loss accumulated into loss[0]
__global__ __launch_bounds__(256) void softmax_xent_bf16_kernel(const float* __restrict__ Z, const int* __restrict__ y,
                                                                uint16_t* __restrict__ dZ, int ldd,
                                                                uint16_t* __restrict__ dZt, int ldt,
                                                                float* __restrict__ loss, int M, int K) {
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
      const uint16_t g = f2bf((pk - (k == yi ? 1.0f : 0.0f)) / (float)M);
      dZ[(int64_t)i * ldd + k] = g;
      dZt[(int64_t)k * ldt + i] = g;
      if (k == yi) l = -logf(fmaxf(pk, 1e-30f));
    }
  }
  if (loss == nullptr) return;      // training steps that do not report the loss
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) atomicAdd(loss, l / (float)M);
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

// Wave-unit GLM IRLS pass (glm_irls_wave_kernel): p + 2 <= 128, not
// multinomial.  n_units waves of rows_per_unit rows (multiple of 64); slab
// [n_units][pw][pw] fp32 with pw = 16 * ceil((p + 2) / 16); dev_out [n_units].
H2OMX_API int h2omx_glm_irls_wave(const float* X, int64_t ld, int64_t n, const float* y, const float* wprior,
                                  const float* offset, const float* means, const float* beta, const void* params,
                                  int n_units, int64_t rows_per_unit, float* slab, double* dev_out,
                                  hipStream_t stream) {
  const GlmParams P = *reinterpret_cast<const GlmParams*>(params);
  if (P.family == 5 || P.p + 2 > 128 || n_units < 1 || rows_per_unit % GW_RB != 0 ||
      (int64_t)n_units * rows_per_unit < n)
    return kBadArg;
  const int nb = (P.p + 2 + 15) / 16;
  // 16-byte column loads need 16-byte aligned column starts
  const bool vec = (ld % 4 == 0) && (reinterpret_cast<uintptr_t>(X) % 16 == 0);
  const int blocks = cdiv(n_units, 4);
#define GWL(NB, V)                                                                                            \
  hipLaunchKernelGGL((glm_irls_wave_kernel<NB, V>), dim3(blocks), dim3(256), 0, stream, X, ld, n, y, wprior,   \
                     offset, means, beta, P, rows_per_unit, n_units, slab, dev_out)
#define GWL_NB(NB) do { if (vec) GWL(NB, true); else GWL(NB, false); } while (0)
  switch (nb) {
    case 1: GWL_NB(1); break;
    case 2: GWL_NB(2); break;
    case 3: GWL_NB(3); break;
    case 4: GWL_NB(4); break;
    case 5: GWL_NB(5); break;
    case 6: GWL_NB(6); break;
    case 7: GWL_NB(7); break;
    case 8: GWL_NB(8); break;
    default: return kBadArg;
  }
#undef GWL_NB
#undef GWL
  return launch_status();
}

// glm_irls_split_kernel: same contract and slab layout as h2omx_glm_irls_wave
// for an NA-free design (`means` is not read)
H2OMX_API int h2omx_glm_irls_split(const float* X, int64_t ld, int64_t n, const float* y, const float* wprior,
                                   const float* offset, const float* means, const float* beta, const void* params,
                                   int n_units, int64_t rows_per_unit, float* slab, double* dev_out,
                                   hipStream_t stream) {
  (void)means;
  const GlmParams P = *reinterpret_cast<const GlmParams*>(params);
  if (P.family == 5 || P.p < 1 || P.p + 2 > 128 || n_units < 1 || rows_per_unit % GW_RB != 0 ||
      (int64_t)n_units * rows_per_unit < n)
    return kBadArg;
  const int nb = (P.p + 2 + 15) / 16;
  const bool vec = (ld % 4 == 0) && (reinterpret_cast<uintptr_t>(X) % 16 == 0);
  const bool logit = P.family == 1 && P.link == 1;
  const int blocks = cdiv(n_units, 4);
#define GSL(NB, V, F)                                                                                          \
  hipLaunchKernelGGL((glm_irls_split_kernel<NB, V, F, V>), dim3(blocks), dim3(256), 0, stream, X, ld, n, y,      \
                     wprior, offset, beta, P, rows_per_unit, n_units, slab, dev_out)
#define GSL_NB(NB)                      \
  do {                                  \
    if (logit) {                        \
      if (vec) GSL(NB, true, 1);        \
      else GSL(NB, false, 1);           \
    } else {                            \
      if (vec) GSL(NB, true, 0);        \
      else GSL(NB, false, 0);           \
    }                                   \
  } while (0)
  switch (nb) {
    case 1: GSL_NB(1); break;
    case 2: GSL_NB(2); break;
    case 3: GSL_NB(3); break;
    case 4: GSL_NB(4); break;
    case 5: GSL_NB(5); break;
    case 6: GSL_NB(6); break;
    case 7: GSL_NB(7); break;
    case 8: GSL_NB(8); break;
    default: return kBadArg;
  }
#undef GSL_NB
#undef GSL
  return launch_status();
}

__global__ __launch_bounds__(256) void dev_sum_kernel(const double* __restrict__ d, int n, double* __restrict__ out) {
  __shared__ double red[4];
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) a += d[i];   // fixed order per thread
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1]) + (red[2] + red[3]);
}

// GLM pass epilogue: out = [sum of the slabs (pw * pw) | sum of dev (1) |
// SLAB_SPLIT * pw * pw partials]; one contiguous read-back for the host
H2OMX_API int h2omx_slab_reduce16_dev(const float* slab, int n_slabs, int pw, const double* dev, double* out,
                                      hipStream_t stream) {
  const int64_t w = (int64_t)pw * pw;
  double* part = out + w + 1;
  hipLaunchKernelGGL(slab_reduce16_kernel, dim3(cdiv(w, 256), SLAB_SPLIT), dim3(256), 0, stream, slab, n_slabs, pw,
                     part);
  hipLaunchKernelGGL(slab_fold_kernel, dim3(cdiv(w, 256)), dim3(256), 0, stream, part, w, out);
  hipLaunchKernelGGL(dev_sum_kernel, dim3(1), dim3(256), 0, stream, dev, n_slabs, out + w);
  return launch_status();
}

// out: fp64 [(SLAB_SPLIT + 1) * pw * pw] scratch; the sum lands in out[0 : pw * pw]
H2OMX_API int h2omx_slab_reduce16(const float* slab, int n_slabs, int pw, double* out, hipStream_t stream) {
  const int64_t w = (int64_t)pw * pw;
  double* part = out + w;
  hipLaunchKernelGGL(slab_reduce16_kernel, dim3(cdiv(w, 256), SLAB_SPLIT), dim3(256), 0, stream, slab, n_slabs, pw,
                     part);
  hipLaunchKernelGGL(slab_fold_kernel, dim3(cdiv(w, 256)), dim3(256), 0, stream, part, w, out);
  return launch_status();
}

H2OMX_API int h2omx_slab_reduce_upper(const float* slab, int n_slabs, int width, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(cdiv(width, 256)), dim3(256), 0, stream, slab, n_slabs, width, out);
  return launch_status();
}

H2OMX_API int h2omx_slab_sum(const float* slab, int n_slabs, int width, double* out, hipStream_t stream) {
  if (n_slabs >= 64 && width < 64 * 1024)   // narrow and deep: column x slab-group parallel
    hipLaunchKernelGGL(slab_sum_wide_kernel, dim3(cdiv(width, 32)), dim3(1024), 0, stream, slab, n_slabs, width, out);
  else
    hipLaunchKernelGGL(slab_sum_kernel<double>, dim3(cdiv(width, 256)), dim3(256), 0, stream, slab, n_slabs, width,
                       out);
  return launch_status();
}

// fp64 column sums of fp32 slabs rounded into an fp32 vector (few slabs)
H2OMX_API int h2omx_slab_sum_f32(const float* slab, int n_slabs, int width, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(slab_sum_kernel<float>, dim3(cdiv(width, 256)), dim3(256), 0, stream, slab, n_slabs, width, out);
  return launch_status();
}

H2OMX_API int h2omx_glm_wz(const float* E, int64_t m, const float* y, const float* wprior, const float* offset,
                           const float* beta, const void* params, float* sw, float* z, double* dev_part, int n_blk,
                           hipStream_t stream) {
  if (m < 1 || n_blk < 1) return kBadArg;
  const GlmParams P = *reinterpret_cast<const GlmParams*>(params);
  hipLaunchKernelGGL(glm_wz_kernel, dim3(n_blk), dim3(256), 0, stream, E, m, y, wprior, offset, beta, P, sw, z,
                     dev_part);
  return launch_status();
}

// GLM gradient (L_BFGS): R [K][n] residual weights + per-block deviance, then
// the per-split partial gradients out [splits][K][p + 1] (host sums the splits)
H2OMX_API int h2omx_glm_grad(const float* X, int64_t ld, int64_t n, const double* beta, const float* y,
                             const float* wprior, const float* offset, const void* params, float* R, double* dev_part,
                             int n_blk, double* out, int splits, hipStream_t stream) {
  const GlmParams P = *reinterpret_cast<const GlmParams*>(params);
  if (n < 1 || n_blk < 1 || splits < 1 || P.K < 1 || P.K > kGradMaxK || P.p < 0) return kBadArg;
  const size_t lds = sizeof(double) * (size_t)P.K * (P.p + 1);
  if (lds > 64 * 1024) return kBadArg;
  hipLaunchKernelGGL(glm_resid_kernel, dim3(n_blk), dim3(256), lds, stream, X, ld, n, beta, y, wprior, offset, P, R,
                     dev_part);
  hipLaunchKernelGGL(glm_xtr_kernel, dim3(P.p + 1, splits), dim3(256), 0, stream, X, ld, n, P.p, P.K, R, out);
  return launch_status();
}

H2OMX_API int h2omx_glm_grad_max_k() { return kGradMaxK; }

H2OMX_API int h2omx_glm_aug(const float* Xc, int p, int64_t m, const float* means, const float* sw, const float* z,
                            float* A, hipStream_t stream) {
  if (p < 1 || m < 1) return kBadArg;
  hipLaunchKernelGGL(glm_aug_kernel, dim3((unsigned)std::min<int64_t>(cdiv(m, 256), 1024), p + 2), dim3(256), 0,
                     stream, Xc, p, m, means, sw, z, A);
  return launch_status();
}

H2OMX_API int h2omx_kmeans_stage(const float* X, int64_t ldx, int d, int64_t row0, int64_t m, float* Xc,
                                 hipStream_t stream) {
  if (d < 1 || m < 1) return kBadArg;
  hipLaunchKernelGGL(kmeans_stage_kernel, dim3((unsigned)std::min<int64_t>(cdiv(m, 256), 1024), d), dim3(256), 0,
                     stream, X, ldx, d, row0, m, Xc);
  return launch_status();
}

// stat: [n_blk][2k] floats (counts | sse per block); k <= 8192 (LDS)
H2OMX_API int h2omx_kmeans_argmin(const float* G, int k, int64_t m, const float* cn, const float* Xc, int d,
                                  int* assign, float* stat, int n_blk, hipStream_t stream) {
  if (k < 1 || k > 8192 || m < 1 || n_blk < 1) return kBadArg;
  hipLaunchKernelGGL(kmeans_argmin_kernel, dim3(n_blk), dim3(256), (size_t)2 * k * sizeof(float), stream, G, k, m,
                     cn, Xc, d, assign, stat);
  return launch_status();
}

H2OMX_API int h2omx_kmeans_onehot(const int* assign, int k, int64_t m, float* OH, hipStream_t stream) {
  if (k < 1 || k > 65535 || m < 1) return kBadArg;
  hipLaunchKernelGGL(kmeans_onehot_kernel, dim3((unsigned)std::min<int64_t>(cdiv(m, 256), 1024), k), dim3(256), 0,
                     stream, assign, k, m, OH);
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

// tile edge of the fp32 GEMM: 0 = by shape (64 when 128-tiles leave CUs short of work), 64, 128
static int g_gemm_tile = 0;
// (1: 64 x 64 wave tiles on 128 x 128 blocks, 2: ... on 128 x 64 blocks)
H2OMX_API int h2omx_gemm_set_tile(int tile) {
  if (tile != 0 && tile != 64 && tile != 128 && tile != 1 && tile != 2) return kBadArg;
  g_gemm_tile = tile;
  return kOk;
}

static int g_gemm_full = 1;   // FULL fast path of gemm_w64_kernel when the shape allows (A/B switch)
H2OMX_API int h2omx_gemm_set_full(int on) {
  g_gemm_full = on ? 1 : 0;
  return kOk;
}

template <int BM, int BN, int EPI>
static void launch_w64(const float* A, const float* B, float* out, const float* bias, const float* Y, float* bws,
                       int M, int N, int K, int ta, int tb, int act, float beta_c, int splitk, hipStream_t stream) {
  const dim3 grid(cdiv(N, BN), cdiv(M, BM), splitk), blk(GW_T);
  const bool aligned = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0;
  const bool full = g_gemm_full && aligned && M % 4 == 0 && N % 4 == 0 && K % 4 == 0;
#define GW_L(TA_, TB_, F_)                                                                                     \
  hipLaunchKernelGGL((gemm_w64_kernel<TA_, TB_, BM, BN, EPI, F_>), grid, blk, 0, stream, A, B, out, bias, Y, bws, M, \
                     N, K, act, beta_c)
#define GW_T2(F_)                        \
  if (!ta && !tb) GW_L(false, false, F_); \
  else if (!ta && tb) GW_L(false, true, F_); \
  else if (ta && !tb) GW_L(true, false, F_); \
  else GW_L(true, true, F_)
  if (full) { GW_T2(true); } else { GW_T2(false); }
#undef GW_T2
#undef GW_L
}

// M, N, K % 4 == 0, aligned operands: gemm_w64_kernel's FULL pipeline
static bool w64_full_ok(const float* A, const float* B, int M, int N, int K, int splitk) {
  (void)splitk;
  // partial edge tiles are fine (masked loads, checked epilogue) but a grid of
  // mostly-empty tiles is not: whole 128 x 64 rows / columns of work or more
  return g_gemm_full && ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0 &&
         M % 4 == 0 && N % 4 == 0 && K % 4 == 0 && M >= 128 && N >= 64;
}

static void launch_gemm(const float* A, const float* B, float* out, const float* bias, int M, int N, int K, int ta,
                        int tb, int act, float beta_c, int splitk, hipStream_t stream) {
  // default: the FULL 64 x 64-wave-tile pipeline on 128 x 64 blocks whenever the shape
  // allows it (8192 x 512 x 512: 50 vs 59 us for gemm64_kernel; same fmaf chain per
  // element, so bit-identical results)
  if (g_gemm_tile == 0 && w64_full_ok(A, B, M, N, K, splitk)) {
    launch_w64<128, 64, 0>(A, B, out, bias, nullptr, nullptr, M, N, K, ta, tb, act, beta_c, splitk, stream);
    return;
  }
  if (g_gemm_tile == 1 || g_gemm_tile == 2) {
    if (g_gemm_tile == 1) launch_w64<128, 128, 0>(A, B, out, bias, nullptr, nullptr, M, N, K, ta, tb, act, beta_c, splitk, stream);
    else launch_w64<128, 64, 0>(A, B, out, bias, nullptr, nullptr, M, N, K, ta, tb, act, beta_c, splitk, stream);
    return;
  }
  const int64_t tiles128 = (int64_t)cdiv(N, GB) * cdiv(M, GB) * splitk;
  const bool t64 = g_gemm_tile == 64 || (g_gemm_tile == 0 && tiles128 < 512);
  if (t64) {
    const dim3 grid(cdiv(N, G64), cdiv(M, G64), splitk), blk(G64T);
    if (!ta && !tb) hipLaunchKernelGGL((gemm64_kernel<false, false>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
    else if (!ta && tb) hipLaunchKernelGGL((gemm64_kernel<false, true>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
    else if (ta && !tb) hipLaunchKernelGGL((gemm64_kernel<true, false>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
    else hipLaunchKernelGGL((gemm64_kernel<true, true>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
    return;
  }
  const dim3 grid(cdiv(N, GB), cdiv(M, GB), splitk);
  const dim3 blk(GTHREADS);
  if (!ta && !tb) hipLaunchKernelGGL((gemm_kernel<false, false>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
  else if (!ta && tb) hipLaunchKernelGGL((gemm_kernel<false, true>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
  else if (ta && !tb) hipLaunchKernelGGL((gemm_kernel<true, false>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
  else hipLaunchKernelGGL((gemm_kernel<true, true>), grid, blk, 0, stream, A, B, out, bias, M, N, K, act, beta_c);
}

H2OMX_API int h2omx_gemm(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int ta,
                         int tb, int act, float beta_c, int splitk, float* ws, hipStream_t stream) {
  if (splitk < 1 || (splitk > 1 && !ws)) return kBadArg;
  float* out = splitk > 1 ? ws : C;
  launch_gemm(A, B, out, bias, M, N, K, ta, tb, act, beta_c, splitk, stream);
  if (splitk > 1)
    hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(cdiv((int64_t)M * N, 256) < 4096 ? cdiv((int64_t)M * N, 256) : 4096),
                       dim3(256), 0, stream, ws, splitk, M, N, C, bias, act, beta_c);
  return launch_status();
}

// back-propagation through an activation: C[M][N] = (A[M][K] B[K][N]) * act'(Y),
// Y = the activation's output [M][N]; bws[cdiv(M, bm)][N] receives the column sums
// of C per bm-row block (bias-gradient partials).  Returns the block count via
// *splits.  tile: 1 = 128 x 128 blocks, 2 = 128 x 64.
H2OMX_API int h2omx_gemm_dact(const float* A, const float* B, float* C, const float* Y, float* bws, int M, int N,
                              int K, int act, int tile, int* splits, hipStream_t stream) {
  if (!A || !B || !C || !Y || !bws || M < 1 || N < 1 || K < 1 || (tile != 1 && tile != 2)) return kBadArg;
  if (tile == 1) launch_w64<128, 128, 1>(A, B, C, nullptr, Y, bws, M, N, K, 0, 0, act, 0.0f, 1, stream);
  else launch_w64<128, 64, 1>(A, B, C, nullptr, Y, bws, M, N, K, 0, 0, act, 0.0f, 1, stream);
  if (splits) *splits = cdiv(M, 128);
  return launch_status();
}

H2OMX_API int h2omx_gemm_skinny_nt(const float* A, const float* B, float* C, const float* bias, int M, int N, int K,
                                   int act, hipStream_t stream) {
  if (N < 1 || N > SKINNY_N) return kBadArg;
  const int blocks = std::min(cdiv(M, 4), 4096);
  hipLaunchKernelGGL(gemm_skinny_nt_kernel, dim3(blocks), dim3(256), 0, stream, A, B, C, bias, M, N, K, act);
  return launch_status();
}

// output layer + softmax cross-entropy gradient in one launch (act none):
// Z = A B^T + bias [M][N], dZ = (softmax(Z) - onehot(y)) / M
H2OMX_API int h2omx_gemm_skinny_softmax(const float* A, const float* B, float* C, const float* bias, int M, int N,
                                        int K, const int* y, float* dZ, hipStream_t stream) {
  if (N < 1 || N > SKINNY_N || !y || !dZ) return kBadArg;
  const int blocks = std::min(cdiv(M, 4), 4096);
  hipLaunchKernelGGL(gemm_skinny_nt_kernel, dim3(blocks), dim3(256), 0, stream, A, B, C, bias, M, N, K, 0, y, dZ);
  return launch_status();
}

H2OMX_API int h2omx_gemm_thin_k(const float* A, const float* B, float* C, int64_t M, int N, int K, const float* act_y,
                                int act, hipStream_t stream) {
  if (K < 1 || K > 8) return kBadArg;
  const int64_t blocks = std::min<int64_t>(cdiv(M * N, 256), 8192);
  hipLaunchKernelGGL(gemm_thin_k_kernel, dim3(blocks), dim3(256), 0, stream, A, B, C, M, N, K, act_y, act);
  return launch_status();
}

// output-layer weight gradient (C <= 8 classes): out[C * N + C] = [dW (dZ^T H) | db
// (column sums of dZ)] - the layer's contiguous gradient span.  ws >= splits * (C * N + C).
H2OMX_API int h2omx_out_wgrad(const float* dZ, const float* H, float* out, float* ws, int M, int N, int C,
                              int splits, hipStream_t stream) {
  if (C < 1 || C > OUT_C || N % 4 || splits < 1 || !ws || (reinterpret_cast<uintptr_t>(H) & 15)) return kBadArg;
  const dim3 grid(cdiv(N, 256), splits);
#define OW_L(C_) hipLaunchKernelGGL(out_wgrad_kernel<C_>, grid, dim3(256), 0, stream, dZ, H, ws, M, N)
  switch (C) {
    case 1: OW_L(1); break;
    case 2: OW_L(2); break;
    case 3: OW_L(3); break;
    case 4: OW_L(4); break;
    case 5: OW_L(5); break;
    case 6: OW_L(6); break;
    case 7: OW_L(7); break;
    default: OW_L(8); break;
  }
#undef OW_L
  // fold: only the reducer's second job (64 columns x 4 slice phases per block, two
  // loads in flight) - its per-element serial loop would chain `splits` loads
  const int T = C * N + C;
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(cdiv(T, 64)), dim3(256), 0, stream, ws, splits, 0, 0, out,
                     nullptr, 0, 0.0f, 0, ws, splits, T, out);
  return launch_status();
}

// dZ_prev = (dZ [M][C] W [C][N]) * act'(Y), column partial sums -> ws[splits][N]
H2OMX_API int h2omx_out_backward(const float* dZ, const float* H, const float* W, float* out, float* wsw, float* wsb,
                                 int M, int N, int C, int splits, int act, hipStream_t stream) {
  if (C < 1 || C > OUT_C || N % 4 || splits < 1 || !wsw || !wsb ||
      ((reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(H) | reinterpret_cast<uintptr_t>(out) |
        reinterpret_cast<uintptr_t>(wsb)) & 15))
    return kBadArg;
  const dim3 grid(cdiv(N, 256), splits);
#define OB_L(C_) \
  hipLaunchKernelGGL(out_backward_kernel<C_>, grid, dim3(256), 0, stream, dZ, H, W, out, wsw, wsb, M, N, act)
  switch (C) {
    case 1: OB_L(1); break;
    case 2: OB_L(2); break;
    case 3: OB_L(3); break;
    case 4: OB_L(4); break;
    case 5: OB_L(5); break;
    case 6: OB_L(6); break;
    case 7: OB_L(7); break;
    default: OB_L(8); break;
  }
#undef OB_L
  return launch_status();
}

H2OMX_API int h2omx_thin_dact(const float* dZ, const float* W, const float* Y, float* out, float* ws, int M, int N,
                              int C, int splits, int act, hipStream_t stream) {
  if (C < 1 || C > OUT_C || N % 4 || splits < 1 || !ws ||
      ((reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(Y) | reinterpret_cast<uintptr_t>(out) |
        reinterpret_cast<uintptr_t>(ws)) & 15))
    return kBadArg;
  const dim3 grid(cdiv(N, 256), splits);
#define TD_L(C_) hipLaunchKernelGGL(thin_dact_kernel<C_>, grid, dim3(256), 0, stream, dZ, W, Y, out, ws, M, N, act)
  switch (C) {
    case 1: TD_L(1); break;
    case 2: TD_L(2); break;
    case 3: TD_L(3); break;
    case 4: TD_L(4); break;
    case 5: TD_L(5); break;
    case 6: TD_L(6); break;
    case 7: TD_L(7); break;
    default: TD_L(8); break;
  }
#undef TD_L
  return launch_status();
}

H2OMX_API int h2omx_act_backward_bias(const float* Y, float* dY, float* ws, int M, int N, int splits, int act,
                                      hipStream_t stream) {
  if (splits < 1 || !ws || N % 4 || (reinterpret_cast<uintptr_t>(Y) & 15) || (reinterpret_cast<uintptr_t>(dY) & 15) ||
      (reinterpret_cast<uintptr_t>(ws) & 15))
    return kBadArg;
  hipLaunchKernelGGL(act_backward_bias_kernel, dim3(cdiv(N, 256), splits), dim3(256), 0, stream, Y, dY, ws, M, N, act);
  return launch_status();
}

// weight-gradient GEMM (split-K) whose reduce launch also sums a bias-gradient workspace
H2OMX_API int h2omx_gemm_wgrad_bias(const float* A, const float* B, float* C, int M, int N, int K, int splitk,
                                    float* ws, const float* bws, int bsplits, int bn, float* db, hipStream_t stream) {
  if (splitk < 2 || !ws || !bws || !db) return kBadArg;
  launch_gemm(A, B, ws, nullptr, M, N, K, 1, 0, 0, 0.0f, splitk, stream);
  const int mb = cdiv((int64_t)M * N, 256) < 4096 ? (int)cdiv((int64_t)M * N, 256) : 4096;
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(mb + cdiv(bn, 64)), dim3(256), 0, stream, ws, splitk, M, N, C,
                     nullptr, 0, 0.0f, mb, bws, bsplits, bn, db);
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

H2OMX_API int h2omx_adadelta_fix(float* W, float* G, float* Eg2, float* Edx2, int64_t n, float rho, float eps,
                                 float l2, const void* fixes, hipStream_t stream) {
  const GradFixes fx = *reinterpret_cast<const GradFixes*>(fixes);
  if (fx.n < 0 || fx.n > MAX_GRAD_FIX) return kBadArg;
  hipLaunchKernelGGL(adadelta_fix_kernel, dim3(cdiv(n, 256)), dim3(256), 0, stream, W, G, Eg2, Edx2, n, rho, eps, l2,
                     fx);
  return launch_status();
}

// out_wgrad without its fold: the S partial rows [S][C * N + C] stay in ws
// (folded later, e.g. by adadelta_fix_kernel)
H2OMX_API int h2omx_out_wgrad_partial(const float* dZ, const float* H, float* ws, int M, int N, int C, int splits,
                                      hipStream_t stream) {
  if (C < 1 || C > OUT_C || N % 4 || splits < 1 || !ws || (reinterpret_cast<uintptr_t>(H) & 15)) return kBadArg;
  const dim3 grid(cdiv(N, 256), splits);
#define OW_L(C_) hipLaunchKernelGGL(out_wgrad_kernel<C_>, grid, dim3(256), 0, stream, dZ, H, ws, M, N)
  switch (C) {
    case 1: OW_L(1); break;
    case 2: OW_L(2); break;
    case 3: OW_L(3); break;
    case 4: OW_L(4); break;
    case 5: OW_L(5); break;
    case 6: OW_L(6); break;
    case 7: OW_L(7); break;
    default: OW_L(8); break;
  }
#undef OW_L
  return launch_status();
}

H2OMX_API int h2omx_sgd_momentum(float* W, const float* G, float* V, int64_t n, float lr, float mom, float l2,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3(cdiv(n, 256)), dim3(256), 0, stream, W, G, V, n, lr, mom, l2);
  return launch_status();
}

H2OMX_API int h2omx_gemm_bf16(const uint16_t* A, int lda, const uint16_t* B, int ldb, int M, int N, int K,
                              const float* bias, int act, const uint16_t* ymask, int ldy, int mask_act, float* cf,
                              uint16_t* cb, int ldc, uint16_t* cbt, int ldt, float beta_c, int splitk, float* ws,
                              float* c_last, hipStream_t stream) {
  if (K % 8 || lda % 8 || ldb % 8 || M < 1 || N < 1 || K < 8 || splitk < 1) return kBadArg;
  if ((reinterpret_cast<uintptr_t>(A) & 15) || (reinterpret_cast<uintptr_t>(B) & 15)) return kBadArg;
  if (cbt && ((ldt & 3) || (reinterpret_cast<uintptr_t>(cbt) & 7))) return kBadArg;
  if (mask_act && !ymask) return kBadArg;
  if (splitk > 1 && (!ws || !cf || cb || cbt || mask_act)) return kBadArg;  // split-K: fp32 out only
  if (c_last && (bias || act || beta_c != 0.0f || cb || cbt || mask_act)) return kBadArg;
  BfEpi ep{bias, ymask, cf, cb, cbt, c_last, ldy, ldc, ldt, act, mask_act, beta_c};
  // 128 x 128 blocks of eight 32 x 64 wave tiles (two waves per SIMD hide each
  // other's LDS / global latency: measured fastest, scripts/gemm_bf16_micro.py);
  // 128 x 64 blocks of four where the output has at most one 64-column block.
  // Variant 0 (four 64 x 64 wave tiles) is kept for A/B runs.
  const int variant = g_bf16_variant >= 0 ? g_bf16_variant : (N <= 64 ? 1 : 2);
  if (variant == 1) {
    const dim3 grid(cdiv(N, 64), cdiv(M, HB), splitk);
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 64, 32, 64>), grid, dim3(256), 0, stream, A, lda, B, ldb, M, N, K, ws,
                       ep);
  } else if (variant == 2) {
    const dim3 grid(cdiv(N, HB), cdiv(M, HB), splitk);
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 128, 32, 64>), grid, dim3(512), 0, stream, A, lda, B, ldb, M, N, K,
                       ws, ep);
  } else {
    const dim3 grid(cdiv(N, HB), cdiv(M, HB), splitk);
    hipLaunchKernelGGL((gemm_bf16_nt_kernel<128, 128, 64, 64>), grid, dim3(256), 0, stream, A, lda, B, ldb, M, N, K,
                       ws, ep);
  }
  if (splitk > 1) {
    const int64_t mn = (int64_t)M * N;
    const int g = cdiv(mn, 256) < 4096 ? cdiv(mn, 256) : 4096;
    if (bias || act || beta_c != 0.0f) {
      if (ldc != N || c_last) return kBadArg;
      hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3(g), dim3(256), 0, stream, ws, splitk, M, N, cf, bias, act,
                         beta_c);
    } else {
      hipLaunchKernelGGL(splitk_reduce_cols_kernel, dim3(g), dim3(256), 0, stream, ws, splitk, M, N, cf, ldc, c_last);
    }
  }
  return launch_status();
}

H2OMX_API int h2omx_cvt_bf16(const float* X, int ldx, int R, int C, uint16_t* out, int ldo, uint16_t* outT, int ldot,
                             hipStream_t stream) {
  if (R < 1 || C < 1) return kOk;
  hipLaunchKernelGGL(cvt_bf16_kernel, dim3(cdiv(out ? (ldo > C ? ldo : C) : C, 64), cdiv(R, 64)), dim3(256), 0,
                     stream, X, ldx, R, C, out, ldo, outT, ldot);
  return launch_status();
}

H2OMX_API int h2omx_rowsum_bf16(const uint16_t* X, int ld, int R, int C, float* out, hipStream_t stream) {
  if (ld % 8 || (reinterpret_cast<uintptr_t>(X) & 15)) return kBadArg;
  hipLaunchKernelGGL(rowsum_bf16_kernel, dim3(cdiv(R, 4)), dim3(256), 0, stream, X, ld, R, C, out);
  return launch_status();
}

H2OMX_API int h2omx_cvt_bf16_multi(const void* jobs, int n_jobs, int max_rows, int max_cols, hipStream_t stream) {
  if (n_jobs < 1 || n_jobs > 8) return kBadArg;
  CvtJobs J{};
  const CvtJob* src = reinterpret_cast<const CvtJob*>(jobs);
  for (int k = 0; k < n_jobs; ++k) J.j[k] = src[k];
  hipLaunchKernelGGL(cvt_bf16_multi_kernel, dim3(cdiv(max_cols, 64), cdiv(max_rows, 64), n_jobs), dim3(256), 0, stream,
                     J);
  return launch_status();
}

H2OMX_API int h2omx_softmax_xent_bf16(const float* Z, const int* y, uint16_t* dZ, int ldd, uint16_t* dZt, int ldt,
                                      float* loss, int M, int K, hipStream_t stream) {
  hipLaunchKernelGGL(softmax_xent_bf16_kernel, dim3(cdiv(M, 256)), dim3(256), 0, stream, Z, y, dZ, ldd, dZt, ldt, loss,
                     M, K);
  return launch_status();
}

H2OMX_API int h2omx_gemm_bf16_variant(int v) {
  g_bf16_variant = v;
  return kOk;
}
