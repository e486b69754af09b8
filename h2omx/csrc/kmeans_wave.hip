// K-Means Lloyd pass (K12 + K13 of SURVEY.md §2.5), wave-unit kernel.  Part
// of libh2omx_dense (dense_kernels.hip holds the workgroup-tile kernel used
// for k > 32 and the GEMM path for d > 128).  Replaces H2O-3's K-Means
// (deployed by the reference, isgasho/h2o-kubernetes templates.rs:28-30).
#include "common.h"

#include <math.h>

// ---------------------------------------------------------------------------
// K-Means Lloyd pass, wave-unit form (d <= 128 with k <= 16, d <= 64 with
// k <= 32).  Every wave runs independently on 64-row chunks (one row per
// lane), no workgroup barriers:
//   * feature f of the chunk arrives as one coalesced 256-B load per wave
//     into x[f]; the registers are parked in the wave's LDS tile [f][65]
//     and immediately reloaded with the wave's NEXT chunk, so the HBM stream
//     stays in flight during all of the chunk's arithmetic;
//   * distances dot(x, c) for all clusters on the VALU as packed fp32 FMAs
//     (v_pk_fma_f32, two clusters per instruction); the centroids are
//     wave-uniform, so one feature's KP values come through the scalar cache
//     (transposed copy CTg [DP][KP], s_load) straight into the FMA's SGPR
//     operand - no LDS traffic for them (an LDS broadcast copy measured
//     LDS-bound); ||c||^2 - 2 dot -> argmin (lowest
//     index on ties);
//   * the tile is read conflict-free both ways: lane = row for the distances,
//     and the cluster sums run transposed: lane = feature, rows
//     of cluster c walked from the ballot of the assignment, so S[c][f]
//     accumulates in registers (no atomics, no barriers); counts are
//     popcounts, the row SSE is picked up with v_readlane.
// Per-wave slabs [k][d] sums | k counts | k SSE, reduced in fp64 by slab_sum.
// ---------------------------------------------------------------------------
constexpr int KW_LD = 65;
typedef float f32x2 __attribute__((ext_vector_type(2)));

// LDS written by some lanes of a wave, read by other lanes of the same wave
__device__ __forceinline__ void kw_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int DP, int KP>
__global__ __launch_bounds__(256) void kmeans_wave_kernel(const float* __restrict__ X, int64_t ld, int64_t n, int d,
                                                          const float* __restrict__ Cp, const float* __restrict__ CTg,
                                                          const float* __restrict__ cnp,
                                                          int k, int* __restrict__ assign, float* __restrict__ slab) {
  constexpr int DH = (DP + 63) / 64;
  extern __shared__ float kw_lds[];
  // wave index made explicitly uniform: the chunk loop is then scalar control flow
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* Xs = kw_lds + wid * DP * KW_LD;
  const int64_t nch = (n + 63) / 64;
  const int64_t W = (int64_t)gridDim.x * 4;
  int64_t ch = (int64_t)blockIdx.x * 4 + wid;
  float S[DH][KP], E[KP];
  int cnt[KP];
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    E[c] = 0.f;
    cnt[c] = 0;
#pragma unroll
    for (int h = 0; h < DH; ++h) S[h][c] = 0.f;
  }
  float x[DP];
  // per-lane 32-bit row offsets from a wave-uniform column offset that steps
  // by ld (global_load saddr form: no 64-bit per-lane address per feature)
  if (ch < nch) {
    const uint32_t ro = (uint32_t)min(ch * 64 + lane, n - 1);
    int64_t co = 0;
#pragma unroll
    for (int f = 0; f < DP; ++f) {
      x[f] = (f < d) ? X[co + ro] : 0.f;
      co += ld;
      asm volatile("" : "+s"(co));   // no DP precomputed column addresses held in SGPRs
    }
  }
  while (ch < nch) {
    const int64_t r = ch * 64 + lane;
    const bool valid = r < n;
    const int64_t nx = ch + W;
    const bool more = nx < nch;
    const uint32_t rn = more ? (uint32_t)min(nx * 64 + lane, n - 1) : 0u;
    // (a) the chunk (in registers) into the wave's LDS tile, NA -> 0
#pragma unroll
    for (int f = 0; f < DP; ++f) {
      const float v = x[f];
      Xs[f * KW_LD + lane] = (v != v) ? 0.f : v;   // NA -> mean (0 in standardized space)
    }
    // (b) the NEXT chunk's loads go out now: in flight during (c) and (d)
    // (scheduling fence: hoisting them above (a) would need a second DP registers)
    __builtin_amdgcn_sched_barrier(0);
    {
      int64_t co = 0;
      int dl = more ? d : 0;
      asm volatile("" : "+s"(dl));   // per-iteration: DP hoisted f < d masks would fill the SGPRs
#pragma unroll
      for (int f = 0; f < DP; ++f) {
        // every x[f] is redefined here (never kept from the previous chunk), so
        // the old values die in (a) and the loads reuse their registers
        float v = 0.f;
        if (f < dl) v = X[co + rn];
        x[f] = v;
        co += ld;
        asm volatile("" : "+s"(co));
      }
    }
    kw_wave_sync();
    // (c) distances from the tile (lane = row) and the broadcast centroids
    f32x2 acc2[KP / 2];   // cluster pairs: packed fp32 FMAs (v_pk_fma_f32)
#pragma unroll
    for (int c = 0; c < KP / 2; ++c) acc2[c] = f32x2{0.f, 0.f};
    float x2 = 0.f;
#pragma unroll
    for (int f = 0; f < DP; ++f) {
      // opaque per feature: the loop-invariant centroid reads stay here instead
      // of being hoisted out of the chunk loop (DP x KP values would spill)
      int co = f * KP;
      asm volatile("" : "+s"(co));
      const float v = Xs[f * KW_LD + lane];
      x2 = fmaf(v, v, x2);
#pragma unroll
      for (int c4 = 0; c4 < KP / 4; ++c4) {
        const float4 cv = *reinterpret_cast<const float4*>(CTg + co + 4 * c4);   // scalar-cache read
        const f32x2 vv{v, v};
        acc2[2 * c4] = __builtin_elementwise_fma(vv, f32x2{cv.x, cv.y}, acc2[2 * c4]);
        acc2[2 * c4 + 1] = __builtin_elementwise_fma(vv, f32x2{cv.z, cv.w}, acc2[2 * c4 + 1]);
      }
    }
    float best = INFINITY;
    int bi = 0;
#pragma unroll
    for (int c = 0; c < KP; ++c) {
      const float dist = cnp[c] - 2.0f * acc2[c / 2][c % 2];
      if (dist < best) { best = dist; bi = c; }
    }
    const float sse = fmaxf(best + x2, 0.f);
    if (valid) assign[r] = bi;
    const int fl0 = lane, fl1 = min(lane + 64, DP - 1);
#pragma unroll
    for (int c = 0; c < KP; ++c) {
      if (c < k) {
        unsigned long long m = __ballot(valid && bi == c);
        cnt[c] += __popcll(m);
        float s0 = 0.f, s1 = 0.f, e = 0.f;
        while (m) {
          const int rr = __ffsll((long long)m) - 1;
          m &= m - 1ull;
          s0 += Xs[fl0 * KW_LD + rr];
          if (DH > 1) s1 += Xs[fl1 * KW_LD + rr];
          e += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sse), rr));
        }
        S[0][c] += s0;
        if (DH > 1) S[DH - 1][c] += s1;
        E[c] += e;
      }
    }
    kw_wave_sync();   // the tile is read before the next chunk overwrites it
    ch = nx;
  }
  const int gw = blockIdx.x * 4 + wid;
  float* out = slab + (int64_t)gw * (k * d + 2 * k);
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    if (c < k) {
      if (lane < d) out[c * d + lane] = S[0][c];
      if (DH > 1 && lane + 64 < d) out[c * d + 64 + lane] = S[DH - 1][c];
      if (lane == 0) {
        out[k * d + c] = (float)cnt[c];
        out[k * d + k + c] = E[c];
      }
    }
  }
}


// ---------------------------------------------------------------------------
// K-Means Lloyd pass, wave-unit form with the cluster sums on the matrix cores
// (kmeans_mfma_kernel; d + 2 <= 128, k <= 32).
//
// kmeans_wave_kernel above parks every 64-row chunk in a per-wave LDS tile
// [DP][65] (29 KB at d = 100: one wave per SIMD) and walks the rows of each
// cluster one at a time (a dependent LDS read per row).  Here:
//   * distances straight from the load registers (lane = row), centroids
//     through the scalar cache as above; no full-tile LDS round trip;
//   * the cluster sums are the GEMM S[c][f] += sum_r onehot[r][c] x[r][f] on
//     v_mfma_f32_16x16x4_f32 (exact fp32 products, a k-ordered fmaf chain):
//     A = onehot (i = cluster, k = row), B = x (k = row, j = feature).  Step s
//     of 16 takes rows 16 (lane / 16) + s: the onehot column comes from the
//     row's lane by one ds_bpermute per step, and each 16-feature block of the
//     chunk is transposed through a 16 x 68 LDS buffer (16 ds_write_b32, 4
//     ds_read_b128 per lane, double-buffered) - 8.7 KB per wave, so LDS no
//     longer limits occupancy (2 waves per SIMD: one wave's loads and matrix
//     work overlap the other's VALU distances);
//   * the counts and the per-cluster SSE are two more B columns (x[d] = 1,
//     x[d + 1] = the row's squared distance), so the same MFMAs produce them.
// Slab layout per wave as kmeans_wave_kernel: [k][d] sums | k counts | k SSE.
// ---------------------------------------------------------------------------
typedef float f32x4_k __attribute__((ext_vector_type(4)));
constexpr int KM_LDP = 68;   // LDS row pitch (floats): conflict-free ds_read_b128 of 16 feature rows

template <int NT, int KD, bool NA>
__global__ __launch_bounds__(256, 2) void kmeans_mfma_kernel(const float* __restrict__ X, int64_t ld, int64_t n, int d,
                                                            const float* __restrict__ CT2,
                                                            const float* __restrict__ cnp, int k,
                                                            int* __restrict__ assign, float* __restrict__ slab) {
  constexpr int DP = NT * 16;            // x registers: d features, count column, SSE column, zero padding
  constexpr int KG = (KD + 15) / 16;     // 16-cluster groups of the MFMA i dimension
  __shared__ float kbuf[4][2][16 * KM_LDP];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* buf0 = &kbuf[wid][0][0];
  float* buf1 = &kbuf[wid][1][0];
  const int64_t nch = (n + 63) / 64;
  const int64_t W = (int64_t)gridDim.x * 4;
  // d >= 16 NT - 17 (NT = ceil((d + 2) / 16)): features below F0 are always data
  constexpr int F0 = DP - 17 > 0 ? DP - 17 : 0;
  f32x4_k acc[KG][NT];
#pragma unroll
  for (int g = 0; g < KG; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[g][t] = f32x4_k{0.f, 0.f, 0.f, 0.f};
  const int kq = lane >> 4, jl = lane & 15;

  for (int64_t ch = (int64_t)blockIdx.x * 4 + wid; ch < nch; ch += W) {
    const int64_t r = ch * 64 + lane;
    const bool valid = r < n;
    const uint32_t ro = (uint32_t)min(r, n - 1);
    // feature pairs: (x[2 i], x[2 i + 1]) is one 64-bit register pair, the
    // operand of the packed distance FMAs below
    f32x2 xx[DP / 2];
    {
      int64_t co = 0;
#pragma unroll
      for (int f = 0; f < DP; ++f) {
        float v = 0.f;
        if (f < F0 || f < d) v = X[co + ro];
        if (NA && v != v) v = 0.f;   // NA -> mean (0 in standardized space)
        xx[f / 2][f % 2] = v;
        co += ld;
        asm volatile("" : "+s"(co));
      }
    }
    // distances: per cluster an (even, odd) feature partial pair, packed fp32
    // FMAs whose centroid operand is an SGPR pair from CT2 [DP / 2][KD][2]
    // (scalar-cache reads; the two halves are summed after the loop)
    f32x2 accp[KD];
#pragma unroll
    for (int c = 0; c < KD; ++c) accp[c] = f32x2{0.f, 0.f};
    f32x2 x2p{0.f, 0.f};
#pragma unroll
    for (int f2 = 0; f2 < DP / 2; ++f2) {
      if (2 * f2 < F0 || 2 * f2 < d) {   // wave-uniform: the padded features cost nothing
        int co = f2 * 2 * KD;
        asm volatile("" : "+s"(co));
        const f32x2 xv = xx[f2];
        x2p = __builtin_elementwise_fma(xv, xv, x2p);
#pragma unroll
        for (int c2 = 0; c2 < KD / 2; ++c2) {
          const float4 cv = *reinterpret_cast<const float4*>(CT2 + co + 4 * c2);   // clusters 2 c2, 2 c2 + 1
          accp[2 * c2] = __builtin_elementwise_fma(xv, f32x2{cv.x, cv.y}, accp[2 * c2]);
          accp[2 * c2 + 1] = __builtin_elementwise_fma(xv, f32x2{cv.z, cv.w}, accp[2 * c2 + 1]);
        }
      }
    }
    const float x2 = x2p.x + x2p.y;
    float best = INFINITY;
    int bi = 0;
#pragma unroll
    for (int c = 0; c < KD; ++c) {
      const float dist = cnp[c] - 2.0f * (accp[c].x + accp[c].y);
      if (dist < best) { best = dist; bi = c; }
    }
    if (valid) assign[r] = bi;
    bi = valid ? bi : -1;                  // rows past n join no cluster
    // count and SSE columns (d and d + 1 < DP by the launcher's NT)
#pragma unroll
    for (int f = F0; f < DP; ++f) {
      if (f == d) xx[f / 2][f % 2] = 1.0f;
      if (f == d + 1) xx[f / 2][f % 2] = fmaxf(best + x2, 0.f);
    }
    // A operands: step s covers rows 16 kq + s; lane (kq, jl) holds onehot[row][16 g + jl]
    float a[KG][16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int bs = __shfl(bi, (lane & 48) + s, kWave);
#pragma unroll
      for (int g = 0; g < KG; ++g) a[g][s] = (bs == 16 * g + jl) ? 1.0f : 0.0f;
    }
    // B operands: block t of 16 features transposed through the wave's LDS buffer
#pragma unroll
    for (int j = 0; j < 16; ++j) buf0[j * KM_LDP + lane] = xx[j / 2][j % 2];
    kw_wave_sync();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float* cur = (t & 1) ? buf1 : buf0;
      float* nxt = (t & 1) ? buf0 : buf1;
      float b[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(cur + jl * KM_LDP + 16 * kq + 4 * q);
        b[4 * q] = v.x; b[4 * q + 1] = v.y; b[4 * q + 2] = v.z; b[4 * q + 3] = v.w;
      }
      if (t + 1 < NT) {
#pragma unroll
        for (int j = 0; j < 16; ++j) nxt[j * KM_LDP + lane] = xx[8 * (t + 1) + j / 2][j % 2];
      }
      kw_wave_sync();   // this block's reads and the next block's writes are done
#pragma unroll
      for (int s = 0; s < 16; ++s)
#pragma unroll
        for (int g = 0; g < KG; ++g) acc[g][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[g][s], b[s], acc[g][t], 0, 0, 0);
    }
  }
  // D layout: lane holds D[i = 4 kq + v][j = jl] -> cluster 16 g + 4 kq + v, feature 16 t + jl
  const int gw = blockIdx.x * 4 + wid;
  float* out = slab + (int64_t)gw * (k * d + 2 * k);
#pragma unroll
  for (int g = 0; g < KG; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int c = 16 * g + 4 * kq + v, f = 16 * t + jl;
        if (c < k) {
          if (f < d) out[c * d + f] = acc[g][t][v];
          else if (f == d) out[k * d + c] = acc[g][t][v];
          else if (f == d + 1) out[k * d + k + c] = acc[g][t][v];
        }
      }
}

// MFMA-sum Lloyd pass: CT2 [8 * nt][kd][2] zero-padded centroids by feature pair,
// cnp [kd] (+inf padding); nt = ceil((d + 2) / 16); n_wg workgroups of 4 waves,
// slab holds 4 * n_wg per-wave slabs; na = 0 asserts an NA-free design
H2OMX_API int h2omx_kmeans_mfma(const float* X, int64_t ld, int64_t n, int d, const float* CT2, const float* cnp,
                                int k, int kd, int nt, int na, int n_wg, int* assign, float* slab,
                                hipStream_t stream) {
  if (n_wg < 1 || n < 1 || d < 1 || k < 1 || k > kd || kd % 4 != 0 || nt != (d + 2 + 15) / 16) return kBadArg;
#define KMM(NT, KD)                                                                                          \
  if (nt == NT && kd == KD) {                                                                                \
    if (na)                                                                                                  \
      hipLaunchKernelGGL((kmeans_mfma_kernel<NT, KD, true>), dim3(n_wg), dim3(256), 0, stream, X, ld, n, d,   \
                         CT2, cnp, k, assign, slab);                                                         \
    else                                                                                                     \
      hipLaunchKernelGGL((kmeans_mfma_kernel<NT, KD, false>), dim3(n_wg), dim3(256), 0, stream, X, ld, n, d,  \
                         CT2, cnp, k, assign, slab);                                                         \
    return launch_status();                                                                                  \
  }
#define KMM_NT(NT) KMM(NT, 4) KMM(NT, 8) KMM(NT, 12) KMM(NT, 16)
  KMM_NT(1) KMM_NT(2) KMM_NT(3) KMM_NT(4) KMM_NT(5) KMM_NT(6) KMM_NT(7) KMM_NT(8)
  KMM(1, 24) KMM(2, 24) KMM(3, 24) KMM(4, 24) KMM(1, 32) KMM(2, 32) KMM(3, 32) KMM(4, 32)
#undef KMM_NT
#undef KMM
  return kBadArg;
}

// wave-unit Lloyd pass: Cp [KP][DP] zero-padded centroids, cnp [KP] (+inf
// padding); n_wg workgroups of 4 waves, slab holds 4 * n_wg per-wave slabs
H2OMX_API int h2omx_kmeans_wave(const float* X, int64_t ld, int64_t n, int d, const float* Cp, const float* CTg,
                                const float* cnp,
                                int k, int kp, int dp, int n_wg, int* assign, float* slab, hipStream_t stream) {
  if (n_wg < 1 || n < 1 || d < 1 || k < 1 || k > kp || d > dp || dp % 16 != 0 || kp % 4 != 0) return kBadArg;
  const size_t lds = (size_t)4 * dp * KW_LD * sizeof(float);   // the 4 waves' row tiles
#define KW_L(DP, KP)                                                                                        \
  if (dp == DP && kp == KP) {                                                                               \
    hipLaunchKernelGGL((kmeans_wave_kernel<DP, KP>), dim3(n_wg), dim3(256), lds, stream, X, ld, n, d, Cp, CTg, \
                       cnp, k, assign, slab);                                                               \
    return launch_status();                                                                                 \
  }
  KW_L(16, 4) KW_L(32, 4) KW_L(48, 4) KW_L(64, 4) KW_L(80, 4) KW_L(96, 4) KW_L(112, 4) KW_L(128, 4)
  KW_L(16, 8) KW_L(32, 8) KW_L(48, 8) KW_L(64, 8) KW_L(80, 8) KW_L(96, 8) KW_L(112, 8) KW_L(128, 8)
  KW_L(16, 12) KW_L(32, 12) KW_L(48, 12) KW_L(64, 12) KW_L(80, 12) KW_L(96, 12) KW_L(112, 12) KW_L(128, 12)
  KW_L(16, 16) KW_L(32, 16) KW_L(48, 16) KW_L(64, 16) KW_L(80, 16) KW_L(96, 16) KW_L(112, 16) KW_L(128, 16)
  KW_L(16, 24) KW_L(32, 24) KW_L(48, 24) KW_L(64, 24)
  KW_L(16, 32) KW_L(32, 32) KW_L(48, 32) KW_L(64, 32)
#undef KW_L
  return kBadArg;
}

