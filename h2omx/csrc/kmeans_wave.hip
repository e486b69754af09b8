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
//     operand - no LDS traffic for them (KW_CT_SCALAR=0: LDS broadcast
//     reads instead, measured LDS-bound); ||c||^2 - 2 dot -> argmin (lowest
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
#ifndef KW_CT_SCALAR
#define KW_CT_SCALAR 1
#endif

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
#if !KW_CT_SCALAR
  float* CT = kw_lds + 4 * DP * KW_LD;   // centroids transposed [f][KP], shared by the 4 waves
  for (int j = threadIdx.x; j < DP * KP; j += blockDim.x) CT[j] = Cp[(j % KP) * DP + j / KP];
  __syncthreads();
#endif
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
#if KW_CT_SCALAR
        const float4 cv = *reinterpret_cast<const float4*>(CTg + co + 4 * c4);   // scalar-cache read
#else
        const float4 cv = *reinterpret_cast<const float4*>(CT + co + 4 * c4);   // broadcast read
#endif
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


// wave-unit Lloyd pass: Cp [KP][DP] zero-padded centroids, cnp [KP] (+inf
// padding); n_wg workgroups of 4 waves, slab holds 4 * n_wg per-wave slabs
H2OMX_API int h2omx_kmeans_wave(const float* X, int64_t ld, int64_t n, int d, const float* Cp, const float* CTg,
                                const float* cnp,
                                int k, int kp, int dp, int n_wg, int* assign, float* slab, hipStream_t stream) {
  if (n_wg < 1 || n < 1 || d < 1 || k < 1 || k > kp || d > dp || dp % 16 != 0 || kp % 4 != 0) return kBadArg;
  const size_t lds = ((size_t)4 * dp * KW_LD + (size_t)dp * kp) * sizeof(float);
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

