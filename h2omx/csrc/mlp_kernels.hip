// Small-batch MLP training step (H2O DeepLearning estimator defaults: 256-row
// mini-batches) as a short chain of latency-optimised fp32 MFMA kernels.
//
// Measured on MI355X (bench_micro/grid_barrier.hip): a grid-wide barrier in
// one persistent kernel costs ~14 us at 256 workgroups, a kernel boundary
// inside a HIP graph ~2 us.  So the step is NOT one persistent kernel; it is
// the minimum chain of dependent launches, each as short as its critical
// path allows:
//
//   F_0 .. F_{L-2}  a_{l+1} = act(a_l W_l^T + b_l)                 (1 launch each)
//   OUT             z = a_{L-1} W_{L-1}^T + b, softmax / squared loss,
//                   g_{L-1} = dLoss/dz, g_{L-2} = (g_{L-1} W_{L-1}) * act'(a_{L-1})
//   Q_j (j = L-2 .. 0), one launch each, independent jobs side by side:
//                   dW_j = g_j^T a_j, db_j (+ dW_{L-1}, db_{L-1} in the first)
//                   g_{j-1} = (g_j W_j) * act'(a_j)                 (j >= 1)
//                   ADADELTA of layers whose gradient is complete and whose
//                   weights no kernel reads any more (layer j + 2, and in
//                   Q_0 layer 1; layer 0 is updated inside its own dW tiles)
//
// Every GEMM job is tiled so that ~one 16 RI x 16 RJ output tile lands on
// each CU; the tile's 4 waves split K and meet in LDS (fixed wave order), so
// a 256 x 512 x 512 product is ~0.9 us of v_mfma_f32_16x16x4f32 per wave
// instead of a 512-long serial K chain.  Operands stream from global memory
// straight into MFMA registers: K-contiguous operands as one float4 per lane
// and k-group (lane group g holds k = 16 t + 4 g + j for MFMA j of group t -
// any k permutation is a valid sum as long as A and B share it), MN-contiguous
// operands as dword loads coalesced over 16 lanes.
#include "common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kT = 256;      // threads per workgroup (4 waves)
constexpr int kMaxR = 2;     // tile side <= 2 x 16

struct Opnd {
  const float* p;
  int ld;
  int kc;    // 1: element (i, k) at p[i * ld + k]; 0: at p[k * ld + i]
  int vec;   // kc operands with 16-byte aligned rows: float4 loads
};

struct GemmJob {
  Opnd A, B;             // A: I x K, B: J x K
  int I, J, K;
  int RI, RJ;            // tile = 16 RI x 16 RJ
  int tiles_j, tiles;
  int epi;               // 0: act(acc + bias), 1: acc * act'(Y), 2: weight gradient
  int act;               // 1 relu, 2 tanh
  float* out;
  int ldo, ldy;
  const float* bias;
  const float* Y;
  // epi 2: bias gradient (tiles of j-tile 0) and in-tile ADADELTA
  float* db;
  float* W;
  float* Eg2;
  float* Edx2;
  float* bW;
  float* bEg2;
  float* bEdx2;
  int ada;
  int pad;
};

struct AdaJob {
  float* W;
  const float* G;
  float* Eg2;
  float* Edx2;
  long long n;
};

constexpr int kMaxJobs = 3, kMaxAda = 4;
struct Phase {
  GemmJob g[kMaxJobs];
  AdaJob a[kMaxAda];
  int ng, na;
  float rho, eps, l2;
  int pad;
};

__device__ __forceinline__ float act_grad_of(float y, int act) {
  return act == 1 ? (y > 0.0f ? 1.0f : 0.0f) : (1.0f - y * y);
}

// H2O ADADELTA (reference/dense.py adadelta_): one parameter
__device__ __forceinline__ void ada_update(float* W, const float gval, float* Eg2, float* Edx2, int64_t e, float rho,
                                           float eps, float l2) {
  const float w = W[e];
  const float g = gval + l2 * w;
  const float eg = rho * Eg2[e] + (1.0f - rho) * g * g;
  const float ed = Edx2[e];
  const float dx = -sqrtf(ed + eps) / sqrtf(eg + eps) * g;
  Eg2[e] = eg;
  Edx2[e] = rho * ed + (1.0f - rho) * dx * dx;
  W[e] = w + dx;
}

// Operand layouts (template codes): kLdV K-contiguous with 16-byte aligned
// rows (one float4 per lane and group), kLdK K-contiguous otherwise (4 dwords),
// kLdM MN-contiguous (4 dwords, each coalesced over 16 lanes).
constexpr int kLdV = 0, kLdK = 1, kLdM = 2;

__device__ __forceinline__ int op_layout(const Opnd& o) { return o.kc ? (o.vec ? kLdV : kLdK) : kLdM; }

// 16 zero floats: the load address of masked-off lanes
__device__ __attribute__((aligned(16))) float g_mlp_zeros[16];

// One 16-k group of a 16 R-row operand slice into registers (see header).
// Branch-free: a masked-off element (row >= rows, k >= kend) is loaded from
// g_mlp_zeros instead of being zeroed after its load - every load is issued
// unconditionally and its value used unconditionally, so the compiler can
// neither sink it into a branch nor lose track of it in the vmcnt accounting
// (masked selects after the loads compiled to a branch + vmcnt(0) per load:
// ~0.4-0.75 us per 16-k group, measured).  kLdV operands need K % 4 == 0.
template <int LY>
__device__ __forceinline__ void load_group(const Opnd& o, int rows, int kend, int i0, int R, int k0, int c, int g,
                                           float (&v)[kMaxR][4]) {
#pragma unroll
  for (int r = 0; r < kMaxR; ++r) {
    const int i = i0 + 16 * r + c;
    const bool rok = r < R && i < rows;
    if constexpr (LY == kLdV) {
      const int k = k0 + 4 * g;
      const float* a = (rok && k < kend) ? o.p + (int64_t)i * o.ld + k : g_mlp_zeros;
      const float4 q = *reinterpret_cast<const float4*>(a);
      v[r][0] = q.x; v[r][1] = q.y; v[r][2] = q.z; v[r][3] = q.w;
    } else if constexpr (LY == kLdK) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + 4 * g + j;
        v[r][j] = *((rok && k < kend) ? o.p + (int64_t)i * o.ld + k : g_mlp_zeros);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + 4 * g + j;
        v[r][j] = *((rok && k < kend) ? o.p + (int64_t)k * o.ld + i : g_mlp_zeros);
      }
    }
  }
}

// One output tile of job `jb`: 4 waves split K, partials meet in LDS.
template <int kDepth, int LA, int LB>
__device__ __attribute__((always_inline)) void tile_gemm(const GemmJob& jb, int tile, float (*red)[32 * 32], float (*dbr)[32], float rho, float eps,
                          float l2) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int ti = tile / jb.tiles_j, tj = tile % jb.tiles_j;
  const int i0 = ti * 16 * jb.RI, j0 = tj * 16 * jb.RJ;
  const int kq = ((jb.K + 3) / 4 + 15) / 16 * 16;
  const int kb = w * kq, ke = min(jb.K, kb + kq);
  const bool dbon = jb.epi == 2 && jb.db != nullptr && tj == 0;
  f32x4 acc[kMaxR][kMaxR];
#pragma unroll
  for (int a = 0; a < kMaxR; ++a)
#pragma unroll
    for (int b = 0; b < kMaxR; ++b) acc[a][b] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float dbacc[kMaxR] = {0.0f, 0.0f};
  // Up to kDepth 16-k groups of loads in flight per wave: a wave's K range is
  // at most a few hundred k, so its whole operand slice is requested before the
  // first MFMA waits (one memory latency per tile instead of one per group -
  // with a single group in flight the 256 x 512 x 512 layer took 13.5 us)
  float va[kDepth][kMaxR][4], vb[kDepth][kMaxR][4];
  const int ng = kb < ke ? (ke - kb + 15) / 16 : 0;
  // Every slot load is unconditional (a group past the wave's range loads
  // zeros: load_group masks k >= ke), so the number of loads in flight is the
  // same on every path and vmcnt waits only for the slot being consumed.
#pragma unroll
  for (int s = 0; s < kDepth; ++s) {
    load_group<LA>(jb.A, jb.I, ke, i0, jb.RI, kb + 16 * s, c, g, va[s]);
    load_group<LB>(jb.B, jb.J, ke, j0, jb.RJ, kb + 16 * s, c, g, vb[s]);
  }
  for (int base = 0; base < ng; base += kDepth) {
#pragma unroll
    for (int s = 0; s < kDepth; ++s) {
      // (tile-shape test once per accumulator and group, not per MFMA)
#pragma unroll
      for (int a = 0; a < kMaxR; ++a)
#pragma unroll
        for (int b = 0; b < kMaxR; ++b)
          if (a < jb.RI && b < jb.RJ) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(va[s][a][j], vb[s][b][j], acc[a][b], 0, 0, 0);
          }
      if (dbon) {
#pragma unroll
        for (int a = 0; a < kMaxR; ++a) dbacc[a] += (va[s][a][0] + va[s][a][1]) + (va[s][a][2] + va[s][a][3]);
      }
      // refill this slot with the group kDepth ahead
      const int nxt = base + s + kDepth;
      load_group<LA>(jb.A, jb.I, ke, i0, jb.RI, kb + 16 * nxt, c, g, va[s]);
      load_group<LB>(jb.B, jb.J, ke, j0, jb.RJ, kb + 16 * nxt, c, g, vb[s]);
    }
  }
  // partial tiles -> LDS (16x16 layout: lane holds D[4 g + v][c])
#pragma unroll
  for (int a = 0; a < kMaxR; ++a)
#pragma unroll
    for (int b = 0; b < kMaxR; ++b)
#pragma unroll
      for (int v = 0; v < 4; ++v) red[w][(16 * a + 4 * g + v) * 32 + 16 * b + c] = acc[a][b][v];
  if (dbon) {
#pragma unroll
    for (int a = 0; a < kMaxR; ++a) {
      float s = dbacc[a];
      s += __shfl_xor(s, 16, kWave);
      s += __shfl_xor(s, 32, kWave);
      if (g == 0) dbr[w][16 * a + c] = s;
    }
  }
  __syncthreads();
  const int ri = 16 * jb.RI, rj = 16 * jb.RJ;
  for (int e = t; e < 32 * 32; e += kT) {
    const int row = e >> 5, col = e & 31;
    const int i = i0 + row, j = j0 + col;
    if (row >= ri || col >= rj || i >= jb.I || j >= jb.J) continue;
    const float v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    const int64_t o = (int64_t)i * jb.ldo + j;
    if (jb.epi == 0) {
      float r = v + (jb.bias ? jb.bias[j] : 0.0f);
      r = jb.act == 1 ? fmaxf(r, 0.0f) : (jb.act == 2 ? tanhf(r) : r);
      jb.out[o] = r;
    } else if (jb.epi == 1) {
      jb.out[o] = v * act_grad_of(jb.Y[(int64_t)i * jb.ldy + j], jb.act);
    } else {
      jb.out[o] = v;
      if (jb.ada) ada_update(jb.W, v, jb.Eg2, jb.Edx2, o, rho, eps, l2);
    }
  }
  if (dbon && t < ri && i0 + t < jb.I) {
    const float s = ((dbr[0][t] + dbr[1][t]) + dbr[2][t]) + dbr[3][t];
    jb.db[i0 + t] = s;
    if (jb.ada) ada_update(jb.bW, s, jb.bEg2, jb.bEdx2, i0 + t, rho, eps, l2);
  }
  __syncthreads();   // LDS reuse by the caller's next tile
}

template <int kDepth>
__global__ __launch_bounds__(kT, 2) void mlp_phase_kernel(Phase ph) {
  __shared__ float red[4][32 * 32];
  __shared__ float dbr[4][32];
  // job selection with constant indices only, copied into a local (uniform,
  // SGPR-resident) descriptor: a runtime index into the kernel-argument array,
  // or a reference into it passed to a call, copies the whole Phase to scratch
  int b = blockIdx.x;
  GemmJob jb;
  bool have = false;
#pragma unroll
  for (int q = 0; q < kMaxJobs; ++q) {
    if (!have && q < ph.ng) {
      if (b < ph.g[q].tiles) {
        jb = ph.g[q];
        have = true;
      } else {
        b -= ph.g[q].tiles;
      }
    }
  }
  if (have) {
    // operand layouts as template parameters: no branch inside the K loop
    switch (op_layout(jb.A) * 3 + op_layout(jb.B)) {
      case 0: tile_gemm<kDepth, kLdV, kLdV>(jb, b, red, dbr, ph.rho, ph.eps, ph.l2); break;
      case 1: tile_gemm<kDepth, kLdV, kLdK>(jb, b, red, dbr, ph.rho, ph.eps, ph.l2); break;
      case 2: tile_gemm<kDepth, kLdV, kLdM>(jb, b, red, dbr, ph.rho, ph.eps, ph.l2); break;
      case 3: tile_gemm<kDepth, kLdK, kLdV>(jb, b, red, dbr, ph.rho, ph.eps, ph.l2); break;
      case 4: tile_gemm<kDepth, kLdK, kLdK>(jb, b, red, dbr, ph.rho, ph.eps, ph.l2); break;
      case 5: tile_gemm<kDepth, kLdK, kLdM>(jb, b, red, dbr, ph.rho, ph.eps, ph.l2); break;
      case 8: tile_gemm<kDepth, kLdM, kLdM>(jb, b, red, dbr, ph.rho, ph.eps, ph.l2); break;
      default: break;   // (A MN-contiguous with a K-contiguous B: no MLP job has it)
    }
  }
  // this workgroup's even share of the ADADELTA updates listed for the phase
#pragma unroll
  for (int q = 0; q < kMaxAda; ++q) {
    if (q >= ph.na) break;
    const AdaJob& aj = ph.a[q];
    const int64_t chunk = (aj.n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min<int64_t>(aj.n, lo + chunk);
    for (int64_t e = lo + threadIdx.x; e < hi; e += kT) ada_update(aj.W, aj.G[e], aj.Eg2, aj.Edx2, e, ph.rho, ph.eps, ph.l2);
  }
}

// Output layer (C <= 8) + loss gradient + the last hidden layer's pre-activation
// gradient, one wave per row: z = a W^T + b, g_out = (softmax(z) - onehot(y)) / M
// (mode 0) or (z - y) / M (mode 1, C = 1), g_prev = (g_out W) * act'(a).
struct OutDesc {
  const float* A;     // a_{L-1} [M][Hd]
  const float* W;     // [C][Hd]
  const float* b;     // [C]
  const int* y;       // class labels (mode 0)
  const float* yr;    // targets (mode 1)
  float* gout;        // [M][C]
  float* gprev;       // [M][Hd]
  int M, Hd, C, act, mode, vec;
  int lda, ldp;       // row strides of A and gprev
  float inv_m;
  int pad;
};

__global__ __launch_bounds__(kT) void mlp_out_kernel(OutDesc d) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= d.M) return;
  const float* a = d.A + (int64_t)m * d.lda;
  float z[8];
#pragma unroll
  for (int cc = 0; cc < 8; ++cc) z[cc] = 0.0f;
  if (d.vec) {
    for (int n = 4 * lane; n < d.Hd; n += 256) {
      const float4 av = *reinterpret_cast<const float4*>(a + n);
#pragma unroll
      for (int cc = 0; cc < 8; ++cc)
        if (cc < d.C) {
          const float4 wv = *reinterpret_cast<const float4*>(d.W + (int64_t)cc * d.Hd + n);
          z[cc] += (av.x * wv.x + av.y * wv.y) + (av.z * wv.z + av.w * wv.w);
        }
    }
  } else {
    for (int n = lane; n < d.Hd; n += 64) {
      const float av = a[n];
#pragma unroll
      for (int cc = 0; cc < 8; ++cc)
        if (cc < d.C) z[cc] += av * d.W[(int64_t)cc * d.Hd + n];
    }
  }
#pragma unroll
  for (int cc = 0; cc < 8; ++cc) {
    float s = z[cc];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
    z[cc] = s + (cc < d.C ? d.b[cc] : 0.0f);
  }
  float gz[8];
  if (d.mode == 0) {
    float mx = -INFINITY;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc)
      if (cc < d.C) mx = fmaxf(mx, z[cc]);
    float den = 0.0f;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc)
      if (cc < d.C) den += __expf(z[cc] - mx);
    const int yi = d.y[m];
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) gz[cc] = cc < d.C ? (__expf(z[cc] - mx) / den - (cc == yi ? 1.0f : 0.0f)) * d.inv_m : 0.0f;
  } else {
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) gz[cc] = cc == 0 ? (z[0] - d.yr[m]) * d.inv_m : 0.0f;
  }
  if (lane < d.C) {
    float v = gz[0];
#pragma unroll
    for (int cc = 1; cc < 8; ++cc)
      if (cc == lane) v = gz[cc];
    d.gout[(int64_t)m * d.C + lane] = v;
  }
  float* gp = d.gprev + (int64_t)m * d.ldp;
  if (d.vec) {
    for (int n = 4 * lane; n < d.Hd; n += 256) {
      const float4 av = *reinterpret_cast<const float4*>(a + n);
      float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
      for (int cc = 0; cc < 8; ++cc)
        if (cc < d.C) {
          const float4 wv = *reinterpret_cast<const float4*>(d.W + (int64_t)cc * d.Hd + n);
          s.x += gz[cc] * wv.x; s.y += gz[cc] * wv.y; s.z += gz[cc] * wv.z; s.w += gz[cc] * wv.w;
        }
      s.x *= act_grad_of(av.x, d.act); s.y *= act_grad_of(av.y, d.act);
      s.z *= act_grad_of(av.z, d.act); s.w *= act_grad_of(av.w, d.act);
      *reinterpret_cast<float4*>(gp + n) = s;
    }
  } else {
    for (int n = lane; n < d.Hd; n += 64) {
      float s = 0.0f;
#pragma unroll
      for (int cc = 0; cc < 8; ++cc)
        if (cc < d.C) s += gz[cc] * d.W[(int64_t)cc * d.Hd + n];
      gp[n] = s * act_grad_of(a[n], d.act);
    }
  }
}

}  // namespace

H2OMX_API int h2omx_mlp_sizes(int* out) {
  if (out == nullptr) return kBadArg;
  out[0] = (int)sizeof(Opnd);
  out[1] = (int)sizeof(GemmJob);
  out[2] = (int)sizeof(AdaJob);
  out[3] = (int)sizeof(Phase);
  out[4] = (int)sizeof(OutDesc);
  out[5] = kMaxJobs;
  out[6] = kMaxAda;
  return kOk;
}

H2OMX_API int h2omx_mlp_phase(const void* phase, hipStream_t stream) {
  if (phase == nullptr) return kBadArg;
  const Phase ph = *static_cast<const Phase*>(phase);
  if (ph.ng < 0 || ph.ng > kMaxJobs || ph.na < 0 || ph.na > kMaxAda) return kBadArg;
  int blocks = 0;
  for (int q = 0; q < ph.ng; ++q) {
    const GemmJob& j = ph.g[q];
    if (j.RI < 1 || j.RI > kMaxR || j.RJ < 1 || j.RJ > kMaxR || j.tiles_j < 1 || j.K < 1 || j.out == nullptr)
      return kBadArg;
    if (j.tiles != j.tiles_j * ((j.I + 16 * j.RI - 1) / (16 * j.RI)) || j.tiles_j != (j.J + 16 * j.RJ - 1) / (16 * j.RJ))
      return kBadArg;
    if ((j.epi == 1 && j.Y == nullptr) || (j.epi == 2 && j.ada && (j.W == nullptr || j.Eg2 == nullptr)))
      return kBadArg;
    blocks += j.tiles;
  }
  if (blocks == 0) blocks = 256;   // ADADELTA-only phase
  // loads in flight per wave (16-k groups): Phase.pad, 0 = default
  switch (ph.pad) {
    case 1: hipLaunchKernelGGL(mlp_phase_kernel<1>, dim3(blocks), dim3(kT), 0, stream, ph); break;
    case 2: hipLaunchKernelGGL(mlp_phase_kernel<2>, dim3(blocks), dim3(kT), 0, stream, ph); break;
    case 4: hipLaunchKernelGGL(mlp_phase_kernel<4>, dim3(blocks), dim3(kT), 0, stream, ph); break;
    case 8: hipLaunchKernelGGL(mlp_phase_kernel<8>, dim3(blocks), dim3(kT), 0, stream, ph); break;
    default: hipLaunchKernelGGL(mlp_phase_kernel<4>, dim3(blocks), dim3(kT), 0, stream, ph); break;
  }
  return launch_status();
}

H2OMX_API int h2omx_mlp_out(const void* desc, hipStream_t stream) {
  if (desc == nullptr) return kBadArg;
  const OutDesc d = *static_cast<const OutDesc*>(desc);
  if (d.C < 1 || d.C > 8 || d.M < 1 || d.Hd < 1 || (d.mode == 1 && d.C != 1)) return kBadArg;
  hipLaunchKernelGGL(mlp_out_kernel, dim3((d.M + 3) / 4), dim3(kT), 0, stream, d);
  return launch_status();
}

// ===========================================================================
// Large-batch fp32 GEMM on the bf16 matrix cores: "x3" split.
//
// C[M][N] = act(A[M][K] . B[N][K]^T + bias), fp32 in, fp32 out (the forward
// products of the 8192-row DL bench, where the fp32 MFMA rate - 157 TF/s -
// bounds a 8192 x 512 x 512 layer at 27 us).  Every fp32 operand is split
// EXACTLY into three bf16 pieces while it is staged to LDS:
//     x = hi + mid + lo,  hi = bf16(x), mid = bf16(x - hi), lo = x - hi - mid
// (round-to-nearest at each step leaves <= 8 significant bits per piece, so
// the three pieces hold all 24 bits of x).  The product keeps the six terms
// hi.hi, hi.mid, mid.hi, hi.lo, lo.hi, mid.mid - every one exact in fp32 -
// and drops mid.lo, lo.mid, lo.lo (<= 2^-24 |a||b|, the size of one fp32
// rounding), accumulating in fp32 on v_mfma_f32_32x32x16_bf16: fp32-equivalent
// accuracy (pinned against float64 in tests/test_dl_step_gpu.py) at 6 bf16
// MFMAs per 16-k step instead of 8 fp32 ones of 4 k each (2.7x the rate).
// 128 x 128 block tile, 4 waves of 64 x 64 (2 x 2 accumulators of 32 x 32),
// 32-k stages: coalesced float4 global loads -> split -> three bf16 planes in
// LDS (rows padded to 40 elements: conflict-free ds_read_b128 fragments);
// the next stage's loads are in flight under the current stage's MFMAs.
// ===========================================================================
namespace {

typedef __bf16 x3_bf16x8 __attribute__((ext_vector_type(8)));
typedef float x3_f32x16 __attribute__((ext_vector_type(16)));
constexpr int X3_BM = 128, X3_BN = 128, X3_BK = 32, X3_ROW = X3_BK + 8;   // bf16 elements per LDS row
constexpr int X3_PLANE = 128 * X3_ROW;                                   // one plane of one operand

__device__ __forceinline__ void x3_split(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// float4 k-run of one row -> the three planes (4 bf16 = 8 bytes each)
__device__ __forceinline__ void x3_store(__bf16* L, int row, int k, const float4 v) {
  __bf16 h[4], m[4], l[4];
  x3_split(v.x, h[0], m[0], l[0]);
  x3_split(v.y, h[1], m[1], l[1]);
  x3_split(v.z, h[2], m[2], l[2]);
  x3_split(v.w, h[3], m[3], l[3]);
  __bf16* p = L + row * X3_ROW + k;
  *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(h);
  *reinterpret_cast<uint2*>(p + X3_PLANE) = *reinterpret_cast<const uint2*>(m);
  *reinterpret_cast<uint2*>(p + 2 * X3_PLANE) = *reinterpret_cast<const uint2*>(l);
}

struct X3Regs {
  float4 a[4], b[4];
};

__device__ __forceinline__ void x3_load(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb,
                                        int M, int N, int K, int m0, int n0, int k0, X3Regs& r) {
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = q * 256 + t, row = f >> 3, k = k0 + (f & 7) * 4;
    const int i = m0 + row, j = n0 + row;
    r.a[q] = (i < M && k < K) ? *reinterpret_cast<const float4*>(A + (int64_t)i * lda + k) : make_float4(0, 0, 0, 0);
    r.b[q] = (j < N && k < K) ? *reinterpret_cast<const float4*>(B + (int64_t)j * ldb + k) : make_float4(0, 0, 0, 0);
  }
}

// kDB: two LDS stage buffers (one barrier per 32-k stage, the next stage's
// split under this stage's MFMAs) - 120 KB of LDS, one workgroup per CU: for
// grids of at most one tile per CU (8192 x 512: 40.1 vs 44.0 us); larger grids
// keep one buffer and two workgroups per CU (8192 x 2048 x 2048: 402 vs 441 us,
// profiles/r5/dl/gemm_x3_r5o.jsonl)
// (K-major operand variants for the data / weight gradients - column gathers
// into the same LDS planes - ran slower than the fp32 MFMA kernels: dact 58.8
// vs 56.2 us, split-K weight gradient 50.1 vs 41.4 us at 8192 x 512 x 512,
// profiles/r5/dl/kernel_stats_r5q.txt; removed)
// kEPI 0: C = act(acc + bias) (forward layers); kEPI 1: C = acc * act'(Y) and
// the column sums of C per 64-row wave block into ws[(row / 64)][N] (the data
// gradient of a hidden layer with its bias-gradient slices; B = W^T, made
// K-contiguous by x3_transpose_kernel first)
template <bool kDB, int kEPI>
__global__ __launch_bounds__(256) void gemm_x3_nt_kernel(const float* __restrict__ A, int lda,
                                                        const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                        int ldc, const float* __restrict__ bias, int M, int N, int K,
                                                        int act, const float* __restrict__ Y, int ldy,
                                                        float* __restrict__ ws) {
  constexpr int NBUF = kDB ? 2 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 La[NBUF][3 * X3_PLANE];
  __shared__ __attribute__((aligned(16))) __bf16 Lb[NBUF][3 * X3_PLANE];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int li = lane & 31, lh = lane >> 5;
  // XCD-aware order: linear block b runs on XCD b % 8; give each XCD a
  // contiguous range of tiles (row-major over the tile grid: shared A rows
  // stay in that XCD's L2)
  const int gx = gridDim.x, nb = gx * gridDim.y;
  int bid = blockIdx.y * gx + blockIdx.x;
  if ((nb & 7) == 0) bid = (bid & 7) * (nb >> 3) + (bid >> 3);
  const int m0 = (bid / gx) * X3_BM, n0 = (bid % gx) * X3_BN;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  x3_f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.0f;
  const int nst = (K + X3_BK - 1) / X3_BK;
  // kEPI 1 (always kDB: one wave per SIMD, 64 VGPRs of room): the tile's Y
  // values (for act') are loaded before the k loop, so the epilogue waits on no
  // global load
  float yg[kEPI == 1 ? 2 : 1][kEPI == 1 ? 32 : 1];
  auto load_y = [&](int b) {
    const int j = min(n0 + wn + 32 * b + li, N - 1);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int i = min(m0 + wm + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * lh, M - 1);
        yg[b][a * 16 + e] = Y[(int64_t)i * ldy + j];
      }
  };
  if (kEPI == 1) {
    load_y(0);
    load_y(1);
  }
  X3Regs r;
  x3_load(A, lda, B, ldb, M, N, K, m0, n0, 0, r);
  auto stage = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = q * 256 + t, row = f >> 3, k = (f & 7) * 4;
      x3_store(La[buf], row, k, r.a[q]);
      x3_store(Lb[buf], row, k, r.b[q]);
    }
  };
  if (kDB) { stage(0); __syncthreads(); }
  for (int st = 0; st < nst; ++st) {
    const int buf = kDB ? (st & 1) : 0;
    if (!kDB) { stage(0); __syncthreads(); }
    if (st + 1 < nst) x3_load(A, lda, B, ldb, M, N, K, m0, n0, (st + 1) * X3_BK, r);
    const __bf16* La_ = La[buf];
    const __bf16* Lb_ = Lb[buf];
#pragma unroll
    for (int kk = 0; kk < X3_BK; kk += 16) {
      x3_bf16x8 fa[2][3], fb[2][3];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          fa[a][p] = *reinterpret_cast<const x3_bf16x8*>(La_ + p * X3_PLANE + (wm + 32 * a + li) * X3_ROW + kk + 8 * lh);
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          fb[b][p] = *reinterpret_cast<const x3_bf16x8*>(Lb_ + p * X3_PLANE + (wn + 32 * b + li) * X3_ROW + kk + 8 * lh);
      // small terms first (fp32 accumulation order: lo-order products then hi.hi);
      // product-major issue (4 independent accumulators between dependent MFMAs;
      // measured the same as accumulator-major)
      constexpr int PA[6] = {1, 2, 0, 1, 0, 0}, PB[6] = {1, 0, 2, 0, 1, 0};
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a][PA[q]], fb[b][PB[q]], acc[a][b], 0, 0, 0);
    }
    if (kDB) {
      if (st + 1 < nst) stage(buf ^ 1);
    }
    __syncthreads();
  }
  // epilogue: lane owns column j, registers e are rows (e & 3) + 8 (e >> 2) + 4 lh
  if (kEPI == 1) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int j = n0 + wn + 32 * b + li;
      float cs = 0.0f;
      if (j < N) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int i = m0 + wm + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * lh;
            if (i < M) {
              const float v = acc[a][b][e] * act_grad_of(yg[b][a * 16 + e], act);
              C[(int64_t)i * ldc + j] = v;
              cs += v;
            }
          }
      }
      cs += __shfl_xor(cs, 32, 64);   // the other 32 rows of the wave block
      if (lh == 0 && j < N && m0 + wm < M) ws[(int64_t)((m0 + wm) >> 6) * N + j] = cs;
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int j = n0 + wn + 32 * b + li;
      if (j >= N) continue;
      const float bj = bias ? bias[j] : 0.0f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int i = m0 + wm + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (i < M) {
          float v = acc[a][b][e] + bj;
          v = act == 1 ? fmaxf(v, 0.0f) : (act == 2 ? tanhf(v) : v);
          C[(int64_t)i * ldc + j] = v;
        }
      }
    }
}

// dst[c][r] = src[r][c] through a padded 32 x 33 LDS tile, one job per
// blockIdx.z (a network's hidden weights, [out][in] -> [in][out], in one
// launch, so the data-gradient GEMMs read K-contiguous rows)
constexpr int X3_TMAX = 8;
struct X3Transpose {
  const float* src[X3_TMAX];
  float* dst[X3_TMAX];
  int R[X3_TMAX], C[X3_TMAX];
};

__global__ __launch_bounds__(256) void x3_transpose_kernel(X3Transpose T) {
  __shared__ float tile[32][33];
  const int z = blockIdx.z;
  const float* __restrict__ src = T.src[z];
  float* __restrict__ dst = T.dst[z];
  const int R = T.R[z], Cn = T.C[z];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  if (c0 >= Cn || r0 >= R) return;   // (grid sized for the largest job)
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + ty + 8 * q, c = c0 + tx;
    if (r < R && c < Cn) tile[ty + 8 * q][tx] = src[(int64_t)r * Cn + c];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = c0 + ty + 8 * q, r = r0 + tx;
    if (r < R && c < Cn) dst[(int64_t)c * R + r] = tile[tx][ty + 8 * q];
  }
}

}  // namespace

// fp32 NT GEMM on the bf16 matrix cores (x3 split, see above); A, B rows
// 16-byte aligned (lda, ldb % 4 == 0), K % 4 == 0
H2OMX_API int h2omx_gemm_x3(const float* A, int lda, const float* B, int ldb, float* C, int ldc, const float* bias,
                            int M, int N, int K, int act, hipStream_t stream) {
  if (A == nullptr || B == nullptr || C == nullptr || M < 1 || N < 1 || K < 1) return kBadArg;
  if ((lda & 3) || (ldb & 3) || (K & 3) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return kBadArg;
  const dim3 grid((N + X3_BN - 1) / X3_BN, (M + X3_BM - 1) / X3_BM);
  if ((int64_t)grid.x * grid.y <= 256)
    hipLaunchKernelGGL((gemm_x3_nt_kernel<true, 0>), grid, dim3(256), 0, stream, A, lda, B, ldb, C, ldc, bias, M, N,
                       K, act, nullptr, 0, nullptr);
  else
    hipLaunchKernelGGL((gemm_x3_nt_kernel<false, 0>), grid, dim3(256), 0, stream, A, lda, B, ldb, C, ldc, bias, M, N,
                       K, act, nullptr, 0, nullptr);
  return launch_status();
}

// Transposes of n <= 8 row-major matrices src_i [R_i][C_i] -> dst_i [C_i][R_i]
// in one launch (the hidden weights before the backward's data gradients).
H2OMX_API int h2omx_x3_transpose(int n, const float* const* src, float* const* dst, const int* R, const int* C,
                                 hipStream_t stream) {
  if (n < 1 || n > X3_TMAX || src == nullptr || dst == nullptr || R == nullptr || C == nullptr) return kBadArg;
  X3Transpose T{};
  int gx = 1, gy = 1;
  for (int z = 0; z < n; ++z) {
    if (src[z] == nullptr || dst[z] == nullptr || R[z] < 1 || C[z] < 1) return kBadArg;
    T.src[z] = src[z]; T.dst[z] = dst[z]; T.R[z] = R[z]; T.C[z] = C[z];
    gx = max(gx, (C[z] + 31) / 32);
    gy = max(gy, (R[z] + 31) / 32);
  }
  hipLaunchKernelGGL(x3_transpose_kernel, dim3(gx, gy, n), dim3(256), 0, stream, T);
  return launch_status();
}

// Data gradient of a Rectifier (act 1) / Tanh (act 2) layer on the x3 GEMM:
// C[M][N] = (dZ[M][K] . Wt[N][K]^T) * act'(Y[M][N]), Wt = W^T (h2omx_x3_transpose).
// ws[(M + 63) / 64][N] receives the column sums of C per 64-row block.  All
// matrices dense row-major, K % 4 == 0.
H2OMX_API int h2omx_gemm_x3_dact(const float* dZ, const float* Wt, const float* Y, float* C, float* ws, int M, int N,
                                 int K, int act, hipStream_t stream) {
  if (dZ == nullptr || Wt == nullptr || Y == nullptr || C == nullptr || ws == nullptr || M < 1 || N < 1 || K < 1 ||
      (act != 1 && act != 2))
    return kBadArg;
  if ((K & 3) || ((uintptr_t)dZ & 15) || ((uintptr_t)Wt & 15)) return kBadArg;
  // (double-buffered at every grid size: the single-buffer variant's two waves
  // per SIMD do not fit the prefetched Y registers)
  const dim3 grid((N + X3_BN - 1) / X3_BN, (M + X3_BM - 1) / X3_BM);
  hipLaunchKernelGGL((gemm_x3_nt_kernel<true, 1>), grid, dim3(256), 0, stream, dZ, K, Wt, K, C, N, nullptr, M, N, K,
                     act, Y, N, ws);
  return launch_status();
}
