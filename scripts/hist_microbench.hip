// LDS histogram atomic micro-benchmark (design experiment for hist_build_kernel).
//
// 11M rows x 28 features, uint8 codes (uniform random bins), one packed
// per-row statistic; every row is live (level 0).  Variants:
//   u64      one 64-bit LDS atomic per (row, feature)            = production
//   u32      one 32-bit LDS atomic per (row, feature)             (16|16 packing)
//   u64x2    64-bit, two interleaved copies picked by lane parity (bank spread)
//   u32x4    32-bit, four interleaved copies picked by lane & 3
// Build: hipcc -O3 --offload-arch=gfx950 scripts/hist_microbench.hip -o /tmp/hmb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename T, int COPIES>
__global__ __launch_bounds__(512) void hist_kernel(const uint8_t* __restrict__ codes, int64_t npad, const T* __restrict__ pk,
                                                   int F, int wgs, T* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* h = reinterpret_cast<T*>(smem);
  const int elems = F * 256 * COPIES;
  for (int j = threadIdx.x; j < elems; j += blockDim.x) h[j] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int copy = lane % COPIES;
  const int64_t units = npad / 16;
  const int64_t u0 = units * blockIdx.x / wgs, u1 = units * (blockIdx.x + 1) / wgs;
  for (int64_t u = u0 + threadIdx.x; u < u1; u += blockDim.x) {
    const int64_t r0 = u * 16;
    T v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = pk[r0 + r];
    for (int f = 0; f < F; ++f) {
      const uint4 c4 = *reinterpret_cast<const uint4*>(codes + (int64_t)f * npad + r0);
      const uint32_t cw[4] = {c4.x, c4.y, c4.z, c4.w};
      T* hb = h + f * 256 * COPIES;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int bin = (cw[r >> 2] >> (8 * (r & 3))) & 0xff;
        atomicAdd(hb + bin * COPIES + copy, v[r]);
      }
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < F * 256; j += blockDim.x) {
    T acc = 0;
    for (int c = 0; c < COPIES; ++c) acc += h[j * COPIES + c];
    out[(int64_t)blockIdx.x * F * 256 + j] = acc;
  }
}

// level >= 1 shapes: a random half of the rows is live (smaller children).
// scan: every row visited, atomics under the live mask (production today).
__global__ __launch_bounds__(512) void scan_masked_kernel(const uint8_t* __restrict__ codes, int64_t npad,
                                                          const unsigned long long* __restrict__ pk,
                                                          const int* __restrict__ live, int F, int wgs,
                                                          unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long hs[];
  for (int j = threadIdx.x; j < F * 256; j += blockDim.x) hs[j] = 0;
  __syncthreads();
  const int64_t units = npad / 16;
  const int64_t u0 = units * blockIdx.x / wgs, u1 = units * (blockIdx.x + 1) / wgs;
  for (int64_t u = u0 + threadIdx.x; u < u1; u += blockDim.x) {
    const int64_t r0 = u * 16;
    unsigned long long v[16];
    int lv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) { v[r] = pk[r0 + r]; lv[r] = live[r0 + r]; }
    for (int f = 0; f < F; ++f) {
      const uint4 c4 = *reinterpret_cast<const uint4*>(codes + (int64_t)f * npad + r0);
      const uint32_t cw[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (lv[r]) atomicAdd(hs + f * 256 + ((cw[r >> 2] >> (8 * (r & 3))) & 0xff), v[r]);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < F * 256; j += blockDim.x) out[(int64_t)blockIdx.x * F * 256 + j] = hs[j];
}

// list: only the live rows (ascending ids), RPL per lane per step, codes
// gathered byte-wise from the column-major matrix.
template <int RPL>
__global__ __launch_bounds__(512) void list_kernel(const uint8_t* __restrict__ codes, int64_t npad,
                                                   const unsigned long long* __restrict__ pk,
                                                   const int* __restrict__ list, int64_t L, int F, int wgs,
                                                   unsigned long long* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long hs[];
  for (int j = threadIdx.x; j < F * 256; j += blockDim.x) hs[j] = 0;
  __syncthreads();
  const int64_t i0 = L * blockIdx.x / wgs, i1 = L * (blockIdx.x + 1) / wgs;
  for (int64_t i = i0 + threadIdx.x * RPL; i < i1; i += (int64_t)blockDim.x * RPL) {
    int rows[RPL];
    unsigned long long v[RPL];
#pragma unroll
    for (int k = 0; k < RPL; ++k) rows[k] = (i + k < i1) ? list[i + k] : -1;
#pragma unroll
    for (int k = 0; k < RPL; ++k) v[k] = rows[k] >= 0 ? pk[rows[k]] : 0ull;
    for (int f = 0; f < F; ++f) {
      int b[RPL];
#pragma unroll
      for (int k = 0; k < RPL; ++k) b[k] = rows[k] >= 0 ? codes[(int64_t)f * npad + rows[k]] : 0;
#pragma unroll
      for (int k = 0; k < RPL; ++k)
        if (rows[k] >= 0) atomicAdd(hs + f * 256 + b[k], v[k]);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < F * 256; j += blockDim.x) out[(int64_t)blockIdx.x * F * 256 + j] = hs[j];
}

template <typename T, int COPIES>
int run(const char* name, const uint8_t* codes, int64_t npad, const void* pk, int F, int wgs, void* out) {
  const size_t lds = (size_t)F * 256 * COPIES * sizeof(T);
  if (lds > 160 * 1024) { printf("%-6s skipped (LDS %zu)\n", name, lds); return 0; }
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int it = 0; it < 3; ++it)
    hipLaunchKernelGGL((hist_kernel<T, COPIES>), dim3(wgs), dim3(512), lds, 0, codes, npad, (const T*)pk, F, wgs, (T*)out);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  const int iters = 20;
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((hist_kernel<T, COPIES>), dim3(wgs), dim3(512), lds, 0, codes, npad, (const T*)pk, F, wgs, (T*)out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("%-6s wgs=%5d lds=%6zu B  %8.1f us/pass  %.2f G atomics/s\n", name, wgs, lds, 1000 * ms / iters,
         (double)npad * F / (ms / iters * 1e-3) / 1e9);
  return 0;
}

int main() {
  const int64_t n = 11000000, npad = (n + 255) / 256 * 256;
  const int F = 28;
  std::vector<uint8_t> hc((size_t)F * npad);
  uint32_t s = 12345;
  for (auto& c : hc) { s = s * 1664525u + 1013904223u; c = (uint8_t)(s >> 24); }
  std::vector<uint64_t> hp(npad);
  for (auto& p : hp) { s = s * 1664525u + 1013904223u; p = ((uint64_t)(s >> 20) << 32) | (s >> 16); }
  uint8_t* codes; void* pk; void* out;
  CK(hipMalloc(&codes, hc.size()));
  CK(hipMalloc(&pk, npad * 8));
  CK(hipMalloc(&out, (size_t)4096 * F * 256 * 8));
  CK(hipMemcpy(codes, hc.data(), hc.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(pk, hp.data(), npad * 8, hipMemcpyHostToDevice));
  for (int wgs : {512, 1024}) {
    run<unsigned long long, 1>("u64", codes, npad, pk, F, wgs, out);
    run<unsigned long long, 2>("u64x2", codes, npad, pk, F, wgs, out);
    run<unsigned int, 1>("u32", codes, npad, pk, F, wgs, out);
    run<unsigned int, 2>("u32x2", codes, npad, pk, F, wgs, out);
    run<unsigned int, 4>("u32x4", codes, npad, pk, F, wgs, out);
  }
  // level >= 1: random half live
  {
    std::vector<int> hl(npad, 0), hlist;
    for (int64_t r = 0; r < n; ++r) { s = s * 1664525u + 1013904223u; if (s >> 31) { hl[r] = 1; hlist.push_back((int)r); } }
    int *live, *list;
    const int64_t L = (int64_t)hlist.size();
    CK(hipMalloc(&live, npad * 4)); CK(hipMalloc(&list, L * 4));
    CK(hipMemcpy(live, hl.data(), npad * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(list, hlist.data(), L * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const size_t lds = (size_t)F * 256 * 8;
    auto timeit = [&](const char* name, auto launch) {
      for (int it = 0; it < 3; ++it) launch();
      hipEventRecord(a);
      for (int it = 0; it < 20; ++it) launch();
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("%-12s live=%lld  %8.1f us/pass  %.2f G live atomics/s\n", name, (long long)L, 1000 * ms / 20,
             (double)L * F / (ms / 20 * 1e-3) / 1e9);
    };
    for (int wgs : {512, 1024}) {
      printf("wgs=%d\n", wgs);
      timeit("scan-masked", [&] { hipLaunchKernelGGL(scan_masked_kernel, dim3(wgs), dim3(512), lds, 0, codes, npad,
                                                     (const unsigned long long*)pk, live, F, wgs, (unsigned long long*)out); });
      timeit("list-r1", [&] { hipLaunchKernelGGL((list_kernel<1>), dim3(wgs), dim3(512), lds, 0, codes, npad,
                                                 (const unsigned long long*)pk, list, L, F, wgs, (unsigned long long*)out); });
      timeit("list-r4", [&] { hipLaunchKernelGGL((list_kernel<4>), dim3(wgs), dim3(512), lds, 0, codes, npad,
                                                 (const unsigned long long*)pk, list, L, F, wgs, (unsigned long long*)out); });
      timeit("list-r8", [&] { hipLaunchKernelGGL((list_kernel<8>), dim3(wgs), dim3(512), lds, 0, codes, npad,
                                                 (const unsigned long long*)pk, list, L, F, wgs, (unsigned long long*)out); });
    }
    CK(hipGetLastError());
    CK(hipFree(live)); CK(hipFree(list));
  }
  CK(hipFree(codes)); CK(hipFree(pk)); CK(hipFree(out));
  return 0;
}
