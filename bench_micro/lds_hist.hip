// Microbenchmark: the histogram kernel's inner loop in isolation.
// Each lane holds 16 random bin codes (4 dwords, L2-resident source) and a
// packed 64-bit value; per "feature" it issues 16 ds_add_u64 into a 256-bin
// slice (bfe + lshl_add per atomic, as the real kernel after simplification).
// Variants: every lane active / a fraction p active with an exec-mask branch
// per atomic / p active branch-free (inactive lanes add 0) / u32 adds /
// the current kernel's per-atomic NA remap (cmp + cndmask).
// Reports CU-cycles per wave-atomic at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int MODE, typename T>
__global__ __launch_bounds__(512) void k(const uint4* __restrict__ src, int iters, int p256, int width,
                                         unsigned long long* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char raw[];
  T* h = reinterpret_cast<T*>(raw);
  constexpr int NF = 28;
  for (int i = threadIdx.x; i < NF * 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t act = 0;
  {
    uint32_t x = (blockIdx.x * 977u + threadIdx.x * 131u) * 0x9E3779B9u;
    for (int r = 0; r < 16; ++r) {
      x ^= x >> 15; x *= 0x2c1b3c6du; x ^= x >> 12;
      if ((int)(x >> 24) < p256) act |= 1u << r;
    }
  }
  T v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = (MODE == 2 && !((act >> r) & 1)) ? (T)0 : (T)(r + 1);
  int idx = (blockIdx.x * 512 + threadIdx.x) & 4095;
  for (int it = 0; it < iters; ++it) {
    const int f = it % NF;
    const uint4 c = src[(idx + it * 64) & 4095];
    const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
    T* hb = h + f * 256;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int bin = (cw[r >> 2] >> (8 * (r & 3))) & 0xff;
      if (MODE == 3 && bin == 255) bin = width - 1;
      if (MODE == 1 || MODE == 3) {
        if ((act >> r) & 1) atomicAdd(hb + bin, v[r]);
      } else {
        atomicAdd(hb + bin, v[r]);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (unsigned long long)h[7];
}

template <int MODE, typename T>
float run(const uint4* src, int blocks, int iters, int p, int width, unsigned long long* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t lds = 28 * 256 * sizeof(T);
  hipLaunchKernelGGL((k<MODE, T>), dim3(blocks), dim3(512), lds, 0, src, iters, p, width, out);
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL((k<MODE, T>), dim3(blocks), dim3(512), lds, 0, src, iters, p, width, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 3;
}

int main() {
  uint32_t* hsrc = new uint32_t[4096 * 4];
  uint32_t s = 1;
  for (int i = 0; i < 4096 * 4; ++i) { s = s * 1664525u + 1013904223u; hsrc[i] = s; }
  uint4* src;
  unsigned long long* out;
  (void)hipMalloc(&src, 4096 * 16);
  (void)hipMemcpy(src, hsrc, 4096 * 16, hipMemcpyHostToDevice);
  (void)hipMalloc(&out, 1 << 20);
  const int blocks = 512, iters = 2048;
  const double wa = (double)blocks * 8 * iters * 16;  // wave-atomics
  auto cyc = [&](float ms) { return (ms * 1e-3) * 256 * 2.4e9 / wa; };
  printf("u64 all lanes           : %.2f cyc/wave-atomic\n", cyc(run<0, unsigned long long>(src, blocks, iters, 256, 256, out)));
  printf("u32 all lanes           : %.2f\n", cyc(run<0, unsigned int>(src, blocks, iters, 256, 256, out)));
  for (int p : {192, 102, 64}) {
    printf("p=%.2f u64 branch      : %.2f\n", p / 256.0, cyc(run<1, unsigned long long>(src, blocks, iters, p, 256, out)));
    printf("p=%.2f u64 zero-add    : %.2f\n", p / 256.0, cyc(run<2, unsigned long long>(src, blocks, iters, p, 256, out)));
    printf("p=%.2f u64 branch+NA   : %.2f\n", p / 256.0, cyc(run<3, unsigned long long>(src, blocks, iters, p, 200, out)));
  }
  return 0;
}
