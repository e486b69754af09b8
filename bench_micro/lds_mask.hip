// Microbenchmark: cost of a 64-bit LDS atomic wave-instruction (ds_add_u64,
// random bins of a 7-feature x 256-bin histogram) as a function of the
// fraction of active lanes, and the cost of the LDS-staged compaction step
// (ds_write_b128 of a 1 KB code tile + ds_read_u8 gather) that replaces 16
// partially-masked atomics by ceil(16 * p) full ones.  Decides whether the
// level >= 1 histogram kernel should compact live rows per wave.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t mix(uint32_t r) {
  r ^= r >> 15; r *= 0x2c1b3c6du; r ^= r >> 12; r *= 0x297a2d39u; r ^= r >> 15;
  return r;
}

// MODE 0: one masked atomic per iteration (lane active with probability p/256)
// MODE 1: staged: per 16 iterations, one ds_write_b128 into a per-wave 1 KB tile,
//         then NITER ds_read_u8 + full atomics (NITER = ceil(16 p / 256))
template <int MODE, typename T = unsigned long long>
__global__ __launch_bounds__(1024) void k(int iters, int p256, unsigned long long* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char hraw[];
  T* h = reinterpret_cast<T*>(hraw);
  constexpr int HE = 7 * 256;
  __shared__ __attribute__((aligned(16))) uint8_t tile[16][1024];
  for (int i = threadIdx.x; i < HE; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = mix(blockIdx.x * 977u + threadIdx.x * 131u);
  if (MODE == 0) {
    for (int it = 0; it < iters; ++it) {
      const uint32_t r = mix(x + (uint32_t)it * 0x9E3779B9u);
      if ((int)(r >> 24) < p256) atomicAdd(&h[((it % 7) << 8) + (r & 255)], (T)1);
    }
  } else {
    const int niter = (16 * p256 + 255) / 256;
    for (int it = 0; it < iters; it += 16) {
      const uint32_t r = mix(x + (uint32_t)it * 0x9E3779B9u);
      uint4 v = make_uint4(r, r * 3u, r * 5u, r * 7u);
      *reinterpret_cast<uint4*>(&tile[wid][lane * 16]) = v;
      for (int j = 0; j < niter; ++j) {
        const int off = (r >> (j & 7)) & 1023;
        const int bin = tile[wid][off];
        atomicAdd(&h[(((it + j) % 7) << 8) + bin], (T)1);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = h[7];
}

template <int MODE, typename T = unsigned long long>
float run(int blocks, int iters, int p256, unsigned long long* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t lds = 7 * 256 * 8;
  hipLaunchKernelGGL((k<MODE, T>), dim3(blocks), dim3(1024), lds, 0, iters, p256, out);
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k<MODE, T>), dim3(blocks), dim3(1024), lds, 0, iters, p256, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 3;
}

int main() {
  unsigned long long* out;
  hipMalloc(&out, 1 << 20);
  const int blocks = 512, iters = 4096;
  const double winst = (double)blocks * 16 * iters;  // wave-iterations of 16-row-equivalent work
  const int ps[] = {256, 192, 128, 90, 64, 32};
  for (int p : ps) {
    const float m0 = run<0>(blocks, iters, p, out);
    const float m1 = run<1>(blocks, iters, p, out);
    const double cyc0 = (m0 * 1e-3) * 256 * 2.4e9 / winst;  // CU-cycles per masked wave-instruction
    const float m2 = run<0, unsigned int>(blocks, iters, p, out);
    const float m3 = run<0, float>(blocks, iters, p, out);
    printf("p=%.2f u32 masked %.3f ms (%.2f cyc)  f32 %.3f ms (%.2f cyc)\n", p / 256.0, m2, (m2 * 1e-3) * 256 * 2.4e9 / winst, m3, (m3 * 1e-3) * 256 * 2.4e9 / winst);
    printf("p=%.2f masked: %.3f ms (%.2f CU-cyc per wave-atomic)  staged: %.3f ms  speedup %.2fx\n", p / 256.0, m0,
           cyc0, m1, m0 / m1);
  }
  return 0;
}
