// Microbenchmark: LDS atomic throughput on gfx950 for histogram design.
// Each block: 512 threads, iterates ITERS times doing one atomic per lane into a
// 256-bin LDS histogram with a given address pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE, typename T>
__global__ __launch_bounds__(512) void k(const uint8_t* __restrict__ bins, int iters, T* out) {
  __shared__ T h[8 * 256 * 3];
  for (int i = threadIdx.x; i < 8 * 256 * 3; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t x = blockIdx.x * 977 + threadIdx.x * 131;
  T v = (T)1;
  for (int it = 0; it < iters; ++it) {
    int b;
    uint32_t r = x + (uint32_t)it * 0x9E3779B9u;
    r ^= r >> 15; r *= 0x2c1b3c6du; r ^= r >> 12;
    if (MODE == 0) b = (lane + it) & 255;           // conflict-free distinct (rotating)
    else if (MODE == 1) b = r & 255;                // random 0..255
    else if (MODE == 2) b = (r & 255) % 3;          // 3 values
    else if (MODE == 4) b = 0;                      // all lanes same address
    else b = (threadIdx.x >> 6) * 256 + (r & 255);  // per-wave private hist, random
    atomicAdd(&h[b], v);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = h[7];
}

template <int MODE, typename T>
float run(const uint8_t* bins, int blocks, int iters, T* out) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((k<MODE, T>), dim3(blocks), dim3(512), 0, 0, bins, iters, out);
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k<MODE, T>), dim3(blocks), dim3(512), 0, 0, bins, iters, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 3;
}

int main() {
  const int N = 1 << 20;
  uint8_t* hb = new uint8_t[N];
  uint32_t s = 12345;
  for (int i = 0; i < N; ++i) { s = s * 1664525u + 1013904223u; hb[i] = s >> 24; }
  uint8_t* db; hipMalloc(&db, N); hipMemcpy(db, hb, N, hipMemcpyHostToDevice);
  void* out; hipMalloc(&out, 1 << 20);
  const int blocks = 512, iters = 4096;
  const double atoms = (double)blocks * 512 * iters;
  auto rep = [&](const char* name, float ms) {
    printf("%-28s %8.3f ms  %8.1f G lane-atomics/s  %6.2f lane-atomics/CU-cycle(2.4GHz)\n", name, ms,
           atoms / ms / 1e6, atoms / (ms * 1e-3) / (256 * 2.4e9));
  };
  rep("f32 distinct", run<0, float>(db, blocks, iters, (float*)out));
  rep("f32 random256", run<1, float>(db, blocks, iters, (float*)out));
  rep("f32 3values", run<2, float>(db, blocks, iters, (float*)out));
  rep("f32 perwave random256", run<3, float>(db, blocks, iters, (float*)out));
  rep("u32 distinct", run<0, uint32_t>(db, blocks, iters, (uint32_t*)out));
  rep("u32 random256", run<1, uint32_t>(db, blocks, iters, (uint32_t*)out));
  rep("u32 3values", run<2, uint32_t>(db, blocks, iters, (uint32_t*)out));
  rep("u64 distinct", run<0, unsigned long long>(db, blocks, iters, (unsigned long long*)out));
  rep("u64 random256", run<1, unsigned long long>(db, blocks, iters, (unsigned long long*)out));
  rep("u64 3values", run<2, unsigned long long>(db, blocks, iters, (unsigned long long*)out));
  rep("u64 perwave random256", run<3, unsigned long long>(db, blocks, iters, (unsigned long long*)out));
  rep("f32 sameaddr", run<4, float>(db, blocks, iters, (float*)out));
  rep("u32 sameaddr", run<4, uint32_t>(db, blocks, iters, (uint32_t*)out));
  rep("u32 perwave random256", run<3, uint32_t>(db, blocks, iters, (uint32_t*)out));
  return 0;
}
