// Cost of a grid-wide barrier inside one persistent kernel vs a kernel
// boundary (graph-captured chain of launches) on MI355X.
// Each "phase": every workgroup writes 4 KB of its own slot, barrier, reads
// the slot of workgroup (b + 1) % G (cross-XCD visibility exercised).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ bool grid_barrier(unsigned* ctr, unsigned target, int* err) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = wall_clock64();
    while ((int)(__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      if (wall_clock64() - t0 > 200000000ull) { atomicExch(err, 1); ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return ok;
}

__global__ __launch_bounds__(256) void persistent(float* buf, unsigned* ctr, int phases, int* err, float* sink) {
  __shared__ unsigned s_base;
  const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x;
  if (t == 0) s_base = __hip_atomic_load(ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned base = s_base;
  float acc = 0.f;
  for (int p = 0; p < phases; ++p) {
    float4* mine = reinterpret_cast<float4*>(buf + (size_t)b * 1024);
    mine[t] = make_float4(p, b, t, 1.f);
    if (!grid_barrier(ctr, base + (unsigned)(p + 1) * G, err)) return;
    const float4 v = reinterpret_cast<const float4*>(buf + (size_t)((b + 1) % G) * 1024)[t];
    acc += v.x + v.y;
  }
  if (b == 0 && t == 0) __hip_atomic_store(ctr + 1, base + (unsigned)phases * G, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (acc == -1.f) sink[0] = acc;
}

__global__ __launch_bounds__(256) void one_phase(float* buf, int p, float* sink) {
  const int G = gridDim.x, b = blockIdx.x, t = threadIdx.x;
  const float4 v = reinterpret_cast<const float4*>(buf + (size_t)((b + 1) % G) * 1024)[t];
  reinterpret_cast<float4*>(buf + (size_t)b * 1024)[t] = make_float4(p + v.x, b, t, 1.f);
}

int main() {
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  printf("CUs %d\n", cus);
  float *buf, *sink; unsigned* ctr; int* err;
  CK(hipMalloc(&buf, 1024 * 4 * 1024)); CK(hipMalloc(&sink, 64)); CK(hipMalloc(&ctr, 64)); CK(hipMalloc(&err, 64));
  CK(hipMemset(ctr, 0, 64)); CK(hipMemset(err, 0, 64));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int G : {64, 128, 256}) {
    for (int P : {1, 9, 33}) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(persistent, dim3(G), dim3(256), 0, s, buf, ctr, P, err, sink);
      CK(hipStreamSynchronize(s));
      const int R = 50;
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < R; ++r) hipLaunchKernelGGL(persistent, dim3(G), dim3(256), 0, s, buf, ctr, P, err, sink);
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      int h_err = 0; CK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
      printf("persistent G=%d phases=%d: %.2f us/launch err=%d\n", G, P, 1000.f * ms / R, h_err);
    }
    // graph of P single-phase kernels
    for (int P : {1, 9, 33}) {
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int p = 0; p < P; ++p) hipLaunchKernelGGL(one_phase, dim3(G), dim3(256), 0, s, buf, p, sink);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      const int R = 50;
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf("graph     G=%d kernels=%d: %.2f us/replay\n", G, P, 1000.f * ms / R);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
