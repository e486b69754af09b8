// Shared helpers for the h2omx HIP kernels (gfx950 / CDNA4 only).
//
// Every kernel library in this directory is compiled with
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC
// and exposes a flat C ABI (extern "C") that the Python layer calls through
// ctypes with raw device pointers and the caller's hipStream_t.  No torch
// headers are needed, which keeps the kernel build fast and the ABI stable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define H2OMX_API extern "C" __attribute__((visibility("default")))

// Wave64 is the CDNA execution width; never assume 32.
constexpr int kWave = 64;

// Return codes of the C entry points (0 = launched).
enum H2omxStatus : int {
  kOk = 0,
  kBadArg = 1,
  kLaunchFailed = 2,
};

static inline int launch_status() {
  return hipGetLastError() == hipSuccess ? kOk : kLaunchFailed;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Stateless 32-bit mixing hash (splitmix-style); used for row bagging and
// per-node column sampling so that every rank draws identical samples
// without any communication.
__device__ __host__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __host__ __forceinline__ uint32_t hash4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return mix32(a ^ mix32(b ^ mix32(c ^ mix32(d + 0x9e3779b9U))));
}

__device__ __host__ __forceinline__ float u01(uint32_t h) {
  return (h >> 8) * (1.0f / 16777216.0f);
}
