// One-shot peer-to-peer all-reduce over IPC-mapped HBM (xGMI between GPUs).
//
// The tree engine's level histograms (<= a few MB of int64), its leaf sums and
// a GLM Gram are latency-bound messages: a ring all-reduce
// spends 2 (N - 1) hops of link latency on them, and a host-issued RCCL call
// also splits the step's HIP graph into segments.  Here every rank keeps a
// symmetric buffer that every peer has mapped (hipIpcGetMemHandle /
// hipIpcOpenMemHandle, exchanged over the rendezvous store), and one kernel
// launch does the whole collective:
//
//   block b:  copy my chunk b into my symmetric buffer (parity = epoch & 1,
//             write-through system-scope stores) -> every wave drains ->
//             post epoch into flags[b][my rank] of every peer -> poll my
//             flags[b][*] >= epoch -> out[chunk b] = sum over ranks
//             r = 0 .. N-1 (fixed order) of sym_r[parity][chunk b]
//             (system-scope loads; p2p_device.h: no cache maintenance)
//
// * Blocks are independent: block b only waits for chunk b of its peers, so
//   there is no grid barrier and no co-residency requirement.
// * The epoch counter lives in device memory and is advanced by the kernel
//   itself (last block to finish), so the launch has no per-call host input
//   and is captured inside the tree step's HIP graph: an N-rank tree is one
//   graph replay with zero host-issued collectives.
// * Buffers alternate by epoch parity: a rank can be at most one collective
//   ahead of any peer (it needs every peer's post of the current epoch), so
//   the parity it overwrites was fully read by everyone.
// * Summation order is the rank order on every rank: float results are
//   bit-identical across ranks (int64 histogram sums are exact anyway).
// * Every poll is bounded by a wall-clock timeout: a peer that never arrives
//   sets the error word and the kernel drains (the host checks that word),
//   so a lost rank can never leave waves spinning on the GPU.
//
// All stores are vector-memory stores/atomics (global_*); flags live in
// uncached device memory.
// (Tensors above the buffer cap - DL gradient buckets - stay on RCCL.)
#include "p2p_device.h"

namespace {

using p2pdev::kMaxBlocks;
using p2pdev::kMaxRanks;
using p2pdev::P2PDesc;
constexpr int kArMaxBlocks = 128;   // blocks of one all-reduce launch (<= kMaxBlocks flag slots)
constexpr int kThreads = 256;

enum Op : int { kSum = 0, kMax = 1 };

template <typename T, int OP>
__device__ __forceinline__ T combine(T a, T b) {
  if constexpr (OP == kSum) return a + b;
  else return a > b ? a : b;
}

// 16-byte vector of T
template <typename T>
struct Vec {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};

template <typename T, int OP>
__device__ __forceinline__ Vec<T> vcombine(const Vec<T>& a, const Vec<T>& b) {
  Vec<T> r;
#pragma unroll
  for (int i = 0; i < Vec<T>::N; ++i) r.v[i] = combine<T, OP>(a.v[i], b.v[i]);
  return r;
}

// a peer's (or this rank's) symmetric-buffer bytes: system-scope loads
template <typename T>
__device__ __forceinline__ Vec<T> vload(const void* p) {
  Vec<T> r;
  const uint4 u = p2pdev::ld_sys16(p);
  __builtin_memcpy(&r, &u, 16);
  return r;
}

template <typename T>
__device__ __forceinline__ void vstore(void* p, const Vec<T>& x) {
  uint4 u;
  __builtin_memcpy(&u, &x, 16);
  *reinterpret_cast<uint4*>(p) = u;
}

template <typename T, int OP, int W>
__device__ void reduce_chunk(const P2PDesc& d, char* data, int64_t parity_off, int64_t v0, int64_t v1) {
  // out[v] = sym_0[v] (+) sym_1[v] (+) ... in rank order; W = world (compile-time for the unroll)
  const char* src[W];
#pragma unroll
  for (int r = 0; r < W; ++r) src[r] = static_cast<const char*>(d.sym[r]) + parity_off;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads) {
    Vec<T> x[W];
#pragma unroll
    for (int r = 0; r < W; ++r) x[r] = vload<T>(src[r] + v * 16);
    Vec<T> acc = x[0];
#pragma unroll
    for (int r = 1; r < W; ++r) acc = vcombine<T, OP>(acc, x[r]);
    vstore<T>(data + v * 16, acc);
  }
}

template <typename T, int OP>
__device__ void reduce_tail(const P2PDesc& d, T* data, int64_t parity_off, int64_t e0, int64_t e1) {
  for (int64_t e = e0 + threadIdx.x; e < e1; e += kThreads) {
    T acc = p2pdev::ld_sys(reinterpret_cast<const T*>(static_cast<const char*>(d.sym[0]) + parity_off) + e);
    for (int r = 1; r < d.world; ++r)
      acc = combine<T, OP>(acc, p2pdev::ld_sys(reinterpret_cast<const T*>(static_cast<const char*>(d.sym[r]) +
                                                                         parity_off) + e));
    data[e] = acc;
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void p2p_allreduce_kernel(P2PDesc d, T* data, int64_t nelem, int nblocks) {
  __shared__ uint32_t s_epoch;
  const int b = blockIdx.x;
  const uint32_t e = p2pdev::begin_epoch(d, &s_epoch);
  const int64_t parity_off = (int64_t)(e & 1u) * d.cap;
  const int64_t nbytes = nelem * (int64_t)sizeof(T);
  const int64_t nvec = nbytes / 16;
  const int64_t per = (nvec + nblocks - 1) / nblocks;
  const int64_t v0 = min<int64_t>(nvec, (int64_t)b * per), v1 = min<int64_t>(nvec, v0 + per);
  // tail elements (bytes past the last full 16-B vector) belong to the last block
  const int64_t t0 = nvec * 16 / (int64_t)sizeof(T);
  const bool tail = (b == nblocks - 1) && t0 < nelem;

  // 1. my chunk into my symmetric buffer
  char* mine = static_cast<char*>(d.sym[d.rank]) + parity_off;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads)
    p2pdev::st_sys16(mine + v * 16, *reinterpret_cast<const uint4*>(reinterpret_cast<char*>(data) + v * 16));
  if (tail)
    for (int64_t i = t0 + threadIdx.x; i < nelem; i += kThreads) p2pdev::st_sys(reinterpret_cast<T*>(mine) + i, data[i]);

  // 2. + 3. publish chunk b to every rank and wait for every rank's chunk b
  p2pdev::post_wait(d, b, e);

  // 4. reduce chunk b over the ranks, in rank order
  char* out = reinterpret_cast<char*>(data);
  switch (d.world) {
    case 2: reduce_chunk<T, OP, 2>(d, out, parity_off, v0, v1); break;
    case 3: reduce_chunk<T, OP, 3>(d, out, parity_off, v0, v1); break;
    case 4: reduce_chunk<T, OP, 4>(d, out, parity_off, v0, v1); break;
    case 5: reduce_chunk<T, OP, 5>(d, out, parity_off, v0, v1); break;
    case 6: reduce_chunk<T, OP, 6>(d, out, parity_off, v0, v1); break;
    case 7: reduce_chunk<T, OP, 7>(d, out, parity_off, v0, v1); break;
    default: reduce_chunk<T, OP, 8>(d, out, parity_off, v0, v1); break;
  }
  if (tail) reduce_tail<T, OP>(d, data, parity_off, t0, nelem);

  // 5. the last block to finish advances the epoch for the next launch
  p2pdev::finish(d, nblocks, e);
}

template <typename T, int OP>
int launch(const P2PDesc& d, void* data, int64_t nelem, hipStream_t st) {
  const int64_t nbytes = nelem * (int64_t)sizeof(T);
  if (nbytes > d.cap) return kBadArg;
  // ~16 KB per block (each block reads world x that over the links), <= kMaxBlocks
  int nblocks = (int)std::min<int64_t>(kArMaxBlocks, std::max<int64_t>(1, (nbytes + 16383) / 16384));
  hipLaunchKernelGGL((p2p_allreduce_kernel<T, OP>), dim3(nblocks), dim3(kThreads), 0, st, d,
                     static_cast<T*>(data), nelem, nblocks);
  return launch_status();
}

}  // namespace

// dtype codes: 0 int64, 1 float32, 2 float64, 3 int32; op: 0 sum, 1 max
H2OMX_API int h2omx_p2p_allreduce(const void* desc, void* data, int64_t nelem, int dtype, int op, hipStream_t st) {
  if (desc == nullptr || data == nullptr || nelem < 0) return kBadArg;
  if (nelem == 0) return kOk;
  const P2PDesc& d = *static_cast<const P2PDesc*>(desc);
  if (d.world < 2 || d.world > kMaxRanks || d.rank < 0 || d.rank >= d.world) return kBadArg;
  if ((reinterpret_cast<uintptr_t>(data) & 15u) != 0) return kBadArg;
  switch (dtype * 2 + op) {
    case 0: return launch<int64_t, kSum>(d, data, nelem, st);
    case 1: return launch<int64_t, kMax>(d, data, nelem, st);
    case 2: return launch<float, kSum>(d, data, nelem, st);
    case 3: return launch<float, kMax>(d, data, nelem, st);
    case 4: return launch<double, kSum>(d, data, nelem, st);
    case 5: return launch<double, kMax>(d, data, nelem, st);
    case 6: return launch<int32_t, kSum>(d, data, nelem, st);
    case 7: return launch<int32_t, kMax>(d, data, nelem, st);
    default: return kBadArg;
  }
}

H2OMX_API int h2omx_p2p_desc_bytes() { return (int)sizeof(P2PDesc); }

// wall_clock64() rate of the current device in kHz (timeout conversion)
H2OMX_API int h2omx_p2p_clock_khz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return -1;
  return khz;
}
H2OMX_API int h2omx_p2p_max_ranks() { return kMaxRanks; }
H2OMX_API int64_t h2omx_p2p_flags_bytes() { return (int64_t)p2pdev::kFlagWords * sizeof(uint32_t); }

// Symmetric-buffer allocation: kind 0 plain (coarse-grained) device memory,
// 1 uncached (the flags), 2 fine-grained (the default data buffers: coherent
// with peer reads at system scope, no reliance on remote-L2 write-back).
// Zeroed; returns the device pointer through *out.
H2OMX_API int h2omx_p2p_alloc(int64_t bytes, int kind, void** out) {
  if (out == nullptr || bytes <= 0 || kind < 0 || kind > 2) return kBadArg;
  void* p = nullptr;
  hipError_t rc = kind == 1   ? hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached)
                  : kind == 2 ? hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocFinegrained)
                              : hipMalloc(&p, (size_t)bytes);
  if (rc != hipSuccess) return kLaunchFailed;
  if (hipMemset(p, 0, (size_t)bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return kLaunchFailed;
  }
  *out = p;
  return kOk;
}

// Pinned, device-mapped host words (the error mirror the host polls without
// a device synchronisation): *host is the CPU address, *dev the GPU one.
H2OMX_API int h2omx_p2p_host_alloc(int64_t bytes, void** host, void** dev) {
  if (host == nullptr || dev == nullptr || bytes <= 0) return kBadArg;
  void* h = nullptr;
  if (hipHostMalloc(&h, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return kLaunchFailed;
  __builtin_memset(h, 0, (size_t)bytes);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return kLaunchFailed;
  }
  *host = h;
  *dev = d;
  return kOk;
}

H2OMX_API int h2omx_p2p_host_free(void* h) { return hipHostFree(h) == hipSuccess ? kOk : kLaunchFailed; }

H2OMX_API int h2omx_p2p_free(void* p) { return hipFree(p) == hipSuccess ? kOk : kLaunchFailed; }

H2OMX_API int h2omx_p2p_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

H2OMX_API int h2omx_p2p_get_handle(void* p, void* handle_out) {
  if (p == nullptr || handle_out == nullptr) return kBadArg;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) return kLaunchFailed;
  __builtin_memcpy(handle_out, &h, sizeof(h));
  return kOk;
}

H2OMX_API int h2omx_p2p_open_handle(const void* handle, void** out) {
  if (handle == nullptr || out == nullptr) return kBadArg;
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return kLaunchFailed;
  *out = p;
  return kOk;
}

H2OMX_API int h2omx_p2p_close_handle(void* p) { return hipIpcCloseMemHandle(p) == hipSuccess ? kOk : kLaunchFailed; }

// Let this device map every other visible device's memory (xGMI); best effort.
H2OMX_API int h2omx_p2p_enable_peers() {
  int n = 0, cur = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || hipGetDevice(&cur) != hipSuccess) return kLaunchFailed;
  for (int i = 0; i < n; ++i) {
    if (i == cur) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, cur, i) == hipSuccess && can) {
      hipError_t rc = hipDeviceEnablePeerAccess(i, 0);
      if (rc != hipSuccess && rc != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    }
  }
  return kOk;
}
