// Device side of the one-shot peer-to-peer exchange (shared by the P2P
// all-reduce in p2p_kernels.hip and the fused multi-rank tree kernels in
// tree_kernels.hip: the tree level's slab reduce + reduce-scatter + split scan
// and the leaf finalisation run as ONE launch each on N ranks, exactly as on one).
//
// Protocol of one collective (every rank launches the same grid):
//   * thread 0 of each block reads the epoch e = ctrl[0] + 1 (the previous
//     collective's last block advanced ctrl[0]);
//   * block b writes (pushes) its payload into the symmetric buffer of the
//     rank(s) that consume it, then posts e into flags[r][b][rank] of every
//     rank r, and waits until its own flags[b][*] hold >= e from every rank
//     (bounded by a wall-clock timeout);
//   * block b reads what was pushed to it, from its OWN symmetric buffer;
//   * the last block to finish advances ctrl[0] to e.
// A rank is at most one collective ahead of any peer (it needs every peer's
// post of the current epoch), so the parity it overwrites was fully read.
//
// Memory model (system scope, no cache maintenance).  Every payload byte is
// stored WRITE-THROUGH at system scope (`st_sys`: global_store ... sc0 sc1, the
// lowering of a relaxed system-scope atomic store) and every storing wave
// drains its stores (`s_waitcnt vmcnt(0)`) before the workgroup barrier behind
// which one wave stores the flags (relaxed system-scope stores).  Every load of
// payload that another rank or workgroup wrote is a system-scope load
// (`ld_sys`: global_load ... sc0 sc1), issued only after the poll of the flag
// matched (the polling wave's loads are in order behind its waited poll; the
// other waves load after the workgroup barrier that wave joins).  So no L2
// write-back (`buffer_wbl2`) and no invalidate (`buffer_inv`) is needed: the
// payload never sits dirty in a cache the reader cannot see, and the reader
// never hits a stale line.  Round 5 used plain payload stores behind a
// system-scope release fence (an L2 write-back per block) and an acquire fence
// (an L2 + L1 invalidate per block) after the poll; `profiles/r6/` records the
// cost of those fences in the N-rank level.  Flags are uncached device memory;
// the symmetric data buffers are fine-grained by default (parallel/p2p.py).
// All stores are vector-memory stores/atomics.
//
// Failure: a poll that times out sets ctrl[2] (and the pinned host word
// host_err, which the host reads without a device sync), writes the abort
// word of every rank's flag buffer, and the block goes on with whatever the
// buffers hold; every later collective of any rank that sees its ctrl[2] or
// its abort word set no longer waits (and records the failure), so a lost
// or late peer drains its stream in microseconds instead of finishing with
// sums that happen to satisfy its polls, and each host raises at its next
// check (parallel/comm.py, Comm._check).  host_err: 1 own timeout, 2 a
// peer's abort.
//
// Loopback: one process standing in for `world` ranks (every sym / flags
// pointer is its own; posts go to every rank slot).  The N-rank launch
// sequence then runs on one GPU - the strong-scaling proxy of bench.py.
#pragma once
#include "common.h"

namespace p2pdev {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;   // flag slots per rank (blocks of one collective)
// flags[kDoneBase + r]: rank r finished its share of a reduce-scatter launch
// (posted by that launch's last block; the consumer launch polls all N)
constexpr int kDoneBase = kMaxBlocks * kMaxRanks;
constexpr int kAbortWord = kDoneBase + kMaxRanks;   // flags[kAbortWord]: set by a peer that timed out
constexpr int kFlagWords = kAbortWord + 16;

struct P2PDesc {
  void* sym[kMaxRanks];        // symmetric data buffers (2 parities x cap bytes + tables), peer-mapped
  uint32_t* flags[kMaxRanks];  // flags[kMaxBlocks][kMaxRanks] + done words per rank, peer-mapped
  uint32_t* ctrl;              // local: [0] epoch, [1] finish ticket, [2] error, [3] timeouts
  uint32_t* host_err;          // pinned host word mirrored from ctrl[2] (nullptr: none)
  int64_t cap;                 // bytes per parity
  int64_t timeout_ticks;       // wall_clock64 ticks before a poll gives up
  int32_t world;
  int32_t rank;
  int32_t loopback;            // 1: this process stands in for every rank
  int32_t pad;
};

// ---- system-scope payload access (write-through stores, coherent loads) ----
template <typename T>
__device__ __forceinline__ void st_sys(T* p, T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "8- or 4-byte payload words");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T ld_sys(const T* p) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "8- or 4-byte payload words");
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys16(void* p, const uint4& v) {
  unsigned long long* q = static_cast<unsigned long long*>(p);
  st_sys(q, (unsigned long long)v.x | ((unsigned long long)v.y << 32));
  st_sys(q + 1, (unsigned long long)v.z | ((unsigned long long)v.w << 32));
}
__device__ __forceinline__ uint4 ld_sys16(const void* p) {
  const unsigned long long* q = static_cast<const unsigned long long*>(p);
  const unsigned long long a = ld_sys(q), b = ld_sys(q + 1);
  return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

// epoch of the collective this launch performs (thread 0 reads, block shares)
__device__ __forceinline__ uint32_t begin_epoch(const P2PDesc& d, uint32_t* s_epoch) {
  if (threadIdx.x == 0) *s_epoch = d.ctrl[0] + 1u;
  __syncthreads();
  return *s_epoch;
}

__device__ __forceinline__ char* parity_base(const P2PDesc& d, int r, uint32_t e) {
  return static_cast<char*>(d.sym[r]) + (int64_t)(e & 1u) * d.cap;
}

// a stream that already lost a peer, or was told so by one, no longer waits
// (its results are discarded by the host); lane 0 records a peer's abort
__device__ __forceinline__ bool failed_state(const P2PDesc& d, int lane) {
  const bool own_fail = __hip_atomic_load(d.ctrl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  const bool peer_abort =
      __hip_atomic_load(d.flags[d.rank] + kAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
  if (peer_abort && !own_fail && lane == 0) {
    __hip_atomic_store(d.ctrl + 2, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d.host_err != nullptr) __hip_atomic_store(d.host_err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return own_fail || peer_abort;
}

// One wave: poll the N words `my[lane]` (lane < world) until each holds >= e.
// On timeout every rank is told (abort word) and the failure is recorded.
__device__ __forceinline__ void wave_wait(const P2PDesc& d, const uint32_t* my, uint32_t e) {
  const int lane = threadIdx.x & (kWave - 1);
  if (failed_state(d, lane)) return;
  const uint64_t t_start = wall_clock64();
  bool timed_out = false;
  for (;;) {
    const uint32_t f = lane < d.world ? __hip_atomic_load(my + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : e;
    if (__all((int32_t)(f - e) >= 0)) break;
    if ((int64_t)(wall_clock64() - t_start) > d.timeout_ticks) {
      timed_out = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (timed_out) {
    // tell every rank (the late one included: it must not later finish on
    // flags this rank posted after giving up)
    if (lane < d.world && !d.loopback)
      __hip_atomic_store(d.flags[lane] + kAbortWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (lane == 0) {
      __hip_atomic_store(d.ctrl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicAdd(d.ctrl + 3, 1u);
      if (d.host_err != nullptr) __hip_atomic_store(d.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Every wave of the block calls this after its payload stores (st_sys): each
// drains its own stores, then - behind the barrier - wave 0 posts e into
// word `slot` of rank r's flag buffer for every rank r (its own rank index,
// or in loopback every rank index).
__device__ __forceinline__ void post(const P2PDesc& d, int slot, uint32_t e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    if (lane < d.world) {
      const int src = d.loopback ? lane : d.rank;
      __hip_atomic_store(d.flags[lane] + slot * kMaxRanks + src, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Whole block: wait until every rank posted e into this rank's slot `slot`;
// the block leaves with every rank's payload for that slot readable (ld_sys).
__device__ __forceinline__ void wait(const P2PDesc& d, int slot, uint32_t e) {
  if (threadIdx.x < kWave) wave_wait(d, d.flags[d.rank] + slot * kMaxRanks, e);
  __syncthreads();
}

// post + wait of the same slot (the all-to-all exchange of block b's chunk)
__device__ __forceinline__ void post_wait(const P2PDesc& d, int b, uint32_t e) {
  post(d, b, e);
  wait(d, b, e);
}

// The last block of the launch advances the epoch for the next collective.
// With `done`, it also posts this rank's done word kDoneBase + rank (loopback:
// every rank's) to every rank: the consumer launch (wait_done) then knows the
// whole grid's payload pushes landed.  Every wave of every block drained its
// stores before the block's ticket (agent-scope atomic), and the last block
// posts only after its ticket returned last.
// Returns (to every thread) whether this block was the last one.
__device__ __forceinline__ bool finish(const P2PDesc& d, int nblocks, uint32_t e, bool done = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    const uint32_t t = atomicAdd(d.ctrl + 1, 1u);
    s_last = t == (uint32_t)nblocks - 1;
    if (s_last) {
      d.ctrl[1] = 0u;
      d.ctrl[0] = e;
    }
  }
  __syncthreads();
  const bool last = s_last != 0;
  if (done && last && threadIdx.x < d.world) {
    const int lane = threadIdx.x;
    const int src = d.loopback ? lane : d.rank;
    __hip_atomic_store(d.flags[lane] + kDoneBase + src, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return last;
}

// Consumer of a `finish(.., done = true)` launch (the NEXT kernel on the
// stream): epoch = ctrl[0] (already advanced), one wave waits for every rank's
// done word, the block leaves with every pushed byte readable (ld_sys).
__device__ __forceinline__ uint32_t wait_done(const P2PDesc& d, uint32_t* s_epoch) {
  if (threadIdx.x == 0) *s_epoch = d.ctrl[0];
  __syncthreads();
  const uint32_t e = *s_epoch;
  if (threadIdx.x < kWave) wave_wait(d, d.flags[d.rank] + kDoneBase, e);
  __syncthreads();
  return e;
}

}  // namespace p2pdev
