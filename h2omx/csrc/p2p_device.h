// Device side of the one-shot peer-to-peer exchange (shared by the P2P
// all-reduce in p2p_kernels.hip and the fused multi-rank tree kernels in
// tree_kernels.hip: the tree level's slab reduce + exchange + split scan and
// the leaf finalisation run as ONE launch each on N ranks, exactly as on one).
//
// Protocol of one collective (every rank launches the same grid):
//   * thread 0 of each block reads the epoch e = ctrl[0] + 1 (the previous
//     collective's last block advanced ctrl[0]);
//   * block b writes its chunk into its own symmetric buffer at parity e & 1,
//     then wave 0 releases at system scope and posts e into flags[r][b][rank]
//     of every rank r, and polls its own flags[b][*] until every rank posted
//     >= e (bounded by a wall-clock timeout);
//   * block b reads the chunk of every rank's buffer in rank order;
//   * the last block to finish advances ctrl[0] to e.
// A rank is at most one collective ahead of any peer (it needs every peer's
// post of the current epoch), so the parity it overwrites was fully read.
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
//
// Memory: flags are uncached device memory; the symmetric data buffers are
// fine-grained by default (parallel/p2p.py), so peer reads over xGMI never
// hit a stale remote-L2 line.  All stores are vector-memory stores/atomics.
#pragma once
#include "common.h"

namespace p2pdev {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;   // flag slots per rank (blocks of one collective)
constexpr int kAbortWord = kMaxBlocks * kMaxRanks;   // flags[kAbortWord]: set by a peer that timed out
constexpr int kFlagWords = kAbortWord + 16;

struct P2PDesc {
  void* sym[kMaxRanks];        // symmetric data buffers (2 parities x cap bytes), peer-mapped
  uint32_t* flags[kMaxRanks];  // flags[kMaxBlocks][kMaxRanks] per rank, peer-mapped
  uint32_t* ctrl;              // local: [0] epoch, [1] finish ticket, [2] error, [3] timeouts
  uint32_t* host_err;          // pinned host word mirrored from ctrl[2] (nullptr: none)
  int64_t cap;                 // bytes per parity
  int64_t timeout_ticks;       // wall_clock64 ticks before a poll gives up
  int32_t world;
  int32_t rank;
  int32_t loopback;            // 1: this process stands in for every rank
  int32_t pad;
};

// epoch of the collective this launch performs (thread 0 reads, block shares)
__device__ __forceinline__ uint32_t begin_epoch(const P2PDesc& d, uint32_t* s_epoch) {
  if (threadIdx.x == 0) *s_epoch = d.ctrl[0] + 1u;
  __syncthreads();
  return *s_epoch;
}

__device__ __forceinline__ char* parity_base(const P2PDesc& d, int r, uint32_t e) {
  return static_cast<char*>(d.sym[r]) + (int64_t)(e & 1u) * d.cap;
}

// Called by the whole block after it wrote its chunk (each thread's stores
// issued).  Wave 0 publishes and waits; the block leaves with every rank's
// chunk b visible.
__device__ __forceinline__ void post_wait(const P2PDesc& d, int b, uint32_t e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    // system-scope release: this XCD's L2 written back before the flag
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane < d.world) {
      const int slot = d.loopback ? lane : d.rank;
      __hip_atomic_store(d.flags[lane] + b * kMaxRanks + slot, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // a stream that already lost a peer, or was told so by one, no longer waits
    // (its results are discarded by the host)
    const bool own_fail = __hip_atomic_load(d.ctrl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    const bool peer_abort =
        __hip_atomic_load(d.flags[d.rank] + kAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    const bool failed = own_fail || peer_abort;
    if (peer_abort && !own_fail && lane == 0) {
      __hip_atomic_store(d.ctrl + 2, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d.host_err != nullptr)
        __hip_atomic_store(d.host_err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint32_t* my = d.flags[d.rank] + b * kMaxRanks;
    const uint64_t t_start = wall_clock64();
    bool timed_out = false;
    while (!failed) {
      const uint32_t f =
          lane < d.world ? __hip_atomic_load(my + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : e;
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
        if (d.host_err != nullptr)
          __hip_atomic_store(d.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// the last block of the launch advances the epoch for the next collective
__device__ __forceinline__ void finish(const P2PDesc& d, int nblocks, uint32_t e) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t done = atomicAdd(d.ctrl + 1, 1u);
    if (done == (uint32_t)nblocks - 1) {
      d.ctrl[1] = 0u;
      d.ctrl[0] = e;
    }
  }
}

}  // namespace p2pdev
