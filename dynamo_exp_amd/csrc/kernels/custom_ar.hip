// One-shot all-reduce over xGMI peer memory for latency-bound TP messages
// (decode: [B, 4096] bf16, <= a few MiB) -- SURVEY §2.14 / §5.8(a).
//
// A ring all-reduce moves 2(N-1)/N of the message over ONE link per
// direction; on the fully connected 8-GPU xGMI mesh a one-shot reduce reads
// every peer's shard over its own link (7 links in parallel) and finishes in
// one step:
//   1. every rank has its input in its own registered buffer (IPC-shared);
//   2. start barrier: block b of rank r stores `2e` into slot [r][b] of every
//      peer's signal array and waits until its own slots [p][b] reach 2e
//      (per-block flags: no grid-wide sync needed);
//   3. each thread reads its 16-B vectors from all `world` buffers, sums in
//      fp32 in rank order (identical result on every rank), stores bf16;
//   4. end barrier with `2e+1`, so no rank overwrites its buffer for the next
//      call while a peer is still reading it.
// The call index e lives on the device: block b of a rank keeps its own
// counter after its flag slots and bumps it once per launch, so a launch
// captured in a hipGraph gets a fresh e on every replay (a host-side value
// would be frozen into the graph and the barrier would pass stale flags).
// Every rank runs the same sequence of all-reduces, so the counters agree.
// Spins are bounded (an unresponsive peer sets *err and the kernel returns
// instead of hanging the GPU).  Signals live in uncached device memory so
// flag stores/loads go straight to the fabric.
#include "common.h"

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;
constexpr int kThreads = 512;
constexpr int kSpinLimit = 1 << 22;  // ~seconds of s_sleep(1) polling

struct Peers {
  const bf16_t* bufs[kMaxRanks];
  uint32_t* sig[kMaxRanks];  // each [kMaxRanks][kMaxBlocks] u32
};

__device__ __forceinline__ void barrier(const Peers& p, int rank, int world, uint32_t value, int* err) {
  const int b = blockIdx.x;
  if ((int)threadIdx.x < world) {
    const int peer = threadIdx.x;
    __hip_atomic_store(p.sig[peer] + rank * kMaxBlocks + b, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = p.sig[rank] + peer * kMaxBlocks + b;
    int spins = 0;
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < value) {
      if (++spins > kSpinLimit) {
        atomicExch(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(kThreads) custom_ar_one_shot(bf16_t* __restrict__ out, Peers p, int rank, int world,
                                                                int64_t n_vec, int* err) {
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) {
    uint32_t* ctr = p.sig[rank] + kMaxRanks * kMaxBlocks + blockIdx.x;  // this block's call counter
    // a vector-memory atomic (never a scalar-cache read of a stale counter)
    s_epoch = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  barrier(p, rank, world, 2 * epoch, err);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int r = 0; r < world; ++r) {
      const u16x8 v = reinterpret_cast<const u16x8*>(p.bufs[r])[i];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        acc[2 * w] += bf16lo(v.w[w]);
        acc[2 * w + 1] += bf16hi(v.w[w]);
      }
    }
    u16x8 o;
#pragma unroll
    for (int w = 0; w < 4; ++w) o.w[w] = pack_bf16x2(acc[2 * w], acc[2 * w + 1]);
    reinterpret_cast<u16x8*>(out)[i] = o;
  }
  barrier(p, rank, world, 2 * epoch + 1, err);
}

}  // namespace

// bufs/sigs: `world` device pointers (peer ones opened from IPC handles).
// n: elements (bf16), multiple of 8.  blocks <= 64 and the same on every call
// (the per-block call counters are indexed by block).  `epoch` is unused (kept
// for ABI stability; the call index is counted on the device).
extern "C" int dx_custom_ar(void* out, const void* const* bufs, void* const* sigs, int rank, int world, int64_t n,
                            uint32_t /*epoch*/, int blocks, int* err, hipStream_t stream) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || n % 8 || blocks < 1 || blocks > kMaxBlocks)
    return -1;
  Peers p{};
  for (int r = 0; r < world; ++r) {
    p.bufs[r] = (const bf16_t*)bufs[r];
    p.sig[r] = (uint32_t*)sigs[r];
  }
  custom_ar_one_shot<<<blocks, kThreads, 0, stream>>>((bf16_t*)out, p, rank, world, n / 8, err);
  return (int)hipGetLastError();
}

// Signal arrays: uncached device memory, zeroed: [kMaxRanks][kMaxBlocks] flags
// followed by [kMaxBlocks] per-block call counters.
extern "C" int dx_custom_ar_alloc_signals(void** ptr) {
  const size_t bytes = sizeof(uint32_t) * (kMaxRanks * kMaxBlocks + kMaxBlocks);
  if (hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached) != hipSuccess) return -1;
  return hipMemset(*ptr, 0, bytes) == hipSuccess ? 0 : -2;
}
