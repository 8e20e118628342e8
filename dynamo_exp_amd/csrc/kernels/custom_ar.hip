// One-shot all-reduce over xGMI peer memory for latency-bound TP messages
// (decode: [B, 4096] bf16, <= a few MiB) -- SURVEY §2.14 / §5.8(a).
//
// A ring all-reduce moves 2(N-1)/N of the message over ONE link per
// direction; on the fully connected 8-GPU xGMI mesh a one-shot reduce reads
// every peer's shard over its own link (7 links in parallel) and finishes in
// one step:
//   1. every rank has its input in its own registered buffer (IPC-shared);
//   2. start barrier: block b of rank r stores `3e` into slot [r][b] of every
//      peer's signal array and waits until its own slots [p][b] reach 3e
//      (per-block flags: no grid-wide sync needed);
//   3. each thread reads its 16-B vectors from all `world` buffers, sums in
//      fp32 in rank order (identical result on every rank), stores bf16;
//   4. end barrier with `3e+2`, so no rank overwrites its buffer for the next
//      call while a peer is still reading it.  (3e+1 is the two-shot kernel's
//      middle barrier.)
// The call index e lives on the device: block b of a rank keeps its own
// counter after its flag slots and bumps it once per launch, so a launch
// captured in a hipGraph gets a fresh e on every replay (a host-side value
// would be frozen into the graph and the barrier would pass stale flags).
// Every rank runs the same sequence of all-reduces, so the counters agree.
// Spins are bounded: an unresponsive peer sets *err and the kernel returns
// without reading or writing any more data (the host polls *err after every
// engine step and fails the worker: parallel/custom_ar.py check()).  The flag
// is sticky and read at kernel entry and inside every spin: once one barrier
// of a rank has failed, its barrier sequence no longer matches its peers', so
// every later launch on that rank returns at once instead of spinning out its
// own timeout (round 4: a graph of 40 collectives after one miss stalled
// 40 x 20 s).  Its peers then miss this rank's flags, time out once and
// fail fast the same way; the host turns the flag into a worker failure.
// Signals live in uncached device memory so flag stores/loads go straight to
// the fabric.
#include "common.h"

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;
constexpr int kThreads = 512;
// a peer that has not arrived after timeout_ms is declared gone (wall clock:
// s_memrealtime ticks at 100 MHz); 0 selects the default.  Generous on
// purpose: ranks of one TP group reach a collective at different host times
// (weight loading, a long prefill step's host work)
constexpr uint32_t kDefaultTimeoutMs = 20000;
constexpr uint64_t kTicksPerMs = 100000;

struct Peers {
  const bf16_t* bufs[kMaxRanks];
  uint32_t* sig[kMaxRanks];  // each [kMaxRanks][kMaxBlocks] u32
};

// Returns false when a peer did not arrive within the spin limit (then *err
// is set and the caller must not touch peer buffers any more).
__device__ __forceinline__ int read_err(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool barrier(const Peers& p, int rank, int world, uint32_t value, int* err,
                                        uint64_t timeout_ticks) {
  __shared__ int s_fail;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) s_fail = 0;
  __syncthreads();
  if ((int)threadIdx.x < world) {
    const int peer = threadIdx.x;
    // system-scope release: writes back this GPU's L2 (the data peers read
    // next, stored by earlier kernels or by this block before the barrier)
    __hip_atomic_store(p.sig[peer] + rank * kMaxBlocks + b, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = p.sig[rank] + peer * kMaxBlocks + b;
    int spins = 0;
    uint64_t t0 = 0;
    // system-scope acquire: no stale copy of a peer's lines survives in L2
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < value) {
      if ((++spins & 1023) == 0) {  // read the clock (and the sticky flag) only now and then
        if (read_err(err)) {  // another block of this rank already gave up
          s_fail = 1;
          break;
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) {
          t0 = now;
        } else if (now - t0 > timeout_ticks) {
          atomicExch(err, 1);
          s_fail = 1;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return s_fail == 0;
}

// Bumps this block's call counter; returns 0 when this rank's sticky error
// flag is set (the launch must return without touching anything else).
__device__ __forceinline__ uint32_t next_epoch(const Peers& p, int rank, const int* err) {
  __shared__ uint32_t s_epoch;
  if (threadIdx.x == 0) {
    uint32_t* ctr = p.sig[rank] + kMaxRanks * kMaxBlocks + blockIdx.x;  // this block's call counter
    // a vector-memory atomic (never a scalar-cache read of a stale counter)
    const uint32_t e = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    s_epoch = read_err(err) ? 0u : e;
  }
  __syncthreads();
  return s_epoch;
}

__device__ __forceinline__ u16x8 sum_ranks(const Peers& p, int world, int64_t i) {
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
  return o;
}

// One-shot: every rank reads the whole message from every peer (decode sizes).
__global__ void __launch_bounds__(kThreads) custom_ar_one_shot(bf16_t* __restrict__ out, Peers p, int rank, int world,
                                                                int64_t n_vec, int* err, uint64_t tmo) {
  const uint32_t epoch = next_epoch(p, rank, err);
  if (epoch == 0) return;  // this rank already failed a barrier
  if (!barrier(p, rank, world, 3 * epoch, err, tmo)) return;  // a late peer: never read half-written buffers
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride)
    reinterpret_cast<u16x8*>(out)[i] = sum_ranks(p, world, i);
  barrier(p, rank, world, 3 * epoch + 2, err, tmo);
}

// Two-shot (reduce-scatter + all-gather through the registered buffers) for
// prefill-size messages: rank r sums chunk r over all ranks and stores it in
// place in ITS OWN buffer (only rank r reads chunk r of any buffer in phase 1,
// and each element is read and written by the same thread), then every rank
// copies chunk s from rank s's buffer.  Each rank moves 2(N-1)/N of the
// message over its N-1 links in parallel instead of the full message per
// peer.  The same vector -> block mapping in both phases means the per-block
// barrier between them orders every phase-2 read after its phase-1 write.
__global__ void __launch_bounds__(kThreads) custom_ar_two_shot(bf16_t* __restrict__ out, Peers p, int rank, int world,
                                                                int64_t n_vec, int* err, uint64_t tmo) {
  const uint32_t epoch = next_epoch(p, rank, err);
  if (epoch == 0) return;  // this rank already failed a barrier
  if (!barrier(p, rank, world, 3 * epoch, err, tmo)) return;
  const int64_t chunk = (n_vec + world - 1) / world;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  {
    const int64_t lo = (int64_t)rank * chunk, hi = min(n_vec, lo + chunk);
    u16x8* mine = reinterpret_cast<u16x8*>(const_cast<bf16_t*>(p.bufs[rank]));
    for (int64_t j = t0; lo + j < hi; j += stride) mine[lo + j] = sum_ranks(p, world, lo + j);
  }
  if (!barrier(p, rank, world, 3 * epoch + 1, err, tmo)) return;
  for (int s = 0; s < world; ++s) {
    const int r = (rank + s) % world;  // start with the local chunk, then spread over the links
    const int64_t lo = (int64_t)r * chunk, hi = min(n_vec, lo + chunk);
    const u16x8* src = reinterpret_cast<const u16x8*>(p.bufs[r]);
    for (int64_t j = t0; lo + j < hi; j += stride) reinterpret_cast<u16x8*>(out)[lo + j] = src[lo + j];
  }
  barrier(p, rank, world, 3 * epoch + 2, err, tmo);
}

// All-gather (any dtype, 16-B vectors): every rank's message sits at the start
// of its registered buffer; rank r copies peer s's message into out[s] over
// link s, all peers in parallel (start with the local one, then rotate so the
// 7 links are loaded evenly).  Decode-step TP gathers (vocab-shard sampler
// partials, full logits for top-k/top-p rows) go here instead of RCCL: the
// same device-side epoch as the all-reduces, so it is graph-capturable and
// shares their barrier sequence (every rank issues the same launches).
__global__ void __launch_bounds__(kThreads) custom_ag(uint4* __restrict__ out, Peers p, int rank, int world,
                                                       int64_t n_vec, int* err, uint64_t tmo) {
  const uint32_t epoch = next_epoch(p, rank, err);
  if (epoch == 0) return;
  if (!barrier(p, rank, world, 3 * epoch, err, tmo)) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int s = 0; s < world; ++s) {
    const int r = (rank + s) % world;
    const uint4* src = reinterpret_cast<const uint4*>(p.bufs[r]);
    uint4* dst = out + (int64_t)r * n_vec;
    for (int64_t j = t0; j < n_vec; j += stride) dst[j] = src[j];
  }
  barrier(p, rank, world, 3 * epoch + 2, err, tmo);
}

}  // namespace

// nbytes per rank, multiple of 16; out holds world * nbytes (rank-major).
static uint64_t timeout_ticks(uint32_t timeout_ms) {
  return (uint64_t)(timeout_ms ? timeout_ms : kDefaultTimeoutMs) * kTicksPerMs;
}

extern "C" int dx_custom_ag(void* out, const void* const* bufs, void* const* sigs, int rank, int world,
                            int64_t nbytes, int blocks, int* err, uint32_t timeout_ms, hipStream_t stream) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || nbytes % 16 || blocks < 1 ||
      blocks > kMaxBlocks)
    return -1;
  Peers p{};
  for (int r = 0; r < world; ++r) {
    p.bufs[r] = (const bf16_t*)bufs[r];
    p.sig[r] = (uint32_t*)sigs[r];
  }
  custom_ag<<<blocks, kThreads, 0, stream>>>((uint4*)out, p, rank, world, nbytes / 16, err,
                                             timeout_ticks(timeout_ms));
  return (int)hipGetLastError();
}

// bufs/sigs: `world` device pointers (peer ones opened from IPC handles).
// n: elements (bf16), multiple of 8.  blocks <= 64 and the same on every call
// (the per-block call counters are indexed by block).  The call index is
// counted on the device; timeout_ms bounds every barrier spin (0: default
// 20 s).  err: this rank's sticky failure flag (device int).  two_shot
// selects the reduce-scatter + all-gather kernel (its phase-1 result
// overwrites this rank's registered buffer).
extern "C" int dx_custom_ar(void* out, const void* const* bufs, void* const* sigs, int rank, int world, int64_t n,
                            uint32_t timeout_ms, int blocks, int* err, int two_shot, hipStream_t stream) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || n % 8 || blocks < 1 || blocks > kMaxBlocks)
    return -1;
  Peers p{};
  for (int r = 0; r < world; ++r) {
    p.bufs[r] = (const bf16_t*)bufs[r];
    p.sig[r] = (uint32_t*)sigs[r];
  }
  if (two_shot)
    custom_ar_two_shot<<<blocks, kThreads, 0, stream>>>((bf16_t*)out, p, rank, world, n / 8, err,
                                                         timeout_ticks(timeout_ms));
  else
    custom_ar_one_shot<<<blocks, kThreads, 0, stream>>>((bf16_t*)out, p, rank, world, n / 8, err,
                                                         timeout_ticks(timeout_ms));
  return (int)hipGetLastError();
}

// Signal arrays: uncached device memory, zeroed: [kMaxRanks][kMaxBlocks] flags
// followed by [kMaxBlocks] per-block call counters.
extern "C" int dx_custom_ar_alloc_signals(void** ptr) {
  const size_t bytes = sizeof(uint32_t) * (kMaxRanks * kMaxBlocks + kMaxBlocks);
  if (hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached) != hipSuccess) return -1;
  return hipMemset(*ptr, 0, bytes) == hipSuccess ? 0 : -2;
}
