// Stand-ins for RCCL point-to-point kernels, used by the hardware-queue and
// ordering tests of the P->D KV data plane (tests/test_wire_hazards_gpu.py,
// tools/hwq_probe.py).  Not on any serving path.
//
// Why they exist: an RCCL send / recv is a kernel that occupies its stream's
// hardware queue (AQL queue) until its peer's matching kernel runs.  HIP maps
// a process's streams onto GPU_MAX_HW_QUEUES (4) queues per priority, so a
// spinning receive can sit ahead of unrelated kernels that share its queue.
// These kernels reproduce exactly that occupancy on ONE GPU, where real RCCL
// cannot run two ranks:
//
// * spin_for(ms): one workgroup holds its queue for `ms` milliseconds (a
//   receive whose sender is still computing).
// * wire_recv / wire_send(k): a rendezvous channel with RCCL p2p semantics.
//   Message k of a channel is matched only when both kernels run: the
//   receive announces itself (state 3k+1), the send waits for that, copies
//   its bytes into the channel's wire buffer and marks it full (3k+2), the
//   receive copies them out and frees the slot (3k+3).  Channel state lives
//   in uncached device memory shared between processes over IPC; every spin
//   is bounded by a wall-clock timeout that sets *err (a deadlock is then a
//   test failure, never a hung GPU).
#include "common.h"

namespace {

constexpr uint64_t kTicksPerMs = 100000;  // s_memrealtime: 100 MHz
constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t ld_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// thread 0 spins until *state == want (or the timeout / sticky error); the
// verdict is broadcast through LDS.  Returns false on timeout.
__device__ bool wait_state(const uint32_t* state, uint32_t want, int* err, uint64_t timeout_ticks) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    int ok = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int spins = 0;
    while (ld_acq(state) != want) {
      if ((++spins & 255) == 0) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          ok = 0;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ok = 0;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(2);
    }
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

__global__ void __launch_bounds__(kThreads) spin_for_kernel(uint64_t ticks, uint32_t* done) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    if (done) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(kThreads) wire_recv_kernel(uint32_t* state, const uint4* wire, uint4* dst,
                                                             int64_t n16, uint32_t k, uint64_t timeout_ticks,
                                                             int* err) {
  if (!wait_state(state, 3u * k, err, timeout_ticks)) return;  // previous message consumed
  if (threadIdx.x == 0) st_rel(state, 3u * k + 1u);             // posted
  if (!wait_state(state, 3u * k + 2u, err, timeout_ticks)) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // (system scope by default) fresh lines for every wave
  for (int64_t i = threadIdx.x; i < n16; i += kThreads) dst[i] = wire[i];
  __atomic_thread_fence(__ATOMIC_RELEASE);
  __syncthreads();
  if (threadIdx.x == 0) st_rel(state, 3u * k + 3u);  // slot free
}

__global__ void __launch_bounds__(kThreads) wire_send_kernel(uint32_t* state, uint4* wire, const uint4* src,
                                                             int64_t n16, uint32_t k, uint64_t timeout_ticks,
                                                             int* err) {
  if (!wait_state(state, 3u * k + 1u, err, timeout_ticks)) return;  // receiver posted
  for (int64_t i = threadIdx.x; i < n16; i += kThreads) wire[i] = src[i];
  __atomic_thread_fence(__ATOMIC_RELEASE);  // every wave writes its stores back before the flag
  __syncthreads();
  if (threadIdx.x == 0) st_rel(state, 3u * k + 2u);
}

}  // namespace

extern "C" int dx_spin_for(uint32_t ms, uint32_t* done, hipStream_t st) {
  if (ms > 60000) return 1;
  hipLaunchKernelGGL(spin_for_kernel, dim3(1), dim3(kThreads), 0, st, (uint64_t)ms * kTicksPerMs, done);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int dx_wire_xfer(int send, uint32_t* state, void* wire, void* buf, int64_t nbytes, uint32_t k,
                            uint32_t timeout_ms, int* err, hipStream_t st) {
  if (nbytes % 16 || !state || !wire || !buf || !err || timeout_ms == 0 || timeout_ms > 60000) return 1;
  if (k > 0x55555554u) return 1;  // 3k + 3 must fit in 32 bits
  const uint64_t to = (uint64_t)timeout_ms * kTicksPerMs;
  if (send)
    hipLaunchKernelGGL(wire_send_kernel, dim3(1), dim3(kThreads), 0, st, state, (uint4*)wire, (const uint4*)buf,
                       nbytes / 16, k, to, err);
  else
    hipLaunchKernelGGL(wire_recv_kernel, dim3(1), dim3(kThreads), 0, st, state, (const uint4*)wire, (uint4*)buf,
                       nbytes / 16, k, to, err);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// uncached device memory for channel states / error flags (IPC-shareable)
extern "C" int dx_wire_alloc(void** p, int64_t nbytes) {
  if (hipExtMallocWithFlags(p, (size_t)nbytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  return hipMemset(*p, 0, (size_t)nbytes) == hipSuccess ? 0 : 2;
}
