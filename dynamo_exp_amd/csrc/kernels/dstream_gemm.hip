// Decode projection GEMM for gfx950 with a deep, decoupled weight stream
// (M ~ 16-256 tokens):      y[M, N] = x[M, K] . w[N, K]^T   bf16, fp32 accumulate
//
// A decode projection at M = 128 moves ~M / 2 weight bytes per FLOP-pair:
// weight-bandwidth bound, and by Little's law a CU needs ~100 KB of weight
// bytes in flight to stream at its share of HBM (~25 GB/s per CU at ~2-4 us
// loaded latency; tools/native/gemv_stream_probe.hip measures the curve).
// The earlier small-M kernels kept 24-48 KB in flight because the weight
// prefetch depth was tied to the depth of the LDS ring that stages x
// (round 2's LDS-DMA weight-streaming kernel: both in LDS; round 3's register-streamed variant: both D = 4
// stages; both removed).  Here they are two
// separate rings:
//   * weights bypass LDS: each wave streams ITS OWN 16 R weight rows as MFMA A
//     fragments straight into VGPRs (16 rows x 64 B per global_load_dwordx4,
//     row = lane & 15, k-group = lane >> 4), DW k-steps (64 k each) ahead --
//     DW = 8 keeps 7 steps x 2 R KB per wave in flight (R = 2, 4 waves:
//     112 KB per CU);
//   * x -- small, L2-resident, shared by all waves of the workgroup -- goes
//     through an LDS ring of DX stages (LDS-DMA, 8 token rows x 128 B per
//     1-KB piece, XOR-swizzled 16-B chunks for conflict-free ds_read_b128 B
//     fragments); only the x ring needs the per-step barrier.
//   * one counted vmcnt per step: every step issues the same pattern (NXW x
//     pieces, then 2 R weight loads; prologue slots that have no real x stage
//     issue a throwaway load instead, past-the-end steps re-read the last
//     stage), so "x(t) and w(t) landed" is one constant count; the wait names
//     the step's weight registers "+v" so no MFMA reading them is scheduled
//     above it, and all loads are inline asm (invisible to the compiler's
//     own vmcnt bookkeeping, which would otherwise drain vmcnt(0));
//   * v_mfma_f32_16x16x32_bf16, A = weight rows, B = token rows: every lane
//     ends with 4 consecutive output columns of one token (8-B stores);
//   * K is split over workgroups when the grid needs it: fp32 slabs, summed
//     in slice order (bit-reproducible) by a second small kernel on the same
//     stream -- the kernel boundary is the cross-XCD hand-off; blocks are
//     remapped so the K-slices of one row tile run consecutively on one XCD.
// The engine's warm-up tuner picks (NW, R, T, DW, DX, splits) per decode
// graph size and projection against hipBLASLt and the other kernels
// (models/llama.py tune_gemms).
//
// SILU (round 6, the decode MLP's gate_up with its SwiGLU fused): the weight
// rows are the gate and up projections interleaved in blocks of 32
// (g0..g31, u0..u31, ...; models/llama.py enable_fused_mlp, the prefill
// gemm256 layout).  With R = 2 each wave owns 16 output columns: block b = 0
// streams their 16 gate rows, b = 1 the 16 up rows 32 further, so every lane
// holds silu(g) * u's operands for 4 output columns in acc[0][j] / acc[1][j]
// and y[M, N / 2] is written directly -- no [M, N] intermediate, no separate
// silu_and_mul launch (split-K: the slices' partials go to the slabs by
// weight row and splitk_reduce_silu_kernel applies the SwiGLU after the sum).
//
// (Round 5 had an fp8 (w8a8) form of this kernel; its first GPU launch
// faulted with an illegal address whose cause was never found, so it was
// removed in round 6 rather than shipped behind a flag: w8a8 decode GEMMs run
// on hipBLASLt's fp8 kernels -- profiles/r5_dstream_fp8_fault.txt.)
#include "common.h"

namespace {

constexpr int KS = 64;   // bf16 k per step: one 128-B line per weight / x row
constexpr int LINE = 128;  // bytes of a row per step (bf16: 64 k, fp8: 128 k)

// s_waitcnt vmcnt(n) naming a step's weight registers "+v": no MFMA that reads
// them can be scheduled above the wait
template <int n, int R>
__device__ __forceinline__ void vm_wait_named(bf16x8_t (&cw)[R][2]) {
  constexpr int enc = 0x0F70 | (n & 15) | ((n >> 4) << 14);
  if constexpr (R == 1)
    asm volatile("s_waitcnt %2" : "+v"(cw[0][0]), "+v"(cw[0][1]) : "i"(enc) : "memory");
  else
    asm volatile("s_waitcnt %4" : "+v"(cw[0][0]), "+v"(cw[0][1]), "+v"(cw[1][0]), "+v"(cw[1][1]) : "i"(enc) : "memory");
}

// P (bandwidth probes, wrong results): 1 = no LDS reads / MFMA, 2 = also no x
// DMA (weights + barrier only), 3 = also no barrier (weights only)
__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

template <int NW, int R, int T, int DW, int DX, int P = 0, bool SILU = false>
__global__ void __launch_bounds__(64 * NW) dstream_kernel(bf16_t* __restrict__ y, int64_t ldy,
                                                          const void* __restrict__ x, int64_t ldx,
                                                          const void* __restrict__ w, float* __restrict__ slabs,
                                                          int* __restrict__ tickets, int M, int N, int K,
                                                          int splits) {
  constexpr int ESZ = 2;                  // bytes per element of x and w (bf16)
  constexpr int KE = LINE / ESZ;          // k per step
  constexpr int BM = 16 * T;              // token rows of the x image
  constexpr int BN = NW * 16 * R;         // weight rows per workgroup
  constexpr int SB = BM * LINE;           // x stage bytes
  constexpr int NXP = BM / 8;             // 1-KB x pieces per stage
  constexpr int NXW = (NXP + NW - 1) / NW;  // pieces per wave (uniform; extras re-load a real piece)
  constexpr int PER = NXW + 2 * R;        // vm ops per wave per step
  // Step t needs x(t) and w(t).  x(t) is issued at step t - DX + 1, first in
  // that step; w(t) at step t - DW + 1, last in it.  DW > DX: w(t) is older,
  // so waiting for x(t) covers it -- ops issued after x(t): that step's
  // weights + DX - 2 whole steps.  DW == DX: both in the same step, w(t)
  // last -- ops after it: DX - 2 whole steps.
  constexpr int WAIT = (DW > DX ? 2 * R : 0) + (DX - 2) * PER;
  static_assert(DX >= 2 && DW >= DX && DW % DX == 0, "ring depths");
  static_assert(WAIT < 64 && R <= 2, "vmcnt range / wait operands");
  // DX x stages + a 1-KB sink for the prologue's placeholder pieces + the split-K flag
  __shared__ __attribute__((aligned(16))) char smem[DX * SB + 1024 + 16];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l15 = lane & 15, lq = lane >> 4;

  // ---- block -> (row tile, K-slice); consecutive ids share an XCD
  const int ntn = N / BN, nwg = ntn * splits;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int nt = id / splits, sl = id - nt * splits;
  const int nk = K / KE / splits;
  const int k0 = sl * nk * KE;

  // ---- weight fragments: block b = rows n0w + 16 b + l15, bytes 16 lq (+64) of a step
  // (SILU: wave gw owns output columns 16 gw .. +15; its gate rows start at
  // wrow(0), its up rows 32 further)
  static_assert(!SILU || R == 2, "the SwiGLU form pairs one gate and one up block per wave");
  const int n0w = nt * BN + wave * 16 * R;
  const int gw = nt * NW + wave;
  auto wrow = [&](int b) { return SILU ? 64 * (gw >> 1) + 16 * (gw & 1) + 32 * b : n0w + 16 * b; };
  uint32_t voff[R];
#pragma unroll
  for (int b = 0; b < R; ++b) voff[b] = (uint32_t)((wrow(b) + l15) * K + k0) * (uint32_t)ESZ + 16u * lq;

  // ---- x image pieces of this wave: piece p holds rows 8p .. 8p + 7 (16-B chunk
  // c of a row stores source chunk c ^ swz(row)); rows >= M re-read row M - 1
  auto swz = [](int r) { return (r >> 1) & 7; };
  uint32_t xoff[NXW], xdst[NXW];
#pragma unroll
  for (int i = 0; i < NXW; ++i) {
    const int p = min(wave * NXW + i, NXP - 1);
    const int row = 8 * p + (lane >> 3);
    const int ch = (lane & 7) ^ swz(row);
    xoff[i] = (uint32_t)(min(row, M - 1) * (int)ldx + k0) * (uint32_t)ESZ + (uint32_t)ch * 16u;
    xdst[i] = (uint32_t)p * 1024u;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // x pieces of step s into slot s % DX; s < 0 (prologue slots without a real
  // stage): the same DMA into the 1-KB sink, so every step issues the same ops
  auto issue_x = [&](int s, int slot) {
    const char* xb = static_cast<const char*>(x) + (int64_t)max(0, min(s, nk - 1)) * LINE;
#pragma unroll
    for (int i = 0; i < NXW; ++i) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane(s < 0 ? lds0 + DX * SB : lds0 + slot * SB + xdst[i]);
      uint32_t keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(xoff[i]), "s"(xb), "s"(dst)
          : "memory");
    }
  };
  auto issue_w = [&](int s, bf16x8_t (&wr)[R][2]) {
    const char* wb = static_cast<const char*>(w) + (int64_t)min(s, nk - 1) * LINE;
#pragma unroll
    for (int b = 0; b < R; ++b) {
      asm volatile("global_load_dwordx4 %0, %1, %2 offset:0" : "=v"(wr[b][0]) : "v"(voff[b]), "s"(wb) : "memory");
      asm volatile("global_load_dwordx4 %0, %1, %2 offset:64" : "=v"(wr[b][1]) : "v"(voff[b]), "s"(wb) : "memory");
    }
  };

  // ---- B fragments: token row 16 j + l15, chunk (4 kb + lq) ^ swz(row)
  int xr[2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) xr[kb] = l15 * LINE + (((4 * kb + lq) ^ swz(l15)) << 4);

  f32x4 acc[R][T];
#pragma unroll
  for (int b = 0; b < R; ++b)
#pragma unroll
    for (int j = 0; j < T; ++j) acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8_t wr[DW][R][2];

  auto compute = [&](int slot, bf16x8_t (&cw)[R][2]) {
    const char* s = smem + slot * SB;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      bf16x8_t xf[T];
#pragma unroll
      for (int j = 0; j < T; ++j) xf[j] = *reinterpret_cast<const bf16x8_t*>(s + j * 16 * LINE + xr[kb]);
#pragma unroll
      for (int b = 0; b < R; ++b)
#pragma unroll
        for (int j = 0; j < T; ++j)
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[b][kb], xf[j], acc[b][j], 0, 0, 0);
    }
  };

  // ---- prologue: virtual steps -(DW-1) .. -1 issue x(v + DX - 1) and w(v + DW - 1)
#pragma unroll
  for (int v = -(DW - 1); v < 0; ++v) {
    if constexpr (P < 2) issue_x(v + DX - 1, ((v + DX - 1) % DX + DX) % DX);
    issue_w(v + DW - 1, wr[v + DW - 1]);
  }
  // ---- steady state (nk % DW == 0, host check): step t waits for x(t), w(t),
  // then refills the x slot and the weight slot step t - 1 consumed
  for (int t0 = 0; t0 < nk; t0 += DW) {
#pragma unroll
    for (int u = 0; u < DW; ++u) {
      const int t = t0 + u;
      vm_wait_named<(P >= 2 ? (DX - 2) * 2 * R : WAIT), R>(wr[u]);
      if constexpr (P < 3) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (P < 2) issue_x(t + DX - 1, (u + DX - 1) % DX);
      issue_w(t + DW - 1, wr[(u + DW - 1) % DW]);
      if constexpr (P == 0) compute(u % DX, wr[u]);
      if constexpr (P != 0) {  // keep the weight loads live
#pragma unroll
        for (int b = 0; b < R; ++b) acc[b][0] += __builtin_bit_cast(f32x4, wr[u][b][0]);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's re-reads

  // ---- epilogue: acc[b][j] register e = (weight row wrow(b) + 4 lq + e, token 16 j + l15)
  if constexpr (SILU) {
    if (splits == 1) {
#pragma unroll
      for (int j = 0; j < T; ++j) {
        const int m = 16 * j + l15;
        if (m >= M) continue;
        const f32x4 g = acc[0][j], u = acc[1][j];
        uint2 pk;
        pk.x = pack_bf16x2(silu_f(g[0]) * u[0], silu_f(g[1]) * u[1]);
        pk.y = pack_bf16x2(silu_f(g[2]) * u[2], silu_f(g[3]) * u[3]);
        *reinterpret_cast<uint2*>(y + (int64_t)m * ldy + 16 * gw + 4 * lq) = pk;
      }
      return;
    }
    float* slab = slabs + (int64_t)sl * BM * N;  // by weight row: splitk_reduce_silu_kernel pairs them
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
      for (int b = 0; b < R; ++b)
        *reinterpret_cast<f32x4*>(slab + (int64_t)(16 * j + l15) * N + wrow(b) + 4 * lq) = acc[b][j];
    return;
  }
  if (splits == 1) {
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const int m = 16 * j + l15;
      if (m >= M) continue;
#pragma unroll
      for (int b = 0; b < R; ++b) {
        uint2 pk;
        pk.x = pack_bf16x2(acc[b][j][0], acc[b][j][1]);
        pk.y = pack_bf16x2(acc[b][j][2], acc[b][j][3]);
        *reinterpret_cast<uint2*>(y + (int64_t)m * ldy + n0w + 16 * b + 4 * lq) = pk;
      }
    }
    return;
  }
  // split-K: plain stores of this slice's fp32 partials; the slices are
  // summed by splitk_reduce_kernel, launched right after on the same stream
  // (the kernel boundary is the cross-XCD hand-off -- no fences, tickets or
  // serialised last-arriver tail inside this kernel; probe: the in-kernel
  // ticket form cost ~8-15 us per launch at 256 workgroups)
  float* slab = slabs + (int64_t)sl * BM * N;
#pragma unroll
  for (int j = 0; j < T; ++j)
#pragma unroll
    for (int b = 0; b < R; ++b)
      *reinterpret_cast<f32x4*>(slab + (int64_t)(16 * j + l15) * N + n0w + 16 * b + 4 * lq) = acc[b][j];
}

// y[m, n .. n + 7] = sum over slices (in slice order: reproducible) of the
// slabs' partials; one thread per 8 outputs, every slice's loads issued
// before the first add (S is a template constant)
template <int S>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16_t* __restrict__ y, int64_t ldy,
                                                            const float* __restrict__ slabs, int M, int N, int BM) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int n8 = N / 8;
  if (i >= (int64_t)M * n8) return;
  const int m = (int)(i / n8), n = (int)(i % n8) * 8;
  f32x4 v[S][2];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const float* p = slabs + ((int64_t)s * BM + m) * N + n;
    v[s][0] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    v[s][1] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
  }
  f32x4 a = v[0][0], b = v[0][1];
#pragma unroll
  for (int s = 1; s < S; ++s) {
    a += v[s][0];
    b += v[s][1];
  }
  uint4 o;
  o.x = pack_bf16x2(a[0], a[1]);
  o.y = pack_bf16x2(a[2], a[3]);
  o.z = pack_bf16x2(b[0], b[1]);
  o.w = pack_bf16x2(b[2], b[3]);
  *reinterpret_cast<uint4*>(y + (int64_t)m * ldy + n) = o;
}

// SILU: y[m, c .. c + 7] (c < N / 2) = silu(g) * u of the slices' summed
// partials, g at weight rows 64 (c / 32) + c % 32 .., u 32 rows further
template <int S>
__global__ void __launch_bounds__(256) splitk_reduce_silu_kernel(bf16_t* __restrict__ y, int64_t ldy,
                                                                 const float* __restrict__ slabs, int M, int N,
                                                                 int BM) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int f8 = N / 16;  // 8-column groups of the N / 2 outputs
  if (i >= (int64_t)M * f8) return;
  const int m = (int)(i / f8), c = (int)(i % f8) * 8;
  const int gr = 64 * (c >> 5) + (c & 31);
  f32x4 g0 = {0.f, 0.f, 0.f, 0.f}, g1 = g0, u0 = g0, u1 = g0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const float* p = slabs + ((int64_t)s * BM + m) * N + gr;
    g0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    g1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
    u0 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 32));
    u1 += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 36));
  }
  uint4 o;
  o.x = pack_bf16x2(silu_f(g0[0]) * u0[0], silu_f(g0[1]) * u0[1]);
  o.y = pack_bf16x2(silu_f(g0[2]) * u0[2], silu_f(g0[3]) * u0[3]);
  o.z = pack_bf16x2(silu_f(g1[0]) * u1[0], silu_f(g1[1]) * u1[1]);
  o.w = pack_bf16x2(silu_f(g1[2]) * u1[2], silu_f(g1[3]) * u1[3]);
  *reinterpret_cast<uint4*>(y + (int64_t)m * ldy + c) = o;
}

void launch_reduce_silu(bf16_t* y, int64_t ldy, const float* slabs, int M, int N, int BM, int splits,
                        hipStream_t st) {
  const int64_t n = (int64_t)M * (N / 16);
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  switch (splits) {
    case 2: hipLaunchKernelGGL(splitk_reduce_silu_kernel<2>, g, b, 0, st, y, ldy, slabs, M, N, BM); break;
    case 4: hipLaunchKernelGGL(splitk_reduce_silu_kernel<4>, g, b, 0, st, y, ldy, slabs, M, N, BM); break;
    case 8: hipLaunchKernelGGL(splitk_reduce_silu_kernel<8>, g, b, 0, st, y, ldy, slabs, M, N, BM); break;
    default: break;
  }
}

void launch_reduce(bf16_t* y, int64_t ldy, const float* slabs, int M, int N, int BM, int splits, hipStream_t st) {
  const int64_t n = (int64_t)M * (N / 8);
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  switch (splits) {
    case 2: hipLaunchKernelGGL(splitk_reduce_kernel<2>, g, b, 0, st, y, ldy, slabs, M, N, BM); break;
    case 4: hipLaunchKernelGGL(splitk_reduce_kernel<4>, g, b, 0, st, y, ldy, slabs, M, N, BM); break;
    case 8: hipLaunchKernelGGL(splitk_reduce_kernel<8>, g, b, 0, st, y, ldy, slabs, M, N, BM); break;
    default: break;
  }
}

template <int NW, int R, int T, int DW, int DX>
int launch(bf16_t* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs, int* tickets, int M,
           int N, int K, int splits, bool reduce, bool silu, hipStream_t st) {
  constexpr int BN = NW * 16 * R;
  if constexpr (DX * 16 * T * LINE + 1024 + 16 > 160 * 1024) {
    return 2;
  } else {
    if (N % BN || (K / KS / splits) % DW || M > 16 * T) return 3;
    const int grid = (N / BN) * splits;
    if constexpr (R == 2) {
      if (silu) {
        if (N % 64 || !reduce) return 3;
        hipLaunchKernelGGL((dstream_kernel<NW, R, T, DW, DX, 0, true>), dim3(grid), dim3(64 * NW), 0, st, y, ldy, x,
                           ldx, w, slabs, tickets, M, N, K, splits);
        if (splits > 1) launch_reduce_silu(y, ldy, slabs, M, N, 16 * T, splits, st);
        return 0;
      }
    }
    if (silu) return 3;
    hipLaunchKernelGGL((dstream_kernel<NW, R, T, DW, DX, 0>), dim3(grid), dim3(64 * NW), 0, st, y, ldy, x, ldx, w,
                       slabs, tickets, M, N, K, splits);
    if (splits > 1 && reduce) launch_reduce(y, ldy, slabs, M, N, 16 * T, splits, st);
    return 0;
  }
}

template <int NW, int R, int T>
int launch_d(int dw, int dx, bf16_t* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs,
             int* tickets, int M, int N, int K, int splits, bool reduce, bool silu, hipStream_t st) {
#define DX_DS_D(DW_, DX_)                                                                                   \
  if (dw == DW_ && dx == DX_)                                                                             \
    return launch<NW, R, T, DW_, DX_>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, reduce, silu, st);
  DX_DS_D(4, 2) DX_DS_D(4, 4) DX_DS_D(8, 2) DX_DS_D(8, 4)
#undef DX_DS_D
  return 2;
}

int run(void* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs, int* tickets, int M, int N,
        int K, int nw, int r, int t, int dw, int dx, int splits, int flags, hipStream_t st) {
  constexpr int ESZ = 2;
  if (M < 1) return 0;
  if (M > 256 || M > 16 * t || !(splits == 1 || splits == 2 || splits == 4 || splits == 8)) return 1;
  if (splits > 1 && (slabs == nullptr || tickets == nullptr)) return 4;
  if (K % (LINE / ESZ * splits) || (K / (LINE / ESZ) / splits) < dw) return 3;
  if (((ldx * ESZ) & 15) || (ldy & 3) || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(w) & 15) || (reinterpret_cast<uintptr_t>(y) & 7))
    return 5;
  if ((flags & 2) && ((flags & 1) || r != 2 || N % 64 ||
                      (splits > 1 && ((ldy & 7) || (reinterpret_cast<uintptr_t>(y) & 15)))))
    return 8;  // the SwiGLU form: see dx_dstream_gemm
  if ((int64_t)N * K * ESZ >= (1ll << 32) || (int64_t)16 * t * ldx * ESZ >= (1ll << 32)) return 6;  // 32-bit offsets
  auto* Y = static_cast<bf16_t*>(y);
  int rc = 2;
#define DX_DS_CASE(NW_, R_, T_) \
  if (nw == NW_ && r == R_ && t == T_) rc = launch_d<NW_, R_, T_>(dw, dx, Y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, !(flags & 1), (flags & 2) != 0, st); else
  DX_DS_CASE(4, 1, 2) DX_DS_CASE(4, 1, 4) DX_DS_CASE(4, 1, 8) DX_DS_CASE(4, 1, 16)
  DX_DS_CASE(4, 2, 2) DX_DS_CASE(4, 2, 4) DX_DS_CASE(4, 2, 8) DX_DS_CASE(4, 2, 16)
  DX_DS_CASE(8, 1, 2) DX_DS_CASE(8, 1, 4) DX_DS_CASE(8, 1, 8) DX_DS_CASE(8, 1, 16)
  DX_DS_CASE(8, 2, 2) DX_DS_CASE(8, 2, 4) DX_DS_CASE(8, 2, 8)
  // 3 / 6 / 7 waves: row tiles of 48 / 96 / 112 (x2) rows, so the Llama projections' N divide into exactly
  // 256 workgroups -- one per CU, no tail wave of workgroups (qkv N 6144 = 128 x 48; gate_up N 28672 = 256 x 112)
  DX_DS_CASE(3, 1, 4) DX_DS_CASE(3, 1, 8) DX_DS_CASE(3, 1, 16) DX_DS_CASE(3, 2, 4) DX_DS_CASE(3, 2, 8)
  DX_DS_CASE(6, 1, 4) DX_DS_CASE(6, 1, 8) DX_DS_CASE(6, 1, 16) DX_DS_CASE(6, 2, 4) DX_DS_CASE(6, 2, 8)
  DX_DS_CASE(7, 1, 4) DX_DS_CASE(7, 1, 8) DX_DS_CASE(7, 1, 16) DX_DS_CASE(7, 2, 4) DX_DS_CASE(7, 2, 8)
  rc = 2;
#undef DX_DS_CASE
  return rc;
}

}  // namespace

// nw (waves) in {3, 4, 6, 7, 8}; r (16-row weight blocks per wave) in {1, 2}; t (16-token blocks, M <= 16 t) in
// {2, 4, 8, 16}; (dw, dx) weight-ring / x-ring depths in {(4, 2), (4, 4), (8, 2), (8, 4)};
// N % (nw * 16 r) == 0, (K / 64 / splits) % dw == 0.  With splits > 1: slabs >= splits * 16 t * N floats
// (tickets unused).  flags bit 0: leave the split-K partials in the slabs
// (slice s, row m at slabs + (s * 16 t + m) * N) for a consumer that sums
// them itself (dx_add_rmsnorm_slabs) -- no reduction launch, y untouched.
// flags bit 1: SILU -- w is a 32-row interleaved gate / up weight, r == 2, N % 64 == 0, and y[M, N / 2] =
// silu(gate) * up (ldy counts the N / 2 output columns); not combinable with bit 0.
extern "C" int dx_dstream_gemm(void* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs,
                               int* tickets, int M, int N, int K, int nw, int r, int t, int dw, int dx, int splits,
                               int flags, hipStream_t st) {
  const int rc = run(y, ldy, x, ldx, w, slabs, tickets, M, N, K, nw, r, t, dw, dx, splits, flags, st);
  DX_CHECK_LAUNCH();
  return rc;
}

// y[M, N] (bf16, row stride ldy) = the slice-ordered sum of split-K partials left by
// dx_dstream_gemm(flags = 1) -- for a consumer that cannot read them directly
extern "C" int dx_splitk_reduce(void* y, int64_t ldy, const float* slabs, int M, int N, int BM, int splits,
                                hipStream_t st) {
  if (M < 1) return 0;
  if (N % 8 || (ldy & 7) || !(splits == 2 || splits == 4 || splits == 8) || M > BM) return 1;
  launch_reduce(static_cast<bf16_t*>(y), ldy, slabs, M, N, BM, splits, st);
  DX_CHECK_LAUNCH();
  return 0;
}

// bandwidth probes of the (nw 4, r 1, t 8, dw 4, dx 4) config (see P above); grid as dx_dstream_gemm
extern "C" int dx_dstream_probe(void* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs,
                                int* tickets, int M, int N, int K, int splits, int probe, hipStream_t st) {
  if (M < 1 || M > 128 || N % 64 || K % (64 * splits) || (K / 64 / splits) % 4 || splits < 1) return 1;
  auto* Y = static_cast<bf16_t*>(y);
  auto* X = static_cast<const bf16_t*>(x);
  auto* W = static_cast<const bf16_t*>(w);
  const int grid = (N / 64) * splits;
#define DX_DP(P_)                                                                                                 \
  if (probe == P_) {                                                                                              \
    hipLaunchKernelGGL((dstream_kernel<4, 1, 8, 4, 4, P_>), dim3(grid), dim3(256), 0, st, Y, ldy, X, ldx, W, slabs, \
                       tickets, M, N, K, splits);                                                                 \
    if (splits > 1) launch_reduce(Y, ldy, slabs, M, N, 128, splits, st);                                        \
    return (int)hipGetLastError();                                                                                \
  }
  DX_DP(0) DX_DP(1) DX_DP(2) DX_DP(3)
#undef DX_DP
  return 2;
}
