// Register-streamed decode projection GEMM for gfx950 (M ~ 16-256 tokens):
//     y[M, N] = x[M, K] . w[N, K]^T      bf16 in / out, fp32 accumulation
//
// Why another small-M kernel.  A decode projection at M = 128 is weight-stream
// bound, and by Little's law a CU has to keep ~64-128 KB of weight bytes in
// flight to run at HBM rate (25-30 GB/s per CU at 6.5-7 TB/s, 2-4 us loaded
// latency).  wstream_gemm.hip stages the weights through a LDS-DMA ring: its
// bytes in flight are capped by the 160 KB of LDS shared with the x image
// (~32-48 KB of weights), and it measured 1.4-4 TB/s.  Here the weights
// bypass LDS: every wave streams ITS OWN weight rows straight into VGPRs as
// MFMA A fragments, D k-steps ahead (8 waves x 12 KB in flight per CU at
// D = 4), while only x -- small, L2-resident, shared by every wave of the
// workgroup -- goes through LDS (LDS-DMA, full 128-B lines, source-side XOR
// swizzle, read back as B fragments with conflict-free ds_read_b128):
//   * workgroup = NW waves x (16 R) weight rows = BN rows, one BM-token tile,
//     one K-slice (split-K over workgroups: fp32 slabs + a ticket, the
//     last arriver sums the slabs in slice order -> bit-reproducible; the
//     reducer re-zeroes the ticket so a captured graph can replay the launch);
//   * one k-step = 64 k: per wave R x 2 weight loads (16 rows x 64 B each,
//     global_load_dwordx4) and BM / (8 NW) x-image LDS-DMA pieces (8 rows x
//     128 B each); D stages in flight, one counted vmcnt + one barrier per
//     step; the LDS slot refilled in step t is the one every wave finished
//     reading in step t - 1 (the barrier of step t orders it);
//   * the weight and x loads are inline asm, invisible to the compiler's
//     s_waitcnt bookkeeping (it drains vmcnt(0) at the first use of a counted
//     load while an LDS-DMA is outstanding: cdna_hip_programming.md §5.7); the
//     counted wait is an asm statement that names the step's weight registers
//     "+v", so no MFMA reading them is scheduled above it, and the barrier is
//     an asm statement with a memory clobber, so no ds_read is hoisted above it;
//   * v_mfma_f32_16x16x32_bf16 with A = weight rows, B = token rows: each lane
//     ends with 4 consecutive output columns of one token (8-byte stores).
// The engine's warm-up tuner adopts a config per decode graph size and
// projection only where it beats hipBLASLt and the other small-M kernels
// (models/llama.py tune_gemms).
#include <type_traits>

#include "common.h"

namespace {

constexpr int KS = 64;  // k per step (one 128-B line per weight / x row)

// P (bandwidth probes, wrong results): 1 = no MFMA, 2 = weights only (no x DMA,
// no MFMA), 3 = weights only with lane-linear rows (8 rows x 128 B per load)
template <int BM, int R, int NW, int D, bool NT, int P = 0>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2, 2))) vstream_kernel(bf16_t* __restrict__ y, int64_t ldy,
                                                      const bf16_t* __restrict__ x, int64_t ldx,
                                                      const bf16_t* __restrict__ w, float* __restrict__ slabs,
                                                      int* __restrict__ tickets, int M, int N, int K, int splits) {
  constexpr int BN = NW * 16 * R;   // weight rows per workgroup
  constexpr int T = BM / 16;        // 16-token MFMA blocks
  constexpr int SB = BM * KS * 2;   // x image bytes per stage
  constexpr int NX = BM / (8 * NW); // LDS-DMA pieces (1 KB) per wave per stage
  constexpr int NL = 2 * R;         // weight loads per wave per stage
  constexpr int PER = NX + NL;      // vm ops per wave per stage
  static_assert(NX >= 1 && BM % (8 * NW) == 0, "x pieces per wave");
  constexpr int PERW = P >= 2 ? NL : PER;
  static_assert((D - 2) * PER < 64 && D >= 2, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[D * SB + 16];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l15 = lane & 15, lq = lane >> 4;

  // ---- block -> (row tile, K-slice): consecutive ids share an XCD, and the
  // K-slices of one row tile are consecutive (the split-K reducer reads its
  // sibling slabs from the same L2)
  const int ntn = N / BN, mtn = (M + BM - 1) / BM, nwg = ntn * splits * mtn;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  // token tiles of one (row tile, K-slice) are consecutive too: launched
  // together on one XCD, the weight tile comes from HBM once and from L2 for
  // the other token tiles
  const int mt = id % mtn, ns_ = id / mtn;
  const int nt = ns_ / splits, sl = ns_ - nt * splits;
  const int nk = K / KS / splits;
  const int k0 = sl * nk * KS;

  // ---- weight fragments: row block b of this wave = rows n0w + 16 b + l15,
  // bytes k * 2 + 64 kb + 16 lq of the step (A operand: row l15, k-group lq)
  const int n0w = nt * BN + wave * 16 * R;
  uint32_t voff[R];
#pragma unroll
  for (int b = 0; b < R; ++b) voff[b] = (uint32_t)((n0w + 16 * b + l15) * K + k0) * 2u + 16u * lq;
  uint32_t voffl[R][2];  // P == 3: load kb of block b = rows 16 b + 8 kb + lane / 8, 16-B chunk lane % 8
#pragma unroll
  for (int b = 0; b < R; ++b)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      voffl[b][kb] = (uint32_t)((n0w + 16 * b + 8 * kb + (lane >> 3)) * K + k0) * 2u + 16u * (lane & 7);

  // ---- x image: piece p = wave * NX + i holds rows 8p .. 8p + 7 (128 B each,
  // 16-B chunk c of a row stores source chunk c ^ swz(row)); rows >= M re-read row M - 1
  auto swz = [](int r) { return (r >> 1) & 7; };
  uint32_t xoff[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int row = 8 * (wave * NX + i) + (lane >> 3);
    const int ch = (lane & 7) ^ swz(row);
    xoff[i] = (uint32_t)(min(mt * BM + row, M - 1) * (int)ldx + k0 + ch * 8) * 2u;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  auto issue = [&](int t, int slot, bf16x8_t (&wr)[R][2]) {
    const bf16_t* wb = w + (int64_t)t * KS;
    const bf16_t* xb = x + (int64_t)t * KS;
#pragma unroll
    for (int b = 0; b < R; ++b) {
      if constexpr (P == 3) {
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(wr[b][0]) : "v"(voffl[b][0]), "s"(wb) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(wr[b][1]) : "v"(voffl[b][1]), "s"(wb) : "memory");
      } else if constexpr (NT) {
        asm volatile("global_load_dwordx4 %0, %1, %2 offset:0 nt" : "=v"(wr[b][0]) : "v"(voff[b]), "s"(wb) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, %2 offset:64 nt" : "=v"(wr[b][1]) : "v"(voff[b]), "s"(wb) : "memory");
      } else {
        asm volatile("global_load_dwordx4 %0, %1, %2 offset:0" : "=v"(wr[b][0]) : "v"(voff[b]), "s"(wb) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, %2 offset:64" : "=v"(wr[b][1]) : "v"(voff[b]), "s"(wb) : "memory");
      }
    }
#pragma unroll
    for (int i = 0; i < (P >= 2 ? 0 : NX); ++i) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds0 + slot * SB + (wave * NX + i) * 1024);
      uint32_t keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(xoff[i]), "s"(xb), "s"(dst)
          : "memory");
    }
  };

  // ---- B fragments: token row 16 j + l15, chunk (4 kb + lq) ^ swz(row) --
  // swz(16 j + l15) = swz(l15), so one per-lane offset per kb
  int xr[2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) xr[kb] = l15 * (KS * 2) + (((4 * kb + lq) ^ swz(l15)) << 4);

  f32x4 acc[R][T];
#pragma unroll
  for (int b = 0; b < R; ++b)
#pragma unroll
    for (int j = 0; j < T; ++j) acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8_t wr[D][R][2];

  auto compute = [&](int slot, bf16x8_t (&cw)[R][2]) {
    const char* s = smem + slot * SB;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      bf16x8_t xf[T];
#pragma unroll
      for (int j = 0; j < T; ++j) xf[j] = *reinterpret_cast<const bf16x8_t*>(s + j * 16 * (KS * 2) + xr[kb]);
#pragma unroll
      for (int b = 0; b < R; ++b)
#pragma unroll
        for (int j = 0; j < T; ++j)
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[b][kb], xf[j], acc[b][j], 0, 0, 0);
    }
  };

  // wait until at most N vm ops of this wave are outstanding; the step's weight
  // registers are named so their consumers stay below the wait
  auto wait_stage = [&](bf16x8_t (&cw)[R][2], auto n_c) {
    constexpr int N_ = decltype(n_c)::value;
    constexpr int enc = 0x0F70 | (N_ & 15) | ((N_ >> 4) << 14);
    if constexpr (R == 1)
      asm volatile("s_waitcnt %2" : "+v"(cw[0][0]), "+v"(cw[0][1]) : "i"(enc) : "memory");
    else
      asm volatile("s_waitcnt %4" : "+v"(cw[0][0]), "+v"(cw[0][1]), "+v"(cw[1][0]), "+v"(cw[1][1]) : "i"(enc) : "memory");
  };

  // ---- D-stage ring: stages t+1 .. t+D-1 in flight while stage t is consumed
#pragma unroll
  for (int s = 0; s < D - 1; ++s) issue(s, s, wr[s]);  // nk >= D (host check)
  // Every step issues one stage -- past the end, a re-read of the last stage
  // into the slot / registers nobody consumes again -- so the wait count is
  // one constant and the loop has no branch: a conditional issue or wait
  // makes the compiler merge two definitions of the ring registers with
  // v_movs placed BEFORE the wait (reading registers whose loads are still in
  // flight).
  for (int t0 = 0; t0 < nk; t0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int t = t0 + u;
      wait_stage(wr[u], std::integral_constant<int, (D - 2) * PERW>{});
      // every wave's x pieces of stage t landed; every wave finished step t-1's reads
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      issue(min(t + D - 1, nk - 1), (u + D - 1) % D, wr[(u + D - 1) % D]);
      if constexpr (P == 0) compute(u, wr[u]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's re-reads

  // ---- epilogue: acc[b][j] register e = (weight row n0w + 16 b + 4 lq + e,
  // token 16 j + l15)
  const int tok0 = mt * BM + l15;
  if (splits == 1) {
#pragma unroll
    for (int j = 0; j < T; ++j) {
      const int m = tok0 + 16 * j;
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
  const int64_t slab_elems = (int64_t)mtn * BM * N;
  {
    float* slab = slabs + (int64_t)sl * slab_elems;
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
      for (int b = 0; b < R; ++b)
        *reinterpret_cast<f32x4*>(slab + (int64_t)(tok0 + 16 * j) * N + n0w + 16 * b + 4 * lq) = acc[b][j];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem + D * SB);
  int* ticket = tickets + nt * mtn + mt;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (tk == splits - 1);
  }
  __syncthreads();
  if (!*flag) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < R; ++b)
#pragma unroll
    for (int j = 0; j < T; ++j) acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s2 = 0; s2 < splits; ++s2) {  // slice order, own slab included (reproducible)
    const float* slab = slabs + (int64_t)s2 * slab_elems;
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
      for (int b = 0; b < R; ++b)
        acc[b][j] += *reinterpret_cast<const f32x4*>(slab + (int64_t)(tok0 + 16 * j) * N + n0w + 16 * b + 4 * lq);
  }
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const int m = tok0 + 16 * j;
    if (m >= M) continue;
#pragma unroll
    for (int b = 0; b < R; ++b) {
      uint2 pk;
      pk.x = pack_bf16x2(acc[b][j][0], acc[b][j][1]);
      pk.y = pack_bf16x2(acc[b][j][2], acc[b][j][3]);
      *reinterpret_cast<uint2*>(y + (int64_t)m * ldy + n0w + 16 * b + 4 * lq) = pk;
    }
  }
}

template <int BM, int R, int NW, int D, bool NT>
int launch(bf16_t* y, int64_t ldy, const bf16_t* x, int64_t ldx, const bf16_t* w, float* slabs, int* tickets, int M,
           int N, int K, int splits, hipStream_t st) {
  constexpr int BN = NW * 16 * R;
  if constexpr (BM % (8 * NW) != 0 || D * BM * KS * 2 + 16 > 160 * 1024) {
    return 2;
  } else {
    if (N % BN || (K / KS / splits) % D) return 3;
    const int grid = (N / BN) * splits * ((M + BM - 1) / BM);
    hipLaunchKernelGGL((vstream_kernel<BM, R, NW, D, NT>), dim3(grid), dim3(64 * NW), 0, st, y, ldy, x, ldx, w, slabs,
                       tickets, M, N, K, splits);
    return 0;
  }
}

template <int BM, int R, int NW>
int launch_d(int d, bool nt, bf16_t* y, int64_t ldy, const bf16_t* x, int64_t ldx, const bf16_t* w, float* slabs,
             int* tickets, int M, int N, int K, int splits, hipStream_t st) {
#define DX_VS_D(D_)                                                                                       \
  if (d == D_)                                                                                            \
    return nt ? launch<BM, R, NW, D_, true>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, st)       \
              : launch<BM, R, NW, D_, false>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, st);
  DX_VS_D(2) DX_VS_D(3) DX_VS_D(4) DX_VS_D(6)
#undef DX_VS_D
  return 2;
}

}  // namespace

// bm (token tile; ceil(M / bm) tiles) in {32, 64, 128, 256}; r (16-row weight blocks per wave) in {1, 2};
// nw (waves) in {4, 8} with bm % (8 nw) == 0; d (stages in flight) in {2, 3, 4, 6} with
// d * bm * 128 B <= 160 KB; N % (nw * 16 r) == 0, (K / 64 / splits) % d == 0.  nt: non-temporal
// weight loads.  With splits > 1: slabs >= splits * ceil(M / bm) * bm * N floats, tickets >=
// N / (nw * 16 r) * ceil(M / bm) zeroed ints (left zeroed on return).
extern "C" int dx_vstream_gemm(void* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs,
                               int* tickets, int M, int N, int K, int bm, int r, int nw, int d, int splits, int nt,
                               hipStream_t st) {
  if (M < 1) return 0;
  if (M > 256 || bm > 256 || splits < 1) return 1;
  if (splits > 1 && (slabs == nullptr || tickets == nullptr)) return 4;
  if (K % (KS * splits) || (K / KS / splits) < d) return 3;
  if ((ldx & 7) || (ldy & 3) || (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 7))
    return 5;
  if ((int64_t)N * K * 2 >= (1ll << 32) || (int64_t)bm * ldx * 2 >= (1ll << 32)) return 6;  // 32-bit offsets
  auto* Y = static_cast<bf16_t*>(y);
  auto* X = static_cast<const bf16_t*>(x);
  auto* W = static_cast<const bf16_t*>(w);
  int rc = 2;
#define DX_VS_CASE(BM_, R_, NW_) \
  if (bm == BM_ && r == R_ && nw == NW_) rc = launch_d<BM_, R_, NW_>(d, nt != 0, Y, ldy, X, ldx, W, slabs, tickets, M, N, K, splits, st); else
  DX_VS_CASE(32, 1, 4) DX_VS_CASE(32, 2, 4)
  DX_VS_CASE(64, 1, 4) DX_VS_CASE(64, 2, 4) DX_VS_CASE(64, 1, 8) DX_VS_CASE(64, 2, 8)
  DX_VS_CASE(128, 1, 4) DX_VS_CASE(128, 2, 4) DX_VS_CASE(128, 1, 8) DX_VS_CASE(128, 2, 8)
  DX_VS_CASE(256, 1, 8) DX_VS_CASE(256, 1, 4)
  rc = 2;
#undef DX_VS_CASE
  DX_CHECK_LAUNCH();
  return rc;
}

// bandwidth probes of two configs (bm 128, r 2, 4 waves / r 1, 8 waves; 4 stages): see P above
extern "C" int dx_vstream_probe(void* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs,
                                int* tickets, int M, int N, int K, int r, int splits, int probe, hipStream_t st) {
  if (M < 1 || M > 128 || K % (64 * splits) || (K / 64 / splits) % 4 || (N % 128) || splits < 1) return 1;
  auto* Y = static_cast<bf16_t*>(y);
  auto* X = static_cast<const bf16_t*>(x);
  auto* W = static_cast<const bf16_t*>(w);
  const int grid = (N / 128) * splits;
#define DX_VP(R_, NW_, P_)                                                                                          \
  if (r == R_ && probe == P_) {                                                                                     \
    hipLaunchKernelGGL((vstream_kernel<128, R_, NW_, 4, false, P_>), dim3(grid), dim3(64 * NW_), 0, st, Y, ldy, X, \
                       ldx, W, slabs, tickets, M, N, K, splits);                                                    \
    return (int)hipGetLastError();                                                                                  \
  }
  DX_VP(2, 4, 1) DX_VP(2, 4, 2) DX_VP(2, 4, 3) DX_VP(1, 8, 1) DX_VP(1, 8, 2) DX_VP(1, 8, 3)
#undef DX_VP
  return 2;
}
