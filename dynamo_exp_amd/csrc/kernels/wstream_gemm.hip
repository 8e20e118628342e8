// Weight-streaming projection GEMM for decode batch sizes (M ~ 33-256) on gfx950:
//     y[M, N] = x[M, K] . w[N, K]^T      bf16 in / out, fp32 accumulation
//
// At M = 128 a projection is weight-bandwidth bound (128 FLOP per weight byte,
// under the MI355X ridge of ~310) but only by ~2x, so the kernel has to keep
// many weight bytes in flight per CU AND run its MFMAs at a fair rate.  The
// register-fed small-M kernels (skinny_gemm.hip) stall on in-order vmcnt: a
// wave's next weight fragments cannot be waited for without also waiting for
// every older load (profiles/README.md "Decode-GEMM studies").  Here both
// operands move HBM/L2 -> LDS by LDS-DMA in an NS-stage ring, so the bytes in
// flight are LDS, not registers, and one counted vmcnt per stage covers them:
//   * workgroup tile = BM tokens x BN weight rows (64 / 128 each), NW = 4 or 8
//     waves as (BN / 32) weight groups x (NW / (BN / 32)) token groups; each wave
//     owns 32 weight rows x BM / WT tokens on v_mfma_f32_16x16x32_bf16 with A = weight
//     rows, B = token rows, so every lane holds 4 consecutive output columns
//     of one token (8-byte stores, the gemm256.hip epilogue layout);
//   * a stage is one KT-deep K step (64 or 128) of both images (w rows, then x
//     rows; lane-linear DMA, the 16-B chunks of a row XOR-swizzled on the
//     source side so 16-lane ds_read_b128 groups hit 16 distinct bank slots); NS - 1 stages
//     are in flight while one is consumed; one barrier per stage, after which
//     the slot read in the previous step is refilled.  Every wave issues its
//     share of the DMA: one wave sustains only ~8 GB/s of LDS-DMA
//     (tools/wstream_probe.py: DMA-only loops run at the same speed with the
//     weights resident in the Infinity Cache), so 8 waves per CU move twice
//     the bytes of 4;
//   * K is split over workgroups (fp32 slabs + a ticket, the last arriver sums
//     the slabs in slice order: bit-reproducible; the reducer resets the ticket
//     so captured graphs can replay the launch), and blocks are remapped so the
//     token tiles and K-slices of one weight tile run on one XCD (the weight
//     tile comes from HBM once and from that XCD's L2 after).
// The engine's warm-up tunes (BM, BN, NS, splits) per decode graph size and
// projection against hipBLASLt and the other small-M kernels
// (models/llama.py tune_gemms).
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt vmcnt(n) with expcnt / lgkmcnt left alone (gfx9 encoding)
template <int n>
__device__ __forceinline__ void wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (n & 15) | ((n >> 4) << 14));
}

template <int BM, int BN, int NS, int KT, int NW>
__global__ void __launch_bounds__(64 * NW) wstream_kernel(bf16_t* __restrict__ y, int64_t ldy,
                                                      const bf16_t* __restrict__ x, int64_t ldx,
                                                      const bf16_t* __restrict__ w, float* __restrict__ slabs,
                                                      int* __restrict__ tickets, int M, int N, int K, int splits,
                                                      int wpol) {
  constexpr int RB = KT * 2;        // image row bytes (128 or 256)
  constexpr int RPI = 1024 / RB;    // image rows per DMA instruction (64 lanes x 16 B)
  constexpr int NKB = KT / 32;      // MFMA k-blocks per stage
  constexpr int R = BM + BN;        // image rows per stage (weights first)
  constexpr int SB = R * RB;        // stage bytes
  constexpr int RW = R / NW;        // image rows DMA'd by one wave per stage
  constexpr int NI = RW / RPI;      // DMA instructions per wave per stage
  constexpr int WW = BN / 32;       // waves along weight rows
  constexpr int WT = NW / WW;       // waves along tokens
  constexpr int TW = BM / WT;       // tokens per wave
  constexpr int TB = TW / 16;       // 16-token MFMA blocks per wave
  static_assert(RW % RPI == 0 && BN % 16 == 0 && TB >= 1 && (KT == 64 || KT == 128), "tile shape");
  // XOR swizzle of a row's 16-B chunks: a 16-lane ds_read_b128 group (rows
  // r0 .. r0 + 15, one chunk) must hit 16 distinct bank slots of 256 B
  auto swz = [](int r) { return KT == 64 ? ((r >> 1) & 7) : (r & 15); };
  __shared__ __attribute__((aligned(16))) char smem[NS * SB + 16];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l15 = lane & 15, lq = lane >> 4;
  const int ww = wave % WW, wt = wave / WW;

  // ---- block -> (K-slice, weight tile, token tile): consecutive ids share an
  // XCD (bijective for any grid size) and run token tiles of one weight tile
  // and weight tiles of one K-slice, so an XCD's L2 holds the x rows of the
  // few K-slices it works on (down at M 128: x is 3.7 MB, a slice 0.9 MB)
  const int ntn = N / BN, mtn = (M + BM - 1) / BM, nwg = ntn * mtn * splits;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int per_sl = ntn * mtn;
  const int sl = id / per_sl, rem = id - sl * per_sl;
  const int nt = rem / mtn, mt = rem - nt * mtn;
  const int nk = K / KT / splits;
  const int64_t k0 = (int64_t)sl * nk * KT;
  const bf16_t* wb = w + (int64_t)nt * BN * K + k0;
  const bf16_t* xb = x + (int64_t)mt * BM * ldx + k0;

  // ---- DMA: instruction i of this wave fills image rows rr0 .. rr0 + RPI - 1
  // (fixed-size arrays: a lambda capturing arrays of template-dependent size
  // loses the kernel's host stub in this clang)
  static_assert(NI <= 16, "DMA instructions per wave");
  int goff[16], loff[16], goffb[16];
  bool isx[16];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int rr0 = wave * RW + RPI * i, row = rr0 + lane / (RB / 16);
    const int ch = (lane % (RB / 16)) ^ swz(row);  // BN % 16 == 0: same XOR in the x image
    isx[i] = rr0 >= BN;
    if (isx[i]) {
      const int xr = row - BN;
      const int gr = min(mt * BM + xr, M - 1) - mt * BM;  // rows past M re-read row M-1
      goff[i] = gr * (int)ldx + ch * 8;
    } else {
      goff[i] = row * K + ch * 8;
      goffb[i] = row * KT + ch * 8;
    }
    loff[i] = rr0 * RB;
  }
  // weights are read once: wpol 1 loads them non-temporal (nt), so the
  // stream does not push the re-read x rows out of L2
  auto issue = [&](int kt, int slot) {
    char* dst = smem + slot * SB;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if (isx[i] && (wpol & 2)) continue;  // probe: no x traffic (results wrong)
      if (!isx[i] && (wpol & 8)) {  // probe: weights in a tile-blocked layout (results wrong)
        const bf16_t* wblk = w + (int64_t)nt * BN * K + (int64_t)(sl * nk + kt) * BN * KT;
        __builtin_amdgcn_global_load_lds(wblk + goffb[i], (lds_void*)(dst + loff[i]), 16, 0, 0);
        continue;
      }
      if (isx[i] || (wpol & 1) == 0)
        __builtin_amdgcn_global_load_lds((isx[i] ? xb : wb) + kt * KT + goff[i], (lds_void*)(dst + loff[i]), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds(wb + kt * KT + goff[i], (lds_void*)(dst + loff[i]), 16, 0, 2);
    }
  };

  // ---- fragments: row = 16-row block base + l15, k chunk 4 kb + lq (XOR swz(l15))
  int cof[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) cof[kb] = ((4 * kb + lq) ^ swz(l15)) << 4;
  const int fw = (ww * 32 + l15) * RB, fx = (BN + wt * TW + l15) * RB;
  f32x4 acc[2][TB];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int slot) {
    const char* s = smem + slot * SB;
    bf16x8_t wf[2][NKB], xf[TB][NKB];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
        wf[b][kb] = *reinterpret_cast<const bf16x8_t*>(s + fw + b * 16 * RB + cof[kb]);
#pragma unroll
    for (int j = 0; j < TB; ++j)
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
        xf[j][kb] = *reinterpret_cast<const bf16x8_t*>(s + fx + j * 16 * RB + cof[kb]);
#pragma unroll
    for (int k = 0; k < NKB; ++k)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < TB; ++j)
          acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[b][k], xf[j][k], acc[b][j], 0, 0, 0);
  };

  // ---- NS-stage ring: stages t+1 .. t+NS-1 in flight while stage t is consumed
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);
  for (int t = 0; t < nk; ++t) {
    if (t + NS - 1 < nk) wait_vm<NI * (NS - 2)>();  // stage t landed (this wave's part)
    else wait_vm<0>();                               // tail: nothing newer was issued
    __builtin_amdgcn_s_waitcnt(0xc07f);              // lgkmcnt(0): step t-1's reads retired
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();                    // every wave's part of stage t landed
    __builtin_amdgcn_sched_barrier(0);
    if (t + NS - 1 < nk) issue(t + NS - 1, (t + NS - 1) % NS);  // the slot read in step t-1
    if (!(wpol & 4)) compute(t % NS);  // probe bit 4: DMA only (results wrong)
  }

  // ---- epilogue: acc[b][j] register r = (weight row nt*BN + ww*32 + 16b + 4lq + r,
  // token mt*BM + wt*TW + 16j + l15)
  const int n0 = nt * BN + ww * 32 + 4 * lq;
  const int tok0 = mt * BM + wt * TW + l15;
  if (splits == 1) {
#pragma unroll
    for (int j = 0; j < TB; ++j) {
      const int m = tok0 + 16 * j;
      if (m >= M) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        uint2 pk;
        pk.x = pack_bf16x2(acc[b][j][0], acc[b][j][1]);
        pk.y = pack_bf16x2(acc[b][j][2], acc[b][j][3]);
        *reinterpret_cast<uint2*>(y + (int64_t)m * ldy + n0 + 16 * b) = pk;
      }
    }
    return;
  }
  const int64_t slab_elems = (int64_t)mtn * BM * N;
  {
    float* slab = slabs + (int64_t)sl * slab_elems;
#pragma unroll
    for (int j = 0; j < TB; ++j)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        *reinterpret_cast<f32x4*>(slab + (int64_t)(tok0 + 16 * j) * N + n0 + 16 * b) = acc[b][j];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem + NS * SB);
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
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s2 = 0; s2 < splits; ++s2) {  // slice order, own slab included (reproducible)
    const float* slab = slabs + (int64_t)s2 * slab_elems;
#pragma unroll
    for (int j = 0; j < TB; ++j)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[b][j] += *reinterpret_cast<const f32x4*>(slab + (int64_t)(tok0 + 16 * j) * N + n0 + 16 * b);
  }
#pragma unroll
  for (int j = 0; j < TB; ++j) {
    const int m = tok0 + 16 * j;
    if (m >= M) continue;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      uint2 pk;
      pk.x = pack_bf16x2(acc[b][j][0], acc[b][j][1]);
      pk.y = pack_bf16x2(acc[b][j][2], acc[b][j][3]);
      *reinterpret_cast<uint2*>(y + (int64_t)m * ldy + n0 + 16 * b) = pk;
    }
  }
}

template <int BM, int BN, int NS, int KT, int NW>
void launch(bf16_t* y, int64_t ldy, const bf16_t* x, int64_t ldx, const bf16_t* w, float* slabs, int* tickets, int M,
            int N, int K, int splits, int wpol, hipStream_t st) {
  const int grid = (N / BN) * ((M + BM - 1) / BM) * splits;
  hipLaunchKernelGGL((wstream_kernel<BM, BN, NS, KT, NW>), dim3(grid), dim3(64 * NW), 0, st, y, ldy, x, ldx, w, slabs, tickets,
                     M, N, K, splits, wpol);
}

// stage counts whose ring fits the 160 KB of LDS, wave counts that tile the workgroup
template <int BM, int BN, int NS, int KT, int NW>
int launch_if_fits(bf16_t* y, int64_t ldy, const bf16_t* x, int64_t ldx, const bf16_t* w, float* slabs, int* tickets,
                   int M, int N, int K, int splits, int wpol, hipStream_t st) {
  if constexpr (NS * (BM + BN) * KT * 2 + 16 <= 160 * 1024 && (BM + BN) % (NW * 1024 / (KT * 2)) == 0 &&
                BM / (NW / (BN / 32)) >= 16) {
    launch<BM, BN, NS, KT, NW>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, wpol, st);
    return 0;
  } else {
    return 2;
  }
}

template <int BM, int BN, int KT, int NW>
int launch_ns(int ns, bf16_t* y, int64_t ldy, const bf16_t* x, int64_t ldx, const bf16_t* w, float* slabs,
              int* tickets, int M, int N, int K, int splits, int wpol, hipStream_t st) {
  switch (ns) {
    case 2: return launch_if_fits<BM, BN, 2, KT, NW>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, wpol, st);
    case 3: return launch_if_fits<BM, BN, 3, KT, NW>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, wpol, st);
    case 4: return launch_if_fits<BM, BN, 4, KT, NW>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, wpol, st);
    case 6: return launch_if_fits<BM, BN, 6, KT, NW>(y, ldy, x, ldx, w, slabs, tickets, M, N, K, splits, wpol, st);
    default: return 2;
  }
}

}  // namespace

// bm, bn in {64, 128}; kt (K per stage) in {64, 128}; wpol bit 0: non-temporal weight loads
// (bits 1 / 2 / 3: bandwidth probes that skip the x DMA / skip the MFMAs / read the
// weights as if tile-blocked -- wrong results); nw (waves) in {4, 8}; ns (stages) in
// {2, 3, 4, 6} with ns * (bm + bn) * kt * 2 B <= 160 KB, (bm + bn) rows split evenly over
// the waves' DMA instructions and >= 16 tokens per wave; N % bn == 0, K % (kt * splits) == 0.
// With splits > 1: slabs >= splits * ceil(M/bm)*bm * N floats, tickets >=
// (N/bn) * ceil(M/bm) zeroed ints (left zeroed on return).
extern "C" int dx_wstream_gemm(void* y, int64_t ldy, const void* x, int64_t ldx, const void* w, float* slabs,
                               int* tickets, int M, int N, int K, int bm, int bn, int ns, int kt, int nw,
                               int splits, int wpol, hipStream_t st) {
  if (M < 1) return 0;
  if (M > 256 || splits < 1) return 1;
  if ((bm != 64 && bm != 128) || (bn != 64 && bn != 128) || (kt != 64 && kt != 128) || (nw != 4 && nw != 8))
    return 2;
  if (N % bn != 0 || K % (kt * splits) != 0) return 3;
  if (splits > 1 && (slabs == nullptr || tickets == nullptr)) return 4;
  if ((ldx & 7) || (ldy & 3) || (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 7))
    return 5;
  if ((int64_t)bn * K >= (1ll << 31) || (int64_t)bm * ldx >= (1ll << 31)) return 6;  // 32-bit DMA offsets
  auto* Y = static_cast<bf16_t*>(y);
  auto* X = static_cast<const bf16_t*>(x);
  auto* W = static_cast<const bf16_t*>(w);
  int rc;
#define DX_WS_CASE(BM_, BN_, KT_, NW_) \
  if (bm == BM_ && bn == BN_ && kt == KT_ && nw == NW_) \
    rc = launch_ns<BM_, BN_, KT_, NW_>(ns, Y, ldy, X, ldx, W, slabs, tickets, M, N, K, splits, wpol, st); \
  else
  DX_WS_CASE(64, 64, 64, 4) DX_WS_CASE(64, 128, 64, 4) DX_WS_CASE(128, 64, 64, 4) DX_WS_CASE(128, 128, 64, 4)
  DX_WS_CASE(64, 64, 128, 4) DX_WS_CASE(64, 128, 128, 4) DX_WS_CASE(128, 64, 128, 4) DX_WS_CASE(128, 128, 128, 4)
  DX_WS_CASE(64, 64, 64, 8) DX_WS_CASE(64, 128, 64, 8) DX_WS_CASE(128, 64, 64, 8) DX_WS_CASE(128, 128, 64, 8)
  DX_WS_CASE(64, 64, 128, 8) DX_WS_CASE(64, 128, 128, 8) DX_WS_CASE(128, 64, 128, 8) DX_WS_CASE(128, 128, 128, 8)
  rc = 2;
#undef DX_WS_CASE
  DX_CHECK_LAUNCH();
  return rc;
}
