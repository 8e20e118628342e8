// Large-M projection GEMM for gfx950 (prefill token counts), two epilogues:
//   EPI_STORE:  y[M, N]   = x[M, K] . w[N, K]^T
//   EPI_SILU:   y[M, N/2] = silu(g) * u, where the N weight rows are the MLP's
//               gate and up projections interleaved in blocks of 32 rows
//               (g0..g31, u0..u31, g32..g63, u32..u63, ...; ops.interleave_gate_up):
//               the SwiGLU of the Llama MLP fused into the gate_up GEMM, so the
//               [M, 2F] intermediate is never written or re-read and the
//               separate silu_and_mul launch disappears.
// bf16 in / out, fp32 accumulation (SURVEY §2.15 "SiLU-gated MLP").
//
// Design (CDNA4 guide §5 "256² 8-phase template", re-derived here):
//   * 256 x 256 output tile per workgroup, K in 64-deep tiles, 8 waves as
//     2 (tokens) x 4 (weight rows); each wave owns 128 tokens x 64 weight rows
//     = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (128 accumulator registers).
//     Operands are swapped (A = weight rows, B = token rows) so that every lane
//     ends up holding 4 consecutive output columns of one token: 8-byte stores,
//     and the gate tile and its up tile sit in the same lanes and registers.
//   * Both operands are staged HBM -> LDS by LDS-DMA (global_load_lds_dwordx4,
//     no staging registers), two 64-KB buffers (x tile + w tile each).  The
//     image is lane-linear (8 rows x 128 B per wave instruction) and XOR-
//     swizzled by choosing each lane's SOURCE chunk: slot s of row r holds
//     chunk s ^ ((r >> 1) & 7), which makes every 16-lane group of the
//     ds_read_b128 fragment reads hit 16 distinct bank slots.
//   * Each K-tile runs in 2 phases, half of the wave's accumulators per phase
//     (32 MFMAs); a phase reads only the fragments it newly needs (the w
//     fragments stay in registers for the whole tile: 24 ds_read_b128 per wave
//     and K-tile):   p1: w + x-half 0 -> Q(x0, w)     p2: x-half 1 -> Q(x1, w)
//     The four "parts" of a buffer (x rows of half 0 / 1, w rows of half
//     0 / 1; 16 KB each) are refilled one phase after their last read.
//   * Waves 4-7 run one barrier (half a phase) behind waves 0-3 (two barriers
//     per phase), so the two waves of each SIMD alternate between their LDS-read
//     segment and their MFMA segment (guide §5 8-phase template, microarch "two
//     waves per SIMD" item 9).  Hazards under that stagger: every wave retires
//     its reads (lgkmcnt(0)) BEFORE the phase's first barrier, so the leading
//     group's refill one phase later cannot overtake the lagging group's reads;
//     the DMA waits sit at the end of each phase and cover the parts read two
//     phases later (one barrier before the lagging group reads them).
//   * Blocks are remapped so that each XCD walks a contiguous range of tiles
//     (bijective for any grid size), in bands of group_m token tiles: the ~32
//     workgroups resident on one XCD then share group_m x tiles and
//     32 / group_m weight tiles through that XCD's L2.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kTile = 256 * 128;   // one operand tile: 256 rows x 64 bf16
constexpr int kBuf = 2 * kTile;    // x tile + w tile
constexpr int kLds = 2 * kBuf;     // double buffered: 128 KB

// EPI_SILU_RS: EPI_SILU whose input rows carry a deferred RMSNorm: g and u
// are scaled by rs[token] (1 / rms of the row) before the activation -- the
// norm's weight is folded into the weight columns (models/llama.py)
enum { EPI_STORE = 0, EPI_SILU = 1, EPI_SILU_RS = 2 };

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

template <int EPI>
__global__ void __launch_bounds__(512) gemm256_kernel(bf16_t* __restrict__ y, int64_t ldy,
                                                      const bf16_t* __restrict__ x, int64_t ldx,
                                                      const bf16_t* __restrict__ w, int M, int N, int K,
                                                      int group_m, const float* __restrict__ rs) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int l15 = lane & 15, lq = lane >> 4;

  // ---- persistent, XCD-aware tile order: the workgroups on one XCD (blocks
  // b, b + 8, ...) walk one contiguous range of logical tiles, stride = their
  // count, so the ~32 tiles in flight on an XCD are always neighbours
  const int mtn = (M + kBM - 1) / kBM, ntn = N / kBN, nwg = mtn * ntn;
  const int G = gridDim.x, bid = blockIdx.x, xcd = bid & 7;
  const int gq = G >> 3, gr8 = G & 7;                 // workgroups on this XCD: gq (+1)
  const int per_xcd = xcd < gr8 ? gq + 1 : gq;
  const int q = nwg >> 3, rr = nwg & 7;               // logical tiles owned by this XCD
  const int t_begin = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  const int t_end = t_begin + (xcd < rr ? q + 1 : q);

  // ---- DMA sources: part P (0 = x half 0, 1 = x half 1, 2 = w half 0, 3 = w half 1),
  // instruction i of this wave covers part rows pr = 16 wave + 8 i + (lane >> 3)
  int prow[4][2];  // part row of this lane's source
  int goff[4][2];
  int loff[4][2];
#pragma unroll
  for (int P = 0; P < 4; ++P)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pr0 = 16 * wave + 8 * i;
      const int pr = pr0 + (lane >> 3);
      const int h = P & 1;
      int row, row0;
      if (P < 2) {
        row = (pr >> 6) * 128 + h * 64 + (pr & 63);
        row0 = (pr0 >> 6) * 128 + h * 64 + (pr0 & 63);
      } else {
        row = (pr >> 5) * 64 + h * 32 + (pr & 31);
        row0 = (pr0 >> 5) * 64 + h * 32 + (pr0 & 31);
      }
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      prow[P][i] = row;
      goff[P][i] = (P < 2 ? 0 : row * K) + ch * 8;  // x rows: + clamped row * ldx per tile
      loff[P][i] = (P < 2 ? 0 : kTile) + row0 * 128;
    }
  const int nkt = K / kBK;
  const bf16_t* xb = x;
  const bf16_t* wb = w;
  int xoff[2][2];  // per tile: x part offsets (rows past M re-read row M-1)
  auto issue = [&](int P, int kt, int buf) {
    kt = min(kt, nkt - 1);  // past the end: harmless reload into a buffer that is not read again
    const bf16_t* src = (P < 2 ? xb : wb) + kt * kBK;
    char* dst = smem + buf * kBuf;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds(src + (P < 2 ? xoff[P][i] : goff[P][i]), (lds_void*)(dst + loff[P][i]), 16,
                                       0, 0);
  };

  // ---- fragment read addresses (row = 16-row tile base + l15; the XOR term of
  // a 16-aligned base is (l15 >> 1))
  const int c0 = (lq ^ (l15 >> 1)) << 4, c1 = ((4 + lq) ^ (l15 >> 1)) << 4;
  const int fx = (wr * 128 + l15) * 128, fw = kTile + (wc * 64 + l15) * 128;

  f32x4 acc[4][8];
  bf16x8_t xf[4][2], wf[4][2];

  auto read_x = [&](const char* b, int xh) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const char* p = b + fx + (xh * 4 + j) * 2048;
      xf[j][0] = *reinterpret_cast<const bf16x8_t*>(p + c0);
      xf[j][1] = *reinterpret_cast<const bf16x8_t*>(p + c1);
    }
  };
  auto read_w = [&](const char* b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const char* p = b + fw + i * 2048;
      wf[i][0] = *reinterpret_cast<const bf16x8_t*>(p + c0);
      wf[i][1] = *reinterpret_cast<const bf16x8_t*>(p + c1);
    }
  };
  // Two 32-MFMA phases per K-tile (one barrier hand-off per phase and wave
  // group; four 16-MFMA phases measured 4-7 % slower, profiles/r2_gemm256.txt):
  //   p1: all w + x-half 0 -> Q(x0, w)    p2: x-half 1 -> Q(x1, w)
  // x half 1 of tile t+1 is refilled in p1 of tile t (its buffer's last read
  // was p2 of tile t-1), the other three parts of tile t+2 in p2; reads of
  // phase q are covered by the wait at the end of phase q-2 (stagger rule).
  auto mma2 = [&](int xh) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][xh * 4 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][s], xf[j][s], acc[i][xh * 4 + j], 0, 0, 0);
  };
  auto compute2 = [&](int xh, int vm) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mma2(xh);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (vm == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // tile t+1's x0 / w landed
    if (vm == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // tile t+1's x1 landed
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto ktile2 = [&](int t, int buf) {
    const char* b = smem + buf * kBuf;
    read_w(b);
    read_x(b, 0);
    issue(1, t + 1, buf ^ 1);
    compute2(0, 2);
    read_x(b, 1);
    issue(0, t + 2, buf);
    issue(2, t + 2, buf);
    issue(3, t + 2, buf);
    compute2(1, 6);
  };

  // tile lid -> (token tile, weight tile): bands of group_m token tiles across
  // all weight tiles, token tile fastest: the ~32 workgroups resident on an XCD
  // cover group_m x (32 / group_m) tiles (8 x 4: 12 KB of new operand bytes per
  // workgroup and K-step through the XCD's L2 instead of 33 KB for one weight
  // tile x 32 token tiles)
  int mt = 0, nt = 0;
  auto select = [&](int lid) {
    const int band = lid / (group_m * ntn), first_m = band * group_m;
    const int gsz = min(mtn - first_m, group_m), in_band = lid - band * group_m * ntn;
    mt = first_m + in_band % gsz;
    nt = in_band / gsz;
    xb = x + (int64_t)mt * kBM * ldx;
    wb = w + (int64_t)nt * kBN * K;
#pragma unroll
    for (int P = 0; P < 2; ++P)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        xoff[P][i] = (min(mt * kBM + prow[P][i], M - 1) - mt * kBM) * (int)ldx + goff[P][i];
  };
  // prologue of a tile: tile 0 of K, then K-tile 1 without its x half 1 (issued in p1 of K-tile 0)
  auto prologue = [&]() {
    issue(0, 0, 0);
    issue(2, 0, 0);
    issue(3, 0, 0);
    issue(1, 0, 0);
    issue(0, 1, 1);
    issue(2, 1, 1);
    issue(3, 1, 1);
  };

  int lid = t_begin + (bid >> 3);
  if (lid >= t_end) return;
  select(lid);
  prologue();
  for (;;) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K-tile 0 landed (the stores of the previous tile, issued after this
    // prologue, are in flight underneath: the wait covers them as well)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wave >= 4) __builtin_amdgcn_s_barrier();  // start the lagging group one barrier late
    __builtin_amdgcn_sched_barrier(0);
    for (int t = 0; t < nkt; t += 2) {
      ktile2(t, 0);
      ktile2(t + 1, 1);
    }
    if (wave < 4) __builtin_amdgcn_s_barrier();  // balance the barrier count: every LDS read of this tile is done
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped tail reloads landed before the buffers are refilled

    const int cmt = mt, cnt = nt;
    const int tok0 = cmt * kBM + wr * 128 + l15;
    // EPI_SILU_RS: the 8 row scales this lane needs, loaded in one batch and
    // retired BEFORE the next tile's prologue DMA is queued (the empty asm
    // consumes them): vmcnt retires in order, and the compiler otherwise
    // waits with vmcnt(0) in the epilogue -- for the whole prologue too (the
    // first version: 15 % slower per GEMM, profiles/r6_fold_pmc.txt)
    float scv[8];
    if (EPI == EPI_SILU_RS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) scv[j] = rs[min(tok0 + 16 * j, M - 1)];
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(scv[j]));
    }

    // the next tile's first K-tiles go out before this tile's stores
    const int nlid = lid + per_xcd;
    const bool more = nlid < t_end;
    if (more) {
      lid = nlid;
      select(lid);
      prologue();
    }

    // ---- epilogue: acc[i][j] register r = (weight row wc*64 + 16 i + 4 lq + r, token 16 j + l15)
    if (EPI == EPI_STORE) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tok = tok0 + 16 * j;
        if (tok >= M) continue;
        bf16_t* yr = y + (int64_t)tok * ldy + cnt * kBN + wc * 64 + 4 * lq;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint2 pk;
          pk.x = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
          pk.y = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
          *reinterpret_cast<uint2*>(yr + 16 * i) = pk;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tok = tok0 + 16 * j;
        if (tok >= M) continue;
        bf16_t* yr = y + (int64_t)tok * ldy + cnt * (kBN / 2) + wc * 32 + 4 * lq;
        const float sc = EPI == EPI_SILU_RS ? scv[j] : 1.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          f32x4 g = acc[i][j], u = acc[2 + i][j];
          if (EPI == EPI_SILU_RS) {
            g *= sc;
            u *= sc;
          }
          uint2 pk;
          pk.x = pack_bf16x2(silu_f(g[0]) * u[0], silu_f(g[1]) * u[1]);
          pk.y = pack_bf16x2(silu_f(g[2]) * u[2], silu_f(g[3]) * u[3]);
          *reinterpret_cast<uint2*>(yr + 16 * i) = pk;
        }
      }
    }
    if (!more) break;
  }
}

// one resident workgroup per CU (128 KB of LDS): a grid of min(tiles, CUs)
// workgroups walks all tiles
int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    // DX_GEMM256_CUS: persistent grid for a CU-masked stream (study knob; profiles/r4_mixed_split_cu_mask.txt)
    if (const char* e = getenv("DX_GEMM256_CUS")) n = std::max(1, atoi(e));
  }
  return n;
}

template <int EPI>
void launch(bf16_t* y, int64_t ldy, const bf16_t* x, int64_t ldx, const bf16_t* w, int M, int N, int K, int gm,
            int persistent, hipStream_t st, const float* rs) {
  const int tiles = ((M + kBM - 1) / kBM) * (N / kBN);
  const int grid = persistent ? std::min(tiles, num_cus()) : tiles;
  hipLaunchKernelGGL((gemm256_kernel<EPI>), dim3(grid), dim3(512), 0, st, y, ldy, x, ldx, w, M, N, K, gm, rs);
}

}  // namespace

// epi: 0 = store y[M, N]; 1 = SwiGLU y[M, N/2] over 32-row interleaved gate/up weights;
// 2 = SwiGLU with the rows' deferred-RMSNorm scales rs[M] (fp32) applied first.
// group_m: token tiles per L2 band.  Requirements: N % 256 == 0, K % 128 == 0,
// 16-byte aligned x / w, x row stride % 8 == 0, y row stride % 4 == 0, y 8-byte aligned.
extern "C" int dx_gemm256(void* y, int64_t ldy, const void* x, int64_t ldx, const void* w, int M, int N, int K,
                          int epi, int group_m, hipStream_t st, const float* rs) {
  if (M < 1) return 0;
  const int persistent = group_m < 1000;  // A/B switch: group_m + 1000 launches one workgroup per tile
  if (!persistent) group_m -= 1000;
  if (group_m < 1) return 7;
  if (N % kBN != 0 || K % (2 * kBK) != 0 || K < 2 * kBK) return 3;
  if ((ldx & 7) || (ldy & 3) || (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 7))
    return 5;
  if ((int64_t)N * K >= (1ll << 31) || (int64_t)kBM * ldx >= (1ll << 31)) return 6;  // 32-bit DMA offsets
  auto* Y = static_cast<bf16_t*>(y);
  auto* X = static_cast<const bf16_t*>(x);
  auto* W = static_cast<const bf16_t*>(w);
  if (epi == EPI_STORE) launch<EPI_STORE>(Y, ldy, X, ldx, W, M, N, K, group_m, persistent, st, nullptr);
  else if (epi == EPI_SILU) launch<EPI_SILU>(Y, ldy, X, ldx, W, M, N, K, group_m, persistent, st, nullptr);
  else if (epi == EPI_SILU_RS && rs != nullptr) launch<EPI_SILU_RS>(Y, ldy, X, ldx, W, M, N, K, group_m, persistent, st, rs);
  else return 2;
  DX_CHECK_LAUNCH();
  return 0;
}
