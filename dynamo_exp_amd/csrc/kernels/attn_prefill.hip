// Paged-KV causal prefill attention (varlen, with cached prefix) for gfx950.
//
// Flash-attention forward on MFMA v_mfma_f32_32x32x16_bf16:
//   * workgroup = 8 waves; every wave owns 32 query rows of ONE query head.
//     The waves of a workgroup share one KV head (GQA group: 4 heads x 2
//     32-token tiles), so every K/V tile staged in LDS is reused by 8 waves;
//     32-row K sub-blocks that lie entirely above a wave's causal diagonal are
//     skipped (no MFMA, no softmax work);
//   * K/V tiles of 64 tokens are gathered from the paged cache (block table)
//     by LDS-DMA (global_load_lds_dwordx4, no staging registers) into a
//     double-buffered, XOR-swizzled LDS image (the swizzle is chosen on the
//     source side), the next tile in flight while the current one computes;
//   * S^T = K . Q^T ("swapped" product): the query row sits on the lane, so the
//     online softmax is lane-local (+1 cross-half exchange) and the S
//     accumulator is directly the B operand of the P.V product
//     O^T = V^T . P^T (guide section 3, "accumulator tile as next operand");
//   * V^T fragments come from the same swizzled image via ds_read_b64_tr_b16
//     (guide T10), K fragments via ds_read_b128; both conflict-free.
//
// Q is read straight from the fused QKV buffer (row stride q_stride) after the
// rope kernel rotated it in place; the new tokens' K/V are already in the paged
// cache, so prefix and new tokens are handled uniformly.
#include "common.h"

#include <type_traits>

namespace {

constexpr int D = 128;
constexpr int BQ = 32;   // query rows per wave
constexpr int BKV = 64;  // kv rows per tile
constexpr int kTileBytes = BKV * D * 2;  // 16 KiB

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// byte offset of 16-B chunk `ch` (0..15) of row `row` inside a [64][128] bf16 tile
__device__ __forceinline__ int tile_off(int row, int ch) { return row * 256 + 16 * (ch ^ swz(row)); }

__device__ __forceinline__ bf16x8_t as_frag(const u16x8& v) { return __builtin_bit_cast(bf16x8_t, v); }

// ---------------------------------------------------------------------------
// The kernel: 8 waves (4 heads x 64 query tokens per workgroup sharing each
// K/V tile), K/V staged by LDS-DMA (global_load_lds) into a double-buffered
// swizzled image, with the per-tile vector work cut down -- the loop is
// issue-bound, not MFMA-bound, at 2 waves/SIMD.  (Earlier register-staged
// 4/8-wave, 4-wave x 2 q-block and 3-stage-DMA variants measured 322-794
// TFLOP/s vs 592-875 for this one: profiles/r1_prefill_attn_*.json; removed.)
// (each MFMA holds the SIMD's vector issue for 8 of its 32 cycles; v_exp 8,
// everything else 4 cycles of issue, MI355X_MICROARCH constants table):
//   * LDS fragment addresses are per-lane constants (the XOR swizzle only
//     depends on row bits 0..3, so +32 rows / +16 rows / the other buffer are
//     immediate offsets): the loop is unrolled over the two buffers;
//   * with block_size >= 64 a full tile lies in one KV block, so the DMA source
//     is a scalar base (one scalar block-table load) + a per-lane constant;
//     only the context's last tile takes the clamped per-lane path;
//   * masking only on diagonal / ragged tiles, by select (no branches);
//     softmax in packed fp32 (v_pk_fma), scale folded into the FMA; the row
//     max as two v_max3 chains; the row sum l as ones . P^T on the matrix
//     pipe (the exact sum of the bf16 P the P.V product uses: with the
//     deferred max, profiles/r4_prefill_attn_variants.txt).
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr float kRescaleLog2 = 8.0f;  // deferred-max threshold (log2 units)

// max / sum of a lane's value and the value of the lane 32 apart: on gfx950 one
// v_permlane32_swap (VALU) instead of a ds_bpermute round trip through LDS in
// the softmax's dependent chain
__device__ __forceinline__ float halves_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// one v_max3_f32 / v_max_f32 as written: fmaxf() on MFMA results makes hipcc
// quieten each operand first (a v_max_f32 x, x, x per value in IEEE mode),
// tripling the row-max VALU work of a tile (48 instead of 16 ops per lane)
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float halves_max_raw(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// V: 0 = the round-3 loop (kept for A/B), 1 = round 4: deferred rescale, row
// sum on the matrix pipe, v_max3 row max, static priority, widened epilogue.
// (Round-4 structural variants -- 4-wave workgroups, ping-pong wave halves,
// two tiles per barrier, a software-pipelined QK / softmax -- all measured
// slower: profiles/r4_prefill_attn_variants.txt.)
template <bool BS64, bool PLS, int V>
__global__ void __launch_bounds__(512, 2) prefill_attn_v2_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_seqlens_q, const int* __restrict__ ctx_lens, const int* __restrict__ work,
    int n_q_heads, int n_kv_heads, int bs_shift, int heads_per_wg, float scale_log2e, int causal) {
  constexpr int kBuf = 2 * kTileBytes;  // one (K, V) stage
  constexpr bool kMfmaSum = V == 1;  // row sum l on the matrix pipe
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int block_size = 1 << bs_shift;
  const int G = n_q_heads / n_kv_heads;
  const int head_groups = G / heads_per_wg;
  // grid = (head groups, work items): x fastest in dispatch order, so every
  // work item (heaviest first) goes out for all heads before the next one --
  // a global longest-first schedule -- and consecutive workgroups land on
  // consecutive XCDs, i.e. with 8 KV-head groups each XCD's L2 serves one KV
  // head's tiles for all work items.
  const int kvh = blockIdx.x / head_groups;
  const int hg = blockIdx.x % head_groups;
  const int seq = work[2 * blockIdx.y];
  const int tok0 = work[2 * blockIdx.y + 1];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q_start = cu_seqlens_q[seq];
  const int qlen = cu_seqlens_q[seq + 1] - q_start;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;
  const int r = lane & 31, h = lane >> 5;

  const int head = kvh * G + hg * heads_per_wg + (wid % heads_per_wg);
  const int wtok0 = tok0 + (wid / heads_per_wg) * BQ;
  const bool row_valid = wtok0 + r < qlen;
  // causal 0 (bidirectional, e.g. a vision tower): every query sees the whole
  // context -- only the ragged last tile is masked
  const int my_pos = causal ? pos0 + wtok0 + r : ctx - 1;
  const int wave_min_pos = causal ? pos0 + wtok0 : ctx - 1;
  const int wave_max_pos = causal ? pos0 + min(wtok0 + BQ, qlen) - 1 : ctx - 1;
  const int token_tiles = 8 / heads_per_wg;
  const int wg_last_tok = min(tok0 + token_tiles * BQ, qlen) - 1;
  const int kv_end = causal ? min(ctx, pos0 + wg_last_tok + 1) : ctx;
  const int n_tiles = (kv_end + BKV - 1) / BKV;

  u16x8 qf[8];
  {
    const bf16_t* qp = q + (int64_t)(q_start + wtok0 + r) * q_stride + (int64_t)head * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      qf[ks] = row_valid ? *reinterpret_cast<const u16x8*>(qp + 16 * ks) : u16x8{{0, 0, 0, 0}};
  }

  // ---- per-lane constant LDS offsets ----
  int koff[8];  // K fragment row r (+32 for the second half: +8192 B), chunk 2ks+h
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) koff[ks] = tile_off(r, 2 * ks + h);
  int voff[4][2];  // V^T fragments: rows 4h+qq and 4h+qq+8 (+16 s2, +32 sub: immediates)
  {
    const int g16 = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int ch = dt * 4 + 2 * g16 + (pp >> 1);
      voff[dt][0] = tile_off(4 * h + qq, ch) + 8 * (pp & 1);
      voff[dt][1] = tile_off(4 * h + qq + 8, ch) + 8 * (pp & 1);
    }
  }
  // ---- DMA slots: instruction k of this wave fills tile rows 4*(KPW*wid+k) .. +3 ----
  constexpr int KPW = 2;  // 1-KB pieces of a 16-KB K (or V) tile per wave
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_stride = (int64_t)block_size * D;
  int src_row[KPW], src_off[KPW];
#pragma unroll
  for (int k = 0; k < KPW; ++k) {
    const int row = (KPW * wid + k) * 4 + (lane >> 4);
    src_row[k] = row;
    src_off[k] = row * D + ((lane & 15) ^ swz(row)) * 8;
  }
  typedef __attribute__((address_space(3))) void lds_void;
  auto dma = [&](const bf16_t* g, char* l) { __builtin_amdgcn_global_load_lds(g, (lds_void*)l, 16, 0, 0); };
  auto issue = [&](char* kb, int j0) {
    char* vb = kb + kTileBytes;
    if (BS64 && j0 + BKV <= ctx) {
      const int blk = bt[j0 >> bs_shift];  // uniform -> scalar load
      const int64_t base = ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(j0 & (block_size - 1)) * D;
#pragma unroll
      for (int k = 0; k < KPW; ++k) {
        dma(k_cache + base + src_off[k], kb + (KPW * wid + k) * 1024);
        dma(v_cache + base + src_off[k], vb + (KPW * wid + k) * 1024);
      }
    } else {
#pragma unroll
      for (int k = 0; k < KPW; ++k) {
        // rows past the context read row ctx-1 (finite); a wave's 4-row group
        // (block_size % 4 == 0) lies in one KV block, so the block-table read is
        // wave-uniform (a scalar load) even with the clamp
        const int j = min(j0 + src_row[k], ctx - 1);
        const int blk = bt[min(j0 + 4 * (KPW * wid + k), ctx - 1) >> bs_shift];
        const int64_t o = ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(j & (block_size - 1)) * D +
                          (src_off[k] - src_row[k] * D);
        dma(k_cache + o, kb + (KPW * wid + k) * 1024);
        dma(v_cache + o, vb + (KPW * wid + k) * 1024);
      }
    }
  };

  f32x16 o_acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o_acc[i] = f32x16{};
  float m_i = -1e30f, l_i = 0.f;
  f32x16 l_acc = f32x16{};  // V1: every row of the 32 x 32 tile = l of the lane's query column
  const bf16x8_t kOnes = __builtin_bit_cast(bf16x8_t, u16x8{{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u}});
  const f32x2 sc2 = {scale_log2e, scale_log2e};

  // segment 1 of a tile: S^T = K . Q^T, mask, online softmax -> this wave's
  // bf16 P fragments (and the O / l rescale); false: nothing of the tile is
  // at or below this wave's diagonal
  auto qk_sm = [&](const char* kb, int t, u16x8 (&pf)[2][2], bool& live1) -> bool {
    const int j0 = t * BKV;
    live1 = j0 + 32 <= wave_max_pos;
    if (j0 > wave_max_pos) return false;
    f32x16 s0 = f32x16{}, s1 = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const u16x8 kf = *reinterpret_cast<const u16x8*>(kb + koff[ks]);
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(kf), as_frag(qf[ks]), s0, 0, 0, 0);
    }
    if (live1) {
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const u16x8 kf = *reinterpret_cast<const u16x8*>(kb + 8192 + koff[ks]);
        s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(kf), as_frag(qf[ks]), s1, 0, 0, 0);
      }
    }
    if ((j0 + BKV - 1 > wave_min_pos) || (j0 + BKV > ctx)) {  // diagonal / ragged tile
      const int lim = min(my_pos, ctx - 1) - j0 - 4 * h;  // keep kv row j0 + 4h + off <= lim + j0 + 4h
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int off = (i & 3) + 8 * (i >> 2);
        s0[i] = off > lim ? -INFINITY : s0[i];
        s1[i] = off + 32 > lim ? -INFINITY : s1[i];
      }
    }
    // (!live1 implies a diagonal tile: the select above already set every
    // valid row's second half to -inf, and its P.V half is skipped below)
    float tmax;
    if constexpr (kMfmaSum) {  // two independent v_max3 chains, no canonicalising moves
      float ta = vmax(s0[0], s1[0]), tb = vmax(s0[1], s1[1]);
#pragma unroll
      for (int i = 2; i < 16; i += 2) {
        ta = vmax3(ta, s0[i], s1[i]);
        tb = vmax3(tb, s0[i + 1], s1[i + 1]);
      }
      tmax = halves_max_raw(vmax(ta, tb));
    } else {
      float ta = -INFINITY, tb = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        ta = fmaxf(ta, fmaxf(s0[i], s1[i]));
        tb = fmaxf(tb, fmaxf(s0[i + 1], s1[i + 1]));
      }
      tmax = fmaxf(ta, tb);
      tmax = PLS ? halves_max(tmax) : fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    }
    // deferred rescale (guide T13): the running max moves only when the
    // tile's max exceeds it by more than kRescaleLog2, so P = 2^(s - m) stays
    // <= 2^kRescaleLog2 (exact enough in bf16 / fp32) and the O / l rescale
    // below is skipped on almost every tile; both halves of a row (lanes r,
    // r + 32) see the same tmax, so they always take the same decision
    const float t_s = tmax * scale_log2e;
    const float m_new = t_s > m_i + (V == 1 ? kRescaleLog2 : 0.f) ? t_s : m_i;
    const float alpha = fast_exp2(m_i - m_new);
    m_i = m_new;
    const f32x2 nm2 = {-m_new, -m_new};
    f32x2 rs2 = {0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int i = 8 * s2 + 2 * w;
        const f32x2 a0 = f32x2{s0[i], s0[i + 1]} * sc2 + nm2;
        const f32x2 a1 = f32x2{s1[i], s1[i + 1]} * sc2 + nm2;
        const f32x2 p0 = {fast_exp2(a0.x), fast_exp2(a0.y)};
        const f32x2 p1 = {fast_exp2(a1.x), fast_exp2(a1.y)};
        pf[0][s2].w[w] = pack_bf16x2(p0.x, p0.y);
        pf[1][s2].w[w] = pack_bf16x2(p1.x, p1.y);
        if constexpr (!kMfmaSum) rs2 += p0 + p1;  // V1: l_acc below
      }
    if constexpr (!kMfmaSum) {
      float rs = rs2.x + rs2.y;
      rs = PLS ? halves_sum(rs) : rs + __shfl_xor(rs, 32, 64);
      l_i = l_i * alpha + rs;
    }
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o_acc[dt] *= alpha;
      if constexpr (kMfmaSum) l_acc *= alpha;
    }
    return true;
  };
  // segment 2: O^T += V^T . P^T (+ l on the matrix pipe)
  auto pv = [&](const char* vb, bool live1, const u16x8 (&pf)[2][2]) {
    // O^T[d][q] += V^T[d][kv] . P^T[kv][q]
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      if (sub == 1 && !live1) break;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_i16x4*)(vb + sub * 8192 + s2 * 4096 + voff[dt][0]));
          const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_i16x4*)(vb + sub * 8192 + s2 * 4096 + voff[dt][1]));
          typedef short i16x8 __attribute__((ext_vector_type(8)));
          const i16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o_acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, vv),
                                                              as_frag(pf[sub][s2]), o_acc[dt], 0, 0, 0);
        }
        // l += ones . P^T: the row sum of exactly the bf16 P the P.V product
        // used (O / l stays an exact weighted mean of V rows under the
        // deferred max), on the matrix pipe instead of 16 packed adds + a
        // cross-half exchange on the issue-bound VALU
        if constexpr (kMfmaSum)
          l_acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kOnes, as_frag(pf[sub][s2]), l_acc, 0, 0, 0);
      }
    }
  };

  {
    auto step = [&](auto bufc, int t) {
      constexpr int BUF = decltype(bufc)::value;
      char* kb = smem + BUF * kBuf;
      if (t + 1 < n_tiles) issue(smem + (BUF ^ 1) * kBuf, t * BKV + BKV);
      u16x8 pf[2][2];
      bool live1;
      if (qk_sm(kb, t, pf, live1)) pv(kb + kTileBytes, live1, pf);
      __syncthreads();  // the compiler's vmcnt(0) here retires this wave's DMA of tile t+1
    };
    if (n_tiles > 0) issue(smem, 0);
    // static priority for the second-dispatched half (guide "Two waves per
    // SIMD" item 4): without it waves 4-7 lose every arbitration
    if (V != 0 && wid >= 4) __builtin_amdgcn_s_setprio(1);
    __syncthreads();
    for (int t = 0; t < n_tiles; t += 2) {
      step(std::integral_constant<int, 0>{}, t);
      if (t + 1 < n_tiles) step(std::integral_constant<int, 1>{}, t + 1);
    }
  }

  // epilogue, widened (guide T21): lane (r, h) holds columns 8 g + 4 h .. + 3
  // of each 8-column group g; one v_permlane32_swap per dword pairs groups
  // (g, g + 1) so each lane stores 16 contiguous bytes: half the stores
  if constexpr (kMfmaSum) l_i = l_acc[0];
  const float inv_l = l_i > 0.f ? 1.f / l_i : 0.f;
  bf16_t* op = out + ((int64_t)(q_start + wtok0 + r) * n_q_heads + head) * D;
  if constexpr (V == 0) {  // A/B baseline: 8-byte stores
    if (!row_valid) return;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        uint2 v;
        v.x = pack_bf16x2(o_acc[dt][4 * g4 + 0] * inv_l, o_acc[dt][4 * g4 + 1] * inv_l);
        v.y = pack_bf16x2(o_acc[dt][4 * g4 + 2] * inv_l, o_acc[dt][4 * g4 + 3] * inv_l);
        *reinterpret_cast<uint2*>(op + dt * 32 + 8 * g4 + 4 * h) = v;
      }
    return;
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; g4 += 2) {
      uint2 a, b;
      a.x = pack_bf16x2(o_acc[dt][4 * g4 + 0] * inv_l, o_acc[dt][4 * g4 + 1] * inv_l);
      a.y = pack_bf16x2(o_acc[dt][4 * g4 + 2] * inv_l, o_acc[dt][4 * g4 + 3] * inv_l);
      b.x = pack_bf16x2(o_acc[dt][4 * g4 + 4] * inv_l, o_acc[dt][4 * g4 + 5] * inv_l);
      b.y = pack_bf16x2(o_acc[dt][4 * g4 + 6] * inv_l, o_acc[dt][4 * g4 + 7] * inv_l);
      const auto sx = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
      const auto sy = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
      a.x = sx[0];
      b.x = sx[1];
      a.y = sy[0];
      b.y = sy[1];
      if (row_valid)  // after the swaps: every lane takes part in them
        *reinterpret_cast<uint4*>(op + dt * 32 + 8 * g4 + 8 * h) = make_uint4(a.x, a.y, b.x, b.y);
    }
}


}  // namespace

extern "C" int dx_prefill_attention(void* out, const void* q, int64_t q_stride, const void* k_cache,
                                    const void* v_cache, const int* block_tables, int bt_stride,
                                    const int* cu_seqlens_q, const int* ctx_lens, const int* work, int n_work,
                                    int n_q_heads, int n_kv_heads, int head_dim, int block_size, float scale,
                                    int causal, int n_waves, hipStream_t stream) {
  if (head_dim != D || n_q_heads % n_kv_heads) return -1;
  const int G = n_q_heads / n_kv_heads;
  const int hpw = G >= 4 ? 4 : G;
  if (G % hpw || (hpw != 1 && hpw != 2 && hpw != 4)) return -2;
  if (n_work == 0) return 0;
  const int bs_shift = __builtin_ctz((unsigned)block_size);
  if (block_size < 4 || (1 << bs_shift) != block_size) return -3;
  dim3 grid(n_kv_heads * (G / hpw), n_work);
  const float sl2e = scale * 1.4426950408889634f;
  // n_waves 92 selects the pre-round-4 loop (A/B runs: tools/attn_ab.py,
  // tools/attn_accuracy.py)
  const bool r3 = n_waves == 92;
#define DX_PA_LAUNCH(BS, VV)                                                                                         \
  prefill_attn_v2_kernel<BS, true, VV><<<grid, 512, 0, stream>>>((bf16_t*)out, (const bf16_t*)q, q_stride,           \
                                                                (const bf16_t*)k_cache, (const bf16_t*)v_cache,       \
                                                                block_tables, bt_stride, cu_seqlens_q, ctx_lens, work, \
                                                                n_q_heads, n_kv_heads, bs_shift, hpw, sl2e, causal)
  if (block_size >= 64) {
    if (r3) DX_PA_LAUNCH(true, 0);
    else DX_PA_LAUNCH(true, 1);
  } else {
    if (r3) DX_PA_LAUNCH(false, 0);
    else DX_PA_LAUNCH(false, 1);
  }
#undef DX_PA_LAUNCH
  return (int)hipGetLastError();
}

// query tokens per work item (the Python work list must use the same value)
extern "C" int dx_prefill_tile_tokens(int n_q_heads, int n_kv_heads, int n_waves) {
  const int G = n_q_heads / n_kv_heads;
  const int hpw = G >= 4 ? 4 : G;
  (void)n_waves;
  return (8 / hpw) * BQ;  // 8 waves x 32 query rows over hpw heads
}
