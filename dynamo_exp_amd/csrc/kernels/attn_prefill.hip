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
//     softmax in packed fp32 (v_pk_fma / v_pk_add), scale folded into the FMA.
typedef float f32x2 __attribute__((ext_vector_type(2)));

// max / sum of a lane's value and the value of the lane 32 apart: on gfx950 one
// v_permlane32_swap (VALU) instead of a ds_bpermute round trip through LDS in
// the softmax's dependent chain
__device__ __forceinline__ float halves_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <bool BS64, bool PLS>
__global__ void __launch_bounds__(512, 2) prefill_attn_v2_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_seqlens_q, const int* __restrict__ ctx_lens, const int* __restrict__ work,
    int n_q_heads, int n_kv_heads, int bs_shift, int heads_per_wg, float scale_log2e) {
  constexpr int kBuf = 2 * kTileBytes;  // one (K, V) stage
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
  const int my_pos = pos0 + wtok0 + r;
  const int wave_min_pos = pos0 + wtok0;
  const int wave_max_pos = pos0 + min(wtok0 + BQ, qlen) - 1;
  const int token_tiles = 8 / heads_per_wg;
  const int wg_last_tok = min(tok0 + token_tiles * BQ, qlen) - 1;
  const int kv_end = min(ctx, pos0 + wg_last_tok + 1);
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
  // ---- DMA slots: instruction k of this wave fills tile rows 4*(2*wid+k) .. +3 ----
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_stride = (int64_t)block_size * D;
  int src_row[2], src_off[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = (2 * wid + k) * 4 + (lane >> 4);
    src_row[k] = row;
    src_off[k] = row * D + ((lane & 15) ^ swz(row)) * 8;
  }
  typedef __attribute__((address_space(3))) void lds_void;
  auto issue = [&](char* kb, int j0) {
    char* vb = kb + kTileBytes;
    if (BS64 && j0 + BKV <= ctx) {
      const int blk = bt[j0 >> bs_shift];  // uniform -> scalar load
      const int64_t base = ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(j0 & (block_size - 1)) * D;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        __builtin_amdgcn_global_load_lds(k_cache + base + src_off[k], (lds_void*)(kb + (2 * wid + k) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(v_cache + base + src_off[k], (lds_void*)(vb + (2 * wid + k) * 1024), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int j = min(j0 + src_row[k], ctx - 1);  // rows past the context read row ctx-1 (finite)
        const int blk = bt[j >> bs_shift];
        const int64_t o = ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(j & (block_size - 1)) * D +
                          (src_off[k] - src_row[k] * D);
        __builtin_amdgcn_global_load_lds(k_cache + o, (lds_void*)(kb + (2 * wid + k) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(v_cache + o, (lds_void*)(vb + (2 * wid + k) * 1024), 16, 0, 0);
      }
    }
  };

  f32x16 o_acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o_acc[i] = f32x16{};
  float m_i = -1e30f, l_i = 0.f;
  const f32x2 sc2 = {scale_log2e, scale_log2e};

  auto step = [&](auto bufc, int t) {
    constexpr int BUF = decltype(bufc)::value;
    char* kb = smem + BUF * kBuf;
    const char* vb = kb + kTileBytes;
    const int j0 = t * BKV;
    if (t + 1 < n_tiles) issue(smem + (BUF ^ 1) * kBuf, j0 + BKV);
    const bool live0 = j0 <= wave_max_pos, live1 = j0 + 32 <= wave_max_pos;
    if (live0) {
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
      float ta = -INFINITY, tb = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        ta = fmaxf(ta, fmaxf(s0[i], s1[i]));
        tb = fmaxf(tb, fmaxf(s0[i + 1], s1[i + 1]));
      }
      float tmax = fmaxf(ta, tb);
      tmax = PLS ? halves_max(tmax) : fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float m_new = fmaxf(m_i, tmax * scale_log2e);
      const float alpha = fast_exp2(m_i - m_new);
      m_i = m_new;
      const f32x2 nm2 = {-m_new, -m_new};
      f32x2 rs2 = {0.f, 0.f};
      u16x8 pf[2][2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int i = 8 * s2 + 2 * w;
          const f32x2 a0 = f32x2{s0[i], s0[i + 1]} * sc2 + nm2;
          const f32x2 a1 = f32x2{s1[i], s1[i + 1]} * sc2 + nm2;
          const f32x2 p0 = {fast_exp2(a0.x), fast_exp2(a0.y)};
          const f32x2 p1 = {fast_exp2(a1.x), fast_exp2(a1.y)};
          rs2 += p0 + p1;
          pf[0][s2].w[w] = pack_bf16x2(p0.x, p0.y);
          pf[1][s2].w[w] = pack_bf16x2(p1.x, p1.y);
        }
      float rs = rs2.x + rs2.y;
      rs = PLS ? halves_sum(rs) : rs + __shfl_xor(rs, 32, 64);
      l_i = l_i * alpha + rs;
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o_acc[dt] *= alpha;
      }
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
        }
      }
    }
    __syncthreads();  // the compiler's vmcnt(0) here retires this wave's DMA of tile t+1
  };

  if (n_tiles > 0) issue(smem, 0);
  __syncthreads();
  for (int t = 0; t < n_tiles; t += 2) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 < n_tiles) step(std::integral_constant<int, 1>{}, t + 1);
  }

  if (!row_valid) return;
  const float inv_l = l_i > 0.f ? 1.f / l_i : 0.f;
  bf16_t* op = out + ((int64_t)(q_start + wtok0 + r) * n_q_heads + head) * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = dt * 32 + 8 * g4 + 4 * h;
      uint2 v;
      v.x = pack_bf16x2(o_acc[dt][4 * g4 + 0] * inv_l, o_acc[dt][4 * g4 + 1] * inv_l);
      v.y = pack_bf16x2(o_acc[dt][4 * g4 + 2] * inv_l, o_acc[dt][4 * g4 + 3] * inv_l);
      *reinterpret_cast<uint2*>(op + d) = v;
    }
}


// ---------------------------------------------------------------------------
// v3: the same workgroup / fragment layout as v2, software-pipelined across
// KV tiles inside each wave (VERDICT r2 "softmax of sub-tile j under the
// MFMAs of j+1"): step t issues the Q.K^T MFMAs of tile t+1 and, in the same
// basic block, the softmax of tile t (VALU / transcendental) and its P.V
// MFMAs, so a wave always has independent MFMA work queued behind its softmax
// instead of the two phases alternating for the whole SIMD.  K/V live in a
// 3-stage LDS ring (96 KB): tile t (V for P.V), tile t+1 (K for Q.K^T), tile
// t+2 in flight by LDS-DMA; one barrier per tile.  Every tile computes both
// 32-row halves (no causal MFMA skipping -- wasted work only on a wave's
// diagonal tile); the causal / ragged mask is a select, taken by a per-wave
// branch around the whole step so each step body stays one basic block.
#define DX_V3_QLDS 1  // Q fragments in LDS: 250 VGPRs, no spills (in VGPRs: 256 + 14 spilled)
template <bool BS64>
__global__ void __launch_bounds__(512, 2) prefill_attn_v3_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_seqlens_q, const int* __restrict__ ctx_lens, const int* __restrict__ work,
    int n_q_heads, int n_kv_heads, int bs_shift, int heads_per_wg, float scale_log2e) {
  constexpr int kBuf = 2 * kTileBytes;  // one (K, V) stage
#ifdef DX_V3_QLDS
  // K/V ring + this wave's Q fragments (8 waves x 32 rows x 256 B = 64 KB)
  __shared__ __attribute__((aligned(16))) char smem[3 * kBuf + 8 * 8 * 1024];
#else
  __shared__ __attribute__((aligned(16))) char smem[3 * kBuf];
#endif
  const int block_size = 1 << bs_shift;
  const int G = n_q_heads / n_kv_heads;
  const int head_groups = G / heads_per_wg;
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
  const int my_pos = pos0 + wtok0 + r;
  const int wave_min_pos = pos0 + wtok0;
  const int token_tiles = 8 / heads_per_wg;
  const int wg_last_tok = min(tok0 + token_tiles * BQ, qlen) - 1;
  const int kv_end = min(ctx, pos0 + wg_last_tok + 1);
  const int n_tiles = (kv_end + BKV - 1) / BKV;
  // tiles [0, n_plain) need no mask for this wave: below its first row's
  // diagonal and inside the context
  const int n_plain = min((wave_min_pos + 1) / BKV, ctx / BKV);

#ifdef DX_V3_QLDS
  char* qlds = smem + 3 * kBuf + wid * 8 * 1024 + lane * 16;  // fragment ks at + ks * 1024
  {
    const bf16_t* qp = q + (int64_t)(q_start + wtok0 + r) * q_stride + (int64_t)head * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      *reinterpret_cast<u16x8*>(qlds + ks * 1024) =
          row_valid ? *reinterpret_cast<const u16x8*>(qp + 16 * ks) : u16x8{{0, 0, 0, 0}};
  }
  auto QF = [&](int ks) { return *reinterpret_cast<const u16x8*>(qlds + ks * 1024); };
#else
  u16x8 qf[8];
  {
    const bf16_t* qp = q + (int64_t)(q_start + wtok0 + r) * q_stride + (int64_t)head * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      qf[ks] = row_valid ? *reinterpret_cast<const u16x8*>(qp + 16 * ks) : u16x8{{0, 0, 0, 0}};
  }
  auto QF = [&](int ks) { return qf[ks]; };
#endif
  int koff[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) koff[ks] = tile_off(r, 2 * ks + h);
  int voff[4][2];
  {
    const int g16 = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int ch = dt * 4 + 2 * g16 + (pp >> 1);
      voff[dt][0] = tile_off(4 * h + qq, ch) + 8 * (pp & 1);
      voff[dt][1] = tile_off(4 * h + qq + 8, ch) + 8 * (pp & 1);
    }
  }
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  const int64_t head_stride = (int64_t)block_size * D;
  int src_row[2], src_off[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = (2 * wid + k) * 4 + (lane >> 4);
    src_row[k] = row;
    src_off[k] = row * D + ((lane & 15) ^ swz(row)) * 8;
  }
  typedef __attribute__((address_space(3))) void lds_void;
  auto issue = [&](char* kb, int j0) {
    char* vb = kb + kTileBytes;
    if (BS64 && j0 + BKV <= ctx) {
      const int blk = bt[j0 >> bs_shift];
      const int64_t base = ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(j0 & (block_size - 1)) * D;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        __builtin_amdgcn_global_load_lds(k_cache + base + src_off[k], (lds_void*)(kb + (2 * wid + k) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(v_cache + base + src_off[k], (lds_void*)(vb + (2 * wid + k) * 1024), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int j = min(j0 + src_row[k], ctx - 1);
        const int blk = bt[j >> bs_shift];
        const int64_t o = ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(j & (block_size - 1)) * D +
                          (src_off[k] - src_row[k] * D);
        __builtin_amdgcn_global_load_lds(k_cache + o, (lds_void*)(kb + (2 * wid + k) * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds(v_cache + o, (lds_void*)(vb + (2 * wid + k) * 1024), 16, 0, 0);
      }
    }
  };

  f32x16 o_acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o_acc[i] = f32x16{};
  float m_i = -1e30f, l_i = 0.f;
  const f32x2 sc2 = {scale_log2e, scale_log2e};

  // Q.K^T of the first tile (prologue; later tiles' S come out of `fused`)
  auto qk = [&](const char* kb, f32x16& s0, f32x16& s1) {
    s0 = f32x16{};
    s1 = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const u16x8 k0 = *reinterpret_cast<const u16x8*>(kb + koff[ks]);
      const u16x8 k1 = *reinterpret_cast<const u16x8*>(kb + 8192 + koff[ks]);
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(k0), as_frag(QF(ks)), s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(k1), as_frag(QF(ks)), s1, 0, 0, 0);
    }
  };

  // One step's hand-placed schedule: 8 slots, each = the K fragments of the
  // next slot (one slot of LDS latency cover), two Q.K^T MFMAs of tile t+1
  // (when `next`), and one chunk of tile t's softmax -- slot 0 the mask and
  // row max, 1-4 the exponentials and P packing, 5 the row sum, 6-7 the O
  // rescale; sched_barrier(0) closes each slot.  Then P.V(t).
  auto fused = [&](const char* kbn, const char* vb, int j0, f32x16& s0, f32x16& s1, f32x16& n0, f32x16& n1,
                   auto maskc, auto nextc) {
    constexpr bool MASK = decltype(maskc)::value, NEXT = decltype(nextc)::value;
    n0 = f32x16{};
    n1 = f32x16{};
    u16x8 kf[2][2];
    if constexpr (NEXT) {
      kf[0][0] = *reinterpret_cast<const u16x8*>(kbn + koff[0]);
      kf[0][1] = *reinterpret_cast<const u16x8*>(kbn + 8192 + koff[0]);
    }
    float alpha = 1.f;
    f32x2 nm2 = {0.f, 0.f}, rs2 = {0.f, 0.f};
    u16x8 pf[2][2];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if constexpr (NEXT) {
        if (ks + 1 < 8) {
          kf[(ks + 1) & 1][0] = *reinterpret_cast<const u16x8*>(kbn + koff[ks + 1]);
          kf[(ks + 1) & 1][1] = *reinterpret_cast<const u16x8*>(kbn + 8192 + koff[ks + 1]);
        }
        n0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(kf[ks & 1][0]), as_frag(QF(ks)), n0, 0, 0, 0);
        n1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(kf[ks & 1][1]), as_frag(QF(ks)), n1, 0, 0, 0);
      }
      if (ks == 0) {
        if constexpr (MASK) {
          const int lim = min(my_pos, ctx - 1) - j0 - 4 * h;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int off = (i & 3) + 8 * (i >> 2);
            s0[i] = off > lim ? -INFINITY : s0[i];
            s1[i] = off + 32 > lim ? -INFINITY : s1[i];
          }
        }
        float ta = -INFINITY, tb = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          ta = fmaxf(ta, fmaxf(s0[i], s1[i]));
          tb = fmaxf(tb, fmaxf(s0[i + 1], s1[i + 1]));
        }
        const float tmax = halves_max(fmaxf(ta, tb));
        const float m_new = fmaxf(m_i, tmax * scale_log2e);
        alpha = fast_exp2(m_i - m_new);
        m_i = m_new;
        nm2 = f32x2{-m_new, -m_new};
      } else if (ks <= 4) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int it = 2 * (ks - 1) + u, s2 = it >> 2, w = it & 3, i = 8 * s2 + 2 * w;
          const f32x2 a0 = f32x2{s0[i], s0[i + 1]} * sc2 + nm2;
          const f32x2 a1 = f32x2{s1[i], s1[i + 1]} * sc2 + nm2;
          const f32x2 p0 = {fast_exp2(a0.x), fast_exp2(a0.y)};
          const f32x2 p1 = {fast_exp2(a1.x), fast_exp2(a1.y)};
          rs2 += p0 + p1;
          pf[0][s2].w[w] = pack_bf16x2(p0.x, p0.y);
          pf[1][s2].w[w] = pack_bf16x2(p1.x, p1.y);
        }
      } else if (ks == 5) {
        l_i = l_i * alpha + halves_sum(rs2.x + rs2.y);
      } else {
        const int d0 = 2 * (ks - 6);
        o_acc[d0] *= alpha;
        o_acc[d0 + 1] *= alpha;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // P.V in 4 groups of 4 MFMAs; the V^T fragments of group g+1 are read
    // during group g (8 reads in flight at most)
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    auto vread = [&](int g, i16x8 (&vv)[4]) {
      const int sub = g >> 1, s2 = g & 1;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(vb + sub * 8192 + s2 * 4096 + voff[dt][0]));
        const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(vb + sub * 8192 + s2 * 4096 + voff[dt][1]));
        vv[dt] = i16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    };
    i16x8 vv[2][4];
    vread(0, vv[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g + 1 < 4) vread(g + 1, vv[(g + 1) & 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o_acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, vv[g & 1][dt]),
                                                            as_frag(pf[g >> 1][g & 1]), o_acc[dt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  f32x16 sc0, sc1;  // S of the current tile
  // step t with the tile in ring slot B (B = t % 3): K of t+1 in slot (B+1)%3,
  // the DMA of t+2 goes to slot (B+2)%3 (read by every wave in step t-1)
  auto step = [&](auto bc, int t) {
    constexpr int B = decltype(bc)::value;
    char* cur = smem + B * kBuf;
    char* nxt = smem + ((B + 1) % 3) * kBuf;
    char* fut = smem + ((B + 2) % 3) * kBuf;
    // the DMA of t+1 (issued in step t-1) is this wave's only one outstanding
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile t+1 resident; slot (B+2)%3 free
    if (t + 2 < n_tiles) issue(fut, (t + 2) * BKV);
    f32x16 n0, n1;
    const int j0 = t * BKV;
    if (t + 1 < n_tiles) {
      if (t < n_plain)
        fused(nxt, cur + kTileBytes, j0, sc0, sc1, n0, n1, std::false_type{}, std::true_type{});
      else
        fused(nxt, cur + kTileBytes, j0, sc0, sc1, n0, n1, std::true_type{}, std::true_type{});
    } else {
      fused(nxt, cur + kTileBytes, j0, sc0, sc1, n0, n1, std::true_type{}, std::false_type{});
    }
    sc0 = n0;
    sc1 = n1;
  };

  if (n_tiles > 0) {
    issue(smem, 0);
    if (n_tiles > 1) issue(smem + kBuf, BKV);
    // tile 0 = this wave's 4 oldest DMAs; tile 1's 4 may stay in flight
    if (n_tiles > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    qk(smem, sc0, sc1);
  }
  for (int t = 0; t < n_tiles; t += 3) {
    step(std::integral_constant<int, 0>{}, t);
    if (t + 1 < n_tiles) step(std::integral_constant<int, 1>{}, t + 1);
    if (t + 2 < n_tiles) step(std::integral_constant<int, 2>{}, t + 2);
  }

  if (!row_valid) return;
  const float inv_l = l_i > 0.f ? 1.f / l_i : 0.f;
  bf16_t* op = out + ((int64_t)(q_start + wtok0 + r) * n_q_heads + head) * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = dt * 32 + 8 * g4 + 4 * h;
      uint2 v;
      v.x = pack_bf16x2(o_acc[dt][4 * g4 + 0] * inv_l, o_acc[dt][4 * g4 + 1] * inv_l);
      v.y = pack_bf16x2(o_acc[dt][4 * g4 + 2] * inv_l, o_acc[dt][4 * g4 + 3] * inv_l);
      *reinterpret_cast<uint2*>(op + d) = v;
    }
}

}  // namespace

// work: int32 [n_work, 2] = (seq index, first new-token index of a
// (4/heads_per_wg)*32-token tile).  out: [T, Hq, D].
extern "C" int dx_prefill_attention(void* out, const void* q, int64_t q_stride, const void* k_cache,
                                    const void* v_cache, const int* block_tables, int bt_stride,
                                    const int* cu_seqlens_q, const int* ctx_lens, const int* work, int n_work,
                                    int n_q_heads, int n_kv_heads, int head_dim, int block_size, float scale,
                                    int n_waves, hipStream_t stream) {
  if (head_dim != D || n_q_heads % n_kv_heads) return -1;
  const int G = n_q_heads / n_kv_heads;
  const int hpw = G >= 4 ? 4 : G;
  if (G % hpw || (hpw != 1 && hpw != 2 && hpw != 4)) return -2;
  if (n_work == 0) return 0;
  const int bs_shift = __builtin_ctz((unsigned)block_size);
  if (block_size <= 0 || (1 << bs_shift) != block_size) return -3;
  dim3 grid(n_kv_heads * (G / hpw), n_work);
  const float sl2e = scale * 1.4426950408889634f;
  // n_waves 90 selects the ds_bpermute half exchange (A/B harness: tools/attn_ab.py; raising
  // the wave priority around the MFMA phases measured 0.5-1 % slower and was dropped)
  const bool pls = n_waves != 90;
#define DX_PA_LAUNCH(BS, P)                                                                                         \
  prefill_attn_v2_kernel<BS, P><<<grid, 512, 0, stream>>>((bf16_t*)out, (const bf16_t*)q, q_stride,                 \
                                                         (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables, \
                                                         bt_stride, cu_seqlens_q, ctx_lens, work, n_q_heads,           \
                                                         n_kv_heads, bs_shift, hpw, sl2e)
  if (n_waves == 93) {  // software-pipelined variant (A/B: tools/attn_ab.py)
    if (block_size >= 64)
      prefill_attn_v3_kernel<true><<<grid, 512, 0, stream>>>((bf16_t*)out, (const bf16_t*)q, q_stride,
                                                             (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                                                             block_tables, bt_stride, cu_seqlens_q, ctx_lens, work,
                                                             n_q_heads, n_kv_heads, bs_shift, hpw, sl2e);
    else
      prefill_attn_v3_kernel<false><<<grid, 512, 0, stream>>>((bf16_t*)out, (const bf16_t*)q, q_stride,
                                                              (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                                                              block_tables, bt_stride, cu_seqlens_q, ctx_lens, work,
                                                              n_q_heads, n_kv_heads, bs_shift, hpw, sl2e);
    return (int)hipGetLastError();
  }
  if (block_size >= 64) {
    if (pls) DX_PA_LAUNCH(true, true);
    else DX_PA_LAUNCH(true, false);
  } else {
    if (pls) DX_PA_LAUNCH(false, true);
    else DX_PA_LAUNCH(false, false);
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
