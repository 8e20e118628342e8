// Fused rotary embedding (neox / rotate-half form, llama3 scaled table) +
// paged KV-cache write, for gfx950.
//
// Input is the fused QKV projection output [T, (Hq + 2*Hkv) * D] (bf16).  Q and
// K are rotated in place; the rotated K and the V rows are scattered into the
// paged cache at `slot_mapping[t]` (slot = block * BS + offset; < 0 = skip,
// used for padded graph slots).  The cache layout is
//   K, V : [num_blocks, Hkv, BS, D]
// so one (block, kv-head) is a contiguous BS x D tile -- the unit the
// attention kernels stream and the P->D transfer packs.
//
// Work item = 4 rotation pairs (8 + 8 bytes) or 8 V elements (16 bytes), so
// every global access is a vector access; the cos/sin table is precomputed on
// the host (guide App. B: no on-device trig).
//
// FP8 cache (F8): K and V are stored as OCP e4m3fn bytes, x / scale clamped to
// +-448 (v_cvt_pk_fp8_f32), with per-tensor scales; the attention kernels
// dequantize on load (decode) or in a pre-pass (prefill, kv_dequant below).
#include <type_traits>

#include "common.h"

namespace {

constexpr int kThreads = 256;

struct __attribute__((aligned(8))) u16x4 {
  uint32_t w[2];
};

// 4 floats -> 4 e4m3 bytes (clamped: a rounding overshoot never makes the NaN code)
__device__ __forceinline__ uint32_t fp8x4(float a, float b, float c, float d, float inv) {
  auto cl = [inv](float x) { return fminf(fmaxf(x * inv, -448.f), 448.f); };
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(cl(a), cl(b), 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(cl(c), cl(d), w, true);
}

// S > 0: the QKV projection's output is still S split-K fp32 slabs (slice s,
// token t at slabs + s * slab_stride + t * row_len, dstream_gemm flags 1); each
// value is their slice-ordered sum rounded to bf16 -- what the reduction kernel
// would have stored -- and the whole bf16 row (rotated Q / K, V) is written to
// qkv, as the unfused path leaves it.
template <int S>
__device__ __forceinline__ void slab_sum(const float* p, int64_t stride, float* o, int n) {
  f32x4 v[S][2];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    v[s][0] = *reinterpret_cast<const f32x4*>(p + s * stride);
    if (n == 8) v[s][1] = *reinterpret_cast<const f32x4*>(p + s * stride + 4);
  }
  f32x4 a = v[0][0], b = v[0][1];
#pragma unroll
  for (int s = 1; s < S; ++s) {
    a += v[s][0];
    if (n == 8) b += v[s][1];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = a[k];
  if (n == 8)
#pragma unroll
    for (int k = 0; k < 4; ++k) o[4 + k] = b[k];
}

template <typename PosT, bool F8, int S = 0>
__global__ void __launch_bounds__(kThreads)
    rope_cache_kernel(bf16_t* __restrict__ qkv, int64_t qkv_stride, const PosT* __restrict__ positions,
                      const float* __restrict__ cos_sin, const int64_t* __restrict__ slot_mapping,
                      void* __restrict__ k_cache_, void* __restrict__ v_cache_, int n_q_heads, int n_kv_heads,
                      int head_dim, int block_size, int rotate_q, float k_inv, float v_inv,
                      const float* __restrict__ slabs, int64_t slab_stride, const float* __restrict__ row_scale) {
  using CT = typename std::conditional<F8, uint8_t, bf16_t>::type;
  CT* k_cache = static_cast<CT*>(k_cache_);
  CT* v_cache = static_cast<CT*>(v_cache_);
  const int64_t t = blockIdx.x;
  const int64_t pos = (int64_t)positions[t];
  const int half = head_dim >> 1;
  const int items_per_head_rot = half >> 2;  // 4 pairs per item
  const int items_per_head_v = head_dim >> 3;
  const int n_rot_items = (n_q_heads + n_kv_heads) * items_per_head_rot;
  const int n_items = n_rot_items + n_kv_heads * items_per_head_v;
  bf16_t* row = qkv + t * qkv_stride;
  const int row_len = (n_q_heads + 2 * n_kv_heads) * head_dim;
  const float* srow = S ? slabs + t * row_len : nullptr;
  // row_scale: the projection's input row carried a deferred RMSNorm (1 / rms,
  // the norm weight folded into the weight columns): Q, K and V are scaled by
  // it here, and Q is written back scaled for the attention kernels
  const float rsc = row_scale != nullptr ? row_scale[t] : 1.f;
  const bool scaled = row_scale != nullptr;
  // 4 (8) bf16 of the projection output at column c: from the row, or the slabs' sum
  auto load4 = [&](int c) -> u16x4 {
    if constexpr (S == 0) {
      return *reinterpret_cast<const u16x4*>(row + c);
    } else {
      float f[8];
      slab_sum<S>(srow + c, slab_stride, f, 4);
      u16x4 r;
      r.w[0] = pack_bf16x2(f[0], f[1]);
      r.w[1] = pack_bf16x2(f[2], f[3]);
      return r;
    }
  };
  const float* cs = cos_sin + pos * head_dim;
  const int64_t slot = slot_mapping ? slot_mapping[t] : -1;
  const int64_t blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? (int)(slot % block_size) : 0;

  for (int it = threadIdx.x; it < n_items; it += kThreads) {
    if (it < n_rot_items) {
      const int head = it / items_per_head_rot;  // 0..Hq-1 are q heads, then k heads
      const int i0 = (it % items_per_head_rot) * 4;
      const bool is_k = head >= n_q_heads;
      bf16_t* hp = row + (int64_t)head * head_dim;
      if (!is_k && !rotate_q) {
        if (S != 0 || scaled) {  // unrotated Q still has to land in the row (scaled)
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            u16x4 r = load4(head * head_dim + i0 + h2 * half);
            r.w[0] = pack_bf16x2(bf16lo(r.w[0]) * rsc, bf16hi(r.w[0]) * rsc);
            r.w[1] = pack_bf16x2(bf16lo(r.w[1]) * rsc, bf16hi(r.w[1]) * rsc);
            *reinterpret_cast<u16x4*>(hp + i0 + h2 * half) = r;
          }
        }
        continue;
      }
      u16x4 a = load4(head * head_dim + i0);
      u16x4 b = load4(head * head_dim + i0 + half);
      // the deferred norm's row scale rides on the rotation coefficients
      const f32x4 c = *reinterpret_cast<const f32x4*>(cs + i0) * rsc;
      const f32x4 s = *reinterpret_cast<const f32x4*>(cs + half + i0) * rsc;
      float x1[4] = {bf16lo(a.w[0]), bf16hi(a.w[0]), bf16lo(a.w[1]), bf16hi(a.w[1])};
      float x2[4] = {bf16lo(b.w[0]), bf16hi(b.w[0]), bf16lo(b.w[1]), bf16hi(b.w[1])};
      float o1[4], o2[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o1[k] = x1[k] * c[k] - x2[k] * s[k];
        o2[k] = x2[k] * c[k] + x1[k] * s[k];
      }
      u16x4 ra, rb;
      ra.w[0] = pack_bf16x2(o1[0], o1[1]);
      ra.w[1] = pack_bf16x2(o1[2], o1[3]);
      rb.w[0] = pack_bf16x2(o2[0], o2[1]);
      rb.w[1] = pack_bf16x2(o2[2], o2[3]);
      *reinterpret_cast<u16x4*>(hp + i0) = ra;
      *reinterpret_cast<u16x4*>(hp + i0 + half) = rb;
      if (is_k && slot >= 0) {
        const int kh = head - n_q_heads;
        CT* dst = k_cache + (((blk * n_kv_heads + kh) * block_size) + off) * (int64_t)head_dim;
        if constexpr (F8) {  // the bf16-rounded values, as the bf16 cache would hold them
          *reinterpret_cast<uint32_t*>(dst + i0) = fp8x4(bf16lo(ra.w[0]), bf16hi(ra.w[0]), bf16lo(ra.w[1]),
                                                         bf16hi(ra.w[1]), k_inv);
          *reinterpret_cast<uint32_t*>(dst + i0 + half) = fp8x4(bf16lo(rb.w[0]), bf16hi(rb.w[0]), bf16lo(rb.w[1]),
                                                                bf16hi(rb.w[1]), k_inv);
        } else {
          *reinterpret_cast<u16x4*>(dst + i0) = ra;
          *reinterpret_cast<u16x4*>(dst + i0 + half) = rb;
        }
      }
    } else {
      const int j = it - n_rot_items;
      const int vh = j / items_per_head_v;
      const int d0 = (j % items_per_head_v) * 8;
      const int col = (n_q_heads + n_kv_heads + vh) * head_dim + d0;
      u16x8 v;
      if constexpr (S == 0) {
        if (slot < 0) continue;
        v = *reinterpret_cast<const u16x8*>(row + col);
        if (scaled)
#pragma unroll
          for (int k = 0; k < 4; ++k) v.w[k] = pack_bf16x2(bf16lo(v.w[k]) * rsc, bf16hi(v.w[k]) * rsc);
      } else {
        float f[8];
        slab_sum<S>(srow + col, slab_stride, f, 8);
#pragma unroll
        for (int k = 0; k < 4; ++k) v.w[k] = pack_bf16x2(f[2 * k], f[2 * k + 1]);
        *reinterpret_cast<u16x8*>(row + col) = v;
        if (slot < 0) continue;
      }
      CT* dst = v_cache + (((blk * n_kv_heads + vh) * block_size) + off) * (int64_t)head_dim + d0;
      if constexpr (F8) {
        uint2 o;
        o.x = fp8x4(bf16lo(v.w[0]), bf16hi(v.w[0]), bf16lo(v.w[1]), bf16hi(v.w[1]), v_inv);
        o.y = fp8x4(bf16lo(v.w[2]), bf16hi(v.w[2]), bf16lo(v.w[3]), bf16hi(v.w[3]), v_inv);
        *reinterpret_cast<uint2*>(dst) = o;
      } else {
        *reinterpret_cast<u16x8*>(dst) = v;
      }
    }
  }
}

// FP8 cache -> bf16 scratch for the prefill attention kernel: grid (blocks per
// sequence, sequences, 2 = K / V); scratch block i * max_blocks + j holds block
// j of sequence i (its block table row remapped to a dense arange), blocks past
// the sequence's context are skipped.
__global__ void __launch_bounds__(kThreads)
    kv_dequant_kernel(const uint8_t* __restrict__ k8, const uint8_t* __restrict__ v8, bf16_t* __restrict__ ks,
                      bf16_t* __restrict__ vs, const int* __restrict__ block_tables, int bt_stride,
                      const int* __restrict__ ctx_lens, const int* __restrict__ dst_table, int max_blocks,
                      int64_t block_elems, int block_size, float k_scale, float v_scale) {
  const int j = blockIdx.x, i = blockIdx.y, which = blockIdx.z;
  if ((int64_t)j * block_size >= ctx_lens[i]) return;
  const int64_t src_blk = block_tables[(int64_t)i * bt_stride + j];
  const uint8_t* src = (which ? v8 : k8) + src_blk * block_elems;
  // packed scratch: sequence i's block j lands in scratch block dst_table[i][j]
  bf16_t* dst = (which ? vs : ks) + (int64_t)dst_table[(int64_t)i * max_blocks + j] * block_elems;
  const float sc = which ? v_scale : k_scale;
  for (int64_t e = (int64_t)threadIdx.x * 8; e < block_elems; e += kThreads * 8) {
    const uint2 w = *reinterpret_cast<const uint2*>(src + e);
    u16x8 o;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t x = h ? w.y : w.x;
      const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)x, false);
      const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)x, true);
      o.w[2 * h] = pack_bf16x2(lo[0] * sc, lo[1] * sc);
      o.w[2 * h + 1] = pack_bf16x2(hi[0] * sc, hi[1] * sc);
    }
    *reinterpret_cast<u16x8*>(dst + e) = o;
  }
}

// Plain KV write (no rotation) for already-rotated K (used by the KV receive
// path tests and by models without rotary embeddings).
__global__ void __launch_bounds__(kThreads)
    kv_write_kernel(const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, int64_t kv_stride,
                    const int64_t* __restrict__ slot_mapping, bf16_t* __restrict__ k_cache,
                    bf16_t* __restrict__ v_cache, int n_kv_heads, int head_dim, int block_size) {
  const int64_t t = blockIdx.x;
  const int64_t slot = slot_mapping[t];
  if (slot < 0) return;
  const int64_t blk = slot / block_size;
  const int off = (int)(slot % block_size);
  const int per_head = head_dim >> 3;
  for (int it = threadIdx.x; it < 2 * n_kv_heads * per_head; it += kThreads) {
    const int which = it / (n_kv_heads * per_head);
    const int j = it % (n_kv_heads * per_head);
    const int h = j / per_head, d0 = (j % per_head) * 8;
    const bf16_t* src = (which ? v : k) + t * kv_stride + (int64_t)h * head_dim + d0;
    bf16_t* dst = (which ? v_cache : k_cache) + (((blk * n_kv_heads + h) * block_size) + off) * (int64_t)head_dim + d0;
    *reinterpret_cast<u16x8*>(dst) = *reinterpret_cast<const u16x8*>(src);
  }
}

}  // namespace

// slabs / splits / slab_bm: the QKV output as split-K partials (splits 2, 4 or 8;
// slice s, token t at slabs + (s * slab_bm + t) * row_len) written whole into qkv;
// splits 0: qkv holds the projection output already
extern "C" int dx_rope_cache(void* qkv, int64_t qkv_stride, const void* positions, int pos_is_i64,
                             const float* cos_sin, const int64_t* slot_mapping, void* k_cache, void* v_cache,
                             int tokens, int n_q_heads, int n_kv_heads, int head_dim, int block_size, int rotate_q,
                             int kv_fp8, float k_scale, float v_scale, const float* slabs, int splits, int slab_bm,
                             hipStream_t stream, const float* row_scale) {
  if (head_dim % 8 || (head_dim / 2) % 4 || (kv_fp8 && (k_scale <= 0.f || v_scale <= 0.f))) return -1;
  if (splits && (!(splits == 2 || splits == 4 || splits == 8) || tokens > slab_bm || slabs == nullptr)) return -2;
  if (splits && row_scale != nullptr) return -3;  // a deferred norm only on a finished projection row
  const int64_t sst = (int64_t)slab_bm * (n_q_heads + 2 * n_kv_heads) * head_dim;
  if (tokens == 0) return 0;
  const float ki = kv_fp8 ? 1.f / k_scale : 1.f, vi = kv_fp8 ? 1.f / v_scale : 1.f;
#define DX_RCS(PT, F8, S_)                                                                                   \
  rope_cache_kernel<PT, F8, S_><<<tokens, kThreads, 0, stream>>>(                                             \
      (bf16_t*)qkv, qkv_stride, (const PT*)positions, cos_sin, slot_mapping, k_cache, v_cache, n_q_heads,      \
      n_kv_heads, head_dim, block_size, rotate_q, ki, vi, slabs, sst, row_scale)
#define DX_RC(PT, F8)                                \
  switch (splits) {                                  \
    case 2: DX_RCS(PT, F8, 2); break;                \
    case 4: DX_RCS(PT, F8, 4); break;                \
    case 8: DX_RCS(PT, F8, 8); break;                \
    default: DX_RCS(PT, F8, 0); break;               \
  }
  if (pos_is_i64) {
    if (kv_fp8) { DX_RC(int64_t, true) }
    else { DX_RC(int64_t, false) }
  } else {
    if (kv_fp8) { DX_RC(int32_t, true) }
    else { DX_RC(int32_t, false) }
  }
#undef DX_RCS
#undef DX_RC
  return (int)hipGetLastError();
}

// dst_table [n_seqs][max_blocks] int32: scratch block of (sequence, block) --
// the caller packs the sequences' live blocks (sum of ceil(ctx / block_size)
// scratch blocks, not n_seqs x max_blocks)
extern "C" int dx_kv_dequant(const void* k8, const void* v8, void* k_scratch, void* v_scratch, const int* block_tables,
                             int bt_stride, const int* ctx_lens, const int* dst_table, int n_seqs, int max_blocks,
                             int n_kv_heads, int block_size, int head_dim, float k_scale, float v_scale,
                             hipStream_t stream) {
  const int64_t be = (int64_t)n_kv_heads * block_size * head_dim;
  if (be % 8) return -1;
  if (n_seqs == 0 || max_blocks == 0) return 0;
  kv_dequant_kernel<<<dim3(max_blocks, n_seqs, 2), kThreads, 0, stream>>>(
      (const uint8_t*)k8, (const uint8_t*)v8, (bf16_t*)k_scratch, (bf16_t*)v_scratch, block_tables, bt_stride,
      ctx_lens, dst_table, max_blocks, be, block_size, k_scale, v_scale);
  return (int)hipGetLastError();
}

extern "C" int dx_kv_write(const void* k, const void* v, int64_t kv_stride, const int64_t* slot_mapping,
                           void* k_cache, void* v_cache, int tokens, int n_kv_heads, int head_dim, int block_size,
                           hipStream_t stream) {
  if (head_dim % 8) return -1;
  if (tokens == 0) return 0;
  kv_write_kernel<<<tokens, kThreads, 0, stream>>>((const bf16_t*)k, (const bf16_t*)v, kv_stride, slot_mapping,
                                                    (bf16_t*)k_cache, (bf16_t*)v_cache, n_kv_heads, head_dim,
                                                    block_size);
  return (int)hipGetLastError();
}
