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
#include "common.h"

namespace {

constexpr int kThreads = 256;

struct __attribute__((aligned(8))) u16x4 {
  uint32_t w[2];
};

template <typename PosT>
__global__ void __launch_bounds__(kThreads)
    rope_cache_kernel(bf16_t* __restrict__ qkv, int64_t qkv_stride, const PosT* __restrict__ positions,
                      const float* __restrict__ cos_sin, const int64_t* __restrict__ slot_mapping,
                      bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache, int n_q_heads, int n_kv_heads,
                      int head_dim, int block_size, int rotate_q) {
  const int64_t t = blockIdx.x;
  const int64_t pos = (int64_t)positions[t];
  const int half = head_dim >> 1;
  const int items_per_head_rot = half >> 2;  // 4 pairs per item
  const int items_per_head_v = head_dim >> 3;
  const int n_rot_items = (n_q_heads + n_kv_heads) * items_per_head_rot;
  const int n_items = n_rot_items + n_kv_heads * items_per_head_v;
  bf16_t* row = qkv + t * qkv_stride;
  const float* cs = cos_sin + pos * head_dim;
  const int64_t slot = slot_mapping ? slot_mapping[t] : -1;
  const int64_t blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? (int)(slot % block_size) : 0;

  for (int it = threadIdx.x; it < n_items; it += kThreads) {
    if (it < n_rot_items) {
      const int head = it / items_per_head_rot;  // 0..Hq-1 are q heads, then k heads
      const int i0 = (it % items_per_head_rot) * 4;
      const bool is_k = head >= n_q_heads;
      if (!is_k && !rotate_q) continue;
      bf16_t* hp = row + (int64_t)head * head_dim;
      u16x4 a = *reinterpret_cast<const u16x4*>(hp + i0);
      u16x4 b = *reinterpret_cast<const u16x4*>(hp + i0 + half);
      const f32x4 c = *reinterpret_cast<const f32x4*>(cs + i0);
      const f32x4 s = *reinterpret_cast<const f32x4*>(cs + half + i0);
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
        bf16_t* dst = k_cache + (((blk * n_kv_heads + kh) * block_size) + off) * (int64_t)head_dim;
        *reinterpret_cast<u16x4*>(dst + i0) = ra;
        *reinterpret_cast<u16x4*>(dst + i0 + half) = rb;
      }
    } else {
      if (slot < 0) continue;
      const int j = it - n_rot_items;
      const int vh = j / items_per_head_v;
      const int d0 = (j % items_per_head_v) * 8;
      const bf16_t* src = row + (int64_t)(n_q_heads + n_kv_heads + vh) * head_dim + d0;
      bf16_t* dst = v_cache + (((blk * n_kv_heads + vh) * block_size) + off) * (int64_t)head_dim + d0;
      *reinterpret_cast<u16x8*>(dst) = *reinterpret_cast<const u16x8*>(src);
    }
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

extern "C" int dx_rope_cache(void* qkv, int64_t qkv_stride, const void* positions, int pos_is_i64,
                             const float* cos_sin, const int64_t* slot_mapping, void* k_cache, void* v_cache,
                             int tokens, int n_q_heads, int n_kv_heads, int head_dim, int block_size, int rotate_q,
                             hipStream_t stream) {
  if (head_dim % 8 || (head_dim / 2) % 4) return -1;
  if (tokens == 0) return 0;
  if (pos_is_i64)
    rope_cache_kernel<int64_t><<<tokens, kThreads, 0, stream>>>(
        (bf16_t*)qkv, qkv_stride, (const int64_t*)positions, cos_sin, slot_mapping, (bf16_t*)k_cache,
        (bf16_t*)v_cache, n_q_heads, n_kv_heads, head_dim, block_size, rotate_q);
  else
    rope_cache_kernel<int32_t><<<tokens, kThreads, 0, stream>>>(
        (bf16_t*)qkv, qkv_stride, (const int32_t*)positions, cos_sin, slot_mapping, (bf16_t*)k_cache,
        (bf16_t*)v_cache, n_q_heads, n_kv_heads, head_dim, block_size, rotate_q);
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
