// KV block gather/scatter for gfx950 -- the block-copy engine behind the
// prefill->decode transfer (pack into / unpack from a contiguous RCCL staging
// buffer), the pinned-host offload tier (src or dst may be host-mapped pinned
// memory: the kernel then streams over PCIe/xGMI with no extra staging) and
// tensor-parallel relayout.
//
// Memory is viewed as [prefix][block][inner] with byte strides; for each
// (prefix p, pair i) it copies `copy_bytes` from
//   src + p*src_prefix_stride + src_ids[i]*src_block_bytes + src_inner_off
// to
//   dst + p*dst_prefix_stride + dst_ids[i]*dst_block_bytes + dst_inner_off.
// With the engine's per-layer cache layout [NB][Hkv][BS][D] a TP re-split of
// the KV heads (decode TP = d x prefill TP) is a contiguous sub-range of each
// block (inner offset r * Hkv/d * BS * D * 2), so relayout needs no permute
// pass -- the reason for that layout.  (Reference semantics: block_copy.cu
// copy_blocks_kernel / permute_scatter_memcpy, kv_rearrange.py.)
//
// 16-byte vector loads/stores, 4 in flight per lane; one launch for all layers
// and all blocks (no per-block memcpy storm, cf. reference copy_blocks_memcpy_3d).
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 4;

__global__ void __launch_bounds__(kThreads)
    kv_copy_kernel(char* __restrict__ dst, const char* __restrict__ src, const int* __restrict__ src_ids,
                   const int* __restrict__ dst_ids, int64_t src_prefix_stride, int64_t dst_prefix_stride,
                   int64_t src_block_bytes, int64_t dst_block_bytes, int64_t src_inner_off, int64_t dst_inner_off,
                   int64_t copy_bytes) {
  const int pair = blockIdx.y;
  const int64_t p = blockIdx.z;
  const char* s = src + p * src_prefix_stride + (int64_t)src_ids[pair] * src_block_bytes + src_inner_off;
  char* d = dst + p * dst_prefix_stride + (int64_t)dst_ids[pair] * dst_block_bytes + dst_inner_off;
  const int64_t nvec = copy_bytes >> 4;
  const u16x8* sv = reinterpret_cast<const u16x8*>(s);
  u16x8* dv = reinterpret_cast<u16x8*>(d);
  const int64_t step = (int64_t)gridDim.x * kThreads * kUnroll;
  for (int64_t base = (int64_t)blockIdx.x * kThreads * kUnroll + threadIdx.x; base < nvec; base += step) {
    u16x8 r[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t i = base + (int64_t)u * kThreads;
      if (i < nvec) r[u] = sv[i];
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t i = base + (int64_t)u * kThreads;
      if (i < nvec) dv[i] = r[u];
    }
  }
}

}  // namespace

extern "C" int dx_kv_copy_blocks(void* dst, const void* src, const int* src_ids, const int* dst_ids, int n_pairs,
                                 int n_prefix, int64_t src_prefix_stride, int64_t dst_prefix_stride,
                                 int64_t src_block_bytes, int64_t dst_block_bytes, int64_t src_inner_off,
                                 int64_t dst_inner_off, int64_t copy_bytes, hipStream_t stream) {
  if (copy_bytes % 16 || src_inner_off % 16 || dst_inner_off % 16 || src_block_bytes % 16 || dst_block_bytes % 16)
    return -1;
  if (n_pairs == 0 || n_prefix == 0 || copy_bytes == 0) return 0;
  const int64_t nvec = copy_bytes / 16;
  int gx = (int)((nvec + kThreads * kUnroll - 1) / (kThreads * kUnroll));
  // enough workgroups to fill 256 CUs, bounded
  const int64_t others = (int64_t)n_pairs * n_prefix;
  if (others >= 2048) gx = 1;
  else if (gx * others > 4096) gx = (int)((4096 + others - 1) / others);
  if (gx < 1) gx = 1;
  dim3 grid(gx, n_pairs, n_prefix);
  kv_copy_kernel<<<grid, kThreads, 0, stream>>>((char*)dst, (const char*)src, src_ids, dst_ids, src_prefix_stride,
                                                dst_prefix_stride, src_block_bytes, dst_block_bytes, src_inner_off,
                                                dst_inner_off, copy_bytes);
  return (int)hipGetLastError();
}
