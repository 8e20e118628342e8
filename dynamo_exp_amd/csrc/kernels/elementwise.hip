// Memory-bound elementwise kernels for gfx950: SiLU-gated MLP activation and
// token-embedding gather.  All accesses are 16-byte vectors (guide G13).
#include "common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// gate_up: [T, 2F] with gate = [:, :F], up = [:, F:] (blk = 0), or gate and up
// interleaved in blocks of blk columns (g[0:blk], u[0:blk], g[blk:2blk], ...;
// the weight layout of the fused SwiGLU GEMM, gemm256.hip)  ->  out: [T, F]
__global__ void __launch_bounds__(kThreads) silu_and_mul_kernel(bf16_t* __restrict__ out,
                                                                const bf16_t* __restrict__ gate_up, int ffn,
                                                                int64_t in_stride, int64_t out_stride, int blk) {
  const int64_t t = blockIdx.y;
  const int nvec = ffn >> 3;
  const u16x8* row = reinterpret_cast<const u16x8*>(gate_up + t * in_stride);
  u16x8* o = reinterpret_cast<u16x8*>(out + t * out_stride);
  const int bv = blk >> 3;  // vectors per block
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < nvec; i += gridDim.x * kThreads) {
    const int gi = bv ? (i / bv) * 2 * bv + i % bv : i;
    const int ui = bv ? gi + bv : i + nvec;
    u16x8 a = row[gi], b = row[ui], r;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      r.w[k] = pack_bf16x2(silu(bf16lo(a.w[k])) * bf16lo(b.w[k]), silu(bf16hi(a.w[k])) * bf16hi(b.w[k]));
    o[i] = r;
  }
}

// out[t, :] = table[ids[t], :]  (ids outside [0, vocab) produce zeros)
template <typename IdT>
__global__ void __launch_bounds__(kThreads) embedding_kernel(bf16_t* __restrict__ out,
                                                             const bf16_t* __restrict__ table,
                                                             const IdT* __restrict__ ids, int hidden, int64_t vocab) {
  const int64_t t = blockIdx.x;
  const int64_t id = (int64_t)ids[t];
  const int nvec = hidden >> 3;
  u16x8* o = reinterpret_cast<u16x8*>(out + t * (int64_t)hidden);
  if (id < 0 || id >= vocab) {
    u16x8 z = {{0, 0, 0, 0}};
    for (int i = threadIdx.x; i < nvec; i += kThreads) o[i] = z;
    return;
  }
  const u16x8* src = reinterpret_cast<const u16x8*>(table + id * (int64_t)hidden);
  for (int i = threadIdx.x; i < nvec; i += kThreads) o[i] = src[i];
}

// Multi-step decode (engine/model_runner.py execute_decode_multi): after a
// captured decode step, feed its sampled tokens back as the next step's inputs
// entirely on the device -- record (token, logprob) of step `step`, then
// ids <- token, pos += 1, ctx += 1, sampling offset += 1 and the new KV slot
// from the block table -- so K decode steps run with one host round trip.
// Rows >= n_real are the graph bucket's padding and stay untouched.
__global__ void __launch_bounds__(kThreads) decode_advance_kernel(
    int64_t* __restrict__ ids, int64_t* __restrict__ pos, int64_t* __restrict__ slots, int* __restrict__ ctx,
    int64_t* __restrict__ offs, const int64_t* __restrict__ out_tok, const float* __restrict__ out_lp,
    int64_t* __restrict__ res_tok, float* __restrict__ res_lp, const int* __restrict__ bt, int bt_stride,
    int block_size, int n_real, int step, int advance) {
  const int b = blockIdx.x * kThreads + threadIdx.x;
  if (b >= n_real) return;
  const int64_t t = out_tok[b];
  res_tok[(int64_t)step * n_real + b] = t;
  res_lp[(int64_t)step * n_real + b] = out_lp[b];
  if (!advance) return;
  const int64_t p = pos[b] + 1;
  ids[b] = t;
  pos[b] = p;
  ctx[b] += 1;
  offs[b] += 1;
  slots[b] = (int64_t)bt[(int64_t)b * bt_stride + p / block_size] * block_size + p % block_size;
}

}  // namespace

extern "C" int dx_decode_advance(void* ids, void* pos, void* slots, void* ctx, void* offs, const void* out_tok,
                                 const void* out_lp, void* res_tok, void* res_lp, const int* bt, int bt_stride,
                                 int block_size, int n_real, int step, int advance, hipStream_t stream) {
  if (n_real <= 0) return 0;
  decode_advance_kernel<<<(n_real + kThreads - 1) / kThreads, kThreads, 0, stream>>>(
      (int64_t*)ids, (int64_t*)pos, (int64_t*)slots, (int*)ctx, (int64_t*)offs, (const int64_t*)out_tok,
      (const float*)out_lp, (int64_t*)res_tok, (float*)res_lp, bt, bt_stride, block_size, n_real, step, advance);
  return (int)hipGetLastError();
}

extern "C" int dx_silu_and_mul(void* out, const void* gate_up, int tokens, int ffn, int64_t in_stride,
                               int64_t out_stride, int blk, hipStream_t stream) {
  if (ffn % 8 || blk % 8 || (blk && ffn % blk)) return -1;
  if (tokens == 0) return 0;
  const int nvec = ffn / 8;
  int gx = (nvec + kThreads - 1) / kThreads;
  if (gx > 64) gx = 64;
  dim3 grid(gx, tokens);
  silu_and_mul_kernel<<<grid, kThreads, 0, stream>>>((bf16_t*)out, (const bf16_t*)gate_up, ffn, in_stride,
                                                     out_stride, blk);
  return (int)hipGetLastError();
}

extern "C" int dx_embedding(void* out, const void* table, const void* ids, int ids_i64, int tokens, int hidden,
                            int64_t vocab, hipStream_t stream) {
  if (hidden % 8) return -1;
  if (tokens == 0) return 0;
  if (ids_i64)
    embedding_kernel<int64_t><<<tokens, kThreads, 0, stream>>>((bf16_t*)out, (const bf16_t*)table,
                                                               (const int64_t*)ids, hidden, vocab);
  else
    embedding_kernel<int32_t><<<tokens, kThreads, 0, stream>>>((bf16_t*)out, (const bf16_t*)table,
                                                               (const int32_t*)ids, hidden, vocab);
  return (int)hipGetLastError();
}
