// Token sampling for gfx950: greedy, temperature, top-k, top-p (nucleus),
// min-p, seeded per request; plus repetition / frequency / presence
// penalties.  One 1024-lane workgroup per row (16 waves, the most a CU can
// give one row); the row (<= 512 KiB) is streamed from L2 once per pass.
//
// * top-k / top-p thresholds: 4-pass radix select (8 bits/pass) on the
//   order-preserving uint32 key of the logit; top-p walks a histogram of
//   probability MASS instead of counts.  Per-wave private LDS histograms keep
//   LDS atomics uncontended (guide G12).
// * sampling: exponential race / Gumbel-max, argmax over survivors of
//   (x - max)/T - log(-log u), u from a counter-based hash of
//   (seed, offset, token) -- exact sampling from the renormalised truncated
//   distribution, no sort, no prefix sum, reproducible per seed.
// * logprob of the chosen token under the unmodified (T=1) distribution.
#include "common.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ uint32_t fkey(float x) {
  uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// uniform in (0, 1)
__device__ __forceinline__ float uniform(uint64_t seed, uint64_t offset, uint32_t i) {
  const uint64_t h = mix64(seed ^ mix64(offset * 0xD1B54A32D192ED03ull + i));
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) {
  return p[i];
}
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, int64_t i) {
  return bf16_to_f32(p[i]);
}

struct ArgMax {
  float v;
  int i;
};
__device__ __forceinline__ ArgMax amax(ArgMax a, ArgMax b) {
  return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}
__device__ __forceinline__ ArgMax wave_argmax(ArgMax a) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = amax(a, b);
  }
  return a;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) sample_kernel(
    int64_t* __restrict__ out_tokens, float* __restrict__ out_logprobs, const T* __restrict__ logits,
    int64_t row_stride, int vocab, const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const float* __restrict__ min_p, const int64_t* __restrict__ seeds,
    const int64_t* __restrict__ offsets) {
  __shared__ float hist[kWaves][256];
  __shared__ float red_f[kWaves];
  __shared__ int red_i[kWaves];
  __shared__ float bcast[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const T* x = logits + (int64_t)row * row_stride;
  const float temp = temperature ? temperature[row] : 0.f;
  const int k = top_k ? top_k[row] : 0;
  const float p = top_p ? top_p[row] : 1.f;
  const float mp = min_p ? min_p[row] : 0.f;

  // ---- pass A: max, argmax, online sum exp(x - max) ----
  ArgMax best{-INFINITY, 0x7fffffff};
  float lm = -INFINITY, ls = 0.f;
  for (int i = tid; i < vocab; i += kThreads) {
    const float v = ld(x, i);
    if (v > best.v) best = ArgMax{v, i};
    if (v > lm) {
      ls = ls * __expf(lm - v) + 1.f;
      lm = v;
    } else {
      ls += __expf(v - lm);
    }
  }
  best = wave_argmax(best);
  // combine (lm, ls) across the wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(lm, o, 64), os = __shfl_xor(ls, o, 64);
    const float nm = fmaxf(lm, om);
    ls = (lm == -INFINITY ? 0.f : ls * __expf(lm - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    lm = nm;
  }
  if (lane == 0) {
    red_f[wid] = best.v;
    red_i[wid] = best.i;
    hist[wid][0] = lm;
    hist[wid][1] = ls;
  }
  __syncthreads();
  if (tid == 0) {
    ArgMax b{red_f[0], red_i[0]};
    float M = hist[0][0];
    for (int w = 1; w < kWaves; ++w) {
      b = amax(b, ArgMax{red_f[w], red_i[w]});
      M = fmaxf(M, hist[w][0]);
    }
    float S = 0.f;
    for (int w = 0; w < kWaves; ++w)
      if (hist[w][0] != -INFINITY) S += hist[w][1] * __expf(hist[w][0] - M);
    bcast[0] = M;
    bcast[1] = __logf(S);
    red_i[0] = b.i;
  }
  __syncthreads();
  const float xmax = bcast[0];
  const float logz = bcast[1];
  int chosen = red_i[0];
  __syncthreads();

  if (temp > 0.f) {
    const float inv_t = 1.f / temp;
    uint32_t thr = 0;  // keep tokens with fkey(x) >= thr
    if (mp > 0.f) thr = fkey(xmax + temp * __logf(mp));
    // ---- top-k: radix select the k-th largest key ----
    if (k > 0 && k < vocab) {
      uint32_t prefix = 0, mask = 0;
      int remaining = k;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = lane; i < 256; i += 64) hist[wid][i] = 0.f;
        __syncthreads();
        for (int i = tid; i < vocab; i += kThreads) {
          const uint32_t kk = fkey(ld(x, i));
          if ((kk & mask) == prefix) atomicAdd(&hist[wid][(kk >> shift) & 0xff], 1.f);
        }
        __syncthreads();
        if (tid < 256) {
          float c = 0.f;
          for (int w = 0; w < kWaves; ++w) c += hist[w][tid];
          hist[0][tid] = c;  // safe: each bin owned by one thread, read-before-write per bin
        }
        __syncthreads();
        if (tid == 0) {
          int cum = 0, sel = 0;
          for (int b = 255; b >= 0; --b) {
            const int c = (int)hist[0][b];
            if (cum + c >= remaining) {
              sel = b;
              break;
            }
            cum += c;
          }
          red_i[1] = sel;
          red_i[2] = remaining - cum;
        }
        __syncthreads();
        prefix |= (uint32_t)red_i[1] << shift;
        mask |= 0xffu << shift;
        remaining = red_i[2];
        __syncthreads();
      }
      thr = max(thr, prefix);
    }
    // ---- top-p over the survivors: radix select on probability mass ----
    if (p < 1.f) {
      float zs = 0.f;
      for (int i = tid; i < vocab; i += kThreads) {
        const float v = ld(x, i);
        if (fkey(v) >= thr) zs += __expf((v - xmax) * inv_t);
      }
      zs = block_reduce_sum(zs, red_f);
      float remaining = p * zs;
      uint32_t prefix = 0, mask = 0;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = lane; i < 256; i += 64) hist[wid][i] = 0.f;
        __syncthreads();
        for (int i = tid; i < vocab; i += kThreads) {
          const float v = ld(x, i);
          const uint32_t kk = fkey(v);
          if (kk >= thr && (kk & mask) == prefix) atomicAdd(&hist[wid][(kk >> shift) & 0xff], __expf((v - xmax) * inv_t));
        }
        __syncthreads();
        if (tid < 256) {
          float c = 0.f;
          for (int w = 0; w < kWaves; ++w) c += hist[w][tid];
          hist[0][tid] = c;
        }
        __syncthreads();
        if (tid == 0) {
          float cum = 0.f;
          int sel = -1, last_nz = 0;
          for (int b = 255; b >= 0; --b) {
            const float c = hist[0][b];
            if (c > 0.f) last_nz = b;
            if (c > 0.f && cum + c >= remaining) {
              sel = b;
              break;
            }
            cum += c;
          }
          if (sel < 0) {  // rounding: take the smallest non-empty bin
            sel = last_nz;
            cum -= hist[0][sel];
          }
          red_i[1] = sel;
          bcast[2] = remaining - cum;
        }
        __syncthreads();
        prefix |= (uint32_t)red_i[1] << shift;
        mask |= 0xffu << shift;
        remaining = bcast[2];
        __syncthreads();
      }
      thr = max(thr, prefix);
    }
    // ---- exponential race over survivors ----
    const uint64_t seed = seeds ? (uint64_t)seeds[row] : 0ull;
    const uint64_t off = offsets ? (uint64_t)offsets[row] : 0ull;
    ArgMax g{-INFINITY, 0x7fffffff};
    for (int i = tid; i < vocab; i += kThreads) {
      const float v = ld(x, i);
      if (fkey(v) < thr) continue;
      const float u = uniform(seed, off, (uint32_t)i);
      const float score = (v - xmax) * inv_t - __logf(-__logf(u));
      if (score > g.v) g = ArgMax{score, i};
    }
    g = wave_argmax(g);
    if (lane == 0) {
      red_f[wid] = g.v;
      red_i[wid] = g.i;
    }
    __syncthreads();
    if (tid == 0) {
      ArgMax b{red_f[0], red_i[0]};
      for (int w = 1; w < kWaves; ++w) b = amax(b, ArgMax{red_f[w], red_i[w]});
      red_i[0] = (b.i == 0x7fffffff) ? chosen : b.i;
    }
    __syncthreads();
    chosen = red_i[0];
  }
  if (tid == 0) {
    out_tokens[row] = chosen;
    if (out_logprobs) out_logprobs[row] = ld(x, chosen) - xmax - logz;
  }
}

// Vocab-parallel (tensor-parallel LM head) sampling, per-rank half: over this
// rank's logits shard (global token ids v0 .. v0+vocab-1) each row produces
//   out[row] = {m, sum exp(x - m), best score, global id of best, x[best]}
// where m is the shard max and "best" is the shard winner of the same
// exponential race as sample_kernel (score x/T - log(-log u(seed, off, id)),
// u keyed by the GLOBAL token id) or the shard argmax for greedy rows (T <= 0).
// Gathering these 5 floats per row from every rank and taking the rank with
// the largest score (ties: lower id) samples exactly from the full softmax at
// temperature T -- the race is shift invariant, so no global max is needed
// before it -- and the logprob is x[best] - M - log(sum_r s_r e^{m_r - M}).
// Rows with top-k / top-p / min-p need global thresholds and use the full
// logits gather instead (models/llama.py sample_sharded).
template <typename T>
__global__ void __launch_bounds__(kThreads) sample_partial_kernel(
    float* __restrict__ out, const T* __restrict__ logits, int64_t row_stride, int vocab, int v0,
    const float* __restrict__ temperature, const int64_t* __restrict__ seeds, const int64_t* __restrict__ offsets) {
  __shared__ float red_m[kWaves], red_s[kWaves], red_b[kWaves];
  __shared__ int red_i[kWaves];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const T* x = logits + (int64_t)row * row_stride;
  const float temp = temperature ? temperature[row] : 0.f;
  const bool race = temp > 0.f;
  const float inv_t = race ? 1.f / temp : 1.f;
  const uint64_t seed = seeds ? (uint64_t)seeds[row] : 0ull;
  const uint64_t off = offsets ? (uint64_t)offsets[row] : 0ull;
  ArgMax best{-INFINITY, 0x7fffffff};
  float lm = -INFINITY, ls = 0.f;
  for (int i = tid; i < vocab; i += kThreads) {
    const float v = ld(x, i);
    if (v > lm) {
      ls = ls * __expf(lm - v) + 1.f;
      lm = v;
    } else {
      ls += __expf(v - lm);
    }
    const float score = race ? v * inv_t - __logf(-__logf(uniform(seed, off, (uint32_t)(v0 + i)))) : v;
    if (score > best.v) best = ArgMax{score, i};
  }
  best = wave_argmax(best);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(lm, o, 64), os = __shfl_xor(ls, o, 64);
    const float nm = fmaxf(lm, om);
    ls = (lm == -INFINITY ? 0.f : ls * __expf(lm - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    lm = nm;
  }
  if (lane == 0) {
    red_m[wid] = lm;
    red_s[wid] = ls;
    red_b[wid] = best.v;
    red_i[wid] = best.i;
  }
  __syncthreads();
  if (tid == 0) {
    ArgMax b{red_b[0], red_i[0]};
    float M = red_m[0];
    for (int w = 1; w < kWaves; ++w) {
      b = amax(b, ArgMax{red_b[w], red_i[w]});
      M = fmaxf(M, red_m[w]);
    }
    float S = 0.f;
    for (int w = 0; w < kWaves; ++w)
      if (red_m[w] != -INFINITY) S += red_s[w] * __expf(red_m[w] - M);
    const int bi = b.i == 0x7fffffff ? 0 : b.i;
    float* o = out + (int64_t)row * 5;
    o[0] = M;
    o[1] = S;
    o[2] = b.v;
    o[3] = (float)(v0 + bi);  // exact: vocab ids < 2^24
    o[4] = ld(x, bi);
  }
}

// Penalties, one workgroup per row; unique (token, count) pairs per row in CSR
// form; `flags` bit0 = token occurs in the output, bit1 = occurs in the prompt.
template <typename T>
__global__ void __launch_bounds__(256)
    penalty_kernel(T* __restrict__ logits, int64_t row_stride, const int* __restrict__ csr,
                   const int* __restrict__ toks, const int* __restrict__ counts, const int* __restrict__ flags,
                   const float* __restrict__ rep, const float* __restrict__ freq, const float* __restrict__ pres) {
  const int row = blockIdx.x;
  T* x = logits + (int64_t)row * row_stride;
  const float rp = rep[row], fp = freq[row], pp = pres[row];
  for (int e = csr[row] + threadIdx.x; e < csr[row + 1]; e += 256) {
    const int t = toks[e];
    float v = ld(x, t);
    if (rp != 1.f) v = v > 0.f ? v / rp : v * rp;
    if (flags[e] & 1) v -= fp * (float)counts[e] + pp;
    if constexpr (sizeof(T) == 4)
      x[t] = v;
    else
      x[t] = f32_to_bf16(v);
  }
}

}  // namespace

extern "C" int dx_sample(int64_t* out_tokens, float* out_logprobs, const void* logits, int logits_f32,
                         int64_t row_stride, int rows, int vocab, const float* temperature, const int* top_k,
                         const float* top_p, const float* min_p, const int64_t* seeds, const int64_t* offsets,
                         hipStream_t stream) {
  if (rows == 0) return 0;
  if (logits_f32)
    sample_kernel<float><<<rows, kThreads, 0, stream>>>(out_tokens, out_logprobs, (const float*)logits, row_stride,
                                                         vocab, temperature, top_k, top_p, min_p, seeds, offsets);
  else
    sample_kernel<bf16_t><<<rows, kThreads, 0, stream>>>(out_tokens, out_logprobs, (const bf16_t*)logits,
                                                          row_stride, vocab, temperature, top_k, top_p, min_p,
                                                          seeds, offsets);
  return (int)hipGetLastError();
}

extern "C" int dx_sample_partial(float* out, const void* logits, int logits_f32, int64_t row_stride, int rows,
                                 int vocab, int v0, const float* temperature, const int64_t* seeds,
                                 const int64_t* offsets, hipStream_t stream) {
  if (rows == 0) return 0;
  if (v0 + vocab > (1 << 24)) return -1;  // ids travel as exact floats
  if (logits_f32)
    sample_partial_kernel<float><<<rows, kThreads, 0, stream>>>(out, (const float*)logits, row_stride, vocab, v0,
                                                                 temperature, seeds, offsets);
  else
    sample_partial_kernel<bf16_t><<<rows, kThreads, 0, stream>>>(out, (const bf16_t*)logits, row_stride, vocab, v0,
                                                                  temperature, seeds, offsets);
  return (int)hipGetLastError();
}

extern "C" int dx_apply_penalties(void* logits, int logits_f32, int64_t row_stride, int rows, const int* csr,
                                  const int* toks, const int* counts, const int* flags, const float* rep,
                                  const float* freq, const float* pres, hipStream_t stream) {
  if (rows == 0) return 0;
  if (logits_f32)
    penalty_kernel<float><<<rows, 256, 0, stream>>>((float*)logits, row_stride, csr, toks, counts, flags, rep, freq,
                                                     pres);
  else
    penalty_kernel<bf16_t><<<rows, 256, 0, stream>>>((bf16_t*)logits, row_stride, csr, toks, counts, flags, rep,
                                                      freq, pres);
  return (int)hipGetLastError();
}
