// RMSNorm and fused residual-add + RMSNorm for gfx950.
//
// One workgroup (256 lanes = 4 waves) per row; every lane keeps its slice of
// the row in registers as 16-byte bf16x8 vectors, so the row is read from HBM
// exactly once (x and residual) and written once (out, residual).  The
// reduction is wave-shuffle + one LDS exchange.  Memory-bound: the target is
// the HBM roofline (guide App. B "Reduction").
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxVecLimit = 8;  // up to 8 x 8 x 256 = 16384 hidden

template <bool kAdd, int kMaxVec, bool kExact>
__global__ void __launch_bounds__(kThreads) rmsnorm_kernel(bf16_t* out, const bf16_t* x,
                                                           bf16_t* residual, const bf16_t* __restrict__ w,
                                                           int hidden, int64_t x_stride, int64_t out_stride,
                                                           int64_t res_stride, float eps) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int nvec = hidden >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + row * x_stride);
  u16x8* rr = kAdd ? reinterpret_cast<u16x8*>(residual + row * res_stride) : nullptr;
  float v[kMaxVec][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * kThreads;
    if (kExact || vi < nvec) {
      u16x8 a = xr[vi];
      if constexpr (kAdd) {
        u16x8 r = rr[vi];
        u16x8 s;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float lo = bf16lo(a.w[k]) + bf16lo(r.w[k]);
          float hi = bf16hi(a.w[k]) + bf16hi(r.w[k]);
          s.w[k] = pack_bf16x2(lo, hi);
          // normalise the bf16-rounded residual (matches a bf16 residual stream)
          v[i][2 * k] = bf16lo(s.w[k]);
          v[i][2 * k + 1] = bf16hi(s.w[k]);
        }
        rr[vi] = s;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[i][2 * k] = bf16lo(a.w[k]);
          v[i][2 * k + 1] = bf16hi(a.w[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) ss += v[i][k] * v[i][k];
    }
  }
  ss = block_reduce_sum(ss, red);
  const float inv = rsqrtf(ss / (float)hidden + eps);
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  u16x8* orow = reinterpret_cast<u16x8*>(out + row * out_stride);
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * kThreads;
    if (kExact || vi < nvec) {
      u16x8 g = wr[vi];
      u16x8 o;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o.w[k] = pack_bf16x2(v[i][2 * k] * inv * bf16lo(g.w[k]), v[i][2 * k + 1] * inv * bf16hi(g.w[k]));
      orow[vi] = o;
    }
  }
}

// residual += bf16(sum of S split-K slabs of a projection's output) (in slice
// order, rounded to bf16 exactly as the reduction kernel would store it);
// out = rmsnorm(residual) * w.  The o / down projections' partials go straight
// into the norm that consumes them: one launch and one bf16 round trip less.
template <int S, int kMaxVec, bool kExact>
__global__ void __launch_bounds__(kThreads) add_rmsnorm_slabs_kernel(bf16_t* out, const float* __restrict__ slabs,
                                                                     int64_t slab_stride, bf16_t* residual,
                                                                     const bf16_t* __restrict__ w, int hidden,
                                                                     int64_t out_stride, int64_t res_stride,
                                                                     float eps) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int nvec = hidden >> 3;
  const float* xr = slabs + row * hidden;
  u16x8* rr = reinterpret_cast<u16x8*>(residual + row * res_stride);
  float v[kMaxVec][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * kThreads;
    if (kExact || vi < nvec) {
      f32x4 p[S][2];
#pragma unroll
      for (int s = 0; s < S; ++s) {  // every slice's loads in flight before the first add
        const float* q = xr + s * slab_stride + 8 * vi;
        p[s][0] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q));
        p[s][1] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q + 4));
      }
      f32x4 a = p[0][0], b = p[0][1];
#pragma unroll
      for (int s = 1; s < S; ++s) {
        a += p[s][0];
        b += p[s][1];
      }
      const float xs[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
      u16x8 r = rr[vi];
      u16x8 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t xb = pack_bf16x2(xs[2 * k], xs[2 * k + 1]);  // the projection's bf16 output
        o.w[k] = pack_bf16x2(bf16lo(xb) + bf16lo(r.w[k]), bf16hi(xb) + bf16hi(r.w[k]));
        v[i][2 * k] = bf16lo(o.w[k]);
        v[i][2 * k + 1] = bf16hi(o.w[k]);
      }
      rr[vi] = o;
#pragma unroll
      for (int k = 0; k < 8; ++k) ss += v[i][k] * v[i][k];
    }
  }
  ss = block_reduce_sum(ss, red);
  const float inv = rsqrtf(ss / (float)hidden + eps);
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  u16x8* orow = reinterpret_cast<u16x8*>(out + row * out_stride);
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * kThreads;
    if (kExact || vi < nvec) {
      u16x8 g = wr[vi];
      u16x8 o;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o.w[k] = pack_bf16x2(v[i][2 * k] * inv * bf16lo(g.w[k]), v[i][2 * k + 1] * inv * bf16hi(g.w[k]));
      orow[vi] = o;
    }
  }
}

template <bool kAdd>
void launch(bf16_t* out, const bf16_t* x, bf16_t* res, const bf16_t* w, int rows, int hidden, int64_t xs, int64_t os,
            int64_t rs, float eps, hipStream_t st) {
  const int nvec = hidden / 8;
  const int nv = (nvec + kThreads - 1) / kThreads;
  const bool exact = nvec % kThreads == 0;
#define DX_RMS_CASE(N)                                                                                  \
  case N:                                                                                               \
    if (exact)                                                                                          \
      rmsnorm_kernel<kAdd, N, true><<<rows, kThreads, 0, st>>>(out, x, res, w, hidden, xs, os, rs, eps); \
    else                                                                                                \
      rmsnorm_kernel<kAdd, N, false><<<rows, kThreads, 0, st>>>(out, x, res, w, hidden, xs, os, rs, eps); \
    break;
  switch (nv) {
    DX_RMS_CASE(1) DX_RMS_CASE(2) DX_RMS_CASE(3) DX_RMS_CASE(4) DX_RMS_CASE(5) DX_RMS_CASE(6) DX_RMS_CASE(7)
    DX_RMS_CASE(8)
    default: break;
  }
#undef DX_RMS_CASE
}

// 1 / rms of each row (fp32), for a norm folded into its consumers: the
// weight is pre-multiplied into the next projection's columns and the
// consumer of that projection's output scales its row by this value
// (models/llama.py "folded norm").  One workgroup per row, one read.
__global__ void __launch_bounds__(kThreads) row_rrms_kernel(float* __restrict__ out, const bf16_t* __restrict__ x,
                                                            int hidden, int64_t x_stride, float eps) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + row * x_stride);
  float ss = 0.f;
  for (int vi = threadIdx.x; vi < (hidden >> 3); vi += kThreads) {
    const u16x8 a = xr[vi];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = bf16lo(a.w[k]), hi = bf16hi(a.w[k]);
      ss += lo * lo + hi * hi;
    }
  }
  ss = block_reduce_sum(ss, red);
  if (threadIdx.x == 0) out[row] = rsqrtf(ss / (float)hidden + eps);
}

}  // namespace

extern "C" int dx_row_rrms(float* out, const void* x, int rows, int hidden, int64_t x_stride, float eps,
                           hipStream_t stream) {
  if (hidden % 8 || (x_stride & 7)) return -1;
  if (rows == 0) return 0;
  row_rrms_kernel<<<rows, kThreads, 0, stream>>>(out, (const bf16_t*)x, hidden, x_stride, eps);
  return (int)hipGetLastError();
}

extern "C" int dx_rmsnorm(void* out, const void* x, const void* w, int rows, int hidden, int64_t x_stride,
                          int64_t out_stride, float eps, hipStream_t stream) {
  if (hidden % 8 || hidden > kMaxVecLimit * 8 * kThreads) return -1;
  if (rows == 0) return 0;
  launch<false>((bf16_t*)out, (const bf16_t*)x, nullptr, (const bf16_t*)w, rows, hidden, x_stride, out_stride, 0,
                eps, stream);
  return (int)hipGetLastError();
}

// slabs: S x [BM][hidden] fp32 partials (slice s, row m at slabs + (s * BM + m) * hidden)
extern "C" int dx_add_rmsnorm_slabs(void* out, const float* slabs, int splits, int BM, void* residual, const void* w,
                                   int rows, int hidden, int64_t out_stride, int64_t res_stride, float eps,
                                   hipStream_t stream) {
  if (hidden % 8 || hidden > 4 * 8 * kThreads || rows > BM) return -1;
  if (rows == 0) return 0;
  const int nvec = hidden / 8;
  const bool exact = nvec % kThreads == 0;
  const int64_t ss = (int64_t)BM * hidden;
  auto* o = static_cast<bf16_t*>(out);
  auto* r = static_cast<bf16_t*>(residual);
  auto* g = static_cast<const bf16_t*>(w);
#define DX_RS(S_, V_, E_)                                                                                     \
  add_rmsnorm_slabs_kernel<S_, V_, E_><<<rows, kThreads, 0, stream>>>(o, slabs, ss, r, g, hidden, out_stride, \
                                                                      res_stride, eps)
#define DX_RS_V(S_, V_)                                       \
  if (exact) DX_RS(S_, V_, true); else DX_RS(S_, V_, false);
#define DX_RS_S(S_)                                           \
  if (nvec <= kThreads) { DX_RS_V(S_, 1) }                    \
  else if (nvec <= 2 * kThreads) { DX_RS_V(S_, 2) }           \
  else { DX_RS_V(S_, 4) }
  switch (splits) {
    case 2: DX_RS_S(2) break;
    case 4: DX_RS_S(4) break;
    case 8: DX_RS_S(8) break;
    default: return -2;
  }
#undef DX_RS_S
#undef DX_RS_V
#undef DX_RS
  return (int)hipGetLastError();
}

extern "C" int dx_add_rmsnorm(void* out, const void* x, void* residual, const void* w, int rows, int hidden,
                              int64_t x_stride, int64_t out_stride, int64_t res_stride, float eps,
                              hipStream_t stream) {
  if (hidden % 8 || hidden > kMaxVecLimit * 8 * kThreads) return -1;
  if (rows == 0) return 0;
  launch<true>((bf16_t*)out, (const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w, rows, hidden, x_stride,
               out_stride, res_stride, eps, stream);
  return (int)hipGetLastError();
}
