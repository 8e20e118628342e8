// FP8 (OCP e4m3fn) activation quantisation for the w8a8 serving path, gfx950.
//
// Every GEMM input of the fp8 model is produced by the kernel that already
// owns the row, so quantisation costs no extra pass over HBM:
//   * rmsnorm_quant  : [residual add +] RMSNorm -> e4m3 row + per-row scale
//                      (input of the QKV and gate|up projections)
//   * silu_mul_quant : silu(gate) * up          -> e4m3 row + per-row scale
//                      (input of the down projection)
//   * quant_rows     : bf16 rows                -> e4m3 rows + scales
//                      (attention output -> O projection)
// Rows up to 16384 elements: 256-thread workgroups; up to 65536: 1024.
// Dynamic per-token scaling: s = max|y| / 448, q = y / s, so the row's
// largest magnitude lands on e4m3's largest normal.  One workgroup (4 waves)
// per row; the row lives in registers between the max reduction and the
// store.  The e4m3 conversion is v_cvt_pk_fp8_f32 (OCP on gfx950, two values
// per instruction); inputs are clamped to +-448 first so a rounding overshoot
// can never produce the format's NaN.  GEMMs then run on hipBLASLt's fp8
// kernels with row-wise (token) x column-wise (channel) scales.
#include <type_traits>

#include "common.h"

namespace {

constexpr float kFp8Max = 448.f;

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

template <int TPB>
__device__ __forceinline__ float block_reduce_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_reduce_max(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < TPB / 64; ++i) r = fmaxf(r, red[i]);
  __syncthreads();
  return r;
}

// 8 floats (already divided by the scale) -> 8 e4m3 bytes
__device__ __forceinline__ uint2 pack_fp8x8(const float* y, float inv_s) {
  float c[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = fminf(fmaxf(y[k] * inv_s, -kFp8Max), kFp8Max);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
  return uint2{(uint32_t)lo, (uint32_t)hi};
}

// store the row from registers: v[i][8] values for vector index threadIdx + i*256
template <int TPB, int kMaxVec, bool kExact>
__device__ __forceinline__ void store_row(uint8_t* out_row, float* scale_out, float (&v)[kMaxVec][8], float amax,
                                          int nvec) {
  const float s = fmaxf(amax, 1e-6f) / kFp8Max;
  const float inv = 1.f / s;
  uint2* o = reinterpret_cast<uint2*>(out_row);
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * TPB;
    if (kExact || vi < nvec) o[vi] = pack_fp8x8(v[i], inv);
  }
  if (threadIdx.x == 0) *scale_out = s;
}

template <int TPB, bool kAdd, int kMaxVec, bool kExact>
__global__ void __launch_bounds__(TPB) rmsnorm_quant_kernel(uint8_t* __restrict__ out, float* __restrict__ scale,
                                                                 const bf16_t* x, bf16_t* residual,
                                                                 const bf16_t* __restrict__ w, int hidden,
                                                                 int64_t x_stride, int64_t res_stride, float eps) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int nvec = hidden >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + row * x_stride);
  u16x8* rr = kAdd ? reinterpret_cast<u16x8*>(residual + row * res_stride) : nullptr;
  float v[kMaxVec][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * TPB;
    if (kExact || vi < nvec) {
      u16x8 a = xr[vi];
      if constexpr (kAdd) {
        u16x8 r = rr[vi], s;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          s.w[k] = pack_bf16x2(bf16lo(a.w[k]) + bf16lo(r.w[k]), bf16hi(a.w[k]) + bf16hi(r.w[k]));
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
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * TPB;
    if (kExact || vi < nvec) {
      u16x8 g = wr[vi];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // round through bf16 like the bf16 path's normalised output
        v[i][2 * k] = bf16lo(pack_bf16x2(v[i][2 * k] * inv * bf16lo(g.w[k]), 0.f));
        v[i][2 * k + 1] = bf16lo(pack_bf16x2(v[i][2 * k + 1] * inv * bf16hi(g.w[k]), 0.f));
        amax = fmaxf(amax, fmaxf(fabsf(v[i][2 * k]), fabsf(v[i][2 * k + 1])));
      }
    }
  }
  amax = block_reduce_max<TPB>(amax, red);
  store_row<TPB, kMaxVec, kExact>(out + row * (int64_t)hidden, scale + row, v, amax, nvec);
}

template <int TPB, int kMaxVec, bool kExact>
__global__ void __launch_bounds__(TPB) silu_mul_quant_kernel(uint8_t* __restrict__ out, float* __restrict__ scale,
                                                                  const bf16_t* __restrict__ gate_up, int ffn,
                                                                  int64_t in_stride) {
  __shared__ float red[16];
  const int64_t t = blockIdx.x;
  const int nvec = ffn >> 3;
  const u16x8* g = reinterpret_cast<const u16x8*>(gate_up + t * in_stride);
  const u16x8* u = reinterpret_cast<const u16x8*>(gate_up + t * in_stride + ffn);
  float v[kMaxVec][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * TPB;
    if (kExact || vi < nvec) {
      u16x8 a = g[vi], b = u[vi];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[i][2 * k] = silu(bf16lo(a.w[k])) * bf16lo(b.w[k]);
        v[i][2 * k + 1] = silu(bf16hi(a.w[k])) * bf16hi(b.w[k]);
        amax = fmaxf(amax, fmaxf(fabsf(v[i][2 * k]), fabsf(v[i][2 * k + 1])));
      }
    }
  }
  amax = block_reduce_max<TPB>(amax, red);
  store_row<TPB, kMaxVec, kExact>(out + t * (int64_t)ffn, scale + t, v, amax, nvec);
}

template <int TPB, int kMaxVec, bool kExact>
__global__ void __launch_bounds__(TPB) quant_rows_kernel(uint8_t* __restrict__ out, float* __restrict__ scale,
                                                              const bf16_t* __restrict__ x, int cols,
                                                              int64_t x_stride) {
  __shared__ float red[16];
  const int64_t t = blockIdx.x;
  const int nvec = cols >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + t * x_stride);
  float v[kMaxVec][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxVec; ++i) {
    const int vi = threadIdx.x + i * TPB;
    if (kExact || vi < nvec) {
      u16x8 a = xr[vi];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[i][2 * k] = bf16lo(a.w[k]);
        v[i][2 * k + 1] = bf16hi(a.w[k]);
        amax = fmaxf(amax, fmaxf(fabsf(v[i][2 * k]), fabsf(v[i][2 * k + 1])));
      }
    }
  }
  amax = block_reduce_max<TPB>(amax, red);
  store_row<TPB, kMaxVec, kExact>(out + t * (int64_t)cols, scale + t, v, amax, nvec);
}

// dispatch on the per-thread vector count (row length <= 8 * 8 * 256 = 16384):
// f(integral_constant<int, N>, integral_constant<bool, exact>) launches
template <typename F>
int dispatch_nv(int nv, bool exact, F&& f) {
  auto go = [&](auto N) {
    if (exact)
      f(N, std::true_type{});
    else
      f(N, std::false_type{});
  };
  switch (nv) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 3: go(std::integral_constant<int, 3>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    case 5: go(std::integral_constant<int, 5>{}); break;
    case 6: go(std::integral_constant<int, 6>{}); break;
    case 7: go(std::integral_constant<int, 7>{}); break;
    case 8: go(std::integral_constant<int, 8>{}); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

}  // namespace

// rows up to 8 x 8 x 256 = 16384 elements use 256-thread workgroups, longer
// ones (Llama-3-70B FFN 28672) 1024 threads, up to 65536
template <typename F>
int launch_rows(int cols, F&& f) {
  if (cols % 8 || cols > 8 * 8 * 1024) return -1;
  const int nvec = cols / 8;
  if (nvec <= 8 * 256)
    return dispatch_nv((nvec + 255) / 256, nvec % 256 == 0,
                       [&](auto N, auto E) { f(std::integral_constant<int, 256>{}, N, E); });
  return dispatch_nv((nvec + 1023) / 1024, nvec % 1024 == 0,
                     [&](auto N, auto E) { f(std::integral_constant<int, 1024>{}, N, E); });
}

extern "C" int dx_rmsnorm_quant(void* out, float* scale, const void* x, void* residual, const void* w, int rows,
                                int hidden, int64_t x_stride, int64_t res_stride, float eps, hipStream_t st) {
  if (rows == 0) return hidden % 8 ? -1 : 0;
  auto o = (uint8_t*)out;
  auto xx = (const bf16_t*)x;
  auto rr = (bf16_t*)residual;
  auto ww = (const bf16_t*)w;
  return launch_rows(hidden, [&](auto T, auto N, auto E) {
    constexpr int tpb = decltype(T)::value;
    if (residual)
      rmsnorm_quant_kernel<tpb, true, decltype(N)::value, decltype(E)::value>
          <<<rows, tpb, 0, st>>>(o, scale, xx, rr, ww, hidden, x_stride, res_stride, eps);
    else
      rmsnorm_quant_kernel<tpb, false, decltype(N)::value, decltype(E)::value>
          <<<rows, tpb, 0, st>>>(o, scale, xx, rr, ww, hidden, x_stride, res_stride, eps);
  });
}

extern "C" int dx_silu_mul_quant(void* out, float* scale, const void* gate_up, int rows, int ffn, int64_t in_stride,
                                 hipStream_t st) {
  if (rows == 0) return ffn % 8 ? -1 : 0;
  return launch_rows(ffn, [&](auto T, auto N, auto E) {
    constexpr int tpb = decltype(T)::value;
    silu_mul_quant_kernel<tpb, decltype(N)::value, decltype(E)::value>
        <<<rows, tpb, 0, st>>>((uint8_t*)out, scale, (const bf16_t*)gate_up, ffn, in_stride);
  });
}

extern "C" int dx_quant_rows(void* out, float* scale, const void* x, int rows, int cols, int64_t x_stride,
                             hipStream_t st) {
  if (rows == 0) return cols % 8 ? -1 : 0;
  return launch_rows(cols, [&](auto T, auto N, auto E) {
    constexpr int tpb = decltype(T)::value;
    quant_rows_kernel<tpb, decltype(N)::value, decltype(E)::value>
        <<<rows, tpb, 0, st>>>((uint8_t*)out, scale, (const bf16_t*)x, cols, x_stride);
  });
}
