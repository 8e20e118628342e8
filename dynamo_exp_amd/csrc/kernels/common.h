// Shared helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64 everywhere (never 32-lane warp idioms);
//   * bf16 activations/KV, fp32 accumulation;
//   * global loads/stores are 16-byte vectors (dwordx4) wherever the layout
//     allows (guide G13: scalar bf16 loads cost 2-2.5x);
//   * launchers take a hipStream_t and never allocate / synchronise, so every
//     launch is hipGraph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DX_WAVE 64

typedef uint16_t bf16_t;  // raw bf16 bits
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

struct __attribute__((aligned(16))) u16x8 {
  uint32_t w[4];
};

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// low / high bf16 of a packed u32 -> f32 (one VALU op each)
__device__ __forceinline__ float bf16lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// f32 -> bf16, round-to-nearest-even; the plain cast lowers to v_cvt_pk_bf16_f32
// on gfx950 which keeps NaNs NaN (microarch "Correctness boundaries").
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  // one v_cvt_pk_bf16_f32 for the pair (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

// raw v_exp_f32 (2^x) without the denormal range fix-up exp2f() adds; inputs
// here are <= 0 softmax exponents where flushing tiny results to 0 is exact
// enough (|err| < 2^-126)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ float wave_reduce_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_reduce_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (16 waves). `red` must hold >= 16 floats.
__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_reduce_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = (threadIdx.x < (unsigned)nw) ? red[threadIdx.x] : 0.f;
  if (wid == 0) r = wave_reduce_sum(r);
  if (threadIdx.x == 0) red[0] = r;
  __syncthreads();
  r = red[0];
  __syncthreads();
  return r;
}

#define DX_CHECK_LAUNCH() (void)hipGetLastError()
