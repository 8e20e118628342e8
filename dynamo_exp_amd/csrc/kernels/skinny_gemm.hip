// Small-M projection GEMM (decode batches) for gfx950:
//     y[M, N] = x[M, K] . w[N, K]^T      bf16 in / out, fp32 accumulation, M <= 256
//
// At decode batch sizes the weight stream is the whole cost, and the GEMM
// library's tile grids for N = 4096-6144 at M <= 256 are too small to keep HBM
// busy (profiles/r1_skinny_gemm.json, weights cold: qkv / o / down at 1.2-2.9 TB/s).  Here:
//   * grid = (N / BN column tiles) x (ceil(M / BM) row tiles) x (S K-slices),
//     remapped so that all row tiles and K-slices of one column tile land on one
//     XCD (round-robin dispatch puts block b on XCD b % 8): the weight tile is
//     pulled from HBM once and re-read from that XCD's L2, and split-K slabs are
//     combined same-XCD (a speed choice only; the combine is correct anywhere);
//   * the 4 waves of a workgroup split the K-slice by interleaved 64-deep steps;
//     each wave loads its weight rows and x rows straight into MFMA fragments
//     (A = w rows, B = x rows of v_mfma_f32_32x32x16_bf16), double-buffered,
//     no LDS in the main loop (guide: "GEMV / M <= 16 decode weights: load
//     straight to VGPRs").  Weight loads use the default cache policy: a
//     fragment instruction covers 32 B of each of 32 rows, and the row's other
//     96 B arrive by the next three instructions from L2 -- non-temporal loads
//     refetched them from HBM (1.3-2x slower, profiles/r1_skinny_gemm_nt.json);
//   * k is permuted inside a step so that each lane's 4 loads of a row form one
//     contiguous 64-B run (the same permutation for both operands, so the dot
//     products are unchanged);
//   * the 4 waves' partial tiles are summed through LDS; with S > 1 every slice
//     writes an fp32 slab and the last arriver on the tile's ticket sums all
//     slabs in slice order, so results are bit-reproducible (agent-scope
//     release before the ticket, acquire after it; the reducer resets the
//     ticket, so a captured graph can replay the launch).
#include "common.h"

namespace {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr int KS = 64;       // k per wave step
constexpr int NB = KS / 16;  // MFMA k-blocks per step
constexpr int NWAVE = 4;

__device__ __forceinline__ bf16x8_t frag(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u32x4_t*>(p));
}

template <int NT, int MT>
struct Stage {
  bf16x8_t w[NT][NB];
  bf16x8_t x[MT][NB];
};

template <int NT, int MT>
__global__ void __launch_bounds__(64 * NWAVE) skinny_gemm_kernel(bf16_t* __restrict__ y, int64_t y_stride,
                                                                 const bf16_t* __restrict__ x, int64_t x_stride,
                                                                 const bf16_t* __restrict__ w,
                                                                 float* __restrict__ slabs, int* __restrict__ tickets,
                                                                 int M, int N, int K, int splits) {
  constexpr int BN = 32 * NT, BM = 32 * MT, NACC = NT * MT;
  // one LDS object (wave partials + the reducer flag; guide: a second
  // __shared__ object can de-pipeline the loop)
  __shared__ __attribute__((aligned(16))) float red[(NWAVE - 1) * NACC * 16 * 64 + 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int n_tiles = N / BN, m_tiles = (M + BM - 1) / BM;
  const int per_col = m_tiles * splits;
  const int total = n_tiles * per_col;
  int id = blockIdx.x;
  if ((total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
  const int nt = id / per_col;
  const int rem = id - nt * per_col;
  const int mt = rem / splits, sl = rem - mt * splits;
  const int kslice = K / splits;
  const int n_w = kslice / (KS * NWAVE);  // steps per wave (host guarantees >= 1, exact)
  const int64_t k0 = (int64_t)sl * kslice + h * (KS / 2) + wave * KS;

  const bf16_t* wp[NT];
  const bf16_t* xp[MT];
#pragma unroll
  for (int i = 0; i < NT; ++i) wp[i] = w + (int64_t)(nt * BN + i * 32 + r) * K + k0;
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int row = min(mt * BM + j * 32 + r, M - 1);  // padded rows recompute the last row
    xp[j] = x + (int64_t)row * x_stride + k0;
  }

  f32x16 acc[NT][MT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  auto load = [&](Stage<NT, MT>& st, int t) {
    const int64_t off = (int64_t)t * (KS * NWAVE);
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) st.w[i][kb] = frag(wp[i] + off + kb * 8);
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) st.x[j][kb] = frag(xp[j] + off + kb * 8);
  };
  auto mma = [&](const Stage<NT, MT>& st) {
#pragma unroll
    for (int kb = 0; kb < NB; ++kb)
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(st.w[i][kb], st.x[j][kb], acc[i][j], 0, 0, 0);
  };

  // branch-free steady state (the compiler's counted vmcnt waits survive), the
  // tail peeled: every wave runs exactly n_w steps
  Stage<NT, MT> s0, s1;
  load(s0, 0);
  int t = 0;
  // sched_barrier pins each prefetch group ahead of the MFMAs of the step
  // before it (left alone, the scheduler sinks the loads next to their use)
  for (; t + 2 < n_w; t += 2) {
    load(s1, t + 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(s0);
    __builtin_amdgcn_sched_barrier(0);
    load(s0, t + 2);
    __builtin_amdgcn_sched_barrier(0);
    mma(s1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (n_w - t == 2) {
    load(s1, t + 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(s0);
    mma(s1);
  } else {
    mma(s0);
  }

  // ---- sum the 4 waves' partial tiles (lane-contiguous LDS image, conflict-free)
  if (wave > 0) {
    float* dst = red + (wave - 1) * NACC * 1024;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) dst[((i * MT + j) * 16 + v) * 64 + lane] = acc[i][j][v];
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int wv = 0; wv < NWAVE - 1; ++wv)
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[i][j][v] += red[(wv * NACC + (i * MT + j)) * 1024 + v * 64 + lane];
  }

  // output element of acc[i][j][4g + q]: row m = mt*BM + 32j + r,
  // column n = nt*BN + 32i + 8g + 4h + q (4 consecutive columns per g)
  auto store_out = [&]() {
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = mt * BM + j * 32 + r;
      if (m >= M) continue;
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = nt * BN + i * 32 + 8 * g + 4 * h;
          uint2 pk;
          pk.x = pack_bf16x2(acc[i][j][4 * g], acc[i][j][4 * g + 1]);
          pk.y = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
          *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n) = pk;
        }
    }
  };

  if (splits == 1) {
    if (wave == 0) store_out();
    return;
  }

  // ---- split-K: publish this slice's slab, take a ticket; the last arriver combines
  const int64_t slab_elems = (int64_t)m_tiles * BM * N;
  if (wave == 0) {
    float* slab = slabs + (int64_t)sl * slab_elems;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = mt * BM + j * 32 + r;
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = nt * BN + i * 32 + 8 * g + 4 * h;
          *reinterpret_cast<f32x4*>(slab + (int64_t)m * N + n) =
              f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(red + (NWAVE - 1) * NACC * 1024);
  int* ticket = tickets + nt * m_tiles + mt;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (tk == splits - 1);
  }
  __syncthreads();
  if (!*flag) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (wave != 0) return;
  // sum every slice's slab (this one's too) in slice order: the result does
  // not depend on which slice arrived last (bit-reproducible runs)
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
  for (int s2 = 0; s2 < splits; ++s2) {
    const float* slab = slabs + (int64_t)s2 * slab_elems;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = mt * BM + j * 32 + r;
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = nt * BN + i * 32 + 8 * g + 4 * h;
          const f32x4 p = *reinterpret_cast<const f32x4*>(slab + (int64_t)m * N + n);
          acc[i][j][4 * g] += p[0];
          acc[i][j][4 * g + 1] += p[1];
          acc[i][j][4 * g + 2] += p[2];
          acc[i][j][4 * g + 3] += p[3];
        }
    }
  }
  store_out();
}

template <int NT, int MT>
void launch(bf16_t* y, int64_t ys, const bf16_t* x, int64_t xs, const bf16_t* w, float* slabs, int* tickets, int M,
            int N, int K, int splits, hipStream_t st) {
  const int grid = (N / (32 * NT)) * ((M + 32 * MT - 1) / (32 * MT)) * splits;
  hipLaunchKernelGGL((skinny_gemm_kernel<NT, MT>), dim3(grid), dim3(64 * NWAVE), 0, st, y, ys, x, xs, w, slabs,
                     tickets, M, N, K, splits);
}

// ---------------------------------------------------------------------------
// Wide variant (bn = 128), for M ~ 64-256 where x re-reads dominate the
// narrow kernel's traffic: the workgroup covers all M rows (BM = 32*MT) x 128
// weight rows; each wave owns 32 weight rows (fragments straight to VGPRs,
// double-buffered) and all waves share the x tile of the step through a
// double-buffered, XOR-swizzled LDS image (register-staged: full 128-B rows
// per 8 lanes, conflict-free ds_read_b128 fragments).  K is split only over
// workgroups (slabs + ticket as above).
template <int MT, int KSW>
__global__ void __launch_bounds__(256) skinny_wide_kernel(bf16_t* __restrict__ y, int64_t y_stride,
                                                          const bf16_t* __restrict__ x, int64_t x_stride,
                                                          const bf16_t* __restrict__ w, float* __restrict__ slabs,
                                                          int* __restrict__ tickets, int M, int N, int K, int splits) {
  constexpr int BN = 128, BM = 32 * MT;
  constexpr int NBW = KSW / 16, RB = KSW * 2, CPR = RB / 16;  // k-blocks, row bytes, 16-B chunks per row
  constexpr int XB = BM * RB;  // one x stage: BM rows x RB bytes
  constexpr int XC = XB / 16 / 256;  // 16-B chunks per thread per stage
  // XOR swizzle of the 16-B chunks of an x row.  With 256-B rows (KSW 128)
  // every ds_read_b128 lane group (16 lanes: rows r with 16 distinct r & 15)
  // must see 16 distinct slots, hence r & 15 -- r & 7 left each slot read by
  // two lanes of a group (2-way conflicts, SQ_LDS_BANK_CONFLICT 3.2 cycles per
  // LDS instruction: profiles/r1_pmc_skinny.txt).  The stores (8-lane groups,
  // banks mod 32) stay conflict-free under either mask.
  constexpr int SWZ = CPR >= 16 ? 15 : 7;
  __shared__ __attribute__((aligned(16))) char smem[2 * XB + 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int n_tiles = N / BN;
  const int total = n_tiles * splits;
  int id = blockIdx.x;
  if ((total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
  const int nt = id / splits, sl = id - nt * splits;
  const int kslice = K / splits;
  const int nsteps = kslice / KSW;
  const int64_t kbeg = (int64_t)sl * kslice;

  const bf16_t* wp = w + (int64_t)(nt * BN + wave * 32 + r) * K + kbeg + h * (KSW / 2);
  const bf16_t* xsrc[XC];
  int xdst[XC];
#pragma unroll
  for (int c = 0; c < XC; ++c) {
    const int q = tid + 256 * c, m = q / CPR, ch = q % CPR;
    xsrc[c] = x + (int64_t)min(m, M - 1) * x_stride + kbeg + ch * 8;
    xdst[c] = m * RB + ((ch ^ (m & SWZ)) << 4);
  }
  f32x16 acc[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[j][v] = 0.f;

  u32x4_t xr[XC];
  bf16x8_t wa[NBW], wb[NBW];
  auto load_x = [&](int t) {
#pragma unroll
    for (int c = 0; c < XC; ++c) xr[c] = *reinterpret_cast<const u32x4_t*>(xsrc[c] + (int64_t)t * KSW);
  };
  auto load_w = [&](bf16x8_t(&dst)[NBW], int t) {
#pragma unroll
    for (int kb = 0; kb < NBW; ++kb) dst[kb] = frag(wp + (int64_t)t * KSW + kb * 8);
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int c = 0; c < XC; ++c) *reinterpret_cast<u32x4_t*>(smem + buf * XB + xdst[c]) = xr[c];
  };
  auto compute = [&](int buf, const bf16x8_t(&wf)[NBW]) {
    const char* xs = smem + buf * XB;
#pragma unroll
    for (int kb = 0; kb < NBW; ++kb)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const bf16x8_t xf =
            *reinterpret_cast<const bf16x8_t*>(xs + (j * 32 + r) * RB + (((h * NBW + kb) ^ (r & SWZ)) << 4));
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[kb], xf, acc[j], 0, 0, 0);
      }
  };
  // one step: prefetch step t+1 (x to registers, w fragments), compute step t
  // from LDS buffer `buf`, then publish x(t+1) into the other buffer
  auto step = [&](int t, int buf, const bf16x8_t(&cur)[NBW], bf16x8_t(&nxt)[NBW]) {
    load_x(t + 1);
    load_w(nxt, t + 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(buf, cur);
    store_x(buf ^ 1);
    __syncthreads();
  };

  load_x(0);
  load_w(wa, 0);
  store_x(0);
  __syncthreads();
  int t = 0;
  for (; t + 2 < nsteps; t += 2) {
    step(t, 0, wa, wb);
    step(t + 1, 1, wb, wa);
  }
  if (nsteps - t == 2) {
    step(t, 0, wa, wb);
    compute(1, wb);
  } else {
    compute(0, wa);
  }

  // acc[j][4g + q]: row m = 32j + r, column n = nt*128 + 32*wave + 8g + 4h + q
  const int n0 = nt * BN + wave * 32 + 4 * h;
  if (splits == 1) {
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int m = j * 32 + r;
      if (m >= M) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 pk;
        pk.x = pack_bf16x2(acc[j][4 * g], acc[j][4 * g + 1]);
        pk.y = pack_bf16x2(acc[j][4 * g + 2], acc[j][4 * g + 3]);
        *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n0 + 8 * g) = pk;
      }
    }
    return;
  }
  const int64_t slab_elems = (int64_t)BM * N;
  {
    float* slab = slabs + (int64_t)sl * slab_elems;
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(slab + (int64_t)(j * 32 + r) * N + n0 + 8 * g) =
            f32x4{acc[j][4 * g], acc[j][4 * g + 1], acc[j][4 * g + 2], acc[j][4 * g + 3]};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem + 2 * XB);
  int* ticket = tickets + nt;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (tk == splits - 1);
  }
  __syncthreads();
  if (!*flag) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < MT; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[j][v] = 0.f;
  for (int s2 = 0; s2 < splits; ++s2) {  // slice order, own slab included (reproducible)
    const float* slab = slabs + (int64_t)s2 * slab_elems;
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 p = *reinterpret_cast<const f32x4*>(slab + (int64_t)(j * 32 + r) * N + n0 + 8 * g);
        acc[j][4 * g] += p[0];
        acc[j][4 * g + 1] += p[1];
        acc[j][4 * g + 2] += p[2];
        acc[j][4 * g + 3] += p[3];
      }
  }
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = j * 32 + r;
    if (m >= M) continue;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 pk;
      pk.x = pack_bf16x2(acc[j][4 * g], acc[j][4 * g + 1]);
      pk.y = pack_bf16x2(acc[j][4 * g + 2], acc[j][4 * g + 3]);
      *reinterpret_cast<uint2*>(y + (int64_t)m * y_stride + n0 + 8 * g) = pk;
    }
  }
}

// 128-deep steps (8 KB of weights per wave in flight) up to 128 rows; 64-deep
// above, where the accumulators take the registers
template <int MT>
void launch_wide(bf16_t* y, int64_t ys, const bf16_t* x, int64_t xs, const bf16_t* w, float* slabs, int* tickets,
                 int M, int N, int K, int splits, hipStream_t st) {
  constexpr int KSW = MT <= 4 ? 128 : 64;
  hipLaunchKernelGGL((skinny_wide_kernel<MT, KSW>), dim3((N / 128) * splits), dim3(256), 0, st, y, ys, x, xs, w,
                     slabs, tickets, M, N, K, splits);
}

}  // namespace

// bn, bm in {32, 64}: narrow kernel, K % (splits * 256) == 0;
// bn = 128: wide kernel, bm = 32 * ceil(M / 32), K % (splits * (bm <= 128 ? 128 : 64)) == 0.
// With splits > 1: slabs >= splits * ceil(M/bm)*bm * N floats and tickets >=
// (N/bn) * ceil(M/bm) zeroed ints.
extern "C" int dx_skinny_gemm(void* y, int64_t y_stride, const void* x, int64_t x_stride, const void* w,
                              float* slabs, int* tickets, int M, int N, int K, int bn, int bm, int splits,
                              hipStream_t st) {
  if (M < 1 || M > 256 || splits < 1) return 1;
  if (splits > 1 && (slabs == nullptr || tickets == nullptr)) return 4;
  if ((x_stride & 7) || (K & 7) || (y_stride & 3)) return 5;
  auto* Y = static_cast<bf16_t*>(y);
  auto* X = static_cast<const bf16_t*>(x);
  auto* W = static_cast<const bf16_t*>(w);
  if (bn == 128) {
    const int mt = (M + 31) / 32;
    if (bm != 32 * mt || N % 128 != 0 || K % (splits * (mt <= 4 ? 128 : 64)) != 0) return 3;
    switch (mt) {
      case 1: launch_wide<1>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
      case 2: launch_wide<2>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
      case 3: launch_wide<3>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
      case 4: launch_wide<4>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
      case 5: launch_wide<5>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
      case 6: launch_wide<6>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
      case 7: launch_wide<7>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
      default: launch_wide<8>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st); break;
    }
    DX_CHECK_LAUNCH();
    return 0;
  }
  if ((bn != 32 && bn != 64) || (bm != 32 && bm != 64)) return 2;
  if (N % bn != 0 || K % (splits * KS * NWAVE) != 0) return 3;
  if (bn == 32 && bm == 32) launch<1, 1>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st);
  else if (bn == 32) launch<1, 2>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st);
  else if (bm == 32) launch<2, 1>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st);
  else launch<2, 2>(Y, y_stride, X, x_stride, W, slabs, tickets, M, N, K, splits, st);
  DX_CHECK_LAUNCH();
  return 0;
}
