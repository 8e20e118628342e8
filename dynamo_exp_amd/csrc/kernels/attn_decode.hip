// Paged-KV decode attention (one query token per sequence, GQA) for gfx950.
//
// Memory-bound: every (token, kv-head) K and V row (2 x 256 B at D=128) is read
// exactly once from HBM per step and shared by the G = Hq/Hkv query heads of
// the group, so the query heads of a group are processed together by one
// workgroup.  Flash-decoding split: grid = (P, Hkv, B) with P balanced
// partitions per sequence: each workgroup takes ceil(ctx / P) tokens (rounded
// to the 4-wave chunk), computed in-kernel from ctx, so one hipGraph captured
// for a batch bucket stays balanced for any context length.  The host picks P
// so the grid has ~512 long-lived workgroups (decode_num_parts): short parts
// (many workgroups of a few chunks each) pay the Q-load / merge prologue and
// epilogue per few KB streamed, and an uneven tail part idles most of the
// chip -- balanced long parts measured 6.0-6.4 TB/s vs 5.0-5.8 with fixed
// 512-token parts (B 64-256, ctx 3072, tools/decode_parts.py).  A reduce kernel
// merges partitions (skipped when P = 1).
//
// Lane layout (wave64): LPT lanes cooperate on one KV row, each owning DPL =
// 128/LPT contiguous dims, i.e. VPL = DPL/8 16-byte loads per row -- so a wave
// instruction covers 64/LPT whole rows (fully coalesced).  Q.K partial dots use
// v_dot2_f32_bf16 and are all-reduced inside the LPT-lane group with DPP
// (row_ror / row_half_mirror / quad_perm; no LDS).  Each lane-group keeps its
// own online-softmax state; a wave's groups are merged in registers (shuffle
// reduce-scatter), then the 4 waves' states once through LDS.
// Each wave streams 16-token chunks (all K/V loads of a chunk issued back to
// back, 8-16 x 16 B per lane in flight); latency is covered by 3-4 waves/SIMD.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr int D = 128;
constexpr int kThreads = 256;
constexpr int kChunk = 16;  // minimum tokens per wave iteration (BS must be a multiple)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// 16-byte K/V row-piece load; NT = non-temporal (once-read stream: the KV
// cache is read exactly once per step, keep it out of L2/MALL residency)
template <bool NT>
__device__ __forceinline__ u32x4_t ld16(const bf16_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  else return *reinterpret_cast<const u32x4_t*>(p);
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// FP8 cache: a lane loads the same 8 dims of a row as on the bf16 path, as 8
// e4m3 bytes (one 8-B non-temporal load), and keeps them raw until use; a
// wave keeps TWO chunks in flight, i.e. as many BYTES as the bf16 path with
// one (twice the tokens), at about the same register cost.  At use they widen to the bf16 pairs the shared dot / FMA code takes (e4m3 ->
// f32 -> bf16 is exact; the per-tensor scales are folded into the softmax
// scale and the output).
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x8 fp8x8_to_bf16(const u32x2_t t) {
  u16x8 o;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)t[h], false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)t[h], true);
    o.w[2 * h] = pack_bf16x2(lo[0], lo[1]);
    o.w[2 * h + 1] = pack_bf16x2(hi[0], hi[1]);
  }
  return o;
}

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

// all-reduce (sum) inside aligned groups of LPT lanes (LPT in {4, 8, 16})
template <int LPT>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (LPT == 16) v += dppf<0x128>(v);  // row_ror:8
  if constexpr (LPT >= 8) v += dppf<0x141>(v);   // row_half_mirror
  v += dppf<0xB1>(v);                            // quad_perm [1,0,3,2]
  v += dppf<0x4E>(v);                            // quad_perm [2,3,0,1]
  return v;
}

// tokens per partition when a context of ctx tokens is split into n balanced
// parts, rounded up to `align` (the workgroup's 4-wave chunk stride)
__device__ __forceinline__ int balanced_part(int ctx, int n, int align) {
  const int per = (ctx + n - 1) / n;
  return (per + align - 1) / align * align;
}

template <int G, int LPT, int CH>
struct Cfg {
  static constexpr int DPL = D / LPT;       // dims per lane
  static constexpr int VPL = DPL / 8;       // 16B vectors per lane per row
  static constexpr int TPW = 64 / LPT;      // rows per wave instruction
  static constexpr int TPL = CH / TPW;      // rows per lane per chunk
  static constexpr int SRC = 4;             // softmax partial states per WG (one per wave after the in-wave merge)
};

// Workgroup epilogue shared by both decode kernels: combine the 4 waves'
// softmax states (so [4][G][D], sm / sl [4][G] in LDS, after a barrier) and
// write the output row (one partition) or the partition's (O, m, l).
template <int G>
__device__ __forceinline__ void finish_workgroup(const float* so, const float* sm, const float* sl,
                                                 bf16_t* __restrict__ out, float* __restrict__ tmp_out,
                                                 float* __restrict__ tmp_ml, int b, int kvh, int pid, int n_parts,
                                                 int n_q_heads, float out_scale) {
  const bool single = n_parts == 1;
  for (int idx = threadIdx.x; idx < G * D; idx += kThreads) {
    const int h = idx / D, d = idx % D;
    float M = -1e30f;
    for (int s2 = 0; s2 < 4; ++s2) M = fmaxf(M, sm[s2 * G + h]);
    float so_sum = 0.f, sl_sum = 0.f;
    for (int s2 = 0; s2 < 4; ++s2) {
      const float f = exp2f(sm[s2 * G + h] - M);
      so_sum += f * so[((int64_t)s2 * G + h) * D + d];
      sl_sum += f * sl[s2 * G + h];
    }
    const int qh = kvh * G + h;
    const float val = sl_sum > 0.f ? so_sum / sl_sum * out_scale : 0.f;
    if (single) {
      out[((int64_t)b * n_q_heads + qh) * D + d] = f32_to_bf16(val);
    } else {
      const int64_t row = ((int64_t)b * n_q_heads + qh) * n_parts + pid;
      tmp_out[row * D + d] = val;
      if (d == 0) {
        tmp_ml[row * 2] = M;
        tmp_ml[row * 2 + 1] = sl_sum;
      }
    }
  }
}

template <int G, int LPT, int CH, bool NT, bool F8 = false>
__global__ void __launch_bounds__(kThreads) decode_attn_kernel(
    bf16_t* __restrict__ out, float* __restrict__ tmp_out, float* __restrict__ tmp_ml, const bf16_t* __restrict__ q,
    int64_t q_stride, const void* __restrict__ k_cache_, const void* __restrict__ v_cache_,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ ctx_lens, int n_kv_heads,
    int block_size, float scale_log2e, float out_scale) {
  using CT = typename std::conditional<F8, uint8_t, bf16_t>::type;
  const CT* k_cache = static_cast<const CT*>(k_cache_);
  const CT* v_cache = static_cast<const CT*>(v_cache_);
  using C = Cfg<G, LPT, CH>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int pid = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int n_parts = gridDim.x;
  const int ctx = ctx_lens[b];
  const int part_size = balanced_part(ctx, n_parts, 4 * CH);
  const int p0 = pid * part_size;
  if (p0 >= ctx) return;
  const int p1 = min(p0 + part_size, ctx);
  // wid through readfirstlane: the chunk loop below is then wave-uniform to the
  // compiler too (scalar branches instead of an exec-masked loop)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = lane / LPT, sub = lane % LPT;
  const int d0 = sub * C::DPL;
  const int n_q_heads = n_kv_heads * G;

  // Q for the G heads of this kv group, my DPL dims, packed bf16 pairs
  uint32_t qw[G][C::VPL * 4];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const bf16_t* qp = q + (int64_t)b * q_stride + (int64_t)(kvh * G + h) * D + d0;
#pragma unroll
    for (int v = 0; v < C::VPL; ++v) {
      u16x8 t = reinterpret_cast<const u16x8*>(qp)[v];
#pragma unroll
      for (int w = 0; w < 4; ++w) qw[h][v * 4 + w] = t.w[w];
    }
  }

  float m[G], l[G], o[G][C::DPL];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m[h] = -1e30f;
    l[h] = 0.f;
#pragma unroll
    for (int d = 0; d < C::DPL; ++d) o[h][d] = 0.f;
  }

  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int64_t head_stride = (int64_t)block_size * D;
  const int n_chunks = (p1 - p0 + CH - 1) / CH;

  // K / V rows as whole 128-bit vector values, zeroed whole when masked: held
  // as 4 x u32 structs, the masking branch's per-dword writes hit an LLVM
  // sub-register liveness bug (gfx950, ROCm 7.2: "No live subrange at use"
  // under -verify-machineinstrs) that reused V registers as temporaries in the
  // G = 1 instance: half of each V vector read back as garbage (round-5 GPU
  // dump: profiles/r5_decode_g1_miscompile.txt).  tests/test_build.py runs the
  // machine verifier over the kernel sources.
  u32x4_t kA[C::TPL][C::VPL] = {}, vA[C::TPL][C::VPL] = {};
  // fp8: raw 8-B vectors, TWO chunks in flight per wave (the raw registers of
  // two fp8 chunks cost what one bf16 chunk does, so the wave keeps the bf16
  // path's bytes in flight at the same occupancy)
  // raw loads: 16 B (16 dims) when a lane owns >= 16 dims, else 8 B
  constexpr bool W16 = F8 && (C::VPL % 2 == 0);
  constexpr int VR = !F8 ? 1 : (W16 ? C::VPL / 2 : C::VPL);
  using RawT = typename std::conditional<W16, u32x4_t, u32x2_t>::type;
  constexpr int NSET = F8 ? 2 : 1;
  constexpr int STRIDE = 4 * NSET;  // chunk distance between a load and its use
  RawT kR[NSET][C::TPL][VR] = {}, vR[NSET][C::TPL][VR] = {};
  auto raw8 = [](const RawT (&r)[VR], int v) -> u32x2_t {  // the 8 fp8 bytes of dims 8v .. 8v+7
    if constexpr (W16) return u32x2_t{r[v >> 1][2 * (v & 1)], r[v >> 1][2 * (v & 1) + 1]};
    else return r[v];
  };


  auto row_base = [&](int c) {
    const int cb = p0 + c * CH;
    const int blk = bt[cb / block_size];
    return ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(cb % block_size) * D + d0;
  };
  auto load_k = [&](int c, auto setc) {
    constexpr int SET = decltype(setc)::value;
    const int64_t base = row_base(c);
#pragma unroll
    for (int i = 0; i < C::TPL; ++i)
#pragma unroll
      for (int v = 0; v < (F8 ? VR : C::VPL); ++v) {
        const CT* p = k_cache + base + (int64_t)(grp + C::TPW * i) * D + (W16 ? 16 : 8) * v;
        if constexpr (F8) kR[SET][i][v] = __builtin_nontemporal_load(reinterpret_cast<const RawT*>(p));
        else kA[i][v] = ld16<NT>(p);
      }
  };
  auto load_v = [&](int c, auto setc) {
    constexpr int SET = decltype(setc)::value;
    const int64_t base = row_base(c);
#pragma unroll
    for (int i = 0; i < C::TPL; ++i)
#pragma unroll
      for (int v = 0; v < (F8 ? VR : C::VPL); ++v) {
        const CT* p = v_cache + base + (int64_t)(grp + C::TPW * i) * D + (W16 ? 16 : 8) * v;
        if constexpr (F8) vR[SET][i][v] = __builtin_nontemporal_load(reinterpret_cast<const RawT*>(p));
        else vA[i][v] = ld16<NT>(p);
      }
  };

  // Software pipeline with one register set: K(c+4) is issued right after
  // Q.K(c) frees kA and V(c+4) right after P.V(c) frees vA, so every wave
  // keeps a chunk of K or V in flight through its softmax / PV work.  (An
  // LDS-DMA ring variant measured slower: profiles/r1_decode_attn_dma.json.)
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, NSET - 1>;
  int c = wid;
  if (c < n_chunks) {
    load_k(c, S0{});
    load_v(c, S0{});
  }
  if (F8 && c + 4 < n_chunks) {
    load_k(c + 4, S1{});
    load_v(c + 4, S1{});
  }
  auto step = [&](const int c, auto setc) {
    constexpr int SET = decltype(setc)::value;
    const bool more = c + STRIDE < n_chunks;  // wave-uniform
    const int cb = p0 + c * CH;
    float s[C::TPL][G];
#pragma unroll
    for (int i = 0; i < C::TPL; ++i) {
      u16x8 kx[C::VPL];  // this row's K: loaded bf16, or fp8 widened right before use
#pragma unroll
      for (int v = 0; v < C::VPL; ++v) {
        if constexpr (F8) kx[v] = fp8x8_to_bf16(raw8(kR[SET][i], v));
        else kx[v] = __builtin_bit_cast(u16x8, kA[i][v]);
      }
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float acc = 0.f;
#pragma unroll
        for (int v = 0; v < C::VPL; ++v)
#pragma unroll
          for (int w = 0; w < 4; ++w)
            acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, qw[h][v * 4 + w]),
                                                  __builtin_bit_cast(bf16x2_t, kx[v].w[w]), acc, false);
        s[i][h] = group_sum<LPT>(acc) * scale_log2e;
      }
    }
    if (more) load_k(c + STRIDE, setc);
    if (cb + CH > p1) {  // partial last chunk (wave-uniform)
#pragma unroll
      for (int i = 0; i < C::TPL; ++i) {
        if (cb + grp + C::TPW * i >= p1) {
#pragma unroll
          for (int h = 0; h < G; ++h) s[i][h] = -INFINITY;
#pragma unroll
          for (int v = 0; v < (F8 ? VR : C::VPL); ++v) {
            if constexpr (F8) vR[SET][i][v] = RawT{};  // e4m3 0x00 = +0
            else vA[i][v] = u32x4_t{0u, 0u, 0u, 0u};
          }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float mc = s[0][h];
#pragma unroll
      for (int i = 1; i < C::TPL; ++i) mc = fmaxf(mc, s[i][h]);
      const float mn = fmaxf(m[h], mc);
      const float alpha = fast_exp2(m[h] - mn);
      m[h] = mn;
      float p[C::TPL];
      float ps = 0.f;
#pragma unroll
      for (int i = 0; i < C::TPL; ++i) {
        p[i] = fast_exp2(s[i][h] - mn);
        ps += p[i];
      }
      l[h] = l[h] * alpha + ps;
#pragma unroll
      for (int d = 0; d < C::DPL; ++d) o[h][d] *= alpha;
#pragma unroll
      for (int i = 0; i < C::TPL; ++i)
#pragma unroll
        for (int v = 0; v < C::VPL; ++v) {
          u16x8 vx;
          if constexpr (F8) vx = fp8x8_to_bf16(raw8(vR[SET][i], v));
          else vx = __builtin_bit_cast(u16x8, vA[i][v]);
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            o[h][v * 8 + 2 * w] += p[i] * bf16lo(vx.w[w]);
            o[h][v * 8 + 2 * w + 1] += p[i] * bf16hi(vx.w[w]);
          }
        }
    }
    if (more) load_v(c + STRIDE, setc);
  };
  if constexpr (F8) {
    for (; c < n_chunks; c += 8) {
      step(c, S0{});
      if (c + 4 < n_chunks) step(c + 4, S1{});
    }
  } else {
    for (; c < n_chunks; c += 4) step(c, S0{});
  }

  // ---- merge the TPW lane groups of each wave in registers (cross-group
  // shuffles), then the 4 waves' states through LDS.  (Round 5: merging all
  // 4 * TPW group states through LDS took 64 KiB at G = 8 -- two workgroups
  // per CU -- and 16 LDS passes per output, a fixed per-workgroup cost that
  // short partitions, e.g. one Llama-3-70B TP4 rank's 2 KV heads, could not
  // amortise.)  The o merge is a reduce-scatter butterfly: at the level that
  // pairs groups g and g ^ 2^i, each lane keeps half of its remaining dims
  // (the upper half when bit i of its group is set) and adds the partner's
  // copy of that half, so after log2(TPW) levels every lane owns
  // DPL / TPW = 2 summed dims: DPL - 2 shuffles per head instead of
  // DPL * log2(TPW), and all 64 lanes write LDS instead of one group.
  constexpr int LEV = __builtin_ctz(C::TPW);
  constexpr int OWN = C::DPL >> LEV;  // dims a lane owns after the butterfly
  static_assert(OWN >= 1 && (C::DPL % (1 << LEV)) == 0, "decode merge: DPL must split over the lane groups");
  int own0 = d0;                      // first of the OWN dims this lane ends with
#pragma unroll
  for (int i = 0; i < LEV; ++i) {
    if (grp & (1 << i)) own0 += C::DPL >> (i + 1);
  }
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float M = m[h];
#pragma unroll
    for (int x = LPT; x < 64; x <<= 1) M = fmaxf(M, __shfl_xor(M, x, 64));
    const float f = exp2f(m[h] - M);
    float lsum = l[h] * f;
#pragma unroll
    for (int x = LPT; x < 64; x <<= 1) lsum += __shfl_xor(lsum, x, 64);
#pragma unroll
    for (int d = 0; d < C::DPL; ++d) o[h][d] *= f;
#pragma unroll
    for (int i = 0; i < LEV; ++i) {
      const int n = C::DPL >> (i + 1);  // dims kept at this level
      const bool up = grp & (1 << i);
#pragma unroll
      for (int j = 0; j < n; ++j) {
        const float lo = o[h][j], hi = o[h][j + n];
        const float got = __shfl_xor(up ? lo : hi, LPT << i, 64);
        o[h][j] = (up ? hi : lo) + got;
      }
    }
    m[h] = M;
    l[h] = lsum;
  }
  float* so = smem;                        // [SRC][G][D]
  float* sm = smem + C::SRC * G * D;       // [SRC][G]
  float* sl = sm + C::SRC * G;             // [SRC][G]
  const int src = wid;
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float* dst = so + ((int64_t)src * G + h) * D + own0;
#pragma unroll
    for (int d = 0; d < OWN; ++d) dst[d] = o[h][d];
    if (lane == 0) {
      sm[src * G + h] = m[h];
      sl[src * G + h] = l[h];
    }
  }
  __syncthreads();
  finish_workgroup<G>(so, sm, sl, out, tmp_out, tmp_ml, b, kvh, pid, n_parts, n_q_heads, out_scale);
}


// ---------------------------------------------------------------------------
// MFMA variant for G = 1 .. 16 query heads per KV head (bf16 or fp8 KV,
// block size a multiple of 16: a 32-token chunk spans two 16-token blocks
// then, looked up per half).  The
// VALU kernel spends 2 x G x D VALU operations per KV row (dot2 + FMA), so
// at G = 8 (one Llama-3-70B TP4 rank's
// 16 q / 2 kv heads, or 70B at TP1) it is issue-bound at 3.3-3.8 TB/s.  Here
// both products run on the matrix pipe and the VALU only does the softmax:
//   * a wave takes 32-token chunks (every 4th); the G heads are the 16 columns
//     of v_mfma_f32_16x16x32_bf16 (padded with zero Q rows);
//   * S = K . Q^T as two 16-token row blocks: K is the A operand straight from
//     global memory (lane = token row, 4 lanes x 64 contiguous bytes per row
//     per load), Q the B operand (dims permuted identically: k-step s, lane
//     group g holds dims 8 (4s + g) .. +8);
//   * the S accumulators hold, per lane, 8 tokens of one head: the softmax is
//     lane-local except the chunk max (two cross-group exchanges), and the
//     accumulators are directly the B operand (P^T, k = token) of
//     O^T = V^T . P^T -- the A row block -> token map is chosen so that lane
//     group g's 8 P values are tokens 8g .. 8g+7 (guide section 3,
//     "accumulator tile as next operand");
//   * V rows are loaded coalesced (4 full rows per wave instruction), stored
//     to the wave's 8 KiB LDS image (XOR-swizzled 256-B rows) and read back
//     as V^T fragments with ds_read_b64_tr_b16 (guide T10): per 16-dim block,
//     tokens 8g .. 8g+3 and 8g+4 .. 8g+7 (two 4-row blocks 8 rows apart in a
//     32-lane half: conflict-free);
//   * O^T accumulators: lane (g, r) holds dims 16 db + 4 g + i of head r, so
//     the online-softmax rescale is lane-local; deferred max (rescale only
//     when the chunk max exceeds the running one by 2^8, guide T13) with the
//     row sum of the bf16-rounded P, so O / l stays an exact weighted mean.
// FP8 (e4m3fn) caches: the same products on bf16 operands widened in
// registers -- K right before its MFMAs (a lane's 4 k-steps are then its 32
// contiguous dims: dim block 4g + s), V before the LDS store (the image and
// the transposed reads stay bf16); half the bytes per token.
// The epilogue and the flash-decoding partitions are the VALU kernel's.
constexpr int MCH = 32;  // tokens per wave chunk

__device__ __forceinline__ int vimg_off(int row, int ch) {  // byte offset of 16-B chunk ch of row in a wave's image
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

typedef __attribute__((address_space(3))) i16x4 lds_i16x4_t;

template <int G, bool NT, bool F8>
__global__ void __launch_bounds__(kThreads) decode_attn_mfma_kernel(
    bf16_t* __restrict__ out, float* __restrict__ tmp_out, float* __restrict__ tmp_ml, const bf16_t* __restrict__ q,
    int64_t q_stride, const void* __restrict__ k_cache_, const void* __restrict__ v_cache_,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ ctx_lens, int n_kv_heads,
    int block_size, float scale_log2e, float out_scale) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "MFMA decode: 1-16 query heads per KV head");
  using CT = typename std::conditional<F8, uint8_t, bf16_t>::type;
  const CT* k_cache = static_cast<const CT*>(k_cache_);
  const CT* v_cache = static_cast<const CT*>(v_cache_);
  constexpr float kRescale = 8.0f;  // deferred-max threshold (log2 units)
  __shared__ __attribute__((aligned(16))) char vimg_all[4 * MCH * D * 2];     // 4 x 8 KiB
  __shared__ __attribute__((aligned(16))) float st_o[4 * G * D], st_m[4 * G], st_l[4 * G];
  const int pid = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int n_parts = gridDim.x;
  const int ctx = ctx_lens[b];
  const int part_size = balanced_part(ctx, n_parts, 4 * MCH);
  const int p0 = pid * part_size;
  if (p0 >= ctx) return;
  const int p1 = min(p0 + part_size, ctx);
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r = lane & 15;
  const int n_q_heads = n_kv_heads * G;
  char* vimg = vimg_all + wid * (MCH * D * 2);

  // Q^T as the B operand: lane (head r, group g), k-step s -> dims 8 dblk .. +8
  // with dblk = 4s + g (bf16: the 4 lanes of a K row read 64 contiguous bytes
  // per load) or 4g + s (fp8: a lane's 32 K bytes are contiguous)
  auto dblk = [&](int s) { return F8 ? 4 * g + s : 4 * s + g; };
  u32x4_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = u32x4_t{0u, 0u, 0u, 0u};
    if (r < G)
      qf[s] = *reinterpret_cast<const u32x4_t*>(q + (int64_t)b * q_stride + (int64_t)(kvh * G + r) * D + 8 * dblk(s));
  }
  // K A-operand rows: row block bb, lane row r -> token 8 (r >> 2) + 4 bb + (r & 3)
  int ktok[2];
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) ktok[bb] = 8 * (r >> 2) + 4 * bb + (r & 3);

  f32x4 oacc[8];
#pragma unroll
  for (int db = 0; db < 8; ++db) oacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_i = -1e30f, l_i = 0.f;

  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int64_t head_stride = (int64_t)block_size * D;
  const int n_chunks = (p1 - p0 + MCH - 1) / MCH;
  // element offsets of a chunk's two 16-token halves: one KV block when
  // block_size % 32 == 0, else (block size 16) two; a second half that starts
  // past the context reuses the first (its rows are masked)
  auto chunk_base = [&](int c, int64_t (&base)[2]) {
    const int cb = p0 + c * MCH;
    const int blk = bt[cb / block_size];
    base[0] = ((int64_t)blk * n_kv_heads + kvh) * head_stride + (int64_t)(cb % block_size) * D;
    if (block_size % MCH == 0 || cb + 16 >= p1) {
      base[1] = base[0] + (block_size % MCH == 0 ? 16 * D : 0);
    } else {
      const int blk2 = bt[(cb + 16) / block_size];
      base[1] = ((int64_t)blk2 * n_kv_heads + kvh) * head_stride + (int64_t)((cb + 16) % block_size) * D;
    }
  };
  // raw K / V registers: bf16 -- K 4 x 16 B (one per k-step) per row block, V
  // 8 loads of 4 full rows; fp8 -- K 2 x 16 B (two k-steps each), V 8 loads
  // of 8 B per lane (4 full 128-B rows), so each lane widens exactly the one
  // 16-B bf16 chunk the bf16 path stores (16-B fp8 loads, two chunks per
  // lane, made the image stores 17x more bank-conflicted:
  // profiles/r5_decode_pmc.txt)
  constexpr int KV = F8 ? 2 : 4, VL = 8;
  using VT = typename std::conditional<F8, u32x2_t, u32x4_t>::type;
  u32x4_t kf[2][KV] = {};
  VT vr[VL] = {};
  auto load16 = [&](const CT* p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p)); };
  auto load8 = [&](const CT* p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(p)); };
  auto load_k = [&](int c) {
    int64_t base[2];
    chunk_base(c, base);
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const int t = ktok[bb];  // 0..31: the half is t / 16 (lane-dependent)
      const int64_t row = (t < 16 ? base[0] : base[1]) + (int64_t)(t & 15) * D;
#pragma unroll
      for (int s2 = 0; s2 < KV; ++s2) {
        if constexpr (F8) kf[bb][s2] = load16(k_cache + row + 32 * g + 16 * s2);
        else kf[bb][s2] = ld16<NT>(k_cache + row + 8 * (4 * s2 + g));
      }
    }
  };
  auto load_v = [&](int c) {
    int64_t base[2];
    chunk_base(c, base);
#pragma unroll
    for (int k = 0; k < VL; ++k) {  // rows 4k + g: the first half for k < 4
      const int64_t row = base[k >> 2] + (int64_t)(4 * (k & 3) + g) * D;
      if constexpr (F8) vr[k] = load8(v_cache + row + 8 * r);
      else vr[k] = ld16<NT>(v_cache + row + 8 * r);
    }
  };
  auto kfrag = [&](int bb, int s2) -> bf16x8_t {  // A fragment of k-step s2
    if constexpr (F8) {
      const u32x4_t w = kf[bb][s2 >> 1];
      const u32x2_t h = (s2 & 1) ? u32x2_t{w[2], w[3]} : u32x2_t{w[0], w[1]};
      return __builtin_bit_cast(bf16x8_t, fp8x8_to_bf16(h));
    } else {
      return __builtin_bit_cast(bf16x8_t, kf[bb][s2]);
    }
  };

  int c = wid;
  if (c < n_chunks) {
    load_k(c);
    load_v(c);
  }
  for (; c < n_chunks; c += 4) {
    const bool more = c + 4 < n_chunks;  // wave-uniform
    const int cb = p0 + c * MCH;
    const bool partial = cb + MCH > p1;
    // S = K . Q^T, two 16-token row blocks
    f32x4 sacc[2];
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      sacc[bb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        sacc[bb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kfrag(bb, s2), __builtin_bit_cast(bf16x8_t, qf[s2]),
                                                           sacc[bb], 0, 0, 0);
    }
    if (more) load_k(c + 4);
    // V rows of this chunk -> the wave's LDS image (rows past the context zeroed:
    // their P is 0, but stale cache bytes may be NaN)
    if (partial) {
#pragma unroll
      for (int k = 0; k < VL; ++k)
        if (cb + 4 * k + g >= p1) vr[k] = VT{};  // e4m3 0x00 = +0
    }
#pragma unroll
    for (int k = 0; k < VL; ++k) {
      if constexpr (F8) {  // 8 fp8 dims -> the bf16 chunk r of row 4k + g
        *reinterpret_cast<u16x8*>(vimg + vimg_off(4 * k + g, r)) = fp8x8_to_bf16(vr[k]);
      } else {
        *reinterpret_cast<u32x4_t*>(vimg + vimg_off(4 * k + g, r)) = vr[k];
      }
    }
    if (more) load_v(c + 4);
    // softmax: lane (g, r) holds tokens 8g + j (j = 4 bb + i) of head r
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = sacc[j >> 2][j & 3] * scale_log2e;
    if (partial) {
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = cb + 8 * g + j >= p1 ? -INFINITY : t[j];
    }
    float cmax = fmaxf(fmaxf(fmaxf(t[0], t[1]), fmaxf(t[2], t[3])), fmaxf(fmaxf(t[4], t[5]), fmaxf(t[6], t[7])));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
    const float m_new = cmax > m_i + kRescale ? cmax : m_i;
    const float alpha = fast_exp2(m_i - m_new);
    m_i = m_new;
    u32x4_t pf;
    float ps = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t pk = pack_bf16x2(fast_exp2(t[2 * w] - m_new), fast_exp2(t[2 * w + 1] - m_new));
      pf[w] = pk;
      ps += bf16lo(pk) + bf16hi(pk);  // the row sum of exactly the bf16 P the product uses
    }
    l_i = l_i * alpha + ps;
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
      for (int db = 0; db < 8; ++db) oacc[db] *= alpha;
    }
    // O^T += V^T . P^T per 16-dim block; V^T fragment of lane 4q + p of group
    // g: rows 8g + q (elements 0-3) and 8g + 4 + q (4-7), columns 16 db + 4p ..
    const bf16x8_t pfrag = __builtin_bit_cast(bf16x8_t, pf);
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      const int qq = r >> 2, pp = r & 3;
      const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_i16x4_t*)(vimg + vimg_off(8 * g + qq, 2 * db + (pp >> 1)) + 8 * (pp & 1)));
      const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_i16x4_t*)(vimg + vimg_off(8 * g + 4 + qq, 2 * db + (pp >> 1)) + 8 * (pp & 1)));
      typedef short i16x8 __attribute__((ext_vector_type(8)));
      const i16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      oacc[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vv), pfrag, oacc[db], 0, 0, 0);
    }
  }

  // wave state -> LDS: lane (g, r < G) holds dims 16 db + 4 g + i of head r;
  // l is this lane's share of the head's row sum (its 8 tokens per chunk)
  float l_tot = l_i + __shfl_xor(l_i, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (r < G) {
#pragma unroll
    for (int db = 0; db < 8; ++db)
      *reinterpret_cast<f32x4*>(st_o + ((int64_t)wid * G + r) * D + 16 * db + 4 * g) = oacc[db];
    if (g == 0) {
      st_m[wid * G + r] = m_i;
      st_l[wid * G + r] = l_tot;
    }
  }
  __syncthreads();
  finish_workgroup<G>(st_o, st_m, st_l, out, tmp_out, tmp_ml, b, kvh, pid, n_parts, n_q_heads, out_scale);
}

// merge flash-decoding partitions: grid (Hq, B), block D threads
__global__ void __launch_bounds__(D) decode_reduce_kernel(bf16_t* __restrict__ out, const float* __restrict__ tmp_out,
                                                          const float* __restrict__ tmp_ml,
                                                          const int* __restrict__ ctx_lens, int n_parts, int align) {
  const int qh = blockIdx.x, b = blockIdx.y, nqh = gridDim.x;
  const int d = threadIdx.x;
  const int ctx = ctx_lens[b];
  if (ctx <= 0) {  // a graph bucket's padding row (context 0): no partition wrote it
    out[((int64_t)b * nqh + qh) * D + d] = 0;
    return;
  }
  const int part_size = balanced_part(ctx, n_parts, align);
  const int np = min((ctx + part_size - 1) / part_size, n_parts);
  const int64_t row0 = ((int64_t)b * nqh + qh) * n_parts;
  float M = -1e30f;
  for (int p = 0; p < np; ++p) M = fmaxf(M, tmp_ml[(row0 + p) * 2]);
  float num = 0.f, den = 0.f;
  for (int p = 0; p < np; ++p) {
    const float w = exp2f(tmp_ml[(row0 + p) * 2] - M) * tmp_ml[(row0 + p) * 2 + 1];
    num += w * tmp_out[(row0 + p) * D + d];
    den += w;
  }
  out[((int64_t)b * nqh + qh) * D + d] = f32_to_bf16(den > 0.f ? num / den : 0.f);
}

template <int G, int LPT, int CH, bool NT, bool F8>
int launch(bf16_t* out, float* tmp_out, float* tmp_ml, const bf16_t* q, int64_t q_stride, const void* kc,
           const void* vc, const int* bt, int bt_stride, const int* ctx, int batch, int n_kv_heads, int block_size,
           int n_parts, float scale, float out_scale, hipStream_t st) {
  using C = Cfg<G, LPT, CH>;
  if (block_size % CH || n_parts < 1) return -1;
  size_t lds = (size_t)C::SRC * G * D * 4 + 2 * C::SRC * G * 4;
  static bool attr_set = false;  // > 64 KiB dynamic LDS needs an explicit opt-in
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)decode_attn_kernel<G, LPT, CH, NT, F8>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  dim3 grid(n_parts, n_kv_heads, batch);
  decode_attn_kernel<G, LPT, CH, NT, F8><<<grid, kThreads, lds, st>>>(out, tmp_out, tmp_ml, q, q_stride, kc, vc, bt,
                                                                     bt_stride, ctx, n_kv_heads, block_size,
                                                                     scale * 1.4426950408889634f, out_scale);
  if (n_parts > 1) {
    dim3 g2(n_kv_heads * G, batch);
    decode_reduce_kernel<<<g2, D, 0, st>>>(out, tmp_out, tmp_ml, ctx, n_parts, 4 * CH);
  }
  return (int)hipGetLastError();
}

template <int G, bool NT, bool F8>
int launch_mfma(bf16_t* out, float* tmp_out, float* tmp_ml, const bf16_t* q, int64_t q_stride, const void* kc,
                const void* vc, const int* bt, int bt_stride, const int* ctx, int batch, int n_kv_heads, int block_size,
                int n_parts, float scale, float out_scale, hipStream_t st) {
  if (block_size % 16 || n_parts < 1) return -1;
  dim3 grid(n_parts, n_kv_heads, batch);
  decode_attn_mfma_kernel<G, NT, F8><<<grid, kThreads, 0, st>>>(out, tmp_out, tmp_ml, q, q_stride, kc, vc, bt,
                                                                bt_stride, ctx, n_kv_heads, block_size,
                                                                scale * 1.4426950408889634f, out_scale);
  if (n_parts > 1) {
    dim3 g2(n_kv_heads * G, batch);
    decode_reduce_kernel<<<g2, D, 0, st>>>(out, tmp_out, tmp_ml, ctx, n_parts, 4 * MCH);
  }
  return (int)hipGetLastError();
}

}  // namespace

// q: [B, Hq, D] rows with stride q_stride (elements) between sequences.
// tmp_out: [B, Hq, n_parts, D] f32, tmp_ml: [B, Hq, n_parts, 2] f32 (only
// touched when n_parts > 1).  block_size must be a multiple of 16 (32 for the
// 32-token-chunk variants).
extern "C" int dx_decode_attention(void* out, float* tmp_out, float* tmp_ml, const void* q, int64_t q_stride,
                                   const void* k_cache, const void* v_cache, const int* block_tables, int bt_stride,
                                   const int* ctx_lens, int batch, int n_q_heads, int n_kv_heads, int head_dim,
                                   int block_size, int n_parts, float scale, int kv_fp8, float k_scale, float v_scale,
                                   hipStream_t stream) {
  if (head_dim != D || block_size % kChunk || n_parts < 1 || n_q_heads % n_kv_heads) return -1;
  if (batch == 0) return 0;
  const int G = n_q_heads / n_kv_heads;
  auto o = (bf16_t*)out;
  auto qq = (const bf16_t*)q;
  // 16-token chunks, non-temporal K/V loads (32-token chunks and temporal
  // loads measured no better: r1 decode studies in profiles/); FP8 caches: the
  // K scale folds into the softmax scale, the V scale into the output; fp8
  // chunk: 16 tokens with two chunks in flight per wave (164 VGPRs, 3
  // waves/SIMD at G 4; a 32-token variant measured no better,
  // profiles/r3_kv_fp8.txt, and was removed in round 4)
#define DX_DEC(GG, LL, L8)                                                                                         \
  return kv_fp8 ? launch<GG, L8, 16, true, true>(o, tmp_out, tmp_ml, qq, q_stride, k_cache, v_cache, block_tables, \
                                                 bt_stride, ctx_lens, batch, n_kv_heads, block_size, n_parts,      \
                                                 scale * k_scale, v_scale, stream)                                 \
                : launch<GG, LL, 16, true, false>(o, tmp_out, tmp_ml, qq, q_stride, k_cache, v_cache, block_tables, \
                                                  bt_stride, ctx_lens, batch, n_kv_heads, block_size, n_parts,     \
                                                  scale, 1.f, stream);
  // the MFMA kernel for 1-16 query heads per KV head (the heads are the 16
  // MFMA columns; DX_DECODE_MFMA=0 selects the VALU kernel, read per call so
  // a test can compare both)
  const char* mf = getenv("DX_DECODE_MFMA");
  if ((G == 1 || G == 2 || G == 4 || G == 8 || G == 16) && block_size % 16 == 0 && !(mf && mf[0] == '0')) {
    const float sc = kv_fp8 ? scale * k_scale : scale, osc = kv_fp8 ? v_scale : 1.f;
#define DX_MF(GG)                                                                                                 \
  return kv_fp8 ? launch_mfma<GG, true, true>(o, tmp_out, tmp_ml, qq, q_stride, k_cache, v_cache, block_tables,  \
                                             bt_stride, ctx_lens, batch, n_kv_heads, block_size, n_parts, sc, osc, \
                                             stream)                                                              \
                : launch_mfma<GG, true, false>(o, tmp_out, tmp_ml, qq, q_stride, k_cache, v_cache, block_tables, \
                                              bt_stride, ctx_lens, batch, n_kv_heads, block_size, n_parts, sc,    \
                                              osc, stream);
    switch (G) {
      case 1: DX_MF(1)
      case 2: DX_MF(2)
      case 4: DX_MF(4)
      case 8: DX_MF(8)
      default: DX_MF(16)
    }
#undef DX_MF
  }
  switch (G) {
    case 1: DX_DEC(1, 4, 4)
    case 2: DX_DEC(2, 8, 8)
    case 4: DX_DEC(4, 16, 8)  // fp8: 8 lanes x 16 dims per row, one 16-B load per row per lane
    case 8: DX_DEC(8, 16, 8)
    default: return -2;
  }
#undef DX_DEC
}
