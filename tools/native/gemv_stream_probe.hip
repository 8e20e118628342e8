// Decode-GEMM weight-stream probe (gfx950): how fast can a grid stream an
// [N][K] bf16 weight matrix when every wave reads 16-row x K slabs in the
// MFMA A-fragment layout (lane l: row l & 15, 16 B at k-group l >> 4), as a
// decode projection kernel would -- no x, no MFMA, loads XOR-reduced so they
// are not dead.  Sweeps the workgroups per launch (work split into row tiles
// x K-slices), waves per workgroup and loads in flight per wave, over the
// projection shapes of Llama-3-8B (TP1) with cold weights (each launch reads
// another copy; 2+ GB rotation >> the 256 MB Infinity Cache).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o gemv_stream_probe gemv_stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// one workgroup = NW waves x 16 rows (a 16*NW-row tile) x one K-slice of kslice
// elements; U loads (1 KB per wave each) issued back to back, then consumed
template <int NW, int U>
__global__ void __launch_bounds__(64 * NW) slab_stream(const unsigned short* __restrict__ w, int N, int K, int splits,
                                                       unsigned* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles = N / (16 * NW);
  const int tile = blockIdx.x % tiles, sl = blockIdx.x / tiles;
  const int kslice = K / splits;
  const int row = tile * 16 * NW + wave * 16 + (lane & 15);
  const char* base = reinterpret_cast<const char*>(w) + ((size_t)row * K + (size_t)sl * kslice) * 2 + 16 * (lane >> 4);
  const int steps = kslice / 32;  // 64 B per row per load
  u32x4 acc = {0, 0, 0, 0};
  for (int t = 0; t < steps; t += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = (t + u < steps) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)(t + u) * 64))
                             : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = 1;
}

template <int NW, int U>
float time_cfg(const unsigned short* w, size_t copy_elems, int copies, int N, int K, int splits, unsigned* out) {
  const int tiles = N / (16 * NW);
  const int grid = tiles * splits;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int c = 0; c < copies; ++c) slab_stream<NW, U><<<grid, 64 * NW>>>(w + c * copy_elems, N, K, splits, out);
  hipEventRecord(a);
  const int reps = 2;
  for (int r = 0; r < reps; ++r)
    for (int c = 0; c < copies; ++c) slab_stream<NW, U><<<grid, 64 * NW>>>(w + c * copy_elems, N, K, splits, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / (reps * copies);
}

struct Shape {
  const char* name;
  int N, K;
};

template <int NW, int U>
void sweep(const Shape& s, const unsigned short* w, size_t pool_elems, unsigned* out) {
  const size_t elems = (size_t)s.N * s.K;
  const int copies = (int)std::min<size_t>(32, pool_elems / elems);
  const int tiles = s.N / (16 * NW);
  for (int splits : {1, 2, 4, 8, 16}) {
    if (s.K % (32 * splits) || (s.K / splits) / 32 < U) continue;
    const int grid = tiles * splits;
    if (grid < 64 || grid > 4096) continue;
    const float us = time_cfg<NW, U>(w, elems, copies, s.N, s.K, splits, out);
    printf("%-8s nw %d U %2d splits %2d grid %5d: %7.1f us  %5.2f TB/s  (%4.0f KB/WG, %3.0f KB in flight/WG)\n",
           s.name, NW, U, splits, grid, us, elems * 2 / (us * 1e-6) / 1e12, elems * 2.0 / grid / 1024, NW * U * 1.0);
  }
}

int main() {
  const size_t pool_bytes = 3ull << 30, pool_elems = pool_bytes / 2;
  unsigned short* w;
  unsigned* out;
  if (hipMalloc(&w, pool_bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  hipMemset(w, 1, pool_bytes);
  hipDeviceSynchronize();
  const Shape shapes[] = {{"o", 4096, 4096}, {"qkv", 6144, 4096}, {"down", 4096, 14336}, {"gate_up", 28672, 4096}};
  for (const Shape& s : shapes) {
    sweep<4, 8>(s, w, pool_elems, out);
    sweep<4, 16>(s, w, pool_elems, out);
    sweep<4, 32>(s, w, pool_elems, out);
    sweep<8, 8>(s, w, pool_elems, out);
    sweep<8, 16>(s, w, pool_elems, out);
    sweep<16, 8>(s, w, pool_elems, out);
    sweep<16, 16>(s, w, pool_elems, out);
    fflush(stdout);
  }
  hipFree(w);
  hipFree(out);
  return 0;
}
