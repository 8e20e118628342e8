// HBM read-bandwidth probe for gfx950: every lane streams 16-B vectors
// (optionally non-temporal) over a 4 GiB buffer, grid-stride, XOR-reduced so the
// loads are not dead.  Prints GB/s per configuration (workgroups per CU x
// loads in flight per lane).  Build: hipcc --offload-arch=gfx950 -O3 -o hbm_probe hbm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) rd(const u32x4* __restrict__ p, size_t n, unsigned* out) {
  u32x4 acc = {0, 0, 0, 0};
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t i = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; i < n; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t j = i + (size_t)u * blockDim.x;
      v[u] = j < n ? (NT ? __builtin_nontemporal_load(p + j) : p[j]) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[0] = 1;  // practically never
}

template <int U, bool NT>
double run(const u32x4* p, size_t n, unsigned* out, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  rd<U, NT><<<blocks, 256>>>(p, n, out);
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) rd<U, NT><<<blocks, 256>>>(p, n, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return (double)n * 16 * reps / (ms * 1e-3) / 1e9;
}

int main() {
  const size_t bytes = 4ull << 30, n = bytes / 16;
  u32x4* p;
  unsigned* out;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  hipMemset(p, 1, bytes);
  hipDeviceSynchronize();
  for (int wpc : {4, 8, 16}) {
    const int blocks = 256 * wpc;
    printf("wg/CU %2d: U1 %.0f  U4 %.0f  U8 %.0f  U8-nt %.0f GB/s\n", wpc, run<1, false>(p, n, out, blocks),
           run<4, false>(p, n, out, blocks), run<8, false>(p, n, out, blocks), run<8, true>(p, n, out, blocks));
  }
  // short kernels (decode-GEMM sized): one launch per `sz` bytes, rotating over
  // the 4 GiB so every launch reads cold data (beyond the 256 MB Infinity Cache)
  for (size_t sz : {16ull << 20, 32ull << 20, 64ull << 20, 128ull << 20, 256ull << 20}) {
    const size_t m = sz / 16, nb = bytes / sz;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (size_t i = 0; i < nb; ++i) rd<8, true><<<1024, 256>>>(p + i * m, m, out);
    (void)hipEventRecord(a);
    for (size_t i = 0; i < nb; ++i) rd<8, true><<<1024, 256>>>(p + i * m, m, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%4zu MB per launch: %.1f us/launch, %.0f GB/s\n", sz >> 20, ms * 1e3 / nb, (double)bytes / (ms * 1e-3) / 1e9);
  }
  hipFree(p);
  hipFree(out);
  return 0;
}
