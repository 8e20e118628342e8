// pybind11 entry points for the gfx950 kernels.  Every function takes raw
// device pointers (uintptr_t, from torch.Tensor.data_ptr()) and the HIP stream
// handle (torch.cuda.current_stream().cuda_stream), so launches are
// graph-capturable and independent of the torch C++ ABI.  Shape/dtype checks
// live in dynamo_exp_amd/ops/kernels.py; the C launchers re-check the kernel
// preconditions and return a nonzero code on violation, which is raised here.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <unistd.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;
using u = uintptr_t;

extern "C" {
int dx_rmsnorm(void*, const void*, const void*, int, int, int64_t, int64_t, float, hipStream_t);
int dx_add_rmsnorm(void*, const void*, void*, const void*, int, int, int64_t, int64_t, int64_t, float, hipStream_t);
int dx_rope_cache(void*, int64_t, const void*, int, const float*, const int64_t*, void*, void*, int, int, int, int,
                  int, int, int, float, float, const float*, int, int, hipStream_t, const float*);
int dx_kv_dequant(const void*, const void*, void*, void*, const int*, int, const int*, const int*, int, int, int, int,
                  int, float, float, hipStream_t);
int dx_kv_write(const void*, const void*, int64_t, const int64_t*, void*, void*, int, int, int, int, hipStream_t);
int dx_silu_and_mul(void*, const void*, int, int, int64_t, int64_t, int, hipStream_t);
int dx_gemm256(void*, int64_t, const void*, int64_t, const void*, int, int, int, int, int, hipStream_t, const float*);
int dx_row_rrms(float*, const void*, int, int, int64_t, float, hipStream_t);
int dx_embedding(void*, const void*, const void*, int, int, int, int64_t, hipStream_t);
int dx_decode_attention(void*, float*, float*, const void*, int64_t, const void*, const void*, const int*, int,
                        const int*, int, int, int, int, int, int, float, int, float, float, hipStream_t);
int dx_prefill_attention(void*, const void*, int64_t, const void*, const void*, const int*, int, const int*,
                         const int*, const int*, int, int, int, int, int, float, int, int, hipStream_t);
int dx_prefill_tile_tokens(int, int, int);
int dx_rmsnorm_quant(void*, float*, const void*, void*, const void*, int, int, int64_t, int64_t, float, hipStream_t);
int dx_decode_advance(void*, void*, void*, void*, void*, const void*, const void*, void*, void*, const int*, int, int,
                      int, int, int, hipStream_t);
int dx_silu_mul_quant(void*, float*, const void*, int, int, int64_t, hipStream_t);
int dx_quant_rows(void*, float*, const void*, int, int, int64_t, hipStream_t);
int dx_custom_ar(void*, const void* const*, void* const*, int, int, int64_t, uint32_t, int, int*, int, hipStream_t);
int dx_custom_ar_alloc_signals(void**);
int dx_custom_ag(void*, const void* const*, void* const*, int, int, int64_t, int, int*, uint32_t, hipStream_t);
int dx_skinny_gemm(void*, int64_t, const void*, int64_t, const void*, float*, int*, int, int, int, int, int, int,
                   hipStream_t);
int dx_dstream_gemm(void*, int64_t, const void*, int64_t, const void*, float*, int*, int, int, int, int, int, int, int,
                    int, int, int, hipStream_t);
int dx_splitk_reduce(void*, int64_t, const float*, int, int, int, int, hipStream_t);
int dx_add_rmsnorm_slabs(void*, const float*, int, int, void*, const void*, int, int, int64_t, int64_t, float,
                         hipStream_t);
int dx_dstream_probe(void*, int64_t, const void*, int64_t, const void*, float*, int*, int, int, int, int, int,
                     hipStream_t);
int dx_sample(int64_t*, float*, const void*, int, int64_t, int, int, const float*, const int*, const float*,
              const float*, const int64_t*, const int64_t*, hipStream_t);
int dx_apply_penalties(void*, int, int64_t, int, const int*, const int*, const int*, const int*, const float*,
                       const float*, const float*, hipStream_t);
int dx_sample_partial(float*, const void*, int, int64_t, int, int, int, const float*, const int64_t*, const int64_t*,
                      hipStream_t);
int dx_kv_copy_blocks(void*, const void*, const int*, const int*, int, int, int64_t, int64_t, int64_t, int64_t,
                      int64_t, int64_t, int64_t, hipStream_t);
int dx_spin_for(uint32_t, uint32_t*, hipStream_t);
int dx_wire_xfer(int, uint32_t*, void*, void*, int64_t, uint32_t, uint32_t, int*, hipStream_t);
int dx_wire_alloc(void**, int64_t);
}

static void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string(what) + " failed with code " + std::to_string(rc));
}

#define P(x) reinterpret_cast<void*>(x)
#define S(x) reinterpret_cast<hipStream_t>(x)

PYBIND11_MODULE(_C_kernels, m) {
  m.doc() = "dynamo_exp_amd gfx950 HIP kernels";
  m.attr("arch") = "gfx950";

  m.def("rmsnorm", [](u out, u x, u w, int rows, int hidden, int64_t xs, int64_t os, float eps, u st) {
    check(dx_rmsnorm(P(out), P(x), P(w), rows, hidden, xs, os, eps, S(st)), "rmsnorm");
  });
  m.def("add_rmsnorm", [](u out, u x, u res, u w, int rows, int hidden, int64_t xs, int64_t os, int64_t rs,
                          float eps, u st) {
    check(dx_add_rmsnorm(P(out), P(x), P(res), P(w), rows, hidden, xs, os, rs, eps, S(st)), "add_rmsnorm");
  });
  m.def("rope_cache", [](u qkv, int64_t qkv_stride, u pos, int pos_i64, u cos_sin, u slots, u kc, u vc, int tokens,
                         int hq, int hkv, int hd, int bs, int rotate_q, int kv_fp8, float ks, float vs, u slabs,
                         int splits, int slab_bm, u st, u row_scale) {
    check(dx_rope_cache(P(qkv), qkv_stride, P(pos), pos_i64, (const float*)cos_sin, (const int64_t*)slots, P(kc),
                        P(vc), tokens, hq, hkv, hd, bs, rotate_q, kv_fp8, ks, vs, (const float*)slabs, splits, slab_bm,
                        S(st), (const float*)row_scale),
          "rope_cache");
  });
  m.def("row_rrms", [](u out, u x, int rows, int hidden, int64_t xs, float eps, u st) {
    check(dx_row_rrms((float*)out, P(x), rows, hidden, xs, eps, S(st)), "row_rrms");
  });
  m.def("kv_dequant", [](u k8, u v8, u ks, u vs, u bt, int bts, u ctx, u dst, int n_seqs, int max_blocks, int hkv,
                         int bs, int hd, float k_scale, float v_scale, u st) {
    check(dx_kv_dequant(P(k8), P(v8), P(ks), P(vs), (const int*)bt, bts, (const int*)ctx, (const int*)dst, n_seqs,
                        max_blocks, hkv, bs, hd, k_scale, v_scale, S(st)),
          "kv_dequant");
  });
  m.def("kv_write", [](u k, u v, int64_t stride, u slots, u kc, u vc, int tokens, int hkv, int hd, int bs, u st) {
    check(dx_kv_write(P(k), P(v), stride, (const int64_t*)slots, P(kc), P(vc), tokens, hkv, hd, bs, S(st)),
          "kv_write");
  });
  m.def("silu_and_mul", [](u out, u gu, int tokens, int ffn, int64_t is, int64_t os, int blk, u st) {
    check(dx_silu_and_mul(P(out), P(gu), tokens, ffn, is, os, blk, S(st)), "silu_and_mul");
  });
  m.def("embedding", [](u out, u table, u ids, int ids_i64, int tokens, int hidden, int64_t vocab, u st) {
    check(dx_embedding(P(out), P(table), P(ids), ids_i64, tokens, hidden, vocab, S(st)), "embedding");
  });
  m.def("decode_attention", [](u out, u tmp_out, u tmp_ml, u q, int64_t qs, u kc, u vc, u bt, int bts, u ctx,
                               int batch, int hq, int hkv, int hd, int bs, int n_parts, float scale, int kv_fp8,
                               float k_scale, float v_scale, u st) {
    check(dx_decode_attention(P(out), (float*)tmp_out, (float*)tmp_ml, P(q), qs, P(kc), P(vc), (const int*)bt, bts,
                              (const int*)ctx, batch, hq, hkv, hd, bs, n_parts, scale, kv_fp8, k_scale, v_scale,
                              S(st)),
          "decode_attention");
  });
  m.def("prefill_attention", [](u out, u q, int64_t qs, u kc, u vc, u bt, int bts, u cu, u ctx, u work, int n_work,
                                int hq, int hkv, int hd, int bs, float scale, int causal, int waves, u st) {
    check(dx_prefill_attention(P(out), P(q), qs, P(kc), P(vc), (const int*)bt, bts, (const int*)cu,
                               (const int*)ctx, (const int*)work, n_work, hq, hkv, hd, bs, scale, causal, waves,
                               S(st)),
          "prefill_attention");
  });
  m.def("prefill_tile_tokens", &dx_prefill_tile_tokens);
  m.def("gemm256", [](u y, int64_t ldy, u x, int64_t ldx, u w, int M, int N, int K, int epi, int gm, u st, u rs) {
    check(dx_gemm256(P(y), ldy, P(x), ldx, P(w), M, N, K, epi, gm, S(st), (const float*)rs), "gemm256");
  });
  m.def("skinny_gemm", [](u y, int64_t ys, u x, int64_t xs, u w, u slabs, u tickets, int M, int N, int K, int bn,
                          int bm, int splits, u st) {
    check(dx_skinny_gemm(P(y), ys, P(x), xs, P(w), (float*)slabs, (int*)tickets, M, N, K, bn, bm, splits, S(st)),
          "skinny_gemm");
  });
  m.def("dstream_gemm", [](u y, int64_t ldy, u x, int64_t ldx, u w, u slabs, u tickets, int M, int N, int K, int nw,
                           int r, int t, int dw, int dx, int splits, int flags, u st) {
    check(dx_dstream_gemm(P(y), ldy, P(x), ldx, P(w), (float*)slabs, (int*)tickets, M, N, K, nw, r, t, dw, dx, splits,
                          flags, S(st)),
          "dstream_gemm");
  });
  m.def("splitk_reduce", [](u y, int64_t ldy, u slabs, int M, int N, int BM, int splits, u st) {
    check(dx_splitk_reduce(P(y), ldy, (const float*)slabs, M, N, BM, splits, S(st)), "splitk_reduce");
  });
  m.def("add_rmsnorm_slabs", [](u out, u slabs, int splits, int BM, u res, u w, int rows, int hidden, int64_t os,
                                int64_t rs, float eps, u st) {
    check(dx_add_rmsnorm_slabs(P(out), (const float*)slabs, splits, BM, P(res), P(w), rows, hidden, os, rs, eps, S(st)),
          "add_rmsnorm_slabs");
  });
  m.def("dstream_probe", [](u y, int64_t ldy, u x, int64_t ldx, u w, u slabs, u tickets, int M, int N, int K,
                            int splits, int probe, u st) {
    check(dx_dstream_probe(P(y), ldy, P(x), ldx, P(w), (float*)slabs, (int*)tickets, M, N, K, splits, probe, S(st)),
          "dstream_probe");
  });
  // fp8 (e4m3fn) w8a8 path: per-row dynamic quantisation fused into the producers
  m.def("rmsnorm_quant", [](u out, u scale, u x, u res, u w, int rows, int hidden, int64_t xs, int64_t rs, float eps,
                            u st) {
    check(dx_rmsnorm_quant(P(out), (float*)scale, P(x), P(res), P(w), rows, hidden, xs, rs, eps, S(st)),
          "rmsnorm_quant");
  });
  m.def("decode_advance", [](u ids, u pos, u slots, u ctx, u offs, u out_tok, u out_lp, u res_tok, u res_lp, u bt,
                             int bts, int bs, int n_real, int step, int advance, u st) {
    check(dx_decode_advance(P(ids), P(pos), P(slots), P(ctx), P(offs), P(out_tok), P(out_lp), P(res_tok), P(res_lp),
                            (const int*)bt, bts, bs, n_real, step, advance, S(st)),
          "decode_advance");
  });
  m.def("silu_mul_quant", [](u out, u scale, u gu, int rows, int ffn, int64_t is, u st) {
    check(dx_silu_mul_quant(P(out), (float*)scale, P(gu), rows, ffn, is, S(st)), "silu_mul_quant");
  });
  m.def("quant_rows", [](u out, u scale, u x, int rows, int cols, int64_t xs, u st) {
    check(dx_quant_rows(P(out), (float*)scale, P(x), rows, cols, xs, S(st)), "quant_rows");
  });
  m.def("sample", [](u out_tok, u out_lp, u logits, int f32, int64_t stride, int rows, int vocab, u temp, u topk,
                     u topp, u minp, u seeds, u offs, u st) {
    check(dx_sample((int64_t*)out_tok, (float*)out_lp, P(logits), f32, stride, rows, vocab, (const float*)temp,
                    (const int*)topk, (const float*)topp, (const float*)minp, (const int64_t*)seeds,
                    (const int64_t*)offs, S(st)),
          "sample");
  });
  m.def("sample_partial", [](u out, u logits, int f32, int64_t stride, int rows, int vocab, int v0, u temp, u seeds,
                             u offs, u st) {
    check(dx_sample_partial((float*)out, P(logits), f32, stride, rows, vocab, v0, (const float*)temp,
                            (const int64_t*)seeds, (const int64_t*)offs, S(st)),
          "sample_partial");
  });
  m.def("apply_penalties", [](u logits, int f32, int64_t stride, int rows, u csr, u toks, u counts, u flags, u rep,
                              u freq, u pres, u st) {
    check(dx_apply_penalties(P(logits), f32, stride, rows, (const int*)csr, (const int*)toks, (const int*)counts,
                             (const int*)flags, (const float*)rep, (const float*)freq, (const float*)pres, S(st)),
          "apply_penalties");
  });
  m.def("kv_copy_blocks", [](u dst, u src, u src_ids, u dst_ids, int n_pairs, int n_prefix, int64_t sps, int64_t dps,
                             int64_t sbb, int64_t dbb, int64_t sio, int64_t dio, int64_t nbytes, u st) {
    check(dx_kv_copy_blocks(P(dst), P(src), (const int*)src_ids, (const int*)dst_ids, n_pairs, n_prefix, sps, dps,
                            sbb, dbb, sio, dio, nbytes, S(st)),
          "kv_copy_blocks");
  });
  // host-pinned memory for the KV offload tier (hipHostMalloc, mapped + coherent
  // off: written by the GPU copy engine / kernels, read back after stream sync)
  m.def("custom_ar", [](u out, std::vector<u> bufs, std::vector<u> sigs, int rank, int world, int64_t n,
                        uint32_t timeout_ms, int blocks, u err, int two_shot, u st) {
    std::vector<const void*> b(bufs.size());
    std::vector<void*> sg(sigs.size());
    for (size_t i = 0; i < bufs.size(); ++i) b[i] = P(bufs[i]);
    for (size_t i = 0; i < sigs.size(); ++i) sg[i] = P(sigs[i]);
    if ((int)b.size() != world || (int)sg.size() != world) throw std::runtime_error("custom_ar: world mismatch");
    check(dx_custom_ar(P(out), b.data(), sg.data(), rank, world, n, timeout_ms, blocks, (int*)err, two_shot, S(st)),
          "custom_ar");
  });
  m.def("custom_ag", [](u out, std::vector<u> bufs, std::vector<u> sigs, int rank, int world, int64_t nbytes,
                        int blocks, u err, uint32_t timeout_ms, u st) {
    std::vector<const void*> b(bufs.size());
    std::vector<void*> sg(sigs.size());
    for (size_t i = 0; i < bufs.size(); ++i) b[i] = P(bufs[i]);
    for (size_t i = 0; i < sigs.size(); ++i) sg[i] = P(sigs[i]);
    if ((int)b.size() != world || (int)sg.size() != world) throw std::runtime_error("custom_ag: world mismatch");
    check(dx_custom_ag(P(out), b.data(), sg.data(), rank, world, nbytes, blocks, (int*)err, timeout_ms, S(st)),
          "custom_ag");
  });
  m.def("custom_ar_alloc_signals", []() {
    void* p = nullptr;
    if (dx_custom_ar_alloc_signals(&p) != 0) throw std::runtime_error("custom_ar signal alloc failed");
    return reinterpret_cast<u>(p);
  });
  m.def("device_free", [](u p) { (void)hipFree(P(p)); });
  m.def("ipc_get_handle", [](u p) {
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, P(p)) != hipSuccess) throw std::runtime_error("hipIpcGetMemHandle failed");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  });
  m.def("ipc_open_handle", [](py::bytes hb) {
    std::string s = hb;
    hipIpcMemHandle_t h;
    if (s.size() != sizeof(h)) throw std::runtime_error("bad IPC handle size");
    memcpy(&h, s.data(), sizeof(h));
    void* p = nullptr;
    hipError_t e;
    {
      // the import can take long (it waits on the exporting process's
      // runtime): other Python threads keep running meanwhile
      py::gil_scoped_release nogil;
      e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    }
    if (e != hipSuccess) throw std::runtime_error("hipIpcOpenMemHandle failed");
    return reinterpret_cast<u>(p);
  });
  m.def("ipc_close_handle", [](u p) { (void)hipIpcCloseMemHandle(P(p)); });
  // (allocation base, offset of p in it): an IPC handle names a whole
  // allocation, so a buffer carved out of a caching-allocator segment is
  // shared as (handle of the base, offset)
  m.def("alloc_base_offset", [](u p) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(P(p))) != hipSuccess)
      throw std::runtime_error("hipMemGetAddressRange failed");
    const u b = reinterpret_cast<u>(base);
    return py::make_tuple(b, p - b);
  });
  // ---- chunked VMM allocations shared as dma-buf fds (one-sided KV transport).
  // hipIpcOpenMemHandle of a single allocation larger than ~1 GiB never
  // returns on this stack (profiles/r6_ipc_probe*.json), and a KV cache is
  // tens to hundreds of GiB: it is reserved as ONE virtual range backed by
  // `chunk`-byte physical allocations, each exportable as a POSIX fd; the
  // owner hands the fds to a peer process over a Unix socket (SCM_RIGHTS,
  // disagg/kv_share.py) and the peer maps the same chunks, in order, into a
  // range of its own.
  m.def("vmm_alloc", [](size_t nbytes, size_t chunk, int device) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    size_t gran = 0;
    check(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) == hipSuccess ? 0 : 1,
          "hipMemGetAllocationGranularity");
    chunk = (chunk + gran - 1) / gran * gran;
    const size_t total = (nbytes + chunk - 1) / chunk * chunk;
    void* va = nullptr;
    check(hipMemAddressReserve(&va, total, gran, nullptr, 0) == hipSuccess ? 0 : 1, "hipMemAddressReserve");
    std::vector<u> hs;
    for (size_t off = 0; off < total; off += chunk) {
      hipMemGenericAllocationHandle_t h;
      check(hipMemCreate(&h, chunk, &prop, 0) == hipSuccess ? 0 : 1, "hipMemCreate");
      check(hipMemMap(static_cast<char*>(va) + off, chunk, 0, h, 0) == hipSuccess ? 0 : 1, "hipMemMap");
      hs.push_back(reinterpret_cast<u>(h));
    }
    hipMemAccessDesc d = {};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    check(hipMemSetAccess(va, total, &d, 1) == hipSuccess ? 0 : 1, "hipMemSetAccess");
    return py::make_tuple(reinterpret_cast<u>(va), total, chunk, hs);
  });
  m.def("vmm_export_fds", [](const std::vector<u>& hs) {
    std::vector<int> fds;
    for (u h : hs) {
      int fd = -1;
      check(hipMemExportToShareableHandle(&fd, reinterpret_cast<hipMemGenericAllocationHandle_t>(h),
                                          hipMemHandleTypePosixFileDescriptor, 0) == hipSuccess ? 0 : 1,
            "hipMemExportToShareableHandle");
      fds.push_back(fd);
    }
    return fds;
  });
  // import: `fds` were received by THIS process; each is closed once mapped
  // (the mapping keeps the memory alive)
  m.def("vmm_import", [](const std::vector<int>& fds, size_t chunk, int device) {
    const size_t total = chunk * fds.size();
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    check(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) == hipSuccess ? 0 : 1,
          "hipMemGetAllocationGranularity");
    void* va = nullptr;
    check(hipMemAddressReserve(&va, total, gran, nullptr, 0) == hipSuccess ? 0 : 1, "hipMemAddressReserve");
    std::vector<u> hs;
    size_t off = 0;
    for (int fd : fds) {
      hipMemGenericAllocationHandle_t h;
      // this runtime reads the fd through the pointer (passing the fd value
      // itself, the other API family's convention, faults in the import)
      int fdv = fd;
      check(hipMemImportFromShareableHandle(&h, &fdv, hipMemHandleTypePosixFileDescriptor) == hipSuccess ? 0 : 1,
            "hipMemImportFromShareableHandle");
      check(hipMemMap(static_cast<char*>(va) + off, chunk, 0, h, 0) == hipSuccess ? 0 : 1, "hipMemMap (import)");
      hs.push_back(reinterpret_cast<u>(h));
      close(fd);
      off += chunk;
    }
    hipMemAccessDesc d = {};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    check(hipMemSetAccess(va, total, &d, 1) == hipSuccess ? 0 : 1, "hipMemSetAccess (import)");
    return py::make_tuple(reinterpret_cast<u>(va), total, hs);
  });
  m.def("vmm_free", [](u va, size_t total, const std::vector<u>& hs) {
    (void)hipMemUnmap(P(va), total);
    for (u h : hs) (void)hipMemRelease(reinterpret_cast<hipMemGenericAllocationHandle_t>(h));
    (void)hipMemAddressFree(P(va), total);
  });
  m.def("close_fd", [](int fd) { close(fd); });
  m.def("host_alloc_pinned", [](size_t nbytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, nbytes, hipHostMallocMapped | hipHostMallocNonCoherent) != hipSuccess)
      throw std::runtime_error("hipHostMalloc failed");
    return reinterpret_cast<u>(p);
  });
  m.def("host_free_pinned", [](u p) { (void)hipHostFree(P(p)); });
  m.def("device_pointer_of_host", [](u p) {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, P(p), 0) != hipSuccess) throw std::runtime_error("hipHostGetDevicePointer failed");
    return reinterpret_cast<u>(d);
  });
  // --- wire stand-ins and stream placement (tests / probes of the P->D data plane, wire_standin.hip)
  m.def("spin_for", [](uint32_t ms, u done, u st) { check(dx_spin_for(ms, (uint32_t*)done, S(st)), "spin_for"); });
  m.def("wire_xfer", [](int send, u state, u wire, u buf, int64_t nbytes, uint32_t k, uint32_t timeout_ms, u err,
                        u st) {
    check(dx_wire_xfer(send, (uint32_t*)state, P(wire), P(buf), nbytes, k, timeout_ms, (int*)err, S(st)),
          "wire_xfer");
  });
  m.def("wire_alloc", [](int64_t nbytes) {
    void* p = nullptr;
    check(dx_wire_alloc(&p, nbytes), "wire_alloc");
    return reinterpret_cast<u>(p);
  });
  // a stream with an explicit priority (lower = higher priority), or with a
  // full CU mask (cu_mask=1): HIP gives a CU-masked stream a hardware queue
  // of its own instead of a shared one from the pool
  m.def("stream_create", [](int priority, int cu_mask) {
    hipStream_t s = nullptr;
    if (cu_mask) {
      int dev = 0, n = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      std::vector<uint32_t> mask((n + 31) / 32, 0xffffffffu);
      if (n % 32) mask.back() = (1u << (n % 32)) - 1u;
      check(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) == hipSuccess ? 0 : 1,
            "hipExtStreamCreateWithCUMask");
    } else {
      check(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority) == hipSuccess ? 0 : 1,
            "hipStreamCreateWithPriority");
    }
    return reinterpret_cast<u>(s);
  });
  m.def("device_read_i32", [](u p) {
    int32_t v = 0;
    check(hipMemcpy(&v, P(p), 4, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1, "device_read_i32");
    return v;
  });
  m.def("stream_destroy", [](u s) { (void)hipStreamDestroy(S(s)); });
  m.def("stream_priority_range", []() {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    return py::make_tuple(lo, hi);
  });
}
