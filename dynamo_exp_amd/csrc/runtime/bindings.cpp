// pybind11 module `_C_runtime`: host-side native runtime pieces.
//   * xxh3-64 + KV block / sequence hashing (reference lib/llm/src/tokens.rs)
//   * RadixIndexer  (KV router index, reference kv_router/indexer.rs)
//   * BlockPool     (engine paged-KV manager with prefix cache + events)
//   * two-part codec (reference pipeline/network/codec/two_part.rs)
//   * EventRing     (shared-memory broadcast ring: TP leader -> followers)
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <string>

#include "block_pool.h"
#include "event_ring.h"
#include "radix_indexer.h"
#include "xxh3.h"

namespace py = pybind11;
using namespace dx;

namespace {

constexpr uint64_t kKvSeed = 1337;

std::vector<uint32_t> to_u32(const py::object& tokens) {
  auto arr = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(tokens);
  if (!arr) throw std::invalid_argument("tokens must be a sequence of ints");
  std::vector<uint32_t> out(arr.size());
  auto r = arr.unchecked<1>();
  for (py::ssize_t i = 0; i < arr.size(); ++i) out[i] = (uint32_t)r(i);
  return out;
}

// local (tokens-only) hash of each full block
std::vector<uint64_t> block_hashes(const std::vector<uint32_t>& t, size_t bs) {
  std::vector<uint64_t> out;
  const size_t nb = bs ? t.size() / bs : 0;
  out.reserve(nb);
  for (size_t b = 0; b < nb; ++b) out.push_back(xxh3::hash64(t.data() + b * bs, bs * 4, kKvSeed));
  return out;
}

// chained sequence hashes: s0 = b0; s_i = xxh3([s_{i-1}, b_i] as 2 x u64 LE)
std::vector<uint64_t> seq_hashes_from_blocks(const std::vector<uint64_t>& bh, bool has_parent, uint64_t parent) {
  std::vector<uint64_t> out;
  out.reserve(bh.size());
  uint64_t prev = parent;
  bool have = has_parent;
  for (uint64_t b : bh) {
    uint64_t s;
    if (!have) {
      s = b;
    } else {
      uint64_t pair[2] = {prev, b};
      s = xxh3::hash64(pair, 16, kKvSeed);
    }
    out.push_back(s);
    prev = s;
    have = true;
  }
  return out;
}

py::bytes encode_two_part(const std::string& header, const std::string& body) {
  std::string buf;
  buf.resize(24 + header.size() + body.size());
  std::string concat = header + body;
  const uint64_t ck = xxh3::hash64(concat.data(), concat.size(), 0);
  auto put_be = [&](size_t off, uint64_t v) {
    for (int i = 0; i < 8; ++i) buf[off + i] = (char)((v >> (56 - 8 * i)) & 0xff);
  };
  put_be(0, header.size());
  put_be(8, body.size());
  put_be(16, ck);
  std::memcpy(&buf[24], concat.data(), concat.size());
  return py::bytes(buf);
}

// returns None if incomplete, else (header, body, consumed); raises on bad checksum / size
py::object decode_two_part(const std::string& buf, int64_t max_size) {
  if (buf.size() < 24) return py::none();
  auto get_be = [&](size_t off) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | (uint8_t)buf[off + i];
    return v;
  };
  const uint64_t hl = get_be(0), bl = get_be(8), ck = get_be(16);
  const uint64_t total = 24 + hl + bl;
  if (max_size > 0 && total > (uint64_t)max_size) throw std::length_error("two-part message too large");
  if (buf.size() < total) return py::none();
  if (xxh3::hash64(buf.data() + 24, hl + bl, 0) != ck) throw std::runtime_error("two-part checksum mismatch");
  return py::make_tuple(py::bytes(buf.data() + 24, hl), py::bytes(buf.data() + 24 + hl, bl), (int64_t)total);
}

// Every complete frame at the front of `b` (a bytes / bytearray read buffer):
// ([(header, body), ...], bytes consumed).  One call per socket read instead
// of a Python loop per frame (the per-token frames of many multiplexed
// streams arrive back to back).
py::tuple split_two_part(py::buffer b, int64_t max_size) {
  py::buffer_info info = b.request();
  const auto* p = static_cast<const uint8_t*>(info.ptr);
  const size_t n = static_cast<size_t>(info.size * info.itemsize);
  auto get_be = [&](size_t off) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[off + i];
    return v;
  };
  py::list out;
  size_t pos = 0;
  while (n - pos >= 24) {
    const uint64_t hl = get_be(pos), bl = get_be(pos + 8), ck = get_be(pos + 16);
    if (hl > (1ull << 40) || bl > (1ull << 40)) throw std::length_error("two-part message too large");
    const uint64_t total = 24 + hl + bl;
    if (max_size > 0 && total > (uint64_t)max_size) throw std::length_error("two-part message too large");
    if (n - pos < total) break;
    const char* d = reinterpret_cast<const char*>(p + pos + 24);
    if (xxh3::hash64(d, hl + bl, 0) != ck) throw std::runtime_error("two-part checksum mismatch");
    out.append(py::make_tuple(py::bytes(d, hl), py::bytes(d + hl, bl)));
    pos += total;
  }
  return py::make_tuple(out, (int64_t)pos);
}

}  // namespace

PYBIND11_MODULE(_C_runtime, m) {
  m.doc() = "dynamo_exp_amd native runtime (hashing, radix indexer, block pool, codec)";
  m.attr("KV_HASH_SEED") = kKvSeed;

  m.def("xxh3_64", [](py::bytes data, uint64_t seed) {
    std::string s = data;
    return xxh3::hash64(s.data(), s.size(), seed);
  }, py::arg("data"), py::arg("seed") = 0);
  m.def("block_hashes", [](py::object tokens, size_t bs) { return block_hashes(to_u32(tokens), bs); });
  m.def("sequence_hashes", [](py::object tokens, size_t bs, py::object parent) {
    auto bh = block_hashes(to_u32(tokens), bs);
    const bool hp = !parent.is_none();
    return seq_hashes_from_blocks(bh, hp, hp ? parent.cast<uint64_t>() : 0);
  }, py::arg("tokens"), py::arg("block_size"), py::arg("parent") = py::none());
  m.def("block_and_sequence_hashes", [](py::object tokens, size_t bs) {
    auto bh = block_hashes(to_u32(tokens), bs);
    return py::make_tuple(bh, seq_hashes_from_blocks(bh, false, 0));
  });
  m.def("chain_hashes", [](std::vector<uint64_t> bh, py::object parent) {
    const bool hp = !parent.is_none();
    return seq_hashes_from_blocks(bh, hp, hp ? parent.cast<uint64_t>() : 0);
  }, py::arg("block_hashes"), py::arg("parent") = py::none());
  m.def("encode_two_part", &encode_two_part);
  m.def("decode_two_part", &decode_two_part, py::arg("buf"), py::arg("max_size") = 0);
  m.def("split_two_part", &split_two_part, py::arg("buf"), py::arg("max_size") = 0);

  py::class_<EventRing>(m, "EventRing")
      .def_static("create", &EventRing::create, py::arg("name"), py::arg("nslots"), py::arg("slot_bytes"),
                  py::arg("nconsumers"))
      .def_static("attach", &EventRing::attach, py::arg("name"), py::arg("consumer"))
      .def("publish", [](EventRing& r, py::bytes b, double timeout_s) {
        std::string s = b;
        py::gil_scoped_release rel;
        return r.publish(reinterpret_cast<const uint8_t*>(s.data()), s.size(), timeout_s);
      }, py::arg("data"), py::arg("timeout_s") = -1.0)
      .def("poll", [](EventRing& r, double timeout_s) -> py::object {
        std::vector<uint8_t> out;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = r.poll(out, timeout_s);
        }
        if (!ok) return py::none();
        return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
      }, py::arg("timeout_s") = -1.0)
      .def("close", &EventRing::close_ring)
      .def_property_readonly("closed", &EventRing::closed)
      .def_property_readonly("head", &EventRing::head)
      .def_property_readonly("name", &EventRing::name)
      .def("unlink", &EventRing::unlink);

  py::class_<RadixIndexer>(m, "RadixIndexer")
      .def(py::init<int64_t>(), py::arg("expiration_ns") = 0)
      .def("apply_stored", [](RadixIndexer& r, WorkerId w, py::object parent, std::vector<uint64_t> ext,
                              std::vector<uint64_t> local) {
        if (ext.size() != local.size()) throw std::invalid_argument("hash lists differ in length");
        const bool hp = !parent.is_none();
        py::gil_scoped_release rel;
        return r.apply_stored(w, hp, hp ? parent.cast<uint64_t>() : 0, ext.data(), local.data(), ext.size());
      })
      .def("apply_removed", [](RadixIndexer& r, WorkerId w, std::vector<uint64_t> ext) {
        py::gil_scoped_release rel;
        return r.apply_removed(w, ext.data(), ext.size());
      })
      .def("remove_worker", [](RadixIndexer& r, WorkerId w) {
        py::gil_scoped_release rel;
        r.remove_worker(w);
      })
      .def("find_matches", [](RadixIndexer& r, std::vector<uint64_t> local, bool early_exit) {
        std::vector<std::pair<WorkerId, uint32_t>> res;
        {
          py::gil_scoped_release rel;
          res = r.find_matches(local.data(), local.size(), early_exit);
        }
        py::dict d;
        for (auto& kv : res) d[py::int_(kv.first)] = kv.second;
        return d;
      }, py::arg("local_hashes"), py::arg("early_exit") = false)
      .def("find_matches_freq", [](RadixIndexer& r, std::vector<uint64_t> local, bool early_exit) {
        std::vector<std::pair<WorkerId, uint32_t>> res;
        std::vector<uint32_t> freq;
        {
          py::gil_scoped_release rel;
          res = r.find_matches(local.data(), local.size(), early_exit, &freq);
        }
        py::dict d;
        for (auto& kv : res) d[py::int_(kv.first)] = kv.second;
        return py::make_tuple(d, freq);
      }, py::arg("local_hashes"), py::arg("early_exit") = false)
      .def("find_matches_for_tokens", [](RadixIndexer& r, py::object tokens, size_t bs, bool early_exit) {
        auto local = block_hashes(to_u32(tokens), bs);
        std::vector<std::pair<WorkerId, uint32_t>> res;
        {
          py::gil_scoped_release rel;
          res = r.find_matches(local.data(), local.size(), early_exit);
        }
        py::dict d;
        for (auto& kv : res) d[py::int_(kv.first)] = kv.second;
        return d;
      }, py::arg("tokens"), py::arg("block_size"), py::arg("early_exit") = false)
      .def("num_nodes", &RadixIndexer::num_nodes)
      .def("num_blocks", &RadixIndexer::num_blocks)
      .def("workers", &RadixIndexer::workers)
      .def("events", &RadixIndexer::events)
      .def("clear", &RadixIndexer::clear);

  py::class_<ShardedRadixIndexer>(m, "ShardedRadixIndexer")
      .def(py::init<size_t, int64_t>(), py::arg("num_shards"), py::arg("expiration_ns") = 0)
      .def("num_shards", &ShardedRadixIndexer::num_shards)
      .def("apply_stored", [](ShardedRadixIndexer& r, WorkerId w, py::object parent, std::vector<uint64_t> ext,
                              std::vector<uint64_t> local) {
        if (ext.size() != local.size()) throw std::invalid_argument("hash lists differ in length");
        const bool hp = !parent.is_none();
        const uint64_t pv = hp ? parent.cast<uint64_t>() : 0;
        py::gil_scoped_release rel;
        r.apply_stored(w, hp, pv, std::move(ext), std::move(local));
      })
      .def("apply_removed", [](ShardedRadixIndexer& r, WorkerId w, std::vector<uint64_t> ext) {
        py::gil_scoped_release rel;
        r.apply_removed(w, std::move(ext));
      })
      .def("remove_worker", [](ShardedRadixIndexer& r, WorkerId w) {
        py::gil_scoped_release rel;
        r.remove_worker(w);
      })
      .def("find_matches_freq", [](ShardedRadixIndexer& r, std::vector<uint64_t> local, bool early_exit) {
        ShardedRadixIndexer::Match m;
        {
          py::gil_scoped_release rel;
          m = r.find_matches(std::move(local), early_exit);
        }
        py::dict d;
        for (auto& kv : m.scores) d[py::int_(kv.first)] = kv.second;
        return py::make_tuple(d, m.frequencies);
      }, py::arg("local_hashes"), py::arg("early_exit") = false)
      .def("flush", [](ShardedRadixIndexer& r) {
        py::gil_scoped_release rel;
        r.flush();
      })
      .def("num_blocks", [](ShardedRadixIndexer& r, WorkerId w) {
        py::gil_scoped_release rel;
        return r.num_blocks(w);
      })
      .def("workers", &ShardedRadixIndexer::workers)
      .def("shard_index", &ShardedRadixIndexer::shard_index);

  py::class_<BlockPool>(m, "BlockPool")
      .def(py::init<int32_t, bool>(), py::arg("num_blocks"), py::arg("enable_caching") = true)
      .def_property_readonly("num_blocks", &BlockPool::num_blocks)
      .def("num_free", &BlockPool::num_free)
      .def("num_used", &BlockPool::num_used)
      .def("num_cached", &BlockPool::num_cached)
      .def("allocate", [](BlockPool& p, int32_t n) -> py::object {
        std::vector<int32_t> out;
        if (!p.allocate(n, out)) return py::none();
        return py::cast(out);
      })
      .def("match_prefix", [](BlockPool& p, std::vector<uint64_t> h) {
        std::vector<int32_t> out;
        p.match_prefix(h.data(), h.size(), out);
        return out;
      })
      .def("count_prefix", [](BlockPool& p, std::vector<uint64_t> h) { return p.count_prefix(h.data(), h.size()); })
      .def("register_block", [](BlockPool& p, int32_t b, uint64_t s, uint64_t l, py::object parent) {
        const bool hp = !parent.is_none();
        return p.register_block(b, s, l, hp, hp ? parent.cast<uint64_t>() : 0);
      })
      .def("free", [](BlockPool& p, std::vector<int32_t> ids, uint32_t priority) {
            p.free_blocks(ids.data(), ids.size(), priority);
          }, py::arg("ids"), py::arg("priority") = 0)
      .def("set_priority", &BlockPool::set_priority)
      .def("inc_ref", [](BlockPool& p, std::vector<int32_t> ids) { p.inc_ref(ids.data(), ids.size()); })
      .def("ref_count", [](BlockPool& p, int32_t b) { return p.block(b).ref; })
      .def("block_seq_hash", [](BlockPool& p, int32_t b) -> py::object {
        const auto& bl = p.block(b);
        if (!bl.registered) return py::none();
        return py::int_(bl.seq_hash);
      })
      .def("block_info", [](BlockPool& p, int32_t b) -> py::object {  // (seq, local, parent|None) if registered
        const auto& bl = p.block(b);
        if (!bl.registered) return py::none();
        return py::make_tuple(bl.seq_hash, bl.local_hash,
                              bl.has_parent ? py::object(py::int_(bl.parent_hash)) : py::object(py::none()));
      })
      .def("reset_cache", &BlockPool::reset_cache)
      .def("set_track_evictions", &BlockPool::set_track_evictions)
      .def("drain_evicted", [](BlockPool& p) {
        py::list out;
        for (auto& e : p.drain_evicted())
          out.append(py::make_tuple(e.block, e.seq_hash, e.local_hash,
                                    e.has_parent ? py::object(py::int_(e.parent_hash)) : py::object(py::none())));
        return out;
      })
      .def("evict_lru", &BlockPool::evict_lru)
      .def("lru_candidates", &BlockPool::lru_candidates)
      .def("drain_events", [](BlockPool& p) {
        py::list out;
        for (auto& e : p.drain_events()) {
          out.append(py::make_tuple(e.kind, e.seq_hash, e.local_hash,
                                    e.has_parent ? py::object(py::int_(e.parent_hash)) : py::object(py::none())));
        }
        return out;
      });
}
