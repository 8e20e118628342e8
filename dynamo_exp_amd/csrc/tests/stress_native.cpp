// Concurrency stress for the native runtime pieces, built standalone with
// -fsanitize=address,undefined and with -fsanitize=thread (the
// reference relies on single-threaded actors and runs no sanitizers; here the
// radix indexer and the block pool are shared by Python threads behind a
// mutex, so they are exercised under concurrent mutation + lookup).
//
//   g++ -std=c++20 -O1 -g -fsanitize=thread -I.. stress_native.cpp -o stress && ./stress
// Exit code 0 and "ok" on success; any invariant violation aborts.
#include <atomic>
#include <cassert>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../runtime/block_pool.h"
#include "../runtime/radix_indexer.h"
#include "../runtime/xxh3.h"

#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                    \
    }                                                                  \
  } while (0)

static void stress_indexer() {
  dx::RadixIndexer idx;
  constexpr int kWorkers = 6, kIters = 4000;
  std::atomic<bool> stop{false};
  std::vector<std::thread> ts;
  // writers: each worker stores chains of blocks (ext hash = worker-unique), removes some
  for (int w = 0; w < kWorkers; ++w) {
    ts.emplace_back([&, w] {
      std::mt19937_64 rng(1000 + w);
      std::vector<uint64_t> mine;
      for (int it = 0; it < kIters; ++it) {
        const size_t n = 1 + rng() % 8;
        std::vector<uint64_t> loc(n), ext(n);
        for (size_t i = 0; i < n; ++i) {
          loc[i] = rng() % 64;  // small alphabet: shared prefixes across workers
          ext[i] = ((uint64_t)w << 48) | (uint64_t)(it * 16 + i);
        }
        const bool has_parent = !mine.empty() && (rng() % 2);
        const uint64_t parent = has_parent ? mine[rng() % mine.size()] : 0;
        if (idx.apply_stored(w, has_parent, parent, ext.data(), loc.data(), n) == n)
          mine.insert(mine.end(), ext.begin(), ext.end());
        if (!mine.empty() && rng() % 3 == 0) {
          const size_t k = 1 + rng() % std::min<size_t>(mine.size(), 4);
          std::vector<uint64_t> rm(mine.end() - k, mine.end());
          mine.resize(mine.size() - k);
          idx.apply_removed(w, rm.data(), rm.size());
        }
        if (rng() % 997 == 0) {
          idx.remove_worker(w);
          mine.clear();
        }
      }
    });
  }
  // readers: routing lookups while the tree changes
  for (int r = 0; r < 3; ++r) {
    ts.emplace_back([&, r] {
      std::mt19937_64 rng(7 + r);
      size_t hits = 0;
      while (!stop.load()) {
        std::vector<uint64_t> q(1 + rng() % 12);
        for (auto& h : q) h = rng() % 64;
        auto sc = idx.find_matches(q.data(), q.size(), rng() % 2);
        for (auto& [w, s] : sc) {
          CHECK(w >= 0 && w < kWorkers);
          CHECK(s <= q.size());
          hits += s;
        }
        (void)idx.num_nodes();
      }
      (void)hits;
    });
  }
  for (int w = 0; w < kWorkers; ++w) ts[w].join();
  stop = true;
  for (size_t i = kWorkers; i < ts.size(); ++i) ts[i].join();
  for (int w = 0; w < kWorkers; ++w) idx.remove_worker(w);
  CHECK(idx.num_nodes() == 0);  // every node pruned once no worker holds it
  std::printf("indexer: %llu events, ok\n", (unsigned long long)idx.events());
}

static void stress_block_pool() {
  constexpr int kBlocks = 512;
  dx::BlockPool pool(kBlocks, true);
  std::vector<std::thread> ts;
  std::atomic<int> failures{0};
  for (int t = 0; t < 6; ++t) {
    ts.emplace_back([&, t] {
      std::mt19937_64 rng(99 + t);
      for (int it = 0; it < 3000; ++it) {
        std::vector<int32_t> got;
        const int n = 1 + rng() % 16;
        if (!pool.allocate(n, got)) {
          failures++;
          continue;
        }
        CHECK((int)got.size() == n);
        // register a chain of content hashes (shared alphabet -> prefix hits)
        uint64_t parent = 0;
        for (int i = 0; i < n; ++i) {
          const uint64_t local = rng() % 32;
          const uint64_t seq = dx::xxh3::hash64(&local, sizeof local, parent ^ 1337);
          pool.register_block(got[i], seq, local, i > 0, parent);
          parent = seq;
        }
        std::vector<uint64_t> probe(4);
        for (auto& h : probe) h = rng();
        std::vector<int32_t> hit;
        const int32_t m = pool.match_prefix(probe.data(), probe.size(), hit);
        CHECK(m == (int32_t)hit.size());
        if (!hit.empty()) pool.free_blocks(hit.data(), hit.size());
        pool.free_blocks(got.data(), got.size());
        if (rng() % 500 == 0) (void)pool.evict_lru(8);
        (void)pool.drain_events();
      }
    });
  }
  for (auto& th : ts) th.join();
  CHECK(pool.num_used() == 0);
  CHECK(pool.num_free() == kBlocks);  // free list + LRU-cached blocks
  std::printf("block pool: %d allocation failures under contention, ok\n", failures.load());
}

// Sharded indexer: writer threads feed events for disjoint worker sets while
// readers broadcast queries; shard actors apply concurrently (TSAN target),
// then a flush + per-worker check against a single tree fed the same events.
static void stress_sharded_indexer() {
  dx::ShardedRadixIndexer sh(4, 1000000);  // 1 ms frequency window too
  dx::RadixIndexer ref;
  constexpr int kWorkers = 8, kIters = 1500;
  std::vector<std::vector<uint64_t>> chains(kWorkers);
  std::mutex ref_mu;
  std::atomic<bool> stop{false};
  std::vector<std::thread> ts;
  for (int t = 0; t < 2; ++t) {
    ts.emplace_back([&, t] {
      std::mt19937_64 rng(77 + t);
      for (int it = 0; it < kIters; ++it) {
        const int w = t + 2 * (int)(rng() % (kWorkers / 2));
        auto& ch = chains[w];
        if (!ch.empty() && rng() % 4 == 0) {
          std::vector<uint64_t> tail(ch.end() - 1, ch.end());
          ch.pop_back();
          sh.apply_removed(w, tail);
          std::lock_guard<std::mutex> g(ref_mu);
          ref.apply_removed(w, tail.data(), tail.size());
        } else {
          std::vector<uint64_t> blk{((uint64_t)w << 40) | (uint64_t)(ch.size() + 1)};
          const bool hp = !ch.empty();
          const uint64_t parent = hp ? ch.back() : 0;
          ch.push_back(blk[0]);
          sh.apply_stored(w, hp, parent, blk, blk);
          std::lock_guard<std::mutex> g(ref_mu);
          ref.apply_stored(w, hp, parent, blk.data(), blk.data(), 1);
        }
      }
    });
  }
  for (int r = 0; r < 2; ++r) {
    ts.emplace_back([&, r] {
      std::mt19937_64 rng(9 + r);
      while (!stop.load()) {
        std::vector<uint64_t> q;
        const int w = (int)(rng() % kWorkers);
        for (int i = 1; i <= 4; ++i) q.push_back(((uint64_t)w << 40) | (uint64_t)i);
        auto m = sh.find_matches(q, false);
        for (auto& kv : m.scores) CHECK(kv.second <= 4);
      }
    });
  }
  for (int i = 0; i < 2; ++i) ts[i].join();
  stop = true;
  for (size_t i = 2; i < ts.size(); ++i) ts[i].join();
  sh.flush();
  for (int w = 0; w < kWorkers; ++w) {
    auto& ch = chains[w];
    if (ch.empty()) continue;
    auto a = sh.find_matches(ch, false);
    auto b = ref.find_matches(ch.data(), ch.size(), false);
    uint32_t bw = 0;
    for (auto& kv : b)
      if (kv.first == w) bw = kv.second;
    CHECK(a.scores[w] == bw && bw == ch.size());
  }
}

int main() {
  const uint8_t empty[1] = {0};
  CHECK(dx::xxh3::hash64(empty, 0, 0) == 0x2D06800538D394C2ull);  // XXH3_64bits("") reference value
  stress_indexer();
  stress_sharded_indexer();
  stress_block_pool();
  std::printf("ok\n");
  return 0;
}
