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

int main() {
  const uint8_t empty[1] = {0};
  CHECK(dx::xxh3::hash64(empty, 0, 0) == 0x2D06800538D394C2ull);  // XXH3_64bits("") reference value
  stress_indexer();
  stress_block_pool();
  std::printf("ok\n");
  return 0;
}
