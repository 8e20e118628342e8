// Paged-KV block pool with prefix caching -- the engine-side block manager.
//
// Mirrors the reference KV manager v2 semantics (lib/llm/src/kv/reuse.rs
// AvailableBlocks: lookup by sequence hash + priority/return-tick eviction
// order; kv/reserved.rs ReservedBlocks: shared immutable matchable blocks;
// kv/manager.rs prepare_prefill_sequence: in-flight, then freed, then new)
// but is actually wired into serving here.  Also emits the
// KV events (Stored / Removed) the router indexes, using the same
// xxh3(seed 1337) block / sequence hashes.
//
// Eviction order of released (reusable, still matchable) blocks is the
// reference's PriorityKey (reuse.rs:250-279): lowest priority first, then
// oldest return tick -- a block's priority is set when it is freed (the
// request's priority) or later by `set_priority` (reuse.rs update_block), its
// return tick is a pool-wide counter bumped on every release.
//
// Two tiers: the device pool (`tier 0`) and an optional pinned-host tier
// (`tier 1`, hipHostMalloc'd by the engine).  A block evicted from HBM can be
// demoted to the host tier instead of being forgotten; a later prefix hit on a
// host block is promoted back (the engine performs the copies, this class only
// does the bookkeeping).
#pragma once
#include <cstdint>
#include <mutex>
#include <set>
#include <stdexcept>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace dx {

// A registered block that was evicted from this pool (its content is still
// intact until the new owner writes it: the engine may demote it first).
struct Evicted {
  int32_t block;
  uint64_t seq_hash, local_hash, parent_hash;
  bool has_parent;
};

struct KvEvent {
  int kind;  // 0 = stored, 1 = removed
  int tier;
  uint64_t seq_hash;
  uint64_t local_hash;
  uint64_t parent_hash;
  bool has_parent;
};

class BlockPool {
 public:
  // (priority, return tick, block): std::set order = eviction order
  using Key = std::tuple<uint32_t, uint64_t, int32_t>;

  struct Block {
    int32_t ref = 0;
    bool registered = false;
    uint64_t seq_hash = 0, local_hash = 0, parent_hash = 0;
    bool has_parent = false;
    uint32_t priority = 0;
    uint64_t return_tick = 0;
    bool in_lru = false;
  };

  explicit BlockPool(int32_t num_blocks, bool enable_caching = true)
      : blocks_(num_blocks), caching_(enable_caching) {
    free_.reserve(num_blocks);
    for (int32_t i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
  }

  int32_t num_blocks() const { return (int32_t)blocks_.size(); }
  int32_t num_free() {
    std::lock_guard<std::mutex> g(mu_);
    return (int32_t)(free_.size() + lru_.size());
  }
  int32_t num_cached() {
    std::lock_guard<std::mutex> g(mu_);
    return (int32_t)cache_.size();
  }
  int32_t num_used() {
    std::lock_guard<std::mutex> g(mu_);
    return (int32_t)blocks_.size() - (int32_t)(free_.size() + lru_.size());
  }

  // Allocate n fresh blocks (evicting LRU cached ones).  Returns false (and
  // allocates nothing) if not enough blocks are available.
  bool allocate(int32_t n, std::vector<int32_t>& out) {
    std::lock_guard<std::mutex> g(mu_);
    if ((size_t)n > free_.size() + lru_.size()) return false;
    for (int32_t i = 0; i < n; ++i) {
      int32_t b;
      if (!free_.empty()) {
        b = free_.back();
        free_.pop_back();
      } else {
        b = std::get<2>(*lru_.begin());
        lru_.erase(lru_.begin());
        Block& bl = blocks_[b];
        bl.in_lru = false;
        evict_locked(b);
      }
      blocks_[b].ref = 1;
      out.push_back(b);
    }
    return true;
  }

  // Longest cached prefix of `seq_hashes`; takes a reference on each hit.
  int32_t match_prefix(const uint64_t* seq_hashes, size_t n, std::vector<int32_t>& out) {
    std::lock_guard<std::mutex> g(mu_);
    if (!caching_) return 0;
    int32_t hits = 0;
    for (size_t i = 0; i < n; ++i) {
      auto it = cache_.find(seq_hashes[i]);
      if (it == cache_.end()) break;
      const int32_t b = it->second;
      Block& bl = blocks_[b];
      unlink_locked(b);
      bl.ref += 1;
      out.push_back(b);
      ++hits;
    }
    return hits;
  }

  // Number of leading hashes cached (no references taken).
  int32_t count_prefix(const uint64_t* seq_hashes, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    if (!caching_) return 0;
    int32_t hits = 0;
    for (size_t i = 0; i < n; ++i) {
      if (cache_.find(seq_hashes[i]) == cache_.end()) break;
      ++hits;
    }
    return hits;
  }

  // Publish a full block under its sequence hash.  If another block already
  // holds that hash the call is a no-op (the duplicate stays private).
  bool register_block(int32_t b, uint64_t seq_hash, uint64_t local_hash, bool has_parent, uint64_t parent_hash) {
    std::lock_guard<std::mutex> g(mu_);
    if (!caching_) return false;
    Block& bl = blocks_.at(b);
    if (bl.registered) return false;
    if (cache_.count(seq_hash)) return false;
    bl.registered = true;
    bl.seq_hash = seq_hash;
    bl.local_hash = local_hash;
    bl.has_parent = has_parent;
    bl.parent_hash = parent_hash;
    cache_[seq_hash] = b;
    events_.push_back(KvEvent{0, 0, seq_hash, local_hash, parent_hash, has_parent});
    return true;
  }

  // Release references; a registered block whose last reference goes
  // becomes reusable (matchable until evicted) with `priority`.
  void free_blocks(const int32_t* ids, size_t n, uint32_t priority = 0) {
    std::lock_guard<std::mutex> g(mu_);
    // free in reverse so the tail of a sequence gets the older return tick and
    // is evicted before its head (same priority)
    for (size_t k = n; k-- > 0;) {
      const int32_t b = ids[k];
      Block& bl = blocks_.at(b);
      if (bl.ref <= 0) throw std::runtime_error("double free of KV block");
      if (--bl.ref == 0) {
        if (bl.registered) {
          bl.priority = priority;
          bl.return_tick = ++return_tick_;
          lru_.insert(Key{bl.priority, bl.return_tick, b});
          bl.in_lru = true;
        } else {
          free_.push_back(b);
        }
      }
    }
  }

  // reference reuse.rs update_block: re-rank a cached block (no-op if the
  // hash is not cached); a block in use keeps the priority for its release.
  bool set_priority(uint64_t seq_hash, uint32_t priority) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = cache_.find(seq_hash);
    if (it == cache_.end()) return false;
    const int32_t b = it->second;
    Block& bl = blocks_[b];
    if (bl.in_lru) {
      lru_.erase(Key{bl.priority, bl.return_tick, b});
      bl.priority = priority;
      lru_.insert(Key{bl.priority, bl.return_tick, b});
    } else {
      bl.priority = priority;
    }
    return true;
  }

  void inc_ref(const int32_t* ids, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t k = 0; k < n; ++k) {
      unlink_locked(ids[k]);
      blocks_.at(ids[k]).ref += 1;
    }
  }

  // Forget every cached block that is not in use (emits Removed events).
  int32_t reset_cache() {
    std::lock_guard<std::mutex> g(mu_);
    int32_t n = 0;
    while (!lru_.empty()) {
      const int32_t b = std::get<2>(*lru_.begin());
      lru_.erase(lru_.begin());
      blocks_[b].in_lru = false;
      evict_locked(b);
      free_.push_back(b);
      ++n;
    }
    return n;
  }

  // Evict up to n LRU cached blocks, returning (block, seq_hash, local, parent)
  // so the engine can demote them to the host tier before reuse.
  std::vector<int32_t> evict_lru(int32_t n) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int32_t> out;
    while (n-- > 0 && !lru_.empty()) {
      const int32_t b = std::get<2>(*lru_.begin());
      lru_.erase(lru_.begin());
      blocks_[b].in_lru = false;
      evict_locked(b);
      free_.push_back(b);
      out.push_back(b);
    }
    return out;
  }

  std::vector<int32_t> lru_candidates(int32_t n) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int32_t> out;
    for (auto it = lru_.begin(); it != lru_.end() && (int32_t)out.size() < n; ++it) out.push_back(std::get<2>(*it));
    return out;
  }

  const Block& block(int32_t b) const { return blocks_.at(b); }

  // Eviction log for host-tier demotion (off unless enabled).
  void set_track_evictions(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    track_evictions_ = on;
  }
  std::vector<Evicted> drain_evicted() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Evicted> e;
    e.swap(evicted_);
    return e;
  }

  std::vector<KvEvent> drain_events() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<KvEvent> e;
    e.swap(events_);
    return e;
  }

 private:
  void unlink_locked(int32_t b) {
    Block& bl = blocks_.at(b);
    if (bl.in_lru) {
      lru_.erase(Key{bl.priority, bl.return_tick, b});
      bl.in_lru = false;
    }
  }

  void evict_locked(int32_t b) {
    Block& bl = blocks_[b];
    if (bl.registered) {
      cache_.erase(bl.seq_hash);
      events_.push_back(KvEvent{1, 0, bl.seq_hash, bl.local_hash, bl.parent_hash, bl.has_parent});
      if (track_evictions_) evicted_.push_back(Evicted{b, bl.seq_hash, bl.local_hash, bl.parent_hash, bl.has_parent});
    }
    bl.registered = false;
    bl.ref = 0;
    bl.priority = 0;
  }

  std::mutex mu_;
  std::vector<Block> blocks_;
  std::vector<int32_t> free_;
  std::set<Key> lru_;  // reusable registered blocks in eviction order
  uint64_t return_tick_ = 0;
  std::unordered_map<uint64_t, int32_t> cache_;
  std::vector<KvEvent> events_;
  std::vector<Evicted> evicted_;
  bool caching_;
  bool track_evictions_ = false;
};

}  // namespace dx
