// Global KV-block radix indexer (the KV router's view of every worker's cache).
//
// Semantics follow the reference RadixTree (lib/llm/src/kv_router/indexer.rs:
// find_matches :239-282, apply_event :284-378, remove_worker :380): nodes are
// keyed by the *local* block hash (tokens only, position-free), each node
// records which workers hold the block, and a per-worker map from the
// worker's *external* sequence hash to the node resolves Stored.parent_hash and
// Removed.block_hashes.  Differences: nodes whose worker set
// empties are pruned from their parent (the reference leaks them), and the
// structure is an index-addressed node arena (no Rc<RefCell>), guarded by one
// mutex so Python threads can share it.
#pragma once
#include <cstdint>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

namespace dx {

using WorkerId = int64_t;

class RadixIndexer {
 public:
  struct Node {
    uint32_t parent = 0;
    uint64_t local_hash = 0;
    std::unordered_map<uint64_t, uint32_t> children;
    std::vector<WorkerId> workers;  // small, unsorted
    uint64_t last_access = 0;
    bool live = false;
  };

  RadixIndexer() {
    nodes_.emplace_back();
    nodes_[0].live = true;
  }

  // Returns number of blocks actually attached (0 if the parent is unknown).
  size_t apply_stored(WorkerId w, bool has_parent, uint64_t parent_ext, const uint64_t* ext_hashes,
                      const uint64_t* local_hashes, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    auto& lookup = lookup_[w];
    uint32_t cur = 0;
    if (has_parent) {
      auto it = lookup.find(parent_ext);
      if (it == lookup.end()) return 0;
      cur = it->second;
    }
    for (size_t i = 0; i < n; ++i) {
      uint32_t child;
      auto& ch = nodes_[cur].children;
      auto it = ch.find(local_hashes[i]);
      if (it != ch.end()) {
        child = it->second;
      } else {
        child = alloc();
        nodes_[child].parent = cur;
        nodes_[child].local_hash = local_hashes[i];
        nodes_[cur].children.emplace(local_hashes[i], child);
      }
      add_worker(child, w);
      nodes_[child].last_access = ++clock_;
      auto prev = lookup.find(ext_hashes[i]);
      if (prev != lookup.end() && prev->second != child) {
        // external hash re-stored at a different place: detach the old node
        drop_worker(prev->second, w);
      }
      lookup[ext_hashes[i]] = child;
      cur = child;
    }
    ++events_;
    return n;
  }

  size_t apply_removed(WorkerId w, const uint64_t* ext_hashes, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    auto lit = lookup_.find(w);
    if (lit == lookup_.end()) return 0;
    size_t removed = 0;
    for (size_t i = 0; i < n; ++i) {
      auto it = lit->second.find(ext_hashes[i]);
      if (it == lit->second.end()) continue;
      const uint32_t node = it->second;
      lit->second.erase(it);
      drop_worker(node, w);
      ++removed;
    }
    ++events_;
    return removed;
  }

  void remove_worker(WorkerId w) {
    std::lock_guard<std::mutex> g(mu_);
    auto lit = lookup_.find(w);
    if (lit == lookup_.end()) return;
    std::vector<uint32_t> nodes;
    nodes.reserve(lit->second.size());
    for (auto& kv : lit->second) nodes.push_back(kv.second);
    lookup_.erase(lit);
    for (uint32_t n : nodes) drop_worker(n, w);
  }

  // Overlap score per worker = number of leading blocks of `local_hashes` the
  // worker holds.  early_exit stops once a single worker remains.
  std::vector<std::pair<WorkerId, uint32_t>> find_matches(const uint64_t* local_hashes, size_t n, bool early_exit,
                                                          std::vector<uint32_t>* freq = nullptr) {
    std::lock_guard<std::mutex> g(mu_);
    std::unordered_map<WorkerId, uint32_t> scores;
    uint32_t cur = 0;
    const uint64_t now = ++clock_;
    for (size_t i = 0; i < n; ++i) {
      auto& ch = nodes_[cur].children;
      auto it = ch.find(local_hashes[i]);
      if (it == ch.end()) break;
      cur = it->second;
      Node& nd = nodes_[cur];
      if (nd.workers.empty()) break;
      for (WorkerId w : nd.workers) scores[w] += 1;
      if (freq) freq->push_back((uint32_t)nd.workers.size());
      nd.last_access = now;
      if (early_exit && nd.workers.size() == 1) break;
    }
    return {scores.begin(), scores.end()};
  }

  size_t num_nodes() {
    std::lock_guard<std::mutex> g(mu_);
    return nodes_.size() - free_.size() - 1;
  }
  size_t num_blocks(WorkerId w) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = lookup_.find(w);
    return it == lookup_.end() ? 0 : it->second.size();
  }
  std::vector<WorkerId> workers() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<WorkerId> out;
    for (auto& kv : lookup_) out.push_back(kv.first);
    return out;
  }
  uint64_t events() const { return events_; }
  void clear() {
    std::lock_guard<std::mutex> g(mu_);
    nodes_.clear();
    free_.clear();
    lookup_.clear();
    nodes_.emplace_back();
    nodes_[0].live = true;
  }

 private:
  uint32_t alloc() {
    if (!free_.empty()) {
      uint32_t id = free_.back();
      free_.pop_back();
      nodes_[id] = Node();
      nodes_[id].live = true;
      return id;
    }
    nodes_.emplace_back();
    nodes_.back().live = true;
    return (uint32_t)nodes_.size() - 1;
  }
  void add_worker(uint32_t n, WorkerId w) {
    auto& ws = nodes_[n].workers;
    for (WorkerId x : ws)
      if (x == w) return;
    ws.push_back(w);
  }
  void drop_worker(uint32_t n, WorkerId w) {
    auto& ws = nodes_[n].workers;
    for (size_t i = 0; i < ws.size(); ++i)
      if (ws[i] == w) {
        ws[i] = ws.back();
        ws.pop_back();
        break;
      }
    prune(n);
  }
  // remove empty leaves upwards
  void prune(uint32_t n) {
    while (n != 0 && nodes_[n].live && nodes_[n].workers.empty() && nodes_[n].children.empty()) {
      const uint32_t p = nodes_[n].parent;
      nodes_[p].children.erase(nodes_[n].local_hash);
      nodes_[n].live = false;
      nodes_[n].children.clear();
      free_.push_back(n);
      n = p;
    }
  }

  std::mutex mu_;
  std::vector<Node> nodes_;
  std::vector<uint32_t> free_;
  std::unordered_map<WorkerId, std::unordered_map<uint64_t, uint32_t>> lookup_;
  uint64_t clock_ = 0;
  uint64_t events_ = 0;
};

}  // namespace dx
