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
//
// Frequency window (reference RadixTree::new_with_frequency, :202-275): with an
// expiration window every matched node keeps the times of its recent matches;
// find_matches reports, per matched depth, how many matches fell inside the
// window before this one (zeros omitted) and records this match.
//
// ShardedRadixIndexer (reference KvIndexerSharded, :677-890): N RadixIndexer
// shards, each owned by one actor thread that applies its workers' events in
// arrival order; a worker is pinned to the least-loaded shard at its first
// event; a match query is broadcast to every shard (each answers after the
// events queued before it) and the answers merged -- scores are disjoint by
// worker, frequencies summed per depth.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
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
    std::deque<int64_t> recent_uses;  // match times (ns), frequency window only
    bool live = false;
  };

  // expiration_ns > 0 turns on the frequency window
  explicit RadixIndexer(int64_t expiration_ns = 0) : expiration_ns_(expiration_ns) {
    nodes_.emplace_back();
    nodes_[0].live = true;
  }

  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
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
  // worker holds.  early_exit stops once a single worker remains.  freq (if
  // given): the frequency window's per-depth counts (see the file comment).
  std::vector<std::pair<WorkerId, uint32_t>> find_matches(const uint64_t* local_hashes, size_t n, bool early_exit,
                                                          std::vector<uint32_t>* freq = nullptr) {
    std::lock_guard<std::mutex> g(mu_);
    std::unordered_map<WorkerId, uint32_t> scores;
    uint32_t cur = 0;
    const uint64_t now = ++clock_;
    const int64_t t = expiration_ns_ > 0 ? now_ns() : 0;
    for (size_t i = 0; i < n; ++i) {
      auto& ch = nodes_[cur].children;
      auto it = ch.find(local_hashes[i]);
      if (it == ch.end()) break;
      cur = it->second;
      Node& nd = nodes_[cur];
      if (nd.workers.empty()) break;
      for (WorkerId w : nd.workers) scores[w] += 1;
      if (expiration_ns_ > 0) {
        while (!nd.recent_uses.empty() && t - nd.recent_uses.front() > expiration_ns_) nd.recent_uses.pop_front();
        if (freq && !nd.recent_uses.empty()) freq->push_back((uint32_t)nd.recent_uses.size());
        nd.recent_uses.push_back(t);
      }
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
  int64_t expiration_ns_ = 0;
};

class ShardedRadixIndexer {
 public:
  struct Match {
    std::unordered_map<WorkerId, uint32_t> scores;
    std::vector<uint32_t> frequencies;
  };

  ShardedRadixIndexer(size_t num_shards, int64_t expiration_ns = 0) {
    if (num_shards == 0) num_shards = 1;
    counts_.assign(num_shards, 0);
    for (size_t i = 0; i < num_shards; ++i) shards_.emplace_back(new Shard(expiration_ns));
    for (auto& sh : shards_) {
      Shard* p = sh.get();
      p->thread = std::thread([p] { p->run(); });
    }
  }
  ~ShardedRadixIndexer() {
    for (auto& sh : shards_) sh->stop();
    for (auto& sh : shards_)
      if (sh->thread.joinable()) sh->thread.join();
  }
  ShardedRadixIndexer(const ShardedRadixIndexer&) = delete;
  ShardedRadixIndexer& operator=(const ShardedRadixIndexer&) = delete;

  size_t num_shards() const { return shards_.size(); }

  // Events are queued to the worker's shard and applied by its actor thread.
  void apply_stored(WorkerId w, bool has_parent, uint64_t parent, std::vector<uint64_t> ext,
                    std::vector<uint64_t> local) {
    shard_of(w)->post([=, e = std::move(ext), l = std::move(local)](RadixIndexer& t) {
      t.apply_stored(w, has_parent, parent, e.data(), l.data(), e.size());
    });
  }
  void apply_removed(WorkerId w, std::vector<uint64_t> ext) {
    shard_of(w)->post([=, e = std::move(ext)](RadixIndexer& t) { t.apply_removed(w, e.data(), e.size()); });
  }
  void remove_worker(WorkerId w) {
    Shard* sh = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = assign_.find(w);
      if (it == assign_.end()) return;
      sh = shards_[it->second].get();
      counts_[it->second] -= 1;
      assign_.erase(it);
    }
    sh->post([w](RadixIndexer& t) { t.remove_worker(w); });
  }

  // Broadcast to every shard; each answers after its earlier events.
  Match find_matches(std::vector<uint64_t> local, bool early_exit) {
    auto hashes = std::make_shared<std::vector<uint64_t>>(std::move(local));
    std::vector<std::future<Match>> futs;
    for (auto& sh : shards_) {
      auto pr = std::make_shared<std::promise<Match>>();
      futs.push_back(pr->get_future());
      sh->post([hashes, early_exit, pr](RadixIndexer& t) {
        Match m;
        auto res = t.find_matches(hashes->data(), hashes->size(), early_exit, &m.frequencies);
        for (auto& kv : res) m.scores.emplace(kv.first, kv.second);
        pr->set_value(std::move(m));
      });
    }
    Match out;
    for (size_t i = 0; i < futs.size(); ++i) {
      Match m = futs[i].get();
      for (auto& kv : m.scores) out.scores.emplace(kv.first, kv.second);
      if (out.frequencies.size() < m.frequencies.size()) out.frequencies.resize(m.frequencies.size(), 0);
      for (size_t k = 0; k < m.frequencies.size(); ++k) out.frequencies[k] += m.frequencies[k];
    }
    return out;
  }

  // Wait until every event queued so far has been applied.
  void flush() {
    std::vector<std::future<void>> futs;
    for (auto& sh : shards_) {
      auto pr = std::make_shared<std::promise<void>>();
      futs.push_back(pr->get_future());
      sh->post([pr](RadixIndexer&) { pr->set_value(); });
    }
    for (auto& f : futs) f.get();
  }

  size_t num_blocks(WorkerId w) {
    Shard* sh = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = assign_.find(w);
      if (it == assign_.end()) return 0;
      sh = shards_[it->second].get();
    }
    flush();
    return sh->tree.num_blocks(w);
  }
  std::vector<WorkerId> workers() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<WorkerId> out;
    for (auto& kv : assign_) out.push_back(kv.first);
    return out;
  }
  int shard_index(WorkerId w) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = assign_.find(w);
    return it == assign_.end() ? -1 : (int)it->second;
  }

 private:
  struct Shard {
    explicit Shard(int64_t exp) : tree(exp) {}
    RadixIndexer tree;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void(RadixIndexer&)>> q;
    bool stopping = false;
    std::thread thread;

    void post(std::function<void(RadixIndexer&)> fn) {
      {
        std::lock_guard<std::mutex> g(mu);
        q.push_back(std::move(fn));
      }
      cv.notify_one();
    }
    void stop() {
      {
        std::lock_guard<std::mutex> g(mu);
        stopping = true;
      }
      cv.notify_one();
    }
    void run() {
      for (;;) {
        std::function<void(RadixIndexer&)> fn;
        {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [this] { return stopping || !q.empty(); });
          if (q.empty()) return;  // stopping and drained
          fn = std::move(q.front());
          q.pop_front();
        }
        fn(tree);
      }
    }
  };

  Shard* shard_of(WorkerId w) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = assign_.find(w);
    if (it != assign_.end()) return shards_[it->second].get();
    size_t best = 0;  // least-loaded shard (reference: min worker count)
    for (size_t i = 1; i < counts_.size(); ++i)
      if (counts_[i] < counts_[best]) best = i;
    counts_[best] += 1;
    assign_.emplace(w, best);
    return shards_[best].get();
  }

  std::mutex mu_;
  std::vector<std::unique_ptr<Shard>> shards_;
  std::vector<size_t> counts_;
  std::unordered_map<WorkerId, size_t> assign_;
};

}  // namespace dx
