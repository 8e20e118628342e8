// dx-ctrld: native control-plane server (the etcd + NATS/JetStream role,
// SURVEY.md §2.14 / §2.17 "C++ control-plane server").
//
// Same wire protocol and semantics as the asyncio reference implementation in
// runtime/control_plane.py (ControlPlaneServer), so every Python client
// (DistributedRuntime, llmctl, serve, the disagg prefill queue) talks to either:
//   * revisioned KV with leases (TTL + keep-alive, revoke/expiry deletes the
//     lease's keys), create-if-absent, create-or-validate, prefix get/delete,
//     prefix watches that start with a consistent snapshot
//     (reference lib/runtime/src/transports/etcd.rs:170-198, :309);
//   * pub/sub with NATS wildcards (`*` one token, `>` the rest);
//   * durable work queues: push, pop with timeout (blocking pull), ack, nak,
//     redelivery after ack_wait, sizes (JetStream pull consumer,
//     examples/llm/utils/nats_queue.py);
//   * a blob store with optional TTL (NATS object store).
// Frames: u32-BE length + msgpack map; requests carry an `id`, responses
// `{id, ok, result|error}`, stream items `{id, ok, item}`.
//
// One thread, epoll, non-blocking sockets: every operation is atomic with
// respect to the others, like the single-threaded asyncio server.  Timers
// (lease expiry, queue redelivery, pop timeouts, blob TTL) run from the epoll
// timeout every 20 ms.
#include <sys/prctl.h>
#include <unistd.h>
#include <arpa/inet.h>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <errno.h>
#include <fcntl.h>
#include <map>
#include <memory>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <optional>
#include <set>
#include <string>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>
#include <unordered_map>
#include <vector>

#include "msgpack.h"

using dx::mp::Value;

namespace {

constexpr size_t kMaxFrame = size_t(1) << 30;
constexpr size_t kMaxOutbox = size_t(512) << 20;  // drop a consumer that stops reading

volatile std::sig_atomic_t g_stop = 0;

double mono() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double wall() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

bool subject_matches(const std::string& pat, const std::string& subj) {
  if (pat == subj) return true;
  auto split = [](const std::string& s) {
    std::vector<std::string> out;
    size_t b = 0;
    for (;;) {
      size_t e = s.find('.', b);
      out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
      if (e == std::string::npos) break;
      b = e + 1;
    }
    return out;
  };
  auto p = split(pat), s = split(subj);
  for (size_t i = 0; i < p.size(); ++i) {
    if (p[i] == ">") return s.size() > i;
    if (i >= s.size()) return false;
    if (p[i] != "*" && p[i] != s[i]) return false;
  }
  return p.size() == s.size();
}

struct Entry {
  Value value;
  int64_t rev = 0;
  std::optional<int64_t> lease;
};

struct Lease {
  double ttl = 10.0;
  double deadline = 0;
  std::set<std::string> keys;
};

struct QMsg {
  int64_t seq = 0;
  Value data;
  int64_t deliveries = 0;
  double deadline = 0;
};

struct Waiter {
  uint64_t conn;
  int64_t rid;
  double deadline;
  double ack_wait;
};

struct Queue {
  std::deque<QMsg> ready;
  std::map<int64_t, QMsg> inflight;
  std::deque<Waiter> waiters;
  int64_t seq = 0;
};

struct Blob {
  Value data;
  double expires = -1;  // < 0: no TTL
};

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  std::string in;
  std::string out;
  size_t out_off = 0;
  bool want_write = false;
  bool dead = false;
};

struct StreamReg {  // watch or subscription owned by a connection
  uint64_t conn;
  int64_t rid;
  std::string pattern;  // prefix (watch) or subject pattern (sub)
};

class Server {
 public:
  Server(std::string host, int port) : host_(std::move(host)), port_(port) {
    lease_next_ = 0x1000 + int64_t(getpid() & 0xFFF) * 0x10000;
  }

  int listen_and_serve() {
    if (!open_listener()) return 1;
    std::printf("ctrld listening on %s:%d\n", host_.c_str(), port_);
    std::fflush(stdout);
    epoll_event evs[256];
    double last_tick = mono();
    while (!g_stop) {
      int n = epoll_wait(ep_, evs, 256, 20);
      if (n < 0) {
        if (errno == EINTR) continue;
        std::perror("epoll_wait");
        return 1;
      }
      for (int k = 0; k < n; ++k) {
        if (evs[k].data.u64 == 0) {
          accept_all();
          continue;
        }
        auto it = conns_.find(evs[k].data.u64);
        if (it == conns_.end()) continue;
        Conn& c = *it->second;
        if (evs[k].events & (EPOLLERR | EPOLLHUP)) c.dead = true;
        if (!c.dead && (evs[k].events & EPOLLIN)) on_readable(c);
        if (!c.dead && (evs[k].events & EPOLLOUT)) flush(c);
      }
      double now = mono();
      if (now - last_tick >= 0.02) {
        tick(now);
        last_tick = now;
      }
      reap_dead();
    }
    return 0;
  }

 private:
  // ------------------------------------------------------------- state
  std::string host_;
  int port_;
  int lfd_ = -1, ep_ = -1;
  uint64_t next_conn_ = 1;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns_;
  std::map<std::string, Entry> kv_;
  int64_t rev_ = 0;
  std::unordered_map<int64_t, Lease> leases_;
  int64_t lease_next_;
  std::map<int64_t, StreamReg> watchers_, subs_;
  int64_t next_wid_ = 1;
  std::unordered_map<std::string, Queue> queues_;
  std::unordered_map<std::string, std::map<std::string, Blob>> blobs_;
  std::map<std::string, int64_t> op_stats_;

  // ------------------------------------------------------------- sockets
  bool open_listener() {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE;
    std::string port = std::to_string(port_);
    if (getaddrinfo(host_.c_str(), port.c_str(), &hints, &res) != 0 || !res) {
      std::fprintf(stderr, "ctrld: cannot resolve %s\n", host_.c_str());
      return false;
    }
    lfd_ = socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (bind(lfd_, res->ai_addr, res->ai_addrlen) != 0 || listen(lfd_, 1024) != 0) {
      std::perror("ctrld: bind/listen");
      freeaddrinfo(res);
      return false;
    }
    freeaddrinfo(res);
    sockaddr_storage ss{};
    socklen_t sl = sizeof ss;
    getsockname(lfd_, reinterpret_cast<sockaddr*>(&ss), &sl);
    if (ss.ss_family == AF_INET) port_ = ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
    else if (ss.ss_family == AF_INET6) port_ = ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port);
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = 0;
    epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &ev);
    return true;
  }

  void accept_all() {
    for (;;) {
      int fd = accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = next_conn_++;
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.u64 = c->id;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
      conns_[c->id] = std::move(c);
    }
  }

  void on_readable(Conn& c) {
    char buf[1 << 16];
    for (;;) {
      ssize_t n = recv(c.fd, buf, sizeof buf, 0);
      if (n > 0) {
        c.in.append(buf, size_t(n));
        continue;
      }
      if (n == 0) c.dead = true;
      else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) c.dead = true;
      break;
    }
    size_t off = 0;
    while (!c.dead && c.in.size() - off >= 4) {
      const uint8_t* p = reinterpret_cast<const uint8_t*>(c.in.data() + off);
      size_t n = (size_t(p[0]) << 24) | (size_t(p[1]) << 16) | (size_t(p[2]) << 8) | size_t(p[3]);
      if (n > kMaxFrame) {
        c.dead = true;
        break;
      }
      if (c.in.size() - off - 4 < n) break;
      Value msg;
      try {
        msg = dx::mp::Decoder(p + 4, n).decode();
      } catch (const std::exception& e) {
        std::fprintf(stderr, "ctrld: bad frame from conn %llu: %s\n", (unsigned long long)c.id, e.what());
        c.dead = true;
        break;
      }
      off += 4 + n;
      dispatch(c, msg);
    }
    c.in.erase(0, off);
  }

  void send(Conn& c, const Value& v) {
    if (c.dead) return;
    std::string body;
    dx::mp::encode(v, body);
    dx::mp::put_be(c.out, body.size(), 4);
    c.out.append(body);
    if (c.out.size() - c.out_off > kMaxOutbox) {
      std::fprintf(stderr, "ctrld: conn %llu outbox overflow, dropping\n", (unsigned long long)c.id);
      c.dead = true;
      return;
    }
    flush(c);
  }

  void send_to(uint64_t conn, const Value& v) {
    auto it = conns_.find(conn);
    if (it != conns_.end()) send(*it->second, v);
  }

  void flush(Conn& c) {
    while (c.out_off < c.out.size()) {
      ssize_t n = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (n > 0) {
        c.out_off += size_t(n);
        continue;
      }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      if (n < 0 && errno == EINTR) continue;
      c.dead = true;
      return;
    }
    if (c.out_off == c.out.size()) {
      c.out.clear();
      c.out_off = 0;
    } else if (c.out_off > (size_t(1) << 20)) {
      c.out.erase(0, c.out_off);
      c.out_off = 0;
    }
    bool want = !c.out.empty();
    if (want != c.want_write) {
      epoll_event ev{};
      ev.events = want ? (EPOLLIN | EPOLLOUT) : EPOLLIN;
      ev.data.u64 = c.id;
      epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &ev);
      c.want_write = want;
    }
  }

  void reap_dead() {
    for (auto it = conns_.begin(); it != conns_.end();) {
      if (!it->second->dead) {
        ++it;
        continue;
      }
      uint64_t id = it->first;
      epoll_ctl(ep_, EPOLL_CTL_DEL, it->second->fd, nullptr);
      close(it->second->fd);
      it = conns_.erase(it);
      drop_streams_of(id);
    }
  }

  void drop_streams_of(uint64_t conn) {
    for (auto* reg : {&watchers_, &subs_})
      for (auto it = reg->begin(); it != reg->end();)
        it = it->second.conn == conn ? reg->erase(it) : std::next(it);
    for (auto& [name, q] : queues_) {
      std::deque<Waiter> keep;
      for (auto& w : q.waiters)
        if (w.conn != conn) keep.push_back(w);
      q.waiters.swap(keep);
    }
  }

  // ------------------------------------------------------------- responses
  static Value ok_result(int64_t rid, Value res) {
    Value r = Value::map();
    r.set("id", Value::integer(rid));
    r.set("ok", Value::boolean(true));
    r.set("result", std::move(res));
    return r;
  }
  static Value ok_item(int64_t rid, Value item) {
    Value r = Value::map();
    r.set("id", Value::integer(rid));
    r.set("ok", Value::boolean(true));
    r.set("item", std::move(item));
    return r;
  }
  static Value err(int64_t rid, const std::string& what) {
    Value r = Value::map();
    r.set("id", Value::integer(rid));
    r.set("ok", Value::boolean(false));
    r.set("error", Value::str(what));
    return r;
  }

  static const Value& need(const Value& m, const char* k) {
    const Value* v = m.get(k);
    if (!v) throw std::runtime_error(std::string("KeyError: '") + k + "'");
    return *v;
  }
  static std::string need_str(const Value& m, const char* k) {
    const Value& v = need(m, k);
    if (v.t != Value::T::Str && v.t != Value::T::Bin) throw std::runtime_error(std::string("TypeError: ") + k);
    return v.s;
  }
  static double opt_num(const Value& m, const char* k, double dflt) {
    const Value* v = m.get(k);
    return (v && !v->is_nil()) ? v->num() : dflt;
  }
  static std::optional<int64_t> opt_int(const Value& m, const char* k) {
    const Value* v = m.get(k);
    if (!v || v->is_nil()) return std::nullopt;
    if (v->t != Value::T::Int) throw std::runtime_error(std::string("TypeError: ") + k);
    return v->i;
  }

  // ------------------------------------------------------------- kv
  void notify(const char* kind, const std::string& key, const Value* value, int64_t rev) {
    if (watchers_.empty()) return;
    Value ev;
    bool built = false;
    for (auto& [wid, w] : watchers_) {
      if (key.compare(0, w.pattern.size(), w.pattern) != 0) continue;
      if (!built) {
        ev = Value::map();
        ev.set("type", Value::str(kind));
        ev.set("key", Value::str(key));
        ev.set("value", value ? *value : Value::nil());
        ev.set("rev", Value::integer(rev));
        built = true;
      }
      send_to(w.conn, ok_item(w.rid, ev));
    }
  }

  int64_t put(const std::string& key, Value value, std::optional<int64_t> lease) {
    if (lease) {
      auto it = leases_.find(*lease);
      if (it == leases_.end()) throw std::runtime_error("KeyError: 'lease " + std::to_string(*lease) + " not found'");
      it->second.keys.insert(key);
    }
    auto old = kv_.find(key);
    if (old != kv_.end() && old->second.lease && old->second.lease != lease) {
      auto ol = leases_.find(*old->second.lease);
      if (ol != leases_.end()) ol->second.keys.erase(key);
    }
    ++rev_;
    Entry& e = kv_[key];
    e.value = std::move(value);
    e.rev = rev_;
    e.lease = lease;
    notify("put", key, &e.value, rev_);
    return rev_;
  }

  int del(const std::string& key) {
    auto it = kv_.find(key);
    if (it == kv_.end()) return 0;
    if (it->second.lease) {
      auto l = leases_.find(*it->second.lease);
      if (l != leases_.end()) l->second.keys.erase(key);
    }
    kv_.erase(it);
    ++rev_;
    notify("delete", key, nullptr, rev_);
    return 1;
  }

  int revoke(int64_t lid) {
    auto it = leases_.find(lid);
    if (it == leases_.end()) return 0;
    std::set<std::string> keys = std::move(it->second.keys);
    leases_.erase(it);
    int n = 0;
    for (auto& k : keys) {
      auto e = kv_.find(k);
      if (e != kv_.end() && e->second.lease == lid) n += del(k);
    }
    return n;
  }

  Value items_with_prefix(const std::string& p) const {
    Value items = Value::arr();
    for (auto it = kv_.lower_bound(p); it != kv_.end() && it->first.compare(0, p.size(), p) == 0; ++it) {
      Value row = Value::arr();
      row.a.push_back(Value::str(it->first));
      row.a.push_back(it->second.value);
      row.a.push_back(Value::integer(it->second.rev));
      items.a.push_back(std::move(row));
    }
    return items;
  }

  // ------------------------------------------------------------- queues
  Value pop_deliver(Queue& q, double ack_wait) {
    QMsg m = std::move(q.ready.front());
    q.ready.pop_front();
    m.deliveries += 1;
    m.deadline = mono() + ack_wait;
    Value r = Value::map();
    r.set("seq", Value::integer(m.seq));
    r.set("data", m.data);
    r.set("deliveries", Value::integer(m.deliveries));
    q.inflight[m.seq] = std::move(m);
    return r;
  }

  void q_wake(Queue& q) {
    while (!q.waiters.empty() && !q.ready.empty()) {
      Waiter w = q.waiters.front();
      q.waiters.pop_front();
      auto it = conns_.find(w.conn);
      if (it == conns_.end() || it->second->dead) continue;
      send(*it->second, ok_result(w.rid, pop_deliver(q, w.ack_wait)));
    }
  }

  // ------------------------------------------------------------- timers
  void tick(double now) {
    std::vector<int64_t> expired;
    for (auto& [id, l] : leases_)
      if (l.deadline < now) expired.push_back(id);
    for (int64_t id : expired) revoke(id);
    for (auto& [name, q] : queues_) {
      std::vector<int64_t> late;
      for (auto& [seq, m] : q.inflight)
        if (m.deadline < now) late.push_back(seq);
      for (auto it = late.rbegin(); it != late.rend(); ++it) {  // oldest ends up first
        q.ready.push_front(std::move(q.inflight[*it]));
        q.inflight.erase(*it);
      }
      if (!late.empty()) q_wake(q);
      std::deque<Waiter> keep;
      for (auto& w : q.waiters) {
        if (w.deadline <= now) send_to(w.conn, ok_result(w.rid, Value::nil()));
        else keep.push_back(w);
      }
      q.waiters.swap(keep);
    }
    for (auto& [bucket, m] : blobs_)
      for (auto it = m.begin(); it != m.end();)
        it = (it->second.expires >= 0 && it->second.expires < now) ? m.erase(it) : std::next(it);
  }

  // ------------------------------------------------------------- dispatch
  void dispatch(Conn& c, const Value& msg) {
    const Value* idv = msg.get("id");
    const Value* opv = msg.get("op");
    int64_t rid = (idv && idv->t == Value::T::Int) ? idv->i : 0;
    if (!opv || opv->t != Value::T::Str) {
      send(c, err(rid, "ValueError: missing op"));
      return;
    }
    const std::string& op = opv->s;
    op_stats_[op] += 1;
    try {
      if (op == "cancel") {
        auto t = opt_int(msg, "target");
        if (t) cancel_stream(c.id, *t);
        return;
      }
      if (op == "watch") {
        std::string p = need_str(msg, "prefix");
        Value snap = Value::map();
        snap.set("type", Value::str("snapshot"));
        snap.set("items", items_with_prefix(p));
        snap.set("rev", Value::integer(rev_));
        send(c, ok_item(rid, std::move(snap)));
        watchers_[next_wid_++] = StreamReg{c.id, rid, p};
        return;
      }
      if (op == "subscribe") {
        subs_[next_wid_++] = StreamReg{c.id, rid, need_str(msg, "subject")};
        Value it = Value::map();
        it.set("type", Value::str("subscribed"));
        send(c, ok_item(rid, std::move(it)));
        return;
      }
      if (op == "q_pop") {
        Queue& q = queues_[need_str(msg, "queue")];
        double timeout = opt_num(msg, "timeout", 1.0);
        double ack_wait = opt_num(msg, "ack_wait", 30.0);
        if (!q.ready.empty()) send(c, ok_result(rid, pop_deliver(q, ack_wait)));
        else if (timeout <= 0) send(c, ok_result(rid, Value::nil()));
        else q.waiters.push_back(Waiter{c.id, rid, mono() + timeout, ack_wait});
        return;
      }
      send(c, ok_result(rid, unary(op, msg)));
    } catch (const std::exception& e) {
      send(c, err(rid, e.what()));
    }
  }

  void cancel_stream(uint64_t conn, int64_t rid) {
    for (auto* reg : {&watchers_, &subs_})
      for (auto it = reg->begin(); it != reg->end();)
        it = (it->second.conn == conn && it->second.rid == rid) ? reg->erase(it) : std::next(it);
    for (auto& [name, q] : queues_) {
      std::deque<Waiter> keep;
      for (auto& w : q.waiters)
        if (!(w.conn == conn && w.rid == rid)) keep.push_back(w);
      q.waiters.swap(keep);
    }
  }

  Value unary(const std::string& op, const Value& m) {
    Value r = Value::map();
    if (op == "ping") {
      r.set("rev", Value::integer(rev_));
      r.set("time", Value::flt(wall()));
    } else if (op == "put") {
      r.set("rev", Value::integer(put(need_str(m, "key"), need(m, "value"), opt_int(m, "lease"))));
    } else if (op == "create") {
      std::string key = need_str(m, "key");
      auto it = kv_.find(key);
      if (it != kv_.end()) {
        r.set("ok", Value::boolean(false));
        r.set("rev", Value::integer(it->second.rev));
      } else {
        r.set("ok", Value::boolean(true));
        r.set("rev", Value::integer(put(key, need(m, "value"), opt_int(m, "lease"))));
      }
    } else if (op == "create_or_validate") {
      std::string key = need_str(m, "key");
      const Value& val = need(m, "value");
      auto it = kv_.find(key);
      if (it == kv_.end()) {
        r.set("ok", Value::boolean(true));
        r.set("rev", Value::integer(put(key, val, opt_int(m, "lease"))));
      } else {
        bool same = it->second.value.t == val.t && it->second.value.s == val.s;
        r.set("ok", Value::boolean(same));
        r.set("rev", Value::integer(it->second.rev));
      }
    } else if (op == "get") {
      auto it = kv_.find(need_str(m, "key"));
      if (it == kv_.end()) return Value::nil();
      r.set("value", it->second.value);
      r.set("rev", Value::integer(it->second.rev));
      r.set("lease", it->second.lease ? Value::integer(*it->second.lease) : Value::nil());
    } else if (op == "get_prefix") {
      r.set("items", items_with_prefix(need_str(m, "prefix")));
      r.set("rev", Value::integer(rev_));
    } else if (op == "delete") {
      r.set("deleted", Value::integer(del(need_str(m, "key"))));
    } else if (op == "delete_prefix") {
      std::string p = need_str(m, "prefix");
      std::vector<std::string> keys;
      for (auto it = kv_.lower_bound(p); it != kv_.end() && it->first.compare(0, p.size(), p) == 0; ++it)
        keys.push_back(it->first);
      int n = 0;
      for (auto& k : keys) n += del(k);
      r.set("deleted", Value::integer(n));
    } else if (op == "lease_grant") {
      int64_t lid = lease_next_++;
      double ttl = opt_num(m, "ttl", 10.0);
      leases_[lid] = Lease{ttl, mono() + ttl, {}};
      r.set("lease", Value::integer(lid));
      r.set("ttl", Value::flt(ttl));
    } else if (op == "lease_keepalive") {
      auto it = leases_.find(need(m, "lease").i);
      if (it == leases_.end()) {
        r.set("ok", Value::boolean(false));
      } else {
        it->second.deadline = mono() + it->second.ttl;
        r.set("ok", Value::boolean(true));
        r.set("ttl", Value::flt(it->second.ttl));
      }
    } else if (op == "lease_revoke") {
      r.set("deleted", Value::integer(revoke(need(m, "lease").i)));
    } else if (op == "lease_alive") {
      r.set("ok", Value::boolean(leases_.count(need(m, "lease").i) > 0));
    } else if (op == "publish") {
      std::string subj = need_str(m, "subject");
      const Value& data = need(m, "data");
      int n = 0;
      Value item;
      bool built = false;
      for (auto& [sid, s] : subs_) {
        if (!subject_matches(s.pattern, subj)) continue;
        if (!built) {
          item = Value::map();
          item.set("subject", Value::str(subj));
          item.set("data", data);
          built = true;
        }
        send_to(s.conn, ok_item(s.rid, item));
        ++n;
      }
      r.set("delivered", Value::integer(n));
    } else if (op == "q_push") {
      Queue& q = queues_[need_str(m, "queue")];
      QMsg msg;
      msg.seq = ++q.seq;
      msg.data = need(m, "data");
      q.ready.push_back(std::move(msg));
      r.set("seq", Value::integer(q.seq));
      q_wake(q);
    } else if (op == "q_ack") {
      Queue& q = queues_[need_str(m, "queue")];
      r.set("ok", Value::boolean(q.inflight.erase(need(m, "seq").i) > 0));
    } else if (op == "q_nak") {
      Queue& q = queues_[need_str(m, "queue")];
      auto it = q.inflight.find(need(m, "seq").i);
      bool found = it != q.inflight.end();
      if (found) {
        q.ready.push_front(std::move(it->second));
        q.inflight.erase(it);
        q_wake(q);
      }
      r.set("ok", Value::boolean(found));
    } else if (op == "q_size") {
      Queue& q = queues_[need_str(m, "queue")];
      r.set("pending", Value::integer(int64_t(q.ready.size())));
      r.set("inflight", Value::integer(int64_t(q.inflight.size())));
    } else if (op == "blob_put") {
      double ttl = opt_num(m, "ttl", 0.0);
      blobs_[need_str(m, "bucket")][need_str(m, "key")] = Blob{need(m, "data"), ttl > 0 ? mono() + ttl : -1.0};
      r.set("ok", Value::boolean(true));
    } else if (op == "blob_get") {
      auto b = blobs_.find(need_str(m, "bucket"));
      if (b == blobs_.end()) return Value::nil();
      auto it = b->second.find(need_str(m, "key"));
      return it == b->second.end() ? Value::nil() : it->second.data;
    } else if (op == "blob_list") {
      Value l = Value::arr();
      auto b = blobs_.find(need_str(m, "bucket"));
      if (b != blobs_.end())
        for (auto& [k, v] : b->second) l.a.push_back(Value::str(k));
      return l;
    } else if (op == "blob_delete") {
      auto b = blobs_.find(need_str(m, "bucket"));
      bool found = b != blobs_.end() && b->second.erase(need_str(m, "key")) > 0;
      r.set("ok", Value::boolean(found));
    } else if (op == "stats") {
      r.set("keys", Value::integer(int64_t(kv_.size())));
      r.set("leases", Value::integer(int64_t(leases_.size())));
      r.set("rev", Value::integer(rev_));
      r.set("watchers", Value::integer(int64_t(watchers_.size())));
      r.set("subs", Value::integer(int64_t(subs_.size())));
      Value qs = Value::map();
      for (auto& [name, q] : queues_) qs.set(name, Value::integer(int64_t(q.ready.size())));
      r.set("queues", std::move(qs));
      Value ops = Value::map();
      for (auto& [name, n] : op_stats_) ops.set(name, Value::integer(n));
      r.set("ops", std::move(ops));
      r.set("server", Value::str("native"));
    } else {
      throw std::runtime_error("ValueError: unknown op " + op);
    }
    return r;
  }
};

void on_signal(int) { g_stop = 1; }

}  // namespace

int main(int argc, char** argv) {
  std::string host = "0.0.0.0";
  int port = 4850;
  if (const char* env = std::getenv("DX_CONTROL_PLANE")) {
    std::string a(env);
    auto colon = a.rfind(':');
    if (colon != std::string::npos) port = std::atoi(a.c_str() + colon + 1);
  }
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--host" && i + 1 < argc) host = argv[++i];
    else if (a == "--port" && i + 1 < argc) port = std::atoi(argv[++i]);
    else if (a == "--exit-with-parent" || a == "--parent-pid") {
      // a child server (e.g. the bench's rank 0) must not outlive its parent,
      // however the parent ends.  The parent-death signal only fires for a
      // death after prctl; a parent that already died shows as a changed
      // getppid().  Compare against the pid the parent passed: a parent that
      // is itself pid 1 (a container entrypoint) is a live parent.
      long expect = -1;
      if (a == "--parent-pid" && i + 1 < argc) expect = std::atol(argv[++i]);
      ::prctl(PR_SET_PDEATHSIG, SIGTERM);
      if (expect > 0 ? (long)::getppid() != expect : ::getppid() == 1) return 0;
    } else if (a == "-h" || a == "--help") {
      std::printf("usage: dx-ctrld [--host H] [--port P] [--exit-with-parent | --parent-pid PID]   (port 0 = ephemeral)\n");
      return 0;
    } else {
      std::fprintf(stderr, "dx-ctrld: unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  std::signal(SIGPIPE, SIG_IGN);
  std::signal(SIGINT, on_signal);
  std::signal(SIGTERM, on_signal);
  Server s(host, port);
  return s.listen_and_serve();
}
