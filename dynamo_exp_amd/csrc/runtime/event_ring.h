// Single-producer / multi-consumer broadcast ring in POSIX shared memory:
// the per-step event plane of the tensor-parallel engine (parallel/tp.py).
//
// The TP leader publishes each step's input events (new requests, aborts,
// KV-transfer events, its step clock) once; every follower rank on the node
// reads the same byte string in the same order.  This replaces a pickled
// gloo broadcast per step (a TCP round trip through the gloo store/pairs) by
// a memcpy into shared memory plus a release store; a follower that is
// already waiting sees it within its spin window.
//
// Layout: Header | nslots x Slot.  A message longer than one slot is split
// into fragments (kMore flag).  The producer reuses slot s for sequence
// number q only after every consumer acknowledged q - nslots, so a slow
// follower back-pressures the leader instead of losing events.  Sequence
// numbers are published with release stores and read with acquire loads.
// Waits spin briefly, then back off with nanosleep; callers release the GIL
// around them.  Peer liveness: the header records the producer's and every
// consumer's pid; a wait that backs off checks them a few times a second and
// throws when the other side died (SIGKILL included: no `closed` flag is ever
// set then), so a follower whose leader vanished -- or a leader whose
// follower vanished with the ring full -- fails instead of spinning forever.
#pragma once

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace dx {

class EventRing {
 public:
  static constexpr uint64_t kMagic = 0x6478657672696e67ull;  // "dxevring"
  static constexpr uint32_t kMaxConsumers = 64;
  static constexpr uint32_t kMore = 1;

  // producer side: creates (and owns) the segment
  static EventRing create(const std::string& name, uint32_t nslots, uint32_t slot_bytes, uint32_t nconsumers) {
    if (nslots < 2 || slot_bytes < 64 || nconsumers > kMaxConsumers) throw std::invalid_argument("EventRing: bad size");
    EventRing r;
    r.name_ = name;
    r.owner_ = true;
    r.bytes_ = sizeof(Header) + (size_t)nslots * slot_stride(slot_bytes);
    int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("EventRing: shm_open(create) failed for " + name);
    if (ftruncate(fd, (off_t)r.bytes_) != 0) {
      close(fd);
      shm_unlink(name.c_str());
      throw std::runtime_error("EventRing: ftruncate failed");
    }
    r.map(fd);
    Header* h = r.hdr();
    h->nslots = nslots;
    h->slot_bytes = slot_bytes;
    h->nconsumers = nconsumers;
    h->head.store(0, std::memory_order_relaxed);
    h->closed.store(0, std::memory_order_relaxed);
    h->producer_pid.store((int32_t)getpid(), std::memory_order_relaxed);
    for (uint32_t i = 0; i < kMaxConsumers; ++i) {
      h->acked[i].v.store(0, std::memory_order_relaxed);
      h->consumer_pid[i].store(0, std::memory_order_relaxed);
    }
    for (uint32_t s = 0; s < nslots; ++s) r.slot(s)->seq.store(0, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    h->magic.store(kMagic, std::memory_order_release);
    return r;
  }

  // consumer side: attaches as consumer `idx` (0 .. nconsumers-1)
  static EventRing attach(const std::string& name, uint32_t idx) {
    EventRing r;
    r.name_ = name;
    int fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("EventRing: shm_open(attach) failed for " + name);
    struct stat st;
    if (fstat(fd, &st) != 0) {
      close(fd);
      throw std::runtime_error("EventRing: fstat failed");
    }
    r.bytes_ = (size_t)st.st_size;
    r.map(fd);
    if (r.hdr()->magic.load(std::memory_order_acquire) != kMagic) throw std::runtime_error("EventRing: bad segment");
    if (idx >= r.hdr()->nconsumers) throw std::invalid_argument("EventRing: consumer index out of range");
    r.consumer_ = (int)idx;
    r.next_ = r.hdr()->acked[idx].v.load(std::memory_order_acquire) + 1;
    r.hdr()->consumer_pid[idx].store((int32_t)getpid(), std::memory_order_release);
    return r;
  }

  EventRing() = default;
  EventRing(const EventRing&) = delete;
  EventRing& operator=(const EventRing&) = delete;
  EventRing(EventRing&& o) noexcept { *this = std::move(o); }
  EventRing& operator=(EventRing&& o) noexcept {
    if (this != &o) {
      release();
      base_ = o.base_;
      bytes_ = o.bytes_;
      name_ = std::move(o.name_);
      owner_ = o.owner_;
      consumer_ = o.consumer_;
      next_ = o.next_;
      o.base_ = nullptr;
      o.owner_ = false;
    }
    return *this;
  }
  ~EventRing() { release(); }

  // Publish one message (blocks while the ring is full).  Returns false if
  // `timeout_s` (< 0: forever) expired waiting for slow consumers.
  bool publish(const uint8_t* data, size_t n, double timeout_s = -1.0) {
    Header* h = hdr();
    const uint32_t sb = h->slot_bytes;
    size_t off = 0;
    do {
      const uint32_t len = (uint32_t)std::min<size_t>(sb, n - off);
      const uint64_t q = h->head.load(std::memory_order_relaxed) + 1;
      if (q > h->nslots && !wait_acked(q - h->nslots, timeout_s)) return false;
      Slot* s = slot((uint32_t)(q % h->nslots));
      s->len = len;
      s->flags = (off + len < n) ? kMore : 0;
      if (len) std::memcpy(s->data, data + off, len);
      s->seq.store(q, std::memory_order_release);
      h->head.store(q, std::memory_order_release);
      off += len;
    } while (off < n);
    return true;
  }

  // Next message for this consumer; false on timeout (`timeout_s` < 0:
  // forever) or when the producer closed the ring and everything was read.
  bool poll(std::vector<uint8_t>& out, double timeout_s = -1.0) {
    out.clear();
    Header* h = hdr();
    for (;;) {
      Slot* s = slot((uint32_t)(next_ % h->nslots));
      if (!wait_seq(s, next_, timeout_s)) return false;
      const uint32_t len = s->len, flags = s->flags;
      const size_t o = out.size();
      out.resize(o + len);
      if (len) std::memcpy(out.data() + o, s->data, len);
      h->acked[consumer_].v.store(next_, std::memory_order_release);
      ++next_;
      if (!(flags & kMore)) return true;
    }
  }

  void close_ring() { hdr()->closed.store(1, std::memory_order_release); }
  bool closed() const { return hdr()->closed.load(std::memory_order_acquire) != 0; }
  uint64_t head() const { return hdr()->head.load(std::memory_order_acquire); }
  const std::string& name() const { return name_; }
  // A pid is gone when it no longer exists or is a zombie (a dead child its
  // parent has not reaped yet still answers kill(pid, 0)).
  static bool pid_alive(int32_t pid) {
    if (pid <= 0) return true;
    if (kill(pid, 0) != 0 && errno == ESRCH) return false;
    char path[64];
    std::snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
    FILE* f = std::fopen(path, "r");
    if (!f) return true;  // no procfs view: trust kill()
    char buf[512];
    size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char* rp = std::strrchr(buf, ')');  // "pid (comm) S ..."
    return !(rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
  }
  bool peers_alive() const {
    const Header* h = hdr();
    if (consumer_ >= 0) return pid_alive(h->producer_pid.load(std::memory_order_acquire));
    for (uint32_t c = 0; c < h->nconsumers; ++c)
      if (!pid_alive(h->consumer_pid[c].load(std::memory_order_acquire))) return false;
    return true;
  }
  void unlink() {
    if (!name_.empty()) shm_unlink(name_.c_str());
  }

 private:
  struct alignas(64) Counter {
    std::atomic<uint64_t> v;
  };
  struct Header {
    std::atomic<uint64_t> magic;
    uint32_t nslots, slot_bytes, nconsumers, pad;
    alignas(64) std::atomic<uint64_t> head;
    alignas(64) std::atomic<uint32_t> closed;
    std::atomic<int32_t> producer_pid;
    std::atomic<int32_t> consumer_pid[kMaxConsumers];
    Counter acked[kMaxConsumers];
  };
  struct Slot {
    std::atomic<uint64_t> seq;
    uint32_t len, flags;
    uint8_t data[1];
  };
  static size_t slot_stride(uint32_t sb) { return (offsetof(Slot, data) + sb + 63) / 64 * 64; }

  Header* hdr() const { return reinterpret_cast<Header*>(base_); }
  Slot* slot(uint32_t i) const {
    return reinterpret_cast<Slot*>(base_ + sizeof(Header) + (size_t)i * slot_stride(hdr()->slot_bytes));
  }

  void map(int fd) {
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("EventRing: mmap failed");
    base_ = static_cast<uint8_t*>(p);
  }
  void release() {
    if (base_) munmap(base_, bytes_);
    if (owner_) unlink();
    base_ = nullptr;
    owner_ = false;
  }

  // spin ~20 us, then back off 5 us -> 200 us
  template <typename Ready>
  bool wait_until(Ready ready, double timeout_s) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int i = 0; i < 2000; ++i) {
      if (ready()) return true;
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    }
    long ns = 5000;
    auto last_check = t0;
    for (;;) {
      if (ready()) return true;
      const auto now = clk::now();
      if (timeout_s >= 0 && std::chrono::duration<double>(now - t0).count() > timeout_s) return ready();
      if (std::chrono::duration<double>(now - last_check).count() > 0.25) {
        last_check = now;
        if (!peers_alive()) {
          if (ready()) return true;
          throw std::runtime_error("EventRing: peer process died (" + name_ + ")");
        }
      }
      struct timespec ts{0, ns};
      nanosleep(&ts, nullptr);
      ns = std::min(ns * 2, 200000L);
    }
  }
  bool wait_acked(uint64_t q, double timeout_s) {
    Header* h = hdr();
    return wait_until([&] {
      for (uint32_t c = 0; c < h->nconsumers; ++c)
        if (h->acked[c].v.load(std::memory_order_acquire) < q) return false;
      return true;
    }, timeout_s);
  }
  bool wait_seq(Slot* s, uint64_t q, double timeout_s) {
    return wait_until([&] {
      return s->seq.load(std::memory_order_acquire) == q ||
             (closed() && hdr()->head.load(std::memory_order_acquire) < q);
    }, timeout_s) && s->seq.load(std::memory_order_acquire) == q;
  }

  uint8_t* base_ = nullptr;
  size_t bytes_ = 0;
  std::string name_;
  bool owner_ = false;
  int consumer_ = -1;
  uint64_t next_ = 1;
};

}  // namespace dx
