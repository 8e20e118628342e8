// libdynamo_llm_capi: KV event publishing for external engines over the
// control plane (see include/dynamo_exp_amd/kv_events.h).  Wire: u32-BE
// length + msgpack map {id, op:"publish", subject, data: bin(json event)};
// every request is answered by one reply frame which is read and checked.
#include "dynamo_exp_amd/kv_events.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../runtime/xxh3.h"

namespace {

constexpr uint64_t kBlockSeed = 1337;

struct Publisher {
  int fd = -1;
  std::string subject;
  int64_t worker_id = 0;
  uint32_t block_size = 0;
  uint64_t next_id = 1;
  std::mutex mu;
};

Publisher* g_pub = nullptr;
std::mutex g_init_mu;

// ---------------------------------------------------------------- msgpack
void mp_str(std::string& o, const std::string& s) {
  size_t n = s.size();
  if (n < 32) {
    o.push_back(char(0xa0 | n));
  } else if (n < 256) {
    o.push_back(char(0xd9));
    o.push_back(char(n));
  } else {
    o.push_back(char(0xda));
    o.push_back(char(n >> 8));
    o.push_back(char(n));
  }
  o += s;
}

void mp_uint(std::string& o, uint64_t v) {
  if (v < 128) {
    o.push_back(char(v));
  } else {
    o.push_back(char(0xcf));
    for (int i = 7; i >= 0; --i) o.push_back(char(v >> (8 * i)));
  }
}

void mp_bin(std::string& o, const std::string& b) {
  uint32_t n = uint32_t(b.size());
  o.push_back(char(0xc6));
  for (int i = 3; i >= 0; --i) o.push_back(char(n >> (8 * i)));
  o += b;
}

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    p += k;
    n -= size_t(k);
  }
  return true;
}

bool recv_all(int fd, char* p, size_t n) {
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) return false;
    p += k;
    n -= size_t(k);
  }
  return true;
}

// reply map contains "ok": true|false; scan for the key followed by 0xc3 (true)
bool reply_ok(const std::string& r) {
  static const char key[] = {char(0xa2), 'o', 'k'};
  size_t pos = r.find(std::string(key, 3));
  return pos != std::string::npos && pos + 3 < r.size() && uint8_t(r[pos + 3]) == 0xc3;
}

dynamo_llm_result_t publish(Publisher* p, const std::string& json) {
  std::lock_guard<std::mutex> g(p->mu);
  std::string m;
  m.push_back(char(0x84));  // fixmap, 4 entries
  mp_str(m, "id");
  mp_uint(m, p->next_id++);
  mp_str(m, "op");
  mp_str(m, "publish");
  mp_str(m, "subject");
  mp_str(m, p->subject);
  mp_str(m, "data");
  mp_bin(m, json);
  uint32_t n = htonl(uint32_t(m.size()));
  if (!send_all(p->fd, reinterpret_cast<const char*>(&n), 4) || !send_all(p->fd, m.data(), m.size()))
    return DYNAMO_ERR;
  uint32_t rn;
  if (!recv_all(p->fd, reinterpret_cast<char*>(&rn), 4)) return DYNAMO_ERR;
  std::string r(ntohl(rn), '\0');
  if (!recv_all(p->fd, r.data(), r.size())) return DYNAMO_ERR;
  return reply_ok(r) ? DYNAMO_OK : DYNAMO_ERR;
}

int connect_to(const std::string& addr) {
  auto colon = addr.rfind(':');
  if (colon == std::string::npos) return -1;
  std::string host = addr.substr(0, colon), port = addr.substr(colon + 1);
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0) return -1;
  int fd = -1;
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype, a->ai_protocol);
    if (fd < 0) continue;
    if (::connect(fd, a->ai_addr, a->ai_addrlen) == 0) break;
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd >= 0) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  return fd;
}

}  // namespace

extern "C" {

dynamo_llm_result_t dynamo_llm_init(const char* ns, const char* component, int64_t worker_id,
                                    uint32_t kv_block_size) {
  std::lock_guard<std::mutex> g(g_init_mu);
  if (g_pub != nullptr || !ns || !component || kv_block_size == 0) return DYNAMO_ERR;
  const char* env = std::getenv("DX_CONTROL_PLANE");
  int fd = connect_to(env && *env ? env : "127.0.0.1:4850");
  if (fd < 0) return DYNAMO_ERR;
  auto* p = new Publisher;
  p->fd = fd;
  p->subject = std::string("namespace.") + ns + ".component." + component + ".kv_events";
  p->worker_id = worker_id;
  p->block_size = kv_block_size;
  g_pub = p;
  return DYNAMO_OK;
}

dynamo_llm_result_t dynamo_llm_shutdown(void) {
  std::lock_guard<std::mutex> g(g_init_mu);
  if (!g_pub) return DYNAMO_ERR;
  ::close(g_pub->fd);
  delete g_pub;
  g_pub = nullptr;
  return DYNAMO_OK;
}

dynamo_llm_result_t dynamo_kv_event_publish_stored(uint64_t event_id, const uint32_t* token_ids,
                                                   const size_t* num_block_tokens, const uint64_t* block_ids,
                                                   size_t num_blocks, const uint64_t* parent_hash,
                                                   uint64_t /*lora_id*/) {
  Publisher* p = g_pub;
  if (!p) return DYNAMO_ERR;
  std::string js = "{\"worker_id\":" + std::to_string(p->worker_id) + ",\"event_id\":" + std::to_string(event_id) +
                   ",\"stored_parent\":" + (parent_hash ? std::to_string(*parent_hash) : std::string("null")) +
                   ",\"stored\":[";
  size_t off = 0;
  for (size_t i = 0; i < num_blocks; ++i) {
    size_t n = num_block_tokens[i];
    if (n != p->block_size) break;  // partial block: drop it and the rest
    uint64_t th = dx::xxh3::hash64(token_ids + off, n * sizeof(uint32_t), kBlockSeed);
    off += n;
    if (i) js += ",";
    js += "{\"block_hash\":" + std::to_string(block_ids[i]) + ",\"tokens_hash\":" + std::to_string(th) + "}";
  }
  js += "],\"removed\":[]}";
  return publish(p, js);
}

dynamo_llm_result_t dynamo_kv_event_publish_removed(uint64_t event_id, const uint64_t* block_ids,
                                                    size_t num_blocks) {
  Publisher* p = g_pub;
  if (!p) return DYNAMO_ERR;
  std::string js = "{\"worker_id\":" + std::to_string(p->worker_id) + ",\"event_id\":" + std::to_string(event_id) +
                   ",\"stored_parent\":null,\"stored\":[],\"removed\":[";
  for (size_t i = 0; i < num_blocks; ++i) {
    if (i) js += ",";
    js += std::to_string(block_ids[i]);
  }
  js += "]}";
  return publish(p, js);
}

}  // extern "C"
