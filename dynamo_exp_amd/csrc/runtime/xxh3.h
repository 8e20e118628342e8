// Self-contained XXH3-64 (seeded) implementation, scalar path.
//
// Written from the public XXH3 specification so the KV router, the engine's
// prefix cache and the two-part wire codec hash identically to the reference
// (xxhash-rust `xxh3_64_with_seed`, seed 1337 for KV blocks; see
// lib/llm/src/kv_router/indexer.rs:64,87 and lib/llm/src/tokens.rs:109-243).
// Verified against the `xxhash` Python package for every length 0..4096 in
// tests/test_runtime_native.py.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace dx {
namespace xxh3 {

constexpr uint64_t P32_1 = 0x9E3779B1ULL, P32_2 = 0x85EBCA77ULL, P32_3 = 0xC2B2AE3DULL;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ULL, P64_2 = 0xC2B2AE3D27D4EB4FULL, P64_3 = 0x165667B19E3779F9ULL,
                   P64_4 = 0x85EBCA77C2B2AE63ULL, P64_5 = 0x27D4EB2F165667C5ULL;

alignas(64) constexpr uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c, 0xde, 0xd4, 0x6d,
    0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f, 0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0,
    0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21, 0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0,
    0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c, 0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b,
    0x1b, 0x53, 0x2e, 0xa3, 0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac,
    0xd8, 0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d, 0x8a, 0x51,
    0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64, 0xea, 0xc5, 0xac, 0x83, 0x34,
    0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb, 0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49,
    0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e, 0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8,
    0xd1, 0x7a, 0xd0, 0x31, 0xce, 0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b,
    0x40, 0x7e,
};

inline uint64_t r64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;  // little-endian host (x86-64)
}
inline uint32_t r32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline void w64(uint8_t* p, uint64_t v) { std::memcpy(p, &v, 8); }
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t swap64(uint64_t x) { return __builtin_bswap64(x); }
inline uint32_t swap32(uint32_t x) { return __builtin_bswap32(x); }

inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
  __uint128_t p = (__uint128_t)a * b;
  return (uint64_t)p ^ (uint64_t)(p >> 64);
}
inline uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}
inline uint64_t avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= 0x165667919E3779F9ULL;
  h ^= h >> 32;
  return h;
}
inline uint64_t rrmxmx(uint64_t h, uint64_t len) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= 0x9FB21C651E98DF25ULL;
  h ^= (h >> 35) + len;
  h *= 0x9FB21C651E98DF25ULL;
  return h ^ (h >> 28);
}

inline uint64_t len_1to3(const uint8_t* in, size_t len, const uint8_t* s, uint64_t seed) {
  const uint8_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
  const uint32_t combined = ((uint32_t)c1 << 16) | ((uint32_t)c2 << 24) | ((uint32_t)c3 << 0) | ((uint32_t)len << 8);
  const uint64_t bitflip = (uint64_t)(r32(s) ^ r32(s + 4)) + seed;
  return xxh64_avalanche((uint64_t)combined ^ bitflip);
}
inline uint64_t len_4to8(const uint8_t* in, size_t len, const uint8_t* s, uint64_t seed) {
  seed ^= (uint64_t)swap32((uint32_t)seed) << 32;
  const uint32_t i1 = r32(in), i2 = r32(in + len - 4);
  const uint64_t bitflip = (r64(s + 8) ^ r64(s + 16)) - seed;
  const uint64_t i64 = i2 + ((uint64_t)i1 << 32);
  return rrmxmx(i64 ^ bitflip, len);
}
inline uint64_t len_9to16(const uint8_t* in, size_t len, const uint8_t* s, uint64_t seed) {
  const uint64_t bf1 = (r64(s + 24) ^ r64(s + 32)) + seed;
  const uint64_t bf2 = (r64(s + 40) ^ r64(s + 48)) - seed;
  const uint64_t lo = r64(in) ^ bf1;
  const uint64_t hi = r64(in + len - 8) ^ bf2;
  const uint64_t acc = len + swap64(lo) + hi + mul128_fold64(lo, hi);
  return avalanche(acc);
}
inline uint64_t len_0to16(const uint8_t* in, size_t len, const uint8_t* s, uint64_t seed) {
  if (len > 8) return len_9to16(in, len, s, seed);
  if (len >= 4) return len_4to8(in, len, s, seed);
  if (len) return len_1to3(in, len, s, seed);
  return xxh64_avalanche(seed ^ (r64(s + 56) ^ r64(s + 64)));
}
inline uint64_t mix16(const uint8_t* in, const uint8_t* s, uint64_t seed) {
  return mul128_fold64(r64(in) ^ (r64(s) + seed), r64(in + 8) ^ (r64(s + 8) - seed));
}
inline uint64_t len_17to128(const uint8_t* in, size_t len, const uint8_t* s, uint64_t seed) {
  uint64_t acc = len * P64_1;
  if (len > 32) {
    if (len > 64) {
      if (len > 96) {
        acc += mix16(in + 48, s + 96, seed);
        acc += mix16(in + len - 64, s + 112, seed);
      }
      acc += mix16(in + 32, s + 64, seed);
      acc += mix16(in + len - 48, s + 80, seed);
    }
    acc += mix16(in + 16, s + 32, seed);
    acc += mix16(in + len - 32, s + 48, seed);
  }
  acc += mix16(in, s, seed);
  acc += mix16(in + len - 16, s + 16, seed);
  return avalanche(acc);
}
inline uint64_t len_129to240(const uint8_t* in, size_t len, const uint8_t* s, uint64_t seed) {
  uint64_t acc = len * P64_1;
  const int rounds = (int)len / 16;
  for (int i = 0; i < 8; ++i) acc += mix16(in + 16 * i, s + 16 * i, seed);
  acc = avalanche(acc);
  for (int i = 8; i < rounds; ++i) acc += mix16(in + 16 * i, s + 16 * (i - 8) + 3, seed);
  acc += mix16(in + len - 16, s + 136 - 17, seed);
  return avalanche(acc);
}

inline void accumulate_512(uint64_t* acc, const uint8_t* in, const uint8_t* s) {
  for (int i = 0; i < 8; ++i) {
    const uint64_t dv = r64(in + 8 * i);
    const uint64_t dk = dv ^ r64(s + 8 * i);
    acc[i ^ 1] += dv;
    acc[i] += (uint64_t)(uint32_t)dk * (dk >> 32);
  }
}
inline void scramble(uint64_t* acc, const uint8_t* s) {
  for (int i = 0; i < 8; ++i) {
    uint64_t a = acc[i];
    a ^= a >> 47;
    a ^= r64(s + 8 * i);
    a *= P32_1;
    acc[i] = a;
  }
}
inline uint64_t hash_long(const uint8_t* in, size_t len, const uint8_t* s, size_t ssize) {
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  const size_t stripes_per_block = (ssize - 64) / 8;
  const size_t block_len = 64 * stripes_per_block;
  const size_t nb_blocks = (len - 1) / block_len;
  for (size_t n = 0; n < nb_blocks; ++n) {
    for (size_t st = 0; st < stripes_per_block; ++st) accumulate_512(acc, in + n * block_len + st * 64, s + st * 8);
    scramble(acc, s + ssize - 64);
  }
  const size_t nb_stripes = ((len - 1) - block_len * nb_blocks) / 64;
  for (size_t st = 0; st < nb_stripes; ++st) accumulate_512(acc, in + nb_blocks * block_len + st * 64, s + st * 8);
  accumulate_512(acc, in + len - 64, s + ssize - 64 - 7);
  uint64_t result = len * P64_1;
  for (int i = 0; i < 4; ++i) result += mul128_fold64(acc[2 * i] ^ r64(s + 11 + 16 * i), acc[2 * i + 1] ^ r64(s + 11 + 16 * i + 8));
  return avalanche(result);
}

inline uint64_t hash64(const void* data, size_t len, uint64_t seed = 0) {
  const uint8_t* in = static_cast<const uint8_t*>(data);
  if (len <= 16) return len_0to16(in, len, kSecret, seed);
  if (len <= 128) return len_17to128(in, len, kSecret, seed);
  if (len <= 240) return len_129to240(in, len, kSecret, seed);
  if (seed == 0) return hash_long(in, len, kSecret, sizeof(kSecret));
  alignas(64) uint8_t secret[192];
  for (int i = 0; i < 12; ++i) {
    w64(secret + 16 * i, r64(kSecret + 16 * i) + seed);
    w64(secret + 16 * i + 8, r64(kSecret + 16 * i + 8) - seed);
  }
  return hash_long(in, len, secret, sizeof(secret));
}

}  // namespace xxh3
}  // namespace dx
