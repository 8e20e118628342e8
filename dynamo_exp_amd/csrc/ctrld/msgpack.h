// Minimal MessagePack value, decoder and encoder for the control-plane wire
// (u32-BE length + msgpack map per frame, runtime/wire.py).  Covers the types
// the Python clients send: nil, bool, int/uint, float32/64, str, bin, array,
// map.  Extension types are rejected.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace dx::mp {

struct Value {
  enum class T : uint8_t { Nil, Bool, Int, Float, Str, Bin, Arr, Map };
  T t = T::Nil;
  bool b = false;
  int64_t i = 0;  // Int (uint64 values above INT64_MAX are not used by the protocol)
  double f = 0;
  std::string s;  // Str / Bin payload
  std::vector<Value> a;
  std::vector<std::pair<Value, Value>> m;

  static Value nil() { return {}; }
  static Value boolean(bool v) { Value x; x.t = T::Bool; x.b = v; return x; }
  static Value integer(int64_t v) { Value x; x.t = T::Int; x.i = v; return x; }
  static Value flt(double v) { Value x; x.t = T::Float; x.f = v; return x; }
  static Value str(std::string v) { Value x; x.t = T::Str; x.s = std::move(v); return x; }
  static Value bin(std::string v) { Value x; x.t = T::Bin; x.s = std::move(v); return x; }
  static Value arr() { Value x; x.t = T::Arr; return x; }
  static Value map() { Value x; x.t = T::Map; return x; }

  bool is_nil() const { return t == T::Nil; }
  // map helpers (string keys)
  const Value* get(std::string_view k) const {
    if (t != T::Map) return nullptr;
    for (auto& kv : m)
      if (kv.first.t == T::Str && kv.first.s == k) return &kv.second;
    return nullptr;
  }
  Value& set(std::string k, Value v) {
    m.emplace_back(str(std::move(k)), std::move(v));
    return m.back().second;
  }
  double num() const {
    if (t == T::Int) return double(i);
    if (t == T::Float) return f;
    throw std::runtime_error("expected a number");
  }
};

class Decoder {
 public:
  Decoder(const uint8_t* p, size_t n) : p_(p), end_(p + n) {}
  Value decode() {
    Value v = one(0);
    if (p_ != end_) throw std::runtime_error("trailing bytes in frame");
    return v;
  }

 private:
  const uint8_t* p_;
  const uint8_t* end_;

  void need(size_t n) {
    if (size_t(end_ - p_) < n) throw std::runtime_error("truncated msgpack");
  }
  uint64_t be(size_t n) {
    need(n);
    uint64_t v = 0;
    for (size_t k = 0; k < n; ++k) v = (v << 8) | p_[k];
    p_ += n;
    return v;
  }
  std::string bytes(size_t n) {
    need(n);
    std::string s(reinterpret_cast<const char*>(p_), n);
    p_ += n;
    return s;
  }
  Value one(int depth) {
    if (depth > 64) throw std::runtime_error("msgpack nesting too deep");
    need(1);
    uint8_t c = *p_++;
    if (c <= 0x7f) return Value::integer(c);
    if (c >= 0xe0) return Value::integer(int8_t(c));
    if ((c & 0xf0) == 0x80) return map_of(c & 0x0f, depth);
    if ((c & 0xf0) == 0x90) return arr_of(c & 0x0f, depth);
    if ((c & 0xe0) == 0xa0) return Value::str(bytes(c & 0x1f));
    switch (c) {
      case 0xc0: return Value::nil();
      case 0xc2: return Value::boolean(false);
      case 0xc3: return Value::boolean(true);
      case 0xc4: return Value::bin(bytes(be(1)));
      case 0xc5: return Value::bin(bytes(be(2)));
      case 0xc6: return Value::bin(bytes(be(4)));
      case 0xca: {
        uint32_t u = uint32_t(be(4));
        float f;
        std::memcpy(&f, &u, 4);
        return Value::flt(f);
      }
      case 0xcb: {
        uint64_t u = be(8);
        double d;
        std::memcpy(&d, &u, 8);
        return Value::flt(d);
      }
      case 0xcc: return Value::integer(int64_t(be(1)));
      case 0xcd: return Value::integer(int64_t(be(2)));
      case 0xce: return Value::integer(int64_t(be(4)));
      case 0xcf: return Value::integer(int64_t(be(8)));
      case 0xd0: return Value::integer(int8_t(be(1)));
      case 0xd1: return Value::integer(int16_t(be(2)));
      case 0xd2: return Value::integer(int32_t(be(4)));
      case 0xd3: return Value::integer(int64_t(be(8)));
      case 0xd9: return Value::str(bytes(be(1)));
      case 0xda: return Value::str(bytes(be(2)));
      case 0xdb: return Value::str(bytes(be(4)));
      case 0xdc: return arr_of(be(2), depth);
      case 0xdd: return arr_of(be(4), depth);
      case 0xde: return map_of(be(2), depth);
      case 0xdf: return map_of(be(4), depth);
      default: throw std::runtime_error("unsupported msgpack type");
    }
  }
  Value arr_of(size_t n, int depth) {
    if (n > size_t(end_ - p_)) throw std::runtime_error("truncated msgpack array");
    Value v = Value::arr();
    v.a.reserve(n);
    for (size_t k = 0; k < n; ++k) v.a.push_back(one(depth + 1));
    return v;
  }
  Value map_of(size_t n, int depth) {
    if (n > size_t(end_ - p_)) throw std::runtime_error("truncated msgpack map");
    Value v = Value::map();
    v.m.reserve(n);
    for (size_t k = 0; k < n; ++k) {
      Value key = one(depth + 1);
      Value val = one(depth + 1);
      v.m.emplace_back(std::move(key), std::move(val));
    }
    return v;
  }
};

inline void put_be(std::string& o, uint64_t v, int n) {
  for (int k = n - 1; k >= 0; --k) o.push_back(char((v >> (8 * k)) & 0xff));
}

inline void encode(const Value& v, std::string& o) {
  using T = Value::T;
  switch (v.t) {
    case T::Nil: o.push_back(char(0xc0)); break;
    case T::Bool: o.push_back(char(v.b ? 0xc3 : 0xc2)); break;
    case T::Int: {
      int64_t x = v.i;
      if (x >= 0) {
        if (x <= 0x7f) o.push_back(char(x));
        else if (x <= 0xff) { o.push_back(char(0xcc)); put_be(o, uint64_t(x), 1); }
        else if (x <= 0xffff) { o.push_back(char(0xcd)); put_be(o, uint64_t(x), 2); }
        else if (x <= 0xffffffffLL) { o.push_back(char(0xce)); put_be(o, uint64_t(x), 4); }
        else { o.push_back(char(0xcf)); put_be(o, uint64_t(x), 8); }
      } else {
        if (x >= -32) o.push_back(char(int8_t(x)));
        else if (x >= -128) { o.push_back(char(0xd0)); put_be(o, uint64_t(uint8_t(int8_t(x))), 1); }
        else if (x >= -32768) { o.push_back(char(0xd1)); put_be(o, uint64_t(uint16_t(int16_t(x))), 2); }
        else if (x >= INT32_MIN) { o.push_back(char(0xd2)); put_be(o, uint64_t(uint32_t(int32_t(x))), 4); }
        else { o.push_back(char(0xd3)); put_be(o, uint64_t(x), 8); }
      }
      break;
    }
    case T::Float: {
      uint64_t u;
      std::memcpy(&u, &v.f, 8);
      o.push_back(char(0xcb));
      put_be(o, u, 8);
      break;
    }
    case T::Str: {
      size_t n = v.s.size();
      if (n <= 31) o.push_back(char(0xa0 | n));
      else if (n <= 0xff) { o.push_back(char(0xd9)); put_be(o, n, 1); }
      else if (n <= 0xffff) { o.push_back(char(0xda)); put_be(o, n, 2); }
      else { o.push_back(char(0xdb)); put_be(o, n, 4); }
      o.append(v.s);
      break;
    }
    case T::Bin: {
      size_t n = v.s.size();
      if (n <= 0xff) { o.push_back(char(0xc4)); put_be(o, n, 1); }
      else if (n <= 0xffff) { o.push_back(char(0xc5)); put_be(o, n, 2); }
      else { o.push_back(char(0xc6)); put_be(o, n, 4); }
      o.append(v.s);
      break;
    }
    case T::Arr: {
      size_t n = v.a.size();
      if (n <= 15) o.push_back(char(0x90 | n));
      else if (n <= 0xffff) { o.push_back(char(0xdc)); put_be(o, n, 2); }
      else { o.push_back(char(0xdd)); put_be(o, n, 4); }
      for (auto& x : v.a) encode(x, o);
      break;
    }
    case T::Map: {
      size_t n = v.m.size();
      if (n <= 15) o.push_back(char(0x80 | n));
      else if (n <= 0xffff) { o.push_back(char(0xde)); put_be(o, n, 2); }
      else { o.push_back(char(0xdf)); put_be(o, n, 4); }
      for (auto& kv : v.m) {
        encode(kv.first, o);
        encode(kv.second, o);
      }
      break;
    }
  }
}

}  // namespace dx::mp
