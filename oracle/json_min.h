// json_min.h — minimal JSON DOM reader/writer for the oracle (test infrastructure only).
// Objects keep keys in a std::map (Go maps are unordered; every consumer here either sorts or
// ignores order), arrays keep order. Numbers are kept as their literal text so int64 / float64
// callers can parse them exactly.
#pragma once
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ojson {

struct Value;
using Object = std::map<std::string, Value>;
using Array = std::vector<Value>;

struct Value {
  enum Kind { Null, Bool, Number, String, Arr, Obj } kind = Null;
  bool b = false;
  std::string s;  // String payload or Number literal
  std::shared_ptr<Array> a;
  std::shared_ptr<Object> o;

  bool is_null() const { return kind == Null; }
  bool is_obj() const { return kind == Obj; }
  bool is_arr() const { return kind == Arr; }
  bool is_str() const { return kind == String; }
  const Value* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    auto it = o->find(k);
    return it == o->end() ? nullptr : &it->second;
  }
  const Array& arr() const {
    static const Array empty;
    return kind == Arr ? *a : empty;
  }
  const Object& obj() const {
    static const Object empty;
    return kind == Obj ? *o : empty;
  }
  std::string str(const std::string& dflt = "") const { return kind == String ? s : dflt; }
  int64_t i64(int64_t dflt = 0) const {
    if (kind == Number) return std::strtoll(s.c_str(), nullptr, 10);
    return dflt;
  }
  double f64(double dflt = 0) const {
    if (kind == Number) return std::strtod(s.c_str(), nullptr);
    return dflt;
  }
  bool boolean(bool dflt = false) const { return kind == Bool ? b : dflt; }
};

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), end_(p + n) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != end_) fail("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* end_;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() {
    while (p_ < end_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  Value value() {
    ws();
    if (p_ >= end_) fail("unexpected end");
    char c = *p_;
    Value v;
    if (c == '{') {
      ++p_;
      v.kind = Value::Obj;
      v.o = std::make_shared<Object>();
      ws();
      if (p_ < end_ && *p_ == '}') { ++p_; return v; }
      for (;;) {
        ws();
        if (p_ >= end_ || *p_ != '"') fail("expected key");
        std::string k = string();
        ws();
        if (p_ >= end_ || *p_ != ':') fail("expected ':'");
        ++p_;
        (*v.o)[k] = value();
        ws();
        if (p_ < end_ && *p_ == ',') { ++p_; continue; }
        if (p_ < end_ && *p_ == '}') { ++p_; break; }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      ++p_;
      v.kind = Value::Arr;
      v.a = std::make_shared<Array>();
      ws();
      if (p_ < end_ && *p_ == ']') { ++p_; return v; }
      for (;;) {
        v.a->push_back(value());
        ws();
        if (p_ < end_ && *p_ == ',') { ++p_; continue; }
        if (p_ < end_ && *p_ == ']') { ++p_; break; }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.kind = Value::String;
      v.s = string();
    } else if (c == 't' || c == 'f' || c == 'n') {
      auto lit = [&](const char* w, size_t n) {
        if ((size_t)(end_ - p_) < n || std::string(p_, n) != w) fail("bad literal");
        p_ += n;
      };
      if (c == 't') { lit("true", 4); v.kind = Value::Bool; v.b = true; }
      else if (c == 'f') { lit("false", 5); v.kind = Value::Bool; v.b = false; }
      else { lit("null", 4); }
    } else {
      const char* s = p_;
      while (p_ < end_ && (std::isdigit((unsigned char)*p_) || *p_ == '-' || *p_ == '+' || *p_ == '.' ||
                           *p_ == 'e' || *p_ == 'E'))
        ++p_;
      if (s == p_) fail("bad value");
      v.kind = Value::Number;
      v.s.assign(s, p_);
    }
    return v;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    }
  }
  std::string string() {
    ++p_;  // opening quote
    std::string out;
    while (p_ < end_ && *p_ != '"') {
      char c = *p_++;
      if (c != '\\') { out += c; continue; }
      if (p_ >= end_) fail("bad escape");
      char e = *p_++;
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          if (end_ - p_ < 4) fail("bad \\u");
          uint32_t cp = std::strtoul(std::string(p_, 4).c_str(), nullptr, 16);
          p_ += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && end_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            uint32_t lo = std::strtoul(std::string(p_ + 2, 4).c_str(), nullptr, 16);
            p_ += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (p_ >= end_) fail("unterminated string");
    ++p_;
    return out;
  }
};

inline Value parse(const std::string& s) { return Parser(s.data(), s.size()).parse(); }

// ---- writer helpers -------------------------------------------------------------------------
inline void quote(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof buf, "\\u%04x", c);
          out += buf;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

}  // namespace ojson
