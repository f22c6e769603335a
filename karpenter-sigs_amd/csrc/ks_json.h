// ks_json.h — JSON DOM reader/writer for snapshot input and results output.
// Objects are key-sorted flat vectors (iteration order equals a std::map's: Go maps are unordered and
// every consumer here either sorts or ignores order; a duplicate key keeps its last value), arrays keep
// order.  Numbers are kept as their literal text so int64 / float64 callers can parse them exactly.
// Snapshots are tens of MB (C5: 45 MB, 100k pods): large arrays near the top of the document (pods,
// stateNodes, clusterPods) are split at element boundaries by a skip scan and their elements parsed by
// worker threads (ks_parallel.h), each into its own slot.
#pragma once
#include <mutex>
#include <deque>
#include <condition_variable>
#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <utility>
#include <vector>

#include "ks_parallel.h"

namespace ksjson {

struct Value;
using Array = std::vector<Value>;

// Key-sorted (key, value) pairs: the subset of std::map's interface the decoders use.
struct Object {
  using Entry = std::pair<std::string, Value>;
  std::vector<Entry> e;
  Object() = default;
  std::vector<Entry>::const_iterator begin() const { return e.begin(); }
  std::vector<Entry>::const_iterator end() const { return e.end(); }
  std::vector<Entry>::iterator begin() { return e.begin(); }
  std::vector<Entry>::iterator end() { return e.end(); }
  size_t size() const { return e.size(); }
  bool empty() const { return e.empty(); }
  const Value* find(std::string_view k) const;
  Value& operator[](const std::string& k);
  void finish();  // sort by key; on duplicates the last one parsed wins
};

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
  const Value* get(std::string_view k) const { return kind == Obj ? o->find(k) : nullptr; }
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

inline const Value* Object::find(std::string_view k) const {
  if (e.size() <= 8) {  // decoder objects are small: a scan beats the binary search
    for (auto& x : e)
      if (x.first == k) return &x.second;
    return nullptr;
  }
  auto it = std::lower_bound(e.begin(), e.end(), k, [](const Entry& x, std::string_view key) { return x.first < key; });
  return it != e.end() && it->first == k ? &it->second : nullptr;
}
inline Value& Object::operator[](const std::string& k) {
  auto it = std::lower_bound(e.begin(), e.end(), k, [](const Entry& x, const std::string& key) { return x.first < key; });
  if (it != e.end() && it->first == k) return it->second;
  return e.insert(it, Entry(k, Value()))->second;
}
inline void Object::finish() {
  std::stable_sort(e.begin(), e.end(), [](const Entry& x, const Entry& y) { return x.first < y.first; });
  size_t w = 0;
  for (size_t i = 0; i < e.size(); i++) {
    if (w > 0 && e[w - 1].first == e[i].first) e[w - 1].second = std::move(e[i].second);  // last wins
    else if (w != i) e[w++] = std::move(e[i]);
    else w++;
  }
  e.resize(w);
}

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), end_(p + n) {}
  Value parse() {
    Value v = value(0);
    ws();
    if (p_ != end_) fail("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* end_;
  static constexpr int kParallelDepth = 3;          // arrays this close to the root may be split
  static constexpr size_t kParallelBytes = 1 << 20;  // ... when they span at least this many bytes
  static constexpr size_t kParallelMinElems = 256;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() {
    while (p_ < end_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  // Skip one value without building it (structure only: strings with escapes, nesting).
  void skip() {
    ws();
    if (p_ >= end_) fail("unexpected end");
    const char c = *p_;
    if (c == '"') {
      skip_string();
    } else if (c == '{' || c == '[') {
      int depth = 0;
      while (p_ < end_) {
        const char x = *p_;
        if (x == '"') {
          skip_string();
          continue;
        }
        ++p_;
        if (x == '{' || x == '[') depth++;
        else if (x == '}' || x == ']') {
          if (--depth == 0) return;
        }
      }
      fail("unterminated container");
    } else {
      while (p_ < end_ && *p_ != ',' && *p_ != ']' && *p_ != '}' && *p_ != ' ' && *p_ != '\n' && *p_ != '\r' &&
             *p_ != '\t')
        ++p_;
    }
  }
  void skip_string() {
    ++p_;
    while (p_ < end_) {
      const char x = *p_++;
      if (x == '\\') {
        if (p_ >= end_) fail("bad escape");
        ++p_;
      } else if (x == '"') {
        return;
      }
    }
    fail("unterminated string");
  }
  // A large array: element extents by a skip scan, then the elements parsed in parallel.
  bool array_parallel(Value& v, int depth) {
    const char* start = p_;
    std::vector<std::pair<const char*, const char*>> ext;
    for (;;) {
      ws();
      const char* b = p_;
      skip();
      ext.push_back({b, p_});
      ws();
      if (p_ < end_ && *p_ == ',') { ++p_; continue; }
      if (p_ < end_ && *p_ == ']') { ++p_; break; }
      fail("expected ',' or ']'");
    }
    if (ext.size() < kParallelMinElems || (size_t)(p_ - start) < kParallelBytes) {
      p_ = start;  // small after all: the sequential path
      return false;
    }
    v.a->resize(ext.size());
    Array& out = *v.a;
    ks::parallel_for((int)ext.size(), 64, [&](int i) {
      Parser sub(ext[(size_t)i].first, (size_t)(ext[(size_t)i].second - ext[(size_t)i].first));
      out[(size_t)i] = sub.value(depth + 1);
    });
    return true;
  }
  Value value(int depth) {
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
      // entries collect on a per-thread stack (nested objects above them), then move into one
      // exactly sized buffer: no growth reallocations
      static thread_local std::vector<Object::Entry> stack;
      const size_t base = stack.size();
      struct Cut {  // an exception from any nested value leaves this thread's stack at `base`
        std::vector<Object::Entry>& s;
        size_t b;
        ~Cut() {
          if (s.size() > b) s.resize(b);
        }
      } cut{stack, base};
      for (;;) {
        ws();
        if (p_ >= end_ || *p_ != '"') fail("expected key");
        std::string k = string();
        ws();
        if (p_ >= end_ || *p_ != ':') fail("expected ':'");
        ++p_;
        Value x = value(depth + 1);
        stack.emplace_back(std::move(k), std::move(x));
        ws();
        if (p_ < end_ && *p_ == ',') { ++p_; continue; }
        if (p_ < end_ && *p_ == '}') { ++p_; break; }
        fail("expected ',' or '}'");
      }
      v.o->e.reserve(stack.size() - base);
      for (size_t i = base; i < stack.size(); i++) v.o->e.push_back(std::move(stack[i]));
      stack.resize(base);
      v.o->finish();
    } else if (c == '[') {
      ++p_;
      v.kind = Value::Arr;
      v.a = std::make_shared<Array>();
      ws();
      if (p_ < end_ && *p_ == ']') { ++p_; return v; }
      if (depth < kParallelDepth && (size_t)(end_ - p_) >= kParallelBytes && ks::parallel_threads() > 1 &&
          array_parallel(v, depth))
        return v;
      for (;;) {
        v.a->push_back(value(depth + 1));
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
    const char* b = p_;  // fast path: no escape before the closing quote
    while (p_ < end_ && *p_ != '"' && *p_ != '\\') ++p_;
    if (p_ < end_ && *p_ == '"') {
      std::string out(b, p_);
      ++p_;
      return out;
    }
    std::string out(b, p_);
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

// Destroy (large) documents on one long-lived worker thread: their ~millions of frees leave the caller's
// critical path (ks_problem_create / ks_cons_create return while the snapshot DOM is still being
// released).  The worker drains its queue and is joined when the library is unloaded (static destructor),
// so no free races process exit.
class Reaper {
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Value*> q_;
  bool stop_ = false;
  std::thread th_;
  void run() {
    for (;;) {
      Value* p;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        p = q_.front();
        q_.pop_front();
      }
      delete p;
    }
  }

 public:
  void push(Value* p) {
    {
      std::lock_guard<std::mutex> l(mu_);
      if (!th_.joinable()) th_ = std::thread([this] { run(); });
      q_.push_back(p);
    }
    cv_.notify_one();
  }
  ~Reaper() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_one();
    if (th_.joinable()) th_.join();
  }
};
inline Reaper& reaper() {
  static Reaper r;
  return r;
}
inline void release_async(Value&& v) { reaper().push(new Value(std::move(v))); }

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

}  // namespace ksjson
