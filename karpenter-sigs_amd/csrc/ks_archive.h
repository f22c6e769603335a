// ks_archive.h — binary snapshot of an encoded problem (SURVEY.md §5 "binary problem file").
//
// One symmetric visitor per host type lists its members once; the same list writes (Out) and reads (In).
// Trivially copyable members and vectors of them go as raw bytes; strings, maps, sets and nested vectors
// as a length followed by their elements.  A snapshot starts with a magic, a format version and the sizes
// of the device-facing structs, so a blob from another build is refused rather than misread.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace ks {

struct ArchiveError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct ArOut {
  std::string buf;
  static constexpr bool reading = false;
  void raw(const void* p, size_t n) { buf.append((const char*)p, n); }
};

struct ArIn {
  const char* p;
  const char* end;
  static constexpr bool reading = true;
  void raw(void* dst, size_t n) {
    if ((size_t)(end - p) < n) throw ArchiveError("binary snapshot truncated");
    std::memcpy(dst, p, n);
    p += n;
  }
  // A length read from the blob must be backed by at least `n` more bytes before anything is allocated for
  // it: a corrupt length is then a parse error, not a multi-GB allocation.
  void need(uint64_t n) const {
    if ((uint64_t)(end - p) < n) throw ArchiveError("binary snapshot length exceeds the remaining bytes");
  }
};

template <class A, class T>
typename std::enable_if<std::is_trivially_copyable<T>::value && !std::is_pointer<T>::value>::type io(A& a, T& v) {
  if constexpr (A::reading) a.raw(&v, sizeof(T));
  else a.raw(&v, sizeof(T));
}

template <class A>
void io_len(A& a, uint64_t& n) {
  io(a, n);
  if (A::reading && n > (1ull << 34)) throw ArchiveError("binary snapshot length out of range");
}

template <class A>
void io(A& a, std::string& s) {
  uint64_t n = s.size();
  io_len(a, n);
  if constexpr (A::reading) {
    a.need(n);
    s.resize(n);
    if (n) a.raw(&s[0], n);
  } else if (n) {
    a.raw(s.data(), n);
  }
}

template <class A, class T>
void io(A& a, std::vector<T>& v) {
  uint64_t n = v.size();
  io_len(a, n);
  constexpr bool raw = std::is_trivially_copyable<T>::value && !std::is_same<T, bool>::value;
  if constexpr (A::reading) {
    if constexpr (raw) {
      a.need(n * sizeof(T));  // raw elements take exactly sizeof(T): the bytes must be there before the allocation
      v.resize(n);
      if (n) a.raw(v.data(), n * sizeof(T));
    } else {
      // an element's encoded size is not bounded below by its in-memory size (an empty PodH is a few bytes,
      // 640 in memory): the vector grows only with elements actually decoded, so a corrupt count runs out of
      // input (ArchiveError) before it can force a large allocation
      a.need(n);
      v.clear();
      v.reserve((size_t)std::min<uint64_t>(n, 1u << 12));
      for (uint64_t i = 0; i < n; i++) {
        T x{};
        io(a, x);
        v.push_back(std::move(x));
      }
    }
  } else if constexpr (raw) {
    if (n) a.raw(v.data(), n * sizeof(T));
  } else {
    for (auto& x : v) io(a, x);
  }
}

template <class A, class K, class V>
void io(A& a, std::pair<K, V>& p) {
  io(a, p.first);
  io(a, p.second);
}

template <class A, class K, class V, class C>
void io(A& a, std::map<K, V, C>& m) {
  uint64_t n = m.size();
  io_len(a, n);
  if constexpr (A::reading) {
    m.clear();
    for (uint64_t i = 0; i < n; i++) {
      std::pair<K, V> kv;
      io(a, kv);
      m.emplace_hint(m.end(), std::move(kv.first), std::move(kv.second));
    }
  } else {
    for (auto& kv : m) {
      K k = kv.first;
      io(a, k);
      io(a, kv.second);
    }
  }
}

template <class A, class T, class C>
void io(A& a, std::set<T, C>& s) {
  uint64_t n = s.size();
  io_len(a, n);
  if constexpr (A::reading) {
    s.clear();
    for (uint64_t i = 0; i < n; i++) {
      T x;
      io(a, x);
      s.emplace_hint(s.end(), std::move(x));
    }
  } else {
    for (auto& x : s) {
      T y = x;
      io(a, y);
    }
  }
}

template <class A, class T>
void io(A& a, std::shared_ptr<T>& p) {
  uint8_t has = p ? 1 : 0;
  io(a, has);
  if constexpr (A::reading) p = has ? std::make_shared<T>() : nullptr;
  if (has) io(a, *p);
}

// variadic member list
template <class A, class... T>
void io_all(A& a, T&... xs) {
  (io(a, xs), ...);
}

}  // namespace ks
