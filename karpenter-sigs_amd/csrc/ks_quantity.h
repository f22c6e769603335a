// ks_quantity.h — k8s resource.Quantity values for the encoder and the result renderer.
//
// The device works on int64 fixed-point vectors (ks_problem.h); this header parses snapshot
// quantity strings into exact nano-unit integers, remembers the apimachinery Format that
// String() depends on, and renders the canonical String() of sums (Merge keeps the Format of the
// first addend that lands on a zero running value; quantity.go Add/Sub).
#pragma once
#include <cctype>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace ks {

enum class QFmt : uint8_t { None = 0, DecExp = 1, BinSI = 2, DecSI = 3 };

struct Qty {
  __int128 n = 0;  // value in nano-units (exact)
  QFmt f = QFmt::None;
  void add(const Qty& y) {
    if (n == 0) f = y.f;
    n += y.n;
  }
};

inline std::string i128str(__int128 v) {
  if (v == 0) return "0";
  bool neg = v < 0;
  unsigned __int128 u = neg ? (unsigned __int128)(-v) : (unsigned __int128)v;
  char buf[64];
  int i = 63;
  buf[i] = 0;
  while (u) { buf[--i] = char('0' + (int)(u % 10)); u /= 10; }
  if (neg) buf[--i] = '-';
  return std::string(buf + i);
}

// resource.ParseQuantity: [sign] digits [. digits] suffix; sub-nano precision rounds up.
inline Qty qty_parse(const std::string& s) {
  Qty q;
  if (s.empty()) throw std::runtime_error("empty quantity");
  if (s == "0") { q.f = QFmt::DecSI; return q; }
  size_t i = 0;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') { neg = s[i] == '-'; i++; }
  __int128 mant = 0;
  int ndigits = 0, frac = 0;
  bool dot = false;
  for (; i < s.size(); i++) {
    char c = s[i];
    if (c >= '0' && c <= '9') {
      if (mant != 0 || c != '0') ndigits++;
      if (ndigits > 36) throw std::runtime_error("quantity too precise: " + s);
      mant = mant * 10 + (c - '0');
      if (dot) frac++;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  std::string suf = s.substr(i);
  int e10 = 0, e2 = 0;
  QFmt f = QFmt::DecSI;
  static const struct { const char* s; int e10, e2; QFmt f; } tab[] = {
      {"", 0, 0, QFmt::DecSI},   {"n", -9, 0, QFmt::DecSI}, {"u", -6, 0, QFmt::DecSI},
      {"m", -3, 0, QFmt::DecSI}, {"k", 3, 0, QFmt::DecSI},  {"M", 6, 0, QFmt::DecSI},
      {"G", 9, 0, QFmt::DecSI},  {"T", 12, 0, QFmt::DecSI}, {"P", 15, 0, QFmt::DecSI},
      {"E", 18, 0, QFmt::DecSI}, {"Ki", 0, 10, QFmt::BinSI}, {"Mi", 0, 20, QFmt::BinSI},
      {"Gi", 0, 30, QFmt::BinSI}, {"Ti", 0, 40, QFmt::BinSI}, {"Pi", 0, 50, QFmt::BinSI},
      {"Ei", 0, 60, QFmt::BinSI},
  };
  bool found = false;
  for (auto& t : tab)
    if (suf == t.s) { e10 = t.e10; e2 = t.e2; f = t.f; found = true; break; }
  if (!found) {
    if (suf.size() >= 2 && (suf[0] == 'e' || suf[0] == 'E')) {
      size_t k = 1;
      if (suf[k] == '+' || suf[k] == '-') k++;
      if (k >= suf.size()) throw std::runtime_error("bad quantity: " + s);
      for (size_t m = k; m < suf.size(); m++)
        if (!std::isdigit((unsigned char)suf[m])) throw std::runtime_error("bad quantity: " + s);
      e10 = std::stoi(suf.substr(1));
      f = QFmt::DecExp;
    } else {
      throw std::runtime_error("bad quantity suffix: " + s);
    }
  }
  for (int k = 0; k < e2; k++) mant *= 2;
  int shift = 9 + e10 - frac;  // to nano
  if (shift > 30) throw std::runtime_error("quantity out of range: " + s);
  if (shift >= 0) {
    for (int k = 0; k < shift; k++) mant *= 10;
  } else {
    __int128 p = 1;
    for (int k = 0; k < -shift; k++) p *= 10;
    __int128 r = mant % p;
    mant /= p;
    if (r) mant += 1;
  }
  q.n = neg ? -mant : mant;
  q.f = f;
  return q;
}

// Quantity.String() (CanonicalizeBytes).
inline std::string qty_str(const Qty& q) {
  if (q.n == 0) return "0";
  QFmt f = q.f;
  const __int128 G = 1000000000;
  if (f == QFmt::BinSI && (q.n % G != 0 || (q.n > -1024 * G && q.n < 1024 * G))) f = QFmt::DecSI;
  if (f == QFmt::None) f = QFmt::DecExp;
  bool neg = q.n < 0;
  __int128 v = neg ? -q.n : q.n;
  if (f == QFmt::BinSI) {
    v /= G;
    int e = 0;
    while (v >= 1024 && v % 1024 == 0 && e < 6) { v /= 1024; e++; }
    static const char* bs[] = {"", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
    return i128str(neg ? -v : v) + bs[e];
  }
  int e = -9;
  while (v >= 10 && v % 10 == 0) { v /= 10; e++; }
  int r = ((e % 3) + 3) % 3;  // fold to a multiple of 3 from above
  for (int k = 0; k < r; k++) { v *= 10; e--; }
  std::string num = i128str(neg ? -v : v);
  if (f == QFmt::DecSI) {
    switch (e) {
      case -9: return num + "n";
      case -6: return num + "u";
      case -3: return num + "m";
      case 0: return num;
      case 3: return num + "k";
      case 6: return num + "M";
      case 9: return num + "G";
      case 12: return num + "T";
      case 15: return num + "P";
      case 18: return num + "E";
      default: return num;
    }
  }
  return e == 0 ? num : num + "e" + std::to_string(e);
}

}  // namespace ks
