// quantity.h — CPU restatement of the k8s.io/apimachinery v0.28.4 `resource.Quantity` subset the
// scheduler hot path uses (test infrastructure only).
//
// Third-party dependency (not vendored under /root/reference): k8s.io/apimachinery v0.28.4
// (go.mod:26).  Call sites on the path: pkg/utils/resources/resources.go:33,56-57,91,120,158,165
// (Merge/Subtract/Cmp/Fits), scheduler.go:376-380 (Sub), existingnode.go:47-50
// (AsApproximateFloat64 sign, Set(0)).  Published algorithm restated: ParseQuantity (suffix table
// n u m "" k M G T P E / Ki..Ei / e<exp>, rounding up to nano precision), Add/Sub (a zero receiver
// adopts the argument's Format), Cmp, and String() = CanonicalizeBytes (trailing decimal zeros
// folded into an exponent that is a multiple of 3; BinarySI only when the value is an integer
// outside (-1024, 1024)).  Values are held exactly as an __int128 count of nano-units.
#pragma once
#include <cctype>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace oq {

enum class Format { None, DecimalExponent, BinarySI, DecimalSI };

struct Quantity {
  __int128 nano = 0;  // value * 1e9, exact
  Format fmt = Format::None;

  bool is_zero() const { return nano == 0; }
  int sign() const { return nano < 0 ? -1 : (nano > 0 ? 1 : 0); }
  void add(const Quantity& y) {
    if (nano == 0) fmt = y.fmt;
    nano += y.nano;
  }
  void sub(const Quantity& y) {
    if (nano == 0) fmt = y.fmt;
    nano -= y.nano;
  }
  int cmp(const Quantity& y) const { return nano < y.nano ? -1 : (nano > y.nano ? 1 : 0); }
  std::string str() const;
};

inline __int128 pow10i(int e) {
  __int128 r = 1;
  for (int i = 0; i < e; i++) r *= 10;
  return r;
}

inline std::string i128_to_string(__int128 v) {
  if (v == 0) return "0";
  bool neg = v < 0;
  unsigned __int128 u = neg ? (unsigned __int128)(-v) : (unsigned __int128)v;
  std::string s;
  while (u) { s.insert(s.begin(), char('0' + (int)(u % 10))); u /= 10; }
  if (neg) s.insert(s.begin(), '-');
  return s;
}

// NewQuantity(value, format) / NewMilliQuantity.
inline Quantity make(int64_t value, Format f) {
  Quantity q;
  q.nano = (__int128)value * 1000000000;
  q.fmt = f;
  return q;
}

// ParseQuantity restatement.  Throws on malformed input (MustParse panics in Go).
inline Quantity parse(const std::string& str) {
  if (str.empty()) throw std::runtime_error("quantity: empty");
  Quantity q;
  if (str == "0") { q.fmt = Format::DecimalSI; return q; }
  size_t pos = 0, end = str.size();
  bool positive = true;
  if (str[0] == '-') { positive = false; pos++; }
  else if (str[0] == '+') pos++;
  while (pos < end && str[pos] == '0') pos++;  // leading zeros
  std::string num, denom;
  size_t i = pos;
  while (i < end && std::isdigit((unsigned char)str[i])) i++;
  num = str.substr(pos, i - pos);
  pos = i;
  if (num.empty()) num = "0";
  if (pos < end && str[pos] == '.') {
    pos++;
    i = pos;
    while (i < end && std::isdigit((unsigned char)str[i])) i++;
    denom = str.substr(pos, i - pos);
    pos = i;
  }
  std::string suf = str.substr(pos);
  int base = 10, exponent = 0;
  Format f;
  if (suf.empty()) { f = Format::DecimalSI; }
  else if (suf == "n") { f = Format::DecimalSI; exponent = -9; }
  else if (suf == "u") { f = Format::DecimalSI; exponent = -6; }
  else if (suf == "m") { f = Format::DecimalSI; exponent = -3; }
  else if (suf == "k") { f = Format::DecimalSI; exponent = 3; }
  else if (suf == "M") { f = Format::DecimalSI; exponent = 6; }
  else if (suf == "G") { f = Format::DecimalSI; exponent = 9; }
  else if (suf == "T") { f = Format::DecimalSI; exponent = 12; }
  else if (suf == "P") { f = Format::DecimalSI; exponent = 15; }
  else if (suf == "E") { f = Format::DecimalSI; exponent = 18; }
  else if (suf == "Ki") { f = Format::BinarySI; base = 2; exponent = 10; }
  else if (suf == "Mi") { f = Format::BinarySI; base = 2; exponent = 20; }
  else if (suf == "Gi") { f = Format::BinarySI; base = 2; exponent = 30; }
  else if (suf == "Ti") { f = Format::BinarySI; base = 2; exponent = 40; }
  else if (suf == "Pi") { f = Format::BinarySI; base = 2; exponent = 50; }
  else if (suf == "Ei") { f = Format::BinarySI; base = 2; exponent = 60; }
  else if (suf[0] == 'e' || suf[0] == 'E') {
    size_t k = 1;
    if (k < suf.size() && (suf[k] == '+' || suf[k] == '-')) k++;
    if (k >= suf.size()) throw std::runtime_error("quantity: bad exponent");
    for (size_t m = k; m < suf.size(); m++)
      if (!std::isdigit((unsigned char)suf[m])) throw std::runtime_error("quantity: bad exponent");
    f = Format::DecimalExponent;
    exponent = std::stoi(suf.substr(1));
  } else {
    throw std::runtime_error("quantity: unknown suffix '" + suf + "'");
  }
  std::string digits = num + denom;
  if (digits.size() > 36) throw std::runtime_error("quantity: too many digits");
  __int128 m = 0;
  for (char c : digits) m = m * 10 + (c - '0');
  // value = m * 10^(-len(denom)) * base^exponent ; store nano = value * 1e9, rounded away from 0.
  int e10 = 9 - (int)denom.size();
  if (base == 10) e10 += exponent;
  else {
    for (int k = 0; k < exponent; k++) m *= 2;
  }
  if (e10 >= 0) {
    if (e10 > 30) throw std::runtime_error("quantity: out of range");
    m *= pow10i(e10);
  } else {
    __int128 p = pow10i(-e10);
    __int128 qv = m / p;
    if (m % p != 0) qv += 1;  // RoundUp at nano scale
    m = qv;
  }
  q.nano = positive ? m : -m;
  q.fmt = f;
  return q;
}

inline std::string Quantity::str() const {
  if (nano == 0) return "0";
  Format f = fmt;
  if (f == Format::BinarySI) {
    __int128 lim = (__int128)1024 * 1000000000;
    if (nano > -lim && nano < lim) f = Format::DecimalSI;
    else if (nano % 1000000000 != 0) f = Format::DecimalSI;
  } else if (f == Format::None) {
    f = Format::DecimalExponent;
  }
  if (f == Format::BinarySI) {
    __int128 v = nano / 1000000000;
    bool neg = v < 0;
    if (neg) v = -v;
    int e = 0;
    while (v >= 1024 && v % 1024 == 0) { v /= 1024; e++; }
    if (neg) v = -v;
    static const char* bs[] = {"", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
    return i128_to_string(v) + (e <= 6 ? bs[e] : "");
  }
  __int128 v = nano;
  bool neg = v < 0;
  if (neg) v = -v;
  int e = -9;
  while (v >= 10 && v % 10 == 0) { v /= 10; e++; }
  int r = e % 3;  // C++ truncated modulo == Go's
  if (r == 1 || r == -2) { v *= 10; e -= 1; }
  else if (r == 2 || r == -1) { v *= 100; e -= 2; }
  if (neg) v = -v;
  std::string s = i128_to_string(v);
  if (f == Format::DecimalSI) {
    switch (e) {
      case -9: return s + "n";
      case -6: return s + "u";
      case -3: return s + "m";
      case 0: return s;
      case 3: return s + "k";
      case 6: return s + "M";
      case 9: return s + "G";
      case 12: return s + "T";
      case 15: return s + "P";
      case 18: return s + "E";
      default: return s;  // outside the SI table (not reachable for realistic inputs)
    }
  }
  if (e == 0) return s;
  return s + "e" + std::to_string(e);
}

}  // namespace oq
