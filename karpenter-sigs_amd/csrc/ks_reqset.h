// ks_reqset.h — fixed-width encoding of pkg/scheduling `Requirements` and its algebra.
//
// A Requirements map (key -> Requirement{complement, values, greaterThan, lessThan},
// pkg/scheduling/requirement.go:33-39, requirements.go:36) is encoded over a per-problem universe:
// every label key the problem mentions gets an id (< 64) and every value of that key a bit, values
// sorted lexicographically.  A record is RSW uint32 words:
//
//   [0,1] present    bit k: key k is in the map
//   [2,3] complement bit k: Requirement.complement
//   [4,5] hasGt      bit k: greaterThan != nil       [6,7] hasLt
//   [8 .. 8+4*NB)    (gt, lt) int64 pairs for the NB "bounded" keys (keys any Gt/Lt mentions)
//   [HDR .. HDR+W)   value bitsets; key k owns words [off_k, off_k + nw_k)
//
// Non-complement keys store their value set; complement keys store the excluded set already
// filtered by the key's bounds (requirement.go:153-157 filters after every Intersection, so the
// stored set is exactly what Len()/Operator()/String() observe).  Values a Requirement never names
// are represented implicitly, which is exact because every value that can appear in a
// non-complement set is in the universe.  The hostname key carries one extra "private" bit: the
// `hostname-placeholder-NNNN` value of the NodeClaim that owns the record (nodeclaim.go:48-52).
//
// All functions are __host__ __device__: the host encoder builds records with them and the HIP
// kernels evaluate Compatible / Intersects / Intersection with them.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KS_HD __host__ __device__ __forceinline__
#else
#define KS_HD inline
#endif

namespace ks {

enum : int { OP_IN = 0, OP_NOTIN = 1, OP_EXISTS = 2, OP_DNE = 3 };

struct KeyMeta {
  int32_t off;      // first value word (relative to HDR)
  int32_t nw;       // number of words
  int32_t nv;       // number of universe values (hostname: + private bit)
  int32_t bslot;    // bound slot or -1
  int32_t vint;     // offset of this key's per-value int table (bounded keys) or -1
  int32_t pad[3];
};

// The layout's table pointers are template parameters so device code keeps their address spaces
// (LDS key table, HBM value tables); the host uses plain pointers (ReqLayout).
template <class KP, class P32, class P64>
struct ReqLayoutT {
  int32_t nkeys, W, NB, HDR, RSW;
  KP keys;
  P32 wordValid;  // [W] valid-bit mask per word (padding bits zero)
  P32 vIsInt;     // [W] bit set when the value parses with strconv.Atoi
  P64 vInt;       // per-value int (indexed by keys[k].vint + bit)
};
using ReqLayout = ReqLayoutT<const KeyMeta*, const uint32_t*, const int64_t*>;

// Record accessors are templates over the record pointer type (LDS / HBM / host).
template <class P> KS_HD uint64_t rd64(P r, int i) { return (uint64_t)r[i] | ((uint64_t)r[i + 1] << 32); }
template <class P> KS_HD void wr64(P r, int i, uint64_t v) { r[i] = (uint32_t)v; r[i + 1] = (uint32_t)(v >> 32); }

template <class P> KS_HD uint64_t rs_present(P r) { return rd64(r, 0); }
template <class P> KS_HD uint64_t rs_compl(P r) { return rd64(r, 2); }
template <class P> KS_HD uint64_t rs_hasgt(P r) { return rd64(r, 4); }
template <class P> KS_HD uint64_t rs_haslt(P r) { return rd64(r, 6); }
template <class P> KS_HD int64_t rs_gt(P r, int slot) { return (int64_t)rd64(r, 8 + 4 * slot); }
template <class P> KS_HD int64_t rs_lt(P r, int slot) { return (int64_t)rd64(r, 8 + 4 * slot + 2); }
template <class P> KS_HD void rs_set_gt(P r, int slot, int64_t v) { wr64(r, 8 + 4 * slot, (uint64_t)v); }
template <class P> KS_HD void rs_set_lt(P r, int slot, int64_t v) { wr64(r, 8 + 4 * slot + 2, (uint64_t)v); }

KS_HD bool bit(uint64_t m, int k) { return (m >> k) & 1ull; }

// Values of word `w` (absolute word index) that lie within (gt, lt) — withinIntPtrs, requirement.go:238-254.
template <class LT>
KS_HD uint32_t within_word(const LT& L, int k, int wrel, bool hg, int64_t gt, bool hl, int64_t lt) {
  if (!hg && !hl) return 0xffffffffu;
  const KeyMeta km = L.keys[k];
  uint32_t isint = L.vIsInt[km.off + wrel];
  uint32_t m = 0;
  for (int b = 0; b < 32; b++) {
    if (!((isint >> b) & 1u)) continue;
    int v = wrel * 32 + b;
    if (v >= km.nv) break;
    int64_t x = L.vInt[km.vint + v];
    if (hg && gt >= x) continue;
    if (hl && lt <= x) continue;
    m |= 1u << b;
  }
  return m;
}

template <class LT, class PR>
KS_HD bool rs_any(const LT& L, PR r, int k) {
  const KeyMeta km = L.keys[k];
  for (int i = 0; i < km.nw; i++)
    if (r[L.HDR + km.off + i]) return true;
  return false;
}

// Requirement.Operator (requirement.go:197-208); a missing key reads as Exists (requirements.go:145-151).
template <class LT, class PR>
KS_HD int rs_op(const LT& L, PR r, int k) {
  if (!bit(rs_present(r), k)) return OP_EXISTS;
  bool any = rs_any(L, r, k);
  if (bit(rs_compl(r), k)) return any ? OP_NOTIN : OP_EXISTS;
  return any ? OP_IN : OP_DNE;
}

KS_HD bool op_neg(int op) { return op == OP_NOTIN || op == OP_DNE; }

// Has(value) for one universe bit (requirement.go:182-187).
template <class LT, class PR>
KS_HD bool rs_member(const LT& L, PR r, int k, int v) {
  if (!bit(rs_present(r), k)) return true;  // Get() of a missing key is Exists
  const KeyMeta km = L.keys[k];
  uint32_t w = r[L.HDR + km.off + (v >> 5)];
  bool in = (w >> (v & 31)) & 1u;
  if (!bit(rs_compl(r), k)) return in;
  if (in) return false;
  if (km.bslot < 0) return true;
  bool hg = bit(rs_hasgt(r), k), hl = bit(rs_haslt(r), k);
  if (!hg && !hl) return true;
  uint32_t wm = within_word(L, k, v >> 5, hg, hg ? rs_gt(r, km.bslot) : 0, hl, hl ? rs_lt(r, km.bslot) : 0);
  return (wm >> (v & 31)) & 1u;
}

struct KeyIx {  // the header part of a per-key Intersection result
  bool dne;     // bounds collapsed: NewRequirement(key, DoesNotExist)
  bool compl_;
  bool hg, hl;
  int64_t gt, lt;
};

template <class LT, class PA, class PB>
KS_HD KeyIx key_ix_header(const LT& L, PA a, PB b, int k) {
  KeyIx x;
  const KeyMeta km = L.keys[k];
  bool ca = bit(rs_compl(a), k), cb = bit(rs_compl(b), k);
  bool ga = bit(rs_hasgt(a), k), gb = bit(rs_hasgt(b), k);
  bool la = bit(rs_haslt(a), k), lb = bit(rs_haslt(b), k);
  x.compl_ = ca && cb;
  x.hg = ga || gb;
  x.hl = la || lb;
  x.gt = 0;
  x.lt = 0;
  if (km.bslot >= 0) {
    int64_t gta = ga ? rs_gt(a, km.bslot) : 0, gtb = gb ? rs_gt(b, km.bslot) : 0;
    int64_t lta = la ? rs_lt(a, km.bslot) : 0, ltb = lb ? rs_lt(b, km.bslot) : 0;
    x.gt = ga && gb ? (gta > gtb ? gta : gtb) : (ga ? gta : gtb);
    x.lt = la && lb ? (lta < ltb ? lta : ltb) : (la ? lta : ltb);
  }
  x.dne = x.hg && x.hl && x.gt >= x.lt;
  return x;
}

// One word of Intersection(a_k, b_k) (requirement.go:128-161) before dropping bounds.
template <class LT, class PA, class PB>
KS_HD uint32_t key_ix_word(const LT& L, PA a, PB b, int k, int wrel, const KeyIx& x) {
  const KeyMeta km = L.keys[k];
  if (x.dne) return 0;
  bool ca = bit(rs_compl(a), k), cb = bit(rs_compl(b), k);
  uint32_t wa = a[L.HDR + km.off + wrel], wb = b[L.HDR + km.off + wrel];
  uint32_t w;
  if (ca && cb) w = wa | wb;
  else if (ca) w = wb & ~wa;
  else if (cb) w = wa & ~wb;
  else w = wa & wb;
  if (x.hg || x.hl) w &= within_word(L, k, wrel, x.hg, x.gt, x.hl, x.lt);
  return w;
}

// Intersection(a_k, b_k).Len() == 0 (only non-complement results can be empty).
template <class LT, class PA, class PB>
KS_HD bool key_ix_empty(const LT& L, PA a, PB b, int k) {
  KeyIx x = key_ix_header(L, a, b, k);
  if (x.dne) return true;
  if (x.compl_) return false;
  const KeyMeta km = L.keys[k];
  for (int i = 0; i < km.nw; i++)
    if (key_ix_word(L, a, b, k, i, x)) return false;
  return true;
}

// Requirements.Compatible (requirements.go:163-174): failing keys of each kind go to the masks.
template <class LT, class PR, class PI>
KS_HD bool rs_compatible(const LT& L, PR r, PI in, uint64_t allowUndefined,
                         uint64_t* undefinedFail = nullptr, uint64_t* intersectFail = nullptr) {
  uint64_t pr = rs_present(r), pi = rs_present(in);
  uint64_t uf = 0, xf = 0;
  uint64_t cand = pi & ~allowUndefined & ~pr;
  while (cand) {
    int k = __builtin_ctzll(cand);
    cand &= cand - 1;
    if (!op_neg(rs_op(L, in, k))) uf |= 1ull << k;
  }
  uint64_t both = pr & pi;
  while (both) {
    int k = __builtin_ctzll(both);
    both &= both - 1;
    if (key_ix_empty(L, r, in, k)) {
      if (op_neg(rs_op(L, in, k)) && op_neg(rs_op(L, r, k))) continue;
      xf |= 1ull << k;
    }
  }
  if (undefinedFail) *undefinedFail = uf;
  if (intersectFail) *intersectFail = xf;
  return (uf | xf) == 0;
}

// Requirements.Intersects (requirements.go:241-258).
template <class LT, class PR, class PI>
KS_HD bool rs_intersects(const LT& L, PR r, PI in) {
  uint64_t both = rs_present(r) & rs_present(in);
  while (both) {
    int k = __builtin_ctzll(both);
    both &= both - 1;
    if (key_ix_empty(L, r, in, k)) {
      if (op_neg(rs_op(L, in, k)) && op_neg(rs_op(L, r, k))) continue;
      return false;
    }
  }
  return true;
}

// out_k = Intersection(a_k, b_k) written into `out` (out may alias a).
template <class LT, class PO, class PA, class PB>
KS_HD void rs_intersect_key(const LT& L, PO out, PA a, PB b, int k) {
  const KeyMeta km = L.keys[k];
  KeyIx x = key_ix_header(L, a, b, k);
  for (int i = 0; i < km.nw; i++) out[L.HDR + km.off + i] = key_ix_word(L, a, b, k, i, x);
  uint64_t one = 1ull << k;
  uint64_t c = rs_compl(out), hg = rs_hasgt(out), hl = rs_haslt(out);
  bool keepBounds = !x.dne && x.compl_;
  c = (x.compl_ && !x.dne) ? (c | one) : (c & ~one);
  hg = (keepBounds && x.hg) ? (hg | one) : (hg & ~one);
  hl = (keepBounds && x.hl) ? (hl | one) : (hl & ~one);
  wr64(out, 2, c);
  wr64(out, 4, hg);
  wr64(out, 6, hl);
  if (km.bslot >= 0) {
    rs_set_gt(out, km.bslot, keepBounds && x.hg ? x.gt : 0);
    rs_set_lt(out, km.bslot, keepBounds && x.hl ? x.lt : 0);
  }
  wr64(out, 0, rs_present(out) | one);
}

// Copy key k of src into out.
template <class LT, class PO, class PS>
KS_HD void rs_copy_key(const LT& L, PO out, PS src, int k) {
  const KeyMeta km = L.keys[k];
  for (int i = 0; i < km.nw; i++) out[L.HDR + km.off + i] = src[L.HDR + km.off + i];
  uint64_t one = 1ull << k;
  for (int h = 0; h < 4; h++) {
    uint64_t o = rd64(out, 2 * h), s = rd64(src, 2 * h);
    wr64(out, 2 * h, (o & ~one) | (s & one));
  }
  if (km.bslot >= 0) {
    rs_set_gt(out, km.bslot, rs_gt(src, km.bslot));
    rs_set_lt(out, km.bslot, rs_lt(src, km.bslot));
  }
}

// Requirements.Add for every key of `in` (requirements.go:118-125): out &= in.
template <class LT, class PO, class PI>
KS_HD void rs_add(const LT& L, PO out, PI in) {
  uint64_t pi = rs_present(in), po = rs_present(out);
  while (pi) {
    int k = __builtin_ctzll(pi);
    pi &= pi - 1;
    if (bit(po, k)) rs_intersect_key(L, out, out, in, k);
    else rs_copy_key(L, out, in, k);
  }
}

// Do a and b agree on every key in `mask` (presence, header, words)?
template <class LT, class PA, class PB>
KS_HD bool rs_equal_keys(const LT& L, PA a, PB b, uint64_t mask) {
  for (int h = 0; h < 4; h++)
    if ((rd64(a, 2 * h) ^ rd64(b, 2 * h)) & mask) return false;
  uint64_t m = mask & rs_present(a);
  while (m) {
    int k = __builtin_ctzll(m);
    m &= m - 1;
    const KeyMeta km = L.keys[k];
    for (int i = 0; i < km.nw; i++)
      if (a[L.HDR + km.off + i] != b[L.HDR + km.off + i]) return false;
    if (km.bslot >= 0 && (rs_gt(a, km.bslot) != rs_gt(b, km.bslot) || rs_lt(a, km.bslot) != rs_lt(b, km.bslot)))
      return false;
  }
  return true;
}

}  // namespace ks
