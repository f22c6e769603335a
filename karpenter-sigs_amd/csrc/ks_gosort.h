// ks_gosort.h — Go 1.21 sort.Slice (pdqsort_func) over (key, payload) arrays, __host__ __device__.
//
// scheduler.go:247 re-sorts s.newNodeClaims by len(Pods) before every placement with the unstable
// sort.Slice; which of several equally-full NodeClaims is tried first decides where the pod goes, so
// the product reproduces Go's exact swap sequence (src/sort/zsortfunc.go: insertionSort, heapSort,
// breakPatterns xorshift, choosePivot ninther, partialInsertionSort, partitionEqual, partition).
// Keys are the claims' pod counts; the payload is the claim id.  The kernels call go_sort_fast first,
// which proves "already sorted" (pdqsort leaves a non-decreasing array untouched: choosePivot then
// counts zero swaps, and partialInsertionSort finds no descent) and skips the emulation.
#pragma once
#include <stdint.h>

#include "ks_reqset.h"  // KS_HD

namespace ks {

template <class P>
struct GoSortT {
  P key;
  P val;

  KS_HD bool less(int i, int j) const { return key[i] < key[j]; }
  KS_HD void swap(int i, int j) {
    int32_t k = key[i]; key[i] = key[j]; key[j] = k;
    int32_t v = val[i]; val[i] = val[j]; val[j] = v;
  }
  KS_HD static int bitsLen(uint32_t x) { int n = 0; while (x) { n++; x >>= 1; } return n; }

  KS_HD void insertionSort(int a, int b) {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && less(j, j - 1); j--) swap(j, j - 1);
  }
  KS_HD void siftDown(int lo, int hi, int first) {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && less(first + child, first + child + 1)) child++;
      if (!less(first + root, first + child)) return;
      swap(first + root, first + child);
      root = child;
    }
  }
  KS_HD void heapSort(int a, int b) {
    int first = a, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) siftDown(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) { swap(first, first + i); siftDown(0, i, first); }
  }
  KS_HD void breakPatterns(int a, int b) {
    int length = b - a;
    if (length < 8) return;
    uint64_t r = (uint64_t)length;
    uint32_t mask = (1u << bitsLen((uint32_t)length)) - 1u;
    int idx = a + (length / 4) * 2 - 1;
    for (int i = 0; i < 3; i++) {
      r ^= r << 13; r ^= r >> 7; r ^= r << 17;
      int other = (int)((uint32_t)r & mask);
      if (other >= length) other -= length;
      swap(idx - 1 + i, a + other);
    }
  }
  KS_HD int median(int a, int b, int c, int& swaps) {
    if (less(b, a)) { swaps++; int t = a; a = b; b = t; }
    if (less(c, b)) { swaps++; int t = b; b = c; c = t; }
    if (less(b, a)) { swaps++; int t = a; a = b; b = t; }
    return b;
  }
  // returns pivot; hint: 0 unknown, 1 increasing, 2 decreasing
  KS_HD int choosePivot(int a, int b, int& hint) {
    int l = b - a, swaps = 0;
    int i = a + l / 4, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= 50) {
        i = median(i - 1, i, i + 1, swaps);
        j = median(j - 1, j, j + 1, swaps);
        k = median(k - 1, k, k + 1, swaps);
      }
      j = median(i, j, k, swaps);
    }
    hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
    return j;
  }
  KS_HD bool partialInsertionSort(int a, int b) {
    int i = a + 1;
    for (int step = 0; step < 5; step++) {
      while (i < b && !less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < 50) return false;
      swap(i, i - 1);
      if (i - a >= 2)
        for (int j = i - 1; j >= 1; j--) { if (!less(j, j - 1)) break; swap(j, j - 1); }
      if (b - i >= 2)
        for (int j = i + 1; j < b; j++) { if (!less(j, j - 1)) break; swap(j, j - 1); }
    }
    return false;
  }
  KS_HD int partitionEqual(int a, int b, int pivot) {
    swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !less(a, i)) i++;
      while (i <= j && less(a, j)) j--;
      if (i > j) break;
      swap(i, j); i++; j--;
    }
    return i;
  }
  KS_HD int partition(int a, int b, int pivot, bool& already) {
    swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && less(i, a)) i++;
    while (i <= j && !less(j, a)) j--;
    if (i > j) { swap(j, a); already = true; return j; }
    swap(i, j); i++; j--;
    for (;;) {
      while (i <= j && less(i, a)) i++;
      while (i <= j && !less(j, a)) j--;
      if (i > j) break;
      swap(i, j); i++; j--;
    }
    swap(j, a);
    already = false;
    return j;
  }
};

// State-carrying iterative pdqsort (exact Go semantics): each frame is either a fresh call
// (wasBalanced = wasPartitioned = true) or the continuation of a loop with carried flags.
template <class P>
struct GoSortExactT {
  GoSortT<P> s;
  // resumePivot >= 0: the top-level call already chose that pivot (increasing hint) and ran a
  // partialInsertionSort that returned false (the kernels' wave-parallel one); continue from there.
  KS_HD void run(int n, int resumePivot = -1) {
    struct Frame { int a, b, limit; bool wb, wp; };
    Frame stack[64];
    int sp = 0;
    stack[sp++] = Frame{0, n, GoSortT<P>::bitsLen((uint32_t)n), true, true};
    bool resume = resumePivot >= 0;
    while (sp > 0) {
      Frame f = stack[--sp];
      int a = f.a, b = f.b, limit = f.limit;
      bool wasBalanced = f.wb, wasPartitioned = f.wp;
      for (;;) {
        int length = b - a;
        int pivot;
        if (resume) {
          resume = false;
          pivot = resumePivot;
        } else {
          if (length <= 12) { s.insertionSort(a, b); break; }
          if (limit == 0) { s.heapSort(a, b); break; }
          if (!wasBalanced) { s.breakPatterns(a, b); limit--; }
          int hint;
          pivot = s.choosePivot(a, b, hint);
          if (hint == 2) {
            for (int i = a, j = b - 1; i < j; i++, j--) s.swap(i, j);
            pivot = (b - 1) - (pivot - a);
            hint = 1;
          }
          if (wasBalanced && wasPartitioned && hint == 1)
            if (s.partialInsertionSort(a, b)) break;
        }
        if (a > 0 && !s.less(a - 1, pivot)) {
          a = s.partitionEqual(a, b, pivot);
          continue;
        }
        bool already = false;
        int mid = s.partition(a, b, pivot, already);
        wasPartitioned = already;
        int leftLen = mid - a, rightLen = b - mid;
        int thr = length / 8;
        if (sp + 2 > 64) return;  // unreachable: depth <= 2*log2(n) + 2
        if (leftLen < rightLen) {
          wasBalanced = leftLen >= thr;
          stack[sp++] = Frame{mid + 1, b, limit, wasBalanced, wasPartitioned};  // continuation
          stack[sp++] = Frame{a, mid, limit, true, true};                      // recursive call
        } else {
          wasBalanced = rightLen >= thr;
          stack[sp++] = Frame{a, mid, limit, wasBalanced, wasPartitioned};
          stack[sp++] = Frame{mid + 1, b, limit, true, true};
        }
        break;
      }
    }
  }
};

using GoSort = GoSortT<int32_t*>;
using GoSortExact = GoSortExactT<int32_t*>;

}  // namespace ks
