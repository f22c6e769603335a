// go_sort.h — CPU restatement of Go 1.21 `sort.Slice` / `sort.SliceStable` (test infrastructure).
//
// The reference calls sort.Slice on its hot path (scheduler.go:247 claims by pod count every pod,
// queue.go:38 pods, requirements.go:90 preferred terms, nodepool.go:210 pools, consolidation.go:79
// candidates).  sort.Slice is Go's unstable pattern-defeating quicksort (src/sort/zsortfunc.go,
// `pdqsort_func`); the tie order it produces is part of the reference's observable behaviour, so
// the oracle restates it step for step.  The Go stdlib source is not present in this container:
// this is a restatement from the published Go 1.21 algorithm — "parity
// unpinned" for tie order, as no reference test pins it.
#pragma once
#include <cstdint>

namespace gosort {

// Less(i, j) and Swap(i, j) over indices of the sequence being sorted.
template <class LessSwap>
struct Sorter {
  LessSwap& d;
  explicit Sorter(LessSwap& x) : d(x) {}

  enum Hint { unknownHint = 0, increasingHint, decreasingHint };

  void insertionSort(int a, int b) {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && d.less(j, j - 1); j--) d.swap(j, j - 1);
  }
  void siftDown(int lo, int hi, int first) {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && d.less(first + child, first + child + 1)) child++;
      if (!d.less(first + root, first + child)) return;
      d.swap(first + root, first + child);
      root = child;
    }
  }
  void heapSort(int a, int b) {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) siftDown(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      d.swap(first, first + i);
      siftDown(lo, i, first);
    }
  }
  static int bitsLen(uint64_t x) {
    int n = 0;
    while (x) { n++; x >>= 1; }
    return n;
  }
  void breakPatterns(int a, int b) {
    int length = b - a;
    if (length >= 8) {
      uint64_t random = (uint64_t)length;  // xorshift seeded with the length
      uint64_t modulus = (uint64_t)1 << bitsLen((uint64_t)length);
      int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        random ^= random << 13;
        random ^= random >> 7;
        random ^= random << 17;
        int other = (int)((unsigned)random & (unsigned)(modulus - 1));
        if (other >= length) other -= length;
        d.swap(idx - 1 + i, a + other);
      }
    }
  }
  void order2(int& a, int& b, int& swaps) {
    if (d.less(b, a)) {
      swaps++;
      int t = a; a = b; b = t;
    }
  }
  int median(int a, int b, int c, int& swaps) {
    order2(a, b, swaps);
    order2(b, c, swaps);
    order2(a, b, swaps);
    return b;
  }
  int medianAdjacent(int a, int& swaps) { return median(a - 1, a, a + 1, swaps); }
  int choosePivot(int a, int b, Hint& hint) {
    const int shortestNinther = 50, maxSwaps = 4 * 3;
    int l = b - a;
    int swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= shortestNinther) {
        i = medianAdjacent(i, swaps);
        j = medianAdjacent(j, swaps);
        k = medianAdjacent(k, swaps);
      }
      j = median(i, j, k, swaps);
    }
    if (swaps == 0) hint = increasingHint;
    else if (swaps == maxSwaps) hint = decreasingHint;
    else hint = unknownHint;
    return j;
  }
  void reverseRange(int a, int b) {
    int i = a, j = b - 1;
    while (i < j) { d.swap(i, j); i++; j--; }
  }
  bool partialInsertionSort(int a, int b) {
    const int maxSteps = 5, shortestShifting = 50;
    int i = a + 1;
    for (int j = 0; j < maxSteps; j++) {
      while (i < b && !d.less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < shortestShifting) return false;
      d.swap(i, i - 1);
      if (i - a >= 2) {  // shift the smaller one to the left (Go uses j >= 1, not j > a)
        for (int k = i - 1; k >= 1; k--) {
          if (!d.less(k, k - 1)) break;
          d.swap(k, k - 1);
        }
      }
      if (b - i >= 2) {  // shift the greater one to the right
        for (int k = i + 1; k < b; k++) {
          if (!d.less(k, k - 1)) break;
          d.swap(k, k - 1);
        }
      }
    }
    return false;
  }
  int partitionEqual(int a, int b, int pivot) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !d.less(a, i)) i++;
      while (i <= j && d.less(a, j)) j--;
      if (i > j) break;
      d.swap(i, j);
      i++; j--;
    }
    return i;
  }
  int partition(int a, int b, int pivot, bool& alreadyPartitioned) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && d.less(i, a)) i++;
    while (i <= j && !d.less(j, a)) j--;
    if (i > j) {
      d.swap(j, a);
      alreadyPartitioned = true;
      return j;
    }
    d.swap(i, j);
    i++; j--;
    for (;;) {
      while (i <= j && d.less(i, a)) i++;
      while (i <= j && !d.less(j, a)) j--;
      if (i > j) break;
      d.swap(i, j);
      i++; j--;
    }
    d.swap(j, a);
    alreadyPartitioned = false;
    return j;
  }
  void pdqsort(int a, int b, int limit) {
    const int maxInsertion = 12;
    bool wasBalanced = true, wasPartitioned = true;
    for (;;) {
      int length = b - a;
      if (length <= maxInsertion) {
        insertionSort(a, b);
        return;
      }
      if (limit == 0) {
        heapSort(a, b);
        return;
      }
      if (!wasBalanced) {
        breakPatterns(a, b);
        limit--;
      }
      Hint hint;
      int pivot = choosePivot(a, b, hint);
      if (hint == decreasingHint) {
        reverseRange(a, b);
        pivot = (b - 1) - (pivot - a);
        hint = increasingHint;
      }
      if (wasBalanced && wasPartitioned && hint == increasingHint) {
        if (partialInsertionSort(a, b)) return;
      }
      if (a > 0 && !d.less(a - 1, pivot)) {
        int mid = partitionEqual(a, b, pivot);
        a = mid;
        continue;
      }
      bool alreadyPartitioned = false;
      int mid = partition(a, b, pivot, alreadyPartitioned);
      wasPartitioned = alreadyPartitioned;
      int leftLen = mid - a, rightLen = b - mid;
      int balanceThreshold = length / 8;
      if (leftLen < rightLen) {
        wasBalanced = leftLen >= balanceThreshold;
        pdqsort(a, mid, limit);
        a = mid + 1;
      } else {
        wasBalanced = rightLen >= balanceThreshold;
        pdqsort(mid + 1, b, limit);
        b = mid;
      }
    }
  }
};

// sort.Slice(x, less): pdqsort_func(data, 0, n, bits.Len(uint(n))).
template <class LessSwap>
void slice(LessSwap& d, int n) {
  Sorter<LessSwap> s(d);
  s.pdqsort(0, n, Sorter<LessSwap>::bitsLen((uint64_t)n));
}

// sort.SliceStable: the result is fully determined by the comparator (stable), so any stable
// algorithm reproduces it; insertion sort keeps this header dependency-free.
template <class LessSwap>
void sliceStable(LessSwap& d, int n) {
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && d.less(j, j - 1); j--) d.swap(j, j - 1);
}

}  // namespace gosort
