// ksort.h -- klib's ks_introsort (ksort.h:142-219 of the reference's klib), restated for sampe.
// Not stable: the order it leaves equal keys in decides which position find_optimal_pair sees
// first, so the reference's exact sequence of comparisons and swaps is kept.  Its control flow
// depends only on the comparisons, so sorting light keys that carry an index gives the same
// permutation as sorting the records themselves (tests/test_ksort.py).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <utility>
#include <vector>

namespace ibwa_sam {

template <class T, class Lt>
void ks_insertsort(T *s, T *t, Lt lt) {
  for (T *i = s + 1; i < t; ++i)
    for (T *j = i; j > s && lt(*j, *(j - 1)); --j) std::swap(*j, *(j - 1));
}
template <class T, class Lt>
void ks_combsort(size_t n, T *a, Lt lt) {
  const double shrink = 1.2473309501039786540366528676643;
  bool do_swap;
  size_t gap = n;
  do {
    if (gap > 2) {
      gap = (size_t)(gap / shrink);
      if (gap == 9 || gap == 10) gap = 11;
    }
    do_swap = false;
    for (T *i = a; i < a + n - gap; ++i) {
      T *j = i + gap;
      if (lt(*j, *i)) {
        std::swap(*i, *j);
        do_swap = true;
      }
    }
  } while (do_swap || gap > 2);
  if (gap != 1) ks_insertsort(a, a + n, lt);
}
template <class T, class Lt>
void ks_introsort(size_t n, T *a, Lt lt) {
  struct Frame {
    T *left, *right;
    int depth;
  };
  if (n < 1) return;
  if (n == 2) {
    if (lt(a[1], a[0])) std::swap(a[0], a[1]);
    return;
  }
  int d;
  for (d = 2; 1ul << d < n; ++d) {}
  std::vector<Frame> stack;
  T *s = a, *t = a + (n - 1);
  d <<= 1;
  for (;;) {
    if (s < t) {
      if (--d == 0) {
        ks_combsort((size_t)(t - s + 1), s, lt);
        t = s;
        continue;
      }
      T *i = s, *j = t, *k = i + ((j - i) >> 1) + 1;
      if (lt(*k, *i)) {
        if (lt(*k, *j)) k = j;
      } else {
        k = lt(*j, *i) ? i : j;
      }
      const T rp = *k;
      if (k != t) std::swap(*k, *t);
      for (;;) {
        do ++i; while (lt(*i, rp));
        do --j; while (i <= j && lt(rp, *j));
        if (j <= i) break;
        std::swap(*i, *j);
      }
      std::swap(*i, *t);
      if (i - s > t - i) {
        if (i - s > 16) stack.push_back({s, i - 1, d});
        s = t - i > 16 ? i + 1 : t;
      } else {
        if (t - i > 16) stack.push_back({i + 1, t, d});
        t = i - s > 16 ? i - 1 : s;
      }
    } else {
      if (stack.empty()) {
        ks_insertsort(a, a + n, lt);
        return;
      }
      s = stack.back().left;
      t = stack.back().right;
      d = stack.back().depth;
      stack.pop_back();
    }
  }
}

// LSD radix sort of 64-bit keys, each with a 32-bit payload (vals may be null), in 11-bit digits
// over the bits in which the keys differ; tk / tv are scratch.  Stable, so for keys without
// duplicates it leaves what any sort leaves.
inline void radix_sort_u64(size_t n, uint64_t *keys, uint32_t *vals, std::vector<uint64_t> &tk, std::vector<uint32_t> &tv) {
  if (n < 2) return;
  uint64_t diff = 0;
  for (size_t i = 1; i < n; ++i) diff |= keys[i] ^ keys[0];
  if (!diff) return;
  const int lo = __builtin_ctzll(diff), hi = 64 - __builtin_clzll(diff);
  tk.resize(n);
  if (vals) tv.resize(n);
  uint64_t *ka = keys, *kb = tk.data();
  uint32_t *va = vals, *vb = vals ? tv.data() : nullptr;
  size_t cnt[2048];
  for (int sh = lo; sh < hi; sh += 11) {
    memset(cnt, 0, sizeof cnt);
    for (size_t i = 0; i < n; ++i) ++cnt[(ka[i] >> sh) & 2047];
    size_t sum = 0;
    for (size_t &c : cnt) {
      const size_t x = c;
      c = sum;
      sum += x;
    }
    for (size_t i = 0; i < n; ++i) {
      const size_t d = cnt[(ka[i] >> sh) & 2047]++;
      kb[d] = ka[i];
      if (va) vb[d] = va[i];
    }
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  if (ka != keys) {
    memcpy(keys, ka, n * sizeof *keys);
    if (vals) memcpy(vals, va, n * sizeof *vals);
  }
}

}  // namespace ibwa_sam
