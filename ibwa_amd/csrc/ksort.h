// ksort.h -- klib's ks_introsort (ksort.h:142-219 of the reference's klib), restated for sampe.
// Not stable: the order it leaves equal keys in decides which position find_optimal_pair sees
// first, so the reference's exact sequence of comparisons and swaps is kept.  Its control flow
// depends only on the comparisons, so sorting light keys that carry an index gives the same
// permutation as sorting the records themselves (tests/test_ksort.py).
#pragma once
#include <stddef.h>

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

}  // namespace ibwa_sam
