// Frequent-item ranking of a numeric vocabulary (FastApriori.scala:55-62: items with
// support >= minCount, sorted by count descending, ties in Java String order of the
// token).  Numeric tokens are ASCII decimals, and Java String order of decimals is
// the order of (digits left-aligned to 10 places, then length); id 0 is the empty
// token "" (sorts first).  One call replaces the host's numpy ranking + LUT build
// (FastApriori._frequent_items) between the histogram readback and the LUT upload.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "fa_common.h"

namespace {

struct F1Key {
  int64_t cnt, key;
  int d;
  int64_t fid;
};

inline void java_decimal_key(int64_t fid, int64_t* key, int* d) {
  if (fid == 0) { *key = -1; *d = 0; return; }
  const int64_t v = fid - 1;
  int digits = 1;
  int64_t p = 10;
  while (digits < 11 && v >= p) { ++digits; p *= 10; }
  int64_t pad = 1;
  for (int i = 0; i < 10 - std::min(digits, 10); ++i) pad *= 10;
  *key = v * pad;
  *d = digits;
}

}  // namespace

// hist: int64 [V] supports by id (fid = token + 1); thr: minimum support.
// ids / cnt (int64 [V] capacity): the frequent ids and counts in rank order;
// lut (int32 [V]): id -> rank, -1 for infrequent ids.  Returns F1.
FA_API int64_t fa_f1_rank_numeric(const int64_t* hist, int64_t V, int64_t thr, int64_t* ids, int64_t* cnt,
                                  int32_t* lut) {
  std::vector<F1Key> f;
  f.reserve(1024);
  for (int64_t v = 0; v < V; ++v) {
    lut[v] = -1;
    if (hist[v] >= thr) {
      F1Key k{hist[v], 0, 0, v};
      java_decimal_key(v, &k.key, &k.d);
      f.push_back(k);
    }
  }
  std::sort(f.begin(), f.end(), [](const F1Key& a, const F1Key& b) {
    if (a.cnt != b.cnt) return a.cnt > b.cnt;
    if (a.key != b.key) return a.key < b.key;
    return a.d < b.d;
  });
  for (size_t i = 0; i < f.size(); ++i) {
    ids[i] = f[i].fid;
    cnt[i] = f[i].cnt;
    lut[f[i].fid] = (int32_t)i;
  }
  return (int64_t)f.size();
}
