// Candidate generation (join + full subset prune), host side.
//
// Reference behaviour (FastApriori.scala:167-193): for every frequent
// (k-1)-itemset x the extensions are ranks y > max(x) such that
// (x - x_i) + y is frequent for every x_i; groups (x, ys) with no ys are
// dropped.  That is classic apriori-gen; we compute it with the equivalent
// equivalence-class join (rows sharing their first k-2 ranks), which only ever
// proposes y's that already pass two of the k subset checks, then binary
// searches the remaining k-2 subsets in the lexicographically sorted F_{k-1}.
//
// The output keeps the reference's (prefix x, extensions ys) grouping because
// the support-counting kernel shares the prefix AND across a group
// (FastApriori.scala:143-154).  Candidates come out in lexicographic order, so
// F_k stays sorted after thresholding — every rank computes the identical list.
#include "fa_common.h"

namespace fa {

struct Cands {
  std::vector<int32_t> prefix;    // index of the prefix row in F_{k-1}
  std::vector<int64_t> ext_off;   // G+1
  std::vector<int32_t> ext;       // C
};

static inline int cmp_row(const int32_t* a, const int32_t* b, int m) {
  for (int i = 0; i < m; ++i) {
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  }
  return 0;
}

static inline bool contains_row(const int32_t* rows, int64_t n, int m, const int32_t* key) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    int c = cmp_row(rows + mid * m, key, m);
    if (c == 0) return true;
    if (c < 0) lo = mid + 1; else hi = mid;
  }
  return false;
}

}  // namespace fa

using namespace fa;

// prev: n rows of m = k-1 ranks, each row ascending, rows lexicographically sorted.
FA_API Cands* fa_apriori_gen(const int32_t* prev, int64_t n, int m, int nthreads, int64_t* sizes) {
  auto* out = new Cands();
  // class end for every row: first row index whose first m-1 ranks differ
  std::vector<int64_t> cls_end(n);
  {
    int64_t i = 0;
    while (i < n) {
      int64_t j = i + 1;
      while (j < n && cmp_row(prev + j * m, prev + i * m, m - 1) == 0) ++j;
      for (int64_t t = i; t < j; ++t) cls_end[t] = j;
      i = j;
    }
  }
  const int64_t grain = 256;
  const int64_t nblocks = (n + grain - 1) / grain;
  std::vector<Cands> parts(nblocks);
  parallel_for(nblocks, nthreads, 1, [&](int64_t b0, int64_t b1, int) {
    std::vector<int32_t> key(m);
    for (int64_t b = b0; b < b1; ++b) {
      Cands& pc = parts[b];
      pc.ext_off.push_back(0);
      for (int64_t i = b * grain; i < std::min(n, (b + 1) * grain); ++i) {
        const int32_t* x = prev + i * m;
        size_t before = pc.ext.size();
        for (int64_t j = i + 1; j < cls_end[i]; ++j) {
          int32_t y = prev[j * m + m - 1];
          bool ok = true;
          // drop x[p] for p < m-1 : key = x without p, then y  (ascending)
          for (int p = 0; p < m - 1 && ok; ++p) {
            int w = 0;
            for (int q = 0; q < m; ++q) if (q != p) key[w++] = x[q];
            key[w] = y;
            ok = contains_row(prev, n, m, key.data());
          }
          if (ok) pc.ext.push_back(y);
        }
        if (pc.ext.size() > before) {
          pc.prefix.push_back((int32_t)i);
          pc.ext_off.push_back((int64_t)pc.ext.size());
        }
      }
    }
  });
  out->ext_off.push_back(0);
  for (auto& pc : parts) {
    int64_t base = (int64_t)out->ext.size();
    out->prefix.insert(out->prefix.end(), pc.prefix.begin(), pc.prefix.end());
    for (size_t g = 1; g < pc.ext_off.size(); ++g) out->ext_off.push_back(base + pc.ext_off[g]);
    out->ext.insert(out->ext.end(), pc.ext.begin(), pc.ext.end());
  }
  sizes[0] = (int64_t)out->prefix.size();
  sizes[1] = (int64_t)out->ext.size();
  return out;
}

FA_API void fa_cands_export(Cands* c, int32_t* prefix, int64_t* ext_off, int32_t* ext) {
  if (!c->prefix.empty()) std::memcpy(prefix, c->prefix.data(), c->prefix.size() * 4);
  std::memcpy(ext_off, c->ext_off.data(), c->ext_off.size() * 8);
  if (!c->ext.empty()) std::memcpy(ext, c->ext.data(), c->ext.size() * 4);
}

FA_API void fa_cands_free(Cands* c) { delete c; }
