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
#include <cstdlib>

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

static inline uint64_t row_hash(const int32_t* r, int m) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)m;
  for (int i = 0; i < m; ++i) h = mix64(h ^ (uint32_t)r[i]);
  return h;
}

// Open-addressing set of the rows of F_{k-1} (indices into `rows`), probed by
// content: O(1) subset checks instead of a binary search per check.  The table
// is split into nthreads partitions by the top hash bits, so it is built in
// parallel with no synchronisation (each thread owns one partition).
struct RowSet {
  const int32_t* rows;
  int m;
  std::vector<int64_t> slot;   // -1 = empty
  int pbits = 0;
  uint64_t pmask;              // slots per partition - 1
  size_t index(uint64_t h, uint64_t probe) const {
    const uint64_t part = pbits ? (h >> (64 - pbits)) : 0;
    return (size_t)((part * (pmask + 1)) + ((h + probe) & pmask));
  }
  RowSet(const int32_t* r, int64_t n, int m_, int nthreads) : rows(r), m(m_) {
    int P = 1;
    while (P * 2 <= std::max(1, nthreads) && P < 64) { P *= 2; ++pbits; }
    size_t per = 16;
    while (per * P < (size_t)n * 2) per <<= 1;
    pmask = per - 1;
    slot.assign(per * P, -1);
    std::vector<uint64_t> h(n);
    parallel_for(n, nthreads, 1 << 14, [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; ++i) h[i] = row_hash(rows + i * m, m);
    });
    parallel_for_threads(P, [&](int t) {
      for (int64_t i = 0; i < n; ++i) {
        if (pbits && (int)(h[i] >> (64 - pbits)) != t) continue;
        uint64_t probe = 0;
        while (slot[index(h[i], probe)] != -1) ++probe;
        slot[index(h[i], probe)] = i;
      }
    });
  }
  template <class Eq>
  bool find(uint64_t h, Eq&& eq) const {
    for (uint64_t probe = 0;; ++probe) {
      const int64_t i = slot[index(h, probe)];
      if (i < 0) return false;
      if (eq(rows + i * m)) return true;
    }
  }
  bool contains(const int32_t* key) const {
    return find(row_hash(key, m), [&](const int32_t* r) { return cmp_row(r, key, m) == 0; });
  }
  // Membership of (x without x[skip]) + y, given the hash state of its first m-1 ranks.
  bool contains_drop(uint64_t state, const int32_t* x, int skip, int32_t y) const {
    return find(mix64(state ^ (uint32_t)y), [&](const int32_t* r) {
      if (r[m - 1] != y) return false;
      for (int q = 0, w = 0; q < m; ++q) {
        if (q == skip) continue;
        if (r[w++] != x[q]) return false;
      }
      return true;
    });
  }
};

}  // namespace fa

using namespace fa;

// Bitset formulation of the same join + prune.  For every (m-1)-prefix Q that
// starts a class of F_{k-1}, Ext(Q) = bitset of the classes' last items (items
// densely renumbered).  The extensions of row x are then
//     { y > x[m-1] } AND Ext(x[0..m-2]) AND  AND_{p < m-1} Ext(x without x[p])
// because (x without x[p]) + y is a row of F_{k-1} exactly when y is in the
// Ext of that prefix.  One hash lookup and one bitset AND per subset check
// instead of one lookup per (row, y) pair: the k = 3 join of a dense F_2
// examines every pair of a class, while the bitsets cost ~F1/64 words per row.
// Returns nullptr when the item universe is too wide for bitsets or the classes
// are small enough that the pair join is cheaper.
static Cands* apriori_gen_bitset(const int32_t* prev, int64_t n, int m, int nthreads) {
  int32_t maxr = 0;
  for (int64_t i = 0; i < n * m; ++i) maxr = std::max(maxr, prev[i]);
  std::vector<int32_t> dense((size_t)maxr + 1, -1);
  for (int64_t i = 0; i < n * m; ++i) dense[prev[i]] = 0;
  std::vector<int32_t> item;
  for (int32_t r = 0; r <= maxr; ++r)
    if (dense[r] >= 0) { dense[r] = (int32_t)item.size(); item.push_back(r); }
  const int nw = (int)((item.size() + 63) / 64);
  if (nw > 64) return nullptr;
  // classes (rows sharing their first m-1 ranks) and their Ext bitsets
  std::vector<int64_t> cls_start;
  std::vector<int32_t> cls_of((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    if (i == 0 || cmp_row(prev + i * m, prev + (i - 1) * m, m - 1) != 0) cls_start.push_back(i);
    cls_of[i] = (int32_t)cls_start.size() - 1;
  }
  const int64_t ncls = (int64_t)cls_start.size();
  // cost model: the pair join probes every (row, later class member) pair m-1
  // times; the bitset form probes m-1 times per row and ANDs nw words per probe.
  // Decided before any bitset is built.
  double pairs = 0;
  for (int64_t c = 0; c < ncls; ++c) {
    const double sz = (double)((c + 1 < ncls ? cls_start[c + 1] : n) - cls_start[c]);
    pairs += sz * (sz - 1) / 2;
  }
  // (per-op costs in ns, measured on the k = 3 / 4 levels of T10I4)
  const double t_bitset = (double)n * (30.0 + m * (15.0 + 1.5 * nw));
  const double t_pairs = 35.0 * pairs * (m - 1) + 40.0 * (double)n;
  if (t_bitset >= t_pairs) return nullptr;
  std::vector<uint64_t> ext((size_t)ncls * nw, 0ull);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t d = dense[prev[i * m + m - 1]];
    ext[(size_t)cls_of[i] * nw + (d >> 6)] |= 1ull << (d & 63);
  }
  // open-addressing map (m-1)-prefix -> class
  size_t cap = 16;
  while (cap < (size_t)ncls * 2) cap <<= 1;
  std::vector<int32_t> slot(cap, -1);
  auto phash = [&](const int32_t* r) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(m - 1);
    for (int q = 0; q < m - 1; ++q) h = mix64(h ^ (uint32_t)r[q]);
    return h;
  };
  for (int64_t c = 0; c < ncls; ++c) {
    size_t at = (size_t)phash(prev + cls_start[c] * m) & (cap - 1);
    while (slot[at] >= 0) at = (at + 1) & (cap - 1);
    slot[at] = (int32_t)c;
  }
  auto out = new Cands();
  out->ext_off.push_back(0);
  const int64_t grain = 1024;
  const int64_t nblocks = (n + grain - 1) / grain;
  std::vector<Cands> parts(nblocks);
  nthreads = std::max(1, std::min<int>(nthreads, (int)(n / 1024)));
  parallel_for(nblocks, nthreads, 1, [&](int64_t b0, int64_t b1, int) {
    std::vector<uint64_t> acc((size_t)nw);
    std::vector<int32_t> key((size_t)std::max(1, m - 1));
    for (int64_t b = b0; b < b1; ++b) {
      struct Local { Cands c; Cands& dst; ~Local() { dst = std::move(c); } } L{Cands(), parts[b]};
      Cands& pc = L.c;
      pc.ext_off.push_back(0);
      for (int64_t i = b * grain; i < std::min(n, (b + 1) * grain); ++i) {
        const int32_t* x = prev + i * m;
        const uint64_t* e0 = ext.data() + (size_t)cls_of[i] * nw;
        // y > x[m-1]: clear dense ids <= d
        const int32_t d = dense[x[m - 1]];
        bool any = false;
        for (int w = 0; w < nw; ++w) {
          uint64_t v = e0[w];
          if (w < (d >> 6)) v = 0;
          else if (w == (d >> 6)) v &= (d & 63) == 63 ? 0ull : (~0ull << ((d & 63) + 1));
          acc[w] = v;
          any |= v != 0;
        }
        for (int p = 0; p < m - 1 && any; ++p) {
          for (int q = 0, t = 0; q < m; ++q) if (q != p) key[t++] = x[q];
          size_t at = (size_t)phash(key.data()) & (cap - 1);
          int32_t c = -1;
          while (slot[at] >= 0) {
            const int32_t cc = slot[at];
            if (cmp_row(prev + cls_start[cc] * m, key.data(), m - 1) == 0) { c = cc; break; }
            at = (at + 1) & (cap - 1);
          }
          if (c < 0) { any = false; break; }
          const uint64_t* ec = ext.data() + (size_t)c * nw;
          any = false;
          for (int w = 0; w < nw; ++w) { acc[w] &= ec[w]; any |= acc[w] != 0; }
        }
        if (!any) continue;
        pc.prefix.push_back((int32_t)i);
        for (int w = 0; w < nw; ++w)
          for (uint64_t v = acc[w]; v; v &= v - 1) pc.ext.push_back(item[w * 64 + __builtin_ctzll(v)]);
        pc.ext_off.push_back((int64_t)pc.ext.size());
      }
    }
  });
  for (auto& pc : parts) {
    int64_t base = (int64_t)out->ext.size();
    out->prefix.insert(out->prefix.end(), pc.prefix.begin(), pc.prefix.end());
    for (size_t g = 1; g < pc.ext_off.size(); ++g) out->ext_off.push_back(base + pc.ext_off[g]);
    out->ext.insert(out->ext.end(), pc.ext.begin(), pc.ext.end());
  }
  return out;
}

// prev: n rows of m = k-1 ranks, each row ascending, rows lexicographically sorted.
FA_API Cands* fa_apriori_gen(const int32_t* prev, int64_t n, int m, int nthreads, int64_t* sizes) {
  if (n > 0 && m >= 2) {
    if (Cands* c = apriori_gen_bitset(prev, n, m, nthreads)) {
      sizes[0] = (int64_t)c->prefix.size();
      sizes[1] = (int64_t)c->ext.size();
      return c;
    }
  }
  auto* out = new Cands();
  // thread start-up costs ~50 us each: small levels run on the calling thread
  nthreads = std::max(1, std::min<int>(nthreads, (int)(n / 1024)));
  // class end for every row: first row index whose first m-1 ranks differ
  std::vector<int64_t> cls_end(n);
  std::vector<char> starts(n + 1, 1);
  parallel_for(n, nthreads, 1 << 14, [&](int64_t b, int64_t e, int) {
    for (int64_t i = std::max<int64_t>(b, 1); i < e; ++i)
      starts[i] = cmp_row(prev + i * m, prev + (i - 1) * m, m - 1) != 0;
  });
  {
    int64_t end = n;
    for (int64_t i = n - 1; i >= 0; --i) {
      cls_end[i] = end;
      if (starts[i]) end = i;
    }
  }
  bool any_join = false;
  for (int64_t i = 0; i + 1 < n && !any_join; ++i) any_join = cls_end[i] > i + 1;
  if (!any_join) {
    out->ext_off.push_back(0);
    sizes[0] = sizes[1] = 0;
    return out;
  }
  RowSet set(prev, n, m, nthreads);
  const int64_t grain = 256;
  const int64_t nblocks = (n + grain - 1) / grain;
  std::vector<Cands> parts(nblocks);
  parallel_for(nblocks, nthreads, 1, [&](int64_t b0, int64_t b1, int) {
    std::vector<uint64_t> st(m);
    for (int64_t b = b0; b < b1; ++b) {
      // built locally and moved: neighbouring blocks run on other threads, and
      // appending through adjacent parts[] headers would false-share
      struct Local { Cands c; Cands& dst; ~Local() { dst = std::move(c); } } L{Cands(), parts[b]};
      Cands& pc = L.c;
      pc.ext_off.push_back(0);
      for (int64_t i = b * grain; i < std::min(n, (b + 1) * grain); ++i) {
        const int32_t* x = prev + i * m;
        size_t before = pc.ext.size();
        if (cls_end[i] > i + 1) {
          // hash state of (x without x[p]) for every p < m-1, shared by all y of the class
          for (int p = 0; p < m - 1; ++p) {
            uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)m;
            for (int q = 0; q < m; ++q) if (q != p) h = mix64(h ^ (uint32_t)x[q]);
            st[p] = h;
          }
        }
        for (int64_t j = i + 1; j < cls_end[i]; ++j) {
          const int32_t y = prev[j * m + m - 1];
          bool ok = true;
          // drop x[p] for p < m-1: (x without x[p]) + y must be frequent
          for (int p = 0; p < m - 1 && ok; ++p) ok = set.contains_drop(st[p], x, p, y);
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
