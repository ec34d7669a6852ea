// Association rules: generation, level-wise redundancy cut, ordering, and the
// CPU first-match recommender.
//
// Reference behaviour (AssociationRules.scala):
//   * genRules (:122-145): for every frequent S with |S| >= 2 and every s in S,
//     rule (S - {s}) -> s with conf = count(S).toDouble / count(S - {s}).
//     The reference finds S - {s} by a linear scan of all (|S|-1)-itemsets;
//     we binary-search the lexicographically sorted level instead (subset index).
//   * cut (:147-182): rules of the smallest antecedent size are all kept; a rule
//     A -> r at size i survives iff for EVERY a in A the rule (A - {a}) -> r was
//     kept at size i-1 and has strictly smaller confidence.
//   * order (:116-120): confidence descending, then consequent token as Int
//     ascending (tie positions are precomputed by the caller, see
//     fastapriori_amd/utils/jvm.py rule_tiebreak_key), then antecedent ranks.
//   * recommend (:80-106): first rule in that order with antecedent subset of the
//     basket and consequent not in the basket; otherwise "0".
#include <chrono>
#include <unordered_map>

#include "fa_common.h"

namespace fa {

struct RuleSet {
  std::vector<int64_t> ante_off;   // R+1
  std::vector<int32_t> ante;       // concatenated antecedent ranks (ascending)
  std::vector<int32_t> cons;
  std::vector<double> conf;
  std::vector<int64_t> stats;      // per antecedent level: before, after, cut microseconds
};

static inline int cmp_row(const int32_t* a, const int32_t* b, int m) {
  for (int i = 0; i < m; ++i)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}

static inline int64_t find_row(const int32_t* rows, int64_t n, int m, const int32_t* key) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    int c = cmp_row(rows + mid * m, key, m);
    if (c == 0) return mid;
    if (c < 0) lo = mid + 1; else hi = mid;
  }
  return -1;
}

struct RawRule { int64_t ante; int32_t cons; double conf; };

}  // namespace fa

using namespace fa;

// rows[k-1]: level-k itemsets (sizes[k-1] rows of k ascending ranks, sorted);
// counts[k-1]: their supports.  levels = K.  tie_pos[r]: position of rank r's
// token in the consequent tiebreak order.
FA_API RuleSet* fa_rules_build(const int32_t* const* rows, const int64_t* const* counts,
                               const int64_t* sizes, int levels, const int64_t* tie_pos,
                               int nthreads, int64_t* n_rules) {
  auto* rs = new RuleSet();
  // raw[L] = rules with antecedent size L (L = 1..levels-1), stored at raw[L-1]
  std::vector<std::vector<RawRule>> raw(std::max(0, levels - 1));
  for (int k = 2; k <= levels; ++k) {
    const int32_t* S = rows[k - 1];
    const int64_t nS = sizes[k - 1];
    const int32_t* A = rows[k - 2];
    const int64_t nA = sizes[k - 2];
    std::vector<RawRule>& out = raw[k - 2];
    out.resize((size_t)(nS * k));
    parallel_for(nS, nthreads, 1024, [&](int64_t b, int64_t e, int) {
      std::vector<int32_t> key(k - 1);
      for (int64_t s = b; s < e; ++s) {
        const int32_t* row = S + s * k;
        for (int p = 0; p < k; ++p) {
          int w = 0;
          for (int q = 0; q < k; ++q) if (q != p) key[w++] = row[q];
          int64_t a = find_row(A, nA, k - 1, key.data());
          // a >= 0 always holds for a complete miner (anti-monotonicity)
          double c = a >= 0 ? (double)counts[k - 1][s] / (double)counts[k - 2][a] : 0.0;
          out[(size_t)(s * k + p)] = RawRule{a, row[p], c};
        }
      }
    });
  }
  // level-wise cut
  std::vector<std::vector<char>> keep(raw.size());
  for (size_t L = 0; L < raw.size(); ++L) {
    const auto t_cut = std::chrono::steady_clock::now();
    keep[L].assign(raw[L].size(), L == 0 ? 1 : 0);
    if (L == 0) {
      rs->stats.push_back((int64_t)raw[0].size()); rs->stats.push_back((int64_t)raw[0].size());
      rs->stats.push_back(0);
      continue;
    }
    // kept rules of the level below, keyed by (antecedent index, consequent)
    std::unordered_map<uint64_t, double> low;
    low.reserve(raw[L - 1].size() * 2);
    for (size_t i = 0; i < raw[L - 1].size(); ++i)
      if (keep[L - 1][i]) low.emplace(((uint64_t)raw[L - 1][i].ante << 32) | (uint32_t)raw[L - 1][i].cons,
                                      raw[L - 1][i].conf);
    const int m = (int)L + 1;          // antecedent size at this level
    const int32_t* Arows = rows[m - 1];
    const int32_t* Brows = rows[m - 2];
    const int64_t nB = sizes[m - 2];
    int64_t kept = 0;
    std::vector<int64_t> kept_t(std::max(1, nthreads), 0);
    parallel_for((int64_t)raw[L].size(), nthreads, 4096, [&](int64_t b, int64_t e, int tid) {
      std::vector<int32_t> key(m - 1);
      for (int64_t i = b; i < e; ++i) {
        const RawRule& r = raw[L][i];
        const int32_t* a = Arows + r.ante * m;
        bool ok = true;
        for (int p = 0; p < m && ok; ++p) {
          int w = 0;
          for (int q = 0; q < m; ++q) if (q != p) key[w++] = a[q];
          int64_t bi = find_row(Brows, nB, m - 1, key.data());
          if (bi < 0) { ok = false; break; }
          auto it = low.find(((uint64_t)bi << 32) | (uint32_t)r.cons);
          if (it == low.end() || it->second >= r.conf) ok = false;
        }
        keep[L][i] = ok ? 1 : 0;
        kept_t[tid] += ok;
      }
    });
    for (auto v : kept_t) kept += v;
    rs->stats.push_back((int64_t)raw[L].size());
    rs->stats.push_back(kept);
    rs->stats.push_back((int64_t)std::chrono::duration_cast<std::chrono::microseconds>(
        std::chrono::steady_clock::now() - t_cut).count());
  }
  // gather kept rules and sort
  struct Ref { int32_t level; int64_t idx; };
  std::vector<Ref> refs;
  for (size_t L = 0; L < raw.size(); ++L)
    for (size_t i = 0; i < raw[L].size(); ++i)
      if (keep[L][i]) refs.push_back(Ref{(int32_t)L, (int64_t)i});
  auto ante_ptr = [&](const Ref& r) { return rows[r.level] + raw[r.level][r.idx].ante * (r.level + 1); };
  std::stable_sort(refs.begin(), refs.end(), [&](const Ref& x, const Ref& y) {
    const RawRule& a = raw[x.level][x.idx];
    const RawRule& b = raw[y.level][y.idx];
    if (a.conf != b.conf) return a.conf > b.conf;
    int64_t ta = tie_pos[a.cons], tb = tie_pos[b.cons];
    if (ta != tb) return ta < tb;
    if (x.level != y.level) return x.level < y.level;
    return cmp_row(ante_ptr(x), ante_ptr(y), x.level + 1) < 0;
  });
  rs->ante_off.push_back(0);
  for (auto& r : refs) {
    const RawRule& rr = raw[r.level][r.idx];
    const int32_t* a = ante_ptr(r);
    rs->ante.insert(rs->ante.end(), a, a + r.level + 1);
    rs->ante_off.push_back((int64_t)rs->ante.size());
    rs->cons.push_back(rr.cons);
    rs->conf.push_back(rr.conf);
  }
  *n_rules = (int64_t)refs.size();
  return rs;
}

FA_API int64_t fa_rules_nante(RuleSet* rs) { return (int64_t)rs->ante.size(); }
FA_API int64_t fa_rules_nstats(RuleSet* rs) { return (int64_t)rs->stats.size(); }

FA_API void fa_rules_export(RuleSet* rs, int64_t* ante_off, int32_t* ante, int32_t* cons,
                            double* conf, int64_t* stats) {
  std::memcpy(ante_off, rs->ante_off.data(), rs->ante_off.size() * 8);
  if (!rs->ante.empty()) std::memcpy(ante, rs->ante.data(), rs->ante.size() * 4);
  if (!rs->cons.empty()) std::memcpy(cons, rs->cons.data(), rs->cons.size() * 4);
  if (!rs->conf.empty()) std::memcpy(conf, rs->conf.data(), rs->conf.size() * 8);
  if (!rs->stats.empty()) std::memcpy(stats, rs->stats.data(), rs->stats.size() * 8);
}

FA_API void fa_rules_free(RuleSet* rs) { delete rs; }

// First-match recommendation on the CPU.  Baskets are CSR of distinct ranks.
// out[i] = recommended rank, or -1 for "0".
FA_API void fa_recommend_cpu(const int64_t* ante_off, const int32_t* ante, const int32_t* cons,
                             int64_t R, int32_t F1, const int64_t* bask_off, const int32_t* bask,
                             int64_t M, int32_t* out, int nthreads) {
  const int64_t words = ((int64_t)F1 + 63) / 64;
  parallel_for(M, nthreads, 256, [&](int64_t b, int64_t e, int) {
    std::vector<uint64_t> bits((size_t)std::max<int64_t>(1, words), 0);
    for (int64_t u = b; u < e; ++u) {
      const int64_t s = bask_off[u], t = bask_off[u + 1];
      for (int64_t i = s; i < t; ++i) bits[bask[i] >> 6] |= 1ull << (bask[i] & 63);
      const int64_t usz = t - s;
      int32_t rec = -1;
      for (int64_t r = 0; r < R && usz > 0; ++r) {
        int32_t c = cons[r];
        if ((bits[c >> 6] >> (c & 63)) & 1) continue;
        const int64_t a0 = ante_off[r], a1 = ante_off[r + 1];
        if (a1 - a0 > usz) continue;
        bool sub = true;
        for (int64_t i = a0; i < a1; ++i)
          if (!((bits[ante[i] >> 6] >> (ante[i] & 63)) & 1)) { sub = false; break; }
        if (sub) { rec = c; break; }
      }
      out[u] = rec;
      for (int64_t i = s; i < t; ++i) bits[bask[i] >> 6] = 0;
    }
  });
}
