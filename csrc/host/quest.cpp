// IBM-Quest-style synthetic transaction generator (Agrawal & Srikant, VLDB'94):
// "T<avg txn len>I<avg pattern len>D<n txns>" with |L| potentially-large
// patterns over N items.  Used for BASELINE.json's configs (T10I4D100K,
// T10I4D100M, T40I10D100M) since no dataset can be downloaded.
//
// Counter-based: transaction t is generated from mix64(seed, t) alone, so any
// shard [begin, end) of the database is identical no matter how the database
// is split across ranks/threads (the pattern table depends only on the seed).
// Departure from the original generator (documented): a pattern that does not
// fit is added with probability 1/2 and otherwise dropped instead of being
// carried to the next transaction (carry-over would serialise generation).
#include <cmath>
#include <cstdio>


#include "fa_common.h"
#include "txndb.h"

namespace fa {

struct QuestParams {
  double avg_len, avg_pat_len;
  int64_t n_patterns, n_items;
  uint64_t seed;
  double correlation = 0.5, corrupt_mean = 0.5, corrupt_sd = 0.1;
};

static int64_t poisson(Rng& r, double mean) {
  if (mean <= 0) return 0;
  if (mean < 40) {
    double L = std::exp(-mean), p = 1.0;
    int64_t k = 0;
    do { ++k; p *= r.uniform(); } while (p > L);
    return k - 1;
  }
  double u1 = std::max(r.uniform(), 1e-300), u2 = r.uniform();
  double z = std::sqrt(-2 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  return std::max<int64_t>(0, (int64_t)std::llround(mean + std::sqrt(mean) * z));
}

static double normal(Rng& r, double mu, double sd) {
  double u1 = std::max(r.uniform(), 1e-300), u2 = r.uniform();
  return mu + sd * std::sqrt(-2 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

struct PatternTable {
  std::vector<std::vector<int32_t>> pats;   // item values in [1, n_items]
  std::vector<double> cdf;
  std::vector<double> corrupt;

  explicit PatternTable(const QuestParams& q) {
    Rng r(mix64(q.seed ^ 0x5157455354ull));
    pats.resize(q.n_patterns);
    cdf.resize(q.n_patterns);
    corrupt.resize(q.n_patterns);
    double tot = 0;
    auto contains = [](const std::vector<int32_t>& v, int32_t x) {
      return std::find(v.begin(), v.end(), x) != v.end();
    };
    for (int64_t p = 0; p < q.n_patterns; ++p) {
      int64_t sz = std::max<int64_t>(1, poisson(r, q.avg_pat_len));
      sz = std::min<int64_t>(sz, q.n_items);
      auto& cur = pats[p];
      if (p > 0) {
        const auto& prev = pats[p - 1];
        double frac = std::min(1.0, -q.correlation * std::log(std::max(r.uniform(), 1e-300)));
        int64_t take = std::min<int64_t>({sz, (int64_t)std::llround(frac * sz), (int64_t)prev.size()});
        std::vector<int32_t> pool(prev);
        for (int64_t i = 0; i < take; ++i) {
          size_t j = (size_t)r.below(pool.size());
          cur.push_back(pool[j]);
          pool[j] = pool.back();
          pool.pop_back();
        }
      }
      while ((int64_t)cur.size() < sz) {
        int32_t x = (int32_t)(1 + r.below((uint64_t)q.n_items));
        if (!contains(cur, x)) cur.push_back(x);
      }
      double w = -std::log(std::max(r.uniform(), 1e-300));
      tot += w;
      cdf[p] = tot;
      corrupt[p] = std::min(1.0, std::max(0.0, normal(r, q.corrupt_mean, q.corrupt_sd)));
    }
    for (auto& c : cdf) c /= tot;
  }

  int64_t pick(Rng& r) const {
    double u = r.uniform();
    int64_t i = std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin();
    return std::min<int64_t>(i, (int64_t)cdf.size() - 1);
  }
};

// Generates transaction t into `out` (sorted, distinct item values).
static void gen_txn(const QuestParams& q, const PatternTable& pt, int64_t t, bool user,
                    std::vector<int32_t>& out, std::vector<int32_t>& tmp) {
  Rng r(mix64(q.seed * 0x9E3779B97F4A7C15ull + (uint64_t)t + (user ? 0x7777777ull : 0)));
  out.clear();
  int64_t target = std::max<int64_t>(1, poisson(r, q.avg_len));
  for (int guard = 0; (int64_t)out.size() < target && guard < 64; ++guard) {
    const auto& pat = pt.pats[pt.pick(r)];
    tmp.assign(pat.begin(), pat.end());
    double c = pt.corrupt[&pat - &pt.pats[0]];
    while (!tmp.empty() && r.uniform() < c) {
      size_t j = (size_t)r.below(tmp.size());
      tmp[j] = tmp.back();
      tmp.pop_back();
    }
    if (tmp.empty()) continue;
    if ((int64_t)(out.size() + tmp.size()) > target && !out.empty()) {
      if (r.uniform() < 0.5) break;
    }
    for (int32_t x : tmp)
      if (std::find(out.begin(), out.end(), x) == out.end()) out.push_back(x);
  }
  std::sort(out.begin(), out.end());
  if (user && !out.empty()) {
    // a user basket: a random non-empty subset of up to 4 items of a transaction
    size_t keep = 1 + (size_t)r.below(std::min<size_t>(4, out.size()));
    for (size_t i = 0; i < keep; ++i) {
      size_t j = i + (size_t)r.below(out.size() - i);
      std::swap(out[i], out[j]);
    }
    out.resize(keep);
    std::sort(out.begin(), out.end());
  }
}

}  // namespace fa

using namespace fa;

static QuestParams make_params(double avg_len, double avg_pat_len, int64_t n_patterns,
                               int64_t n_items, uint64_t seed) {
  QuestParams q;
  q.avg_len = avg_len; q.avg_pat_len = avg_pat_len;
  q.n_patterns = std::max<int64_t>(1, n_patterns);
  q.n_items = std::max<int64_t>(1, n_items);
  q.seed = seed;
  return q;
}

// Generates transactions [txn_begin, txn_end) as a numeric-mode TxnDB
// (id = item value + 1, matching the parser's numeric id space).
FA_API TxnDB* fa_quest_generate(int64_t txn_begin, int64_t txn_end, double avg_len,
                                double avg_pat_len, int64_t n_patterns, int64_t n_items,
                                uint64_t seed, int user_mode, int nthreads) {
  QuestParams q = make_params(avg_len, avg_pat_len, n_patterns, n_items, seed);
  PatternTable pt(q);
  auto* db = new TxnDB();
  db->numeric = true;
  db->vocab = q.n_items + 2;
  int64_t n = std::max<int64_t>(0, txn_end - txn_begin);
  int nt = std::max(1, nthreads);
  if (n < (int64_t)nt * 1024) nt = 1;
  db->chunks.assign(nt, TxnChunk());
  parallel_for_threads(nt, [&](int t) {
    int64_t lo = txn_begin + n * t / nt, hi = txn_begin + n * (t + 1) / nt;
    // appended on this thread's stack, moved into the shared array at the end
    // (adjacent TxnChunk headers false-share when appended to in place)
    struct Local { TxnChunk ch; TxnChunk& dst; ~Local() { dst = std::move(ch); } } L{TxnChunk(), db->chunks[t]};
    TxnChunk& ch = L.ch;
    ch.lens.reserve(hi - lo);
    ch.items.reserve((size_t)((hi - lo) * (avg_len + 1)));
    std::vector<int32_t> out, tmp;
    for (int64_t i = lo; i < hi; ++i) {
      gen_txn(q, pt, i, user_mode != 0, out, tmp);
      for (int32_t x : out) ch.items.push_back(x + 1);
      ch.lens.push_back((int64_t)ch.items.size());
    }
  });
  return db;
}

// Writes transactions [0, n_txn) as text ("v1 v2 ...\n" per line).
FA_API int fa_quest_write(const char* path, int64_t n_txn, double avg_len, double avg_pat_len,
                          int64_t n_patterns, int64_t n_items, uint64_t seed, int user_mode,
                          int nthreads) {
  QuestParams q = make_params(avg_len, avg_pat_len, n_patterns, n_items, seed);
  PatternTable pt(q);
  FILE* f = std::fopen(path, "wb");
  if (!f) return 1;
  const int64_t block = 1 << 16;
  int nt = std::max(1, nthreads);
  std::vector<std::string> bufs(nt);
  for (int64_t b0 = 0; b0 < n_txn; b0 += block * nt) {
    parallel_for_threads(nt, [&](int t) {
      std::string& s = bufs[t];
      s.clear();
      std::vector<int32_t> out, tmp;
      char num[16];
      int64_t lo = b0 + block * t, hi = std::min(n_txn, lo + block);
      for (int64_t i = lo; i < hi; ++i) {
        gen_txn(q, pt, i, user_mode != 0, out, tmp);
        for (size_t j = 0; j < out.size(); ++j) {
          int len = std::snprintf(num, sizeof num, "%d", out[j]);
          if (j) s.push_back(' ');
          s.append(num, len);
        }
        s.push_back('\n');
      }
    });
    for (auto& s : bufs) std::fwrite(s.data(), 1, s.size(), f);
  }
  return std::fclose(f) == 0 ? 0 : 2;
}

// ---------------------------------------------------------------------------
// Wide-vocabulary documents (webdocs-scale config; no real webdocs file can be
// fetched).  A document is
//   * a background bag: length ~ lognormal(mean_len, sigma), words drawn without
//     replacement from a Zipf-Mandelbrot law p(k) ~ 1/(k+q)^s over n_items ids
//     (q bounds the head's document frequency like stop-word filtering does), and
//   * one topic (Zipf(1) over n_topics topics); each of the topic's 5-15 core
//     words (drawn from ranks [100, 20100)) joins the document with probability
//     0.8 — the correlated structure that makes deeper itemsets frequent.
// Counter-based per document like the Quest generator.
// ---------------------------------------------------------------------------
namespace fa {
struct ZipfTable {
  std::vector<double> cdf;
  ZipfTable(int64_t n, double s, double q) : cdf((size_t)n) {
    double acc = 0;
    for (int64_t k = 0; k < n; ++k) { acc += 1.0 / std::pow((double)(k + 1) + q, s); cdf[k] = acc; }
    for (auto& c : cdf) c /= acc;
  }
  int64_t sample(Rng& r) const {
    const double u = r.uniform();
    return std::min<int64_t>((int64_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()),
                             (int64_t)cdf.size() - 1);
  }
};
}  // namespace fa

namespace fa {
// The document model above, built once per call and shared by the threads.
struct ZipfModel {
  int64_t n_items, n_topics;
  double mu, sigma;
  uint64_t seed;
  ZipfTable words, topic_law;
  std::vector<std::vector<int64_t>> topics;
  ZipfModel(double mean_len, double sigma_, int64_t n_items_, double s, double q, int64_t n_topics_, uint64_t seed_)
      : n_items(std::max<int64_t>(1, n_items_)), n_topics(std::max<int64_t>(1, n_topics_)),
        mu(std::log(std::max(1.0, mean_len)) - 0.5 * sigma_ * sigma_), sigma(sigma_), seed(seed_),
        words(std::max<int64_t>(1, n_items_), s, q), topic_law(std::max<int64_t>(1, n_topics_), 1.0, 0.0),
        topics((size_t)std::max<int64_t>(1, n_topics_)) {
    Rng r(mix64(seed ^ 0x70F1C5ull));
    const int64_t lo = std::min<int64_t>(100, n_items - 1), span = std::max<int64_t>(1, std::min<int64_t>(20000, n_items - lo));
    for (auto& t : topics) {
      const int64_t c = 5 + (int64_t)r.below(11);
      for (int64_t j = 0; j < c; ++j) t.push_back(lo + (int64_t)r.below((uint64_t)span));
    }
  }
  // document i -> sorted distinct word ids (0-based) in row
  void doc(int64_t i, std::vector<int64_t>& row, std::vector<int64_t>& table) const {
    Rng r(mix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)i));
    const double g = std::sqrt(-2 * std::log(std::max(r.uniform(), 1e-300))) * std::cos(6.283185307179586 * r.uniform());
    int64_t L = (int64_t)std::llround(std::exp(mu + sigma * g));
    L = std::max<int64_t>(1, std::min<int64_t>({L, 20000, n_items}));
    row.clear();
    size_t cap = 64;
    while (cap < (size_t)L * 2 + 64) cap <<= 1;
    table.assign(cap, -1);
    auto add = [&](int64_t it) {
      size_t h = (size_t)mix64((uint64_t)it) & (cap - 1);
      while (table[h] != -1) { if (table[h] == it) return; h = (h + 1) & (cap - 1); }
      table[h] = it;
      row.push_back(it);
    };
    for (int64_t w : topics[(size_t)topic_law.sample(r)])
      if (r.uniform() < 0.8) add(w);
    for (int64_t guard = 0; (int64_t)row.size() < L && guard < L * 8; ++guard) add(words.sample(r));
    std::sort(row.begin(), row.end());
  }
};

// String token of word id x for the string-vocabulary variant: "w" + base-26
// letters of x + 1 (distinct for distinct ids, never a decimal number).
inline int word_token(int64_t x, char* buf) {
  char tmp[24];
  int n = 0;
  uint64_t v = (uint64_t)x + 1;
  while (v) { tmp[n++] = (char)('a' + (v % 26)); v /= 26; }
  buf[0] = 'w';
  for (int j = 0; j < n; ++j) buf[1 + j] = tmp[n - 1 - j];
  return n + 1;
}
}  // namespace fa

FA_API TxnDB* fa_zipf_generate(int64_t txn_begin, int64_t txn_end, double mean_len, double sigma, int64_t n_items,
                               double s, double q, int64_t n_topics, uint64_t seed, int nthreads) {
  ZipfModel zm(mean_len, sigma, n_items, s, q, n_topics, seed);
  auto* db = new TxnDB();
  db->numeric = true;
  db->vocab = zm.n_items + 2;
  const int64_t n = std::max<int64_t>(0, txn_end - txn_begin);
  int nt = std::max(1, nthreads);
  if (n < (int64_t)nt * 256) nt = 1;
  db->chunks.assign(nt, TxnChunk());
  parallel_for_threads(nt, [&](int t) {
    const int64_t lo = txn_begin + n * t / nt, hi = txn_begin + n * (t + 1) / nt;
    // appended on this thread's stack, moved into the shared array at the end
    // (adjacent TxnChunk headers false-share when appended to in place)
    struct Local { TxnChunk ch; TxnChunk& dst; ~Local() { dst = std::move(ch); } } L{TxnChunk(), db->chunks[t]};
    TxnChunk& ch = L.ch;
    ch.lens.reserve(hi - lo);
    std::vector<int64_t> row, table;
    for (int64_t i = lo; i < hi; ++i) {
      zm.doc(i, row, table);
      for (int64_t x : row) ch.items.push_back((int32_t)(x + 2));   // value x+1, numeric id value+1
      ch.lens.push_back((int64_t)ch.items.size());
    }
  });
  return db;
}

// The same documents written as a text file: numeric tokens (value x + 1, as the
// in-memory generator) or, with string_tokens, word-like strings (word_token) so
// the file exercises the dictionary (string-vocabulary) path of the parser/miner.
FA_API int fa_zipf_write(const char* path, int64_t n_txn, double mean_len, double sigma, int64_t n_items, double s,
                         double q, int64_t n_topics, uint64_t seed, int string_tokens, int nthreads) {
  ZipfModel zm(mean_len, sigma, n_items, s, q, n_topics, seed);
  FILE* f = std::fopen(path, "wb");
  if (!f) return 1;
  const int64_t block = 1 << 13;
  int nt = std::max(1, nthreads);
  std::vector<std::string> bufs(nt);
  for (int64_t b0 = 0; b0 < n_txn; b0 += block * nt) {
    parallel_for_threads(nt, [&](int t) {
      std::string& out = bufs[t];
      out.clear();
      std::vector<int64_t> row, table;
      char tok[32];
      const int64_t lo = b0 + block * t, hi = std::min(n_txn, lo + block);
      for (int64_t i = lo; i < hi; ++i) {
        zm.doc(i, row, table);
        for (size_t j = 0; j < row.size(); ++j) {
          const int len = string_tokens ? word_token(row[j], tok)
                                        : std::snprintf(tok, sizeof tok, "%lld", (long long)(row[j] + 1));
          if (j) out.push_back(' ');
          out.append(tok, (size_t)len);
        }
        out.push_back('\n');
      }
    });
    for (auto& b : bufs) std::fwrite(b.data(), 1, b.size(), f);
  }
  return std::fclose(f) == 0 ? 0 : 2;
}
