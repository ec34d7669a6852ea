// Native self-test of the host runtime (libfa_host sources linked statically),
// built twice by tests/test_native_sanitizers.py:
//   * -fsanitize=address,undefined  (memory errors, UB)
//   * -fsanitize=thread             (data races in the thread pool and every
//                                    parallel_for user: parser, generators,
//                                    apriori_gen, rules, CPU kernels, writer)
// Each check compares a parallel native routine against a simple serial
// recomputation in this file; any mismatch or sanitizer report fails the run.
// SURVEY.md §5.2 (race detection / sanitizers).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

extern "C" {
void* fa_parse_buffer(const char* data, int64_t size, int mode, int nthreads);
void fa_txndb_info(void* db, int64_t* info);
void fa_txndb_export(void* db, int64_t* offsets, int32_t* items, int32_t* extras, int nthreads);
void fa_txndb_export_dict(void* db, char* buf, int64_t* str_off, uint64_t* hashes);
void fa_txndb_free(void* db);
void* fa_quest_generate(int64_t b, int64_t e, double avg_len, double avg_pat, int64_t n_pat, int64_t n_items,
                        uint64_t seed, int user_mode, int nthreads);
void* fa_zipf_generate(int64_t b, int64_t e, double mean_len, double sigma, int64_t n_items, double s, double q,
                       int64_t n_topics, uint64_t seed, int nthreads);
void* fa_apriori_gen(const int32_t* prev, int64_t n, int m, int nthreads, int64_t* sizes);
void fa_cands_export(void* c, int32_t* prefix, int64_t* ext_off, int32_t* ext);
void fa_cands_free(void* c);
void* fa_rules_build(const int32_t* const* rows, const int64_t* const* counts, const int64_t* sizes, int levels,
                     const int64_t* tie_pos, int nthreads, int64_t* n_rules);
int64_t fa_rules_nante(void* rs);
int64_t fa_rules_nstats(void* rs);
void fa_rules_export(void* rs, int64_t* ante_off, int32_t* ante, int32_t* cons, double* conf, int64_t* stats);
void fa_rules_free(void* rs);
void fa_recommend_cpu(const int64_t* ante_off, const int32_t* ante, const int32_t* cons, int64_t R, int32_t F1,
                      const int64_t* bask_off, const int32_t* bask, int64_t M, int32_t* out, int nthreads);
int fa_write_freq_itemsets(const char* path, const char* tokbuf, const int64_t* tokoff, int32_t F1,
                           const int32_t* const* rows, const int64_t* const* counts, const int64_t* sizes,
                           int levels, int with_counts, int nthreads);
void fa_cpu_histogram(const int32_t* items, int64_t nnz, int64_t V, int64_t* out, int nthreads);
void fa_cpu_build_bitmaps(const int64_t* roff, const int32_t* ranks, const int32_t* src, int64_t ncols, int64_t Wp,
                          uint64_t* bm, int nthreads);
void fa_cpu_pair_gram(const uint64_t* bm, int32_t F1, int64_t Wp, int64_t W, const int32_t* wword, int64_t* out,
                      int nthreads);
void fa_cpu_pair_horizontal(const int64_t* roff, const int32_t* ranks, int64_t T, const int32_t* wrow, int32_t F1,
                            int64_t* out, int nthreads);
void fa_cpu_row_hash(const int64_t* roff, const int32_t* ranks, int64_t T, int64_t* h1, int64_t* h2, int nthreads);
}

static int g_fail = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

struct Db {
  std::vector<int64_t> off;
  std::vector<int32_t> items, extras;
  int64_t vocab = 0;
  bool numeric = true;
  std::vector<std::string> dict;
};

static Db export_db(void* h, int nt) {
  int64_t info[6];
  fa_txndb_info(h, info);
  Db d;
  d.off.assign(info[0] + 1, 0);
  d.items.assign(std::max<int64_t>(info[1], 1), 0);
  d.extras.assign(std::max<int64_t>(info[2], 1), 0);
  d.numeric = info[3] != 0;
  d.vocab = info[4];
  fa_txndb_export(h, d.off.data(), d.items.data(), d.extras.data(), nt);
  if (!d.numeric) {
    std::vector<char> buf(std::max<int64_t>(info[5], 1));
    std::vector<int64_t> so(info[4] + 1);
    std::vector<uint64_t> hs(std::max<int64_t>(info[4], 1));
    fa_txndb_export_dict(h, buf.data(), so.data(), hs.data());
    for (int64_t i = 0; i < info[4]; ++i) d.dict.emplace_back(buf.data() + so[i], (size_t)(so[i + 1] - so[i]));
  }
  fa_txndb_free(h);
  d.items.resize(info[1]);
  d.extras.resize(info[2]);
  return d;
}

// Java trim().split("\\s+") over Hadoop lines, serially, as token strings.
static std::vector<std::vector<std::string>> serial_parse(const std::string& s) {
  std::vector<std::string> lines;
  std::string cur;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '\n' || s[i] == '\r') {
      lines.push_back(cur);
      cur.clear();
      if (s[i] == '\r' && i + 1 < s.size() && s[i + 1] == '\n') ++i;
    } else {
      cur.push_back(s[i]);
    }
  }
  if (!cur.empty()) lines.push_back(cur);
  std::vector<std::vector<std::string>> out;
  for (auto& l : lines) {
    size_t a = 0, b = l.size();
    while (a < b && (uint8_t)l[a] <= 0x20) ++a;
    while (b > a && (uint8_t)l[b - 1] <= 0x20) --b;
    std::vector<std::string> toks;
    std::string t = l.substr(a, b - a);
    if (t.empty()) {
      toks.push_back("");
    } else {
      std::string w;
      for (char c : t) {
        if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v') {
          if (!w.empty()) toks.push_back(w), w.clear();
        } else {
          w.push_back(c);
        }
      }
      if (!w.empty()) toks.push_back(w);
    }
    out.push_back(toks);
  }
  return out;
}

static void test_parser(int nt) {
  std::mt19937_64 rng(7);
  const char* words[] = {"1", "2", "17", "apple", "x", "3", "banana", "42"};
  const char* seps[] = {" ", "\t", "  ", " \t "};
  const char* ends[] = {"\n", "\r\n", "\r", "\n\n"};
  for (int rep = 0; rep < 3; ++rep) {
    std::string s;
    const bool dict = rep == 2;
    for (int i = 0; i < 4000; ++i) {
      int n = (int)(rng() % 7);
      if (rng() % 9 == 0) s += "  ";
      for (int j = 0; j < n; ++j) {
        s += words[rng() % (dict ? 8 : 4)];
        if (j + 1 < n) s += seps[rng() % 4];
      }
      s += ends[rng() % 4];
    }
    Db d = export_db(fa_parse_buffer(s.data(), (int64_t)s.size(), dict ? 1 : 0, nt), nt);
    auto ref = serial_parse(s);
    CHECK((int64_t)ref.size() == (int64_t)d.off.size() - 1);
    // distinct tokens per line + extras (duplicates) must equal the serial token multiset
    std::map<std::string, int64_t> want, got;
    for (auto& l : ref)
      for (auto& t : l) want[t]++;
    auto tok = [&](int32_t id) -> std::string {
      if (!d.numeric) return d.dict[id];
      return id == 0 ? std::string() : std::to_string(id - 1);
    };
    for (int32_t id : d.items) got[tok(id)]++;
    for (int32_t id : d.extras) got[tok(id)]++;
    CHECK(want == got);
  }
}

static void test_generators(int nt) {
  // shard invariance: [0,n) == [0,a) ++ [a,n)
  for (int z = 0; z < 2; ++z) {
    auto gen = [&](int64_t b, int64_t e) {
      return export_db(z ? fa_zipf_generate(b, e, 40.0, 0.5, 200000, 1.05, 50.0, 50, 3, nt)
                         : fa_quest_generate(b, e, 10.0, 4.0, 200, 300, 3, 0, nt), nt);
    };
    Db all = gen(0, 6000), a = gen(0, 2500), b = gen(2500, 6000);
    std::vector<int32_t> cat(a.items);
    cat.insert(cat.end(), b.items.begin(), b.items.end());
    CHECK(cat == all.items);
    CHECK(all.off.back() == a.off.back() + b.off.back());
  }
}

static void test_apriori_gen(int nt) {
  std::mt19937_64 rng(11);
  for (int m = 2; m <= 4; ++m) {
    const int F1 = 22;
    // at most half of the C(F1, m) possible rows (C(22, 2) = 231)
    int64_t total = 1;
    for (int q = 0; q < m; ++q) total = total * (F1 - q) / (q + 1);
    const int64_t target = std::min<int64_t>(300, total / 2);
    std::set<std::vector<int32_t>> prev;
    while ((int64_t)prev.size() < target) {
      std::vector<int32_t> r;
      std::set<int32_t> s;
      while ((int)s.size() < m) s.insert((int32_t)(rng() % F1));
      r.assign(s.begin(), s.end());
      prev.insert(r);
    }
    std::vector<int32_t> flat;
    for (auto& r : prev) flat.insert(flat.end(), r.begin(), r.end());
    int64_t sizes[2];
    void* c = fa_apriori_gen(flat.data(), (int64_t)prev.size(), m, nt, sizes);
    std::vector<int32_t> pre(std::max<int64_t>(sizes[0], 1)), ext(std::max<int64_t>(sizes[1], 1));
    std::vector<int64_t> off(sizes[0] + 1);
    fa_cands_export(c, pre.data(), off.data(), ext.data());
    fa_cands_free(c);
    std::set<std::vector<int32_t>> got, want;
    std::vector<std::vector<int32_t>> rows(prev.begin(), prev.end());
    for (int64_t g = 0; g < sizes[0]; ++g)
      for (int64_t e = off[g]; e < off[g + 1]; ++e) {
        std::vector<int32_t> x = rows[pre[g]];
        x.push_back(ext[e]);
        got.insert(x);
      }
    for (auto& x : rows)
      for (int32_t y = x.back() + 1; y < F1; ++y) {
        std::vector<int32_t> cand = x;
        cand.push_back(y);
        bool ok = true;
        for (int drop = 0; drop < m && ok; ++drop) {
          std::vector<int32_t> sub;
          for (int q = 0; q <= m; ++q)
            if (q != drop) sub.push_back(cand[q]);
          ok = prev.count(sub) > 0;
        }
        if (ok) want.insert(cand);
      }
    CHECK(got == want);
  }
}

static void test_kernels_and_rules(int nt) {
  Db d = export_db(fa_quest_generate(0, 3000, 8.0, 3.0, 60, 40, 5, 0, nt), nt);
  const int64_t T = (int64_t)d.off.size() - 1;
  const int32_t F1 = (int32_t)d.vocab;   // numeric ids: value + 1 (0 = the empty token)
  // histogram
  std::vector<int64_t> h(F1, 0), hr(F1, 0);
  fa_cpu_histogram(d.items.data(), (int64_t)d.items.size(), F1, h.data(), nt);
  for (int32_t x : d.items) hr[x]++;
  CHECK(h == hr);
  // rows of ids as ranks (already sorted, distinct); bitmaps; pairs two ways
  std::vector<int64_t> pa((size_t)F1 * F1, 0), pb((size_t)F1 * F1, 0);
  fa_cpu_pair_horizontal(d.off.data(), d.items.data(), T, nullptr, F1, pa.data(), nt);
  const int64_t W = (T + 63) / 64, Wp = W;
  std::vector<uint64_t> bm((size_t)F1 * Wp, 0);
  fa_cpu_build_bitmaps(d.off.data(), d.items.data(), nullptr, T, Wp, bm.data(), nt);
  fa_cpu_pair_gram(bm.data(), F1, Wp, W, nullptr, pb.data(), nt);
  for (int32_t i = 0; i < F1; ++i)
    for (int32_t j = i + 1; j < F1; ++j) CHECK(pa[(size_t)i * F1 + j] == pb[(size_t)i * F1 + j]);
  std::vector<int64_t> h1(T), h2(T);
  fa_cpu_row_hash(d.off.data(), d.items.data(), T, h1.data(), h2.data(), nt);
  for (int64_t t = 1; t < T; ++t) {
    const bool same = std::equal(d.items.begin() + d.off[t - 1], d.items.begin() + d.off[t],
                                 d.items.begin() + d.off[t], d.items.begin() + d.off[t + 1]);
    if (same) CHECK(h1[t] == h1[t - 1] && h2[t] == h2[t - 1]);
  }
  // rules: levels 1..2 from the pair counts (min count 1), then recommendation
  std::vector<int32_t> r1, r2;
  std::vector<int64_t> c1, c2;
  for (int32_t i = 0; i < F1; ++i) r1.push_back(i), c1.push_back(std::max<int64_t>(h[i], 1));
  for (int32_t i = 0; i < F1; ++i)
    for (int32_t j = i + 1; j < F1; ++j)
      if (pa[(size_t)i * F1 + j] > 0) {
        r2.push_back(i), r2.push_back(j);
        c2.push_back(std::min(pa[(size_t)i * F1 + j], std::min(c1[i], c1[j])));
      }
  const int32_t* rows[2] = {r1.data(), r2.data()};
  const int64_t* cnts[2] = {c1.data(), c2.data()};
  int64_t sizes[2] = {F1, (int64_t)c2.size()};
  std::vector<int64_t> tie(F1);
  for (int32_t i = 0; i < F1; ++i) tie[i] = i;
  int64_t n_rules = 0;
  void* rs = fa_rules_build(rows, cnts, sizes, 2, tie.data(), nt, &n_rules);
  const int64_t R = n_rules;
  std::vector<int64_t> aoff(R + 1), stats(std::max<int64_t>(fa_rules_nstats(rs), 1));
  std::vector<int32_t> ante(std::max<int64_t>(fa_rules_nante(rs), 1)), cons(std::max<int64_t>(R, 1));
  std::vector<double> conf(std::max<int64_t>(R, 1));
  fa_rules_export(rs, aoff.data(), ante.data(), cons.data(), conf.data(), stats.data());
  fa_rules_free(rs);
  for (int64_t r = 1; r < R; ++r) CHECK(conf[r - 1] >= conf[r]);
  std::vector<int32_t> out(T);
  fa_recommend_cpu(aoff.data(), ante.data(), cons.data(), R, F1, d.off.data(), d.items.data(), T, out.data(), nt);
  for (int64_t u = 0; u < std::min<int64_t>(T, 200); ++u) {   // serial first match
    int32_t want = -1;
    std::set<int32_t> B(d.items.begin() + d.off[u], d.items.begin() + d.off[u + 1]);
    for (int64_t r = 0; r < R && want < 0 && !B.empty(); ++r) {
      if (B.count(cons[r])) continue;
      bool sub = true;
      for (int64_t a = aoff[r]; a < aoff[r + 1] && sub; ++a) sub = B.count(ante[a]) > 0;
      if (sub) want = cons[r];
    }
    CHECK(out[u] == want);
  }
  // writer
  std::string tokbuf;
  std::vector<int64_t> tokoff{0};
  for (int32_t i = 0; i < F1; ++i) tokbuf += std::to_string(i), tokoff.push_back((int64_t)tokbuf.size());
  const char* path = "/tmp/fa_selftest_freq.txt";
  CHECK(fa_write_freq_itemsets(path, tokbuf.data(), tokoff.data(), F1, rows, cnts, sizes, 2, 1, nt) == 0);
  FILE* f = std::fopen(path, "rb");
  CHECK(f != nullptr);
  if (f) {
    int64_t lines = 0;
    for (int ch; (ch = std::fgetc(f)) != EOF;) lines += ch == '\n';
    std::fclose(f);
    CHECK(lines == sizes[0] + sizes[1]);
    std::remove(path);
  }
}

int main(int argc, char** argv) {
  const int nt = argc > 1 ? std::atoi(argv[1]) : 8;
  test_parser(nt);
  test_generators(nt);
  test_apriori_gen(nt);
  test_kernels_and_rules(nt);
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("selftest ok\n");
  return 0;
}
