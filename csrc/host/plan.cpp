// Work-item planner for the trie-shared level kernel (csrc/hip/count.hip
// k_count_trie).
//
// Reference behaviour being scheduled: FastApriori.scala:132-160 counts every
// (prefix x, extensions ys) group by AND-ing x's bitmaps once and then each y.
// The groups arrive in lexicographic prefix order (apriori_gen.cpp), so
// neighbouring groups share leading items: the kernel keeps three partial ANDs
// in registers — P1 (first D1 items), P2 (first D2 items) and p (the whole
// (k-1)-prefix) — and a piece only recomputes the parts whose items changed.
//
// This file chooses D1/D2 from the longest-common-prefix (LCP) histogram of
// consecutive groups, then cuts the group sequence into
//   pieces      (group, ext range <= emax, flags: 2 = recompute P2, 1 = recompute p)
//   work items  (consecutive pieces inside one D1-class, <= emax extensions)
//   passes      (consecutive work items whose extensions fit the LDS accumulator)
// and sorts the work items of a pass by estimated cost so the lanes of a wave
// run loops of similar length.
#include "fa_common.h"

namespace fa {

static inline int lcp_rows(const int32_t* a, const int32_t* b, int m) {
  int i = 0;
  while (i < m && a[i] == b[i]) ++i;
  return i;
}

}  // namespace fa

using namespace fa;

// Reads of slab rows the kernel performs for split depths (d1, d2), estimated
// from nchg[d] = number of groups whose LCP with the previous group is < d.
static int64_t plan_cost(const std::vector<int64_t>& nchg, int64_t G, int64_t C, int m, int d1, int d2,
                         int64_t emax) {
  const int64_t nw = std::max<int64_t>(nchg[d1], (C + emax - 1) / emax);
  return nw * d1 + std::max<int64_t>(nchg[d2], nw) * (d2 - d1) + G * (m - d2) + C;
}

// P: int32 [G][m] prefix rows (lexicographic), ext_off: int64 [G+1].
// d1 < 0 -> choose (d1, d2) by plan_cost.  Outputs (caller-sized):
//   pieces int32 [4 * maxp], witems int32 [2 * maxp], passes int64 [3 * maxp]
//   (work-item begin, end, ext base), info int64 [8]:
//   {n_pieces, n_witems, n_passes, d1, d2, est_reads, reads_unshared, 0}.
// maxp must be >= G + C / emax + 1.
FA_API int fa_plan_trie(const int32_t* P, int64_t G, int m, const int64_t* ext_off, int64_t emax, int64_t cap,
                        int d1, int d2, int32_t* pieces, int32_t* witems, int64_t* passes, int64_t maxp,
                        int64_t* info) {
  if (G <= 0 || m <= 0 || emax <= 0 || cap <= 0) return 1;
  const int64_t C = ext_off[G] - ext_off[0];
  std::vector<uint8_t> lcp((size_t)G, 0);
  std::vector<int64_t> nchg((size_t)m + 1, 0);
  for (int64_t g = 1; g < G; ++g) lcp[g] = (uint8_t)std::min(255, lcp_rows(P + (g - 1) * m, P + g * m, m));
  {
    std::vector<int64_t> hist((size_t)m + 1, 0);
    hist[0] += 1;                                    // the first group changes at every depth
    for (int64_t g = 1; g < G; ++g) hist[lcp[g]] += 1;
    // nchg[d] = #groups with lcp < d
    int64_t run = 0;
    for (int d = 0; d <= m; ++d) { nchg[d] = run; run += hist[d]; }
    // lcp can equal m only for duplicate rows (never: rows are distinct)
  }
  if (d1 < 0) {
    int64_t best = -1;
    for (int a = 0; a <= m; ++a)
      for (int b = a; b <= m; ++b) {
        const int64_t c = plan_cost(nchg, G, C, m, a, b, emax);
        if (best < 0 || c < best) { best = c; d1 = a; d2 = b; }
      }
  }
  if (!(0 <= d1 && d1 <= d2 && d2 <= m)) return 2;

  int64_t np = 0, nw = 0, npass = 0;
  int64_t w_open = -1, w_ext = 0;                    // current work item
  int64_t pass_base = ext_off[0], pass_ext = 0, pass_w0 = 0;
  int64_t reads = 0, reads_unshared = 0;
  auto close_w = [&]() {
    if (w_open >= 0) { witems[2 * nw] = (int32_t)w_open; witems[2 * nw + 1] = (int32_t)np; ++nw; }
    w_open = -1; w_ext = 0;
  };
  auto close_pass = [&](int64_t next_base) {
    close_w();
    if (nw > pass_w0) {
      passes[3 * npass] = pass_w0; passes[3 * npass + 1] = nw; passes[3 * npass + 2] = pass_base;
      ++npass;
    }
    pass_w0 = nw; pass_base = next_base; pass_ext = 0;
  };
  for (int64_t g = 0; g < G; ++g) {
    int64_t e = ext_off[g];
    const int64_t e_end = ext_off[g + 1];
    bool first_chunk = true;
    while (e < e_end) {
      const int64_t chunk = std::min<int64_t>(e_end - e, emax);
      if (np >= maxp) return 3;
      if (pass_ext + chunk > cap) close_pass(e);
      const bool row_new = first_chunk;
      const bool new_w = w_open < 0 || (row_new && lcp[g] < d1) || w_ext + chunk > emax;
      int flags;
      if (new_w) {
        close_w();
        w_open = np;
        flags = 3;
        reads += d1 + (d2 - d1) + (m - d2);
      } else {
        flags = row_new ? (1 | (lcp[g] < d2 ? 2 : 0)) : 0;
        reads += ((flags & 2) ? d2 - d1 : 0) + ((flags & 1) ? m - d2 : 0);
      }
      reads += chunk;
      reads_unshared += m + chunk;
      pieces[4 * np + 0] = (int32_t)(g * m);
      pieces[4 * np + 1] = (int32_t)(e - pass_base);
      pieces[4 * np + 2] = (int32_t)(e + chunk - pass_base);
      pieces[4 * np + 3] = flags;
      ++np;
      w_ext += chunk;
      pass_ext += chunk;
      e += chunk;
      first_chunk = false;
    }
  }
  close_pass(ext_off[G]);

  // order the work items of every pass by estimated cost (descending)
  std::vector<int64_t> cost;
  std::vector<int32_t> tmp;
  std::vector<int64_t> idx;
  for (int64_t q = 0; q < npass; ++q) {
    const int64_t w0 = passes[3 * q], w1 = passes[3 * q + 1];
    const int64_t n = w1 - w0;
    cost.assign((size_t)n, 0);
    for (int64_t w = w0; w < w1; ++w) {
      int64_t c = d1;
      for (int64_t p = witems[2 * w]; p < witems[2 * w + 1]; ++p) {
        const int f = pieces[4 * p + 3];
        c += ((f & 2) ? d2 - d1 : 0) + ((f & 1) ? m - d2 : 0) + (pieces[4 * p + 2] - pieces[4 * p + 1]);
      }
      cost[w - w0] = c;
    }
    idx.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return cost[a] > cost[b]; });
    tmp.assign(witems + 2 * w0, witems + 2 * w1);
    for (int64_t i = 0; i < n; ++i) {
      witems[2 * (w0 + i)] = tmp[2 * idx[i]];
      witems[2 * (w0 + i) + 1] = tmp[2 * idx[i] + 1];
    }
  }
  info[0] = np; info[1] = nw; info[2] = npass; info[3] = d1; info[4] = d2;
  info[5] = reads; info[6] = reads_unshared; info[7] = 0;
  return 0;
}
