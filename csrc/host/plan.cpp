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
#include <algorithm>
#include <cstring>
#include <vector>

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

// Piece records for k_count_trie: 32 B per piece (8 int32), so a piece is two
// 16-B loads with no dependent index chain and the kernel loads the next piece's
// record while it counts the current one.  (A piece used to cost three
// serialised global latencies: its descriptor, then its prefix ids, then its
// first extension ids.)
//   a.x = ext begin (pass-local, bits 0-16) | n_ext << 17 (6 bits) | flags << 23
//         (2 bits) | long << 25 (prefix ids not inline: read gpre)
//   a.y = gpre offset of the piece's prefix row
//   a.z, a.w = extension ids 0-3 (u16 slab rows)
//   b   = prefix ids D1 .. m-1 (u16 slab rows, <= 8 of them; else long)
// rec must hold 8 * n_pieces int32 and be 16-B aligned.  Returns 0, or 2 when a
// field does not fit its bits.
FA_API int fa_trie_records(const int32_t* pieces, const int32_t* witems, const int64_t* passes, int64_t npass,
                           const int32_t* gpre, const int32_t* gext, int m, int d1, int32_t* rec) {
  auto pk = [](int32_t x, int32_t y) { return (uint32_t)(x & 0xFFFF) | ((uint32_t)(y & 0xFFFF) << 16); };
  const bool inl = m - d1 <= 8;
  for (int64_t q = 0; q < npass; ++q) {
    const int64_t base = passes[3 * q + 2];
    for (int64_t w = passes[3 * q]; w < passes[3 * q + 1]; ++w) {
      for (int64_t p = witems[2 * w]; p < witems[2 * w + 1]; ++p) {
        const int32_t* pc = pieces + 4 * p;
        const int32_t lo = pc[1], n = pc[2] - pc[1];
        if (lo < 0 || lo >= (1 << 17) || n < 0 || n >= 64) return 2;
        uint32_t* r = reinterpret_cast<uint32_t*>(rec + 8 * p);
        int32_t ex4[4] = {0, 0, 0, 0};
        for (int32_t k = 0; k < std::min<int32_t>(n, 4); ++k) ex4[k] = gext[base + lo + k];
        r[0] = (uint32_t)lo | ((uint32_t)n << 17) | ((uint32_t)(pc[3] & 3) << 23) | (inl ? 0u : 1u << 25);
        r[1] = (uint32_t)pc[0];
        r[2] = pk(ex4[0], ex4[1]);
        r[3] = pk(ex4[2], ex4[3]);
        int32_t ids[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (inl)
          for (int t = d1; t < m; ++t) ids[t - d1] = gpre[pc[0] + t];
        for (int k = 0; k < 4; ++k) r[4 + k] = pk(ids[2 * k], ids[2 * k + 1]);
      }
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------
// One-call level planner: everything the level kernels need, computed in C++
// and written into one (pinned) int32 buffer so the driver issues a single
// host->device copy per level.
//
//   params (double[10]): lds_bytes, min_saving (0 = always trie, >1 = never),
//                       conflict16, conflict8, pass_weight, rounds, emax_max, W,
//                       LDS bytes per accumulator (4, or 2 for packed 16-bit counters),
//                       class layout of slab passes (1: where it saves reads, 2: always)
//   info (int64[24]) out:
//     0 kernel (0 slab, 1 trie)  1 sw  2 cap  3 n_used  4 n_pieces  5 n_witems
//     6 n_passes  7 d1  8 d2  9 trie reads  10 slab reads  11 emax
//     12 off item_map  13 off used  14 off gext  15 off gpre  16 off pieces/loc_off
//     17 off witems  18 total int32 written  19 off gpm (slab)  20 off piece records (slab)
//     21 slab wave-step reads, size-sorted  22 the same, class layout (0: not tried)
//     23 class layout used by some pass (record flags set: k_count_slab_rec<.., kCls>)
//   passes (int64[3 * maxpass]): slab: (piece begin, piece end, ext base);
//                                trie: (witem begin, witem end, ext base)
// Returns 0, 3 (buffer too small), 4 (no slab width fits: use the bitmap kernel).
// ---------------------------------------------------------------------------
// Width order 16, 32, 8, 4: measured per slab column on MI355X (T40I10D100M levels
// 7-10, k_count_slab_rec), 64-B rows read ~0.43x and 256-B rows ~0.55x as many
// columns per second as 128-B rows (the 256-B form holds 16 uint4 of prefix AND
// per thread: fewer waves, longer row scans per LDS bank).
static int slab_width(int64_t n_used, int64_t C, double lds, int64_t* cap_out, double accb = 4,
                      double map_lds = 0) {
  for (int sw : {16, 32, 8, 4}) {
    // + the LDS copy of the rank -> slab-row map (u16 per frequent item, k_count_slab_rec)
    const int64_t cap = (int64_t)((lds - (double)n_used * (sw + 2) * 8 - map_lds) / accb);
    if (cap >= std::min<int64_t>(C, 8192) || (sw == 4 && cap >= 1024)) { *cap_out = cap; return sw; }
  }
  return 0;
}

// LDS bytes of k_count_slab_rec's copy of the rank -> slab-row map (u16 per
// frequent item; 0 = the map stays in global memory).  count.hip mirrors this.
static inline int64_t fa_slab_map_lds(int64_t F1) { return F1 <= 8192 ? ((F1 * 2 + 15) & ~(int64_t)15) : 0; }

// ---------------------------------------------------------------------------
// Class layout of a slab pass (k_count_slab_rec<.., kCls>).  Pieces whose prefixes
// share their first m-1 items (siblings in the candidate trie: one equivalence
// class of the (k-2)-prefix, FastApriori.scala:132-160 groups by the (k-1)-prefix
// only) are counted by one thread in a row: it ANDs the m-1 shared rows once (q),
// then per piece one row (p = q & last item) and its extensions.  On T40I10D100K
// levels 7-11 this reads 0.63-0.67x the slab rows of the size-sorted layout.
// A wave's 64 lanes must branch alike, so classes of equal length s (<= 8 pieces)
// fill the lanes of one "wave row" (s steps), classes sorted by their extension
// counts so the lanes' extension loops match, and the wave rows go to the 16 waves
// of the workgroup longest first onto the least-loaded wave.  Slot s of a pass is
// step s / 1024 of thread s % 1024 (count.hip kSlabThreads); idle slots keep both
// partial ANDs and have no extensions.  Record flags: kRecKeepQ = the shared
// m-1 rows are the previous piece's, kRecKeepP = the whole prefix is.
// ---------------------------------------------------------------------------
struct SlabPiece { int64_t g, lo, hi; };
constexpr int kSlabWg = 1024;              // count.hip kSlabThreads
constexpr int kClsMaxRun = 8;              // pieces per class run (longer classes are cut)
constexpr double kClsMinGain = 0.8;        // class layout only when its wave-step reads are < 0.8x
constexpr uint8_t kRecKeepQ = 1, kRecKeepP = 2;

// Critical path of a pass in slab-row reads per lane: the SIMT cost of a wave step (the
// longest extension loop of its lanes, a recompute if any lane needs one, + 1 for the
// record and loop), summed over each wave's steps; the busiest wave, since all 16 meet
// at every slab's barrier.
static int64_t slot_cost(const std::vector<SlabPiece>& pcs, const std::vector<int64_t>& slots,
                         const std::vector<uint8_t>& flags, int m) {
  int64_t wc[kSlabWg / 64] = {0};
  const int64_t n = (int64_t)slots.size();
  for (int64_t w0 = 0; w0 < n; w0 += 64) {
    bool q = false, p = false, any = false;
    int64_t e = 0;
    for (int64_t s = w0; s < std::min(n, w0 + 64); ++s) {
      if (slots[s] < 0) continue;
      any = true;
      q = q || !(flags[s] & kRecKeepQ);
      p = p || !(flags[s] & kRecKeepP);
      e = std::max(e, pcs[slots[s]].hi - pcs[slots[s]].lo);
    }
    if (any) wc[(w0 % kSlabWg) / 64] += (q ? m - 1 : 0) + (p ? 1 : 0) + e + 1;
  }
  return *std::max_element(wc, wc + kSlabWg / 64);
}

static void cls_layout(const std::vector<SlabPiece>& pcs, int64_t i, int64_t j, const int32_t* Pf,
                       const int64_t* poff, int m, std::vector<int64_t>& slots, std::vector<uint8_t>& flags) {
  struct Run { int64_t k0; int s; };
  std::vector<Run> runs;
  for (int64_t k = i; k < j; ++k) {
    bool same = k > i && runs.back().s < kClsMaxRun;
    if (same && pcs[k].g != pcs[k - 1].g) {
      const int32_t* a = Pf + poff[pcs[k - 1].g];
      const int32_t* b = Pf + poff[pcs[k].g];
      same = std::equal(a, a + m - 1, b);
    }
    if (same) runs.back().s += 1;
    else runs.push_back({k, 1});
  }
  // runs longest first; equal lengths keep their lexicographic order, so the lanes of a
  // wave read mostly the same prefix rows (LDS broadcast) -- measured better than
  // ordering them by extension counts
  std::stable_sort(runs.begin(), runs.end(), [&](const Run& x, const Run& y) { return x.s > y.s; });
  // wave rows of <= 64 runs of one length, costliest first, each to the wave with the
  // least estimated reads so far: the waves meet at every slab's barrier, so the
  // critical path is the busiest wave (slot_cost)
  constexpr int NWv = kSlabWg / 64;
  struct Row { int64_t r0, r1, cost; };
  std::vector<Row> rows;
  for (int64_t r = 0; r < (int64_t)runs.size();) {
    int64_t r1 = r + 1;
    while (r1 < (int64_t)runs.size() && r1 - r < 64 && runs[r1].s == runs[r].s) ++r1;
    int64_t c = 0;
    for (int e = 0; e < runs[r].s; ++e) {
      int64_t mx = 0;
      bool newp = e == 0;
      for (int64_t x = r; x < r1; ++x) {
        const int64_t k = runs[x].k0 + e;
        mx = std::max(mx, pcs[k].hi - pcs[k].lo);
        newp = newp || pcs[k].g != pcs[k - 1].g;
      }
      c += (e == 0 ? m - 1 : 0) + (newp ? 1 : 0) + mx + 1;   // + 1: per-step record and loop cost
    }
    rows.push_back({r, r1, c});
    r = r1;
  }
  std::stable_sort(rows.begin(), rows.end(), [](const Row& x, const Row& y) { return x.cost > y.cost; });
  std::vector<std::vector<std::pair<int64_t, int64_t>>> rows_of(NWv);   // (first run, end run)
  int64_t load[NWv] = {0}, wcost[NWv] = {0};
  for (const Row& rw : rows) {
    const int w = (int)(std::min_element(wcost, wcost + NWv) - wcost);
    rows_of[w].push_back({rw.r0, rw.r1});
    load[w] += runs[rw.r0].s;
    wcost[w] += rw.cost;
  }
  const int64_t T = *std::max_element(load, load + NWv);
  slots.assign((size_t)(T * kSlabWg), -1);
  flags.assign((size_t)(T * kSlabWg), kRecKeepQ | kRecKeepP);
  for (int w = 0; w < NWv; ++w) {
    int64_t t = 0;
    for (const auto& row : rows_of[w]) {
      const int s = runs[row.first].s;
      for (int64_t r = row.first; r < row.second; ++r) {
        const int64_t lane = r - row.first;
        for (int e = 0; e < s; ++e) {
          const int64_t k = runs[r].k0 + e;
          const size_t at = (size_t)((t + e) * kSlabWg + w * 64 + lane);
          slots[at] = k;
          flags[at] = e == 0 ? 0 : (uint8_t)(kRecKeepQ | (pcs[k].g == pcs[k - 1].g ? kRecKeepP : 0));
        }
      }
      t += s;
    }
  }
}

FA_API int fa_level_plan(const int32_t* Pf, const int64_t* poff, int64_t G, const int64_t* ext_off,
                         const int32_t* ext, int32_t F1, const double* params, int32_t* buf, int64_t buf_cap,
                         int64_t* passes, int64_t max_pass, int64_t* info) {
  const double lds = params[0], min_saving = params[1], conf16 = params[2], conf8 = params[3];
  const double pass_w = params[4], rounds = params[5];
  const int64_t emax_max = (int64_t)params[6];
  const double W = params[7];
  const double accb = params[8] > 0 ? params[8] : 4;   // LDS bytes per accumulator (2: packed 16-bit)
  const int64_t C = ext_off[G] - ext_off[0];
  for (int i = 0; i < 24; ++i) info[i] = 0;
  if (G <= 0 || C <= 0) return 1;
  // prefix lengths: uniform for one level, mixed when several levels share a launch
  const int m0 = (int)(poff[1] - poff[0]);
  bool uniform = true;
  int64_t sum_m = 0;
  for (int64_t g = 0; g < G; ++g) {
    const int mg = (int)(poff[g + 1] - poff[g]);
    uniform = uniform && mg == m0;
    sum_m += mg;
  }
  // used items and the rank -> slab-row map
  std::vector<uint8_t> mark((size_t)std::max(F1, 1), 0);
  for (int64_t i = poff[0]; i < poff[G]; ++i) mark[Pf[i]] = 1;
  for (int64_t e = 0; e < C; ++e) mark[ext[ext_off[0] + e]] = 1;
  int64_t pos = 0;
  auto need = [&](int64_t n) { return pos + n <= buf_cap; };
  if (!need(2 * (int64_t)F1 + C)) return 3;
  int32_t* item_map = buf + pos; info[12] = pos; pos += F1;
  int32_t* used = buf + pos; info[13] = pos;
  int64_t n_used = 0;
  for (int32_t r = 0; r < F1; ++r) {
    if (mark[r]) { item_map[r] = (int32_t)n_used; used[n_used++] = r; } else item_map[r] = -1;
  }
  pos += n_used;
  int32_t* gext = buf + pos; info[14] = pos; pos += C;
  for (int64_t e = 0; e < C; ++e) gext[e] = item_map[ext[ext_off[0] + e]];
  info[3] = n_used;

  // slab-kernel reads: pieces of <= 8 extensions, each ANDs its whole prefix
  int64_t pieces8 = 0, slab_reads = C;
  for (int64_t g = 0; g < G; ++g) {
    const int64_t np = std::max<int64_t>(1, (ext_off[g + 1] - ext_off[g] + 7) / 8);
    pieces8 += np;
    slab_reads += np * (poff[g + 1] - poff[g]);
  }
  info[10] = slab_reads;

  // ---- trie kernel (one level: uniform prefix length): slab width by the time model, then the plan
  if (uniform && min_saving <= 1.0) {
    const int m = m0;
    const int32_t* P = Pf + poff[0];
    int best_sw = 0;
    int64_t best_cap = 0;
    double best_t = 0;
    const double reads_est = (double)C + 0.5 * (double)G * m;
    for (int sw : {32, 16, 8}) {
      const int64_t cap = (int64_t)((lds - (double)n_used * sw * 8) / accb);
      if (cap < std::min<int64_t>(C, 1024)) continue;
      const int64_t passes_n = (C + cap - 1) / cap;
      double t = reads_est * W * 8 * (sw == 32 ? 1.0 : sw == 16 ? conf16 : conf8) / 60e12;
      if (passes_n > 1) t += pass_w * passes_n * (double)n_used * W * 8 / 5e12;
      if (best_sw == 0 || t < best_t) { best_sw = sw; best_cap = cap; best_t = t; }
    }
    if (best_sw) {
      const int64_t ngrp = 4096 / best_sw;
      const int64_t emax = std::max<int64_t>(2, std::min<int64_t>(emax_max,
                                             std::min<int64_t>(C, best_cap) / (int64_t)(rounds * ngrp)));
      const int64_t maxp = G + C / emax + 2;
      if (!need(G * m + 6 * maxp)) return 3;
      int32_t* gpre = buf + pos;
      const int64_t o_gpre = pos;
      for (int64_t i = 0; i < G * m; ++i) gpre[i] = item_map[P[i]];
      int32_t* pieces = buf + pos + G * m;
      int32_t* witems = pieces + 4 * maxp;
      std::vector<int64_t> pas(3 * (size_t)maxp);
      int64_t tinfo[8];
      const int rc = fa_plan_trie(P, G, m, ext_off, emax, best_cap, -1, -1, pieces, witems, pas.data(), maxp, tinfo);
      if (rc != 0) return 10 + rc;
      info[9] = tinfo[5];
      if (min_saving <= 0.0 || (double)tinfo[5] <= min_saving * (double)slab_reads) {
        if (tinfo[2] > max_pass) return 3;
        const int64_t np = tinfo[0], nw = tinfo[1];
        std::memmove(pieces + 4 * np, witems, sizeof(int32_t) * 2 * nw);
        info[0] = 1; info[1] = best_sw; info[2] = best_cap; info[4] = np; info[5] = nw; info[6] = tinfo[2];
        info[7] = tinfo[3]; info[8] = tinfo[4]; info[11] = emax;
        info[15] = o_gpre; info[16] = o_gpre + G * m; info[17] = o_gpre + G * m + 4 * np;
        pos = o_gpre + G * m + 4 * np + 2 * nw;
        for (int64_t q = 0; q < 3 * tinfo[2]; ++q) passes[q] = pas[q];
        // 32-B piece records (fa_trie_records), 16-B aligned
        pos = (pos + 3) & ~(int64_t)3;
        if (!need(8 * np)) return 3;
        if (fa_trie_records(pieces, pieces + 4 * np, passes, tinfo[2], gpre, gext, m, (int)tinfo[3], buf + pos))
          return 5;
        info[20] = pos;
        pos += 8 * np;
        info[18] = pos;
        return 0;
      }
    }
  }

  // ---- slab kernel: pieces of <= 8 extensions, passes of <= cap, size-sorted per pass
  int64_t cap = 0;
  const int sw = slab_width(n_used, C, lds, &cap, accb, (double)fa_slab_map_lds(F1));
  if (sw == 0) return 4;
  std::vector<SlabPiece> pcs;
  pcs.reserve((size_t)pieces8);
  for (int64_t g = 0; g < G; ++g) {
    const int64_t a = ext_off[g] - ext_off[0], b = ext_off[g + 1] - ext_off[0];
    if (a == b) { pcs.push_back({g, a, a}); continue; }
    for (int64_t x = a; x < b; x += 8) pcs.push_back({g, x, std::min(b, x + 8)});
  }
  const int64_t NP = (int64_t)pcs.size();
  // passes: consecutive pieces while their extensions fit the accumulator; then the
  // slot order of each pass (slot s = step s / 1024 of thread s % 1024): size-sorted
  // pieces, or (class layout, see cls_layout) sibling runs with sharing flags
  const bool cls_ok = params[9] > 0 && uniform && m0 >= 2 && m0 <= 12;
  std::vector<int64_t> slot;        // piece index, -1 = idle slot
  std::vector<uint8_t> sflag;       // kRecKeepQ | kRecKeepP
  std::vector<int64_t> pass_rng;    // (piece begin, piece end, slot begin, slot end, ext base, class slot end)
  std::vector<int64_t> cslot;       // the class layout's slots and flags
  std::vector<uint8_t> cflag;
  int64_t cost_sorted = 0, cost_cls = 0;
  {
    int64_t i = 0;
    std::vector<int64_t> ord;
    std::vector<int64_t> cs;
    std::vector<uint8_t> cf;
    while (i < NP) {
      const int64_t base = pcs[i].lo;
      int64_t j = i;
      while (j < NP && pcs[j].hi - base <= cap) ++j;
      if (j == i) j = i + 1;   // a single piece always fits (<= 8 extensions)
      // stable order by extension count (8..0, descending): counting sort
      int64_t bucket[10] = {0};
      for (int64_t k = i; k < j; ++k) bucket[8 - (pcs[k].hi - pcs[k].lo) + 1] += 1;
      for (int b = 1; b < 10; ++b) bucket[b] += bucket[b - 1];
      ord.resize((size_t)(j - i));
      for (int64_t k = i; k < j; ++k) ord[bucket[8 - (pcs[k].hi - pcs[k].lo)]++] = k;
      std::vector<uint8_t> of(ord.size(), 0);
      const int64_t c_sorted = slot_cost(pcs, ord, of, m0);
      cost_sorted += c_sorted;
      const int64_t s0 = (int64_t)slot.size();
      slot.insert(slot.end(), ord.begin(), ord.end());
      sflag.insert(sflag.end(), of.begin(), of.end());
      if (cls_ok) {
        cls_layout(pcs, i, j, Pf, poff, m0, cs, cf);
        cost_cls += slot_cost(pcs, cs, cf, m0);
        cslot.insert(cslot.end(), cs.begin(), cs.end());
        cflag.insert(cflag.end(), cf.begin(), cf.end());
      }
      pass_rng.insert(pass_rng.end(), {i, j, s0, (int64_t)slot.size(), base, (int64_t)cslot.size()});
      i = j;
    }
  }
  // one layout for the whole level (one kernel per level): the class layout when its
  // wave-step reads are below kClsMinGain of the size-sorted layout's (params[9] = 2: always)
  if (cls_ok && (params[9] >= 2 || (double)cost_cls < kClsMinGain * (double)cost_sorted)) {
    slot.swap(cslot);
    sflag.swap(cflag);
    for (size_t q = 0; q < pass_rng.size(); q += 6) {
      pass_rng[q + 2] = q ? pass_rng[q - 1] : 0;
      pass_rng[q + 3] = pass_rng[q + 5];
    }
  }
  const int64_t npass = (int64_t)pass_rng.size() / 6;
  if (npass > max_pass) return 3;
  const int64_t NS = (int64_t)slot.size();
  int64_t pre_total = 0;
  for (int64_t s = 0; s < NS; ++s)
    if (slot[s] >= 0) pre_total += poff[pcs[slot[s]].g + 1] - poff[pcs[slot[s]].g];
  if (!need(pre_total + 4 * NS)) return 3;
  int32_t* gpre = buf + pos;
  int32_t* loc = gpre + pre_total;
  int32_t* gpm = loc + 2 * NS;
  info[15] = pos; info[16] = pos + pre_total; info[19] = pos + pre_total + 2 * NS;
  int64_t wpos = 0;
  for (int64_t q = 0; q < npass; ++q) {
    const int64_t base = pass_rng[6 * q + 4];
    for (int64_t s = pass_rng[6 * q + 2]; s < pass_rng[6 * q + 3]; ++s) {
      if (slot[s] < 0) {   // idle slot: no prefix, no extensions
        gpm[2 * s] = 0; gpm[2 * s + 1] = 0; loc[2 * s] = 0; loc[2 * s + 1] = 0;
        continue;
      }
      const SlabPiece& pc = pcs[slot[s]];
      const int64_t mg = poff[pc.g + 1] - poff[pc.g];
      gpm[2 * s] = (int32_t)wpos;
      gpm[2 * s + 1] = (int32_t)mg;
      for (int64_t t = 0; t < mg; ++t) gpre[wpos++] = item_map[Pf[poff[pc.g] + t]];
      loc[2 * s] = (int32_t)(pc.lo - base);
      loc[2 * s + 1] = (int32_t)(pc.hi - base);
    }
    passes[3 * q] = pass_rng[6 * q + 2]; passes[3 * q + 1] = pass_rng[6 * q + 3]; passes[3 * q + 2] = base;
  }
  info[0] = 0; info[1] = sw; info[2] = cap; info[4] = NS; info[6] = npass;
  info[18] = pos + pre_total + 4 * NS;
  info[21] = cost_sorted; info[22] = cost_cls;
  info[23] = std::any_of(sflag.begin(), sflag.end(), [](uint8_t f) { return f != 0; }) ? 1 : 0;
  // piece records for k_count_slab_rec: 48 B per piece (16-B aligned), so a piece's
  // whole description is three 16-B loads with no dependent index chain:
  //   a = {ext begin (pass-local), n_ext | m << 8 | (m > 12) << 16 | class flags << 17 | last prefix id << 19,
  //        prefix ids 0-3 (u16)}
  //   b = extension ids 0-7 (u16),  c = prefix ids 4-11 (u16), or c.x = gpre offset when m > 12
  {
    const int64_t rpos = (info[18] + 3) & ~(int64_t)3;
    if (rpos + 12 * NS > buf_cap) return 3;
    int32_t* rec = buf + rpos;
    const int32_t* gext_all = buf + info[14];
    auto pk = [](int32_t x, int32_t y) { return (uint32_t)(x & 0xFFFF) | ((uint32_t)(y & 0xFFFF) << 16); };
    for (int64_t q = 0; q < npass; ++q) {
      const int64_t base = passes[3 * q + 2];
      for (int64_t p = passes[3 * q]; p < passes[3 * q + 1]; ++p) {
        const int32_t lo = loc[2 * p], hi = loc[2 * p + 1];
        const int32_t mg = gpm[2 * p + 1];
        const int32_t* pre = gpre + gpm[2 * p];
        uint32_t* r = reinterpret_cast<uint32_t*>(rec + 12 * p);
        int32_t ids[12] = {0};
        for (int t = 0; t < std::min(mg, 12); ++t) ids[t] = pre[t];
        r[0] = (uint32_t)lo;
        // an idle slot keeps both partial ANDs and has no extensions: it reads nothing
        r[1] = (uint32_t)(hi - lo) | ((uint32_t)(slot[p] < 0 ? m0 : mg) << 8) | (mg > 12 ? 1u << 16 : 0u) |
               ((uint32_t)sflag[p] << 17) | (mg >= 1 && mg <= 12 ? (uint32_t)ids[mg - 1] << 19 : 0u);
        r[2] = pk(ids[0], ids[1]);
        r[3] = pk(ids[2], ids[3]);
        int32_t ex8[8] = {0};
        for (int32_t e = lo; e < hi; ++e) ex8[e - lo] = gext_all[base + e];
        for (int k = 0; k < 4; ++k) r[4 + k] = pk(ex8[2 * k], ex8[2 * k + 1]);
        for (int k = 0; k < 4; ++k) r[8 + k] = pk(ids[4 + 2 * k], ids[5 + 2 * k]);
        if (mg > 12) r[8] = (uint32_t)gpm[2 * p];
      }
    }
    info[20] = rpos;
    info[18] = rpos + 12 * NS;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Work plan of a level bundle for the depth-2 prefix-reuse kernel
// (k_count_slab<.., kDfs>; Python reference: ops.primitives.plan_bundle_dfs).
// Level j: groups g (prefix = row pi[j][g] of pv[j], m[j] items), candidates
// eo[j][g] .. eo[j][g+1] extending them by ex[j][c].  Level j+1's prefix rows are
// level j's candidates, so level j+1 group g' hangs under level-j candidate
// pi[j+1][g'].  Even levels are roots; the odd level after each is read as
// depth-2 nodes.  buf (int32) receives, at the offsets written to info:
//   item_map [F1] | used [n_used] | gpre | gpm [NP][2] | prng [NP][2] | node1 [N1][4] | node2 [N2][2]
// info: 0 n_used 1 NP 2 N1 3 N2 4 C 5..11 offsets of the seven arrays 12 total
// 13 accumulator passes (rows of passes, see below; one pass unless cap > 0 and L = 2).
// Returns 0, or 3 when buf or passes is too small.
// ---------------------------------------------------------------------------
FA_API int fa_plan_dfs(int L, const int32_t* const* pv, const int32_t* m, const int32_t* const* pi,
                       const int64_t* const* eo, const int32_t* const* ex, const int64_t* G, const int64_t* Cn,
                       int32_t F1, int piece_nodes, int32_t* buf, int64_t buf_cap, int64_t* info, int64_t cap,
                       int64_t* passes, int64_t max_pass) {
  for (int i = 0; i < 16; ++i) info[i] = 0;
  if (L <= 0) return 0;
  std::vector<int64_t> off(L + 1, 0);
  for (int j = 0; j < L; ++j) off[j + 1] = off[j] + Cn[j];
  int64_t NP = 0, N1 = 0, N2 = 0, npre = 0;
  for (int j = 0; j < L; j += 2) {
    for (int64_t g = 0; g < G[j]; ++g)
      NP += std::max<int64_t>(1, (eo[j][g + 1] - eo[j][g] + piece_nodes - 1) / piece_nodes);
    N1 += Cn[j];
    npre += G[j] * m[j];
    if (j + 1 < L) N2 += Cn[j + 1];
  }
  // + 8: node1 is read as int4 and node2 as int2 (count.hip), so their offsets are
  // rounded up to 4 and 2 int32
  const int64_t need = 2 * (int64_t)F1 + npre + 4 * NP + 4 * N1 + 2 * std::max<int64_t>(N2, 1) + 64 + 8;
  if (need > buf_cap) return 3;
  int64_t pos = 0;
  int32_t* item_map = buf + pos; info[5] = pos; pos += F1;
  int32_t* used = buf + pos; info[6] = pos;
  std::vector<uint8_t> mark((size_t)std::max(F1, 1), 0);
  for (int64_t g = 0; g < G[0]; ++g)
    for (int t = 0; t < m[0]; ++t) mark[pv[0][(int64_t)pi[0][g] * m[0] + t]] = 1;
  for (int64_t c = 0; c < Cn[0]; ++c) mark[ex[0][c]] = 1;
  int64_t n_used = 0;
  for (int32_t r = 0; r < F1; ++r) {
    if (mark[r]) { item_map[r] = (int32_t)n_used; used[n_used++] = r; } else item_map[r] = -1;
  }
  pos += n_used;
  int32_t* gpre = buf + pos; info[7] = pos; pos += npre;
  int32_t* gpm = buf + pos; info[8] = pos; pos += 2 * NP;
  int32_t* prng = buf + pos; info[9] = pos; pos += 2 * NP;
  pos = (pos + 3) & ~(int64_t)3;
  int32_t* node1 = buf + pos; info[10] = pos; pos += 4 * N1;
  pos = (pos + 1) & ~(int64_t)1;
  int32_t* node2 = buf + pos; info[11] = pos; pos += 2 * std::max<int64_t>(N2, 1);
  struct Piece { int32_t po, pl, b, e; int64_t cost; };
  std::vector<Piece> pcs;
  pcs.reserve((size_t)NP);
  int64_t gp = 0, n1 = 0, n2 = 0;
  std::vector<int64_t> n2b, n2e;
  for (int j = 0; j < L; j += 2) {
    const int mj = m[j];
    for (int64_t g = 0; g < G[j]; ++g)
      for (int t = 0; t < mj; ++t) gpre[gp + g * mj + t] = item_map[pv[j][(int64_t)pi[j][g] * mj + t]];
    n2b.assign((size_t)Cn[j], 0);
    n2e.assign((size_t)Cn[j], 0);
    if (j + 1 < L) {
      for (int64_t g = 0; g < G[j + 1]; ++g) {
        const int32_t c = pi[j + 1][g];
        n2b[c] = n2 + eo[j + 1][g];
        n2e[c] = n2 + eo[j + 1][g + 1];
      }
      for (int64_t c = 0; c < Cn[j + 1]; ++c) {
        node2[2 * (n2 + c)] = item_map[ex[j + 1][c]];
        node2[2 * (n2 + c) + 1] = (int32_t)(off[j + 1] + c);
      }
    }
    for (int64_t c = 0; c < Cn[j]; ++c) {
      int32_t* nd = node1 + 4 * (n1 + c);
      nd[0] = item_map[ex[j][c]];
      nd[1] = (int32_t)(off[j] + c);
      nd[2] = (int32_t)n2b[c];
      nd[3] = (int32_t)n2e[c];
    }
    for (int64_t g = 0; g < G[j]; ++g) {
      const int64_t a = eo[j][g], b = eo[j][g + 1];
      for (int64_t x = a; x < std::max(b, a + 1); x += piece_nodes) {
        const int64_t y = std::min(b, x + piece_nodes);
        int64_t cost = mj + (y - x);
        for (int64_t c = x; c < y; ++c) cost += n2e[c] - n2b[c];
        pcs.push_back({(int32_t)(gp + g * mj), (int32_t)mj, (int32_t)(n1 + x), (int32_t)(n1 + y), cost});
      }
    }
    gp += G[j] * mj;
    n1 += Cn[j];
    if (j + 1 < L) n2 += Cn[j + 1];
  }
  // accumulator passes (two levels, cap > 0): consecutive pieces while their level-k
  // nodes plus those nodes' children fit the LDS accumulator.  The nodes of a pass
  // are one contiguous candidate range [A0, A1) and their children one contiguous
  // range [B0, B1) (children follow their parents' order), so the pass counts into
  // acc[0, A1 - A0) and acc[A1 - A0, ..) and the launcher flushes the two ranges to
  // out[A0 ..] and out[C_k + B0 ..].  Output indices in node1 / node2 become
  // pass-local.  Each pass row: (piece begin, piece end, A0, nA, C_k + B0).
  int64_t npass = 0;
  const int64_t NPc = (int64_t)pcs.size();
  if (cap > 0 && L == 2) {
    std::vector<int64_t> chst((size_t)Cn[0] + 1, 0);      // children before node c
    for (int64_t c = 0; c < Cn[0]; ++c) chst[c + 1] = chst[c] + (node1[4 * c + 3] - node1[4 * c + 2]);
    int64_t p0 = 0;
    while (p0 < NPc) {
      const int64_t a0 = pcs[p0].b;
      int64_t p1 = p0;
      while (p1 < NPc) {
        const int64_t a1 = pcs[p1].e;
        if (p1 > p0 && (a1 - a0) + (chst[a1] - chst[a0]) > cap) break;
        ++p1;
      }
      if (npass >= max_pass) return 3;
      const int64_t a1 = pcs[p1 - 1].e, na = a1 - a0, b0 = chst[a0];
      for (int64_t c = a0; c < a1; ++c) node1[4 * c + 1] = (int32_t)(c - a0);
      for (int64_t j = chst[a0]; j < chst[a1]; ++j) node2[2 * j + 1] = (int32_t)(na + j - b0);
      int64_t* ps = passes + 5 * npass;
      ps[0] = p0; ps[1] = p1; ps[2] = a0; ps[3] = na; ps[4] = off[1] + b0;
      ++npass;
      p0 = p1;
    }
  } else {
    if (max_pass < 1) return 3;
    passes[0] = 0; passes[1] = NPc; passes[2] = 0; passes[3] = off[L]; passes[4] = off[L];
    npass = 1;
  }
  // cost-sorted pieces within each pass (the lanes of a wave then run loops of similar length)
  for (int64_t q = 0; q < npass; ++q)
    std::stable_sort(pcs.begin() + passes[5 * q], pcs.begin() + passes[5 * q + 1],
                     [](const Piece& x, const Piece& y) { return x.cost > y.cost; });
  for (size_t i = 0; i < pcs.size(); ++i) {
    gpm[2 * i] = pcs[i].po; gpm[2 * i + 1] = pcs[i].pl;
    prng[2 * i] = pcs[i].b; prng[2 * i + 1] = pcs[i].e;
  }
  info[0] = n_used; info[1] = (int64_t)pcs.size(); info[2] = N1; info[3] = N2; info[4] = off[L];
  info[12] = pos;
  info[13] = npass;
  return 0;
}
