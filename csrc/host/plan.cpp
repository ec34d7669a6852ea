// Level planner of the slab kernel (csrc/hip/count.hip k_count_slab_rec).
//
// Reference behaviour being scheduled: FastApriori.scala:132-160 counts every
// (prefix x, extensions ys) group by AND-ing x's bitmaps once and then each y.
// Here a group becomes pieces of <= 8 extensions; a piece is one 48-B record the
// kernel's thread reads once per slab.  Passes are consecutive pieces whose
// extensions fit the LDS accumulator; within a pass pieces are laid out by size
// (lanes of a wave then loop equally long) or, on deep levels, as sibling runs
// (the class layout: pieces sharing their first m-1 prefix items go to one thread
// in a row, which keeps that AND in registers).
#include <algorithm>
#include <cstring>
#include <vector>

#include "fa_common.h"

using namespace fa;

// ---------------------------------------------------------------------------
// One-call level planner: everything the level kernels need, computed in C++
// and written into one (pinned) int32 buffer so the driver issues a single
// host->device copy per level.
//
//   params (double[4]): lds_bytes, W (bitmap words), LDS bytes per accumulator (4),
//                       class layout of slab passes (0 off, 1 where it saves reads, 2 always)
//   info (int64[24]) out:
//     1 sw  2 cap  3 n_used  4 n_pieces  6 n_passes  10 slab reads
//     12 off item_map  13 off used  14 off gext  15 off gpre  16 off loc (piece ext ranges)
//     18 total int32 written  19 off gpm  20 off piece records
//     21 slab wave-step reads, size-sorted  22 the same, class layout (0: not tried)
//     23 class layout used by some pass (record flags set: k_count_slab_rec<.., kCls>)
//   passes (int64[3 * maxpass]): (piece begin, piece end, ext base)
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
  const double lds = params[0];
  const double accb = params[2] > 0 ? params[2] : 4;   // LDS bytes per accumulator
  const double cls_mode = params[3];
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
  // records carry the last prefix item's slab row in 13 bits (bits 19-31 of r[1])
  const bool cls_ok = cls_mode > 0 && uniform && m0 >= 2 && m0 <= 12 && n_used < 8192;
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
  // wave-step reads are below kClsMinGain of the size-sorted layout's (cls_mode 2: always)
  if (cls_ok && (cls_mode >= 2 || (double)cost_cls < kClsMinGain * (double)cost_sorted)) {
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
