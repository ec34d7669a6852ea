// CPU implementations of the mining primitives.
//
// These serve two roles: (1) the device path for CPU tensors, used by the
// gloo multi-process tests and the BASELINE "CPU world_size=1 plumbing"
// config; (2) an independent reference for the HIP kernels in csrc/hip/.
// Layout conventions are identical to the HIP side:
//   bitmaps  uint64 [F1][Wp], bit (c & 63) of word c >> 6 = column c;
//   wword    optional int32 per word: weight of every column in that word
//            (columns are grouped by dedup weight class, padded to 64);
//   counts   int64.
#include <atomic>

#include "fa_common.h"

using namespace fa;

FA_API void fa_cpu_histogram(const int32_t* items, int64_t nnz, int64_t V, int64_t* out,
                             int nthreads) {
  if (V <= 0) return;
  int nt = std::max(1, nthreads);
  if (V > (1 << 22) || nnz < (1 << 16)) nt = 1;
  std::vector<std::vector<int64_t>> loc(nt);
  parallel_for_threads(nt, [&](int t) {
    auto& h = loc[t];
    h.assign((size_t)V, 0);
    int64_t b = nnz * t / nt, e = nnz * (t + 1) / nt;
    for (int64_t i = b; i < e; ++i) h[items[i]]++;
  });
  for (int t = 0; t < nt; ++t)
    for (int64_t v = 0; v < V; ++v) out[v] += loc[t][v];
}

FA_API void fa_cpu_txn_freq_count(const int64_t* off, const int32_t* items, int64_t n,
                                  const int32_t* lut, int32_t* out, int nthreads) {
  parallel_for(n, nthreads, 1 << 14, [&](int64_t b, int64_t e, int) {
    for (int64_t t = b; t < e; ++t) {
      int32_t c = 0;
      for (int64_t i = off[t]; i < off[t + 1]; ++i) c += lut[items[i]] >= 0;
      out[t] = c;
    }
  });
}

// Compressed rows (FastApriori.scala:66-70): kept transaction x -> the ranks
// lut[id] >= 0 of its ids, ascending, at ranks[roff[x] ..].  Rows are short
// (insertion sort); rows are independent, so threads take row ranges.
FA_API void fa_cpu_compress(const int64_t* off, const int32_t* items, const int32_t* lut, const int32_t* kept,
                            int64_t T, const int64_t* roff, int32_t* ranks, int nthreads) {
  parallel_for(T, nthreads, 1 << 14, [&](int64_t b, int64_t e, int) {
    for (int64_t x = b; x < e; ++x) {
      const int64_t t = kept[x];
      int32_t* out = ranks + roff[x];
      int64_t n = 0;
      for (int64_t i = off[t]; i < off[t + 1]; ++i) {
        const int32_t r = lut[items[i]];
        if (r < 0) continue;
        int64_t j = n++;
        while (j > 0 && out[j - 1] > r) { out[j] = out[j - 1]; --j; }
        out[j] = r;
      }
    }
  });
}

// Column c holds compressed row src[c] (src == nullptr: identity; -1: padding).
// out must be zero-initialised, [F1][Wp].
FA_API void fa_cpu_build_bitmaps(const int64_t* roff, const int32_t* ranks, const int32_t* src,
                                 int64_t ncols, int64_t Wp, uint64_t* out, int nthreads) {
  const int64_t W = (ncols + 63) / 64;
  parallel_for(W, nthreads, 256, [&](int64_t wb, int64_t we, int) {
    for (int64_t c = wb * 64; c < std::min(ncols, we * 64); ++c) {
      int64_t row = src ? (int64_t)src[c] : c;
      if (row < 0) continue;
      const uint64_t bit = 1ull << (c & 63);
      const int64_t w = c >> 6;
      for (int64_t i = roff[row]; i < roff[row + 1]; ++i) out[(int64_t)ranks[i] * Wp + w] |= bit;
    }
  });
}

// Same hash as the device k_row_hash (csrc/hip/prep.hip).
FA_API void fa_cpu_row_hash(const int64_t* roff, const int32_t* ranks, int64_t T, int64_t* h1,
                            int64_t* h2, int nthreads) {
  parallel_for(T, nthreads, 1 << 14, [&](int64_t b, int64_t e, int) {
    for (int64_t x = b; x < e; ++x) {
      uint64_t a = 0x243F6A8885A308D3ull, c = 0x13198A2E03707344ull;
      for (int64_t i = roff[x]; i < roff[x + 1]; ++i) {
        uint64_t r = (uint32_t)ranks[i];
        a = mix64(a ^ r);
        c = mix64(c + r * 0xD6E8FEB86659FD93ull);
      }
      a = mix64(a ^ (uint64_t)(roff[x + 1] - roff[x]));
      h1[x] = (int64_t)(a >> 1);
      h2[x] = (int64_t)(c >> 1);
    }
  });
}

// Upper-triangular pair supports from bitmaps (out[i*F1+j], i<j).  out zeroed.
FA_API void fa_cpu_pair_gram(const uint64_t* bm, int32_t F1, int64_t Wp, int64_t W,
                             const int32_t* wword, int64_t* out, int nthreads) {
  parallel_for(F1, nthreads, 1, [&](int64_t i0, int64_t i1, int) {
    for (int64_t i = i0; i < i1; ++i) {
      const uint64_t* a = bm + i * Wp;
      for (int64_t j = i + 1; j < F1; ++j) {
        const uint64_t* b = bm + j * Wp;
        int64_t s = 0;
        if (wword) {
          for (int64_t w = 0; w < W; ++w) s += (int64_t)__builtin_popcountll(a[w] & b[w]) * wword[w];
        } else {
          for (int64_t w = 0; w < W; ++w) s += __builtin_popcountll(a[w] & b[w]);
        }
        out[i * F1 + j] = s;
      }
    }
  });
}

// Pair supports from compressed rows (sorted ranks): every pair (a < c) of a
// row gets +weight.  out zeroed, [F1][F1].
FA_API void fa_cpu_pair_horizontal(const int64_t* roff, const int32_t* ranks, int64_t T,
                                   const int32_t* wrow, int32_t F1, int64_t* out, int nthreads) {
  int nt = std::max(1, nthreads);
  if ((int64_t)F1 * F1 > (1 << 22) || T < 4096) nt = 1;
  std::vector<std::vector<int64_t>> loc(nt);
  parallel_for_threads(nt, [&](int tid) {
    int64_t* acc = out;
    if (nt > 1) { loc[tid].assign((size_t)F1 * F1, 0); acc = loc[tid].data(); }
    int64_t b = T * tid / nt, e = T * (tid + 1) / nt;
    for (int64_t x = b; x < e; ++x) {
      const int64_t w = wrow ? wrow[x] : 1;
      if (w == 0) continue;
      for (int64_t i = roff[x]; i < roff[x + 1]; ++i)
        for (int64_t j = i + 1; j < roff[x + 1]; ++j) acc[(int64_t)ranks[i] * F1 + ranks[j]] += w;
    }
  });
  if (nt > 1)
    for (int t = 0; t < nt; ++t)
      for (int64_t i = 0; i < (int64_t)F1 * F1; ++i) out[i] += loc[t][i];
}

// Prefix-shared candidate support (FastApriori.scala:132-160 semantics):
// group g = prefix ranks prefix[g][0..m) + extensions ext[ext_off[g]..ext_off[g+1]).
//
// Tiled like the GPU slab kernel: the columns are cut into tiles of kTileWords
// words (2 KB of every item row), a thread takes a tile and runs EVERY group over
// it -- the prefix AND once per group (the reference's commonArray), then each
// extension's AND + popcount -- so a level streams each used item row from DRAM
// once per tile instead of once per group, and the group loop reads L1/L2-resident
// tiles.  A group whose prefix AND is empty on a tile skips its extensions there.
// Each thread accumulates into its own count vector; the vectors are summed last.
FA_API void fa_cpu_count_candidates(const uint64_t* bm, int64_t Wp, int64_t W,
                                    const int32_t* prefix, int32_t m, const int64_t* ext_off,
                                    const int32_t* ext, int64_t G, const int32_t* wword,
                                    int64_t* out, int nthreads) {
  constexpr int64_t kTileWords = 256;
  const int64_t e_base = ext_off[0];
  const int64_t C = ext_off[G] - e_base;
  if (C <= 0 || W <= 0) {
    for (int64_t e = 0; e < C; ++e) out[e] = 0;
    return;
  }
  const int64_t ntile = (W + kTileWords - 1) / kTileWords;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, ntile));
  std::vector<std::vector<int64_t>> loc((size_t)nt);
  std::atomic<int64_t> next{0};
  parallel_for_threads(nt, [&](int tid) {
    auto& acc = loc[(size_t)tid];
    acc.assign((size_t)C, 0);
    uint64_t common[kTileWords];
    for (;;) {
      const int64_t t = next.fetch_add(1);
      if (t >= ntile) break;
      const int64_t w0 = t * kTileWords, nw = std::min(kTileWords, W - w0);
      for (int64_t g = 0; g < G; ++g) {
        const int32_t* p = prefix + g * m;
        const uint64_t* r0 = bm + (int64_t)p[0] * Wp + w0;
        for (int64_t w = 0; w < nw; ++w) common[w] = r0[w];
        for (int q = 1; q < m; ++q) {
          const uint64_t* rq = bm + (int64_t)p[q] * Wp + w0;
          for (int64_t w = 0; w < nw; ++w) common[w] &= rq[w];
        }
        uint64_t any = 0;
        for (int64_t w = 0; w < nw; ++w) any |= common[w];
        if (!any) continue;
        for (int64_t e = ext_off[g]; e < ext_off[g + 1]; ++e) {
          const uint64_t* re = bm + (int64_t)ext[e] * Wp + w0;
          int64_t s = 0;
          if (wword) {
            for (int64_t w = 0; w < nw; ++w) s += (int64_t)__builtin_popcountll(common[w] & re[w]) * wword[w0 + w];
          } else {
            for (int64_t w = 0; w < nw; ++w) s += __builtin_popcountll(common[w] & re[w]);
          }
          acc[(size_t)(e - e_base)] += s;
        }
      }
    }
  });
  for (int64_t e = 0; e < C; ++e) {
    int64_t s = 0;
    for (int t = 0; t < nt; ++t) s += loc[(size_t)t][(size_t)e];
    out[e] = s;
  }
}

// Open-addressing probe table for the heavy-hitter F1 exact pass
// (csrc/hip/prep.hip k_f1_exact): keys[S] = -1 or a candidate id, linear
// probing from the multiplicative hash (id * a) >> (32 - log_s).  slot[i]
// receives the position of ids[i].
FA_API void fa_build_probe_table(const int64_t* ids, int64_t n, int log_s, uint32_t a, int32_t* keys,
                                 int64_t* slot) {
  const uint32_t S = 1u << log_s;
  for (uint32_t i = 0; i < S; ++i) keys[i] = -1;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t h = ((uint32_t)ids[i] * a) >> (32 - log_s);
    while (keys[h] != -1 && keys[h] != (int32_t)ids[i]) h = (h + 1) & (S - 1);
    keys[h] = (int32_t)ids[i];
    slot[i] = h;
  }
}
