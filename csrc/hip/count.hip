// Support-counting kernels for k = 2 and k >= 3.
//
// Reference sites: FastApriori.scala:212-241 (genTwoFreqItems: all F1(F1-1)/2
// pairs, AND of two byte-per-transaction arrays + weighted sum) and
// :132-160 (genNextFreqItemsets: prefix AND once per group, then AND + sum per
// extension).  Here:
//   * k_pair_queue16 / k_pair_blocked : sparse data — rows re-laid out per rank
//     block; every tile of the pair matrix is counted in LDS (packed u16 / u32)
//     from its two blocks' segments, one global atomic per non-zero entry.
//   * k_pair_gram_mfma4  : dense data — bit-matrix Gram B^T B on the int8 matrix
//     cores (per weight class with a scale); k_pair_gram_popc the v_bcnt form
//     for short weight classes.
//   * k_count_candidates : k >= 3 — prefix-shared AND + popcount per group of
//     candidates over a super-chunk of bitmap words; wave reductions into an
//     LDS accumulator, one coalesced global atomic per candidate per chunk.
// All accumulation is integer, so results are exact and order-independent.
#include <algorithm>
#include <cstdlib>

#include "fa_hip.h"

namespace fa {

// ---------------------------------------------------------------------------
// k = 2, horizontal
// ---------------------------------------------------------------------------
constexpr int kPB = 128;

__device__ __forceinline__ void tri_index(int pid, int nb, int& bi, int& bj) {
  bi = 0;
  int rem = pid;
  while (rem >= nb - bi) { rem -= nb - bi; ++bi; }
  bj = bi + rem;
}

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* __restrict__ a, int64_t lo, int64_t hi,
                                                   int32_t key) {
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Each workgroup owns one 128x128 tile (bi, bj) of the pair matrix (u32 in LDS)
// and a chunk of rows.  Its 8 wavefronts run fully decoupled: each takes
// 64-row batches of the chunk, stages the batch's sorted ranks into a
// wave-private LDS span (u16), and every lane scans its row for the bi / bj
// segments and scatters the pairs into the shared tile with ds_add_u32.  There
// is no workgroup barrier in the main loop; global-load latency is hidden by a
// two-deep register pipeline (row offsets two batches ahead, ranks one ahead)
// and by the 16 resident waves per CU.  The logical block id is XCD-remapped so
// the nbp tiles of one chunk run on one XCD and re-read the chunk from its L2.
constexpr int kPW = 16;                // waves per workgroup (1024 threads)
constexpr int kWSpan = 1024;           // ranks staged per wave batch
constexpr int kWPer = kWSpan / 64;     // per lane

__device__ __forceinline__ void wave_lds_fence() { wave_lds_sync(); }

// ---------------------------------------------------------------------------
// k = 2, blocked layout.  Rows are re-laid out per 128-rank block:
//   cnt[b][x]   u8   number of ranks of row x in block b
//   base[b][q]  i64  where block b's data of 64-row batch q starts in lr
//   lr[...]     u8   local ranks (rank - 128*b), block-major, batch-major, row order
// A tile (bi, bj) then reads two bytes per row and only its two blocks' segments.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
  (void)lane;
  return wave_scan_incl_dpp(v);
}

// one wave per 64-row batch; lane = row
__global__ __launch_bounds__(256) void k_block_counts(const int64_t* __restrict__ roff,
                                                      const int32_t* __restrict__ ranks, int64_t T, int nb,
                                                      uint8_t* __restrict__ cnt, int64_t* __restrict__ bsum,
                                                      int64_t nbatch, int pb) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nbatch) return;
  const int lane = threadIdx.x & 63;
  const int64_t x = q * 64 + lane;
  const bool valid = x < T;
  int64_t i = valid ? roff[x] : 0;
  const int64_t e = valid ? roff[x + 1] : 0;
  for (int b = 0; b < nb; ++b) {
    const int edge = (b + 1) * pb;
    int c = 0;
    while (i < e && ranks[i] < edge) { ++i; ++c; }
    if (valid) cnt[(int64_t)b * T + x] = (uint8_t)c;
    int tot = c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if (lane == 0) bsum[(int64_t)b * nbatch + q] = tot;
  }
}

__global__ __launch_bounds__(256) void k_block_scatter(const int64_t* __restrict__ roff,
                                                       const int32_t* __restrict__ ranks, int64_t T, int nb,
                                                       const uint8_t* __restrict__ cnt,
                                                       const int64_t* __restrict__ base, int64_t nbatch,
                                                       uint8_t* __restrict__ lr, int pb) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nbatch) return;
  const int lane = threadIdx.x & 63;
  const int64_t x = q * 64 + lane;
  const bool valid = x < T;
  int64_t i = valid ? roff[x] : 0;
  for (int b = 0; b < nb; ++b) {
    const int c = valid ? cnt[(int64_t)b * T + x] : 0;
    const int incl = wave_incl_scan(c, lane);
    int64_t o = base[(int64_t)b * nbatch + q] + (incl - c);
    for (int k = 0; k < c; ++k) lr[o + k] = (uint8_t)(ranks[i + k] - b * pb);
    i += c;
  }
}

// Wave-cooperative versions (nb <= kWBMaxNB): a wave owns batch q (64 rows =
// lanes) and streams the rows' contiguous ranks 64 at a time, coalesced.
//   counts : row l's block-b count = sum over windows of popc(ballot(block == b)
//            & the window lanes inside row l);
//   scatter: row owners put (block base + rows-before prefix - row start -
//            earlier-block items of the row) per block in an LDS table; a rank
//            at position p of row r in block b goes to table[r][b] + p (ranks
//            are sorted, so a row's block-b items are contiguous).
// Rows are non-empty (compress keeps rows with >= 2 frequent items).
constexpr int kWBMaxNB = 8;

struct BatchSpan {
  int64_t base;
  int n, srel, erel;
};

__device__ __forceinline__ BatchSpan batch_span(const int64_t* __restrict__ roff, int64_t x0, int64_t T) {
  const int lane = threadIdx.x & 63;
  BatchSpan b;
  b.base = roff[x0];
  b.n = (int)(roff[min(x0 + 64, T)] - b.base);
  b.srel = (int)(roff[min(x0 + lane, T)] - b.base);
  b.erel = (int)(roff[min(x0 + lane + 1, T)] - b.base);
  return b;
}

__device__ __forceinline__ unsigned long long lane_span(int lo, int hi) {   // bits [lo, hi) clamped to [0, 64]
  lo = max(lo, 0); hi = min(hi, 64);
  if (hi <= lo) return 0ull;
  const unsigned long long h = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
  return h & ~((1ull << lo) - 1);
}

__global__ __launch_bounds__(256) void k_block_counts_w(const int64_t* __restrict__ roff,
                                                        const int32_t* __restrict__ ranks, int64_t T, int nb,
                                                        uint8_t* __restrict__ cnt, int64_t* __restrict__ bsum,
                                                        int64_t nbatch, int lpb) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nbatch) return;
  const int lane = threadIdx.x & 63;
  const int64_t x = q * 64 + lane;
  const BatchSpan bs = batch_span(roff, q * 64, T);
  int c[kWBMaxNB];
#pragma unroll
  for (int b = 0; b < kWBMaxNB; ++b) c[b] = 0;
  constexpr int U = 4;
  for (int p0 = 0; p0 < bs.n; p0 += 64 * U) {
    int r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + 64 * u + lane;
      r[u] = p < bs.n ? ranks[bs.base + p] >> lpb : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q0 = p0 + 64 * u;
      const unsigned long long rm = lane_span(bs.srel - q0, bs.erel - q0);
#pragma unroll
      for (int b = 0; b < kWBMaxNB; ++b)
        if (b < nb) c[b] += __popcll(__ballot(r[u] == b) & rm);
    }
  }
#pragma unroll
  for (int b = 0; b < kWBMaxNB; ++b) {
    if (b >= nb) break;
    if (x < T) cnt[(int64_t)b * T + x] = (uint8_t)c[b];
    const int tot = wave_last(wave_scan_incl_dpp(x < T ? c[b] : 0));
    if (lane == 0) bsum[(int64_t)b * nbatch + q] = tot;
  }
}

__global__ __launch_bounds__(256) void k_block_scatter_w(const int64_t* __restrict__ roff,
                                                         const int32_t* __restrict__ ranks, int64_t T, int nb,
                                                         const uint8_t* __restrict__ cnt,
                                                         const int64_t* __restrict__ base, int64_t nbatch,
                                                         uint8_t* __restrict__ lr, int lpb) {
  __shared__ int64_t offt[4][64 * kWBMaxNB];
  __shared__ unsigned long long swords[4][4];
  const int wv = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 4 + wv;
  if (q >= nbatch) return;
  const int lane = threadIdx.x & 63;
  const int64_t x = q * 64 + lane;
  const BatchSpan bs = batch_span(roff, q * 64, T);
  int before = 0;
#pragma unroll
  for (int b = 0; b < kWBMaxNB; ++b) {
    if (b >= nb) break;
    const int c = x < T ? cnt[(int64_t)b * T + x] : 0;
    const int pre = wave_scan_incl_dpp(c) - c;
    offt[wv][lane * kWBMaxNB + b] = base[(int64_t)b * nbatch + q] + pre - bs.srel - before;
    before += c;
  }
  const unsigned long long le = lanes_le_mask();
  constexpr int U = 4;
  for (int p0 = 0; p0 < bs.n; p0 += 64 * U) {
    int r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + 64 * u + lane;
      r[u] = p < bs.n ? ranks[bs.base + p] : -1;
    }
    const int cs0 = __popcll(__ballot(x < T && bs.srel < p0));
    unsigned long long S[U];
    window_starts<U>(swords[wv], x < T ? bs.srel : -(1 << 30), p0, S);   // (also orders the offt writes)
    int cs = cs0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = cs + __popcll(S[u] & le) - 1;
      cs += __popcll(S[u]);
      if (r[u] >= 0) {
        const int b = r[u] >> lpb;
        lr[offt[wv][(row & 63) * kWBMaxNB + b] + p0 + 64 * u + lane] = (uint8_t)(r[u] - (b << lpb));
      }
    }
  }
}

constexpr int kBSpan = 1024;   // staged bytes per block segment per wave batch

__global__ __launch_bounds__(1024) void k_pair_blocked(
    const uint8_t* __restrict__ cnt, const int64_t* __restrict__ base, const uint8_t* __restrict__ lr,
    int64_t T, int64_t nbatch, const int32_t* __restrict__ wrow, int32_t F1, int nb, int nbp, int64_t chunk_b,
    uint32_t* __restrict__ out) {
  __shared__ uint32_t tile[kPB * kPB];
  __shared__ uint8_t wsi[kPW][kBSpan];
  __shared__ uint8_t wsj[kPW][kBSpan];
  __shared__ int32_t wmeta[kPW][4][64];   // pair prefix, i-start, j-start, nj | weight<<8 (weight < 2^23) ...
  const uint32_t logical = xcd_remap(blockIdx.x, gridDim.x);
  const int pid = logical % nbp;
  const int64_t ch = logical / nbp;
  int bi, bj;
  tri_index(pid, nb, bi, bj);
  const int rb0 = bi * kPB, cb0 = bj * kPB;
  const bool diag = bi == bj;
  for (int i = threadIdx.x; i < kPB * kPB; i += blockDim.x) tile[i] = 0;
  __syncthreads();
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* si = wsi[wv];
  uint8_t* sj = diag ? wsi[wv] : wsj[wv];
  int32_t* mpre = wmeta[wv][0];
  int32_t* mist = wmeta[wv][1];
  int32_t* mjst = wmeta[wv][2];
  int32_t* mnw = wmeta[wv][3];
  const int64_t q0 = ch * chunk_b, q1 = min(nbatch, q0 + chunk_b);
  const uint8_t* ci_row = cnt + (int64_t)bi * T;
  const uint8_t* cj_row = cnt + (int64_t)bj * T;
  // pipeline: counts of the next batch are loaded while this one scatters
  auto load = [&](int64_t q, int& ci, int& cj, uint32_t& w) {
    const int64_t x = q * 64 + lane;
    const bool valid = x < T;
    ci = valid ? ci_row[x] : 0;
    cj = diag ? ci : (valid ? cj_row[x] : 0);
    w = valid ? (wrow ? (uint32_t)wrow[x] : 1u) : 0u;
  };
  int ci = 0, cj = 0, ci_n = 0, cj_n = 0;
  uint32_t w = 0, w_n = 0;
  int64_t q = q0 + wv;
  if (q < q1) load(q, ci, cj, w);
  for (; q < q1; q += kPW) {
    if (q + kPW < q1) load(q + kPW, ci_n, cj_n, w_n);
    const int ni = w ? ci : 0, nj = w ? cj : 0;
    const int P = (ni > 0 && nj > 0) ? ni * nj : 0;
    const int incl = wave_incl_scan(P, lane);
    const int total = wave_last(incl);
    if (total > 0) {
      const int inci = wave_incl_scan(ci, lane);
      const int incj = diag ? inci : wave_incl_scan(cj, lane);
      const int tot_i = wave_last(inci), tot_j = wave_last(incj);
      const int64_t bsi = base[(int64_t)bi * nbatch + q];
      const int64_t bsj = base[(int64_t)bj * nbatch + q];
      const bool staged = tot_i <= kBSpan && tot_j <= kBSpan;
      if (staged) {
        for (int k = lane; k < tot_i; k += 64) si[k] = lr[bsi + k];
        if (!diag)
          for (int k = lane; k < tot_j; k += 64) sj[k] = lr[bsj + k];
      }
      mpre[lane] = incl - P;
      mist[lane] = inci - ci;
      mjst[lane] = incj - cj;
      mnw[lane] = nj;
      wave_lds_fence();
      auto scatter = [&](const uint8_t* __restrict__ A, const uint8_t* __restrict__ B) {
        for (int f = lane; f < total; f += 64) {
          int owner = 0;
#pragma unroll
          for (int step = 32; step > 0; step >>= 1)
            if (mpre[owner + step] <= f) owner += step;
          const int loc = f - mpre[owner];
          const int cols = mnw[owner];
          const int ii = (int)(((float)loc + 0.5f) * __builtin_amdgcn_rcpf((float)cols));
          const int jj = loc - ii * cols;
          if (diag && jj <= ii) continue;
          const int ra = A[mist[owner] + ii];
          const int rb = B[mjst[owner] + jj];
          const uint32_t wt = wrow ? (uint32_t)wrow[q * 64 + owner] : 1u;
          atomicAdd(&tile[ra * kPB + rb], wt);
        }
      };
      if (staged) scatter(si, sj);
      else scatter(lr + bsi, lr + bsj);
      wave_lds_fence();
    }
    ci = ci_n; cj = cj_n; w = w_n;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kPB * kPB; i += blockDim.x) {
    const uint32_t v = tile[i];
    if (!v) continue;
    const int r = rb0 + i / kPB, c = cb0 + i % kPB;
    if (r < F1 && c < F1) atomicAdd(&out[(int64_t)r * F1 + c], v);
  }
}

// 256x256 tile of packed 16-bit counters (128 KB of LDS, 10 tiles for F1 <= 1024
// instead of 36): two counters per u32 word, incremented with ds_add_u32 of
// 1 or 1<<16.  A workgroup's chunk is <= 65535 unit-weight rows, so no counter
// can carry into its neighbour before the flush.
constexpr int kPB16 = 256;

// ---------------------------------------------------------------------------
// k = 2, unit-weight rows: one lane per (row, item-in-block-bi) position.
//
// Blocked layout with 256-rank blocks and a 256x256 packed-u16 LDS tile.  Instead
// of flattening pairs by a dependent LDS binary search per pair,
// a lane takes one position p of the batch's block-bi local ranks and loops
// over its row's block-bj ranks.  The batch's local-rank bytes are staged in
// per-wave LDS (coalesced loads); the row of position p comes from the
// row-start mask of the window (window_starts over non-empty rows) and a
// compaction table of the non-empty rows, so the dependency chain per pair is
// one LDS byte read and one LDS atomic.
// ---------------------------------------------------------------------------
constexpr int kRowsDw = 2;                  // staged dwords per lane and block
constexpr int kRowsStage = 64 * kRowsDw * 4; // 512 staged local-rank bytes per wave and block
constexpr int kRowsWin = kRowsStage / 64;    // 8 windows

// Batches [q0, q1) of tile (bi, bj) into the packed-u16 LDS tile (no barriers).
constexpr int kTriTab = 64 * 63 / 2;

struct PairRowsLds {
  uint32_t tile[kPB16 * kPB16 / 2];
  uint32_t sa[kPW][kRowsStage / 4];
  uint32_t sb[kPW][kRowsStage / 4];
  uint8_t rowtab[kPW][64];
  unsigned long long swd[kPW][kRowsWin];
  int2 rowinfo[kPW][64];   // flattened pairs: (pair start, A start | B start << 10 | ci << 20) per row with pairs
  uint16_t tri[kTriTab];   // diagonal flat decode: t = j (j - 1) / 2 + i -> i | j << 8 (rows of <= 64 items)
};

// kDiag (bi == bj) is a template parameter: a runtime select between the two
// count loads made the compiler wait for the prefetched load right after issue.
//
// Software pipeline with two register sets X / Y (the loop is unrolled twice, so
// nothing is copied between iterations: a copy of a register that a load is
// still filling would wait for it).  Per batch: "meta" = the rows' block counts
// and the two segment bases, issued two batches ahead; "bytes" = the segments'
// aligned dwords (addresses from meta), issued one batch ahead.  Every load is
// unconditional -- cnt, base and lr are padded past their ends by the launcher
// (batches past the chunk read real or padding data that is never processed) --
// so the compiler's wait counts are exact and a wait never drains the loads
// issued for later batches.
struct PairBatch {
  int ci, cj;            // this lane's row: items in block bi / bj
  int64_t vb;            // lane 0: segment base in block bi, lane 1: in block bj
  uint32_t da[kRowsDw], db[kRowsDw];
};

template <bool kDiag>
__device__ __forceinline__ void pair_rows16_chunk_t(PairRowsLds& L, const uint8_t* __restrict__ cnt,
                                                    const int64_t* __restrict__ base,
                                                    const uint8_t* __restrict__ lr, int64_t T, int64_t nbatch,
                                                    int bi, int bj, int64_t q0, int64_t q1) {
  uint32_t* tile = L.tile;
  auto& sa = L.sa;
  auto& sb = L.sb;
  auto& rowtab = L.rowtab;
  auto& swd = L.swd;
  constexpr bool diag = kDiag;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned long long le = lanes_le_mask(), lt = le >> 1;
  const uint8_t* ci_row = cnt + (int64_t)bi * T;
  const uint8_t* cj_row = cnt + (int64_t)bj * T;
  const int64_t bsel = (lane & 1) ? (int64_t)bj * nbatch : (int64_t)bi * nbatch;
  auto load_meta = [&](PairBatch& B, int64_t qq) {
    const int64_t x = qq * 64 + lane;
    B.ci = ci_row[x];
    if (!kDiag) B.cj = cj_row[x];
    B.vb = base[bsel + qq];            // lane-varying address: a vector load
  };
  auto load_bytes = [&](PairBatch& B) {
    const int64_t oa = (int64_t)__builtin_amdgcn_readlane((int)B.vb, 0) |
                       ((int64_t)__builtin_amdgcn_readlane((int)(B.vb >> 32), 0) << 32);
    const uint32_t* pa = reinterpret_cast<const uint32_t*>(lr + (oa & ~(int64_t)3));
#pragma unroll
    for (int k = 0; k < kRowsDw; ++k) B.da[k] = pa[lane + 64 * k];   // lr is padded by >= 1 KiB
    if (!kDiag) {
      const int64_t ob = (int64_t)__builtin_amdgcn_readlane((int)B.vb, 1) |
                         ((int64_t)__builtin_amdgcn_readlane((int)(B.vb >> 32), 1) << 32);
      const uint32_t* pb = reinterpret_cast<const uint32_t*>(lr + (ob & ~(int64_t)3));
#pragma unroll
      for (int k = 0; k < kRowsDw; ++k) B.db[k] = pb[lane + 64 * k];
    }
  };
  auto process = [&](PairBatch& X, int64_t qq) {
    const int ci = (qq * 64 + lane < T) ? X.ci : 0;
    const int cj = diag ? ci : ((qq * 64 + lane < T) ? X.cj : 0);
    const int64_t oa = (int64_t)__builtin_amdgcn_readlane((int)X.vb, 0) |
                       ((int64_t)__builtin_amdgcn_readlane((int)(X.vb >> 32), 0) << 32);
    const int64_t ob = diag ? oa : ((int64_t)__builtin_amdgcn_readlane((int)X.vb, 1) |
                                    ((int64_t)__builtin_amdgcn_readlane((int)(X.vb >> 32), 1) << 32));
    const int inci = wave_scan_incl_dpp(ci);
    const int incj = diag ? inci : wave_scan_incl_dpp(cj);
    const int SA = wave_last(inci);
    const int SB = diag ? SA : wave_last(incj);
    const bool has = diag ? ci >= 2 : (ci > 0 && cj > 0);
    if (__ballot(has) == 0ull) return;
    const int sha = (int)(oa & 3), shb = (int)(ob & 3);
    const bool stA = SA + sha <= kRowsStage, stB = diag || SB + shb <= kRowsStage;
#pragma unroll
    for (int k = 0; k < kRowsDw; ++k) {
      sa[wv][lane + 64 * k] = X.da[k];
      if (!diag) sb[wv][lane + 64 * k] = X.db[k];
    }
    // flattened pairs (staged batches): one lane per (row, pair) instead of per
    // (row, position) -- see the flat branch below; rowtab then lists the rows with pairs
    const bool flat = stA && stB;
    const int npr = diag ? ci * (ci - 1) / 2 : ci * cj;
    const bool own = flat ? npr > 0 : ci > 0;
    const unsigned long long M = __ballot(own);
    const int incp = flat ? wave_scan_incl_dpp(npr) : 0;
    if (own) {
      if (flat) {
        const int a0 = inci - ci, b0 = diag ? a0 : incj - cj;
        L.rowinfo[wv][__popcll(M & lt)] = make_int2(incp - npr, a0 | (b0 << 10) | (ci << 20));
      } else {
        rowtab[wv][__popcll(M & lt)] = (uint8_t)lane;
      }
    }
    wave_lds_sync();
    if (flat) {
      // Pair t of row r (t < npr) is enumerated with the row's item in block bi
      // varying fastest, so consecutive lanes hit different tile rows (bank
      // swizzle of pair_tile16_word):
      //   off-diagonal: t = j * ci + i (i < ci, j < cj);  diagonal: t = j (j - 1) / 2 + i
      //   (i < j < ci), decoded with a float square root and a +-1 fix-up.
      // The owner row of flat index f comes from the row-start masks of its 64-wide
      // window, as the positions do in run_windows.
      const int NP = wave_last(incp);
      const int pst = incp - npr;
      const uint8_t* As = reinterpret_cast<const uint8_t*>(sa[wv]) + sha;
      const uint8_t* Bs = diag ? As : reinterpret_cast<const uint8_t*>(sb[wv]) + shb;
      const int srel = npr > 0 ? pst : -(1 << 30);
      int cs = 0;
      for (int f0 = 0; f0 < NP; f0 += 256) {
        unsigned long long S[4];
        window_starts<4>(swd[wv], srel, f0, S);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int fb = f0 + 64 * w;
          if (fb >= NP) break;
          const int kk = cs + __popcll(S[w] & le) - 1;
          cs += __popcll(S[w]);
          const int2 ri = L.rowinfo[wv][kk & 63];
          const int p_st = ri.x, px = ri.y;
          const int f = fb + lane;
          const int t = f - p_st;
          const int c = (px >> 20) & 0xFF;
          int i, j;
          if (diag) {
            // the triangular index does not depend on the row: a table (rows of <= 64
            // items) instead of a quarter-rate square root and its fix-ups
            if (c <= 64) {
              const int e = L.tri[t < kTriTab ? t : 0];
              i = e & 0xFF;
              j = e >> 8;
            } else {
              j = (int)((1.0f + __builtin_sqrtf(8.0f * (float)t + 1.0f)) * 0.5f);
              if (j * (j - 1) / 2 > t) --j;
              else if (j * (j + 1) / 2 <= t) ++j;
              i = t - j * (j - 1) / 2;
            }
          } else {
            j = (int)(((float)t + 0.5f) * __builtin_amdgcn_rcpf((float)c));
            i = t - j * c;
          }
          if (f < NP) {
            const int a = (int)As[(px & 0x3FF) + i];
            const int b = (int)Bs[((px >> 10) & 0x3FF) + j];
            atomicAdd(&tile[a * (kPB16 / 2) + ((b >> 1) ^ (a & 31))], (b & 1) ? 0x10000u : 1u);
          }
        }
      }
      wave_lds_sync();
      return;
    }
    const int jbeg = diag ? 0 : incj - cj;          // row owner view: my row's block-bj span
    const int jend = diag ? inci : incj;
    const int srow = ci > 0 ? inci - ci : -(1 << 30);
    // A and B are either both LDS stages or both global: each call site then has
    // one address space, so the byte reads are ds_read_u8 / global_load_ubyte
    // (a pointer that may be either compiles to flat loads, whose waits also
    // drain the prefetched global loads)
    auto run_windows = [&](const uint8_t* __restrict__ A, const uint8_t* __restrict__ B) {
      auto scatter = [&](int p0, unsigned long long Sw, int& cs) {
        const int k = cs + __popcll(Sw & le) - 1;
        cs += __popcll(Sw);
        const int row = rowtab[wv][k & 63];
        const int p = p0 + lane;
        int j0 = __shfl(jbeg, row, 64);
        const int j1 = __shfl(jend, row, 64);
        if (diag) j0 = p + 1;
        if (p < SA) {
          // word of (a, b) = a * 128 + ((b >> 1) ^ (a & 31)): the bank (word mod 32)
          // depends on a as well as b, so the lanes of one row (different a, same b
          // in the off-diagonal tiles) hit different banks (pair_tile16_word)
          const int a = (int)A[p];
          const int rowb = a * (kPB16 / 2), xa = a & 31;
          for (int j = j0; j < j1; ++j) {
            const int b = (int)B[j];
            atomicAdd(&tile[rowb + ((b >> 1) ^ xa)], (b & 1) ? 0x10000u : 1u);
          }
        }
      };
      int cs = 0;                                    // non-empty rows started before the window
      if (SA <= kRowsStage) {
        // row-start masks, 4 windows per LDS round trip
#pragma unroll
        for (int w0 = 0; w0 < kRowsWin; w0 += 4) {
          if (64 * w0 >= SA) break;
          unsigned long long S[4];
          window_starts<4>(swd[wv], srow, 64 * w0, S);
#pragma unroll
          for (int w = 0; w < 4; ++w)
            if (64 * (w0 + w) < SA) scatter(64 * (w0 + w), S[w], cs);
        }
      } else {
        for (int p0 = 0; p0 < SA; p0 += 64) {
          unsigned long long S[1];
          window_starts<1>(swd[wv], srow, p0, S);
          scatter(p0, S[0], cs);
        }
      }
    };
    if (stA && stB) {
      const uint8_t* As = reinterpret_cast<const uint8_t*>(sa[wv]) + sha;
      run_windows(As, diag ? As : reinterpret_cast<const uint8_t*>(sb[wv]) + shb);
    } else {
      run_windows(lr + oa, diag ? lr + oa : lr + ob);
    }
    wave_lds_sync();
  };
  // batch t lives in set t % 3: its meta is issued two batches before its bytes'
  // turn, its bytes one batch before it is processed
  int64_t q = q0 + wv;
  if (q >= q1) return;
  PairBatch X, Y, Z;
  load_meta(X, q);
  load_meta(Y, q + kPW);
  load_meta(Z, q + 2 * kPW);
  load_bytes(X);
  for (;;) {
    load_bytes(Y);
    process(X, q);
    load_meta(X, q + 3 * kPW);
    if ((q += kPW) >= q1) break;
    load_bytes(Z);
    process(Y, q);
    load_meta(Y, q + 3 * kPW);
    if ((q += kPW) >= q1) break;
    load_bytes(X);
    process(Z, q);
    load_meta(Z, q + 3 * kPW);
    if ((q += kPW) >= q1) break;
  }
}

__device__ __forceinline__ void pair_rows16_chunk(PairRowsLds& L, const uint8_t* __restrict__ cnt,
                                                  const int64_t* __restrict__ base,
                                                  const uint8_t* __restrict__ lr, int64_t T, int64_t nbatch,
                                                  int bi, int bj, int64_t q0, int64_t q1) {
  if (bi == bj) pair_rows16_chunk_t<true>(L, cnt, base, lr, T, nbatch, bi, bj, q0, q1);
  else pair_rows16_chunk_t<false>(L, cnt, base, lr, T, nbatch, bi, bj, q0, q1);
}

// Packed-u16 tile -> global counts.  With an even row stride (ld) the two
// counters of a word go out as one 64-bit atomic (two adjacent u32 counts; a
// u32 count never carries: it is bounded by the rows of the shard < 2^31).
// (row, column) of word i of a swizzled rows16 tile (see pair_rows16_chunk)
__device__ __forceinline__ void pair_tile16_word(int i, int rb0, int cb0, int& r, int& c) {
  const int a = i >> 7;
  r = rb0 + a;
  c = cb0 + 2 * ((i & 127) ^ (a & 31));
}

__device__ __forceinline__ void pair_tile16_flush(const uint32_t* tile, int bi, int bj, int32_t F1, int64_t ld,
                                                  uint32_t* __restrict__ out) {
  const int rb0 = bi * kPB16, cb0 = bj * kPB16;
  const bool pair64 = (ld & 1) == 0;
  for (int i = threadIdx.x; i < kPB16 * kPB16 / 2; i += blockDim.x) {
    const uint32_t v = tile[i];
    if (!v) continue;
    int r, c;
    pair_tile16_word(i, rb0, cb0, r, c);
    if (r >= F1) continue;
    uint32_t* o = out + (int64_t)r * ld + c;
    if (pair64 && c + 1 < F1) {
      atomicAdd(reinterpret_cast<unsigned long long*>(o),
                (unsigned long long)(v & 0xFFFFu) | ((unsigned long long)(v >> 16) << 32));
    } else {
      if ((v & 0xFFFF) && c < F1) atomicAdd(o, v & 0xFFFF);
      if ((v >> 16) && c + 1 < F1) atomicAdd(o + 1, v >> 16);
    }
  }
}

// Work-queue schedule of the same tiles: one persistent workgroup per CU, a
// queue of sub-chunks (<= 32767 rows) per tile.  A workgroup starts on its home
// tile (blockIdx % nbp) and keeps its LDS tile across sub-chunks: after each
// one, counters with bit 15 set give 32768 to the global count ("drain"), so
// every counter stays < 32768 + 32767 and a tile is flushed only when the
// workgroup moves to another tile (then: the tile with the most sub-chunks
// left) or ends.  (A one-chunk-per-workgroup schedule flushed a full 64K-counter
// tile per 65K rows: ~1e9 global atomics on T10I4D100M.)
// Every workgroup exits once all queues are exhausted (each grab increments a
// queue counter, which never decreases).
constexpr int64_t kQSubB = 511;   // batches per sub-chunk: 32704 rows

__global__ __launch_bounds__(1024) void k_pair_queue16(
    const uint8_t* __restrict__ cnt, const int64_t* __restrict__ base, const uint8_t* __restrict__ lr,
    int64_t T, int64_t nbatch, int32_t F1, int64_t ld, int nb, int nbp, int* __restrict__ qctr, int nsub,
    uint32_t* __restrict__ out) {
  __shared__ PairRowsLds L;
  __shared__ int s_take[2];
  for (int t = threadIdx.x; t < kTriTab; t += blockDim.x) {
    int j = 1;
    while ((j + 1) * j / 2 <= t) ++j;            // t in [j (j - 1) / 2, j (j + 1) / 2)
    L.tri[t] = (uint16_t)((t - j * (j - 1) / 2) | (j << 8));
  }                                             // (ordered before use by the first tile's barriers)
  int cur = -1;                                 // tile held in LDS
  int t = (int)(blockIdx.x % (unsigned)nbp);    // tile to take work from
  for (;;) {
    if (threadIdx.x == 0) {
      int got = -1, tt = t;
      if (tt >= 0) {
        const int g = atomicAdd(&qctr[tt], 1);
        if (g < nsub) got = g;
      }
      if (got < 0) {
        // this tile is exhausted: the tile with the most sub-chunks left, if any
        int best = -1, left = 0;
        for (int x = 0; x < nbp; ++x) {
          const int l = nsub - __hip_atomic_load(&qctr[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (l > left) { left = l; best = x; }
        }
        tt = best;
        if (tt >= 0) {
          const int g = atomicAdd(&qctr[tt], 1);
          got = g < nsub ? g : -2;              // -2: lost a race, look again
        }
      }
      s_take[0] = tt;
      s_take[1] = got;
    }
    __syncthreads();
    const int tt = s_take[0], got = s_take[1];
    __syncthreads();
    if (got == -2) { t = -1; continue; }
    if (tt < 0 || got < 0) break;
    t = tt;
    if (tt != cur) {
      if (cur >= 0) {
        int bi, bj;
        tri_index(cur, nb, bi, bj);
        pair_tile16_flush(L.tile, bi, bj, F1, ld, out);
      }
      __syncthreads();
      for (int i = threadIdx.x; i < kPB16 * kPB16 / 2; i += blockDim.x) L.tile[i] = 0;
      __syncthreads();
      cur = tt;
    }
    int bi, bj;
    tri_index(cur, nb, bi, bj);
    const int64_t q0 = (int64_t)got * kQSubB, q1 = min(nbatch, q0 + kQSubB);
    pair_rows16_chunk(L, cnt, base, lr, T, nbatch, bi, bj, q0, q1);
    __syncthreads();
    // drain: bit 15 of either counter -> 32768 to the global count
    const int rb0 = bi * kPB16, cb0 = bj * kPB16;
    for (int i = threadIdx.x; i < kPB16 * kPB16 / 2; i += blockDim.x) {
      const uint32_t v = L.tile[i];
      const uint32_t hb = v & 0x80008000u;
      if (!hb) continue;
      L.tile[i] = v - hb;
      int r, c;
      pair_tile16_word(i, rb0, cb0, r, c);
      if (r >= F1) continue;
      if ((hb & 0x8000u) && c < F1) atomicAdd(&out[(int64_t)r * ld + c], 32768u);
      if ((hb >> 16) && c + 1 < F1) atomicAdd(&out[(int64_t)r * ld + c + 1], 32768u);
    }
    __syncthreads();
  }
  if (cur >= 0) {
    int bi, bj;
    tri_index(cur, nb, bi, bj);
    pair_tile16_flush(L.tile, bi, bj, F1, ld, out);
  }
}

// ---------------------------------------------------------------------------
// F_2 = pairs with count >= minCount (FastApriori.scala:236-238), compacted on the
// device in triangle order (row i ascending, then j): three small kernels instead of
// the gather / compare / scan / two index_copy passes of torch.  The counts come
// either as the pair kernel's matrix (pc[i * ld + j], j > i) or as the all-reduced
// flat triangle (pc[tri(i) + j - i - 1], ld < 0).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t pc_tri_base(int64_t i, int64_t F1) { return i * F1 - i * (i + 1) / 2; }

__device__ __forceinline__ uint32_t pc_at(const uint32_t* __restrict__ pc, int64_t ld, int64_t F1, int64_t i,
                                          int64_t j) {
  return ld >= 0 ? pc[i * ld + j] : pc[pc_tri_base(i, F1) + (j - i - 1)];
}

// one workgroup per row i: its kept pairs
__global__ __launch_bounds__(256) void k_pairs_keep_count(const uint32_t* __restrict__ pc, int64_t ld, int F1,
                                                          int64_t mc, int32_t* __restrict__ row_cnt) {
  __shared__ int part[4];
  const int i = blockIdx.x;
  int c = 0;
  for (int j = i + 1 + threadIdx.x; j < F1; j += 256) c += (int64_t)pc_at(pc, ld, F1, i, j) >= mc;
  c = (int)wave_sum_u32((uint32_t)c);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) row_cnt[i] = part[0] + part[1] + part[2] + part[3];
}

// exclusive row offsets (one workgroup), |F_2| into n_out[0]
__global__ __launch_bounds__(1024) void k_pairs_scan(const int32_t* __restrict__ row_cnt, int F1,
                                                     int64_t* __restrict__ row_off, int64_t* __restrict__ n_out) {
  __shared__ int64_t part[16];
  __shared__ int64_t carry;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int b = 0; b < F1; b += 1024) {
    const int i = b + threadIdx.x;
    const int v = i < F1 ? row_cnt[i] : 0;
    const int incl = wave_scan_incl_dpp(v);
    if (lane == 63) part[wv] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int q = 0; q < wv; ++q) before += part[q];
    if (i < F1) row_off[i] = before + incl - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) n_out[0] = carry;
}

// one workgroup per row: its kept pairs in j order at row_off[i]
__global__ __launch_bounds__(256) void k_pairs_emit(const uint32_t* __restrict__ pc, int64_t ld, int F1, int64_t mc,
                                                    const int64_t* __restrict__ row_off, int32_t* __restrict__ rows,
                                                    int32_t* __restrict__ cnt) {
  __shared__ int part[4];
  __shared__ int64_t carry;
  const int i = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = row_off[i];
  __syncthreads();
  for (int j0 = i + 1; j0 < F1; j0 += 256) {
    const int j = j0 + threadIdx.x;
    const uint32_t v = j < F1 ? pc_at(pc, ld, F1, i, j) : 0u;
    const int keep = (j < F1 && (int64_t)v >= mc) ? 1 : 0;
    const int incl = wave_scan_incl_dpp(keep);
    if (lane == 63) part[wv] = incl;
    __syncthreads();
    int64_t at = carry;
    for (int q = 0; q < wv; ++q) at += part[q];
    at += incl - keep;
    if (keep) {
      rows[2 * at] = i;
      rows[2 * at + 1] = j;
      cnt[at] = (int32_t)v;
    }
    __syncthreads();
    if (threadIdx.x == 255) carry = at + keep;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Item-major bitmaps in one of two layouts, word w of item row r at
//   (w >> 3) * bs + r * rs + (w & 7):
// row-major [F1][Wp] (rs = Wp, bs = 8) -- the multi-pass levels' -- or 8-word blocks
// [Wp / 8][F1][8] (rs = 8, bs = 8 F1) -- the Gram's: a Gram stage reads 256 rows x 8
// words as 16 KB contiguous and the build writes each 64-B block of every row into one
// 8 F1-word run, where row-major puts those 64 B 12.5 MB apart (T40I10D100M: 512 rows a
// stage; scripts/microbench/bitmap_fetch.cpp: stage fetches 15.3 -> 7.7 ms, build
// stores 4.4 -> 2.2 ms).  woff (0..7) starts the view inside a block (weight classes
// and candidate-mode slices that begin off a block boundary).
// ---------------------------------------------------------------------------
struct BmView {
  const uint64_t* p;
  int64_t rs, bs;
  int woff;
  __device__ __forceinline__ int64_t idx(int row, int64_t w) const {
    w += woff;
    return (w >> 3) * bs + (int64_t)row * rs + (w & 7);
  }
  __device__ __forceinline__ uint64_t operator()(int row, int64_t w) const { return p[idx(row, w)]; }
};

// ---------------------------------------------------------------------------
// k = 2, dense bit-matrix Gram with popcounts.  Tile 64x64 items, K-step 32 words.
// ---------------------------------------------------------------------------
constexpr int kGT = 64, kGK = 32, kGS = kGT + 1;   // LDS row stride (u64) breaks bank aliasing

template <bool kWeighted>
__global__ __launch_bounds__(256) void k_pair_gram_popc(
    BmView bm, int32_t F1, int64_t W,
    const int32_t* __restrict__ wword, int nt, int ntp, int64_t kchunk, uint32_t* __restrict__ out) {
  __shared__ uint64_t As[kGK * kGS];
  __shared__ uint64_t Bs[kGK * kGS];
  __shared__ int32_t Ws[kGK];
  const int tp = blockIdx.x % ntp;
  const int64_t kc = blockIdx.x / ntp;
  int ti, tj;
  tri_index(tp, nt, ti, tj);
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  uint32_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0;
  const int64_t k_begin = kc * kchunk, k_end = min(W, k_begin + kchunk);
  for (int64_t k0 = k_begin; k0 < k_end; k0 += kGK) {
#pragma unroll
    for (int it = 0; it < (kGT * kGK) / 256; ++it) {
      const int idx = threadIdx.x + it * 256;
      const int r = idx / kGK, k = idx % kGK;
      const int ra = ti * kGT + r, rb = tj * kGT + r;
      const int64_t kk = k0 + k;
      As[k * kGS + r] = (ra < F1 && kk < k_end) ? bm(ra, kk) : 0ull;
      Bs[k * kGS + r] = (rb < F1 && kk < k_end) ? bm(rb, kk) : 0ull;
    }
    if (kWeighted && threadIdx.x < kGK) {
      const int64_t kk = k0 + threadIdx.x;
      Ws[threadIdx.x] = kk < k_end ? wword[kk] : 0;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < kGK; ++k) {
      uint64_t a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[k * kGS + ty * 4 + i]; b[i] = Bs[k * kGS + tx * 4 + i]; }
      if (kWeighted) {
        const uint32_t wk = (uint32_t)Ws[k];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] += popc64_acc(a[i] & b[j], 0) * wk;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = popc64_acc(a[i] & b[j], acc[i][j]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = ti * kGT + ty * 4 + i, c = tj * kGT + tx * 4 + j;
      if (r < c && c < F1 && acc[i][j]) atomicAdd(&out[(int64_t)r * F1 + c], acc[i][j]);
    }
}

// ---------------------------------------------------------------------------
// k = 2, dense bit-matrix Gram on the matrix cores (one weight class per launch).
//
// count[a][b] = sum_t bit_a(t) bit_b(t) = (B^T B)[a][b] with B the T x F1 0/1
// matrix: a GEMM with K = transactions.  Bits are unpacked to int8 in registers
// (a nibble n -> 4 bytes by (n * 0x204081) & 0x01010101, no carries) and fed
// to v_mfma_i32_32x32x32_i8 with exact int32 accumulation.  A workgroup owns an
// item tile (4 waves, each a square of 32 x 32 MFMA tiles) and a chunk of bitmap
// words, staged through LDS 8 words (512 transactions) at a time
// with coalesced 64-byte row reads; partial tiles are added with one atomic
// per element.  Lane (r, h) supplies A[r][16h + j] and B[16h + j][c] from the
// same 16 transactions, so the K pairing is exact whatever the hardware's
// k-order inside a lane half is (the same for A and B).
// ---------------------------------------------------------------------------
typedef int fa_v4i __attribute__((ext_vector_type(4)));
typedef int fa_v16i __attribute__((ext_vector_type(16)));
constexpr int kMW = 16;      // words staged per step
constexpr int kMS = kMW + 1; // LDS row stride (words): 136 B rows -> conflict-free ds_read_b64

__device__ __forceinline__ fa_v4i unpack16_i8(uint32_t b) {
  fa_v4i r;
  r.x = (int)(((b & 0xFu) * 0x00204081u) & 0x01010101u);
  r.y = (int)((((b >> 4) & 0xFu) * 0x00204081u) & 0x01010101u);
  r.z = (int)((((b >> 8) & 0xFu) * 0x00204081u) & 0x01010101u);
  r.w = (int)((((b >> 12) & 0xFu) * 0x00204081u) & 0x01010101u);
  return r;
}

// Bit-matrix Gram on the matrix cores with a 128 x 128 register tile per wave (4 x 4
// MFMA tiles, 256 accumulator registers, one wave per SIMD) and a 256 x 256 workgroup
// tile.  A 2 x 2-tile form (removed) spent more VALU on unpacking bits to int8 than the MFMA
// pipe needs (~14 VALU per 32x32x32 MFMA, i.e. longer than the MFMA's 32 cycles);
// with 4 x 4 tiles every unpacked fragment feeds four MFMAs instead of two.  The
// next stage's words are loaded into registers while the current one is counted.
// On diagonal tiles the wave below the diagonal has no (row < col) entry and skips
// its MFMAs.
constexpr int kM4 = 4;                 // 32 x 32 MFMA tiles per wave side
constexpr int kMT4 = 64 * kM4;         // items per workgroup tile side (2 x 2 waves)
constexpr int kM4Ld = kMT4 * kMW / 256;   // staged words per thread and operand

// kFp4: the same tiles on the block-scaled FP4 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4,
// e2m1 operands): one 64-transaction k-step per bitmap word instead of two
// 32-transaction i8 steps, at the i8 instruction's cycles (twice the K per MFMA).  A
// bit becomes the e2m1 nibble 0b0001 (0.5; both block scales 2^1 make each product 1).
// The transactions may sit in any k order that A and B share, so element (dword d,
// nibble n) of a lane takes transaction 4n + d of its 32: dword d is (x >> d) &
// 0x11111111, two VALU ops, where bits -> i8 bytes cost ~3 per 4 bits.  The f32 sums
// are exact integers while a workgroup's chunk holds <= 2^24 transactions
// (fa_hip_pair_gram_mfma caps kchunk).
typedef int fa_v8i __attribute__((ext_vector_type(8)));
typedef float fa_v16f __attribute__((ext_vector_type(16)));
constexpr int kFp4Scale = 128;   // E8M0 2^1

__device__ __forceinline__ fa_v8i unpack32_fp4(uint32_t x) {
  fa_v8i r;
  r[0] = (int)(x & 0x11111111u);
  r[1] = (int)((x >> 1) & 0x11111111u);
  r[2] = (int)((x >> 2) & 0x11111111u);
  r[3] = (int)((x >> 3) & 0x11111111u);
  r[4] = 0; r[5] = 0; r[6] = 0; r[7] = 0;
  return r;
}

template <bool kFp4>
__global__ __launch_bounds__(256) void k_pair_gram_mfma4(BmView bm, int32_t F1,
                                                         int64_t W, int nt, int ntp, int64_t kchunk,
                                                         uint32_t* __restrict__ out, uint32_t scale) {
  using AccT = std::conditional_t<kFp4, fa_v16f, fa_v16i>;
  __shared__ uint64_t As[kMT4 * kMS];
  __shared__ uint64_t Bs[kMT4 * kMS];
  const uint32_t logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tp = (int)(logical % (uint32_t)ntp);
  const int64_t kc = logical / (uint32_t)ntp;
  int ti, tj;
  tri_index(tp, nt, ti, tj);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wr = (wv >> 1) * 32 * kM4, wc = (wv & 1) * 32 * kM4;   // the wave's 128 x 128 sub-tile
  const bool live = !(ti == tj && wr > wc);
  AccT acc[kM4][kM4];
#pragma unroll
  for (int i = 0; i < kM4; ++i)
#pragma unroll
    for (int j = 0; j < kM4; ++j) acc[i][j] = AccT{0};
  const int64_t k_begin = kc * kchunk, k_end = min(W, k_begin + kchunk);
  uint64_t pa[kM4Ld], pb[kM4Ld];
  auto fetch = [&](int64_t k0) {
#pragma unroll
    for (int it = 0; it < kM4Ld; ++it) {
      const int idx = threadIdx.x + it * 256;
      const int row = idx / kMW, w = idx % kMW;
      const int ra = ti * kMT4 + row, rb = tj * kMT4 + row;
      const int64_t kk = k0 + w;
      pa[it] = (ra < F1 && kk < k_end) ? bm(ra, kk) : 0ull;
      pb[it] = (rb < F1 && kk < k_end) ? bm(rb, kk) : 0ull;
    }
  };
  if (k_begin < k_end) fetch(k_begin);
  for (int64_t k0 = k_begin; k0 < k_end; k0 += kMW) {
#pragma unroll
    for (int it = 0; it < kM4Ld; ++it) {
      const int idx = threadIdx.x + it * 256;
      const int row = idx / kMW, w = idx % kMW;
      As[row * kMS + w] = pa[it];
      Bs[row * kMS + w] = pb[it];
    }
    __syncthreads();
    if (k0 + kMW < k_end) fetch(k0 + kMW);
    if (live) {
#pragma unroll 1
      for (int w = 0; w < kMW; ++w) {
        uint64_t a[kM4], b[kM4];
#pragma unroll
        for (int i = 0; i < kM4; ++i) {
          a[i] = As[(wr + 32 * i + r) * kMS + w];
          b[i] = Bs[(wc + 32 * i + r) * kMS + w];
        }
        if constexpr (kFp4) {
          // one 64-transaction k-step: lane half h takes transactions 32h .. 32h + 31
          fa_v8i fb[kM4];
#pragma unroll
          for (int j = 0; j < kM4; ++j) fb[j] = unpack32_fp4((uint32_t)(b[j] >> (32 * h)));
#pragma unroll
          for (int i = 0; i < kM4; ++i) {
            const fa_v8i fa = unpack32_fp4((uint32_t)(a[i] >> (32 * h)));
#pragma unroll
            for (int j = 0; j < kM4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa, fb[j], acc[i][j], 4, 4, 0, kFp4Scale, 0,
                                                                          kFp4Scale);
          }
        } else {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {                  // two 32-transaction k-steps per word
          const int sh = 32 * s2 + 16 * h;
          fa_v4i fb[kM4];
#pragma unroll
          for (int j = 0; j < kM4; ++j) fb[j] = unpack16_i8((uint32_t)(b[j] >> sh) & 0xFFFFu);
#pragma unroll
          for (int i = 0; i < kM4; ++i) {
            const fa_v4i fa = unpack16_i8((uint32_t)(a[i] >> sh) & 0xFFFFu);
#pragma unroll
            for (int j = 0; j < kM4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb[j], acc[i][j], 0, 0, 0);
          }
        }
        }
      }
    }
    __syncthreads();
  }
  if (!live) return;
  // C/D layout (gfx950, 32x32): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int i = 0; i < kM4; ++i)
#pragma unroll
    for (int j = 0; j < kM4; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int row = ti * kMT4 + wr + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
        const int col = tj * kMT4 + wc + 32 * j + r;
        const uint32_t v = kFp4 ? (uint32_t)(acc[i][j][g] + 0.5f) : (uint32_t)acc[i][j][g];
        if (row < col && col < F1 && v) atomicAdd(&out[(int64_t)row * F1 + col], v * scale);
      }
}

// The FP4 Gram, software-pipelined (the product path; k_pair_gram_mfma4<true> above
// is kept as its reference form).  k_pair_gram_mfma4 kept the matrix pipe busy 41 % of
// the kernel (PMC, T40I10D100M): one wave per SIMD (256 accumulator registers), all 256
// VGPRs taken (16-word register prefetch of both operands), so each word's LDS reads
// went out behind the MFMAs and their s_waitcnt left the pipe idle, plus a 64-bit shift
// per operand to pick the lane half's 32 transactions.  Here
//   * a stage is 8 words (half the prefetch registers) double-buffered in LDS, one
//     barrier per stage;
//   * the two 32-bit halves of a word sit in separate LDS planes (row stride 9 dwords,
//     the hi plane 32 dwords off the lo plane mod 64): one conflict-free ds_read_b32 per
//     operand, no shift;
//   * the unpacked operands are double-buffered and the raw words read two words
//     ahead: word w's 16 MFMAs go out with word w + 1's unpacking interleaved between
//     them (sched_group_barrier) and word w + 2's LDS reads in front, so neither the
//     matrix pipe nor the unpacking waits on LDS.
// The prefetch loads are branch-free (clamped addresses, masked values).
constexpr int kGW = 8;                       // words per stage
constexpr int kGRow = kGW + 1;                 // plane row stride (dwords)
constexpr int kGPl = kMT4 * kGRow + 32;     // plane size (dwords): hi plane = lo + 32 mod 64 banks
constexpr int kGLd = kMT4 * kGW / 256;       // staged words per thread and operand

__global__ __launch_bounds__(256) void k_pair_gram_fp4(BmView bm, int32_t F1,
                                                       int64_t W, int nt, int ntp, int64_t kchunk,
                                                       uint32_t* __restrict__ out, uint32_t scale) {
  __shared__ uint32_t S[2][2][2 * kGPl];      // [buffer][A, B][lo plane, hi plane]
  const uint32_t logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tp = (int)(logical % (uint32_t)ntp);
  const int64_t kc = logical / (uint32_t)ntp;
  int ti, tj;
  tri_index(tp, nt, ti, tj);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int wr = (wv >> 1) * 32 * kM4, wc = (wv & 1) * 32 * kM4;
  const bool live = !(ti == tj && wr > wc);
  fa_v16f acc[kM4][kM4];
#pragma unroll
  for (int i = 0; i < kM4; ++i)
#pragma unroll
    for (int j = 0; j < kM4; ++j) acc[i][j] = fa_v16f{0};
  const int64_t k_begin = kc * kchunk, k_end = min(W, k_begin + kchunk);
  uint64_t pa[kGLd], pb[kGLd];
  uint32_t oka = 0, okb = 0;
  auto fetch = [&](int64_t k0) {
    oka = okb = 0;
#pragma unroll
    for (int it = 0; it < kGLd; ++it) {
      const int idx = threadIdx.x + it * 256;
      const int row = idx / kGW, w = idx % kGW;
      const int ra = ti * kMT4 + row, rb = tj * kMT4 + row;
      const int64_t kk = k0 + w;
      const bool okk = kk < k_end;
      pa[it] = bm(ra < F1 ? ra : 0, okk ? kk : k_begin);
      pb[it] = bm(rb < F1 ? rb : 0, okk ? kk : k_begin);
      oka |= (uint32_t)(ra < F1 && okk) << it;
      okb |= (uint32_t)(rb < F1 && okk) << it;
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int it = 0; it < kGLd; ++it) {
      const int idx = threadIdx.x + it * 256;
      const int row = idx / kGW, w = idx % kGW;
      const uint64_t a = ((oka >> it) & 1) ? pa[it] : 0ull;
      const uint64_t b = ((okb >> it) & 1) ? pb[it] : 0ull;
      S[buf][0][row * kGRow + w] = (uint32_t)a;
      S[buf][0][kGPl + row * kGRow + w] = (uint32_t)(a >> 32);
      S[buf][1][row * kGRow + w] = (uint32_t)b;
      S[buf][1][kGPl + row * kGRow + w] = (uint32_t)(b >> 32);
    }
  };
  if (k_begin < k_end) {
    fetch(k_begin);
    stage(0);
  }
  __syncthreads();
  // the lane's row offsets in its half's plane
  int oa[kM4], ob[kM4];
#pragma unroll
  for (int i = 0; i < kM4; ++i) {
    oa[i] = h * kGPl + (wr + 32 * i + r) * kGRow;
    ob[i] = h * kGPl + (wc + 32 * i + r) * kGRow;
  }
  int buf = 0;
  for (int64_t k0 = k_begin; k0 < k_end; k0 += kGW) {
    const bool more = k0 + kGW < k_end;
    if (more) fetch(k0 + kGW);                   // global loads in flight during the MFMAs
    if (live) {
      const uint32_t* As = S[buf][0];
      const uint32_t* Bs = S[buf][1];
      fa_v8i fa0[kM4], fb0[kM4], fa1[kM4], fb1[kM4];
      uint32_t ra[kM4], rb[kM4], qa[kM4], qb[kM4];   // raw words one and two ahead
#pragma unroll
      for (int i = 0; i < kM4; ++i) {
        fa0[i] = unpack32_fp4(As[oa[i]]);
        fb0[i] = unpack32_fp4(Bs[ob[i]]);
        ra[i] = As[oa[i] + 1];
        rb[i] = Bs[ob[i] + 1];
      }
      // word w's MFMAs on (fa, fb), the unpacking of word w + 1 (raw words (ca, cb),
      // read one step earlier, so it never waits on LDS) into (na, nb) between them,
      // and the reads of word w + 2 into (la, lb) ahead of them; branch-free: the
      // stage's last two steps re-read words 0 and 1
      auto step = [&](fa_v8i* fa, fa_v8i* fb, fa_v8i* na, fa_v8i* nb, const uint32_t* ca, const uint32_t* cb,
                      uint32_t* la, uint32_t* lb, int wl) {
#pragma unroll
        for (int i = 0; i < kM4; ++i) {
          la[i] = As[oa[i] + wl];
          lb[i] = Bs[ob[i] + wl];
        }
#pragma unroll
        for (int i = 0; i < kM4; ++i)
#pragma unroll
          for (int j = 0; j < kM4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[i], fb[j], acc[i][j], 4, 4, 0, kFp4Scale,
                                                                        0, kFp4Scale);
#pragma unroll
        for (int i = 0; i < kM4; ++i) {
          na[i] = unpack32_fp4(ca[i]);
          nb[i] = unpack32_fp4(cb[i]);
        }
        // the 8 LDS reads, then one MFMA and 5 VALU (the unpacking, 7 per operand) at a
        // time (scripts/microbench/gram_mfma.cpp mode 3: 43.7 cycles per MFMA per SIMD,
        // MFMA alone 41.4; reads one word ahead with 3 MFMAs in front: 59.0)
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
        for (int q = 1; q < kM4 * kM4; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
        }
        __builtin_amdgcn_sched_barrier(0);          // each step its own scheduling region
      };
#pragma unroll 1
      for (int w = 0; w < kGW; w += 2) {
        step(fa0, fb0, fa1, fb1, ra, rb, qa, qb, (w + 2) & (kGW - 1));
        step(fa1, fb1, fa0, fb0, qa, qb, ra, rb, (w + 3) & (kGW - 1));
      }
    }
    if (more) stage(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  if (!live) return;
#pragma unroll
  for (int i = 0; i < kM4; ++i)
#pragma unroll
    for (int j = 0; j < kM4; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int row = ti * kMT4 + wr + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
        const int col = tj * kMT4 + wc + 32 * j + r;
        const uint32_t v = (uint32_t)(acc[i][j][g] + 0.5f);
        if (row < col && col < F1 && v) atomicAdd(&out[(int64_t)row * F1 + col], v * scale);
      }
}

// ---------------------------------------------------------------------------
// k >= 3: prefix-shared candidate counting.
// Workgroup = (super-chunk sc of 256*kWPT words) x (group block gb).  Each thread
// keeps its kWPT words of the prefix AND in registers, streams every
// extension's words, and the 4 waves reduce into an LDS accumulator.
// ---------------------------------------------------------------------------
constexpr int kWPT = 8;
constexpr int kMaxBlockExt = 1024;

template <bool kWeighted>
__global__ __launch_bounds__(256) void k_count_candidates(
    const uint64_t* __restrict__ bm, int64_t Wp, int64_t W, const int32_t* __restrict__ prefix, int m,
    const int64_t* __restrict__ ext_off, const int32_t* __restrict__ ext,
    const int32_t* __restrict__ gb_start, int ngb, const int32_t* __restrict__ wword,
    uint32_t* __restrict__ out) {
  __shared__ uint32_t acc[kMaxBlockExt];
  const uint32_t logical = xcd_remap(blockIdx.x, gridDim.x);
  const int gb = logical % ngb;
  const int64_t sc = logical / ngb;
  const int g0 = gb_start[gb], g1 = gb_start[gb + 1];
  const int64_t e_base = ext_off[g0];
  const int n_ext = (int)(ext_off[g1] - e_base);
  for (int i = threadIdx.x; i < n_ext; i += blockDim.x) acc[i] = 0;
  const int64_t w0 = sc * (256 * kWPT) + threadIdx.x;
  bool valid[kWPT];
  int32_t wt[kWPT];
#pragma unroll
  for (int q = 0; q < kWPT; ++q) {
    valid[q] = w0 + q * 256 < W;
    wt[q] = (kWeighted && valid[q]) ? wword[w0 + q * 256] : 1;
  }
  __syncthreads();
  for (int g = g0; g < g1; ++g) {
    uint64_t p[kWPT];
    const int32_t* pr = prefix + (int64_t)g * m;
    {
      const uint64_t* row = bm + (int64_t)pr[0] * Wp + w0;
#pragma unroll
      for (int q = 0; q < kWPT; ++q) p[q] = valid[q] ? row[q * 256] : 0ull;
    }
    for (int j = 1; j < m; ++j) {
      const uint64_t* row = bm + (int64_t)pr[j] * Wp + w0;
#pragma unroll
      for (int q = 0; q < kWPT; ++q) p[q] &= valid[q] ? row[q * 256] : 0ull;
    }
    for (int64_t e = ext_off[g]; e < ext_off[g + 1]; ++e) {
      const uint64_t* row = bm + (int64_t)ext[e] * Wp + w0;
      uint32_t s = 0;
#pragma unroll
      for (int q = 0; q < kWPT; ++q) {
        const uint64_t v = valid[q] ? (p[q] & row[q * 256]) : 0ull;
        if (kWeighted) s += popc64_acc(v, 0) * (uint32_t)wt[q];
        else s = popc64_acc(v, s);
      }
      s = wave_sum_u32(s);
      if (lane_id() == 0 && s) atomicAdd(&acc[e - e_base], s);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_ext; i += blockDim.x)
    if (acc[i]) atomicAdd(&out[e_base + i], acc[i]);
}

// ---------------------------------------------------------------------------
// k >= 3, slab-stationary counting (the default path).
//
// A slab = SW consecutive bitmap words (64*SW columns).  Each workgroup walks
// slabs b = blockIdx.x, +gridDim.x, ...: it builds the slab of every item used
// by this level's candidates directly in LDS from the compressed rows
// (ds_or_b64), then every thread takes candidate groups, ANDs the group's
// prefix rows once into registers and popcounts each extension row against it,
// adding into a per-candidate LDS accumulator that lives across all slabs.
// One pass reads the compressed rows once and touches HBM for nothing else;
// the global bitmap is never materialised.  One coalesced atomic per candidate
// per workgroup at the end.
// ---------------------------------------------------------------------------
constexpr int kSlabThreads = 1024;

// Slab build modes: per-column rank prefetch (dedup: columns gather rows through
// src), wave-cooperative coalesced build (columns = rows, contiguous ranks), or
// a copy from the materialised used-item bitmap (multi-pass levels).
enum { kBuildCols = 0, kBuildContig = 1, kBuildBM = 2 };

// Coalesced slab build for one 64-column word q of the tile: the 64 rows'
// ranks are one contiguous span, read 2 x 64 at a time; a rank's column is the
// last row whose start is <= its position (6-step binary search over the row
// starts held one per lane, __shfl).  Empty rows are skipped by the search.
// nsub waves share one word: wave h of them takes window groups h, h + nsub, ...
// A rank's column (bit) is the row owning its position: rows are non-empty, so
// it is (row starts before the window) + popc(start mask & lanes <= me) - 1.
// rank -> slab row (-1: not used) from the global int32 map, or from the
// workgroup's u16 copy in LDS (k_count_slab_rec; 0xFFFF = not used)
struct MapGlobal {
  const int32_t* __restrict__ p;
  __device__ __forceinline__ int operator()(int r) const { return p[r]; }
};
struct MapLds {
  const uint16_t* p;
  __device__ __forceinline__ int operator()(int r) const {
    const int v = p[r];
    return v == 0xFFFF ? -1 : v;
  }
};

// The CSR span of a 64-column word: this lane's row start, the word's first and end
// positions (loaded ahead of the build by k_count_slab_rec: one HBM round trip less
// in every slab's build phase).
struct WordSpan {
  int64_t st, base, end;
};
__device__ __forceinline__ WordSpan word_span(const int64_t* __restrict__ roff, int64_t col0, int64_t ncols) {
  const int lane = threadIdx.x & 63;
  return WordSpan{roff[min(col0 + lane, ncols)], roff[col0], roff[min(col0 + 64, ncols)]};
}

template <class Map>
__device__ __forceinline__ void slab_build_word_span(uint64_t* __restrict__ slab, int swp, int q, const WordSpan& ws,
                                                     const int32_t* __restrict__ ranks, Map item_map, int h,
                                                     int nsub, unsigned long long* words, int swz);

template <class Map = MapGlobal>
__device__ __forceinline__ void slab_build_word_m(uint64_t* __restrict__ slab, int swp, int q, int64_t col0,
                                                  int64_t ncols, const int64_t* __restrict__ roff,
                                                  const int32_t* __restrict__ ranks, Map item_map, int h,
                                                  int nsub, unsigned long long* words, int swz = 0) {
  slab_build_word_span(slab, swp, q, word_span(roff, col0, ncols), ranks, item_map, h, nsub, words, swz);
}

template <class Map>
__device__ __forceinline__ void slab_build_word_span(uint64_t* __restrict__ slab, int swp, int q, const WordSpan& ws,
                                                     const int32_t* __restrict__ ranks, Map item_map, int h,
                                                     int nsub, unsigned long long* words, int swz) {
  const int lane = threadIdx.x & 63;
  const int64_t st = ws.st, base = ws.base, end = ws.end;
  const int srel = (int)(st - base);
  const int n = (int)(end - base);
  const unsigned long long le = lanes_le_mask();
  constexpr int U = 2;                                // windows per step (4 measured slower)
  const int step = 64 * U * nsub;
  // software pipeline: the ranks of the next two steps are loaded before this step's
  // window masks and LDS atomics, so the HBM latency of a step overlaps the previous ones
  int rn[U], rn2[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int p = 64 * U * h + 64 * u + lane;
    rn[u] = p < n ? ranks[base + p] : -1;
    rn2[u] = p + step < n ? ranks[base + p + step] : -1;
  }
  for (int p0 = 64 * U * h; p0 < n; p0 += step) {
    int r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = rn[u];
      rn[u] = rn2[u];
      const int p = p0 + 2 * step + 64 * u + lane;
      rn2[u] = p < n ? ranks[base + p] : -1;
    }
    // starts before p0: rows with srel < p0 (ballot over the row owners)
    const int cs0 = __popcll(__ballot(srel < p0));
    unsigned long long S[U];
    window_starts<U>(words, srel, p0, S);
    int cs = cs0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int l = cs + __popcll(S[u] & le) - 1;
      const int uu = r[u] >= 0 ? item_map(r[u]) : -1;
      if (uu >= 0) atomicOr((unsigned long long*)(slab + (size_t)uu * swp + (q ^ ((uu << 2) & swz))), 1ull << l);
      cs += __popcll(S[u]);
    }
  }
}

__device__ __forceinline__ void slab_build_word(uint64_t* __restrict__ slab, int swp, int q, int64_t col0,
                                                int64_t ncols, const int64_t* __restrict__ roff,
                                                const int32_t* __restrict__ ranks,
                                                const int32_t* __restrict__ item_map, int h, int nsub,
                                                unsigned long long* words, int swz = 0) {
  slab_build_word_m(slab, swp, q, col0, ncols, roff, ranks, MapGlobal{item_map}, h, nsub, words, swz);
}

// Multi-pass levels copy the slab tile of every used item from the
// materialised bitmap.  A plain strided loop (load, store, next) pays one global
// round trip per 16 B a thread copies (~8-10 per slab at 1024 threads);
// here every thread issues all its loads (after one batched load of the
// bitmap row ids) before its first LDS store.  ROWW: LDS row stride in words;
// kSwz: an XOR of the word slot by ((u << 2) & (SW - 4)) (rotated row layouts).
// ld > 0: a row-major bitmap of row stride ld; ld < 0: the 8-word block layout of
// block stride -ld (BmView: the Gram's bitmap, reused by the levels after it; slab
// starts and word pairs stay inside one block).
template <int SW, int ROWW, bool kSwz>
__device__ __forceinline__ void slab_copy_bm(uint4* lds4, int n_used, const uint64_t* __restrict__ bm, int64_t Wp,
                                             const int32_t* __restrict__ bm_rows, int64_t w0, int64_t W) {
  constexpr int QW = SW / 2;                 // uint4 per row
  constexpr int KMAX = 4;                    // loads in flight per thread
  const int total = n_used * QW;
  for (int base = 0; base < total; base += KMAX * kSlabThreads) {
    int32_t br[KMAX];
    uint4 v[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int i = base + (int)threadIdx.x + k * kSlabThreads;
      br[k] = i < total ? (bm_rows ? bm_rows[i / QW] : i / QW) : 0;
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int i = base + (int)threadIdx.x + k * kSlabThreads;
      const int64_t w = w0 + 2 * (i % QW);
      v[k] = make_uint4(0, 0, 0, 0);
      // rows are Wp (a multiple of 64) words long and zero past W: a pair whose
      // first word is valid may be read whole
      const int64_t at = Wp > 0 ? (int64_t)br[k] * Wp + w : (w >> 3) * -Wp + (int64_t)br[k] * 8 + (w & 7);
      if (i < total && w < W) v[k] = *reinterpret_cast<const uint4*>(bm + at);
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int i = base + (int)threadIdx.x + k * kSlabThreads;
      if (i < total) {
        const int u = i / QW, q = i % QW;
        const int qq = kSwz ? (q ^ (((u << 2) & (SW - 4)) >> 1)) : q;
        lds4[(size_t)u * (ROWW / 2) + qq] = v[k];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k >= 3, slab-stationary counting from piece records (the slab path of
// fa_level_plan).
//
// Slab build (above) and thread-per-piece counting, with the piece metadata laid
// out for latency.  PMC of the earlier per-group kernel on the T10I4D100M level 3-4
// bundle: waves wait ~64 % of their cycles, only ~3 % of it on LDS -- every piece
// walked a chain of dependent global loads (gpm -> prefix ids -> slab rows,
// gext_off -> each extension id).  Here a piece is one 48-B record (plan.cpp):
//   a = {ext begin, n_ext | m << 8 | long-prefix flag << 16, prefix ids 0-3 (u16)}
//   b = {extension ids 0-7 (u16)}
//   c = {prefix ids 4-11 (u16)}, or c.x = gpre offset when m > 12
// loaded one piece ahead.  A thread's pieces are the same on every slab, so the
// load after its last piece fetches its first piece for the next slab.  The
// rank -> slab-row map of the slab build is copied to LDS as u16 (one dependent
// global load less per rank).
// ---------------------------------------------------------------------------
constexpr int kMapLdsMax = 8192;   // plan.cpp fa_slab_map_lds: F1 <= this keeps the map in LDS

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
  // popcount + add in one VALU op (the compiler otherwise splits the sum into
  // v_bcnt(x, 0) + v_add3 trees: 25 % more VALU in the extension loop)
  uint32_t r;
  __asm__("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
  return r;
}

__device__ __forceinline__ uint32_t and3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x80);
}

__device__ __forceinline__ int u16_at(const int4& v, int k) {
  const int w = (k >> 1) == 0 ? v.x : (k >> 1) == 1 ? v.y : (k >> 1) == 2 ? v.z : v.w;
  return (k & 1) ? (int)((uint32_t)w >> 16) : (w & 0xFFFF);
}

template <int SW, bool kWeighted, int kBuild, bool kCls = false, bool kAcc16 = false>
__global__ __launch_bounds__(kSlabThreads) void k_count_slab_rec(
    const int64_t* __restrict__ roff, const int32_t* __restrict__ ranks, const int32_t* __restrict__ src,
    int64_t ncols, const int32_t* __restrict__ item_map, int F1, int n_used, const int32_t* __restrict__ gpre,
    const int4* __restrict__ rec, int G_arg, int C, const int32_t* __restrict__ wword, uint32_t* __restrict__ out,
    const uint64_t* __restrict__ bm, int64_t Wp, const int32_t* __restrict__ bm_rows, int flags,
    const int32_t* __restrict__ g_dev) {
  // g_dev: the piece count from device memory (device-planned bundles, levels.hip)
  const int G = g_dev ? *g_dev : G_arg;
  extern __shared__ uint4 lds4[];
  __shared__ unsigned long long build_words[kSlabThreads / 64 * 2];
  constexpr int SWP = SW + 2;                       // row stride: odd number of 16-B slots
  constexpr int RS = SWP / 2;
  uint64_t* slab = reinterpret_cast<uint64_t*>(lds4);
  // kAcc16 (flags & 8): two u16 counters per accumulator word (unit weights; twice the
  // candidates per accumulator pass), drained into the u32 global counts before they can
  // carry: a slab adds at most SW * 64 to a counter.  A template parameter: a runtime
  // flag put a scalar branch pair around every accumulator add of the extension loop.
  constexpr bool acc16 = !kWeighted && kAcc16;
  const int nacc = acc16 ? (C + 1) >> 1 : C;
  constexpr int kFlush16 = 65535 / (SW * 64);
  uint32_t* acc = reinterpret_cast<uint32_t*>(slab + (size_t)n_used * SWP);
  uint16_t* smap = reinterpret_cast<uint16_t*>(acc + ((nacc + 3) & ~3));
  const bool map_lds = kBuild == kBuildContig && F1 <= kMapLdsMax;
  for (int i = threadIdx.x; i < nacc; i += blockDim.x) acc[i] = 0;
  if (map_lds) {
    for (int i = threadIdx.x; i < F1; i += blockDim.x) {
      const int v = item_map[i];
      smap[i] = v < 0 ? (uint16_t)0xFFFF : (uint16_t)v;
    }
  }
  const int64_t W = (ncols + 63) >> 6;
  const int64_t nslabs = (W + SW - 1) / SW;
  const int4 z4 = make_int4(0, 0, 0, 0);
  // candidate distribution (flags bits 8-15: this rank, 16-23: ranks - 1): the rank counts
  // the 64-piece chunks part, part + nparts, ... over all rows, one chunk per wave step, so
  // a wave still walks 64 consecutive records (the lane deal stays valid)
  const int ppart = (flags >> 8) & 0xFF, npart = ((flags >> 16) & 0xFF) + 1;
  const int gstep = kSlabThreads * npart;
  const int g0 = (ppart + npart * (int)(threadIdx.x >> 6)) * 64 + (int)(threadIdx.x & 63);
  int4 ra = z4, rb = z4, rc = z4;
  if (g0 < G) { ra = rec[3 * g0]; rb = rec[3 * g0 + 1]; rc = rec[3 * g0 + 2]; }

  auto and_row = [&](uint4 (&p)[SW / 2], int u) {
    const uint4* r = lds4 + (size_t)u * RS;
#pragma unroll
    for (int q = 0; q < SW / 2; ++q) {
      const uint4 v = r[q];
      p[q].x &= v.x; p[q].y &= v.y; p[q].z &= v.z; p[q].w &= v.w;
    }
  };
  // two prefix rows per VALU op: v_bitop3_b32 p & a & b (truth table 0x80); the
  // prefix ANDs were ~60 % of the counting VALU of the deep bundles (m ~ 5, 1-2
  // extensions per piece)
  auto and_row2 = [&](uint4 (&p)[SW / 2], int u, int w) {
    const uint4* r = lds4 + (size_t)u * RS;
    const uint4* t = lds4 + (size_t)w * RS;
#pragma unroll
    for (int q = 0; q < SW / 2; ++q) {
      const uint4 v = r[q], x = t[q];
      p[q].x = and3(p[q].x, v.x, x.x); p[q].y = and3(p[q].y, v.y, x.y);
      p[q].z = and3(p[q].z, v.z, x.z); p[q].w = and3(p[q].w, v.w, x.w);
    }
  };
  // AND of prefix rows [j0, j1) of the piece (ids 1-3 in ra, 4-11 in rc), two at a time
  auto pid = [&](int j) { return j < 4 ? u16_at(ra, 4 + j) : u16_at(rc, j - 4); };
  auto and_prefix = [&](uint4 (&p)[SW / 2], int j0, int j1) {
#pragma unroll
    for (int j = 1; j < 12; j += 2) {
      if (j >= j0 && j < j1) {
        if (j + 1 < j1) and_row2(p, pid(j), pid(j + 1));
        else and_row(p, pid(j));
      }
    }
  };
  auto acc_add = [&](int e, uint32_t v) {
    if (acc16) atomicAdd(&acc[e >> 1], v << ((e & 1) << 4));
    else atomicAdd(&acc[e], v);
  };
  auto flush = [&]() {
    for (int i = threadIdx.x; i < nacc; i += blockDim.x) {
      const uint32_t v = acc[i];
      if (!v) continue;
      if (acc16) {
        if (v & 0xFFFFu) atomicAdd(&out[2 * i], v & 0xFFFFu);
        if ((v >> 16) && 2 * i + 1 < C) atomicAdd(&out[2 * i + 1], v >> 16);
        acc[i] = 0;
      } else {
        atomicAdd(&out[i], v);
      }
    }
  };
  int nsl = 0;                                      // slabs counted since the last u16 drain
  // contiguous build with one word per wave (SW <= 8; at SW = 16 the span spills): the word's CSR span for the
  // next slab is loaded before this slab's counting, so the build starts without
  // waiting on the row offsets
  constexpr int kNW = kSlabThreads / 64;
  constexpr bool kOneWord = kBuild == kBuildContig && SW <= 8 && SW * (kNW > SW ? kNW / SW : 1) == kNW;
  const int my_q = (int)(threadIdx.x >> 6) / (kNW > SW ? kNW / SW : 1);
  WordSpan span{0, 0, 0};
  auto load_span = [&](int64_t sb_) {
    const int64_t col0 = (sb_ * SW + my_q) * 64;
    if (kOneWord && sb_ < nslabs && col0 < ncols) span = word_span(roff, col0, ncols);
  };
  load_span(blockIdx.x);

  for (int64_t sb = blockIdx.x; sb < nslabs; sb += gridDim.x) {
    const int64_t w0 = sb * SW;
    __syncthreads();
    if (acc16 && ++nsl > kFlush16) {               // (the barrier after the build orders it)
      flush();
      nsl = 1;
    }
    if (kBuild == kBuildBM) {
      slab_copy_bm<SW, SWP, false>(lds4, n_used, bm, Wp, bm_rows, w0, W);
    } else {
      {
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (int i = threadIdx.x; i < n_used * RS; i += blockDim.x) lds4[i] = z;
      }
      __syncthreads();
      if (kBuild == kBuildContig) {
        constexpr int NW = kSlabThreads / 64;
        constexpr int NSUB = NW > SW ? NW / SW : 1;
        const int wv = threadIdx.x >> 6;
        if (kOneWord) {
          // one word per wave: its span was loaded ahead (during the previous slab's count)
          const int q = wv / NSUB;
          if ((w0 + q) * 64 < ncols) {
            if (map_lds)
              slab_build_word_span(slab, SWP, q, span, ranks, MapLds{smap}, wv % NSUB, NSUB, build_words + wv * 2, 0);
            else
              slab_build_word_span(slab, SWP, q, span, ranks, MapGlobal{item_map}, wv % NSUB, NSUB,
                                   build_words + wv * 2, 0);
          }
        } else {
          for (int q = wv / NSUB; q < SW; q += NW / NSUB) {
            if ((w0 + q) * 64 >= ncols) continue;
            if (map_lds)
              slab_build_word_m(slab, SWP, q, (w0 + q) * 64, ncols, roff, ranks, MapLds{smap}, wv % NSUB, NSUB,
                                build_words + wv * 2);
            else
              slab_build_word_m(slab, SWP, q, (w0 + q) * 64, ncols, roff, ranks, MapGlobal{item_map}, wv % NSUB,
                                NSUB, build_words + wv * 2);
          }
        }
      } else {
        // dedup layout: column j of the tile gathers row src[col]
        for (int j = threadIdx.x; j < SW * 64; j += blockDim.x) {
          const int64_t col = w0 * 64 + j;
          if (col >= ncols) break;
          const int64_t row = src ? (int64_t)src[col] : col;
          if (row < 0) continue;
          const unsigned long long bit = 1ull << (j & 63);
          uint64_t* base = slab + (j >> 6);
          for (int64_t r = roff[row], r1 = roff[row + 1]; r < r1; ++r) {
            const int uu = item_map[ranks[r]];
            if (uu >= 0) atomicOr((unsigned long long*)(base + (size_t)uu * SWP), bit);
          }
        }
      }
    }
    __syncthreads();
    load_span(sb + gridDim.x);                      // in flight during the counting below
    uint32_t wt[SW];
#pragma unroll
    for (int q = 0; q < SW; ++q) wt[q] = kWeighted ? ((w0 + q < W) ? (uint32_t)wword[w0 + q] : 0u) : 1u;
    // kCls (plan.cpp cls_layout): q = AND of the first m-1 prefix rows, kept while
    // the record says the piece is a sibling of this thread's previous one (flag 1),
    // p = q & the last prefix row, kept for the next piece of the same prefix (flag 2)
    uint4 p[SW / 2], qv[SW / 2];
    for (int g = g0; g < G; g += gstep) {
      // this thread's next piece (after its last one: its first, for the next slab)
      const int gn = g + gstep < G ? g + gstep : g0;
      const int4 na = rec[3 * gn], nb = rec[3 * gn + 1], nc = rec[3 * gn + 2];
      const int n_ext = ra.y & 0xFF, m = (ra.y >> 8) & 0xFF;
      if constexpr (kCls) {
        const int fl = (ra.y >> 17) & 3;
        if (!(fl & 1)) {
          const uint4* r0 = lds4 + (size_t)(ra.z & 0xFFFF) * RS;
#pragma unroll
          for (int q = 0; q < SW / 2; ++q) qv[q] = r0[q];
          and_prefix(qv, 1, m - 1);
        }
        if (!(fl & 2)) {
          // the last prefix id rides in the record's bits 19-31 (a runtime u16_at index
          // would put the record in scratch memory)
          const uint4* rl = lds4 + (size_t)((uint32_t)ra.y >> 19) * RS;
#pragma unroll
          for (int q = 0; q < SW / 2; ++q) {
            const uint4 v = rl[q];
            p[q].x = qv[q].x & v.x; p[q].y = qv[q].y & v.y; p[q].z = qv[q].z & v.z; p[q].w = qv[q].w & v.w;
          }
        }
      } else {
      {
        const uint4* r0 = lds4 + (size_t)(ra.z & 0xFFFF) * RS;
#pragma unroll
        for (int q = 0; q < SW / 2; ++q) p[q] = r0[q];
      }
      if (!((ra.y >> 16) & 1)) {
        and_prefix(p, 1, m);
      } else {
        const int32_t* pr = gpre + rc.x;            // long prefixes (m > 12): ids from the plan's gpre
        int j = 1;
        for (; j + 1 < m; j += 2) and_row2(p, pr[j], pr[j + 1]);
        if (j < m) and_row(p, pr[j]);
      }
      }
      // an all-zero prefix skips its extensions; dense levels (flags & 4: every frequent
      // prefix expects >= 4 rows per slab) skip the test instead (32 VALU ops per piece at SW = 16)
      uint32_t any = flags & 4;
      if (!any) {
#pragma unroll
        for (int q = 0; q < SW / 2; ++q) any |= p[q].x | p[q].y | p[q].z | p[q].w;
      }
      if (any) {
        const int e0 = ra.x;
        // UE extension rows in flight per step (2 x 64 B at SW <= 8; wider rows one at a time)
        constexpr int UE = SW <= 8 ? 2 : 1;
#pragma unroll
        for (int k = 0; k < 8; k += UE) {
          if (k >= n_ext) break;
          uint32_t s[UE];
          const uint4* r[UE];
#pragma unroll
          for (int x = 0; x < UE; ++x) {
            s[x] = 0;
            r[x] = lds4 + (size_t)u16_at(rb, k + x < n_ext ? k + x : k) * RS;
          }
#pragma unroll
          for (int q = 0; q < SW / 2; ++q) {
#pragma unroll
            for (int x = 0; x < UE; ++x) {
              const uint4 v = r[x][q];
              if (kWeighted) {
                s[x] += (uint32_t)(__popc(p[q].x & v.x) + __popc(p[q].y & v.y)) * wt[2 * q] +
                        (uint32_t)(__popc(p[q].z & v.z) + __popc(p[q].w & v.w)) * wt[2 * q + 1];
              } else {
                s[x] = bcnt_acc(p[q].x & v.x, s[x]); s[x] = bcnt_acc(p[q].y & v.y, s[x]);
                s[x] = bcnt_acc(p[q].z & v.z, s[x]); s[x] = bcnt_acc(p[q].w & v.w, s[x]);
              }
            }
          }
#pragma unroll
          for (int x = 0; x < UE; ++x)
            if (k + x < n_ext && s[x]) acc_add(e0 + k + x, s[x]);
        }
      }
      ra = na; rb = nb; rc = nc;
    }
  }
  __syncthreads();
  flush();
}

// ---------------------------------------------------------------------------
// Vertical bitmaps of contiguous rows (no src gather), every rank's row in one LDS
// tile: wave-cooperative like the slab build -- a wave owns one 64-row word of the
// workgroup's WT-word column block, streams the 64 rows' contiguous ranks 64 at a time
// (coalesced, two windows in flight) and ORs each rank's bit into its item's tile row
// (slab_build_word_span).  prep.hip k_build_bitmaps walks one row per lane instead
// (one cache line per lane and load: 7.7 ms per T40I10D100M build).
// ---------------------------------------------------------------------------
struct MapIdent {
  __device__ __forceinline__ int operator()(int r) const { return r; }
};

// 16 waves (the tile allows 2 workgroups per CU): at WT = 8 two waves split each word's
// rows (T40I10D100M full build 12.5 ms at 4 waves, 8.3 at 8)
constexpr int kBwThreads = 1024;

template <class Map>
__global__ __launch_bounds__(kBwThreads) void k_build_bitmaps_w(const int64_t* __restrict__ roff,
                                                         const int32_t* __restrict__ ranks, int64_t ncols, int F1,
                                                         int64_t rs, int64_t bs, int WT, uint64_t* __restrict__ bm,
                                                         Map map) {
  extern __shared__ uint64_t btile[];   // [F1][WT]
  __shared__ unsigned long long bwords[kBwThreads / 64 * 2];
  for (int i = threadIdx.x; i < F1 * WT; i += blockDim.x) btile[i] = 0ull;
  __syncthreads();
  const int wv = threadIdx.x >> 6;
  constexpr int NW = kBwThreads / 64;
  const int nsub = NW > WT ? NW / WT : 1;            // waves per word (WT divides NW or NW divides WT)
  for (int q = wv / nsub; q < WT; q += NW / nsub) {
    const int64_t col0 = ((int64_t)blockIdx.x * WT + q) * 64;
    if (col0 < ncols)
      slab_build_word_span(btile, WT, q, word_span(roff, col0, ncols), ranks, map, wv % nsub, nsub, bwords + wv * 2,
                           0);
  }
  __syncthreads();
  const int64_t w0 = (int64_t)blockIdx.x * WT;
  for (int i = threadIdx.x; i < F1 * WT; i += blockDim.x) {
    const int u = i / WT, w = i - u * WT;
    bm[((w0 + w) >> 3) * bs + (int64_t)u * rs + ((w0 + w) & 7)] = btile[i];
  }
}

}  // namespace fa

using namespace fa;

// Contiguous rows, all F1 output rows in one tile (F1 * WT * 8 B of LDS): the wave
// build above.  Returns 2 when it does not apply (the caller's thread-per-row kernel).
// blocked: the 8-word block layout (BmView; Wp a multiple of 8).
FA_API int fa_hip_build_bitmaps_wave(const int64_t* roff, const int32_t* ranks, int64_t ncols, int32_t F1, int64_t Wp,
                                     int WT, uint64_t* bm, const int32_t* item_map, int blocked, hipStream_t st) {
  const size_t lds = (size_t)F1 * WT * 8;
  if (F1 <= 0 || WT <= 0 || Wp % WT || Wp % 8 || lds > 64 * 1024) return 2;
  const int64_t rs = blocked ? 8 : Wp, bs = blocked ? 8 * (int64_t)F1 : 8;
  dim3 g((unsigned)(Wp / WT));
  if (item_map) {
    (void)hipFuncSetAttribute((const void*)k_build_bitmaps_w<MapGlobal>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL(k_build_bitmaps_w<MapGlobal>, g, dim3(kBwThreads), lds, st, roff, ranks, ncols, F1, rs, bs, WT, bm,
                       MapGlobal{item_map});
  } else {
    (void)hipFuncSetAttribute((const void*)k_build_bitmaps_w<MapIdent>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL(k_build_bitmaps_w<MapIdent>, g, dim3(kBwThreads), lds, st, roff, ranks, ncols, F1, rs, bs, WT, bm,
                       MapIdent{});
  }
  FA_LAUNCH_RET();
}

// Flattened pairs in every staged tile (k_pair_queue16): measured against flattening only
// the off-diagonal tiles, only the diagonal ones and none (T10I4D100M pair call, square-root
// decode of the diagonal tiles: 13.9 / 13.7 / 14.8 / 14.5 ms; with the triangular decode
// table PairRowsLds::tri the all-tiles form won the headline A/B, 45.5-46.3 vs 47.1-47.3 ms).

// Gram of words [0, W) of the bitmap view (bm, rs, bs, woff: BmView) on the matrix
// cores, every count multiplied by scale before it is added to out (a weight class of
// a deduplicated layout: its columns all carry the same weight, FastApriori.scala:233-235).
FA_API int fa_hip_pair_gram_mfma(const uint64_t* bm, int32_t F1, int64_t rs, int64_t bs, int woff, int64_t W,
                                 uint32_t* out, int target_wgs, uint32_t scale, int fp4, hipStream_t st) {
  if (woff < 0 || woff > 7) return -22;
  const BmView v{bm, rs, bs, woff};
  if (W <= 0 || F1 < 2) return 0;
  const int nt = (F1 + kMT4 - 1) / kMT4;
  const int ntp = nt * (nt + 1) / 2;
  int64_t nk = std::max<int64_t>(1, (target_wgs + ntp - 1) / ntp);
  int64_t kchunk = (W + nk - 1) / nk;
  kchunk = std::max<int64_t>(kMW, (kchunk + kMW - 1) / kMW * kMW);
  // fp4: the FP4 form (T40I10D100M pair phase 68 -> 46 ms); 0: the i8 form (a test oracle)
  if (fp4) kchunk = std::min<int64_t>(kchunk, (int64_t)1 << 18);   // f32-exact sums: <= 2^24 transactions
  nk = (W + kchunk - 1) / kchunk;
  if (fp4)
    hipLaunchKernelGGL(k_pair_gram_fp4, dim3((unsigned)(nk * ntp)), dim3(256), 0, st, v, F1, W, nt,
                       ntp, kchunk, out, scale);
  else
    hipLaunchKernelGGL(k_pair_gram_mfma4<false>, dim3((unsigned)(nk * ntp)), dim3(256), 0, st, v, F1, W, nt,
                       ntp, kchunk, out, scale);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_pair_gram_popc(const uint64_t* bm, int32_t F1, int64_t rs, int64_t bs, int woff, int64_t W,
                                 const int32_t* wword, uint32_t* out, int target_wgs, hipStream_t st) {
  if (woff < 0 || woff > 7) return -22;
  if (W <= 0 || F1 < 2) return 0;
  const BmView v{bm, rs, bs, woff};
  const int nt = (F1 + kGT - 1) / kGT;
  const int ntp = nt * (nt + 1) / 2;
  int64_t nk = std::max<int64_t>(1, (target_wgs + ntp - 1) / ntp);
  int64_t kchunk = (W + nk - 1) / nk;
  kchunk = std::max<int64_t>(kGK, (kchunk + kGK - 1) / kGK * kGK);
  nk = (W + kchunk - 1) / kchunk;
  dim3 g((unsigned)(nk * ntp));
  if (wword)
    hipLaunchKernelGGL(k_pair_gram_popc<true>, g, dim3(256), 0, st, v, F1, W, wword, nt, ntp, kchunk, out);
  else
    hipLaunchKernelGGL(k_pair_gram_popc<false>, g, dim3(256), 0, st, v, F1, W, wword, nt, ntp, kchunk, out);
  FA_LAUNCH_RET();
}

// gb_start: ngb+1 group boundaries; every block must hold <= 1024 extensions.
FA_API int fa_hip_count_candidates(const uint64_t* bm, int64_t Wp, int64_t W, const int32_t* prefix,
                                   int m, const int64_t* ext_off, const int32_t* ext,
                                   const int32_t* gb_start, int ngb, const int32_t* wword,
                                   uint32_t* out, hipStream_t st) {
  if (ngb <= 0 || W <= 0) return 0;
  const int64_t nsc = (W + 256 * kWPT - 1) / (256 * kWPT);
  dim3 g((unsigned)(nsc * ngb));
  if (wword)
    hipLaunchKernelGGL(k_count_candidates<true>, g, dim3(256), 0, st, bm, Wp, W, prefix, m, ext_off, ext, gb_start, ngb, wword, out);
  else
    hipLaunchKernelGGL(k_count_candidates<false>, g, dim3(256), 0, st, bm, Wp, W, prefix, m, ext_off, ext, gb_start, ngb, wword, out);
  FA_LAUNCH_RET();
}

// ---------------------------------------------------------------------------
// A window's own rows, in the bitmap domain (FastApriori._window_rows): a window of a
// window-by-window level counts k-candidates over its items U only, so only the rows
// holding >= k of U matter.  k_win_alive: per 64-row word q of the level's bitmap, the
// mask of rows with >= k bits among U's bitmap rows (a bit-sliced counter: one plane per
// count bit, ripple-carry adds) and its popcount.  k_win_compact: every U row's words
// compressed to the alive rows (software PEXT, Hacker's Delight 7-4, with the six move
// masks of the word's alive mask computed once for all of U) and written at the alive
// rows' running bit offset: one wave per 64 words assembles its output span in LDS,
// stores the words inside it and ORs the two it shares with its neighbours.  The result
// is a row-major bitmap of U over the alive rows only -- no pass over the transaction
// rows, no trimmed copy of them.
// bm element (bitmap row r, word q): ld > 0 row-major (row stride ld), ld < 0 the 8-word
// blocked layout of block stride -ld (slab_copy_bm).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t bm_word(const uint64_t* __restrict__ bm, int64_t ld, int64_t r, int64_t q) {
  return ld > 0 ? bm[r * ld + q] : bm[(q >> 3) * -ld + r * 8 + (q & 7)];
}

constexpr int kWinPlanes = 11;   // counts up to 2047 items
constexpr int kWinAhead = 8;     // item words loaded ahead (k_win_alive)
constexpr int kWinBatch = 8;     // items per LDS round (k_win_compact)

__global__ __launch_bounds__(256) void k_win_alive(const uint64_t* __restrict__ bm, int64_t ld,
                                                   const int32_t* __restrict__ rows, int n_items, int64_t W, int k,
                                                   int planes, uint64_t* __restrict__ alive, int32_t* __restrict__ cnt) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= W) return;
  uint64_t pl[kWinPlanes];
#pragma unroll
  for (int p = 0; p < kWinPlanes; ++p) pl[p] = 0ull;
  // kWinAhead item words in flight per thread (one at a time left the kernel waiting on
  // HBM latency: ~355 us per T40I10D100M window)
  uint64_t nx[kWinAhead];
#pragma unroll
  for (int j = 0; j < kWinAhead; ++j) nx[j] = j < n_items ? bm_word(bm, ld, rows[j], q) : 0ull;
  for (int u0 = 0; u0 < n_items; u0 += kWinAhead) {
#pragma unroll
    for (int j = 0; j < kWinAhead; ++j) {
      uint64_t c = nx[j];
      const int un = u0 + kWinAhead + j;
      nx[j] = un < n_items ? bm_word(bm, ld, rows[un], q) : 0ull;
#pragma unroll
      for (int p = 0; p < kWinPlanes; ++p) {
        if (p >= planes) break;
        const uint64_t t = pl[p] & c;
        pl[p] ^= c;
        c = t;
      }
    }
  }
  // count >= k, bit-sliced, from the top plane down
  uint64_t gt = 0ull, eq = ~0ull;
#pragma unroll
  for (int p = kWinPlanes - 1; p >= 0; --p) {
    if (p >= planes) continue;
    if ((k >> p) & 1) {
      eq &= pl[p];
    } else {
      gt |= eq & pl[p];
      eq &= ~pl[p];
    }
  }
  const uint64_t a = (k >> planes) ? 0ull : (gt | eq);
  alive[q] = a;
  cnt[q] = __popcll(a);
}

__global__ __launch_bounds__(256) void k_win_compact(const uint64_t* __restrict__ bm, int64_t ld,
                                                     const int32_t* __restrict__ rows, int n_items, int64_t W,
                                                     const uint64_t* __restrict__ alive,
                                                     const int64_t* __restrict__ off, uint64_t* __restrict__ out,
                                                     int64_t ldo) {
  // four independent waves per workgroup, each with its own buffers and only wave-level
  // LDS ordering (wave_lds_sync): a __syncthreads fence drains the wave's outstanding
  // stores and loads (s_waitcnt vmcnt(0)) at every round
  __shared__ unsigned long long bufs[4][kWinBatch][66];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long (&buf)[kWinBatch][66] = bufs[wv];
  const int64_t q0 = ((int64_t)blockIdx.x * 4 + wv) * 64, q = q0 + lane;
  if (q0 >= W) return;
  const int64_t qe = min(W, q0 + 64) - 1;                 // the wave's last word
  const uint64_t m0 = q < W ? alive[q] : 0ull;
  const int n = __popcll(m0);
  const int64_t base = off[q0];                            // the wave's first output bit
  const int64_t end = off[qe] + __popcll(alive[qe]);      // one past its last
  if (end == base) return;                                 // (uniform: no alive row in these words)
  const int s = (int)(base & 63) + (q < W ? (int)(off[q] - base) : 0);
  const int nwords = (int)(((base & 63) + (end - base) + 63) >> 6);
  const int64_t w0 = base >> 6;
  // the six move masks of m0 (compress, Hacker's Delight 7-4)
  uint64_t mv[6];
  {
    uint64_t m = m0, mk = ~m0 << 1;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      uint64_t mp = mk ^ (mk << 1);
      mp ^= mp << 2; mp ^= mp << 4; mp ^= mp << 8; mp ^= mp << 16; mp ^= mp << 32;
      mv[i] = mp & m;
      m = (m ^ mv[i]) | (mv[i] >> (1 << i));
      mk &= ~mp;
    }
  }
  // kWinBatch items per round: their words loaded together, one LDS buffer each
  for (int u0 = 0; u0 < n_items; u0 += kWinBatch) {
    const int nb = min(kWinBatch, n_items - u0);
    uint64_t x[kWinBatch];
#pragma unroll
    for (int b = 0; b < kWinBatch; ++b) x[b] = (n && b < nb) ? bm_word(bm, ld, rows[u0 + b], q) : 0ull;
    for (int i = lane; i < nb * 66; i += 64) (&buf[0][0])[i] = 0ull;
    wave_lds_sync();
    if (n) {
      const int w = s >> 6, sh = s & 63;
#pragma unroll
      for (int b = 0; b < kWinBatch; ++b) {
        if (b >= nb) break;
        uint64_t y = x[b] & m0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const uint64_t t = y & mv[i];
          y = (y ^ t) | (t >> (1 << i));
        }
        atomicOr(&buf[b][w], (unsigned long long)(y << sh));
        if (sh + n > 64) atomicOr(&buf[b][w + 1], (unsigned long long)(y >> (64 - sh)));
      }
    }
    wave_lds_sync();
    for (int b = 0; b < nb; ++b) {
      const int64_t u = u0 + b;
      for (int j = lane; j < nwords; j += 64) {
        const unsigned long long v = buf[b][j];
        const int64_t gw = w0 + j;
        uint64_t* o = ldo > 0 ? out + u * ldo + gw : out + (gw >> 3) * -ldo + u * 8 + (gw & 7);
        if (j == 0 || j == nwords - 1) {
          if (v) atomicOr(reinterpret_cast<unsigned long long*>(o), v);   // shared with a neighbour wave
        } else {
          *o = v;
        }
      }
    }
    wave_lds_sync();                                     // (the buffers are cleared next round)
  }
}

FA_API int fa_hip_win_alive(const uint64_t* bm, int64_t ld, const int32_t* rows, int n_items, int64_t W, int k,
                            uint64_t* alive, int32_t* cnt, hipStream_t st) {
  if (W <= 0) return 0;
  int planes = 1;
  while ((1 << planes) <= n_items) ++planes;
  if (n_items < 1 || planes > kWinPlanes || k < 1 || ld == 0) return 1;
  hipLaunchKernelGGL(k_win_alive, dim3((unsigned)((W + 255) / 256)), dim3(256), 0, st, bm, ld, rows, n_items, W, k,
                     planes, alive, cnt);
  FA_LAUNCH_RET();
}

// out: zeroed, row-major [n_items][ldo] words (ldo >= ceil(K / 64)), or ldo < 0: the 8-word
// blocked layout [Wp / 8][n_items][8] (ldo = -8 n_items; what the slab copies stream best);
// off: exclusive prefix of k_win_alive's counts [W]
FA_API int fa_hip_win_compact(const uint64_t* bm, int64_t ld, const int32_t* rows, int n_items, int64_t W,
                              const uint64_t* alive, const int64_t* off, uint64_t* out, int64_t ldo, hipStream_t st) {
  if (W <= 0 || n_items < 1) return 0;
  if (ld == 0 || ldo == 0) return 1;
  hipLaunchKernelGGL(k_win_compact, dim3((unsigned)((W + 255) / 256)), dim3(256), 0, st, bm, ld, rows, n_items, W,
                     alive, off, out, ldo);
  FA_LAUNCH_RET();
}

// Slab counting from piece records (k_count_slab_rec; records: plan.cpp, 3 x int4
// per piece).  LDS: slab + accumulator (16-B aligned) + u16 map when F1 <= 8192
// and the slab is built from contiguous rows.  Returns 3 when that exceeds the LDS.
// g_dev (optional): the piece count read by the kernel from device memory (G is then
// ignored; device-planned bundles, levels.hip fa_hip_dl_plan).
// cls bit 0: the records carry class-layout flags (plan.cpp cls_layout): unit weights
// run k_count_slab_rec<.., kCls> (the flags are hints: the plain kernel ignores them and
// recomputes every prefix, with the same counts).  cls bit 1: dense level, no
// all-zero-prefix test (the counts are the same either way).  cls bit 2: u16 packed
// accumulators (unit weights: half the LDS per candidate, drained every 65535 / (SW * 64)
// slabs).
// Test hook: at most this many workgroups per slab count (0: no cap).  One workgroup
// then walks every slab, so the packed-u16 accumulators' mid-run drain (every
// kFlush16 slabs) runs on inputs of a few hundred thousand rows.
static int g_slab_max_wg = 0;
FA_API void fa_hip_debug_slab_max_wg(int n) { g_slab_max_wg = n; }
// Candidate distribution of the slab counts launched next (fastapriori_amd
// FastApriori._piece_part with --strategy candidate): this rank counts the 64-piece
// chunks part, part + nparts, ... (k_count_slab_rec flags bits 8-23); (0, 1): every piece.
static int g_piece_part = 0, g_piece_nparts = 1;
FA_API int fa_hip_set_piece_part(int part, int nparts) {
  if (nparts < 1 || nparts > 256 || part < 0 || part >= nparts) return 1;
  g_piece_part = part;
  g_piece_nparts = nparts;
  return 0;
}

FA_API int fa_hip_count_slab_rec_cls(const int64_t* roff, const int32_t* ranks, const int32_t* src, int64_t ncols,
                                     const int32_t* item_map, int F1, int n_used, const int32_t* gpre,
                                     const void* rec, int G, int C, const int32_t* wword, uint32_t* out, int sw,
                                     int n_wg, const uint64_t* bm, int64_t Wp, hipStream_t st,
                                     const int32_t* bm_rows, const int32_t* g_dev, int cls) {
  if ((G <= 0 && !g_dev) || C <= 0 || ncols <= 0) return 0;
  // the class-layout flags name a thread's previous piece in the undivided plan: with the
  // pieces divided among ranks the plain kernel recomputes every prefix instead
  if (g_piece_nparts > 1) cls &= ~1;
  const bool acc16 = (cls & 4) && !wword;   // two u16 counters per accumulator word
  const int64_t n_acc = acc16 ? (C + 1) / 2 : C;
  const bool contig = !bm && !src;
  const size_t map_b = (contig && F1 <= kMapLdsMax) ? (size_t)(((int64_t)F1 * 2 + 15) & ~(int64_t)15) : 0;
  const size_t lds = (size_t)n_used * (sw + 2) * 8 + (size_t)((n_acc + 3) & ~(int64_t)3) * 4 + map_b;
  if (lds > 160 * 1024 - 256) return 3;             // static build_words scratch
  if (g_slab_max_wg > 0) n_wg = std::min(n_wg, g_slab_max_wg);
  using KernT = void (*)(const int64_t*, const int32_t*, const int32_t*, int64_t, const int32_t*, int, int,
                         const int32_t*, const int4*, int, int, const int32_t*, uint32_t*, const uint64_t*, int64_t,
                         const int32_t*, int, const int32_t*);
  KernT kern = nullptr;
#define FA_REC_MODE(S, B)                                                                              \
  kern = wword ? (KernT)k_count_slab_rec<S, true, B>                                                   \
         : (cls & 1) ? (acc16 ? (KernT)k_count_slab_rec<S, false, B, true, true>                       \
                              : (KernT)k_count_slab_rec<S, false, B, true, false>)                      \
                     : (acc16 ? (KernT)k_count_slab_rec<S, false, B, false, true>                      \
                              : (KernT)k_count_slab_rec<S, false, B, false, false>);
#define FA_REC_CASE(S)                                    \
  if (sw == S) {                                          \
    if (bm) { FA_REC_MODE(S, kBuildBM) }                  \
    else if (src) { FA_REC_MODE(S, kBuildCols) }          \
    else { FA_REC_MODE(S, kBuildContig) }                 \
  }
  FA_REC_CASE(4)
  FA_REC_CASE(8)
  FA_REC_CASE(16)
  FA_REC_CASE(32)
#undef FA_REC_CASE
#undef FA_REC_MODE
  if (!kern) return 1;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int flags = ((cls & 2) ? 4 : 0) | (acc16 ? 8 : 0) | (g_piece_part << 8) | ((g_piece_nparts - 1) << 16);
  hipLaunchKernelGGL(kern, dim3((unsigned)n_wg), dim3(kSlabThreads), lds, st, roff, ranks, src, ncols, item_map, F1,
                     n_used, gpre, (const int4*)rec, G, C, wword, out, bm, Wp, bm_rows, flags, g_dev);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_count_slab_rec(const int64_t* roff, const int32_t* ranks, const int32_t* src, int64_t ncols,
                                 const int32_t* item_map, int F1, int n_used, const int32_t* gpre, const void* rec,
                                 int G, int C, const int32_t* wword, uint32_t* out, int sw, int n_wg,
                                 const uint64_t* bm, int64_t Wp, hipStream_t st, const int32_t* bm_rows,
                                 const int32_t* g_dev) {
  return fa_hip_count_slab_rec_cls(roff, ranks, src, ncols, item_map, F1, n_used, gpre, rec, G, C, wword, out, sw,
                                   n_wg, bm, Wp, st, bm_rows, g_dev, 0);
}

FA_API int fa_hip_block_counts(const int64_t* roff, const int32_t* ranks, int64_t T, int32_t F1, uint8_t* cnt,
                               int64_t* bsum, int pb, hipStream_t st) {
  if (T <= 0) return 0;
  const int nb = (F1 + pb - 1) / pb;
  const int64_t nbatch = (T + 63) / 64;
  const int lpb = __builtin_ctz((unsigned)pb);
  if (nb <= kWBMaxNB && (1 << lpb) == pb)
    hipLaunchKernelGGL(k_block_counts_w, dim3((unsigned)((nbatch + 3) / 4)), dim3(256), 0, st, roff, ranks, T, nb,
                       cnt, bsum, nbatch, lpb);
  else
    hipLaunchKernelGGL(k_block_counts, dim3((unsigned)((nbatch + 3) / 4)), dim3(256), 0, st, roff, ranks, T, nb, cnt,
                       bsum, nbatch, pb);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_block_scatter(const int64_t* roff, const int32_t* ranks, int64_t T, int32_t F1,
                                const uint8_t* cnt, const int64_t* base, uint8_t* lr, int pb, hipStream_t st) {
  if (T <= 0) return 0;
  const int nb = (F1 + pb - 1) / pb;
  const int64_t nbatch = (T + 63) / 64;
  const int lpb = __builtin_ctz((unsigned)pb);
  if (nb <= kWBMaxNB && (1 << lpb) == pb)
    hipLaunchKernelGGL(k_block_scatter_w, dim3((unsigned)((nbatch + 3) / 4)), dim3(256), 0, st, roff, ranks, T, nb,
                       cnt, base, nbatch, lr, lpb);
  else
    hipLaunchKernelGGL(k_block_scatter, dim3((unsigned)((nbatch + 3) / 4)), dim3(256), 0, st, roff, ranks, T, nb, cnt,
                       base, nbatch, lr, pb);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_pair_blocked(const uint8_t* cnt, const int64_t* base, const uint8_t* lr, int64_t T,
                               const int32_t* wrow, int32_t F1, uint32_t* out, int64_t chunk_rows, hipStream_t st) {
  if (T <= 0 || F1 < 2) return 0;
  const int nb = (F1 + kPB - 1) / kPB;
  const int nbp = nb * (nb + 1) / 2;
  const int64_t nbatch = (T + 63) / 64;
  const int64_t chunk_b = std::max<int64_t>(kPW, (chunk_rows + 63) / 64);
  const int64_t nch = (nbatch + chunk_b - 1) / chunk_b;
  hipLaunchKernelGGL(k_pair_blocked, dim3((unsigned)(nch * nbp)), dim3(64 * kPW), 0, st, cnt, base, lr, T, nbatch,
                     wrow, F1, nb, nbp, chunk_b, out);
  FA_LAUNCH_RET();
}

// Work-queue schedule (k_pair_queue16): qctr = nbp zeroed ints, out has row stride ld.
FA_API int fa_hip_pair_queue16(const uint8_t* cnt, const int64_t* base, const uint8_t* lr, int64_t T, int32_t F1,
                               int64_t ld, int* qctr, uint32_t* out, int n_wg, hipStream_t st) {
  if (T <= 0 || F1 < 2) return 0;
  const int nb = (F1 + kPB16 - 1) / kPB16;
  const int nbp = nb * (nb + 1) / 2;
  const int64_t nbatch = (T + 63) / 64;
  const int nsub = (int)((nbatch + kQSubB - 1) / kQSubB);
  if (n_wg <= 0) {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    n_wg = ncu;
  }
  n_wg = (int)std::min<int64_t>(n_wg, (int64_t)nsub * nbp);
  hipLaunchKernelGGL(k_pair_queue16, dim3((unsigned)n_wg), dim3(64 * kPW), 0, st, cnt, base, lr, T, nbatch, F1, ld,
                     nb, nbp, qctr, nsub, out);
  FA_LAUNCH_RET();
}

// F_2 of the pair counts (matrix with row stride ld, or the flat triangle when ld < 0):
// rows int32 [|F_2|][2], cnt int32 [|F_2|] in triangle order, |F_2| into n_out (device
// int64); row_cnt int32 [F1] and row_off int64 [F1] scratch.
FA_API int fa_hip_pairs_compact(const uint32_t* pc, int64_t ld, int32_t F1, int64_t mc, int32_t* row_cnt,
                                int64_t* row_off, int32_t* rows, int32_t* cnt, int64_t* n_out, hipStream_t st) {
  if (F1 < 2) return 1;
  hipLaunchKernelGGL(k_pairs_keep_count, dim3((unsigned)F1), dim3(256), 0, st, pc, ld, F1, mc, row_cnt);
  hipLaunchKernelGGL(k_pairs_scan, dim3(1), dim3(1024), 0, st, row_cnt, F1, row_off, n_out);
  hipLaunchKernelGGL(k_pairs_emit, dim3((unsigned)F1), dim3(256), 0, st, pc, ld, F1, mc, row_off, rows, cnt);
  FA_LAUNCH_RET();
}
