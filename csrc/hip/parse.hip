// Device-side parsing of a transaction file's bytes (numeric and dictionary vocabularies).
//
// Same input semantics as the host parser (csrc/host/parse.cpp, Utils.scala:19-27):
//   * lines end at '\n', at '\r\n' or at a lone '\r' (Hadoop LineRecordReader);
//   * each line -> trim() (bytes <= 0x20) -> split on [ \t\x0B\f]+; a blank line
//     is the single token "" (id 0);
//   * numeric ids: id = value + 1 for canonical decimals "0" | [1-9][0-9]* with
//     value <= 2^31 - 2; any other token raises the `bad` flag and the caller
//     re-parses the shard on the host (dictionary mode);
//   * ids inside one line are distinct, in first-occurrence order; every
//     repeated occurrence goes to `extras` (F1 counts occurrences).
//
// Pipeline (the file's bytes are already in HBM, padded to 64 + a multiple of 64):
//   k_line_count  16 KB tiles, 64 bytes per thread (4 x 16-byte loads): line ends per tile
//   k_line_ends   same tiles; block scan of per-thread counts -> position of every line end
//   (numeric ids: the tile parser below; dictionary ids: k_parse_lines_dict, then
//   k_compact_lines, one thread per line copying ids and extras to their offsets)
#include "fa_hip.h"

namespace fa {

constexpr int kLT = 256;              // threads per line-scan block
constexpr int kLB = 64;               // bytes per thread
constexpr int kLTile = kLT * kLB;     // 16 KB
constexpr int kPT = 128;              // threads per parse block
constexpr int kSeen = 64;             // distinct ids kept in LDS per thread

__device__ __forceinline__ bool is_term_at(const uint8_t* __restrict__ buf, int64_t n, int64_t i, uint32_t c) {
  return c == '\n' || (c == '\r' && (i + 1 >= n || buf[i + 1] != '\n'));
}

// Line ends among this thread's 64 bytes: count (mode 0) or write (mode 1).
template <int MODE>
__device__ __forceinline__ int scan_bytes(const uint8_t* __restrict__ buf, int64_t n, int64_t base,
                                          int64_t* __restrict__ out, int64_t lo = 0) {
  int cnt = 0;
  if (base >= n) return 0;
  const uint4* p = reinterpret_cast<const uint4*>(buf + base);
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const uint4 w = p[v];
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t x = ws[q];
      // any '\n' (0x0a) or '\r' (0x0d) byte in this dword?  (zero-byte test on x ^ pattern)
      const uint32_t a = x ^ 0x0a0a0a0au, b = x ^ 0x0d0d0d0du;
      const uint32_t za = (a - 0x01010101u) & ~a & 0x80808080u;
      const uint32_t zb = (b - 0x01010101u) & ~b & 0x80808080u;
      if (!(za | zb)) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t i = base + v * 16 + q * 4 + k;
        const uint32_t c = (x >> (8 * k)) & 0xffu;
        if (i >= lo && i < n && is_term_at(buf, n, i, c)) {
          if (MODE == 1) out[cnt] = i;
          ++cnt;
        }
      }
    }
  }
  return cnt;
}

__global__ __launch_bounds__(kLT) void k_line_count(const uint8_t* __restrict__ buf, int64_t n,
                                                    int32_t* __restrict__ tile_cnt) {
  __shared__ int part[kLT / kWave];
  const int64_t base = (int64_t)blockIdx.x * kLTile + (int64_t)threadIdx.x * kLB;
  const uint32_t c = wave_sum_u32((uint32_t)scan_bytes<0>(buf, n, base, nullptr));
  if (lane_id() == 0) part[threadIdx.x >> 6] = (int)c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kLT / kWave; ++w) t += part[w];
    tile_cnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kLT) void k_line_ends(const uint8_t* __restrict__ buf, int64_t n,
                                                   const int64_t* __restrict__ tile_base,
                                                   int64_t* __restrict__ ends) {
  __shared__ int part[kLT / kWave];
  const int64_t base = (int64_t)blockIdx.x * kLTile + (int64_t)threadIdx.x * kLB;
  const int mine = scan_bytes<0>(buf, n, base, nullptr);
  const int incl = wave_scan_incl_dpp(mine);
  if (lane_id() == 63) part[threadIdx.x >> 6] = incl;
  __syncthreads();
  int before = 0;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) before += part[w];
  if (mine) scan_bytes<1>(buf, n, base, ends + tile_base[blockIdx.x] + before + incl - mine);
}

__global__ __launch_bounds__(256) void k_compact_lines(
    const int32_t* __restrict__ scratch, const int32_t* __restrict__ xscratch, const int64_t* __restrict__ bound_off,
    const int32_t* __restrict__ dcnt, const int32_t* __restrict__ xcnt, const int64_t* __restrict__ off,
    const int64_t* __restrict__ xoff, int64_t nl, int32_t* __restrict__ items, int32_t* __restrict__ extras) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= nl) return;
  const int64_t bo = bound_off[j];
  const int32_t d = dcnt[j], x = xcnt[j];
  int32_t* dst = items + off[j];
  for (int q = 0; q < d; ++q) dst[q] = scratch[bo + q];
  if (x) {
    int32_t* xd = extras + xoff[j];
    for (int q = 0; q < x; ++q) xd[q] = xscratch[bo + q];
  }
}

// ---------------------------------------------------------------------------
// Tile parser of numeric lines (the default path).  A region [lo, hi) of the
// shard's bytes in HBM (lo a line start; hi just after a terminator, or the shard
// end) is cut into 16 KB tiles from a = lo & ~63; k_tline_count counts each
// tile's line ends and the caller scans them into tile_base.
//   k_tparse   one workgroup per tile stages the tile, kHalo bytes before it and
//              64 after it in LDS with coalesced 16-byte loads.  Each thread
//              takes the lines that END in its 64 bytes (the previous line end
//              from a block max-scan, or found in the halo), parses them from
//              LDS a dword at a time and writes each line's distinct ids to its
//              own slots of scratch at (line start - sbase) / 2: tokens are
//              separated, so a line of len bytes holds <= (len + 1) / 2 of them
//              and the slots of consecutive lines never overlap.  Repeats go to
//              xscratch; dcnt / xcnt / slot base (-1: blank line = the single
//              token "") per line.  Duplicates inside a line: a 128-bit filter of
//              the ids seen; only on a filter hit are the first kSeenT ids (LDS
//              column) and the rest (scratch) compared.  Lines longer than the
//              halo read their bytes from HBM.
//   k_tcompact one wave per 64 lines copies their ids to the scanned offsets
//              (items flattened over the lanes: coalesced stores) and counts
//              every id, repeats included (F1 counts occurrences, FastApriori
//              .scala:55), into an LDS histogram of kHistCap bins, added into
//              the block's own row of hpart (no atomics; rows summed once by
//              k_hist_reduce).  An id >= kHistCap sets flags[2]: the caller's
//              histogram pass runs instead.  Repeats beyond the caller's xcap set
//              flags[3] (the caller parses again with room for all of them).
// The old thread-per-line kernel read every byte with a dependent global load
// (62 ms for the 3.9 GB T10I4D100M file on MI355X); these read HBM coalesced.
// ---------------------------------------------------------------------------
constexpr int kTT = kLT;
constexpr int kTBy = kLB;
constexpr int kTTile = kTT * kTBy;       // = kLTile: k_tline_count uses the same tiles
constexpr int kHalo = 2048;
constexpr int kTLds = kHalo + kTTile + 64;
constexpr int kSeenT = 16;
constexpr int kHistCap = 8192;

__global__ __launch_bounds__(kLT) void k_tline_count(const uint8_t* __restrict__ buf, int64_t a, int64_t lo,
                                                     int64_t hi, int32_t* __restrict__ tile_cnt) {
  __shared__ int part[kLT / kWave];
  const int64_t base = a + (int64_t)blockIdx.x * kLTile + (int64_t)threadIdx.x * kLB;
  const uint32_t c = wave_sum_u32((uint32_t)scan_bytes<0>(buf, hi, base, nullptr, lo));
  if (lane_id() == 0) part[threadIdx.x >> 6] = (int)c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kLT / kWave; ++w) t += part[w];
    tile_cnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kTT) void k_tparse(const uint8_t* __restrict__ buf, int64_t buf_len, int64_t a,
                                                int64_t lo, int64_t hi, int tail, int64_t sbase,
                                                const int64_t* __restrict__ tile_base, int32_t* __restrict__ dcnt,
                                                int32_t* __restrict__ xcnt, int64_t* __restrict__ lbase,
                                                int32_t* __restrict__ scratch, int32_t* __restrict__ xscratch,
                                                int32_t* __restrict__ tile_dx, int32_t* __restrict__ flags) {
  // The tile image in LDS: file byte o (relative to l0) in dword (o >> 2) + (o >> 6).
  // One dword of padding per 64 bytes: the threads' 64-byte chunks (and the lines they
  // parse, lock-stepped at similar offsets) then fall on different banks; unpadded,
  // a 64-byte stride puts all 32 lanes of a ds_read_b32 half on 2 banks (16-way).
  __shared__ uint32_t sw[kTLds / 4 + kTLds / 64 + 1];
  __shared__ int32_t seen[kSeenT * kTT];      // column per thread: conflict-free
  __shared__ int wsum[kTT / kWave];
  __shared__ long long wmax[kTT / kWave];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t t0 = a + (int64_t)blockIdx.x * kTTile;
  const int64_t l0 = t0 - kHalo;               // LDS byte 0 is file byte l0 (16-byte aligned)
  for (int q = tid; q < kTLds / 16; q += kTT) {
    const int64_t p = l0 + 16 * (int64_t)q;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (p >= 0 && p + 16 <= buf_len) v = *reinterpret_cast<const uint4*>(buf + p);
    uint32_t* d = sw + 4 * q + (q >> 2);       // a 16-byte piece never straddles a 64-byte chunk
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  auto lds_dw = [&](int64_t o) -> uint32_t { return sw[(o >> 2) + (o >> 6)]; };
  auto lds_b = [&](int64_t o) -> uint32_t { return (lds_dw(o) >> (8 * (o & 3))) & 0xffu; };
  // line ends among this thread's bytes [c0, c0 + 64) that lie in [lo, hi)
  const int64_t c0 = t0 + (int64_t)tid * kTBy;
  unsigned long long M = 0ull;
  {
    const int lb0 = kHalo + tid * kTBy;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t x = lds_dw(lb0 + 16 * v + 4 * q);
        const uint32_t xa = x ^ 0x0a0a0a0au, xb = x ^ 0x0d0d0d0du;
        const uint32_t za = (xa - 0x01010101u) & ~xa & 0x80808080u;
        const uint32_t zb = (xb - 0x01010101u) & ~xb & 0x80808080u;
        if (!(za | zb)) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int o = v * 16 + q * 4 + k;
          const int64_t i = c0 + o;
          const uint32_t c = (x >> (8 * k)) & 0xffu;
          const bool t = c == '\n' || (c == '\r' && (i + 1 >= hi || lds_b(lb0 + o + 1) != '\n'));
          if (t && i >= lo && i < hi) M |= 1ull << o;
        }
      }
    }
  }
  // the shard's last line has no terminator: it ends at hi
  const int64_t lastb = hi - 1;
  const bool has_tail = tail && lastb >= lo && lastb >= c0 && lastb < c0 + kTBy && !((M >> (lastb - c0)) & 1ull);
  const int cnt = __popcll(M) + (has_tail ? 1 : 0);
  const int incl = wave_scan_incl_dpp(cnt);
  long long m = M ? (long long)(c0 + 63 - __clzll(M)) : -1ll;     // last line end of this thread
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(m, (unsigned)o, 64);
    if (lane >= o) m = t > m ? t : m;
  }
  if (lane == 63) { wsum[wv] = incl; wmax[wv] = m; }
  __syncthreads();
  int before = 0;
  long long pm = __shfl_up(m, 1u, 64);
  if (lane == 0) pm = -1;
  for (int w = 0; w < wv; ++w) {
    before += wsum[w];
    pm = wmax[w] > pm ? wmax[w] : pm;
  }
  bool bad = false;
  int32_t mx = 0;
  int dsum = 0, xsum = 0;                      // ids and repeats of this thread's lines
  if (cnt > 0) {
    int64_t g = tile_base[blockIdx.x] + before + incl - cnt;     // this thread's first line
    int64_t s0;
    if (pm >= 0) {
      s0 = pm + 1;
    } else {
      // the previous line end is in the halo, before lo (s0 = lo), or further back in HBM
      s0 = -1;
      const int64_t stop = lo > l0 ? lo : l0;
      for (int64_t p = t0 - 1; p >= stop; --p) {
        const uint32_t c = lds_b(p - l0);
        if (c == '\n' || (c == '\r' && lds_b(p + 1 - l0) != '\n')) { s0 = p + 1; break; }
      }
      if (s0 < 0 && lo < l0) {
        for (int64_t p = l0 - 1; p >= lo; --p) {
          const uint32_t c = buf[p];
          if (c == '\n' || (c == '\r' && buf[p + 1] != '\n')) { s0 = p + 1; break; }
        }
      }
      if (s0 < 0) s0 = lo;
    }
    auto byte_at = [&](int64_t p) -> uint32_t { return p >= l0 ? lds_b(p - l0) : (uint32_t)buf[p]; };
    unsigned long long mm = M;
    for (int left = cnt; left > 0 && !bad; --left, ++g) {
      int64_t e0;
      if (mm) {
        e0 = c0 + __builtin_ctzll(mm);
        mm &= mm - 1ull;
      } else {
        e0 = hi;                                   // the unterminated last line
      }
      const int64_t ls = s0;                       // untrimmed line [ls, e0)
      s0 = e0 + 1;
      int64_t s = ls, e = e0;
      while (s < e && byte_at(s) <= 0x20u) ++s;
      while (e > s && byte_at(e - 1) <= 0x20u) --e;
      if (s == e) {
        dcnt[g] = 1; xcnt[g] = 0; lbase[g] = -1;   // blank line: the single token ""
        dsum += 1;
        continue;
      }
      const int64_t bo = (ls - sbase) >> 1;        // this line's slots in scratch / xscratch
      int D = 0, X = 0, nd = 0;
      uint64_t v = 0;
      bool lead0 = false;
      unsigned long long f0 = 0ull, f1 = 0ull;
      for (int64_t q = s & ~(int64_t)3; q <= e && !bad; q += 4) {
        const uint32_t w = q >= l0 ? lds_dw(q - l0) : *reinterpret_cast<const uint32_t*>(buf + q);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t p = q + k;
          if (p < s || p > e || bad) continue;
          const uint32_t c = p == e ? 32u : ((w >> (8 * k)) & 0xffu);
          const uint32_t dg = c - '0';
          if (dg <= 9u) {
            if (nd == 0) { v = 0; lead0 = dg == 0; }
            v = v * 10 + dg;
            if (++nd > 10) bad = true;
            continue;
          }
          if (c == ' ' || c == '\t' || c == 0x0Bu || c == '\f') {
            if (nd) {
              if ((lead0 && nd > 1) || v > 2147483646ull) { bad = true; continue; }
              const int32_t id = (int32_t)(v + 1);
              nd = 0;
              const uint32_t hb = ((uint32_t)id * 0x9E3779B1u) >> 25;
              const unsigned long long bit = 1ull << (hb & 63u);
              bool dup = false;
              if (((hb & 64u) ? f1 : f0) & bit) {
                const int lim = D < kSeenT ? D : kSeenT;
                for (int r = 0; r < lim && !dup; ++r) dup = seen[r * kTT + tid] == id;
                for (int r = kSeenT; r < D && !dup; ++r) dup = scratch[bo + r] == id;
              }
              if (dup) {
                xscratch[bo + X++] = id;
              } else {
                if (D < kSeenT) seen[D * kTT + tid] = id;
                scratch[bo + D++] = id;
                if (hb & 64u) f1 |= bit; else f0 |= bit;
                mx = id > mx ? id : mx;
              }
            }
            continue;
          }
          bad = true;   // neither digit nor separator (nor trimmed blank)
        }
      }
      dcnt[g] = D;
      xcnt[g] = X;
      lbase[g] = bo;
      dsum += D;
      xsum += X;
    }
  }
  // the tile's id / repeat totals (k_scan_small turns them into the compaction's bases)
  // and ONE flag update per workgroup, skipped when the max id is already known: a
  // device-scope atomic per wave on one word serialises across the chip (the earlier
  // thread-per-line kernel spent most of its 62 ms on them)
  __shared__ int red[kTT / kWave][4];
  const unsigned long long anybad = __ballot(bad);
  int32_t r = mx;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const int32_t t = __shfl_xor(r, o, 64); r = t > r ? t : r; }
  const int wd = (int)wave_sum_u32((uint32_t)dsum), wx = (int)wave_sum_u32((uint32_t)xsum);
  if (lane == 0) { red[wv][0] = wd; red[wv][1] = wx; red[wv][2] = r; red[wv][3] = anybad ? 1 : 0; }
  __syncthreads();
  if (tid == 0) {
    int D = 0, X = 0, R = 0, B = 0;
    for (int w = 0; w < kTT / kWave; ++w) {
      D += red[w][0]; X += red[w][1]; R = red[w][2] > R ? red[w][2] : R; B |= red[w][3];
    }
    tile_dx[2 * blockIdx.x] = D;
    tile_dx[2 * blockIdx.x + 1] = X;
    if (B) atomicOr(&flags[0], 1);
    if (R > *reinterpret_cast<volatile int32_t*>(&flags[1])) atomicMax(&flags[1], R);
  }
}

// Exclusive scan of n counts (K interleaved int32 arrays) by one workgroup: out[K*i + k]
// = base[k] + in[K*0 + k] + ... + in[K*(i-1) + k] for i = 0..n; base (device, may be
// null = 0); total (device, may alias base) receives out[K*n + k].
template <int K>
__global__ __launch_bounds__(1024) void k_scan_small(const int32_t* __restrict__ in, int64_t n,
                                                     int64_t* __restrict__ out, const int64_t* base,
                                                     int64_t* total) {
  __shared__ int64_t part[16][K];
  __shared__ int64_t carry[K];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x < K) carry[threadIdx.x] = base ? base[threadIdx.x] : 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < n; b0 += 1024) {
    const int64_t i = b0 + threadIdx.x;
    int v[K], incl[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      v[k] = i < n ? in[K * i + k] : 0;
      incl[k] = wave_scan_incl_dpp(v[k]);
      if (lane == 63) part[wv][k] = incl[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int64_t before = carry[k];
      for (int q = 0; q < wv; ++q) before += part[q][k];
      if (i < n) out[K * i + k] = before + incl[k] - v[k];
      if (threadIdx.x == 1023) part[15][k] = before + incl[k];   // (read after the barrier below)
    }
    __syncthreads();
    if (threadIdx.x < K) carry[threadIdx.x] = part[15][threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x < K) {
    out[K * n + threadIdx.x] = carry[threadIdx.x];
    if (total) total[threadIdx.x] = carry[threadIdx.x];
  }
}

// Compaction of a region's lines, workgroups striding over its tiles: lines
// [tile_base[t], tile_base[t+1]) of tile t take ids from tile_xb[2t] on (repeats from
// tile_xb[2t+1]: k_scan_small of k_tparse's tile totals, the region's running offsets
// included).  Per chunk of 256 lines a block scan gives every line its offset (off[j],
// the shard's CSR row offsets); each wave then copies its 64 lines' ids flattened over
// the lanes (coalesced stores).  hpart (may be null): kHistCap counters per block,
// added to (one row per workgroup: no atomics).
__global__ __launch_bounds__(256) void k_tcompact(const int64_t* __restrict__ tile_base,
                                                  const int64_t* __restrict__ tile_xb, int64_t ntiles, int tail,
                                                  const int32_t* __restrict__ dcnt, const int32_t* __restrict__ xcnt,
                                                  const int64_t* __restrict__ lbase,
                                                  const int32_t* __restrict__ scratch,
                                                  const int32_t* __restrict__ xscratch, int32_t* __restrict__ items,
                                                  int32_t* __restrict__ extras, int64_t xcap,
                                                  int64_t* __restrict__ off, unsigned long long* __restrict__ hpart,
                                                  int32_t* __restrict__ flags) {
  __shared__ uint32_t h[kHistCap];
  __shared__ int wsum[4][2];
  if (hpart)
    for (int b = threadIdx.x; b < kHistCap; b += 256) h[b] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  bool over = false, xover = false;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    // (the region's unterminated last line, when tail, belongs to its last tile)
    const int64_t j0 = tile_base[t], j1 = tile_base[t + 1] + (t == ntiles - 1 ? tail : 0);
    int64_t ib = tile_xb[2 * t], xb = tile_xb[2 * t + 1];
    for (int64_t c0 = j0; c0 < j1; c0 += 256) {
      const int64_t j = c0 + threadIdx.x;
      int d = 0, x = 0;
      int64_t lb = 0;
      if (j < j1) { d = dcnt[j]; x = xcnt[j]; lb = lbase[j]; }
      const int incl = wave_scan_incl_dpp(d);
      const int xincl = wave_scan_incl_dpp(x);
      if (lane == 63) { wsum[wv][0] = incl; wsum[wv][1] = xincl; }
      __syncthreads();
      int64_t bd = ib, bx = xb;
      for (int q = 0; q < wv; ++q) { bd += wsum[q][0]; bx += wsum[q][1]; }
      int64_t td = 0, tx = 0;
      for (int q = 0; q < 4; ++q) { td += wsum[q][0]; tx += wsum[q][1]; }
      if (j < j1) off[j] = bd + incl - d;
      const int tot = wave_last(incl);
      const int excl = incl - d;
      // wave-uniform trip count: every lane takes part in the shuffles; four gathers are
      // issued before the first of their stores (they are independent of each other)
      constexpr int kU = 4;
      for (int kb = 0; kb < tot; kb += 64 * kU) {
        int32_t id[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int k = kb + 64 * u + lane;
          int L = 0;                             // the lane whose line holds flattened id k
#pragma unroll
          for (int st = 32; st > 0; st >>= 1)
            if (__shfl(incl, L + st - 1, 64) <= k) L += st;
          const int64_t lbL = __shfl(lb, L, 64);
          const int exL = __shfl(excl, L, 64);
          id[u] = (k < tot && lbL >= 0) ? scratch[lbL + (k - exL)] : 0;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int k = kb + 64 * u + lane;
          if (k < tot) {
            items[bd + k] = id[u];
            if (hpart) {
              if ((uint32_t)id[u] < (uint32_t)kHistCap) atomicAdd(&h[id[u]], 1u); else over = true;
            }
          }
        }
      }
      if (x > 0) {                               // repeated ids of the line (rare)
        const int64_t xo = bx + xincl - x;
        for (int q = 0; q < x; ++q) {
          const int32_t id = xscratch[lb + q];
          if (xo + q < xcap) extras[xo + q] = id; else xover = true;
          if (hpart) {
            if ((uint32_t)id < (uint32_t)kHistCap) atomicAdd(&h[id], 1u); else over = true;
          }
        }
      }
      ib += td;
      xb += tx;
      __syncthreads();                           // wsum is reused by the next chunk
    }
  }
  if (hpart) {
    __syncthreads();
    unsigned long long* row = hpart + (int64_t)blockIdx.x * kHistCap;
    for (int b = threadIdx.x; b < kHistCap; b += 256)
      if (h[b]) row[b] += h[b];
  }
  if (__ballot(over) != 0ull && lane == 0) atomicOr(&flags[2], 1);
  if (__ballot(xover) != 0ull && lane == 0) atomicOr(&flags[3], 1);
}

// hist[b] = sum of the rows' counters (int64 [kHistCap])
__global__ __launch_bounds__(256) void k_hist_reduce(const unsigned long long* __restrict__ hpart, int rows,
                                                     int64_t* __restrict__ hist) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= kHistCap) return;
  unsigned long long t = 0ull;
  for (int r = 0; r < rows; ++r) t += hpart[(int64_t)r * kHistCap + b];
  hist[b] = (int64_t)t;
}

// ---------------------------------------------------------------------------
// Dictionary (string) vocabularies on the device.  Same tokenisation; every token
// gets the host parser's 64-bit identity hash (csrc/host/fa_common.h hash_bytes:
// FNV-1a over the bytes, then the splitmix64 finaliser of h ^ length) and is
// inserted into a global open-addressing table keyed by that hash (0 = empty; a
// hash of 0 is stored as 1).  A token's id here is its table slot; k_slot_ids
// turns occupied slots into dense ids (slot order, i.e. hash order) afterwards.
// The slot's (byte offset, length) of one occurrence lets the host decode the
// strings it needs (frequent items) without a dictionary of every token.
// flags[0] |= 2 when a probe sequence exceeds kMaxProbe (table too full), |= 4 when
// k_dict_verify finds two distinct tokens sharing a hash: the caller then falls
// back to the host parser.
// ---------------------------------------------------------------------------
constexpr int kMaxProbe = 256;

__device__ __forceinline__ uint64_t dmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int32_t dict_insert(unsigned long long* __restrict__ keys, int64_t* __restrict__ tpos,
                                               int32_t* __restrict__ tlen, uint32_t mask, uint64_t h, int64_t pos,
                                               int32_t len) {
  if (h == 0) h = 1;
  uint32_t at = (uint32_t)(h >> 20) & mask;
  for (int p = 0; p < kMaxProbe; ++p) {
    const unsigned long long k = keys[at];
    if (k == h) return (int32_t)at;
    if (k == 0) {
      const unsigned long long old = atomicCAS(&keys[at], 0ull, (unsigned long long)h);
      if (old == 0) {
        tpos[at] = pos;
        tlen[at] = len;
        return (int32_t)at;
      }
      if (old == h) return (int32_t)at;
    }
    at = (at + 1) & mask;
  }
  return -1;
}

__global__ __launch_bounds__(kPT) void k_parse_lines_dict(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ ends, int64_t nl,
    const int64_t* __restrict__ bound_off, int32_t* __restrict__ scratch, int32_t* __restrict__ xscratch,
    int32_t* __restrict__ dcnt, int32_t* __restrict__ xcnt, int32_t* __restrict__ flags,
    unsigned long long* __restrict__ keys, int64_t* __restrict__ tpos, int32_t* __restrict__ tlen, uint32_t mask) {
  __shared__ int32_t seen[kSeen * kPT];
  const int tid = threadIdx.x;
  const int64_t j = (int64_t)blockIdx.x * kPT + tid;
  bool full = false;
  if (j < nl) {
    int64_t s = j ? ends[j - 1] + 1 : 0;
    int64_t e = ends[j];
    while (s < e && buf[s] <= 0x20) ++s;
    while (e > s && buf[e - 1] <= 0x20) --e;
    const int64_t bo = bound_off[j];
    int D = 0, X = 0;
    auto add = [&](int64_t ts, int64_t te, uint64_t h) {
      const int32_t id = dict_insert(keys, tpos, tlen, mask, dmix64(h ^ (uint64_t)(te - ts)), ts, (int32_t)(te - ts));
      if (id < 0) { full = true; return; }
      bool dup = false;
      const int lim = D < kSeen ? D : kSeen;
      for (int q = 0; q < lim && !dup; ++q) dup = seen[q * kPT + tid] == id;
      for (int q = kSeen; q < D && !dup; ++q) dup = scratch[bo + q] == id;
      if (dup) {
        xscratch[bo + X++] = id;
      } else {
        if (D < kSeen) seen[D * kPT + tid] = id;
        scratch[bo + D++] = id;
      }
    };
    if (s == e) {
      add(s, s, 0xCBF29CE484222325ull);     // blank line: the single token ""
    } else {
      int64_t ts = -1;
      uint64_t h = 0;
      for (int64_t i = s; i <= e && !full; ++i) {
        const uint32_t c = i < e ? buf[i] : (uint32_t)' ';
        if (c == ' ' || c == '\t' || c == 0x0B || c == '\f') {
          if (ts >= 0) { add(ts, i, h); ts = -1; }
          continue;
        }
        if (ts < 0) { ts = i; h = 0xCBF29CE484222325ull; }
        h = (h ^ c) * 0x100000001B3ull;
      }
    }
    dcnt[j] = D;
    xcnt[j] = X;
  }
  if (__ballot(full) != 0ull && lane_id() == 0) atomicOr(&flags[0], 2);
}

// Identity check of the table: a slot is keyed by the 64-bit hash alone, so two
// distinct tokens with one hash would share an id.  After k_parse_lines_dict every
// slot's representative (tpos, tlen) is written; this pass re-tokenises every line
// and compares each token's bytes with its slot's representative.  flags[0] |= 4 on
// any difference (the caller then parses the shard on the host, which reports the
// collision as an error, csrc/host/parse.cpp).
__device__ __forceinline__ bool dict_same(const uint8_t* __restrict__ buf, const unsigned long long* __restrict__ keys,
                                          const int64_t* __restrict__ tpos, const int32_t* __restrict__ tlen,
                                          uint32_t mask, uint64_t h, int64_t pos, int32_t len) {
  if (h == 0) h = 1;
  uint32_t at = (uint32_t)(h >> 20) & mask;
  for (int p = 0; p < kMaxProbe; ++p) {
    const unsigned long long k = keys[at];
    if (k == h) {
      if (tlen[at] != len) return false;
      const int64_t q = tpos[at];
      for (int32_t i = 0; i < len; ++i)
        if (buf[q + i] != buf[pos + i]) return false;
      return true;
    }
    if (k == 0) return false;
    at = (at + 1) & mask;
  }
  return false;
}

__global__ __launch_bounds__(kPT) void k_dict_verify(const uint8_t* __restrict__ buf, const int64_t* __restrict__ ends,
                                                     int64_t nl, int32_t* __restrict__ flags,
                                                     const unsigned long long* __restrict__ keys,
                                                     const int64_t* __restrict__ tpos, const int32_t* __restrict__ tlen,
                                                     uint32_t mask) {
  const int64_t j = (int64_t)blockIdx.x * kPT + threadIdx.x;
  bool bad = false;
  if (j < nl) {
    int64_t s = j ? ends[j - 1] + 1 : 0;
    int64_t e = ends[j];
    while (s < e && buf[s] <= 0x20) ++s;
    while (e > s && buf[e - 1] <= 0x20) --e;
    if (s < e) {        // (a blank line's token "" has length 0: nothing to compare)
      int64_t ts = -1;
      uint64_t h = 0;
      for (int64_t i = s; i <= e && !bad; ++i) {
        const uint32_t c = i < e ? buf[i] : (uint32_t)' ';
        if (c == ' ' || c == '\t' || c == 0x0B || c == '\f') {
          if (ts >= 0) {
            bad = !dict_same(buf, keys, tpos, tlen, mask, dmix64(h ^ (uint64_t)(i - ts)), ts, (int32_t)(i - ts));
            ts = -1;
          }
          continue;
        }
        if (ts < 0) { ts = i; h = 0xCBF29CE484222325ull; }
        h = (h ^ c) * 0x100000001B3ull;
      }
    }
  }
  if (__ballot(bad) != 0ull && lane_id() == 0) atomicOr(&flags[0], 4);
}

// dense id of every occupied slot (exclusive scan of occupancy done by the caller)
__global__ __launch_bounds__(256) void k_slot_remap(int32_t* __restrict__ ids, int64_t n,
                                                    const int32_t* __restrict__ slot_id) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    ids[i] = slot_id[ids[i]];
}

}  // namespace fa

using namespace fa;

FA_API int fa_hip_parse_lines_dict(const uint8_t* buf, const int64_t* ends, int64_t nl, const int64_t* bound_off,
                                   int32_t* scratch, int32_t* xscratch, int32_t* dcnt, int32_t* xcnt,
                                   int32_t* flags, void* keys, int64_t* tpos, int32_t* tlen, int64_t cap,
                                   hipStream_t st) {
  if (nl <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) || cap > ((int64_t)1 << 31)) return 1;
  hipLaunchKernelGGL(k_parse_lines_dict, dim3((unsigned)((nl + kPT - 1) / kPT)), dim3(kPT), 0, st, buf, ends, nl,
                     bound_off, scratch, xscratch, dcnt, xcnt, flags, (unsigned long long*)keys, tpos, tlen,
                     (uint32_t)(cap - 1));
  FA_LAUNCH_RET();
}

FA_API int fa_hip_dict_verify(const uint8_t* buf, const int64_t* ends, int64_t nl, int32_t* flags, const void* keys,
                              const int64_t* tpos, const int32_t* tlen, int64_t cap, hipStream_t st) {
  if (nl <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) || cap > ((int64_t)1 << 31)) return 1;
  hipLaunchKernelGGL(k_dict_verify, dim3((unsigned)((nl + kPT - 1) / kPT)), dim3(kPT), 0, st, buf, ends, nl, flags,
                     (const unsigned long long*)keys, tpos, tlen, (uint32_t)(cap - 1));
  FA_LAUNCH_RET();
}

FA_API int fa_hip_slot_remap(int32_t* ids, int64_t n, const int32_t* slot_id, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_slot_remap, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 65536)), dim3(256), 0, st, ids,
                     n, slot_id);
  FA_LAUNCH_RET();
}

FA_API int64_t fa_hip_parse_tiles(int64_t n) { return (n + kLTile - 1) / kLTile; }

FA_API int fa_hip_line_count(const uint8_t* buf, int64_t n, int32_t* tile_cnt, hipStream_t st) {
  const int64_t tiles = (n + kLTile - 1) / kLTile;
  if (tiles <= 0) return 0;
  if (tiles >= (int64_t)INT32_MAX) return 3;
  hipLaunchKernelGGL(k_line_count, dim3((unsigned)tiles), dim3(kLT), 0, st, buf, n, tile_cnt);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_line_ends(const uint8_t* buf, int64_t n, const int64_t* tile_base, int64_t* ends,
                            hipStream_t st) {
  const int64_t tiles = (n + kLTile - 1) / kLTile;
  if (tiles <= 0) return 0;
  hipLaunchKernelGGL(k_line_ends, dim3((unsigned)tiles), dim3(kLT), 0, st, buf, n, tile_base, ends);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_compact_lines(const int32_t* scratch, const int32_t* xscratch, const int64_t* bound_off,
                                const int32_t* dcnt, const int32_t* xcnt, const int64_t* off, const int64_t* xoff,
                                int64_t nl, int32_t* items, int32_t* extras, hipStream_t st) {
  if (nl <= 0) return 0;
  hipLaunchKernelGGL(k_compact_lines, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, st, scratch, xscratch,
                     bound_off, dcnt, xcnt, off, xoff, nl, items, extras);
  FA_LAUNCH_RET();
}

FA_API int64_t fa_hip_tparse_tiles(int64_t lo, int64_t hi) {
  const int64_t a = lo & ~(int64_t)63;
  return hi > lo ? (hi - a + kLTile - 1) / kLTile : 0;
}

FA_API int fa_hip_tparse_hist_cap() { return kHistCap; }

FA_API int fa_hip_tline_count(const uint8_t* buf, int64_t lo, int64_t hi, int32_t* tile_cnt, hipStream_t st) {
  const int64_t a = lo & ~(int64_t)63;
  const int64_t tiles = fa_hip_tparse_tiles(lo, hi);
  if (tiles <= 0) return 0;
  if (tiles >= (int64_t)INT32_MAX || lo < 0) return 3;
  hipLaunchKernelGGL(k_tline_count, dim3((unsigned)tiles), dim3(kLT), 0, st, buf, a, lo, hi, tile_cnt);
  FA_LAUNCH_RET();
}

// buf_len: bytes of buf readable (a multiple of 16, >= hi + 64 rounded up); tail = 1: a
// last line without terminator ends at hi; sbase: byte position of scratch slot 0
// (scratch and xscratch hold >= (hi - sbase) / 2 + 1 ids)
FA_API int fa_hip_tparse(const uint8_t* buf, int64_t buf_len, int64_t lo, int64_t hi, int tail, int64_t sbase,
                         const int64_t* tile_base, int32_t* dcnt, int32_t* xcnt, int64_t* lbase, int32_t* scratch,
                         int32_t* xscratch, int32_t* tile_dx, int32_t* flags, hipStream_t st) {
  const int64_t a = lo & ~(int64_t)63;
  const int64_t tiles = fa_hip_tparse_tiles(lo, hi);
  if (tiles <= 0) return 0;
  if (sbase > lo || (buf_len & 15) || buf_len < hi + 64) return 3;
  hipLaunchKernelGGL(k_tparse, dim3((unsigned)tiles), dim3(kTT), 0, st, buf, buf_len, a, lo, hi, tail, sbase,
                     tile_base, dcnt, xcnt, lbase, scratch, xscratch, tile_dx, flags);
  FA_LAUNCH_RET();
}

// k = 1: tile_base [n + 1] from per-tile line counts; k = 2: the tiles' id / repeat
// bases [2 (n + 1)] from k_tparse's totals, starting at and advancing cursor (int64 [2])
FA_API int fa_hip_scan_small(int k, const int32_t* in, int64_t n, int64_t* out, int64_t* cursor, hipStream_t st) {
  if (n < 0) return 3;
  if (k == 1)
    hipLaunchKernelGGL(k_scan_small<1>, dim3(1), dim3(1024), 0, st, in, n, out, (const int64_t*)cursor, cursor);
  else if (k == 2)
    hipLaunchKernelGGL(k_scan_small<2>, dim3(1), dim3(1024), 0, st, in, n, out, (const int64_t*)cursor, cursor);
  else
    return 3;
  FA_LAUNCH_RET();
}

FA_API int fa_hip_tcompact(const int64_t* tile_base, const int64_t* tile_xb, int64_t ntiles, int tail,
                           const int32_t* dcnt,
                           const int32_t* xcnt, const int64_t* lbase, const int32_t* scratch, const int32_t* xscratch,
                           int32_t* items, int32_t* extras, int64_t xcap, int64_t* off, int grid,
                           unsigned long long* hpart, int32_t* flags, hipStream_t st) {
  if (ntiles <= 0) return 0;
  if (grid < 1) return 3;
  hipLaunchKernelGGL(k_tcompact, dim3((unsigned)grid), dim3(256), 0, st, tile_base, tile_xb, ntiles, tail, dcnt, xcnt,
                     lbase, scratch, xscratch, items, extras, xcap, off, hpart, flags);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_hist_reduce(const unsigned long long* hpart, int rows, int64_t* hist, hipStream_t st) {
  hipLaunchKernelGGL(k_hist_reduce, dim3((kHistCap + 255) / 256), dim3(256), 0, st, hpart, rows, hist);
  FA_LAUNCH_RET();
}
