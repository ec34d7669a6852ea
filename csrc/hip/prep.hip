// Preprocessing kernels: token histogram, per-transaction frequent counts,
// transaction compression to sorted rank lists, row hashing for dedup, and the
// vertical (item-major) bitmap build.
//
// Reference sites: FastApriori.scala:55-57 (histogram),
// :66-70 (compress + size filter), :71-79 (dedup), :195-210 (vertical transpose,
// done there as F1 separate Spark jobs producing 1 byte per transaction).
#include "fa_hip.h"

namespace fa {

// ---------------------------------------------------------------------------
// Histogram over token ids.  V <= kLdsBins: LDS-privatised per workgroup, one
// global atomic per non-zero bin per workgroup; otherwise global atomics.
// ---------------------------------------------------------------------------
constexpr int kLdsBins = 16384;

// The LDS bins are dynamic: V * nrep words, so a T10-scale vocabulary (V ~ 1000) leaves
// room for many workgroups per CU (a static 64 KB array allowed two).  nrep = 4 gives each
// wave its own copy of the bins when they fit, so the four waves' atomics never collide.
template <bool kLds, bool kVec>
__global__ __launch_bounds__(256) void k_histogram(const int32_t* __restrict__ items, int64_t nnz,
                                                   int32_t V, int nrep, uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t sh[];
  uint32_t* mine = sh;
  if (kLds) {
    for (int i = threadIdx.x; i < V * nrep; i += blockDim.x) sh[i] = 0;
    mine = sh + (nrep > 1 ? (threadIdx.x >> 6) % nrep : 0) * V;
    __syncthreads();
  }
  auto add = [&](int32_t v) {
    if (kLds) atomicAdd(&mine[v], 1u); else atomicAdd(&counts[v], 1u);
  };
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = kVec ? (nnz >> 2) : 0;
  const int4* it4 = reinterpret_cast<const int4*>(items);
  for (int64_t i = gid; i < n4; i += stride) {
    int4 v = it4[i];
    add(v.x); add(v.y); add(v.z); add(v.w);
  }
  for (int64_t i = (n4 << 2) + gid; i < nnz; i += stride) add(items[i]);
  if (kLds) {
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      uint32_t c = 0;
      for (int r = 0; r < nrep; ++r) c += sh[r * V + i];
      if (c) atomicAdd(&counts[i], c);
    }
  }
}

// ---------------------------------------------------------------------------
// F1 ranking on the device (FastApriori.scala:55-62; the order of csrc/host/f1.cpp
// fa_f1_rank_numeric): the frequent ids (support >= thr) by support descending, ties
// by a unique tie key -- Java String order of the decimal token (string: the digits
// left-aligned to 10 places, then the length; id 0 = "" first) or the integer value
// (numeric: id 0 last).  Every workgroup stages all V (support, tie key) pairs in
// LDS and each thread ranks one id by counting the ids ahead of it, so the id -> rank
// LUT is written without a host round trip: the compression kernels queue right
// behind it while the host reads the ranking back.  pack (int64 [2 V + 1]): [0] the
// number of frequent ids F, [1 .. F] the ids in rank order, [V + 1 .. V + F] their supports.
// ---------------------------------------------------------------------------
constexpr int kF1RankMax = 2048;

__device__ __forceinline__ int64_t f1_tie_key(int64_t fid, int numeric) {
  if (numeric) return fid == 0 ? INT64_MAX : fid - 1;
  if (fid == 0) return -16;                       // "" sorts first (key -1, length 0)
  const int64_t v = fid - 1;
  int digits = 1;
  int64_t p = 10;
  while (digits < 11 && v >= p) { ++digits; p *= 10; }
  int64_t pad = 1;
  for (int i = 0; i < 10 - min(digits, 10); ++i) pad *= 10;
  return v * pad * 16 + digits;                   // (key, length) in one order-preserving int64
}

__global__ __launch_bounds__(256) void k_f1_rank(const int64_t* __restrict__ hist, int32_t V, int64_t thr,
                                                 int numeric, int32_t* __restrict__ lut, int64_t* __restrict__ pack) {
  __shared__ int64_t sc[kF1RankMax], sk[kF1RankMax];
  __shared__ int nf[4];
  int mine = 0;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const int64_t c = hist[i];
    sc[i] = c >= thr ? c : -1;
    sk[i] = f1_tie_key(i, numeric);
    mine += c >= thr;
  }
  __syncthreads();
  const int v = (int)blockIdx.x * blockDim.x + (int)threadIdx.x;
  if (v < V) {
    const int64_t c = sc[v], k = sk[v];
    if (c < 0) {
      lut[v] = -1;
    } else {
      int r = 0;
      for (int j = 0; j < V; ++j) {               // (every lane reads the same word: a broadcast)
        const int64_t cj = sc[j];
        r += (cj > c) | ((cj == c) & (sk[j] < k));
      }
      lut[v] = r;
      pack[1 + r] = v;
      pack[1 + V + r] = c;
    }
  }
  if (blockIdx.x == 0) {
    mine = (int)wave_sum_u32((uint32_t)mine);
    if ((threadIdx.x & 63) == 0) nf[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) pack[0] = (int64_t)nf[0] + nf[1] + nf[2] + nf[3];
  }
}

// ---------------------------------------------------------------------------
// Heavy-hitter F1 for wide vocabularies (webdocs-scale: millions of ids, where
// a V-bin histogram means one global atomic per token plus a V-sized
// all-reduce).  Pass 1: a 2-row count-min sketch (2 x 16K u32 bins = 128 KB of
// LDS per workgroup, one workgroup per CU), each workgroup storing its private
// sketch to partial[wg] (summed by the caller).  Pass 2: exact counts for the
// sketch's candidates only, through an LDS open-addressing table (keys -1 =
// empty, linear probing).  Both hashes are multiplicative; the host mirrors
// them (fastapriori_amd/ops/primitives.py: _sk_hash) to build the table.
// ---------------------------------------------------------------------------
constexpr int kSkLog = 14, kSkW = 1 << kSkLog;
constexpr uint32_t kSkA0 = 0x9E3779B1u, kSkA1 = 0x85EBCA77u;

template <bool kVec, class F>
__device__ __forceinline__ void for_each_item(const int32_t* __restrict__ items, int64_t nnz, F&& f) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = kVec ? (nnz >> 2) : 0;
  const int4* it4 = reinterpret_cast<const int4*>(items);
  for (int64_t i = gid; i < n4; i += stride) {
    const int4 v = it4[i];
    f(v.x); f(v.y); f(v.z); f(v.w);
  }
  for (int64_t i = (n4 << 2) + gid; i < nnz; i += stride) f(items[i]);
}

template <bool kVec>
__global__ __launch_bounds__(1024) void k_f1_sketch(const int32_t* __restrict__ items, int64_t nnz,
                                                    uint32_t* __restrict__ partial) {
  __shared__ uint32_t sh[2 * kSkW];
  for (int i = threadIdx.x; i < 2 * kSkW; i += blockDim.x) sh[i] = 0;
  __syncthreads();
  for_each_item<kVec>(items, nnz, [&](int32_t v) {
    atomicAdd(&sh[((uint32_t)v * kSkA0) >> (32 - kSkLog)], 1u);
    atomicAdd(&sh[kSkW + (((uint32_t)v * kSkA1) >> (32 - kSkLog))], 1u);
  });
  __syncthreads();
  uint32_t* out = partial + (size_t)blockIdx.x * 2 * kSkW;
  for (int i = threadIdx.x; i < 2 * kSkW; i += blockDim.x) out[i] = sh[i];
}

template <bool kVec>
__global__ __launch_bounds__(1024) void k_f1_exact(const int32_t* __restrict__ items, int64_t nnz,
                                                   const int32_t* __restrict__ keys, int log_s,
                                                   uint32_t* __restrict__ counts) {
  __shared__ int32_t sk[kSkW];
  __shared__ uint32_t sc[kSkW];
  const int S = 1 << log_s;
  for (int i = threadIdx.x; i < S; i += blockDim.x) { sk[i] = keys[i]; sc[i] = 0; }
  __syncthreads();
  for_each_item<kVec>(items, nnz, [&](int32_t v) {
    for (uint32_t h = ((uint32_t)v * kSkA0) >> (32 - log_s);; h = (h + 1) & (S - 1)) {
      const int32_t k = sk[h];
      if (k == v) { atomicAdd(&sc[h], 1u); break; }
      if (k < 0) break;
    }
  });
  __syncthreads();
  for (int i = threadIdx.x; i < S; i += blockDim.x)
    if (sc[i]) atomicAdd(&counts[i], sc[i]);
}

// ---------------------------------------------------------------------------
// Number of frequent ids in every transaction (ids are distinct per line).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_txn_freq_count(const int64_t* __restrict__ off,
                                                        const int32_t* __restrict__ items, int64_t n,
                                                        const int32_t* __restrict__ lut,
                                                        int32_t* __restrict__ cnt) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  int32_t c = 0;
  for (int64_t i = off[t], e = off[t + 1]; i < e; ++i) c += lut[items[i]] >= 0;
  cnt[t] = c;
}

// The same with the workgroup's 256-row input span loaded coalesced and mapped
// through the LUT into LDS as one flag byte per token; each thread then sums its
// row's flags from LDS.  (Thread-per-row loads touch one cache line per lane and
// load: 15.6 ms for T40I10D100M's 4 G tokens.)  Spans past SPAN bytes read their
// rows directly.
template <int SPAN>
__global__ __launch_bounds__(256) void k_txn_freq_count_span(const int64_t* __restrict__ off,
                                                             const int32_t* __restrict__ items, int64_t n,
                                                             const int32_t* __restrict__ lut,
                                                             int32_t* __restrict__ cnt) {
  constexpr int PER = SPAN / 256;
  __shared__ __attribute__((aligned(16))) uint8_t fl[SPAN];
  const int64_t x0 = (int64_t)blockIdx.x * 256;
  const int64_t x1 = min(n, x0 + 256);
  const int64_t x = x0 + threadIdx.x;
  const int64_t base = off[x0], n_in = off[x1] - base;
  const int64_t s = x < x1 ? off[x] : 0, e = x < x1 ? off[x + 1] : 0;
  if (n_in <= SPAN) {
    int32_t v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int64_t i = threadIdx.x + k * 256;
      v[k] = i < n_in ? items[base + i] : 0;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int64_t i = threadIdx.x + k * 256;
      if (i < n_in) fl[i] = lut[v[k]] >= 0 ? 1 : 0;
    }
    __syncthreads();
    if (x < x1) {
      // the row's flag bytes [s, e) read a dword at a time (flags are 0 / 1 bytes:
      // popcount of the masked dword = number of frequent tokens in it)
      int32_t c = 0;
      const int sr = (int)(s - base), er = (int)(e - base);
      if (er > sr) {
        const uint32_t* fw = reinterpret_cast<const uint32_t*>(fl);
        const int w0 = sr >> 2, w1 = (er - 1) >> 2;
        for (int w = w0; w <= w1; ++w) {
          const int lo = w == w0 ? (sr & 3) : 0, hi = w == w1 ? ((er - 1) & 3) + 1 : 4;
          const uint32_t m = (hi == 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u)) & ~((1u << (8 * lo)) - 1u);
          c += __popc(fw[w] & m);
        }
      }
      cnt[x] = c;
    }
  } else if (x < x1) {
    int32_t c = 0;
    for (int64_t i = s; i < e; ++i) c += lut[items[i]] >= 0;
    cnt[x] = c;
  }
}

// ---------------------------------------------------------------------------
// Compression: kept transaction x -> its frequent ranks, sorted ascending, at
// ranks[roff[x] .. roff[x+1]).  Short rows are sorted in registers with an
// unrolled bitonic network (static indices only, so nothing spills to
// scratch); rows longer than N go to an overflow list for the next tier.
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void bitonic_regs(uint32_t (&a)[N]) {
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l > i) {
          uint32_t x = a[i], y = a[l];
          uint32_t lo = x < y ? x : y, hi = x < y ? y : x;
          if ((i & k) == 0) { a[i] = lo; a[l] = hi; } else { a[i] = hi; a[l] = lo; }
        }
      }
    }
  }
}

template <int N>
__global__ __launch_bounds__(256) void k_compress_regs(
    const int64_t* __restrict__ off, const int32_t* __restrict__ items, const int32_t* __restrict__ lut,
    const int32_t* __restrict__ rows, int64_t nrows, const int32_t* __restrict__ kept,
    const int64_t* __restrict__ roff, int32_t* __restrict__ ranks, int8_t* __restrict__ over_flag,
    uint8_t* __restrict__ bcnt = nullptr, int64_t bld = 0, int nb = 0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < nrows;
  int64_t s = 0, L = 0, x = 0;
  if (valid) {
    x = rows ? rows[i] : (int32_t)i;
    const int64_t t = kept[x];
    s = off[t];
    L = off[t + 1] - s;
    over_flag[i] = L > N ? 1 : 0;
  }
  const bool mine = valid && L <= N;
  // loads only up to the longest row of the wave (a wave-uniform bound: the slots past
  // it are skipped by a scalar branch instead of issuing N mostly-masked loads)
  int Lw = mine ? (int)L : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const int t = __shfl_xor(Lw, o, 64); Lw = t > Lw ? t : Lw; }
  Lw = __builtin_amdgcn_readfirstlane(Lw);
  if (!mine) return;
  uint32_t a[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    a[j] = 0xFFFFFFFFu;
    if (j < Lw) {
      const int32_t r = j < L ? lut[items[s + j]] : -1;
      a[j] = r < 0 ? 0xFFFFFFFFu : (uint32_t)r;
    }
  }
  bitonic_regs<N>(a);
  const int64_t o = roff[x];
  const int64_t c = roff[x + 1] - o;
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (j < c) ranks[o + j] = (int32_t)a[j];
  if (bcnt) {
    // 256-rank block counts of the row (see k_cmp_emit); <= 64 items: no byte carries
    unsigned long long pc = 0;
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < c) pc += 1ull << ((a[j] >> 8) << 3);
    for (int b = 0; b < nb; ++b) bcnt[(int64_t)b * bld + x] = (uint8_t)(pc >> (8 * b));
  }
}

// Tier 1 with LDS staging: a workgroup's 256 kept rows usually come from one
// contiguous span of the input CSR, so the span is loaded coalesced (and
// mapped through the LUT) into LDS, each thread sorts its row from LDS, and the
// sorted output span is written back coalesced.  Rows longer than N go to the
// overflow list; their (garbage) slots in the output span are rewritten by the
// next tier, which runs later on the same stream.
constexpr int kCSpan = 8192;

// SPAN = staged input tokens per workgroup (32 KB at N = 16; 64 KB for the
// 64-token tier of long-ish rows, e.g. T40I10's 40-token transactions, whose
// 256-row spans do not fit 8192 and would otherwise be gathered row by row).
// BT = uint16_t (ranks < 0xFFFF, the caller's check): the span at half the LDS, so
// twice the workgroups per CU (the 64 KB u32 span allowed two, 8 waves per CU).
template <int N, int SPAN = kCSpan, typename BT = uint32_t>
__global__ __launch_bounds__(256) void k_compress_staged(
    const int64_t* __restrict__ off, const int32_t* __restrict__ items, const int32_t* __restrict__ lut,
    int64_t T, const int32_t* __restrict__ kept, const int64_t* __restrict__ roff,
    int32_t* __restrict__ ranks, int8_t* __restrict__ over_flag) {
  constexpr int kCSpan = SPAN;
  constexpr int kCPer = kCSpan / 256;   // span elements per thread, loaded with full ILP
  constexpr BT kNone = (BT)~(BT)0;      // not frequent: sorts last
  __shared__ BT buf[kCSpan];
  const int64_t x0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t x1 = min(T, x0 + (int64_t)blockDim.x);
  const int64_t x = x0 + threadIdx.x;
  // independent loads first: this row's bounds and the span bounds
  const int64_t t = x < x1 ? (int64_t)kept[x] : 0;
  const int64_t tf = kept[x0], tl = kept[x1 - 1];
  const int64_t s = off[t], e_row = off[t + 1];
  const int64_t base = off[tf];
  const int64_t n_in = off[tl + 1] - base;
  const int64_t obase = roff[x0];
  const int64_t n_out = roff[x1] - obase;
  const int64_t o_row = x < x1 ? roff[x] : 0, o_end = x < x1 ? roff[x + 1] : 0;
  const bool staged = n_in <= kCSpan;
  if (staged) {
    // in chunks of at most 32 loads per thread: 64 in flight at the 64-token tier held
    // 64 more VGPRs than the row sort needs and capped the workgroups per CU
    constexpr int kCh = kCPer < 32 ? kCPer : 32;
#pragma unroll
    for (int k0 = 0; k0 < kCPer; k0 += kCh) {
      int32_t v[kCh];
#pragma unroll
      for (int k = 0; k < kCh; ++k) {
        const int64_t i = threadIdx.x + (k0 + k) * 256;
        v[k] = i < n_in ? items[base + i] : 0;
      }
#pragma unroll
      for (int k = 0; k < kCh; ++k) {
        const int64_t i = threadIdx.x + (k0 + k) * 256;
        if (i < n_in) v[k] = lut[v[k]];
      }
#pragma unroll
      for (int k = 0; k < kCh; ++k) {
        const int64_t i = threadIdx.x + (k0 + k) * 256;
        if (i < n_in) buf[i] = v[k] < 0 ? kNone : (BT)v[k];
      }
    }
  }
  __syncthreads();
  uint32_t a[N];
  const int64_t L = e_row - s;
  const bool mine = x < x1 && L <= N;
  if (x < x1) over_flag[x] = L > N ? 1 : 0;
  if (mine) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      uint32_t v = 0xFFFFFFFFu;
      if (j < L) {
        if (staged) { const BT b = buf[s - base + j]; v = b == kNone ? 0xFFFFFFFFu : (uint32_t)b; }
        else { const int32_t r = lut[items[s + j]]; v = r < 0 ? 0xFFFFFFFFu : (uint32_t)r; }
      }
      a[j] = v;
    }
    bitonic_regs<N>(a);
  }
  __syncthreads();   // everyone is done reading the input span
  const int64_t o = o_row - obase, c = o_end - o_row;
  if (mine) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < c) {
        if (staged) buf[o + j] = (BT)a[j];
        else ranks[obase + o + j] = (int32_t)a[j];
      }
  }
  __syncthreads();
  if (staged)
    for (int64_t i = threadIdx.x; i < n_out; i += blockDim.x) ranks[obase + i] = (int32_t)buf[i];
}

// Long rows: one 256-thread workgroup per row, bitonic sort in LDS (<= 16384).
constexpr int kLongMax = 16384;
__global__ __launch_bounds__(256) void k_compress_lds(
    const int64_t* __restrict__ off, const int32_t* __restrict__ items, const int32_t* __restrict__ lut,
    const int32_t* __restrict__ rows, const int32_t* __restrict__ kept, const int64_t* __restrict__ roff,
    int32_t* __restrict__ ranks, int32_t* __restrict__ too_long, int32_t* __restrict__ n_too_long) {
  __shared__ uint32_t sh[kLongMax];
  const int32_t x = rows[blockIdx.x];
  const int64_t t = kept[x];
  const int64_t s = off[t];
  const int64_t L = off[t + 1] - s;
  if (L > kLongMax) {
    if (threadIdx.x == 0) too_long[atomicAdd(n_too_long, 1)] = x;
    return;
  }
  int P = 1;
  while (P < L) P <<= 1;
  for (int j = threadIdx.x; j < P; j += blockDim.x) {
    int32_t r = j < L ? lut[items[s + j]] : -1;
    sh[j] = r < 0 ? 0xFFFFFFFFu : (uint32_t)r;
  }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          uint32_t a = sh[i], b = sh[l];
          bool up = (i & k) == 0;
          if ((a > b) == up) { sh[i] = b; sh[l] = a; }
        }
      }
      __syncthreads();
    }
  }
  const int64_t o = roff[x];
  const int64_t c = roff[x + 1] - o;
  for (int j = threadIdx.x; j < c; j += blockDim.x) ranks[o + j] = (int32_t)sh[j];
}

// Long rows, F1 <= 65536: one wave per row and no sort.  The row's tokens are
// read coalesced 256 at a time, mapped through the LUT, and each frequent rank
// sets its bit in a per-wave LDS bitmap (ds_or_b64).  Lane l owns words
// l + 64m; a popcount + DPP prefix scan over the words gives every lane its
// output position, so ranks come out ascending.  Lanes clear their own words.
constexpr int kCwMaxWords = 16;   // words per lane -> F1 <= 16 * 64 * 64

__global__ __launch_bounds__(256) void k_compress_wave(
    const int64_t* __restrict__ off, const int32_t* __restrict__ items, const int32_t* __restrict__ lut,
    const int32_t* __restrict__ rows, int64_t nrows, const int32_t* __restrict__ kept,
    const int64_t* __restrict__ roff, int32_t* __restrict__ ranks, int M, const int8_t* __restrict__ flags) {
  // flags (optional): only rows i with flags[i] != 0 (the rows an earlier tier left)
  __shared__ unsigned long long bm[4][kCwMaxWords * 64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long* b = bm[w];
  for (int m = 0; m < M; ++m) b[lane + 64 * m] = 0;
  wave_lds_sync();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t i = (int64_t)blockIdx.x * 4 + w; i < nrows; i += nw) {
    if (flags && !flags[i]) continue;             // wave-uniform: one row per wave
    const int32_t x = rows ? rows[i] : (int32_t)i;
    const int64_t t = kept[x];
    const int64_t s = off[t], L = off[t + 1] - s;
    const int64_t o = roff[x];
    for (int64_t j0 = 0; j0 < L; j0 += 256) {
      int32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = j0 + lane + 64 * k;
        v[k] = j < L ? items[s + j] : -1;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = v[k] >= 0 ? lut[v[k]] : -1;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (v[k] >= 0) atomicOr(&b[v[k] >> 6], 1ull << (v[k] & 63));
    }
    wave_lds_sync();
    int base = 0;
    for (int m = 0; m < M; ++m) {
      const int widx = lane + 64 * m;
      unsigned long long word = b[widx];
      b[widx] = 0;
      const int c = __popcll(word);
      const int incl = wave_scan_incl_dpp(c);
      int64_t pos = o + base + incl - c;
      base += wave_last(incl);
      while (word) {
        ranks[pos++] = widx * 64 + (__ffsll((long long)word) - 1);
        word &= word - 1;
      }
    }
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------
// Order-sensitive 128-bit hash of each compressed row (rows are sorted, so equal
// sets <=> equal sequences).  Used to find duplicate transactions.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t dmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_row_hash(const int64_t* __restrict__ roff,
                                                  const int32_t* __restrict__ ranks, int64_t T,
                                                  int64_t* __restrict__ h1, int64_t* __restrict__ h2) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= T) return;
  uint64_t a = 0x243F6A8885A308D3ull, b = 0x13198A2E03707344ull;
  const int64_t s = roff[x], e = roff[x + 1];
  for (int64_t i = s; i < e; ++i) {
    uint64_t r = (uint32_t)ranks[i];
    a = dmix64(a ^ r);
    b = dmix64(b + r * 0xD6E8FEB86659FD93ull);
  }
  a = dmix64(a ^ (uint64_t)(e - s));
  // keep the sign bit clear so signed sorts order like unsigned ones
  h1[x] = (int64_t)(a >> 1);
  h2[x] = (int64_t)(b >> 1);
}

// Dedup probe (models.apriori FastApriori._want_dedup): the row hash h1 of the
// first min(T, n_max) compressed rows marks a bit of a 2^22-bit occupancy bitmap;
// the marked bits estimate the distinct rows by linear counting.  T is read from
// device memory (the compression scan's total), so the probe is queued behind the
// emit pass and its result travels with the compression sizes in one readback.
constexpr int kProbeBits = 1 << 22;

// Only rows of <= kCmpProbeLen items are hashed (the emit pass has written them; longer
// rows are finished by later tiers); hashed counts them.
constexpr int kCmpProbeLen = 16;

// Pass 1 (thread per row): the row's slot, or kNoSlot (past T, or a row longer than
// kCmpProbeLen), and the workgroup's hashed-row count -- plain stores: 2^18 scattered
// atomicOr into a 512 KB global bitmap cost ~58 us (device-scope atomics are served
// behind the XCDs' L2s), more than all the hashing.
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr int kProbeRange = 1 << 16;                 // slots per pass-2 workgroup (8 KB of LDS)

__global__ __launch_bounds__(256) void k_dedup_probe(const int64_t* __restrict__ roff,
                                                     const int32_t* __restrict__ ranks,
                                                     const int64_t* __restrict__ T_dev, int64_t n_max,
                                                     uint32_t* __restrict__ slots, uint32_t* __restrict__ part) {
  const int64_t n = min(T_dev[0], n_max);
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t slot = kNoSlot;
  if (x < n) {
    const int64_t s = roff[x], e = roff[x + 1];
    const int L = (int)(e - s);
    if (L <= kCmpProbeLen) {
      uint32_t v[kCmpProbeLen];
#pragma unroll
      for (int j = 0; j < kCmpProbeLen; ++j) v[j] = j < L ? (uint32_t)ranks[s + j] : 0u;
      uint64_t a = 0x243F6A8885A308D3ull;
#pragma unroll
      for (int j = 0; j < kCmpProbeLen; ++j)
        if (j < L) a = dmix64(a ^ (uint64_t)v[j]);
      a = dmix64(a ^ (uint64_t)L);
      slot = (uint32_t)((a >> 1) & (kProbeBits - 1));      // = (h1 of k_row_hash) mod 2^22
    }
  }
  if (x < n_max) slots[x] = slot;
  __shared__ uint32_t wsum[4];
  const uint32_t c = wave_sum_u32(slot != kNoSlot ? 1u : 0u);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// Pass 2: workgroup j owns slots [j * kProbeRange, (j + 1) * kProbeRange) as an LDS
// bitmap, marks the slots of every hashed row that fall in it, and adds its occupied
// count (one atomic per workgroup); workgroup 0 also sums pass 1's row counts.
// out[0]: occupied slots, out[1]: hashed rows (out[0] zeroed by the caller).
__global__ __launch_bounds__(1024) void k_probe_count(const uint32_t* __restrict__ slots, int64_t n_max,
                                                      const uint32_t* __restrict__ part, int nparts,
                                                      unsigned long long* __restrict__ out) {
  __shared__ uint32_t bits[kProbeRange / 32];
  __shared__ uint32_t wsum[16];
  for (int i = threadIdx.x; i < kProbeRange / 32; i += 1024) bits[i] = 0u;
  __syncthreads();
  const uint32_t lo = (uint32_t)blockIdx.x * kProbeRange;
  const uint4* s4 = reinterpret_cast<const uint4*>(slots);
  const int64_t n4 = n_max >> 2;
  auto mark = [&](uint32_t v) {
    const uint32_t d = v - lo;                       // kNoSlot and other ranges: d >= kProbeRange
    if (d < (uint32_t)kProbeRange) atomicOr(&bits[d >> 5], 1u << (d & 31));
  };
  // eight 16-B loads in flight per thread (the pass streams 4 B per probed row per workgroup)
  constexpr int U = 8;
  int64_t i = threadIdx.x;
  for (; i + (U - 1) * 1024 < n4; i += U * 1024) {
    uint4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = s4[i + k * 1024];
#pragma unroll
    for (int k = 0; k < U; ++k) { mark(v[k].x); mark(v[k].y); mark(v[k].z); mark(v[k].w); }
  }
  for (; i < n4; i += 1024) {
    const uint4 v = s4[i];
    mark(v.x); mark(v.y); mark(v.z); mark(v.w);
  }
  for (int64_t j = (n4 << 2) + threadIdx.x; j < n_max; j += 1024) mark(slots[j]);
  __syncthreads();
  uint32_t c = 0, h = 0;
  for (int i = threadIdx.x; i < kProbeRange / 32; i += 1024) c += __popc(bits[i]);
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < nparts; i += 1024) h += part[i];
  c = wave_sum_u32(c);
  h = wave_sum_u32(h);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) wsum[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < 16; ++k) t += wsum[k];
    if (t) atomicAdd(out, (unsigned long long)t);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wsum[w] = h;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < 16; ++k) t += wsum[k];
    out[1] = t;
  }
}

// ---------------------------------------------------------------------------
// Vertical bitmap build from the compressed rows.  Workgroup (wx, ry) owns the
// WT-word column block wx and the rank slice [ry*R, ry*R+R): it ORs bits into an
// LDS tile with ds_or_b32, then writes each rank's WT words (coalesced per row).
// Column c holds compressed row src[c] (src == nullptr: identity; -1: padding).
// Every word of [F1][Wp] is written, so the output needs no zeroing.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_build_bitmaps(
    const int64_t* __restrict__ roff, const int32_t* __restrict__ ranks, const int32_t* __restrict__ src,
    int64_t ncols, int32_t F1, int64_t Wp, int WT, int R, uint64_t* __restrict__ bm,
    const int32_t* __restrict__ item_map, const int32_t* __restrict__ used) {
  extern __shared__ uint32_t tile[];   // [R][2*WT]
  const int hw = 2 * WT;
  // output rows [u0, u1); with an item map (u = item_map[rank], used[] = sorted ranks of
  // the mapped items) the rank window is [used[u0], used[u1]) and rows are u - u0
  const int u0 = blockIdx.y * R;
  const int u1 = min(F1, u0 + R);
  const int nr = u1 - u0;
  const int r0 = item_map ? used[u0] : u0;
  const int r1 = item_map ? (u1 < F1 ? used[u1] : 0x7FFFFFFF) : u1;
  for (int i = threadIdx.x; i < nr * hw; i += blockDim.x) tile[i] = 0;
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * WT * 64;
  for (int j = threadIdx.x; j < WT * 64; j += blockDim.x) {
    const int64_t c = c0 + j;
    if (c >= ncols) break;
    const int64_t row = src ? (int64_t)src[c] : c;
    if (row < 0) continue;
    int64_t s = roff[row];
    const int64_t e = roff[row + 1];
    // ranks are sorted: skip to r0, stop at r1
    int64_t lo = s, hi = e;
    while (lo < hi) {
      int64_t mid = (lo + hi) >> 1;
      if (ranks[mid] < r0) lo = mid + 1; else hi = mid;
    }
    const uint32_t bit = 1u << (j & 31);
    const int word = j >> 5;
    for (int64_t i = lo; i < e; ++i) {
      const int r = ranks[i];
      if (r >= r1) break;
      const int u = item_map ? item_map[r] : r;
      if (u >= 0) atomicOr(&tile[(u - u0) * hw + word], bit);
    }
  }
  __syncthreads();
  uint32_t* out = reinterpret_cast<uint32_t*>(bm);
  const int64_t base = c0 >> 5;
  for (int i = threadIdx.x; i < nr * hw; i += blockDim.x) {
    const int r = i / hw, w = i - r * hw;
    out[(int64_t)(u0 + r) * (2 * Wp) + base + w] = tile[i];
  }
}

// ---------------------------------------------------------------------------
// Transaction trimming before level k (an item matters only if it occurs in a
// level-k candidate, a row only if it keeps >= k such items), as count -> scan
// of block sums -> emit, wave-cooperative: a wave owns
// 64 consecutive rows and streams their (contiguous) ranks 64 at a time,
// coalesced; lane l also owns row l.  The alive table is in LDS.
//   count: row l's alive count = sum over windows of popc(ballot(alive) & the
//          window lanes inside row l);
//   emit:  a rank's slot in its new row = the row's alive ranks in earlier
//          windows (carried by the row's owner lane) + alive lanes of the same
//          row below it in this window (ballot prefix), so the new CSR is
//          written without any staging buffer.
// Rows are dropped when they keep < min_len items (or weight 0).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int block_excl_scan256(int v, int* wtot, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int incl = wave_scan_incl_dpp(v);
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  int before = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) { before += k < w ? wtot[k] : 0; tot += wtot[k]; }
  __syncthreads();
  *total = tot;
  return before + incl - v;
}

__device__ __forceinline__ unsigned long long lane_range(int lo, int hi) {   // bits [lo, hi), 0 <= lo, hi <= 64
  const unsigned long long h = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
  const unsigned long long l = lo >= 64 ? ~0ull : ((1ull << lo) - 1);
  return hi > lo ? (h & ~l) : 0ull;
}

constexpr int kTrimAliveLds = 32768;

struct TrimWave {
  int64_t base;   // first rank position of the wave's rows
  int n;          // ranks in the wave's rows
  int srel, erel; // this lane's row [srel, erel) relative to base
};

__device__ __forceinline__ TrimWave trim_wave_setup(const int64_t* __restrict__ roff, int64_t row0, int64_t T) {
  const int lane = threadIdx.x & 63;
  TrimWave tw;
  tw.base = roff[row0];
  const int64_t end = roff[min(row0 + 64, T)];
  tw.n = (int)(end - tw.base);
  tw.srel = (int)(roff[min(row0 + lane, T)] - tw.base);
  tw.erel = (int)(roff[min(row0 + lane + 1, T)] - tw.base);
  return tw;
}

template <bool kLdsAlive>
__global__ __launch_bounds__(256) void k_trim_scan_count(const int64_t* __restrict__ roff,
                                                         const int32_t* __restrict__ ranks, int64_t T,
                                                         const int8_t* __restrict__ alive, int F1, int min_len,
                                                         const int32_t* __restrict__ wrow, int32_t* __restrict__ cnt,
                                                         int32_t* __restrict__ bk_rows, int32_t* __restrict__ bk_nnz) {
  extern __shared__ int8_t al[];                 // F1 bytes when kLdsAlive
  __shared__ int wtot[4];
  if (kLdsAlive)
    for (int i = threadIdx.x; i < F1; i += blockDim.x) al[i] = alive[i];
  __syncthreads();
  const int8_t* A = kLdsAlive ? al : alive;
  const int lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63);
  const int64_t row = row0 + lane;
  int c = 0;
  if (row0 < T) {
    const TrimWave tw = trim_wave_setup(roff, row0, T);
    constexpr int U = 8;                           // windows in flight per wave (memory-level parallelism)
    for (int p0 = 0; p0 < tw.n; p0 += 64 * U) {
      int32_t r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + 64 * u + lane;
        r[u] = p < tw.n ? ranks[tw.base + p] : 0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q0 = p0 + 64 * u;
        const unsigned long long b = __ballot(q0 + lane < tw.n && A[r[u]] != 0);
        c += __popcll(b & lane_range(max(tw.srel - q0, 0), min(max(tw.erel - q0, 0), 64)));
      }
    }
  }
  const bool keep = row < T && c >= min_len && (!wrow || wrow[row] > 0);
  if (row < T) cnt[row] = keep ? c : -1;
  int tr, tn;
  (void)block_excl_scan256(keep ? 1 : 0, wtot, &tr);
  (void)block_excl_scan256(keep ? c : 0, wtot, &tn);
  if (threadIdx.x == 0) { bk_rows[blockIdx.x] = tr; bk_nnz[blockIdx.x] = tn; }
}

constexpr int kTrimHist = 256;

template <bool kLdsAlive>
__global__ __launch_bounds__(256) void k_trim_emit(const int64_t* __restrict__ roff, const int32_t* __restrict__ ranks,
                                                   const int8_t* __restrict__ alive, int F1, int64_t T,
                                                   const int32_t* __restrict__ cnt, const int64_t* __restrict__ base_rows,
                                                   const int64_t* __restrict__ base_nnz, int64_t* __restrict__ nroff,
                                                   int32_t* __restrict__ nranks, int32_t* __restrict__ kept,
                                                   int64_t* __restrict__ hist) {
  extern __shared__ int8_t al[];                 // F1 bytes when kLdsAlive
  __shared__ uint32_t hs[kTrimHist];
  __shared__ unsigned long long sw[4 * 4];        // per-wave window_starts scratch
  __shared__ int wtot[4];
  if (kLdsAlive)
    for (int i = threadIdx.x; i < F1; i += blockDim.x) al[i] = alive[i];
  hs[threadIdx.x] = 0;
  const int8_t* A = kLdsAlive ? al : alive;
  const int lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63);
  const int64_t row = row0 + lane;
  const int32_t c = row < T ? cnt[row] : -1;
  const bool keep = c >= 0;
  int nk, nn;
  const int rk = block_excl_scan256(keep ? 1 : 0, wtot, &nk);     // (contains __syncthreads)
  const int ok = block_excl_scan256(keep ? c : 0, wtot, &nn);
  const int64_t obase = base_nnz[blockIdx.x] + ok;                 // this row's first new slot
  if (keep) {
    nroff[base_rows[blockIdx.x] + rk] = obase;
    kept[base_rows[blockIdx.x] + rk] = (int32_t)row;
    atomicAdd(&hs[min(c, kTrimHist - 1)], 1u);
  }
  if (row0 < T && __ballot(keep) != 0ull) {
    const TrimWave tw = trim_wave_setup(roff, row0, T);
    // next output slot of my row (row owner view), -1 when the row is dropped
    int64_t nxt = keep ? obase : -1;
    unsigned long long* words = sw + (threadIdx.x >> 6) * 4;
    const unsigned long long le = lanes_le_mask();
    int cs = 0;                                                    // row starts before the window
    constexpr int U = 4;
    for (int p0 = 0; p0 < tw.n; p0 += 64 * U) {
      int32_t r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + 64 * u + lane;
        r[u] = p < tw.n ? ranks[tw.base + p] : 0;
      }
      unsigned long long S[U];
      window_starts<U>(words, tw.srel, p0, S);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q0 = p0 + 64 * u, p = q0 + lane;
        const bool a = p < tw.n && A[r[u]] != 0;
        const unsigned long long B = __ballot(a);
        const unsigned long long sle = S[u] & le;
        const int owner = cs + __popcll(sle) - 1;
        const int rs = sle ? 63 - __clzll(sle) : 0;                // my row's first lane in this window
        const int64_t dst = __shfl(nxt, owner & 63, 64);
        if (a && dst >= 0) nranks[dst + __popcll(B & lane_range(rs, lane))] = r[u];
        if (nxt >= 0) nxt += __popcll(B & lane_range(max(tw.srel - q0, 0), min(max(tw.erel - q0, 0), 64)));
        cs += __popcll(S[u]);
      }
    }
  }
  __syncthreads();
  // 64 striped copies (summed by the caller): one shared copy would serialise
  // ~10 bins x every block on a few L2 lines
  if (hist && hs[threadIdx.x])
    atomicAdd((unsigned long long*)&hist[(blockIdx.x & 63) * kTrimHist + threadIdx.x], (unsigned long long)hs[threadIdx.x]);
}


// ---------------------------------------------------------------------------
// Two-pass fused compression (short rows).  Replaces per-row counts + a
// 100M-entry nonzero/cumsum in torch: each workgroup owns 256 consecutive
// input rows (one contiguous CSR span, loaded coalesced into LDS and mapped
// through the LUT once per pass).
//   pass 1 (k_cmp_agg):  per-workgroup (kept rows, kept items) + the kept-row
//                        length histogram (clamped to 255);
//   host:                exclusive scan of the 2 x nWG aggregates;
//   pass 2 (k_cmp_emit): block scans give every kept row its index and output
//                        offset; writes kept[], roff[], and the sorted ranks of
//                        rows <= 16 tokens (register bitonic network), staged
//                        through LDS for coalesced stores; longer rows are
//                        appended to an overflow list for the next tiers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cmp_block_scan2(int a, int b, int& ea, int& eb, int& ta, int& tb, int* sh) {
  // exclusive scans of a and b over the 256-thread workgroup (4 waves)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ia = wave_scan_incl_dpp(a), ib = wave_scan_incl_dpp(b);
  if (lane == 63) { sh[w] = ia; sh[4 + w] = ib; }
  __syncthreads();
  int pa = 0, pb = 0;
  for (int k = 0; k < w; ++k) { pa += sh[k]; pb += sh[4 + k]; }
  ta = sh[0] + sh[1] + sh[2] + sh[3];
  tb = sh[4] + sh[5] + sh[6] + sh[7];
  ea = pa + ia - a;
  eb = pb + ib - b;
}

// Loads the workgroup's span into LDS as mapped ranks (0xFFFFFFFF = not frequent).
// 16 KB spans (4096 tokens per 256 rows: every T10I4 workgroup) keep 8
// workgroups resident per CU, which hides the dependent offset -> token -> LUT
// loads of these short-lived workgroups.
constexpr int kCmpSpan = 4096;
constexpr int kCmpPer = kCmpSpan / 256;
__device__ __forceinline__ bool cmp_stage(uint32_t* buf, const int32_t* __restrict__ items,
                                          const int32_t* __restrict__ lut, int64_t base, int64_t n_in) {
  if (n_in > kCmpSpan) return false;
  int32_t v[kCmpPer];
#pragma unroll
  for (int k = 0; k < kCmpPer; ++k) {
    const int64_t i = threadIdx.x + k * 256;
    v[k] = i < n_in ? items[base + i] : 0;
  }
#pragma unroll
  for (int k = 0; k < kCmpPer; ++k) {
    const int64_t i = threadIdx.x + k * 256;
    if (i < n_in) v[k] = lut[v[k]];
  }
#pragma unroll
  for (int k = 0; k < kCmpPer; ++k) {
    const int64_t i = threadIdx.x + k * 256;
    if (i < n_in) buf[i] = v[k] < 0 ? 0xFFFFFFFFu : (uint32_t)v[k];
  }
  return true;
}

constexpr int kCmpN = 16;          // rows of <= kCmpN tokens are sorted by k_cmp_emit
constexpr int kCmpStripes = 64;    // histogram copies
// Rows of kCmpN < L <= kCmpMid tokens in a staged span are sorted by k_cmp_emit too,
// with wave-wide bitonic networks on the span already in LDS (rows of <= 32 tokens
// two per network, one per 32-lane half) -- at most kCmpMidPerWave per wave, the
// rest go to the overflow tiers.  (The thread-per-row 64-token tier,
// k_compress_regs<64>, gathers every such row again from HBM: 1.6-1.7 ms per
// T10I4D100M run.)
constexpr int kCmpMid = 64;
constexpr int kCmpMidPerWave = 8;

// the same rows in k_cmp_agg and k_cmp_emit (their overflow counts must agree)
__device__ __forceinline__ bool cmp_mid(bool kept, int64_t L, bool staged) {
  const bool cand = kept && staged && L > kCmpN && L <= kCmpMid;
  const unsigned long long m = __ballot(cand);
  return cand && __popcll(m & (lanes_le_mask() >> 1)) < kCmpMidPerWave;
}

// Two ascending bitonic sorts at once (independent exchange chains interleave):
// one value per lane of a and of b; KMAX = 64 sorts each across the wave, 32 sorts
// each 32-lane half on its own (the last merge stage ascends in both halves).
// (DPP / ds_swizzle exchanges instead of ds_bpermute measured no faster: 3.9 vs 3.8 ms)
template <int KMAX>
__device__ __forceinline__ void wave_sort2(uint32_t& a, uint32_t& b) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 2; k <= KMAX; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint32_t oa = (uint32_t)__shfl_xor((int)a, j, 64);
      const uint32_t ob = (uint32_t)__shfl_xor((int)b, j, 64);
      const bool up = k == KMAX || (lane & k) == 0;
      const bool keep_min = up == ((lane & j) == 0);
      a = keep_min ? min(a, oa) : max(a, oa);
      b = keep_min ? min(b, ob) : max(b, ob);
    }
  }
}

// the i-th set bit of a wave-uniform mask (i < popcount)
__device__ __forceinline__ int nth_bit(unsigned long long m, int i) {
  for (; i > 0; --i) m &= m - 1;
  return __builtin_ctzll(m);
}

// a frequent rank's count in its row's packed 256-rank block counts (byte b = block b;
// exact while a row holds < 256 items of a block, the pair layout's u8 guard)
__device__ __forceinline__ unsigned long long blk_inc(uint32_t v) {
  return v == 0xFFFFFFFFu ? 0ull : 1ull << ((v >> 8) << 3);
}

// per-workgroup totals of the rows' block counts: aggb[b * gridDim.x + workgroup]
__device__ __forceinline__ void cmp_block_totals(unsigned long long pc, int nb, int32_t* __restrict__ aggb) {
  __shared__ int bs[8][4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b >= nb) break;
    const int t = wave_last(wave_scan_incl_dpp((int)((pc >> (8 * b)) & 255)));
    if (lane == 0) bs[b][w] = t;
  }
  __syncthreads();
  if ((int)threadIdx.x < nb)
    aggb[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] =
        bs[threadIdx.x][0] + bs[threadIdx.x][1] + bs[threadIdx.x][2] + bs[threadIdx.x][3];
}

__global__ __launch_bounds__(256) void k_cmp_agg(const int64_t* __restrict__ off, const int32_t* __restrict__ items,
                                                 const int32_t* __restrict__ lut, int64_t n,
                                                 int32_t* __restrict__ agg, uint32_t* __restrict__ hist,
                                                 int32_t* __restrict__ aggb, int nb) {
  __shared__ uint32_t buf[kCmpSpan];
  __shared__ uint32_t lh[256];
  __shared__ int sh[8];
  const int64_t r0 = (int64_t)blockIdx.x * 256, r1 = min(n, r0 + 256);
  const int64_t r = r0 + threadIdx.x;
  lh[threadIdx.x] = 0;
  const int64_t base = off[r0], n_in = off[r1] - base;
  const int64_t s = r < r1 ? off[r] : 0, e = r < r1 ? off[r + 1] : 0;
  const bool staged = cmp_stage(buf, items, lut, base, n_in);
  __syncthreads();
  int c = 0;
  unsigned long long pc = 0;
  for (int64_t i = s; i < e; ++i) {
    const uint32_t v = staged ? buf[i - base] : (uint32_t)lut[items[i]];
    c += v != 0xFFFFFFFFu;
    if (aggb) pc += blk_inc(v);
  }
  const int kept = c >= 2;
  if (aggb) cmp_block_totals(kept ? pc : 0ull, nb, aggb);
  int ea, eb, ta, tb;
  cmp_block_scan2(kept, kept ? c : 0, ea, eb, ta, tb, sh);
  if (kept) atomicAdd(&lh[min(c, 255)], 1u);
  const bool mid = cmp_mid(kept, e - s, staged);
  const unsigned long long ob = __ballot(kept && e - s > kCmpN && !mid);
  __shared__ int ov_w[4];
  if ((threadIdx.x & 63) == 0) ov_w[threadIdx.x >> 6] = __popcll(ob);
  __syncthreads();
  if (threadIdx.x == 0) {
    agg[3 * blockIdx.x] = ta; agg[3 * blockIdx.x + 1] = tb;
    agg[3 * blockIdx.x + 2] = ov_w[0] + ov_w[1] + ov_w[2] + ov_w[3];
  }
  // striped histogram copies: 390K workgroups adding into one 256-bin row would
  // serialise on a few hot addresses (~10 distinct row lengths)
  if (lh[threadIdx.x]) atomicAdd(&hist[(blockIdx.x & (kCmpStripes - 1)) * 256 + threadIdx.x], lh[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_cmp_emit(const int64_t* __restrict__ off, const int32_t* __restrict__ items,
                                                  const int32_t* __restrict__ lut, int64_t n,
                                                  const int64_t* __restrict__ pre_rows,
                                                  const int64_t* __restrict__ pre_items,
                                                  const int64_t* __restrict__ pre_over,
                                                  int32_t* __restrict__ kept_out, int64_t* __restrict__ roff,
                                                  int32_t* __restrict__ ranks, int32_t* __restrict__ over,
                                                  uint8_t* __restrict__ bcnt, int nb,
                                                  const int64_t* __restrict__ preb, uint8_t* __restrict__ lr,
                                                  int64_t lr_cap, int64_t* __restrict__ lbase,
                                                  int64_t* __restrict__ ovb) {
  constexpr int N = kCmpN;
  __shared__ uint32_t buf[kCmpSpan];
  __shared__ int sh[8];
  // fused pair layout (lr != null): row x's block-b segment start in the workgroup's
  // block-b span minus the row's first block-b index, tabx[x * nb + b]
  extern __shared__ int32_t tabx[];
  __shared__ int64_t wgb[8];
  const bool blk = bcnt != nullptr;
  const int64_t r0 = (int64_t)blockIdx.x * 256, r1 = min(n, r0 + 256);
  const int64_t r = r0 + threadIdx.x;
  const int64_t base = off[r0], n_in = off[r1] - base;
  const int64_t s = r < r1 ? off[r] : 0, e = r < r1 ? off[r + 1] : 0;
  const int64_t xr0 = pre_rows[blockIdx.x], obase = pre_items[blockIdx.x];
  const bool staged = cmp_stage(buf, items, lut, base, n_in);
  __syncthreads();
  const int64_t L = e - s;
  uint32_t a[N];
  int c = 0;
  unsigned long long pc = 0;      // packed 256-rank block counts of the row (blk_inc)
  if (L <= N) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      uint32_t v = 0xFFFFFFFFu;
      if (j < L) v = staged ? buf[s - base + j] : (uint32_t)lut[items[s + j]];
      a[j] = v;
      c += v != 0xFFFFFFFFu;
      if (blk) pc += blk_inc(v);
    }
  } else {
    for (int64_t i = s; i < e; ++i) {
      const uint32_t v = staged ? buf[i - base] : (uint32_t)lut[items[i]];
      c += v != 0xFFFFFFFFu;
      if (blk) pc += blk_inc(v);
    }
  }
  const int kept = c >= 2;
  const bool mid = cmp_mid(kept, L, staged);
  const int ov = kept && L > N && !mid;
  int ea, eb, ta, tb;
  cmp_block_scan2(kept, kept ? c : 0, ea, eb, ta, tb, sh);
  // overflow rows go to their slot of the scanned per-workgroup counts (no atomics:
  // a counter shared by every workgroup serialises), ballot ranks inside the waves
  __shared__ int ov_w[4];
  const int w = threadIdx.x >> 6;
  const unsigned long long ob = __ballot(ov);
  if ((threadIdx.x & 63) == 0) ov_w[w] = __popcll(ob);
  __syncthreads();
  const int64_t ov_base = pre_over[blockIdx.x];
  const int64_t xk = xr0 + ea;
  int64_t ovi = -1;
  if (kept) {
    kept_out[xk] = (int32_t)r;
    roff[xk + 1] = obase + eb + c;
    if (ov) {
      int64_t before = ov_base;
      for (int k = 0; k < w; ++k) before += ov_w[k];
      ovi = before + __popcll(ob & (lanes_le_mask() >> 1));
      over[ovi] = (int32_t)xk;
    }
  }
  const bool mine = kept && L <= N;
  if (mine) bitonic_regs<N>(a);
  if (blk) {
    // per-row item counts of the pair kernel's 256-rank blocks, bcnt[b * T + row]
    // (T = kept rows, the scan total), counted by value while the row was loaded.
    // Fused pair layout (lr): every block's data in kept-row order, block-major --
    // the row's block-b segment starts at the workgroup's block-b offset (preb: the
    // scan of k_cmp_agg's per-workgroup totals) + the block scan below; the first
    // row of every 64-row batch also writes the batch's base (pair_queue16's base).
    const int64_t bld = pre_rows[gridDim.x];
    const unsigned long long pk = kept ? pc : 0ull;
    const unsigned long long fpre = (pk << 8) * 0x0101010101010101ull;   // byte b: items in blocks < b
    __shared__ int bs2[8][4];
    const int lane_ = threadIdx.x & 63;
    int exb[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      exb[b] = 0;
      if (b < nb) {
        const int cb = (int)((pk >> (8 * b)) & 255);
        const int incl = wave_scan_incl_dpp(cb);
        exb[b] = incl - cb;
        if (lane_ == 63) bs2[b][w] = incl;
      }
    }
    if (lr && (int)threadIdx.x < nb) wgb[threadIdx.x] = preb[(int64_t)threadIdx.x * gridDim.x + blockIdx.x];
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (b < nb) {
        for (int k = 0; k < w; ++k) exb[b] += bs2[b][k];
        if (kept) bcnt[(int64_t)b * bld + xk] = (uint8_t)(pk >> (8 * b));
        if (lr) {
          const int t = exb[b] - (int)((fpre >> (8 * b)) & 255);
          tabx[threadIdx.x * nb + b] = t;
          if (kept && (xk & 63) == 0) lbase[(int64_t)b * ((bld + 63) >> 6) + (xk >> 6)] = wgb[b] + exb[b];
          if (ovi >= 0) ovb[ovi * nb + b] = wgb[b] + t;
        }
      }
    }
    if (lr && mine) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j < c) {
          const int b = (int)(a[j] >> 8);
          // b < nb and the position inside lr hold by construction (a frequent rank is
          // < F1 <= 256 nb; the layout's spans are the scanned block counts): no guards
          // in this 16-step loop
          lr[wgb[b] + (int64_t)(tabx[threadIdx.x * nb + b] + j)] = (uint8_t)a[j];
        }
      }
    }
  }
  // mid rows (staged, kCmpN < L <= 64): wave-wide bitonic sorts on the input span
  // while it is still in LDS.  Slots: rows of <= 32 tokens two per slot (one per
  // 32-lane half), then longer rows one per slot; slots are sorted two at a time.
  // Lane l of a slot holds element l (l & 31 in halves) of its row.
  const int lane = threadIdx.x & 63;
  const unsigned long long m32 = __ballot(mid && L <= 32), m64 = __ballot(mid && L > 32);
  const int n32 = __popcll(m32), s32 = (n32 + 1) >> 1, nslot = s32 + __popcll(m64);
  // the row (lane id in the wave) this lane holds in slot t, -1: none
  auto slot_row = [&](int t) -> int {
    if (t < s32) {
      const int i = 2 * t + (lane >> 5);
      return i < n32 ? nth_bit(m32, i) : -1;
    }
    return t < nslot ? nth_bit(m64, t - s32) : -1;
  };
  uint32_t midv[kCmpMidPerWave];
#pragma unroll
  for (int t = 0; t < kCmpMidPerWave; ++t) {
    midv[t] = 0xFFFFFFFFu;
    if (t < nslot) {                             // wave-uniform: every lane takes part in the shuffles
      const int rw = slot_row(t);
      const int src = rw < 0 ? 0 : rw;
      const int idx = t < s32 ? (lane & 31) : lane;
      const int rs = __shfl((int)(s - base), src, 64);
      const int rl = __shfl((int)L, src, 64);
      if (rw >= 0 && idx < rl) midv[t] = buf[rs + idx];
    }
  }
#pragma unroll
  for (int t = 0; t < kCmpMidPerWave; t += 2) {
    if (t < nslot) {
      if (t + 1 < s32) {
        wave_sort2<32>(midv[t], midv[t + 1]);
      } else if (t >= s32) {
        wave_sort2<64>(midv[t], midv[t + 1]);
      } else {                                   // slot t: halves; slot t + 1 (if any): a long row
        uint32_t none = 0xFFFFFFFFu;
        wave_sort2<32>(midv[t], none);
        if (t + 1 < nslot) wave_sort2<64>(midv[t + 1], none);
      }
    }
  }
  __syncthreads();   // everyone is done reading the input span
  if (staged && tb <= kCmpSpan) {
    if (mine) {
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (j < c) buf[eb + j] = a[j];
    }
    {
      // mid rows into the staged output (their rows are always staged), and into the
      // fused pair layout (their block counts were written with the short rows')
#pragma unroll
      for (int t = 0; t < kCmpMidPerWave; ++t) {
        if (t < nslot) {                         // wave-uniform
          const int rw = slot_row(t);
          const int src = rw < 0 ? 0 : rw;
          const int idx = t < s32 ? (lane & 31) : lane;
          const int rc = __shfl(c, src, 64), reb = __shfl(eb, src, 64);
          const bool in = rw >= 0 && idx < rc;
          if (in) {
            buf[reb + idx] = midv[t];
            if (lr) {
              const int b = (int)(midv[t] >> 8);
              lr[wgb[b] + (int64_t)(tabx[(w * 64 + rw) * nb + b] + idx)] = (uint8_t)midv[t];
            }
          }
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < tb; i += blockDim.x) ranks[obase + i] = (int32_t)buf[i];
  } else if (mine) {
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (j < c) ranks[obase + eb + j] = (int32_t)a[j];
  }
}
// Block counts of the rows the emit pass left to later tiers (rows[i] = row id):
// thread per row over its final ranks (counts need no order).
__global__ __launch_bounds__(256) void k_block_counts_rows(const int64_t* __restrict__ roff,
                                                           const int32_t* __restrict__ ranks,
                                                           const int32_t* __restrict__ rows, int64_t nrows,
                                                           uint8_t* __restrict__ bcnt, int64_t bld, int nb,
                                                           const int8_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows || (flags && !flags[i])) return;
  const int64_t x = rows[i];
  int c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t k = roff[x], e = roff[x + 1]; k < e; ++k) {
    const int b = ranks[k] >> 8;
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] += b == q;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (q < nb) bcnt[(int64_t)q * bld + x] = (uint8_t)min(c[q], 255);
}

// bsum[b * nbatch + q] = items of 64-row batch q in block b (rows >= T count 0).
// A wave takes 16 batches of one block: lane l sums the 16 count bytes of rows
// 64q + 16(l % 4) .. +16 of batch q = q0 + l / 4 (four dword loads; a block's bytes
// start at b * bld, so they may be unaligned), then a quad DPP sum per batch.
__global__ __launch_bounds__(256) void k_block_bsum(const uint8_t* __restrict__ bcnt, int64_t bld, int64_t T,
                                                    int nb, int64_t nbatch, int64_t* __restrict__ bsum) {
  const int64_t ng = (nbatch + 15) / 16;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= nb * ng) return;
  const int lane = threadIdx.x & 63;
  const int64_t b = t / ng, q = (t - b * ng) * 16 + (lane >> 2);
  const int64_t x0 = q * 64 + 16 * (lane & 3);
  const uint8_t* src = bcnt + b * bld + x0;
  uint32_t s = 0;
  if (q < nbatch) {
    if (x0 + 16 <= T) {
      uint32_t acc = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t d;
        __builtin_memcpy(&d, src + 4 * k, 4);
        acc += (d & 0x00FF00FFu) + ((d >> 8) & 0x00FF00FFu);
      }
      s = (acc & 0xFFFFu) + (acc >> 16);
    } else {
      for (int k = 0; k < 16; ++k)
        if (x0 + k < T) s += src[k];
    }
  }
  s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  s += (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  if ((lane & 3) == 0 && q < nbatch) bsum[b * nbatch + q] = s;
}

}  // namespace fa

using namespace fa;

FA_API int fa_hip_block_counts_rows(const int64_t* roff, const int32_t* ranks, const int32_t* rows, int64_t nrows,
                                    uint8_t* bcnt, int64_t bld, int nb, const int8_t* flags, hipStream_t st) {
  if (nrows <= 0) return 0;
  if (nb > 8) return 1;
  hipLaunchKernelGGL(k_block_counts_rows, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, st, roff, ranks, rows,
                     nrows, bcnt, bld, nb, flags);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_block_bsum(const uint8_t* bcnt, int64_t bld, int64_t T, int nb, int64_t* bsum, hipStream_t st) {
  if (T <= 0) return 0;
  const int64_t nbatch = (T + 63) / 64;
  const int64_t ng = (nbatch + 15) / 16;
  hipLaunchKernelGGL(k_block_bsum, dim3((unsigned)((nb * ng + 3) / 4)), dim3(256), 0, st, bcnt, bld, T, nb,
                     nbatch, bsum);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_histogram(const int32_t* items, int64_t nnz, int32_t V, uint32_t* counts,
                            hipStream_t st) {
  if (nnz <= 0) return 0;
  int64_t blocks = std::min<int64_t>((nnz + 256 * 16 - 1) / (256 * 16), 2048);
  const bool aligned = ((uintptr_t)items & 15) == 0;
  dim3 g((unsigned)blocks), b(256);
  if (V <= kLdsBins) {
    const int nrep = V * 4 <= kLdsBins / 4 ? 4 : 1;   // per-wave copies while they stay <= 16 KB
    const size_t lds = (size_t)V * nrep * 4;
    if (aligned) hipLaunchKernelGGL((k_histogram<true, true>), g, b, lds, st, items, nnz, V, nrep, counts);
    else hipLaunchKernelGGL((k_histogram<true, false>), g, b, lds, st, items, nnz, V, nrep, counts);
  } else {
    if (aligned) hipLaunchKernelGGL((k_histogram<false, true>), g, b, 0, st, items, nnz, V, 1, counts);
    else hipLaunchKernelGGL((k_histogram<false, false>), g, b, 0, st, items, nnz, V, 1, counts);
  }
  FA_LAUNCH_RET();
}

// F1 ranking + id -> rank LUT on the device (k_f1_rank); hist int64 [V], V <= kF1RankMax.
FA_API int fa_hip_f1_rank(const int64_t* hist, int32_t V, int64_t thr, int numeric, int32_t* lut, int64_t* pack,
                          hipStream_t st) {
  if (V < 1 || V > kF1RankMax || thr < 1) return 1;
  hipLaunchKernelGGL(k_f1_rank, dim3((unsigned)((V + 255) / 256)), dim3(256), 0, st, hist, V, thr, numeric, lut, pack);
  FA_LAUNCH_RET();
}

// Long documents: one wave per row, a ballot per 64 tokens.
__global__ __launch_bounds__(256) void k_txn_freq_count_wave(const int64_t* __restrict__ off,
                                                             const int32_t* __restrict__ items, int64_t n,
                                                             const int32_t* __restrict__ lut,
                                                             int32_t* __restrict__ cnt) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t t = (int64_t)blockIdx.x * 4 + w; t < n; t += nw) {
    const int64_t s = off[t], L = off[t + 1] - s;
    int32_t c = 0;
    for (int64_t j0 = 0; j0 < L; j0 += 256) {
      int32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = j0 + lane + 64 * k;
        v[k] = j < L ? items[s + j] : -1;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) c += __popcll(__ballot(v[k] >= 0 && lut[v[k]] >= 0));
    }
    if (lane == 0) cnt[t] = c;
  }
}

static int f1_grid(int64_t nnz) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(256, (nnz + 1024 * 64 - 1) / (1024 * 64)));
}

// partial: [f1_grid(nnz)][2 * 16384] u32; returns the number of partial sketches via *nwg.
FA_API int fa_hip_f1_sketch(const int32_t* items, int64_t nnz, uint32_t* partial, int* nwg, hipStream_t st) {
  const int g = f1_grid(nnz);
  *nwg = g;
  if (nnz <= 0) return 0;
  if (((uintptr_t)items & 15) == 0) hipLaunchKernelGGL(k_f1_sketch<true>, dim3(g), dim3(1024), 0, st, items, nnz, partial);
  else hipLaunchKernelGGL(k_f1_sketch<false>, dim3(g), dim3(1024), 0, st, items, nnz, partial);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_f1_exact(const int32_t* items, int64_t nnz, const int32_t* keys, int log_s, uint32_t* counts,
                           hipStream_t st) {
  if (nnz <= 0) return 0;
  if (log_s < 6 || log_s > kSkLog) return 1;
  const int g = f1_grid(nnz);
  if (((uintptr_t)items & 15) == 0)
    hipLaunchKernelGGL(k_f1_exact<true>, dim3(g), dim3(1024), 0, st, items, nnz, keys, log_s, counts);
  else
    hipLaunchKernelGGL(k_f1_exact<false>, dim3(g), dim3(1024), 0, st, items, nnz, keys, log_s, counts);
  FA_LAUNCH_RET();
}

// Frequent tokens per row, wave-cooperative (rows of ~8-48 tokens): a wave owns 64
// consecutive rows, streams their contiguous tokens 64 at a time (four windows in
// flight, coalesced), and row l (lane l) adds popc(ballot(frequent) & the window lanes
// inside its span).  k_txn_freq_count_span stages 64 tokens per thread in registers
// and flags in LDS instead: 14 ms for T40I10D100M's 4 G tokens, ~1.1 TB/s.
__global__ __launch_bounds__(256) void k_txn_freq_count_wv(const int64_t* __restrict__ off,
                                                           const int32_t* __restrict__ items, int64_t n,
                                                           const int32_t* __restrict__ lut, int32_t* __restrict__ cnt) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t x0 = q * 64;
  if (x0 >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t base = off[x0];
  const int nt = (int)(off[min(x0 + 64, n)] - base);
  const int srel = (int)(off[min(x0 + lane, n)] - base);
  const int erel = (int)(off[min(x0 + lane + 1, n)] - base);
  int c = 0;
  constexpr int U = 8;
  // the next U windows' tokens are loaded before this step's LUT gathers: the token
  // stream and the gathers overlap instead of alternating
  int v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = 64 * u + lane < nt ? items[base + 64 * u + lane] : -1;
  for (int p0 = 0; p0 < nt; p0 += 64 * U) {
    int nv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + 64 * (U + u) + lane;
      nv[u] = p < nt ? items[base + p] : -1;
    }
    int lv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) lv[u] = v[u] >= 0 ? lut[v[u]] : -1;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool f = lv[u] >= 0;
      const unsigned long long b = __ballot(f);
      const int lo = max(srel - (p0 + 64 * u), 0), hi = min(erel - (p0 + 64 * u), 64);
      if (hi > lo) {
        const unsigned long long m = (hi >= 64 ? ~0ull : ((1ull << hi) - 1)) & ~((1ull << lo) - 1);
        c += __popcll(b & m);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = nv[u];
  }
  if (x0 + lane < n) cnt[x0 + lane] = c;
}

FA_API int fa_hip_txn_freq_count(const int64_t* off, const int32_t* items, int64_t n, int64_t nnz,
                                 const int32_t* lut, int32_t* cnt, hipStream_t st) {
  if (n <= 0) return 0;
  if (nnz > 8 * n && nnz <= 48 * n) {
    hipLaunchKernelGGL(k_txn_freq_count_wv, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, off, items, n, lut,
                       cnt);
    FA_LAUNCH_RET();
  }
  if (nnz > 48 * n)
    hipLaunchKernelGGL(k_txn_freq_count_wave, dim3((unsigned)std::min<int64_t>((n + 3) / 4, 8192)), dim3(256), 0, st,
                       off, items, n, lut, cnt);
  else if (nnz > 8 * n)
    hipLaunchKernelGGL(k_txn_freq_count_span<16384>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, off, items,
                       n, lut, cnt);
  else
    hipLaunchKernelGGL(k_txn_freq_count, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, off, items, n, lut, cnt);
  FA_LAUNCH_RET();
}

// tier: 16 / 64 register networks over `rows` (nullptr = all kept rows 0..nrows)
FA_API int fa_hip_compress_regs(int tier, const int64_t* off, const int32_t* items, const int32_t* lut,
                                const int32_t* rows, int64_t nrows, const int32_t* kept,
                                const int64_t* roff, int32_t* ranks, int8_t* over_flag, hipStream_t st) {
  if (nrows <= 0) return 0;
  dim3 g((unsigned)((nrows + 255) / 256));
  if (tier == 16)
    hipLaunchKernelGGL(k_compress_regs<16>, g, dim3(256), 0, st, off, items, lut, rows, nrows, kept, roff, ranks, over_flag);
  else if (tier == 32)
    hipLaunchKernelGGL(k_compress_regs<32>, g, dim3(256), 0, st, off, items, lut, rows, nrows, kept, roff, ranks, over_flag);
  else if (tier == 64)
    hipLaunchKernelGGL(k_compress_regs<64>, g, dim3(256), 0, st, off, items, lut, rows, nrows, kept, roff, ranks, over_flag);
  else
    return 1;
  FA_LAUNCH_RET();
}

// The 64-token tier that also writes the rows' 256-rank block counts (bcnt[b * bld + row]).
FA_API int fa_hip_compress_regs_bc(const int64_t* off, const int32_t* items, const int32_t* lut, const int32_t* rows,
                                   int64_t nrows, const int32_t* kept, const int64_t* roff, int32_t* ranks,
                                   int8_t* over_flag, uint8_t* bcnt, int64_t bld, int nb, hipStream_t st) {
  if (nrows <= 0) return 0;
  if (nb < 1 || nb > 8) return 1;
  hipLaunchKernelGGL(k_compress_regs<64>, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, st, off, items, lut,
                     rows, nrows, kept, roff, ranks, over_flag, bcnt, bld, nb);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_compress_staged(const int64_t* off, const int32_t* items, const int32_t* lut, int64_t T,
                                  const int32_t* kept, const int64_t* roff, int32_t* ranks, int8_t* over_flag,
                                  hipStream_t st) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(k_compress_staged<16>, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, st, off, items, lut,
                     T, kept, roff, ranks, over_flag);
  FA_LAUNCH_RET();
}

// 64-token staged tier for long-ish rows (64 KB input span per workgroup); rows
// longer than 64 tokens are flagged for the wave / LDS tiers
// F1 < 0xFFFF (ranks fit u16): the span staged as u16
FA_API int fa_hip_compress_staged64(const int64_t* off, const int32_t* items, const int32_t* lut, int64_t T,
                                    const int32_t* kept, const int64_t* roff, int32_t* ranks, int8_t* over_flag,
                                    int F1, hipStream_t st) {
  if (T <= 0) return 0;
  const dim3 g((unsigned)((T + 255) / 256));
  if (F1 > 0 && F1 < 0xFFFF)
    hipLaunchKernelGGL((k_compress_staged<64, 16384, uint16_t>), g, dim3(256), 0, st, off, items, lut, T, kept, roff,
                       ranks, over_flag);
  else
    hipLaunchKernelGGL((k_compress_staged<64, 16384>), g, dim3(256), 0, st, off, items, lut, T, kept, roff, ranks,
                       over_flag);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_compress_lds(const int64_t* off, const int32_t* items, const int32_t* lut,
                               const int32_t* rows, int64_t nrows, const int32_t* kept,
                               const int64_t* roff, int32_t* ranks, int32_t* too_long,
                               int32_t* n_too_long, hipStream_t st) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(k_compress_lds, dim3((unsigned)nrows), dim3(256), 0, st, off, items, lut, rows, kept, roff, ranks, too_long, n_too_long);
  FA_LAUNCH_RET();
}

// rows == nullptr: kept rows 0..nrows-1.  Requires F1 <= 65536.
// flags (optional): int8 [nrows], only rows with a non-zero flag are compressed
FA_API int fa_hip_compress_wave(const int64_t* off, const int32_t* items, const int32_t* lut, const int32_t* rows,
                                int64_t nrows, const int32_t* kept, const int64_t* roff, int32_t* ranks, int F1,
                                const int8_t* flags, hipStream_t st) {
  if (nrows <= 0) return 0;
  const int M = (F1 + 4095) / 4096;
  if (M > kCwMaxWords) return 1;
  const int64_t g = std::min<int64_t>((nrows + 3) / 4, 8192);
  hipLaunchKernelGGL(k_compress_wave, dim3((unsigned)g), dim3(256), 0, st, off, items, lut, rows, nrows, kept, roff,
                     ranks, std::max(M, 1), flags);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_row_hash(const int64_t* roff, const int32_t* ranks, int64_t T, int64_t* h1,
                           int64_t* h2, hipStream_t st) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(k_row_hash, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, st, roff, ranks, T, h1, h2);
  FA_LAUNCH_RET();
}

// ws: u32 [n_max + ceil(n_max / 256)] scratch (no zeroing); tail: int64 [2] (marked
// slots, hashed rows), tail[0] zeroed
FA_API int fa_hip_dedup_probe(const int64_t* roff, const int32_t* ranks, const int64_t* T_dev, int64_t n_max,
                              uint32_t* ws, unsigned long long* tail, hipStream_t st) {
  if (n_max <= 0) return 0;
  if (n_max > (int64_t)1 << 24) return 1;
  const int nparts = (int)((n_max + 255) / 256);
  uint32_t* part = ws + n_max;
  hipLaunchKernelGGL(k_dedup_probe, dim3((unsigned)nparts), dim3(256), 0, st, roff, ranks, T_dev, n_max, ws, part);
  hipLaunchKernelGGL(k_probe_count, dim3(kProbeBits / kProbeRange), dim3(1024), 0, st, ws, n_max, part, nparts, tail);
  FA_LAUNCH_RET();
}

// Wp must be a multiple of WT.  LDS = R * 2 * WT * 4 bytes.
FA_API int fa_hip_build_bitmaps_wave(const int64_t* roff, const int32_t* ranks, int64_t ncols, int32_t F1, int64_t Wp,
                                     int WT, uint64_t* bm, const int32_t* item_map, int blocked, hipStream_t st);

FA_API int fa_hip_build_bitmaps(const int64_t* roff, const int32_t* ranks, const int32_t* src,
                                int64_t ncols, int32_t F1, int64_t Wp, int WT, int R, uint64_t* bm,
                                const int32_t* item_map, const int32_t* used, int blocked, hipStream_t st) {
  if (F1 <= 0 || Wp <= 0) return 0;
  if (Wp % WT) return 1;
  // contiguous rows with every output row in one tile: the wave-cooperative build (count.hip)
  // (T40I10D100M: the full 998-item Gram bitmap 22.8 -> 14.1 ms per build, the used-item
  // subsets of the multi-pass levels ~1.9 ms).  blocked (the Gram's 8-word block layout,
  // count.hip BmView) only there: the caller checks that it applies.
  if (!src && R >= F1) {
    const int rc = fa_hip_build_bitmaps_wave(roff, ranks, ncols, F1, Wp, WT, bm, item_map, blocked, st);
    if (rc != 2) return rc;
  }
  if (blocked) return -22;
  dim3 g((unsigned)(Wp / WT), (unsigned)((F1 + R - 1) / R));
  size_t lds = (size_t)R * 2 * WT * 4;
  hipLaunchKernelGGL(k_build_bitmaps, g, dim3(256), lds, st, roff, ranks, src, ncols, F1, Wp, WT, R, bm, item_map,
                     used);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_trim_scan_count(const int64_t* roff, const int32_t* ranks, int64_t T, const int8_t* alive, int F1,
                                  int min_len, const int32_t* wrow, int32_t* cnt, int32_t* bk_rows, int32_t* bk_nnz,
                                  hipStream_t st) {
  if (T <= 0) return 0;
  const dim3 g((unsigned)((T + 255) / 256)), b(256);
  if (F1 <= kTrimAliveLds)
    hipLaunchKernelGGL(k_trim_scan_count<true>, g, b, F1, st, roff, ranks, T, alive, F1, min_len, wrow, cnt, bk_rows, bk_nnz);
  else
    hipLaunchKernelGGL(k_trim_scan_count<false>, g, b, 0, st, roff, ranks, T, alive, F1, min_len, wrow, cnt, bk_rows, bk_nnz);
  FA_LAUNCH_RET();
}

// hist: int64 [64][256] striped row-length histogram (length clamped to 255) or nullptr.
FA_API int fa_hip_trim_emit(const int64_t* roff, const int32_t* ranks, const int8_t* alive, int F1, int64_t T,
                            const int32_t* cnt, const int64_t* base_rows, const int64_t* base_nnz, int64_t* nroff,
                            int32_t* nranks, int32_t* kept, int64_t* hist, hipStream_t st) {
  if (T <= 0) return 0;
  const dim3 g((unsigned)((T + 255) / 256)), b(256);
  if (F1 <= kTrimAliveLds)
    hipLaunchKernelGGL(k_trim_emit<true>, g, b, F1, st, roff, ranks, alive, F1, T, cnt, base_rows, base_nnz, nroff,
                       nranks, kept, hist);
  else
    hipLaunchKernelGGL(k_trim_emit<false>, g, b, 0, st, roff, ranks, alive, F1, T, cnt, base_rows, base_nnz, nroff,
                       nranks, kept, hist);
  FA_LAUNCH_RET();
}

// Two-pass fused compression: agg int32 [3 * nwg], hist u32 [64 * 256] striped copies (zeroed by the caller).
// aggb (optional, nb <= 8 256-rank blocks): int32 [nb * nwg] per-workgroup block totals
// (the fused pair layout of k_cmp_emit).
// ---------------------------------------------------------------------------
// Exclusive scans of k_cmp_agg's per-workgroup aggregates for k_cmp_emit, in three
// small kernels (chunk sums, one scan of the chunk sums, chunk rescans) instead of
// torch's conversion, three cumsums and a fourth for the block totals (~10 kernels
// and two host allocations rounds per run).  Sequences: s < 3 the interleaved agg
// (kept rows, kept items, overflow rows) of nwg workgroups -> pre[s][0 .. nwg];
// s = 3 (aggb != null) the block-major block totals, nb * nwg -> preb[0 .. nb * nwg].
// Also roff[0] = 0.
// ---------------------------------------------------------------------------
constexpr int kScanChunk = 4096;      // elements per workgroup (256 threads x 16)

__device__ __forceinline__ int64_t cs_len(int s, int64_t nwg, int nb) { return s < 3 ? nwg : nb * nwg; }
__device__ __forceinline__ int32_t cs_at(const int32_t* __restrict__ agg, const int32_t* __restrict__ aggb, int s,
                                         int64_t i) {
  return s < 3 ? agg[3 * i + s] : aggb[i];
}

__global__ __launch_bounds__(256) void k_cmp_scan_sums(const int32_t* __restrict__ agg,
                                                       const int32_t* __restrict__ aggb, int64_t nwg, int nb,
                                                       int64_t* __restrict__ part, int64_t pstride) {
  const int s = blockIdx.y;
  const int64_t n = cs_len(s, nwg, nb), c0 = (int64_t)blockIdx.x * kScanChunk;
  if (c0 >= n) return;
  int64_t t = 0;
#pragma unroll 4
  for (int k = 0; k < kScanChunk / 256; ++k) {
    const int64_t i = c0 + k * 256 + threadIdx.x;
    if (i < n) t += cs_at(agg, aggb, s, i);
  }
  __shared__ int64_t w4[4];
  t = (int64_t)wave_sum_u64((unsigned long long)t);
  if ((threadIdx.x & 63) == 0) w4[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) part[s * pstride + blockIdx.x] = w4[0] + w4[1] + w4[2] + w4[3];
}

// exclusive scan of every sequence's chunk sums (one workgroup; <= 1024 chunks each)
__global__ __launch_bounds__(1024) void k_cmp_scan_parts(int64_t* __restrict__ part, int64_t pstride, int nseq,
                                                         int64_t nwg, int nb) {
  __shared__ int64_t wsum[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int s = 0; s < nseq; ++s) {
    const int64_t nch = (cs_len(s, nwg, nb) + kScanChunk - 1) / kScanChunk;
    const int64_t v = threadIdx.x < nch ? part[s * pstride + threadIdx.x] : 0;
    // 64-bit inclusive wave scan (shuffles)
    int64_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int64_t before = 0;
    for (int q = 0; q < wv; ++q) before += wsum[q];
    if (threadIdx.x < nch) part[s * pstride + threadIdx.x] = before + incl - v;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_cmp_scan_out(const int32_t* __restrict__ agg,
                                                      const int32_t* __restrict__ aggb, int64_t nwg, int nb,
                                                      const int64_t* __restrict__ part, int64_t pstride,
                                                      int64_t* __restrict__ pre, int64_t* __restrict__ preb,
                                                      int64_t* __restrict__ roff) {
  const int s = blockIdx.y;
  const int64_t n = cs_len(s, nwg, nb), c0 = (int64_t)blockIdx.x * kScanChunk;
  if (s == 0 && blockIdx.x == 0 && threadIdx.x == 0) roff[0] = 0;
  if (c0 >= n) return;
  int64_t* out = s < 3 ? pre + s * (nwg + 1) : preb;
  // each thread: 16 consecutive elements; thread sums scanned across the workgroup
  constexpr int PER = kScanChunk / 256;
  int32_t v[PER];
  int64_t t = 0;
  const int64_t i0 = c0 + (int64_t)threadIdx.x * PER;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    v[k] = i0 + k < n ? cs_at(agg, aggb, s, i0 + k) : 0;
    t += v[k];
  }
  __shared__ int64_t w4[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t incl = t;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) w4[wv] = incl;
  __syncthreads();
  int64_t run = part[s * pstride + blockIdx.x] + incl - t;
  for (int q = 0; q < wv; ++q) run += w4[q];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (i0 + k < n) out[i0 + k] = run;
    run += v[k];
    if (i0 + k == n - 1) out[n] = run;          // the sequence total
  }
}

FA_API int fa_hip_cmp_scan(const int32_t* agg, const int32_t* aggb, int64_t nwg, int nb, int64_t* part,
                           int64_t* pre, int64_t* preb, int64_t* roff, hipStream_t st) {
  if (nwg <= 0) return 0;
  const int nseq = aggb ? 4 : 3;
  const int64_t nmax = aggb ? std::max<int64_t>(nwg, (int64_t)nb * nwg) : nwg;
  const int64_t nch = (nmax + kScanChunk - 1) / kScanChunk;
  if (nch > 1024) return 1;                       // (n <= 4M workgroups' rows)
  const dim3 g((unsigned)nch, (unsigned)nseq);
  hipLaunchKernelGGL(k_cmp_scan_sums, g, dim3(256), 0, st, agg, aggb, nwg, nb, part, nch);
  hipLaunchKernelGGL(k_cmp_scan_parts, dim3(1), dim3(1024), 0, st, part, nch, nseq, nwg, nb);
  hipLaunchKernelGGL(k_cmp_scan_out, g, dim3(256), 0, st, agg, aggb, nwg, nb, part, nch, pre, preb, roff);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_cmp_agg(const int64_t* off, const int32_t* items, const int32_t* lut, int64_t n, int32_t* agg,
                          uint32_t* hist, int32_t* aggb, int nb, hipStream_t st) {
  if (n <= 0) return 0;
  if (aggb && (nb < 1 || nb > 8)) return 1;
  hipLaunchKernelGGL(k_cmp_agg, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, off, items, lut, n, agg, hist,
                     aggb, nb);
  FA_LAUNCH_RET();
}

// bcnt (optional, nb <= 8): u8 [nb * T] per-row block counts.  lr (optional, needs bcnt
// and preb = the exclusive scan of fa_hip_cmp_agg's aggb, nb * nwg + 1 entries): the
// pair kernel's blocked local-rank layout, u8 [lr_cap]; lbase: int64 [nb * ceil(T / 64)]
// batch bases (zeroed padding past it is the caller's); ovb: int64 [rows * nb] the
// overflow rows' segment bases, finished by fa_hip_lr_rows after the later tiers.
FA_API int fa_hip_cmp_emit(const int64_t* off, const int32_t* items, const int32_t* lut, int64_t n,
                           const int64_t* pre_rows, const int64_t* pre_items, const int64_t* pre_over, int32_t* kept,
                           int64_t* roff, int32_t* ranks, int32_t* over, uint8_t* bcnt, int nb, const int64_t* preb,
                           uint8_t* lr, int64_t lr_cap, int64_t* lbase, int64_t* ovb, hipStream_t st) {
  if (n <= 0) return 0;
  if (bcnt && (nb < 1 || nb > 8)) return 1;
  if (lr && (!bcnt || !preb || !lbase || !ovb)) return 1;
  const size_t dyn = lr ? (size_t)256 * nb * sizeof(int32_t) : 0;
  hipLaunchKernelGGL(k_cmp_emit, dim3((unsigned)((n + 255) / 256)), dim3(256), dyn, st, off, items, lut, n, pre_rows,
                     pre_items, pre_over, kept, roff, ranks, over, bcnt, nb, preb, lr, lr_cap, lbase, ovb);
  FA_LAUNCH_RET();
}

// The fused pair layout of the rows k_cmp_emit left to the later tiers (rows[i] = kept
// row, flags: optional), thread per row over its final sorted ranks.
__global__ __launch_bounds__(256) void k_lr_rows(const int64_t* __restrict__ roff, const int32_t* __restrict__ ranks,
                                                 const int32_t* __restrict__ rows, int64_t nrows,
                                                 const int64_t* __restrict__ ovb, int nb, uint8_t* __restrict__ lr,
                                                 int64_t lr_cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows) return;
  const int64_t x = rows[i];
  const int64_t r0 = roff[x], r1 = roff[x + 1];
  for (int64_t k = r0; k < r1; ++k) {
    const int v = ranks[k];
    const int b = v >> 8;
    const int64_t pos = b < nb ? ovb[i * nb + b] + (k - r0) : -1;
    if (pos >= 0 && pos < lr_cap) lr[pos] = (uint8_t)v;
  }
}

FA_API int fa_hip_lr_rows(const int64_t* roff, const int32_t* ranks, const int32_t* rows, int64_t nrows,
                          const int64_t* ovb, int nb, uint8_t* lr, int64_t lr_cap, hipStream_t st) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(k_lr_rows, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, st, roff, ranks, rows, nrows,
                     ovb, nb, lr, lr_cap);
  FA_LAUNCH_RET();
}
