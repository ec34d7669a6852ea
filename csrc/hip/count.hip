// Support-counting kernels for k = 2 and k >= 3.
//
// Reference sites: FastApriori.scala:212-241 (genTwoFreqItems: all F1(F1-1)/2
// pairs, AND of two byte-per-transaction arrays + weighted sum) and
// :132-160 (genNextFreqItemsets: prefix AND once per group, then AND + sum per
// extension).  Here:
//   * k_pair_horizontal  : sparse data — every transaction's sorted rank list
//     scatters its pairs into an LDS-resident 128x128 count tile (ds_add_u32),
//     one global atomic per non-zero tile entry per workgroup.
//   * k_pair_gram_popc   : dense data — bit-matrix Gram B^T diag(w) B over the
//     vertical bitmaps, 64x64 item tiles staged through LDS, v_bcnt popcounts.
//   * k_count_candidates : k >= 3 — prefix-shared AND + popcount per group of
//     candidates over a super-chunk of bitmap words; wave reductions into an
//     LDS accumulator, one coalesced global atomic per candidate per chunk.
// All accumulation is integer, so results are exact and order-independent.
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

__global__ __launch_bounds__(256) void k_pair_horizontal(
    const int64_t* __restrict__ roff, const int32_t* __restrict__ ranks, int64_t T,
    const int32_t* __restrict__ wrow, int32_t F1, int nb, int nbp, int64_t chunk,
    uint32_t* __restrict__ out) {
  __shared__ uint32_t tile[kPB * kPB];
  const int pid = blockIdx.x % nbp;
  const int64_t ch = blockIdx.x / nbp;
  int bi, bj;
  tri_index(pid, nb, bi, bj);
  const int rb0 = bi * kPB, cb0 = bj * kPB;
  const bool diag = bi == bj;
  for (int i = threadIdx.x; i < kPB * kPB; i += blockDim.x) tile[i] = 0;
  __syncthreads();
  const int64_t x0 = ch * chunk, x1 = min(T, x0 + chunk);
  for (int64_t x = x0 + threadIdx.x; x < x1; x += blockDim.x) {
    const int64_t s = roff[x], e = roff[x + 1];
    if (e - s < 2) continue;
    const uint32_t w = wrow ? (uint32_t)wrow[x] : 1u;
    if (w == 0) continue;   // dedup: non-representative row
    const int64_t i0 = lower_bound_i32(ranks, s, e, rb0);
    const int64_t i1 = lower_bound_i32(ranks, i0, e, rb0 + kPB);
    if (i0 == i1) continue;
    int64_t j0, j1;
    if (diag) { j0 = i0; j1 = i1; }
    else {
      j0 = lower_bound_i32(ranks, i1, e, cb0);
      j1 = lower_bound_i32(ranks, j0, e, cb0 + kPB);
    }
    for (int64_t i = i0; i < i1; ++i) {
      const int a = (ranks[i] - rb0) * kPB - cb0;
      for (int64_t j = diag ? i + 1 : j0; j < j1; ++j) atomicAdd(&tile[a + ranks[j]], w);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kPB * kPB; i += blockDim.x) {
    const uint32_t v = tile[i];
    if (!v) continue;
    const int r = rb0 + i / kPB, c = cb0 + i % kPB;
    if (r < F1 && c < F1) atomicAdd(&out[(int64_t)r * F1 + c], v);
  }
}

// ---------------------------------------------------------------------------
// k = 2, dense bit-matrix Gram with popcounts.  Tile 64x64 items, K-step 32 words.
// ---------------------------------------------------------------------------
constexpr int kGT = 64, kGK = 32, kGS = kGT + 1;   // LDS row stride (u64) breaks bank aliasing

template <bool kWeighted>
__global__ __launch_bounds__(256) void k_pair_gram_popc(
    const uint64_t* __restrict__ bm, int32_t F1, int64_t Wp, int64_t W,
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
      As[k * kGS + r] = (ra < F1 && kk < k_end) ? bm[(int64_t)ra * Wp + kk] : 0ull;
      Bs[k * kGS + r] = (rb < F1 && kk < k_end) ? bm[(int64_t)rb * Wp + kk] : 0ull;
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

}  // namespace fa

using namespace fa;

FA_API int fa_hip_pair_horizontal(const int64_t* roff, const int32_t* ranks, int64_t T,
                                  const int32_t* wrow, int32_t F1, uint32_t* out, int target_wgs,
                                  hipStream_t st) {
  if (T <= 0 || F1 < 2) return 0;
  const int nb = (F1 + kPB - 1) / kPB;
  const int nbp = nb * (nb + 1) / 2;
  int64_t nch = std::max<int64_t>(1, (target_wgs + nbp - 1) / nbp);
  nch = std::min<int64_t>(nch, std::max<int64_t>(1, T / 512));
  const int64_t chunk = (T + nch - 1) / nch;
  nch = (T + chunk - 1) / chunk;
  hipLaunchKernelGGL(k_pair_horizontal, dim3((unsigned)(nch * nbp)), dim3(256), 0, st, roff, ranks,
                     T, wrow, F1, nb, nbp, chunk, out);
  FA_LAUNCH_RET();
}

FA_API int fa_hip_pair_gram_popc(const uint64_t* bm, int32_t F1, int64_t Wp, int64_t W,
                                 const int32_t* wword, uint32_t* out, int target_wgs, hipStream_t st) {
  if (W <= 0 || F1 < 2) return 0;
  const int nt = (F1 + kGT - 1) / kGT;
  const int ntp = nt * (nt + 1) / 2;
  int64_t nk = std::max<int64_t>(1, (target_wgs + ntp - 1) / ntp);
  int64_t kchunk = (W + nk - 1) / nk;
  kchunk = std::max<int64_t>(kGK, (kchunk + kGK - 1) / kGK * kGK);
  nk = (W + kchunk - 1) / kchunk;
  dim3 g((unsigned)(nk * ntp));
  if (wword)
    hipLaunchKernelGGL(k_pair_gram_popc<true>, g, dim3(256), 0, st, bm, F1, Wp, W, wword, nt, ntp, kchunk, out);
  else
    hipLaunchKernelGGL(k_pair_gram_popc<false>, g, dim3(256), 0, st, bm, F1, Wp, W, wword, nt, ntp, kchunk, out);
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
