// freqItemset writer: exact reference format (Utils.scala:29-41, :51-63).
//
// Each itemset becomes its tokens in rank-DESCENDING order joined by one space
// (optionally followed by "[count]", the saveFreqItemsetWithCount format), and
// the lines are sorted with java.lang.String ordering: UTF-16 code units.  For
// pure-ASCII vocabularies that is plain byte order; otherwise every line is
// compared through its UTF-16 image.
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "fa_common.h"

namespace fa {

static void utf8_to_utf16be(const char* s, size_t n, std::string& out) {
  out.clear();
  size_t i = 0;
  auto put = [&](uint32_t u) { out.push_back((char)(u >> 8)); out.push_back((char)(u & 0xFF)); };
  while (i < n) {
    uint8_t c = (uint8_t)s[i];
    uint32_t cp;
    int len;
    if (c < 0x80) { cp = c; len = 1; }
    else if ((c >> 5) == 6 && i + 1 < n) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); len = 2; }
    else if ((c >> 4) == 14 && i + 2 < n) { cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); len = 3; }
    else if ((c >> 3) == 30 && i + 3 < n) {
      cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F); len = 4;
    } else { cp = 0xFFFD; len = 1; }   // malformed byte: Java decodes it as U+FFFD
    if (cp >= 0x10000) {
      cp -= 0x10000;
      put(0xD800 + (cp >> 10));
      put(0xDC00 + (cp & 0x3FF));
    } else {
      put(cp);
    }
    i += len;
  }
}

}  // namespace fa

using namespace fa;

// Lines go into one flat buffer (lengths, then a scan, then the bytes, all in parallel);
// pure-ASCII lines sort on a 64-bit key of their first 8 bytes (big-endian, zero-padded:
// a line that is a prefix of another sorts first, as in String.compareTo) with a byte
// comparison of the rest only between equal keys, in parallel chunks merged pairwise;
// the sorted lines are gathered into one output buffer and written with one fwrite.
// (One std::string per line and a single-threaded sort of them: ~5 ms for the 33 K
// itemsets of T10I4D100M on the GPU box, inside the reference's timed window.)
FA_API int fa_write_freq_itemsets(const char* path, const char* tokbuf, const int64_t* tokoff,
                                  int32_t F1, const int32_t* const* rows,
                                  const int64_t* const* counts, const int64_t* sizes, int levels,
                                  int with_counts, int nthreads) {
  bool ascii = true;
  for (int64_t i = 0; i < tokoff[F1] && ascii; ++i) ascii = (uint8_t)tokbuf[i] < 0x80;
  // line index: (level, row)
  std::vector<int64_t> base(levels + 1, 0);
  for (int k = 1; k <= levels; ++k) base[k] = base[k - 1] + sizes[k - 1];
  const int64_t n = base[levels];
  auto level_of = [&](int64_t li) {
    int k = 1;
    while (li >= base[k]) ++k;
    return k;
  };
  auto count_str = [&](int k, int64_t row, char* num) {
    return std::snprintf(num, 32, "[%lld]", (long long)counts[k - 1][row]);
  };
  // 1. line lengths and offsets
  std::vector<int64_t> loff((size_t)n + 1, 0);
  parallel_for(n, nthreads, 4096, [&](int64_t b, int64_t e, int) {
    char num[32];
    int k = level_of(b);
    for (int64_t li = b; li < e; ++li) {
      while (li >= base[k]) ++k;
      const int64_t row = li - base[k - 1];
      const int32_t* r = rows[k - 1] + row * k;
      int64_t len = k - 1;
      for (int j = 0; j < k; ++j) len += tokoff[r[j] + 1] - tokoff[r[j]];
      if (with_counts) len += count_str(k, row, num);
      loff[li + 1] = len;
    }
  });
  for (int64_t i = 0; i < n; ++i) loff[i + 1] += loff[i];
  // 2. the line bytes (tokens in rank-descending order, one space apart)
  std::vector<char> text((size_t)std::max<int64_t>(loff[n], 1));
  parallel_for(n, nthreads, 4096, [&](int64_t b, int64_t e, int) {
    char num[32];
    int k = level_of(b);
    for (int64_t li = b; li < e; ++li) {
      while (li >= base[k]) ++k;
      const int64_t row = li - base[k - 1];
      const int32_t* r = rows[k - 1] + row * k;
      char* o = text.data() + loff[li];
      for (int j = k - 1; j >= 0; --j) {   // rows are ascending: emit descending
        const int64_t tl = tokoff[r[j] + 1] - tokoff[r[j]];
        std::memcpy(o, tokbuf + tokoff[r[j]], (size_t)tl);
        o += tl;
        if (j) *o++ = ' ';
      }
      if (with_counts) {
        const int len = count_str(k, row, num);
        std::memcpy(o, num, (size_t)len);
      }
    }
  });
  // 3. the order
  std::vector<int64_t> order((size_t)n);
  for (int64_t i = 0; i < n; ++i) order[i] = i;
  if (ascii) {
    std::vector<uint64_t> key((size_t)n);
    parallel_for(n, nthreads, 8192, [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; ++i) {
        uint64_t k = 0;
        const int64_t len = loff[i + 1] - loff[i];
        const unsigned char* t = reinterpret_cast<const unsigned char*>(text.data() + loff[i]);
        for (int j = 0; j < 8; ++j) k = (k << 8) | (j < len ? t[j] : 0u);
        key[i] = k;
      }
    });
    auto less = [&](int64_t a, int64_t b) {
      if (key[a] != key[b]) return key[a] < key[b];
      const int64_t la = loff[a + 1] - loff[a], lb = loff[b + 1] - loff[b];
      if (la <= 8 || lb <= 8) return la < lb;     // equal 8-byte keys: the shorter is a prefix
      const int c = std::memcmp(text.data() + loff[a] + 8, text.data() + loff[b] + 8, (size_t)std::min(la, lb) - 8);
      return c != 0 ? c < 0 : la < lb;
    };
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, n / 4096));
    std::vector<int64_t> cut((size_t)T + 1);
    for (int t = 0; t <= T; ++t) cut[t] = n * t / T;
    parallel_for_threads(T, [&](int t) { std::sort(order.begin() + cut[t], order.begin() + cut[t + 1], less); });
    for (int w = 1; w < T; w *= 2) {
      const int nm = (T + 2 * w - 1) / (2 * w);
      parallel_for_threads(std::min(nm, std::max(nthreads, 1)), [&](int tid) {
        for (int m = tid; m < nm; m += std::min(nm, std::max(nthreads, 1))) {
          const int a0 = 2 * w * m, a1 = std::min(T, a0 + w), a2 = std::min(T, a0 + 2 * w);
          if (a1 < a2)
            std::inplace_merge(order.begin() + cut[a0], order.begin() + cut[a1], order.begin() + cut[a2], less);
        }
      });
    }
  } else {
    std::vector<std::string> keys((size_t)n);
    parallel_for(n, nthreads, 4096, [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; ++i) utf8_to_utf16be(text.data() + loff[i], (size_t)(loff[i + 1] - loff[i]), keys[i]);
    });
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return keys[a] < keys[b]; });
  }
  // 4. the output: sorted lines with '\n', gathered in parallel, one write
  std::vector<int64_t> ooff((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i) ooff[i + 1] = ooff[i] + (loff[order[i] + 1] - loff[order[i]]) + 1;
  std::vector<char> out((size_t)std::max<int64_t>(ooff[n], 1));
  parallel_for(n, nthreads, 8192, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      const int64_t l = order[i], len = loff[l + 1] - loff[l];
      std::memcpy(out.data() + ooff[i], text.data() + loff[l], (size_t)len);
      out[(size_t)(ooff[i] + len)] = '\n';
    }
  });
  FILE* f = std::fopen(path, "wb");
  if (!f) return 1;
  const size_t wrote = n ? std::fwrite(out.data(), 1, (size_t)ooff[n], f) : 0;
  const int rc = std::fclose(f);
  return (rc == 0 && wrote == (size_t)ooff[n]) ? 0 : 2;
}
