// freqItemset writer: exact reference format (Utils.scala:29-41, :51-63).
//
// Each itemset becomes its tokens in rank-DESCENDING order joined by one space
// (optionally followed by "[count]", the saveFreqItemsetWithCount format), and
// the lines are sorted with java.lang.String ordering: UTF-16 code units.  For
// pure-ASCII vocabularies that is plain byte order; otherwise every line is
// compared through its UTF-16 image.
#include <cstdio>

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
  std::vector<std::string> lines((size_t)n);
  parallel_for(n, nthreads, 4096, [&](int64_t b, int64_t e, int) {
    char num[32];
    int k = 1;
    for (int64_t li = b; li < e; ++li) {
      while (li >= base[k]) ++k;
      const int64_t row = li - base[k - 1];
      const int32_t* r = rows[k - 1] + row * k;
      std::string& s = lines[li];
      for (int j = k - 1; j >= 0; --j) {   // rows are ascending: emit descending
        s.append(tokbuf + tokoff[r[j]], (size_t)(tokoff[r[j] + 1] - tokoff[r[j]]));
        if (j) s.push_back(' ');
      }
      if (with_counts) {
        int len = std::snprintf(num, sizeof num, "[%lld]", (long long)counts[k - 1][row]);
        s.append(num, len);
      }
    }
  });
  std::vector<int64_t> order((size_t)n);
  for (int64_t i = 0; i < n; ++i) order[i] = i;
  if (ascii) {
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return lines[a] < lines[b]; });
  } else {
    std::vector<std::string> keys((size_t)n);
    parallel_for(n, nthreads, 4096, [&](int64_t b, int64_t e, int) {
      for (int64_t i = b; i < e; ++i) utf8_to_utf16be(lines[i].data(), lines[i].size(), keys[i]);
    });
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return keys[a] < keys[b]; });
  }
  FILE* f = std::fopen(path, "wb");
  if (!f) return 1;
  std::string buf;
  buf.reserve(1 << 20);
  for (int64_t i = 0; i < n; ++i) {
    buf.append(lines[order[i]]);
    buf.push_back('\n');
    if (buf.size() > (1 << 20)) { std::fwrite(buf.data(), 1, buf.size(), f); buf.clear(); }
  }
  std::fwrite(buf.data(), 1, buf.size(), f);
  return std::fclose(f) == 0 ? 0 : 2;
}
