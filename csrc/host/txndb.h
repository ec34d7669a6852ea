// In-memory transaction shard produced by the parser or the synthetic generator.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fa {

struct TxnChunk {
  std::vector<int64_t> lens;   // cumulative item count at the end of each line (within chunk)
  std::vector<int32_t> items;  // distinct ids per line, concatenated
};

struct TxnDB {
  std::vector<TxnChunk> chunks;
  std::vector<int32_t> extras;     // one id per repeated occurrence inside a line
  bool numeric = true;
  int64_t vocab = 0;               // id space size
  std::vector<std::string> dict;   // dict mode: id -> token bytes
};

int64_t next_line_start(const char* d, int64_t size, int64_t pos);

}  // namespace fa
