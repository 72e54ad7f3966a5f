// L1 — the libfm loader's per-cell work in C++ (SURVEY §8f items 2 and 4:
// "loader in C++", "libfm encoder"), host code in libhhfm.so (no GPU).
//
//   hhfm_libfm_encode replaces NewLoadData.py:16-34: read_csv(sep=' ') of
//                     "label tok tok ..." lines, the column-major
//                     first-occurrence token -> id map over columns 1..
//                     (identical tokens in different columns share one id)
//                     and the per-cell applymap
//   hhfm_loader_split replaces NewLoadData.py:39-58's walk over the
//                     shuffled rows: a row goes to Test iff its key (every
//                     column but label and item) is unseen and fewer than
//                     test_size rows went to Test so far
//
// Tokens are compared as byte strings.  That is what pandas does for libfm
// files, whose feature tokens are "index:value" strings; a column of purely
// numeric tokens would be parsed as integers by pandas (the Python loader
// keeps that path: hhfm_amd.NewLoadData, encoder="python").
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/hhfm.h"

namespace {

struct KeyHash {
  size_t operator()(const std::vector<int64_t>& k) const {
    uint64_t h = 1469598103934665603ull;
    for (int64_t v : k) {
      h ^= (uint64_t)v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
      h *= 1099511628211ull;
    }
    return (size_t)h;
  }
};

}  // namespace

extern "C" int hhfm_libfm_encode(const char* buf, int64_t len, int32_t ncols, int64_t max_rows,
                                 double* labels, int64_t* ids, int64_t* rows_out,
                                 int64_t* features_M, int64_t* distinct) {
  if (!buf || len < 0 || ncols < 2 || max_rows < 0 || !labels || !ids || !rows_out ||
      !features_M || !distinct)
    return HHFM_EINVAL;
  // split into lines and single-space separated fields (read_csv(sep=' ')
  // skips blank lines; a trailing '\r' is dropped)
  std::vector<std::string_view> tok;   // row-major [rows][ncols]
  int64_t rows = 0;
  const char* p = buf;
  const char* end = buf + len;
  while (p < end) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    const char* le = nl ? nl : end;
    const char* lend = (le > p && le[-1] == '\r') ? le - 1 : le;
    if (lend > p) {
      if (rows >= max_rows) return HHFM_EINVAL;
      int c = 0;
      const char* f = p;
      for (const char* q = p;; ++q) {
        if (q == lend || *q == ' ') {
          if (c >= ncols) return HHFM_EINVAL;
          tok.emplace_back(f, (size_t)(q - f));
          ++c;
          if (q == lend) break;
          f = q + 1;
        }
      }
      if (c != ncols) return HHFM_EINVAL;
      char* e = nullptr;
      const std::string lab(tok[(size_t)rows * ncols].data(), tok[(size_t)rows * ncols].size());
      labels[rows] = strtod(lab.c_str(), &e);
      if (lab.empty() || *e != '\0') return HHFM_EINVAL;
      ++rows;
    }
    p = nl ? nl + 1 : end;
  }
  // column-major first-occurrence ids over columns 1..ncols-1
  std::unordered_map<std::string_view, int64_t> id;
  id.reserve((size_t)rows * 2 + 16);
  for (int c = 1; c < ncols; ++c) {
    std::unordered_set<std::string_view> col;
    for (int64_t r = 0; r < rows; ++r) {
      const std::string_view t = tok[(size_t)r * ncols + c];
      auto it = id.find(t);
      int64_t v;
      if (it == id.end()) {
        v = (int64_t)id.size();
        id.emplace(t, v);
      } else {
        v = it->second;
      }
      ids[r * (ncols - 1) + (c - 1)] = v;
      col.insert(t);
    }
    distinct[c - 1] = (int64_t)col.size();   // value_counts() length
  }
  *rows_out = rows;
  *features_M = (int64_t)id.size();
  return HHFM_OK;
}

extern "C" int hhfm_loader_split(const int64_t* data, int64_t rows, int32_t ncols,
                                 int32_t item_col, int64_t test_size, uint8_t* is_test) {
  if (rows < 0 || ncols < 3 || item_col < 1 || item_col >= ncols || test_size < 0)
    return HHFM_EINVAL;
  if (rows == 0) return HHFM_OK;
  if (!data || !is_test) return HHFM_EINVAL;
  std::unordered_set<std::vector<int64_t>, KeyHash> seen;
  seen.reserve((size_t)test_size * 2 + 16);
  std::vector<int64_t> key((size_t)ncols - 2);
  int64_t n_test = 0;
  for (int64_t r = 0; r < rows; ++r) {
    const int64_t* line = data + r * ncols;
    size_t k = 0;
    for (int c = 1; c < ncols; ++c)
      if (c != item_col) key[k++] = line[c];
    // `key not in set_key and i < test_size` (NewLoadData.py:51): the set
    // is only consulted (and grown) while Test still has room
    if (n_test < test_size && seen.insert(key).second) {
      is_test[r] = 1;
      ++n_test;
    } else {
      is_test[r] = 0;
    }
  }
  return HHFM_OK;
}
