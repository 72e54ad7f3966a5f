// H3 / H5 on the device — the evaluation harness's per-element work
// (SURVEY §8f items 2 and 4).
//
//   hhfm_pf_contains replaces the `neg in self.data.positive_feedback[key]`
//                    rejection test of Train.sample_negative (FM.py:291-293)
//                    and the target test of evaluate_TopK (FM.py:343-355:
//                    `item in positive_feedback[key]`)
//   hhfm_topk_walk   replaces the per-row walk over the 20 predictions of
//                    Train.evaluate_TopK (FM.py:344-357)
//
// positive_feedback (a dict key -> set(item), key = every column but the
// item, NewLoadData.py:49-56) is laid out as two sorted device arrays built
// once on the host: the distinct keys, lexicographically sorted
// [nkeys][key_cols] int32, and the (key rank << 32 | item) codes of every
// (key, item) pair, sorted int64.  A membership test is a binary search for
// the key followed by one for the code: no hashing, no collisions, exact.
// The draws themselves stay on the host (numpy's RNG stream, so the samples
// are the reference's); the walk returns ranks, the host turns them into
// the reference's float64 HR / NDCG / PRE values.
#include "hhfm_common.h"

namespace hhfm {

// row key (every column but item_col, in column order) vs keys[m]
HHFM_DEV int key_cmp(const int32_t* row, int ncols, int item_col, const int32_t* key) {
  int c2 = 0;
  for (int c = 0; c < ncols; ++c) {
    if (c == item_col) continue;
    const int32_t a = row[c], b = key[c2++];
    if (a != b) return a < b ? -1 : 1;
  }
  return 0;
}

// one thread per (row, candidate); cand == nullptr: the row's own item
__global__ __launch_bounds__(256) void pf_contains_kernel(
    const int32_t* __restrict__ keys, int64_t nkeys, int key_cols,
    const int64_t* __restrict__ codes, int64_t ncodes, const int32_t* __restrict__ rows,
    int64_t B, int ncols, int item_col, const int32_t* __restrict__ cand, int num,
    uint8_t* __restrict__ out) {
  const int64_t n = B * num;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = x / num;
    const int32_t* row = rows + b * ncols;
    const int32_t item = cand ? cand[x] : row[item_col];
    // lower_bound over the sorted keys
    int64_t lo = 0, hi = nkeys;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (key_cmp(row, ncols, item_col, keys + mid * key_cols) > 0) lo = mid + 1;
      else hi = mid;
    }
    uint8_t hit = 0;
    if (lo < nkeys && key_cmp(row, ncols, item_col, keys + lo * key_cols) == 0) {
      const int64_t code = (lo << 32) | (int64_t)(uint32_t)item;
      int64_t a = 0, e = ncodes;
      while (a < e) {
        const int64_t mid = (a + e) >> 1;
        if (codes[mid] < code) a = mid + 1;
        else e = mid;
      }
      hit = a < ncodes && codes[a] == code;
    }
    out[x] = hit;
  }
}

// evaluate_TopK's walk (FM.py:344-357), one thread per row:
//   outcome = n >= 0  the target found at walk position n (< TopK)
//           = -1      walk reached n > TopK-1: the reference appends 0, 0, 0
//           = -2      predictions exhausted: the reference appends nothing
// A target that is itself a train positive of its key makes every non-hit a
// `continue` (n is not advanced), the reference's quirk.
__global__ __launch_bounds__(256) void topk_walk_kernel(
    const int32_t* __restrict__ pred, int64_t B, int P, const int32_t* __restrict__ target,
    const uint8_t* __restrict__ positive, int TopK, int32_t* __restrict__ outcome) {
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    const int32_t item = target[b];
    const bool pos = positive[b] != 0;
    int n = 0, res = -2;
    for (int p = 0; p < P; ++p) {
      if (n > TopK - 1) { res = -1; break; }
      if (pred[b * P + p] == item) { res = n; break; }
      if (!pos) ++n;
    }
    outcome[b] = res;
  }
}

static unsigned grid_1d(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_pf_contains(const int32_t* keys, int64_t nkeys, int32_t key_cols,
                                const int64_t* codes, int64_t ncodes, const int32_t* rows,
                                int64_t B, int32_t ncols, int32_t item_col,
                                const int32_t* cand, int32_t num, uint8_t* out,
                                void* stream) {
  if (B < 0 || nkeys < 0 || ncodes < 0 || ncols < 2 || ncols > 64) return HHFM_EINVAL;
  if (item_col < 0 || item_col >= ncols || key_cols != ncols - 1) return HHFM_EINVAL;
  if (cand ? num < 1 : num != 1) return HHFM_EINVAL;
  if (B == 0) return HHFM_OK;
  if (!rows || !out || (nkeys && !keys) || (ncodes && !codes)) return HHFM_EINVAL;
  hipLaunchKernelGGL(pf_contains_kernel, dim3(grid_1d(B * num)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), keys, nkeys, key_cols, codes,
                     ncodes, rows, B, ncols, item_col, cand, num, out);
  return (int)hipGetLastError();
}

extern "C" int hhfm_topk_walk(const int32_t* pred, int64_t B, int32_t P, const int32_t* target,
                              const uint8_t* positive, int32_t TopK, int32_t* outcome,
                              void* stream) {
  if (B < 0 || P < 1 || TopK < 1) return HHFM_EINVAL;
  if (B == 0) return HHFM_OK;
  if (!pred || !target || !positive || !outcome) return HHFM_EINVAL;
  hipLaunchKernelGGL(topk_walk_kernel, dim3(grid_1d(B)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), pred, B, P, target, positive, TopK,
                     outcome);
  return (int)hipGetLastError();
}
