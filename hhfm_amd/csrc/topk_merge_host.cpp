// Host (CPU-memory) top-K merge — same contract as hhfm_topk_merge; used by
// the gloo multi-process path and by tests that run without a GPU.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/hhfm.h"

extern "C" int hhfm_topk_merge_host(const float* in_score, const int32_t* in_idx,
                                    int32_t R, int64_t B, int32_t K,
                                    float* out_score, int32_t* out_idx) {
  if (R < 1 || B < 0 || K < 1) return HHFM_EINVAL;
  if (B == 0) return HHFM_OK;
  if (!in_score || !in_idx || !out_score || !out_idx) return HHFM_EINVAL;
  std::vector<std::pair<float, int32_t>> cand((size_t)R * K);
  auto better = [](const std::pair<float, int32_t>& a,
                   const std::pair<float, int32_t>& b) {
    return a.first > b.first || (a.first == b.first && a.second < b.second);
  };
  for (int64_t b = 0; b < B; ++b) {
    for (int32_t r = 0; r < R; ++r)
      for (int32_t x = 0; x < K; ++x) {
        const int64_t o = ((int64_t)r * B + b) * K + x;
        cand[(size_t)r * K + x] = {in_score[o], in_idx[o]};
      }
    std::partial_sort(cand.begin(), cand.begin() + K, cand.end(), better);
    for (int32_t x = 0; x < K; ++x) {
      out_score[b * K + x] = cand[x].first;
      out_idx[b * K + x] = cand[x].second;
    }
  }
  return HHFM_OK;
}
