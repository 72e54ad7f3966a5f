// Wave-level top-K primitives (64-lane CDNA wavefronts).
//
// A top-K list lives one entry per lane (lanes [0, KPAD)), sorted by the
// tf.nn.top_k order: score descending, index ascending on equal scores
// (FM.py:185 / OurModel7.py:295 fetch tf.nn.top_k(score, 20)).
#pragma once
#include "hhfm_common.h"

namespace hhfm {

constexpr float kNegInf = -__builtin_huge_valf();
constexpr int32_t kNoIdx = 0x7fffffff;

// strict total order used everywhere: a ranks before b
HHFM_DEV bool better(float as, int32_t ai, float bs, int32_t bi) {
  return as > bs || (as == bs && ai < bi);
}

HHFM_DEV int lane_id() { return threadIdx.x & (kWave - 1); }

HHFM_DEV float shfl_f(float v, int src) { return __shfl(v, src, kWave); }
HHFM_DEV int32_t shfl_i(int32_t v, int src) { return __shfl(v, src, kWave); }

// v from lane (self ^ d), d a power of two < 64, without the LDS crossbar
// where a DPP pattern exists (ds_bpermute costs an LDS round trip per step):
//   d = 1, 2: quad_perm; d = 4: row_shl/row_shr 4 + lane select; d = 8:
//   row_ror 8; d = 16: ds_swizzle xor mode (no address VGPR); d = 32:
//   v_permlane32_swap.
HHFM_DEV int32_t xor_lane(int32_t v, int d) {
  switch (d) {
    case 1: return __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false);   // [1,0,3,2]
    case 2: return __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false);   // [2,3,0,1]
    case 4: {
      const int32_t up = __builtin_amdgcn_update_dpp(v, v, 0x104, 0xF, 0xF, false);  // row_shl:4
      const int32_t dn = __builtin_amdgcn_update_dpp(v, v, 0x114, 0xF, 0xF, false);  // row_shr:4
      return (lane_id() & 4) ? dn : up;
    }
    case 8: return __builtin_amdgcn_update_dpp(v, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    case 16: return __builtin_amdgcn_ds_swizzle(v, 0x401F);                    // xor 16 in 32
    default: {   // 32: swap(a=v, b=v) leaves a = [v_lo | v_lo], b = [v_hi | v_hi]
      const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
      return (int32_t)(lane_id() < 32 ? r[1] : r[0]);
    }
  }
}
HHFM_DEV float xor_lane(float v, int d) {
  return __int_as_float(xor_lane(__float_as_int(v), d));
}

// One compare-exchange step of a bitonic network: keep the better of
// (self, lane^d) when keep_better, else the worse.
HHFM_DEV void cx(float& s, int32_t& i, int d, bool keep_better) {
  const float ps = xor_lane(s, d);
  const int32_t pi = xor_lane(i, d);
  const bool pb = better(ps, pi, s, i);
  const bool take = keep_better ? pb : !pb;
  s = take ? ps : s;
  i = take ? pi : i;
}

// Bitonic sort, descending (best first), independently inside every aligned
// group of N lanes (N power of two <= 64).
template <int N>
HHFM_DEV void bitonic_sort_desc(float& s, int32_t& i) {
  const int l = lane_id() & (N - 1);
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
    const bool desc = (l & size) == 0 || size == N;
#pragma unroll
    for (int d = size >> 1; d >= 1; d >>= 1) {
      const bool lower = (l & d) == 0;
      cx(s, i, d, lower == desc);
    }
  }
}

// Sort a bitonic sequence held in aligned groups of N lanes, descending.
template <int N>
HHFM_DEV void bitonic_merge_desc(float& s, int32_t& i) {
  const int l = lane_id() & (N - 1);
#pragma unroll
  for (int d = N >> 1; d >= 1; d >>= 1) cx(s, i, d, (l & d) == 0);
}

// Top-KPAD of the union of two descending lists A (self, lanes [0,KPAD)) and
// B (lanes [0,KPAD) of bs/bi): elementwise best of A[l] and B[KPAD-1-l] is
// bitonic and holds exactly the KPAD best; the merge network sorts it.
template <int KPAD>
HHFM_DEV void merge_lists(float& as, int32_t& ai, float bs, int32_t bi) {
  const int l = lane_id();
  const int src = (l < KPAD) ? (KPAD - 1 - l) : l;
  const float rs = shfl_f(bs, src);
  const int32_t ri = shfl_i(bi, src);
  if (better(rs, ri, as, ai)) {
    as = rs;
    ai = ri;
  }
  bitonic_merge_desc<KPAD>(as, ai);
}

// ---------------------------------------------------------------------------
// dense top-K over materialised scores [B][N] (wave per query)
// ---------------------------------------------------------------------------
template <int KPAD>
__global__ __launch_bounds__(256) void topk_dense_kernel(const float* __restrict__ S,
                                                         int64_t B, int32_t N, int64_t lds,
                                                         int K, int32_t base,
                                                         float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i) {
  const int l = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t b = wave; b < B; b += nwave) {
    const float* row = S + b * lds;
    float ls = kNegInf;
    int32_t li = kNoIdx;
    float thr = kNegInf;
    for (int32_t c0 = 0; c0 < N; c0 += kWave) {
      const int32_t i = c0 + l;
      const float s = i < N ? row[i] : kNegInf;
      const bool pass = i < N && s >= thr;
      const uint64_t m = __ballot(pass);
      const int cnt = __popcll(m);
      if (cnt == 0) continue;
      if (cnt > 8) {
        float cs = pass ? s : kNegInf;
        int32_t ci = pass ? i : kNoIdx;
        bitonic_sort_desc<64>(cs, ci);
        merge_lists<KPAD>(ls, li, cs, ci);
      } else {
        uint64_t mm = m;
        while (mm) {
          const int L = __builtin_ctzll(mm);
          mm &= mm - 1;
          const float sc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), L));
          const int32_t ic = c0 + L;
          const int pos = __popcll(__ballot(l < KPAD && better(ls, li, sc, ic)));
          if (pos < K) {
            const float ps = __shfl_up(ls, 1, kWave);
            const int32_t pi = __shfl_up(li, 1, kWave);
            if (l > pos) { ls = ps; li = pi; }
            else if (l == pos) { ls = sc; li = ic; }
          }
        }
      }
      if (l >= KPAD) { ls = kNegInf; li = kNoIdx; }
      thr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ls), K - 1));
    }
    if (l < K) {
      out_s[b * K + l] = ls;
      out_i[b * K + l] = li == kNoIdx ? kNoIdx : li + base;
    }
  }
}

static inline void launch_topk_dense(const float* S, int64_t B, int32_t N, int64_t lds, int K,
                              int32_t base, float* os, int32_t* oi, hipStream_t st) {
  int64_t blocks = (B + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (K <= 32)
    hipLaunchKernelGGL(topk_dense_kernel<32>, dim3((int)blocks), dim3(256), 0, st, S, B, N, lds,
                       K, base, os, oi);
  else
    hipLaunchKernelGGL(topk_dense_kernel<64>, dim3((int)blocks), dim3(256), 0, st, S, B, N, lds,
                       K, base, os, oi);
}

}  // namespace hhfm
