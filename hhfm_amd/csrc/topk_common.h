// Wave-level top-K primitives (64-lane CDNA wavefronts).
//
// A top-K list lives one entry per lane (lanes [0, KPAD)), sorted by the
// tf.nn.top_k order: score descending, index ascending on equal scores
// (FM.py:185 / OurModel7.py:295 fetch tf.nn.top_k(score, 20)).
#pragma once
#include "hhfm_common.h"

#ifndef HHFM_TOPK_NV
#define HHFM_TOPK_NV 32   // scores per lane per chunk in topk_dense
#endif
#ifndef HHFM_TOPK_NT
#define HHFM_TOPK_NT 1    // non-temporal score loads in topk_dense
#endif

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
//
// The row is read in chunks of NV·64 scores, all NV loads of a lane issued
// before any is used (one memory latency per chunk, not one per 64 scores).
// Before filtering a chunk, the threshold is raised to the K-th best of the
// chunk's 64 lane maxima: K distinct lanes each hold a score at least that
// large, so it never exceeds the row's K-th best score and every top-K
// candidate still passes `s >= thr` — while nearly all others fail.  The
// chunk's candidates (typically 20–40) are compacted through LDS (ballot +
// mbcnt positions) into one register per lane, sorted by one 64-lane bitonic
// network and merged into the list in one step.  More than 64 candidates
// (heavy ties) fall back to per-64-score filtering.
// ---------------------------------------------------------------------------
// Fold one chunk of NV·64 scores (lane l holds v[j] = score of index
// cb + 64 j + l = src[64 j + l]; indices >= n are ignored) into the wave's
// running top-K list (ls, li: lanes [0, KPAD), sorted) with threshold thr.
// cs / ci: 64 LDS slots private to the wave.  The rare heavy-tie path
// re-reads src in a rolled loop (keeps the kernel's code small: a fully
// unrolled fallback made these kernels instruction-fetch bound).
template <int KPAD, int NV>
HHFM_DEV void topk_fold_chunk(const float (&v)[NV], const float* src, int32_t cb, int32_t n,
                              int K, float& ls, int32_t& li, float& thr, float* cs_lds,
                              int32_t* ci_lds) {
  const int l = lane_id();
  if (thr == kNegInf) {   // list not full yet: K-th best lane maximum bounds the K-th score
    float mx = v[0];
#pragma unroll
    for (int j = 1; j < NV; ++j) mx = fmaxf(mx, cb + j * kWave + l < n ? v[j] : kNegInf);
    if (cb + l >= n) mx = kNegInf;
    int32_t dummy = l;
    bitonic_sort_desc<64>(mx, dummy);
    thr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mx), K - 1));
  }
  // cheap test first: most chunks after the first hold few or no candidates
  int mine = 0;
#pragma unroll
  for (int j = 0; j < NV; ++j) mine += (cb + j * kWave + l < n && v[j] >= thr) ? 1 : 0;
  if (__ballot(mine > 0) == 0) return;
  int total = 0;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int32_t i = cb + j * kWave + l;
    const bool pass = i < n && v[j] >= thr;
    const uint64_t m = __ballot(pass);
    if (pass) {
      const int pos = total + (int)__builtin_amdgcn_mbcnt_hi(
                                  (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (pos < kWave) {
        cs_lds[pos] = v[j];
        ci_lds[pos] = i;
      }
    }
    total += __popcll(m);
  }
  if (total <= kWave) {
    __builtin_amdgcn_wave_barrier();
    float cs = l < total ? cs_lds[l] : kNegInf;
    int32_t ci = l < total ? ci_lds[l] : kNoIdx;
    __builtin_amdgcn_wave_barrier();   // the next chunk rewrites the slots
    // the smallest network that covers the candidates (lanes >= total hold -inf,
    // so the whole 64-lane sequence is sorted once the first group is)
    if (total <= 2) bitonic_sort_desc<2>(cs, ci);
    else if (total <= 4) bitonic_sort_desc<4>(cs, ci);
    else if (total <= 8) bitonic_sort_desc<8>(cs, ci);
    else if (total <= 16) bitonic_sort_desc<16>(cs, ci);
    else if (total <= 32) bitonic_sort_desc<32>(cs, ci);
    else bitonic_sort_desc<64>(cs, ci);
    merge_lists<KPAD>(ls, li, cs, ci);
  } else {   // heavy ties: filter 64 scores at a time
#pragma unroll 1
    for (int j = 0; j < NV; ++j) {
      const int32_t i = cb + j * kWave + l;
      const float x = i < n ? src[j * kWave + l] : kNegInf;
      const bool pass = i < n && x >= thr;
      if (__ballot(pass) == 0) continue;
      float cs = pass ? x : kNegInf;
      int32_t ci = pass ? i : kNoIdx;
      bitonic_sort_desc<64>(cs, ci);
      merge_lists<KPAD>(ls, li, cs, ci);
      if (l >= KPAD) { ls = kNegInf; li = kNoIdx; }
      thr = fmaxf(thr, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ls), K - 1)));
    }
  }
  if (l >= KPAD) { ls = kNegInf; li = kNoIdx; }
  thr = fmaxf(thr, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ls), K - 1)));
}

// Order-preserving float -> int32 key (signed compare == float compare).
HHFM_DEV int32_t fkey(float f) {
  const int32_t b = __float_as_int(f);
  return b >= 0 ? b : (b ^ 0x7fffffff);
}

// kth (optional): kth[b] = fkey of query b's K-th score (the threshold seed)
template <int KPAD, int NV>
__global__ __launch_bounds__(256) void topk_dense_kernel(const float* __restrict__ S,
                                                         int64_t B, int32_t N, int64_t lds,
                                                         int K, int32_t base,
                                                         float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i,
                                                         int32_t* __restrict__ kth) {
  __shared__ float cand_s[4][kWave];
  __shared__ int32_t cand_i[4][kWave];
  const int l = lane_id(), wv = (threadIdx.x >> 6) & 3;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t b = wave; b < B; b += nwave) {
    const float* row = S + b * lds;
    float ls = kNegInf;
    int32_t li = kNoIdx;
    float thr = kNegInf;
    for (int32_t cb = 0; cb < N; cb += NV * kWave) {
      float v[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int32_t i = cb + j * kWave + l;
        v[j] = i < N ? (HHFM_TOPK_NT ? __builtin_nontemporal_load(row + i) : row[i]) : kNegInf;
      }
      topk_fold_chunk<KPAD, NV>(v, row + cb, cb, N, K, ls, li, thr, cand_s[wv], cand_i[wv]);
    }
    if (l < K) {
      out_s[b * K + l] = ls;
      out_i[b * K + l] = li == kNoIdx ? kNoIdx : li + base;
      if (kth && l == K - 1) kth[b] = fkey(ls);
    }
  }
}

// Few queries (the reference's 300-row topk calls, the threshold seed's
// 1,024): WPQ waves of one workgroup share a query, each folding a
// contiguous 1/WPQ of the row into its own exact top-K, then the first wave
// merges the WPQ lists (merge_lists keeps the strict (score desc, index asc)
// order, so the result is the one-wave result bit for bit).  WPQ x more
// waves in flight for a latency-bound pass.
template <int KPAD, int NV, int WPQ>
__global__ __launch_bounds__(256) void topk_dense_split_kernel(const float* __restrict__ S,
                                                               int64_t B, int32_t N, int64_t lds,
                                                               int K, int32_t base,
                                                               float* __restrict__ out_s,
                                                               int32_t* __restrict__ out_i,
                                                               int32_t* __restrict__ kth) {
  constexpr int QB = 4 / WPQ;   // queries per workgroup
  __shared__ float cand_s[4][kWave];
  __shared__ int32_t cand_i[4][kWave];
  __shared__ float ms[4][KPAD];
  __shared__ int32_t mi[4][KPAD];
  const int l = lane_id(), wv = (threadIdx.x >> 6) & 3;
  const int qw = wv / WPQ, part = wv - qw * WPQ;
  // each part a multiple of 64 items (the last one may be short or empty)
  const int32_t span = (((N + WPQ - 1) / WPQ) + kWave - 1) / kWave * kWave;
  const int32_t lo = part * span < N ? part * span : N;
  const int32_t hi = lo + span < N ? lo + span : N;
  for (int64_t b0 = (int64_t)blockIdx.x * QB; b0 < B; b0 += (int64_t)gridDim.x * QB) {
    const int64_t b = b0 + qw;
    float ls = kNegInf;
    int32_t li = kNoIdx;
    if (b < B) {
      const float* row = S + b * lds;
      float thr = kNegInf;
      for (int32_t cb = lo; cb < hi; cb += NV * kWave) {
        float v[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const int32_t i = cb + j * kWave + l;
          v[j] = i < hi ? (HHFM_TOPK_NT ? __builtin_nontemporal_load(row + i) : row[i]) : kNegInf;
        }
        topk_fold_chunk<KPAD, NV>(v, row + cb, cb, hi, K, ls, li, thr, cand_s[wv], cand_i[wv]);
      }
    }
    if (l < KPAD) {
      ms[wv][l] = ls;
      mi[wv][l] = li;
    }
    __syncthreads();
    if (part == 0 && b < B) {
#pragma unroll
      for (int p = 1; p < WPQ; ++p) {
        const float bs = l < KPAD ? ms[wv + p][l] : kNegInf;
        const int32_t bi = l < KPAD ? mi[wv + p][l] : kNoIdx;
        merge_lists<KPAD>(ls, li, bs, bi);
        if (l >= KPAD) { ls = kNegInf; li = kNoIdx; }
      }
      if (l < K) {
        out_s[b * K + l] = ls;
        out_i[b * K + l] = li == kNoIdx ? kNoIdx : li + base;
        if (kth && l == K - 1) kth[b] = fkey(ls);
      }
    }
    __syncthreads();   // ms / mi are rewritten by the next query group
  }
}

// waves per query: 4 for <= 1,024 queries of >= 1,024 items (each folds a
// 64-aligned quarter, the first merges); one_wave (HHFM_PLAN_ONE_WAVE) keeps
// one wave per query at every size
static inline int topk_dense_wpq(int64_t B, int32_t N, bool one_wave) {
  if (one_wave || N < 1024) return 1;
  // (2 waves per query at 3,000 queries measured 48.4 vs 46.2 µs for C3)
  return B <= 1024 ? 4 : 1;
}

static inline void launch_topk_dense(const float* S, int64_t B, int32_t N, int64_t lds, int K,
                              int32_t base, float* os, int32_t* oi, hipStream_t st,
                              bool one_wave = false, int32_t* kth = nullptr) {
  const int wpq = topk_dense_wpq(B, N, one_wave);
  if (wpq > 1) {
    const int qb = 4 / wpq;
    int64_t blocks = (B + qb - 1) / qb;
    if (blocks > 8192) blocks = 8192;
#define HHFM_TOPK_SPLIT(KP, W)                                                                   \
  hipLaunchKernelGGL((topk_dense_split_kernel<KP, HHFM_TOPK_NV, W>), dim3((int)blocks), dim3(256), 0, \
                     st, S, B, N, lds, K, base, os, oi, kth)
    if (K <= 32) {
      if (wpq == 4) HHFM_TOPK_SPLIT(32, 4); else HHFM_TOPK_SPLIT(32, 2);
    } else {
      if (wpq == 4) HHFM_TOPK_SPLIT(64, 4); else HHFM_TOPK_SPLIT(64, 2);
    }
#undef HHFM_TOPK_SPLIT
    return;
  }
  int64_t blocks = (B + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (K <= 32)
    hipLaunchKernelGGL((topk_dense_kernel<32, HHFM_TOPK_NV>), dim3((int)blocks), dim3(256), 0, st, S, B, N, lds,
                       K, base, os, oi, kth);
  else
    hipLaunchKernelGGL((topk_dense_kernel<64, HHFM_TOPK_NV>), dim3((int)blocks), dim3(256), 0, st, S, B, N, lds,
                       K, base, os, oi, kth);
}

}  // namespace hhfm
