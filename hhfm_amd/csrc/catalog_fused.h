// K2 small-catalog path (C3: evaluate_TopK over Frappe's 4,082 items;
// Newcode/OurModel7.py:294-295, FM.py:180-185): scores + exact top-K in ONE
// kernel launch — the [B, N] score matrix is never written and the split
// lists are merged inside the launch (no topk_merge kernel).  Included by
// catalog_topk.hip (uses its tile constants, split-bf16 helpers and the
// wave-level top-K primitives of topk_common.h).
//
// S workgroups per 32 queries, each = 8 waves x one range of 8·T item tiles
// (wave w takes the range's tiles [w·T, w·T + T)):
//   0. the 32 query vectors formed in LDS (catalog_queries' arithmetic), each
//      wave's MFMA B operands built from them (catalog_main's split pieces);
//      the wave's first item tiles are already in flight;
//   1. every wave scores its T tiles with catalog_main's exact MFMA sequence
//      (same products, same order: the same bits as the selecting and STORE
//      kernels) and keeps the T x 16 scores of its lanes in registers;
//   2. threshold: every (wave, lane half, tile) is a group of 16 items of one
//      query.  Each lane offers its two largest tile maxima, 32 values per
//      query; their K-th largest t is the maximum of K distinct groups, so K
//      items of the range score >= t (~K·1.2 of a 1,024-item range do);
//   3. the survivors (score >= t) go to a per-query LDS list.  A list past
//      kFusedCap (heavy exact ties) raises the threshold to the K-th best
//      (score, index) PAIR among those collected and filters again — each
//      round drops at least kFusedCap - K items, so it ends, and the pair
//      order keeps tf.nn.top_k's ties;
//   4. per query the entries at or above the final threshold are sorted by
//      one 32-lane key network: the range's exact top K;
//   5. S > 1: the sorted lists are stored write-through (sc1), every storing
//      wave drains, and one lane adds to the query group's arrival counter
//      (agent scope); the workgroup whose add comes last loads the S lists
//      with sc1 loads, merges them and writes the top K, then re-arms the
//      counter (MI355X_MICROARCH.md § visibility, the first row of the
//      hand-off table; no fence, no second launch).
// Exactness: every range contributes a superset of its top K under the strict
// (score desc, index asc) order, so the lists equal the dense path's.
//
// Selection arithmetic is branch-free on the VALU: entries are 64-bit keys
// compared by v_cmp_u64 (the (score, index) pair compare compiled to
// SALU/exec-mask sequences that cost ~20 cycles per instruction here), the
// survivors leave registers through a select tree, and barriers are LDS-only
// (the item tiles in flight stay in flight across them).
#pragma once

namespace hhfm {

// diagnostic: s_memtime at the phase boundaries, every wave's phase
// durations summed into g_fused_t (read by hhfm_debug_fused_timing; timing
// only; 1 = on)
#ifndef HHFM_FUSED_TIMING
#define HHFM_FUSED_TIMING 0
#endif
#if HHFM_FUSED_TIMING && !defined(HHFM_DIAG_BUILD)
#error "HHFM_FUSED_TIMING: diagnostic builds only (-DHHFM_DIAG_BUILD)"
#endif
#if HHFM_FUSED_TIMING
// [0] query phase, [1] scores, [2] threshold, [3] survivors (+ overflow
// rounds), [4] range sort and hand-off, [5] waves, [6] merging workgroups,
// [7] merge
__device__ unsigned long long g_fused_t[8];
#define HHFM_TMARK(v) v = __builtin_amdgcn_s_memtime()
#else
#define HHFM_TMARK(v) (void)0
#endif

constexpr int kFusedCap = 128;    // list entries held per query
// arrival counters (one per 32 queries) at the workspace's start
constexpr int kFusedMaxGroups = HHFM_CATALOG_WS_ZERO / 4;
constexpr int kFusedMaxS = 16;    // item ranges (workgroups) per 32 queries
constexpr int kFusedTiles = 4;    // item tiles per wave: a range = 8 x 4 tiles = 1,024 items
constexpr int kFusedMaxCtx = 8;   // context (and time) fields the fused kernel takes
constexpr int kFusedWaves = 8;

// workgroup barrier that orders LDS only: outstanding global loads (the next
// item tiles) stay in flight across it (__syncthreads waits for them)
HHFM_DEV void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// bitonic sort of scores in aligned groups of N lanes (no indices: only the
// K-th value is wanted), Q independent sorts interleaved stage by stage
template <int N, int Q>
HHFM_DEV void sort_desc_scores_n(float (&s)[Q]) {
  const int l = lane_id() & (N - 1);
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
    const bool desc = (l & size) == 0 || size == N;
#pragma unroll
    for (int d = size >> 1; d >= 1; d >>= 1) {
      const bool keep_max = ((l & d) == 0) == desc;
      float ps[Q];
#pragma unroll
      for (int u = 0; u < Q; ++u) ps[u] = xor_lane(s[u], d);
#pragma unroll
      for (int u = 0; u < Q; ++u) s[u] = keep_max ? fmaxf(s[u], ps[u]) : fminf(s[u], ps[u]);
    }
  }
}

// Entry keys: one uint64 per (score, index), larger = better under the
// strict (score desc, index asc) order of tf.nn.top_k — the high word the
// order-preserving bits of the score, the low word ~index.  Compares and
// swaps are then a v_cmp_u64 and two v_cndmask (no exec-mask branches: the
// (score, index) pair compare compiled to SALU/exec sequences that cost
// ~20 cycles per instruction here).  Key 0 is below every entry (empty).
HHFM_DEV uint32_t ukey(float f) {
  const uint32_t b = __float_as_uint(f);
  return b ^ ((uint32_t)((int32_t)b >> 31) | 0x80000000u);
}
HHFM_DEV float ukey_inv(uint32_t k) {
  return __uint_as_float(k ^ ((k & 0x80000000u) ? 0x80000000u : 0xffffffffu));
}
HHFM_DEV uint64_t ekey(float s, int32_t i) {
  return ((uint64_t)ukey(s) << 32) | (uint32_t)~i;
}
HHFM_DEV uint64_t xor_lane64(uint64_t v, int d) {
  const uint32_t lo = (uint32_t)xor_lane((int32_t)(uint32_t)v, d);
  const uint32_t hi = (uint32_t)xor_lane((int32_t)(uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
// bitonic sort of keys, descending, in aligned groups of N lanes
template <int N>
HHFM_DEV void sort_keys_desc(uint64_t& k) {
  const int l = lane_id() & (N - 1);
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
    const bool desc = (l & size) == 0 || size == N;
#pragma unroll
    for (int d = size >> 1; d >= 1; d >>= 1) {
      const uint64_t p = xor_lane64(k, d);
      const bool keep_max = ((l & d) == 0) == desc;
      k = ((p > k) == keep_max) ? p : k;
    }
  }
}
// the best N of the union of two descending key lists A (self) and B, in
// aligned groups of N lanes: max(A[l], B[N-1-l]) is bitonic, then merged
template <int N>
HHFM_DEV void merge_keys(uint64_t& a, uint64_t b) {
  const int l = lane_id();
  const int src = (l & ~(N - 1)) | (N - 1 - (l & (N - 1)));
  const uint32_t blo = (uint32_t)__shfl((int32_t)(uint32_t)b, src, kWave);
  const uint32_t bhi = (uint32_t)__shfl((int32_t)(uint32_t)(b >> 32), src, kWave);
  const uint64_t r = ((uint64_t)bhi << 32) | blo;
  a = r > a ? r : a;
  const int lg = l & (N - 1);
#pragma unroll
  for (int d = N >> 1; d >= 1; d >>= 1) {
    const uint64_t p = xor_lane64(a, d);
    a = ((p > a) == ((lg & d) == 0)) ? p : a;
  }
}
// v[r] for a lane-dependent r in [0, 16): a 4-level tree of bitwise blends
// (v_bfi_b32).  Written as selects, the compiler turns them into a load
// through a selected address and moves the score array to scratch.
HHFM_DEV float select16(const float (&v)[16], int r) {
  auto bl = [](uint32_t a, uint32_t b, uint32_t m) { return (b & m) | (a & ~m); };
  const uint32_t m0 = 0u - (uint32_t)(r & 1), m1 = 0u - (uint32_t)((r >> 1) & 1);
  const uint32_t m2 = 0u - (uint32_t)((r >> 2) & 1), m3 = 0u - (uint32_t)((r >> 3) & 1);
  uint32_t a[8], b[4], c[2];
#pragma unroll
  for (int x = 0; x < 8; ++x) a[x] = bl(__float_as_uint(v[2 * x]), __float_as_uint(v[2 * x + 1]), m0);
#pragma unroll
  for (int x = 0; x < 4; ++x) b[x] = bl(a[2 * x], a[2 * x + 1], m1);
#pragma unroll
  for (int x = 0; x < 2; ++x) c[x] = bl(b[2 * x], b[2 * x + 1], m2);
  return __uint_as_float(bl(c[0], c[1], m3));
}

template <bool BF16, int KT, bool FM, bool SPLIT, int T>
__global__ __launch_bounds__(kFusedWaves * 64) void catalog_fused(
    const int32_t* __restrict__ qidx, int64_t B, int ncols, int mode, int ucol, int c0, int c1,
    int t0, int t1, const char* __restrict__ E, int64_t M, int64_t item_row_begin, int32_t N,
    const float* __restrict__ w, int K, float* __restrict__ out_s, int32_t* __restrict__ out_i,
    int32_t gbase, int S, uint32_t* __restrict__ arrive, uint64_t* __restrict__ part) {
  constexpr int k = BF16 ? KT * 16 : KT * 8;
  constexpr int64_t ROWB = (int64_t)KT * 32;
  constexpr int EPC = BF16 ? 8 : 4;
  constexpr int NW = kFusedWaves;
  constexpr int NU = SPLIT ? (BF16 ? KT : KT / 2) : 1;
  constexpr int R = 32 / (2 * NW);     // tile maxima a lane offers
  constexpr int kQS = kFusedCap + 1;   // list slots per query (the last: spare)
  // item tiles in flight per wave (one for bf16 k >= 128: its 96 registers of
  // query pieces leave no room for a second)
  constexpr int PD = BF16 && KT >= 8 ? 1 : 2;
  static_assert(T % PD == 0, "tiles per wave a multiple of the prefetch depth");

  __shared__ float hq[kQPerWave][k + 4];
  __shared__ float cq_l[kQPerWave];
  __shared__ float pq[kQPerWave][64];   // FM: per query, catalog_queries' 64 lane values
  __shared__ float gmx[kQPerWave][33];  // per query the 32 offered group values
  __shared__ uint64_t thr_k[kQPerWave];   // entries with a key >= pass
  __shared__ int32_t cnt[kQPerWave], cprev[kQPerWave], redo[kQPerWave];
  __shared__ int32_t ovf[2];
  __shared__ uint64_t cbuf[kQPerWave * kQS];   // entry keys
  __shared__ uint64_t fscr[NW][kWave];         // range sort: compacted keys
  __shared__ int32_t last_sh;                  // this workgroup merges its group

  const int wv = threadIdx.x / kWave;
  const int l = lane_id();
  const int j = l & 31, h = l >> 5;
  const int g = blockIdx.x / S, split = blockIdx.x - (blockIdx.x / S) * S;
  const int64_t q0 = (int64_t)g * kQPerWave;
  const bool live = q0 + j < B;   // this lane's query exists (rows past B add nothing)
  const int ntiles = (N + kTile - 1) / kTile;
  const int tile0 = (split * NW + wv) * T;   // this wave's first tile
  int rnd = 0;   // survivor rounds so far (selects the overflow flag word)

#if HHFM_FUSED_TIMING
  uint64_t tm0 = 0, tm1 = 0, tacc[6] = {0, 0, 0, 0, 0, 0};
#endif
  HHFM_TMARK(tm0);
  // the query rows' raw ids first (8 threads per query; only the first 256
  // threads form queries): their loads are the oldest, so waiting for them
  // leaves the tile loads below in flight (vmcnt counts in order)
  const int pq_q = threadIdx.x >> 3;
  const int64_t pq_b = q0 + pq_q;
  const bool pq_on = threadIdx.x < 8 * kQPerWave && pq_b < B;
  int32_t idu = 0, idc[kFusedMaxCtx], idt[kFusedMaxCtx];
#pragma unroll
  for (int f = 0; f < kFusedMaxCtx; ++f) idc[f] = idt[f] = 0;
  if (pq_on) {
    const int32_t* p = qidx + pq_b * (int64_t)ncols;
    idu = p[ucol];
#pragma unroll
    for (int f = 0; f < kFusedMaxCtx; ++f) {
      if (f < c1 - c0) idc[f] = p[c0 + f];
      if (f < t1 - t0) idt[f] = p[t0 + f];
    }
  }
  asm volatile("" ::: "memory");   // keep the tile loads behind them
  // the wave's tile tt -> catalog tile (clamped: every load is issued, so
  // the counted waits stay exact)
  auto tile_of = [&](int tt) {
    const int t = tile0 + (tt < T ? tt : T - 1);
    return t < ntiles ? t : ntiles - 1;
  };
  auto item_of = [&](int tile) {
    const int item = tile * kTile + j;
    return item < N ? item : N - 1;
  };
  uint4 ar[PD][KT];
  float wr[PD];
  auto load_tile = [&](int tile, uint4 (&a)[KT], float& wv_) {
    const char* row = E + (item_row_begin + item_of(tile)) * ROWB + 16 * h;
#pragma unroll
    for (int t = 0; t < KT; ++t) a[t] = *reinterpret_cast<const uint4*>(row + 32 * t);
    if constexpr (FM) wv_ = w ? w[item_row_begin + item_of(tile)] : 0.f;
  };
#pragma unroll
  for (int d = 0; d < PD; ++d) {
    wr[d] = 0.f;
    load_tile(tile_of(d), ar[d], wr[d]);
  }

  // ---- 0. query vectors (catalog_queries' arithmetic, bit for bit) ----
  // 8 threads per query; thread tp loads 16-B chunks tp, tp + 8, ... of each
  // field's row (every id and row load of the workgroup issued before any
  // is used).  FM's item-independent q·f = Σ_e h_e f_e: lane L = e mod 64 of
  // catalog_queries accumulates e then e + 64 (chunks tp and tp + 64/EPC of
  // one thread hold both), the 64 lane values go through LDS and one wave per
  // query sums them with catalog_queries' own butterfly (group_sum).
  {
    constexpr int CPR = k / EPC;              // 16-B chunks per row
    constexpr int CPT = (CPR + 7) / 8;        // chunks per thread
    const int qq = threadIdx.x >> 3, tp = threadIdx.x & 7;
    const int64_t b = q0 + qq;
    if (threadIdx.x < 8 * kQPerWave) {
      idu = clamp_id(idu, M);
#pragma unroll
      for (int f = 0; f < kFusedMaxCtx; ++f) {
        idc[f] = clamp_id(idc[f], M);
        idt[f] = clamp_id(idt[f], M);
      }
      // lane L = e mod 64 accumulates e, then e + 64: chunk slot cc % LPT
      constexpr int LPT = 64 / (8 * EPC) > 0 ? 64 / (8 * EPC) : 1;
      float part[LPT][EPC];
#pragma unroll
      for (int c = 0; c < LPT; ++c)
#pragma unroll
        for (int v = 0; v < EPC; ++v) part[c][v] = 0.f;
      auto cvt = [&](const uint4& u, float (&x)[EPC]) {
        if constexpr (BF16) {
          const uint32_t r4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            x[2 * v] = __uint_as_float(r4[v] << 16);
            x[2 * v + 1] = __uint_as_float(r4[v] & 0xffff0000u);
          }
        } else {
          x[0] = __uint_as_float(u.x); x[1] = __uint_as_float(u.y);
          x[2] = __uint_as_float(u.z); x[3] = __uint_as_float(u.w);
        }
      };
      const int nc = c1 - c0, nt = t1 - t0;
#pragma unroll
      for (int cc = 0; cc < CPT; ++cc) {
        const int ch = tp + 8 * cc;
        if (ch < CPR) {
          auto ld = [&](int32_t id) {
            return *reinterpret_cast<const uint4*>(E + (int64_t)id * ROWB + 16 * ch);
          };
          // every field row of a chunk loaded before any is summed (one memory
          // latency, not one per field)
          const uint4 ru = ld(idu);
          uint4 rc[kFusedMaxCtx], rt[kFusedMaxCtx];
#pragma unroll
          for (int f = 0; f < kFusedMaxCtx; ++f) {
            rc[f] = make_uint4(0, 0, 0, 0);
            rt[f] = make_uint4(0, 0, 0, 0);
            if (f < nc) rc[f] = ld(idc[f]);
            if (f < nt) rt[f] = ld(idt[f]);
          }
          float uu[EPC], cx[EPC], tm[EPC], r[EPC];
          cvt(ru, uu);
#pragma unroll
          for (int v = 0; v < EPC; ++v) {
            cx[v] = 0.f;
            tm[v] = 0.f;
          }
          // ctx fields, then time fields, in field order
#pragma unroll
          for (int f = 0; f < kFusedMaxCtx; ++f) {
            if (f >= nc) break;
            cvt(rc[f], r);
#pragma unroll
            for (int v = 0; v < EPC; ++v) cx[v] += r[v];
          }
#pragma unroll
          for (int f = 0; f < kFusedMaxCtx; ++f) {
            if (f >= nt) break;
            cvt(rt[f], r);
#pragma unroll
            for (int v = 0; v < EPC; ++v) tm[v] += r[v];
          }
#pragma unroll
          for (int v = 0; v < EPC; ++v) {
            float hv = 0.f;
            if (b < B) {
              if (mode == HHFM_MODE_FM) {
                hv = uu[v] + cx[v];                     // FM.py:177
                part[cc % LPT][v] += hv * cx[v];        // FM.py:178-183
              } else {
                hv = uu[v];                             // OurModel7.py:270-292
                if (c1 > c0) hv = hv + cx[v];
                if (t1 > t0) hv = hv + tm[v];
              }
            }
            hq[qq][EPC * ch + v] = hv;
          }
        }
      }
      if (mode == HHFM_MODE_FM) {
#pragma unroll
        for (int c = 0; c < LPT; ++c) {
          const int ch = tp + 8 * c;
          if (ch < CPR && EPC * ch < 64)
#pragma unroll
            for (int v = 0; v < EPC; ++v) pq[qq][EPC * ch + v] = part[c][v];
        }
      }
    }
    if (threadIdx.x < kQPerWave) {
      cnt[threadIdx.x] = 0;
      // the lowest finite score: items past N (held as -inf) never pass
      thr_k[threadIdx.x] = (uint64_t)ukey(-__FLT_MAX__) << 32;
    }
    if (threadIdx.x < 2) ovf[threadIdx.x] = 0;
    lds_barrier();
    if (mode == HHFM_MODE_FM) {
      for (int q2 = wv; q2 < kQPerWave; q2 += NW) {
        float x = l < k ? pq[q2][l] : 0.f;
        x = group_sum<kWave>(x);
        if (l == 0) cq_l[q2] = x;
      }
      lds_barrier();
    }
  }

  // B operand (catalog_main): this lane's query j, k slices {EPC(2t+h) ..}
  float bq[KT][EPC];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int e = 0; e < EPC; ++e) bq[t][e] = hq[j][(2 * t + h) * EPC + e];
  bf16x8 qp[3][NU];
  if constexpr (SPLIT) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (BF16) x[e] = bq[u][e];
        else x[e] = bq[2 * u + (e >> 2)][e & 3];
      }
      split3x8(x, qp[0][u], qp[1][u], qp[2][u]);
    }
  }
  const float cq = FM ? cq_l[j] : 0.f;
#if HHFM_FUSED_TIMING
  HHFM_TMARK(tm1);
  tacc[0] += tm1 - tm0;
#endif

  {
    HHFM_TMARK(tm0);
    // ---- 1. scores of this wave's T tiles, kept in registers ----
    float sc[T][16];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) {
      const int tile = tile0 + tt;
      uint4 (&ar_)[KT] = ar[tt % PD];
      // this slot is refilled with tile tt + PD, chunk by chunk
      const int nxt = tile_of(tt + PD);
      const char* nrow = E + (item_row_begin + item_of(nxt)) * ROWB + 16 * h;
      f32x16 acc = {0};
      const float wcur = wr[tt % PD];
      if constexpr (SPLIT && BF16) {
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const bf16x8 ai = __builtin_bit_cast(bf16x8, ar_[t]);
          ar_[t] = *reinterpret_cast<const uint4*>(nrow + 32 * t);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ai, qp[2][t], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ai, qp[1][t], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ai, qp[0][t], acc, 0, 0, 0);
        }
      } else if constexpr (SPLIT) {
#pragma unroll
        for (int u = 0; u < KT / 2; ++u) {
          const float x[8] = {__uint_as_float(ar_[2 * u].x), __uint_as_float(ar_[2 * u].y),
                              __uint_as_float(ar_[2 * u].z), __uint_as_float(ar_[2 * u].w),
                              __uint_as_float(ar_[2 * u + 1].x), __uint_as_float(ar_[2 * u + 1].y),
                              __uint_as_float(ar_[2 * u + 1].z), __uint_as_float(ar_[2 * u + 1].w)};
          ar_[2 * u] = *reinterpret_cast<const uint4*>(nrow + 32 * (2 * u));
          ar_[2 * u + 1] = *reinterpret_cast<const uint4*>(nrow + 32 * (2 * u + 1));
          bf16x8 i0, i1, i2;
          split3x8(x, i0, i1, i2);
          const bf16x8 p0 = qp[0][u], p1 = qp[1][u], p2 = qp[2][u];
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i2, p0, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i1, p1, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i0, p2, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i1, p0, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i0, p1, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i0, p0, acc, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          float av[EPC];
          if constexpr (BF16) {
            const uint32_t r4[4] = {ar_[t].x, ar_[t].y, ar_[t].z, ar_[t].w};
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              av[2 * v] = __uint_as_float(r4[v] << 16);
              av[2 * v + 1] = __uint_as_float(r4[v] & 0xffff0000u);
            }
          } else {
            av[0] = __uint_as_float(ar_[t].x); av[1] = __uint_as_float(ar_[t].y);
            av[2] = __uint_as_float(ar_[t].z); av[3] = __uint_as_float(ar_[t].w);
          }
          ar_[t] = *reinterpret_cast<const uint4*>(nrow + 32 * t);
#pragma unroll
          for (int e = 0; e < EPC; ++e)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bq[t][e], acc, 0, 0, 0);
        }
      }
      if constexpr (FM) {   // D[i][j] += w_i·1 + 1·(q_j·f_j)   (catalog_main)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h == 0 ? wcur : 1.f, h == 0 ? 1.f : cq, acc,
                                                   0, 0, 0);
        wr[tt % PD] = w ? w[item_row_begin + item_of(nxt)] : 0.f;
      }
      const int ibase = tile * kTile;
      if (ibase + kTile <= N) {   // wave-uniform: only the catalog's last tiles are partial
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[tt][r] = acc[r];
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
          sc[tt][r] = ibase + row < N ? acc[r] : kNegInf;
        }
      }
      // one tile in flight: keeps the compiler from hoisting later tiles' loads
      asm volatile("" ::: "memory");
    }
#if HHFM_FUSED_TIMING
    HHFM_TMARK(tm1);
    tacc[1] += tm1 - tm0;
    tm0 = tm1;
#endif

    // ---- 2. threshold: K-th largest of the 32 offered tile maxima ----
    {
      float mr[R];   // this lane's R largest tile maxima, descending
#pragma unroll
      for (int r = 0; r < R; ++r) mr[r] = kNegInf;
#pragma unroll
      for (int tt = 0; tt < T; ++tt) {
        float m = sc[tt][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) m = fmaxf(m, sc[tt][r]);
#pragma unroll
        for (int r = 0; r < R; ++r) {   // insert: the larger stays, the smaller moves on
          const float hi = fmaxf(mr[r], m);
          m = fminf(mr[r], m);
          mr[r] = hi;
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) gmx[j][(wv * 2 + h) * R + r] = mr[r];
    }
    lds_barrier();
    {   // wave wv: queries QW wv + 2u + h, one per 32-lane half
      constexpr int QW = kQPerWave / NW, U = QW / 2;
      float m[U];
#pragma unroll
      for (int u = 0; u < U; ++u) m[u] = gmx[wv * QW + 2 * u + h][j];
      sort_desc_scores_n<32, U>(m);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float t = shfl_f(m[u], (h << 5) + K - 1);
        const int qq = wv * QW + 2 * u + h;
        // a raised pair threshold of equal score stays (its key is larger)
        const uint64_t tk = (uint64_t)ukey(t) << 32;
        if (j == 0 && tk > thr_k[qq]) thr_k[qq] = tk;
      }
    }
    if (threadIdx.x < kQPerWave) cprev[threadIdx.x] = cnt[threadIdx.x];
    lds_barrier();
#if HHFM_FUSED_TIMING
    HHFM_TMARK(tm1);
    tacc[2] += tm1 - tm0;
    tm0 = tm1;
#endif

    // ---- 3. survivors to the per-query lists (re-filtered on overflow) ----
    const int qbase = j * kQS;
    bool first = true;
#pragma unroll 1
    for (;;) {
      // this round's filter: every live query in the chunk's first round,
      // afterwards only the queries whose list overflowed (redo); rows past B
      // never pass (their zero query ties every item at 0)
      const bool mine = live && (first || redo[j]);
      const uint64_t tk = thr_k[j];
      const uint32_t tlo = (uint32_t)tk;
      // NaN: no score passes
      const float ts = mine ? ukey_inv((uint32_t)(tk >> 32)) : __builtin_nanf("");
      // item index of (tile tt, row r) = ib + 32 tt + row(r); laundered so the
      // compiler does not hoist 16 T indices out of the loop into registers
      int32_t ib = tile0 * kTile + 4 * h;
      asm volatile("" : "+v"(ib));
      uint32_t pm[T];   // pass bits of the lane's 16 rows per tile
      // a score threshold (low word 0 on every lane) is `score >= t` (items
      // past N hold -inf); a raised pair threshold takes the key test
      if (__ballot(mine && tlo != 0) == 0) {
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
          uint32_t m = 0;
#pragma unroll
          for (int r = 15; r >= 0; --r) m = m + m + (sc[tt][r] >= ts ? 1u : 0u);
          pm[tt] = m;
        }
      } else {
        // key >= (ukey(ts), ~ti)  <=>  x > ts, or x == ts and index <= ti
        const int32_t ti = ~(int32_t)tlo;
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
          uint32_t m = 0;
#pragma unroll
          for (int r = 15; r >= 0; --r) {
            const int32_t it = ib + tt * kTile + (r & 3) + 8 * (r >> 2);
            const float x = sc[tt][r];
            const bool pass = (it < N) & ((x > ts) | ((x == ts) & (it <= ti)));
            m = m + m + (pass ? 1u : 0u);
          }
          pm[tt] = m;
        }
      }
      int n = 0;
#pragma unroll
      for (int tt = 0; tt < T; ++tt) n += __popc(pm[tt]);
      int pos = atomicAdd(&cnt[j], n);
      asm volatile("" : "+v"(ib));   // recompute the indices below (no 16 T live values)
      // one survivor per lane per step (lowest row first); a lane without one
      // writes the query's spare slot (no exec-mask branches)
#pragma unroll
      for (int tt = 0; tt < T; ++tt) {
        uint32_t m = pm[tt];
#pragma unroll 1
        while (__ballot(m != 0) != 0) {
          const int r = __builtin_ctz(m | 0x10000u) & 15;
          const float x = select16(sc[tt], r);
          const int32_t it = ib + tt * kTile + (r & 3) + 8 * (r >> 2);
          const int slot = m ? (pos < kFusedCap ? pos : kFusedCap) : kFusedCap;
          cbuf[qbase + slot] = ekey(x, it);
          pos += m ? 1 : 0;
          m &= m - 1;
        }
      }
      // a lane whose last slot lies past the cap flags the overflow in this
      // round's flag word (two words alternate, so the reset of the next
      // round's word never races with this round's writers)
      if (pos > kFusedCap) ovf[rnd & 1] = 1;
      lds_barrier();
      const bool over = ovf[rnd & 1] != 0;
      if (threadIdx.x == 0) ovf[(rnd + 1) & 1] = 0;   // last read before this barrier
      ++rnd;
      first = false;
      if (!over) break;
      // overflowed queries (rare: heavy exact ties): the K-th best key among
      // the kFusedCap collected becomes the threshold (at least K items reach
      // it; only K of the collected do), the earlier chunks' entries [0,
      // cprev) below it are dropped, and the chunk is filtered again for
      // those queries only
#pragma unroll 1
      for (int qq = wv; qq < kQPerWave; qq += NW) {
        const bool of = cnt[qq] > kFusedCap;   // wave-uniform
        if (l == 0) redo[qq] = of ? 1 : 0;
        if (!of) continue;
        const uint64_t e0 = cbuf[qq * kQS + l], e1 = cbuf[qq * kQS + l + 64];
        uint64_t k0 = e0, k1 = e1;
        sort_keys_desc<64>(k0);
        sort_keys_desc<64>(k1);
        merge_keys<64>(k0, k1);   // the best 64 of the 128, sorted
        const uint32_t nlo = __builtin_amdgcn_readlane((int32_t)(uint32_t)k0, K - 1);
        const uint32_t nhi = __builtin_amdgcn_readlane((int32_t)(uint32_t)(k0 >> 32), K - 1);
        const uint64_t nk = ((uint64_t)nhi << 32) | nlo;
        const int np = cprev[qq];
        const bool a0 = l < np && e0 >= nk;
        const bool a1 = l + 64 < np && e1 >= nk;
        const uint64_t b0 = __ballot(a0), b1 = __ballot(a1);
        const int p0 = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0u));
        const int p1 = __popcll(b0) + (int)__builtin_amdgcn_mbcnt_hi(
                                          (uint32_t)(b1 >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
        __builtin_amdgcn_wave_barrier();   // every lane's reads before any write
        if (a0) cbuf[qq * kQS + p0] = e0;
        if (a1) cbuf[qq * kQS + p1] = e1;
        if (l == 0) {
          const int kept = __popcll(b0) + __popcll(b1);
          thr_k[qq] = nk;
          cnt[qq] = kept;
          cprev[qq] = kept;
        }
      }
      lds_barrier();
    }
#if HHFM_FUSED_TIMING
    HHFM_TMARK(tm1);
    tacc[3] += tm1 - tm0;
#endif
  }

  // ---- 4. per query: the range's entries at or above the final threshold,
  // sorted (its exact top K) ----
  // Two queries per pass, one per 32-lane half: a half's lanes load its
  // query's entries 32 at a time, the passing ones are compacted into the
  // wave's LDS scratch and one 32-lane key network sorts them (typically
  // ~K·1.2 pass).  A query with more than 32 passing takes the 64-lane
  // network (+ merges past 64), one query at a time.
  HHFM_TMARK(tm0);
  typedef __attribute__((address_space(1))) uint64_t gu64;
  typedef __attribute__((address_space(1))) uint32_t gu32;
  // rank r of query qq: the output (S = 1) or the range's list, stored
  // write-through (sc1) for the merging workgroup
  auto emit = [&](int qq, int r, uint64_t key) {
    if (S == 1) {
      const int64_t b = q0 + qq;
      if (b < B && r < K) {
        out_s[b * K + r] = ukey_inv((uint32_t)(key >> 32));
        const int32_t it = ~(int32_t)(uint32_t)key;
        out_i[b * K + r] = it == kNoIdx ? kNoIdx : it + gbase;
      }
    } else {
      gu64* dst = (gu64*)(part + (((int64_t)blockIdx.x * kQPerWave + qq) << 5) + r);
      __hip_atomic_store(dst, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  {
    constexpr int QW = kQPerWave / NW, U = QW / 2;
#pragma unroll 1
    for (int u = 0; u < U; ++u) {
      const int qq = wv * QW + 2 * u + h;
      const int nq = cnt[qq] < kFusedCap ? cnt[qq] : kFusedCap;
      const uint64_t tk = thr_k[qq];
      int nv = 0;   // passing entries of this half's query so far
#pragma unroll 1
      for (int c = 0; c < kFusedCap; c += 32) {
        if (__ballot(c < nq) == 0) break;   // both halves done
        const uint64_t e = cbuf[qq * kQS + (c + j < nq ? c + j : kFusedCap)];
        const bool ok = c + j < nq && e >= tk;
        const uint64_t bm = __ballot(ok);
        const uint32_t hm = h ? (uint32_t)(bm >> 32) : (uint32_t)bm;
        const int pre = __popc(hm & ((1u << j) - 1u));
        if (ok && nv + pre < 32) fscr[wv][(h << 5) + nv + pre] = e;
        nv += __popc(hm);
      }
      if (__ballot(nv > 32) == 0) {
        uint64_t key = j < nv ? fscr[wv][(h << 5) + j] : 0ull;
        sort_keys_desc<32>(key);
        emit(qq, j, key);
      } else {   // rare: one query at a time over the whole wave
#pragma unroll 1
        for (int hh = 0; hh < 2; ++hh) {
          const int q2 = wv * QW + 2 * u + hh;
          const int n2 = cnt[q2] < kFusedCap ? cnt[q2] : kFusedCap;
          const uint64_t t2 = thr_k[q2];
          uint64_t top = 0;
#pragma unroll 1
          for (int c = 0; c < n2; c += kWave) {
            const uint64_t e = cbuf[q2 * kQS + (c + l < n2 ? c + l : kFusedCap)];
            uint64_t key = (c + l < n2 && e >= t2) ? e : 0ull;
            sort_keys_desc<64>(key);
            if (c == 0) top = key;
            else merge_keys<32>(top, key);
            if (l >= 32) top = 0;
          }
          if (l < 32) emit(q2, l, top);
        }
      }
    }
  }
#if HHFM_FUSED_TIMING
  HHFM_TMARK(tm1);
  tacc[4] += tm1 - tm0;
  tm0 = tm1;
#endif

  // ---- 5. S > 1: hand-off, the last arriving workgroup merges ----
  bool merged = false;
  if (S > 1) {
    // every storing wave drains its sc1 stores, then the barrier, then ONE
    // lane's agent-scope add for the whole workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (threadIdx.x == 0) {
      const uint32_t old = __hip_atomic_fetch_add((gu32*)(arrive + g), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      last_sh = old == (uint32_t)(S - 1);
    }
    lds_barrier();
    merged = last_sh != 0;   // uniform
    if (merged) {
      // no instruction: keeps the sc1 loads below the barrier
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      constexpr int QW = kQPerWave / NW;
      constexpr int kMaxS = kFusedMaxS;
#pragma unroll 1
      for (int u = 0; u < QW; ++u) {
        const int qq = wv * QW + u;
        // lane (h, j) holds rank j of the lists h, h + 2, ...: all loads in
        // flight before the merges
        uint64_t v[kMaxS / 2];
#pragma unroll
        for (int x = 0; x < kMaxS / 2; ++x) {
          const int sl = 2 * x + h;
          v[x] = 0;
          if (2 * x < S) {   // wave-uniform
            const gu64* src =
                (const gu64*)(part + ((((int64_t)g * S + (sl < S ? sl : 0)) * kQPerWave + qq) << 5) + j);
            const uint64_t t = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[x] = sl < S ? t : 0ull;
          }
        }
        uint64_t a = v[0];
#pragma unroll
        for (int x = 1; x < kMaxS / 2; ++x)
          if (2 * x < S) merge_keys<32>(a, v[x]);
        merge_keys<32>(a, xor_lane64(a, 32));   // the odd lists' half into the even's
        const int64_t b = q0 + qq;
        if (b < B && l < K) {
          out_s[b * K + l] = ukey_inv((uint32_t)(a >> 32));
          const int32_t it = ~(int32_t)(uint32_t)a;
          out_i[b * K + l] = it == kNoIdx ? kNoIdx : it + gbase;
        }
      }
      // re-arm the counter for the next call (stream order publishes it)
      if (threadIdx.x == 0)
        __hip_atomic_store((gu32*)(arrive + g), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#if HHFM_FUSED_TIMING
  HHFM_TMARK(tm1);
  tacc[5] += tm1 - tm0;
  if (l == 0) {
#pragma unroll
    for (int p = 0; p < 5; ++p) atomicAdd(&g_fused_t[p], tacc[p]);
    atomicAdd(&g_fused_t[5], 1ull);
    if (merged) {
      atomicAdd(&g_fused_t[6], 1ull);
      atomicAdd(&g_fused_t[7], tacc[5]);
    }
  }
#endif
  (void)merged;
}

}  // namespace hhfm
