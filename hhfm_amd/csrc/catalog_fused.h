// K2 small-catalog path (C3: evaluate_TopK over Frappe's 4,082 items;
// Newcode/OurModel7.py:294-295, FM.py:180-185): scores + exact top-K in ONE
// kernel, the [B, N] score matrix never written.  Included by
// catalog_topk.hip (uses its tile constants, split-bf16 helpers and the
// wave-level top-K primitives of topk_common.h).
//
// A workgroup = 8 waves = 32 queries x a range of 8·T item tiles (S
// workgroups per query group cover the catalog; their lists are merged by
// topk_merge, S = 1 writes the final lists).
//   0. the 32 query vectors formed in LDS (catalog_queries' arithmetic), each
//      wave's MFMA B operands built from them (catalog_main's split pieces);
//   1. every wave scores its T tiles with catalog_main's exact MFMA sequence
//      (same products, same order: the same bits as the selecting and STORE
//      kernels) and KEEPS the T x 16 scores of its lanes in registers;
//   2. threshold: every (lane half, tile) is a group of 16 items of one query,
//      8T groups per query in the workgroup.  The K-th largest group maximum
//      t is a lower bound of the query's K-th best score in the range (K
//      distinct groups hold a score >= t), so every item of the range's
//      top-K scores >= t — while only ~K·(1 + small) items do (K = 20, 64
//      groups: ~24 of 1,024);
//   3. the survivors (score >= t) go to a per-query LDS list (slot from an
//      LDS counter); more than kFusedCap of them (heavy exact ties) raises
//      the threshold to the K-th best (score, index) PAIR among those
//      collected and filters again — each round drops at least kFusedCap - K
//      items, so it ends, and the pair order keeps tf.nn.top_k's ties;
//   4. per query the survivors are sorted by one bitonic network (32 lanes,
//      two queries per wave, or 64-lane chunks merged into the list) and the
//      top K written.
// Exactness: the candidates are a superset of the range's top K under the
// strict (score desc, index asc) order, so the lists equal the dense path's.
#pragma once

namespace hhfm {

// diagnostic knock-outs (timing only, wrong results; default 0): 1 no
// survivor phases (3-4), 2 no threshold phase either, 4 no MFMAs
#ifndef HHFM_FUSED_KO
#define HHFM_FUSED_KO 0
#endif
// diagnostic: s_memtime at the phase boundaries, every wave's phase
// durations summed into g_fused_t (read by hhfm_debug_fused_timing; timing
// only; 1 = on)
#ifndef HHFM_FUSED_TIMING
#define HHFM_FUSED_TIMING 0
#endif
#if HHFM_FUSED_TIMING
// [0..5] phases 0-1 (ids, query rows, LDS), 1-2 (B operands), 2-3 (scores),
// 3-4 (threshold), 4-5 (survivors), 5-6 (sort, write); [6] waves; [7] sum of
// the first mark's spread (wave start - earliest start is not known: raw start)
__device__ unsigned long long g_fused_t[8];
#define HHFM_TMARK(i) tmk[i] = __builtin_amdgcn_s_memtime()
#else
#define HHFM_TMARK(i) (void)0
#endif

constexpr int kFusedCap = 128;   // survivors held per query and workgroup
constexpr int kFusedMaxCtx = 8;   // context (and time) fields the fused kernel takes

// waves per workgroup and tiles per wave: a lane keeps T x 16 scores; 8 waves
// of 4 tiles (two waves per SIMD within 256 registers) rather than 4 of 8 —
// each wave's chain of dependent tile loads is half as long (4 x 8 measured
// 50-60 us per call against ... with 8 x 4: profiles/r05_c3_fused_ab.txt)
constexpr int kFusedWaves = 8, kFusedTiles = 4;

// bitonic sort of scores in aligned groups of N lanes (no indices: only the
// K-th value is wanted)
template <int N>
HHFM_DEV void sort_desc_scores(float& s) {
  const int l = lane_id() & (N - 1);
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
    const bool desc = (l & size) == 0 || size == N;
#pragma unroll
    for (int d = size >> 1; d >= 1; d >>= 1) {
      const float ps = xor_lane(s, d);
      s = (((l & d) == 0) == desc) ? fmaxf(s, ps) : fminf(s, ps);
    }
  }
}

// Q independent score sorts (one per register), interleaved stage by stage
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

// Q independent (score, index) bitonic sorts in aligned groups of N lanes,
// interleaved stage by stage (tf.nn.top_k order, as bitonic_sort_desc)
template <int N, int Q>
HHFM_DEV void bitonic_sort_desc_n(float (&s)[Q], int32_t (&i)[Q]) {
  const int l = lane_id() & (N - 1);
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
    const bool desc = (l & size) == 0 || size == N;
#pragma unroll
    for (int d = size >> 1; d >= 1; d >>= 1) {
      const bool keep_better = ((l & d) == 0) == desc;
      float ps[Q];
      int32_t pi[Q];
#pragma unroll
      for (int u = 0; u < Q; ++u) {
        ps[u] = xor_lane(s[u], d);
        pi[u] = xor_lane(i[u], d);
      }
#pragma unroll
      for (int u = 0; u < Q; ++u) {
        const bool pb = better(ps[u], pi[u], s[u], i[u]);
        const bool take = keep_better ? pb : !pb;
        s[u] = take ? ps[u] : s[u];
        i[u] = take ? pi[u] : i[u];
      }
    }
  }
}

// pass (score, index) at or above the pair threshold (ts, ti): better or equal
HHFM_DEV bool at_least(float s, int32_t i, float ts, int32_t ti) {
  return s > ts || (s == ts && i <= ti);
}

template <bool BF16, int KT, bool FM, bool SPLIT, int T>
__global__ __launch_bounds__(kFusedWaves * 64) void catalog_fused(
    const int32_t* __restrict__ qidx, int64_t B, int ncols, int mode, int ucol, int c0, int c1,
    int t0, int t1, const char* __restrict__ E, int64_t M, int64_t item_row_begin, int32_t N,
    const float* __restrict__ w, int K, int S, float* __restrict__ out_s,
    int32_t* __restrict__ out_i, int64_t ostride_b, int64_t ostride_s, int32_t gbase) {
  constexpr int k = BF16 ? KT * 16 : KT * 8;
  constexpr int64_t ROWB = (int64_t)KT * 32;
  constexpr int EPC = BF16 ? 8 : 4;
  constexpr int NW = kFusedWaves;
  // groups per query: every (wave, lane half, run of T/4 tiles) — 64 groups,
  // 16 (T = 4) or 32 (T = 8) items each
  constexpr int TG = T / 4, NG = 64;
  static_assert(T == 4 || T == 8, "fused catalog kernel: 4 or 8 tiles per wave");
  constexpr int NU = SPLIT ? (BF16 ? KT : KT / 2) : 1;

  __shared__ float hq[kQPerWave][k + 4];
  __shared__ float cq_l[kQPerWave];
  __shared__ float pq[kQPerWave][64];   // FM: per query, catalog_queries' 64 lane values
  __shared__ float gmax[kQPerWave][64];
  __shared__ float thr_s[kQPerWave];
  __shared__ int32_t thr_i[kQPerWave];
  __shared__ int32_t cnt[kQPerWave];
  __shared__ int32_t again;
  // per query kFusedCap (score, index bits) slots + a spare
  __shared__ float2 cbuf[kQPerWave * (kFusedCap + 1)];

  const int g = blockIdx.x / S, split = blockIdx.x - (blockIdx.x / S) * S;
  const int wv = threadIdx.x / kWave;
  const int l = lane_id();
  const int j = l & 31, h = l >> 5;
  const int64_t q0 = (int64_t)g * kQPerWave;
  const int ntiles = (N + kTile - 1) / kTile;
  const int tile0 = (split * NW + wv) * T;

#if HHFM_FUSED_TIMING
  uint64_t tmk[12] = {};
#endif
  HHFM_TMARK(0);
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
  // item operands of the wave's first PD tiles (all T when they fit in 64
  // registers), issued before the query phase so their latency overlaps it
  constexpr int PD = KT <= 4 && T <= 4 ? T : 2;
  uint4 ar[PD][KT];
  float wr[PD];
  auto item_of = [&](int tile) {
    int item = tile * kTile + j;
    return item < N ? item : N - 1;
  };
  auto load_tile = [&](int tile, uint4 (&a)[KT], float& wv_) {
    const char* row = E + (item_row_begin + item_of(tile)) * ROWB + 16 * h;
#pragma unroll
    for (int t = 0; t < KT; ++t) a[t] = *reinterpret_cast<const uint4*>(row + 32 * t);
    if constexpr (FM) wv_ = w ? w[item_row_begin + item_of(tile)] : 0.f;
  };
#pragma unroll
  for (int d = 0; d < PD; ++d) {
    wr[d] = 0.f;
    load_tile(tile0 + d < ntiles ? tile0 + d : ntiles - 1, ar[d], wr[d]);
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
      // every field row of a chunk is loaded before any is summed (loads
      // interleaved with the sums were each followed by a vmcnt(0): one
      // memory latency per field, in series)
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
          // ctx fields, then time fields, in field order: uniform trip counts
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
    __syncthreads();
    if (mode == HHFM_MODE_FM) {
      for (int q2 = wv; q2 < kQPerWave; q2 += NW) {
        float x = l < k ? pq[q2][l] : 0.f;
        x = group_sum<kWave>(x);
        if (l == 0) cq_l[q2] = x;
      }
    }
  }
  if (threadIdx.x < kQPerWave) cnt[threadIdx.x] = 0;
  if (threadIdx.x == 0) again = 0;
  __syncthreads();
  HHFM_TMARK(1);

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
  auto QP = [&](int pc, int u) -> bf16x8 { return qp[pc][u]; };
  const float cq = FM ? cq_l[j] : 0.f;

  HHFM_TMARK(2);
#if HHFM_FUSED_KO & 8   // knock-out: stop after the query phase (tile loads consumed)
  {
    float z = __uint_as_float(ar[0][0].x) + __uint_as_float(QP(0, 0)[0]);
    if (z == 1234.5f) out_s[0] = z;
    return;
  }
#endif
  // ---- 1. scores of this wave's T tiles, kept in registers ----
  float sc[T][16];
#pragma unroll
  for (int tt = 0; tt < T; ++tt) {
    const int tile = tile0 + tt;
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[tt][r] = kNegInf;
    if (tile >= ntiles) continue;   // wave-uniform
    uint4 (&ar_)[KT] = ar[tt % PD];
    // PD < T: this slot is refilled with tile tt + PD chunk by chunk
    const bool refill = PD < T && tt + PD < T;
    const int nxt = tile + PD < ntiles ? tile + PD : ntiles - 1;
    const char* nrow = E + (item_row_begin + item_of(nxt)) * ROWB + 16 * h;
    f32x16 acc = {0};
    const float wcur = wr[tt % PD];
    if constexpr (HHFM_FUSED_KO & 4) {
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        acc[t] += __uint_as_float(ar_[t].x) * (float)QP(0, 0)[t & 7];
        if (refill) ar_[t] = *reinterpret_cast<const uint4*>(nrow + 32 * t);
      }
    } else if constexpr (SPLIT && BF16) {
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const bf16x8 ai = __builtin_bit_cast(bf16x8, ar_[t]);
        if (refill) ar_[t] = *reinterpret_cast<const uint4*>(nrow + 32 * t);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ai, QP(2, t), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ai, QP(1, t), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ai, QP(0, t), acc, 0, 0, 0);
      }
    } else if constexpr (SPLIT) {
#pragma unroll
      for (int u = 0; u < KT / 2; ++u) {
        const float x[8] = {__uint_as_float(ar_[2 * u].x), __uint_as_float(ar_[2 * u].y),
                            __uint_as_float(ar_[2 * u].z), __uint_as_float(ar_[2 * u].w),
                            __uint_as_float(ar_[2 * u + 1].x), __uint_as_float(ar_[2 * u + 1].y),
                            __uint_as_float(ar_[2 * u + 1].z), __uint_as_float(ar_[2 * u + 1].w)};
        if (refill) ar_[2 * u] = *reinterpret_cast<const uint4*>(nrow + 32 * (2 * u));
        if (refill) ar_[2 * u + 1] = *reinterpret_cast<const uint4*>(nrow + 32 * (2 * u + 1));
        bf16x8 i0, i1, i2;
        split3x8(x, i0, i1, i2);
        const bf16x8 q0 = QP(0, u), q1 = QP(1, u), q2 = QP(2, u);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i2, q0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i1, q1, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i0, q2, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i1, q0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i0, q1, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i0, q0, acc, 0, 0, 0);
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
        if (refill) ar_[t] = *reinterpret_cast<const uint4*>(nrow + 32 * t);
#pragma unroll
        for (int e = 0; e < EPC; ++e)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bq[t][e], acc, 0, 0, 0);
      }
    }
    if constexpr (FM) {   // D[i][j] += w_i·1 + 1·(q_j·f_j)   (catalog_main)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h == 0 ? wcur : 1.f, h == 0 ? 1.f : cq, acc,
                                                 0, 0, 0);
      if (refill) wr[tt % PD] = w ? w[item_row_begin + item_of(nxt)] : 0.f;
    }
    const int ibase = tile * kTile;
    if (ibase + kTile <= N) {   // wave-uniform: only the catalog's last tile is partial
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
    // (the unrolled loop otherwise holds every tile's A operand at once)
    asm volatile("" ::: "memory");
  }

#if HHFM_FUSED_KO & 2
  {
    float z = 0.f;
#pragma unroll
    for (int tt = 0; tt < T; ++tt)
#pragma unroll
      for (int r = 0; r < 16; ++r) z += sc[tt][r];
    if (z == 1234.5f) out_s[0] = z;
    return;
  }
#endif
  HHFM_TMARK(3);
  // ---- 2. threshold from the group maxima ----
  float tmax[T];   // this lane's group maxima (also: tiles with nothing to pass)
#pragma unroll
  for (int tt = 0; tt < T; ++tt) {
    float m = sc[tt][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) m = fmaxf(m, sc[tt][r]);
    tmax[tt] = m;
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float m = tmax[g * TG];
#pragma unroll
    for (int u = 1; u < TG; ++u) m = fmaxf(m, tmax[g * TG + u]);
    gmax[j][(wv * 4 + g) * 2 + h] = m;
  }
  __syncthreads();
  {   // this wave's kQPerWave / NW queries side by side (independent networks)
    constexpr int QW = kQPerWave / NW;
    float m[QW];
#pragma unroll
    for (int u = 0; u < QW; ++u) m[u] = l < NG ? gmax[wv + NW * u][l] : kNegInf;
    sort_desc_scores_n<64, QW>(m);
#pragma unroll
    for (int u = 0; u < QW; ++u) {
      const float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m[u]), K - 1));
      if (l == 0) {
        thr_s[wv + NW * u] = t;
        thr_i[wv + NW * u] = kNoIdx;   // every item scoring t passes
      }
    }
  }
  __syncthreads();

#if HHFM_FUSED_KO & 1
  {
    float z = thr_s[j];
#pragma unroll
    for (int tt = 0; tt < T; ++tt)
#pragma unroll
      for (int r = 0; r < 16; ++r) z += sc[tt][r];
    if (z == 1234.5f) out_s[0] = z;
    return;
  }
#endif
  HHFM_TMARK(4);
  // ---- 3. survivors to the per-query lists (re-filtered on overflow) ----
  for (;;) {
    // queries past B (a zero vector: every HHFM score ties at 0) add nothing
    const float ts = q0 + j < B ? thr_s[j] : __builtin_huge_valf();
    const int32_t ti = q0 + j < B ? thr_i[j] : -1;
    // item index of (tile tt, row r) = ib + 32 tt + row(r); laundered so the
    // compiler does not hoist 16 T indices out of the loop into registers
    int32_t ib = tile0 * kTile + 4 * h;
    asm volatile("" : "+v"(ib));
    uint32_t pm[T];   // pass bits of the lane's 16 rows per tile
    int n = 0;
    // the first round (t finite, ti = kNoIdx on every lane) is `score >= t`
    // (items past N hold -inf); a raised pair threshold takes the full test
    if (__ballot(ti != kNoIdx || !(ts > kNegInf)) == 0) {
#pragma unroll
      for (int tt = 0; tt < T; ++tt) {
        uint32_t m = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) m |= sc[tt][r] >= ts ? 1u << r : 0u;
        pm[tt] = m;
      }
    } else {
#pragma unroll
      for (int tt = 0; tt < T; ++tt) {
        uint32_t m = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int32_t it = ib + tt * kTile + (r & 3) + 8 * (r >> 2);
          const float x = sc[tt][r];
          const bool pass = (it < N) & ((x > ts) | ((x == ts) & (it <= ti)));
          m |= pass ? 1u << r : 0u;
        }
        pm[tt] = m;
      }
    }
#pragma unroll
    for (int tt = 0; tt < T; ++tt) n += __popc(pm[tt]);
    HHFM_TMARK(7);
    int pos = n ? atomicAdd(&cnt[j], n) : 0;
    HHFM_TMARK(8);
    asm volatile("" : "+v"(ib));   // recompute the indices below (no 16 T live values)
    // (score, index) as one 8-B slot; slots past the list's end go to the
    // query's spare slot kFusedCap
    constexpr int kQS = kFusedCap + 1;   // slots per query (the last: spare)
    const int qbase = j * kQS;
#pragma unroll
    for (int tt = 0; tt < T; ++tt) {
      const uint32_t m = pm[tt];
      if (__ballot(m != 0) != 0) {
        // only the passing rows write (exec-masked stores; branch-free
        // writes of every row to a dummy slot measured 2 % slower)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool pb = (m >> r) & 1u;
          if (pb)
            cbuf[qbase + min(pos, kFusedCap)] =
                make_float2(sc[tt][r], __int_as_float(ib + tt * kTile + (r & 3) + 8 * (r >> 2)));
          pos += pb ? 1 : 0;
        }
      }
      // one tile's slots at a time (the compiler otherwise forms all 16 T
      // slot addresses up front)
      asm volatile("" : "+v"(pos) : : "memory");
    }
    HHFM_TMARK(9);
    // a lane whose last slot lies past the cap flags the overflow: the
    // common case (no list overflowed) then costs one barrier
    if (pos > kFusedCap) again = 1;
    __syncthreads();
    HHFM_TMARK(10);
    if (!again) break;
    // overflowed queries: the K-th best pair among the kFusedCap collected
    // becomes the threshold (at least K items reach it), and the range is
    // filtered again from an empty list
    for (int qq = wv; qq < kQPerWave; qq += NW) {
      if (cnt[qq] <= kFusedCap) continue;   // wave-uniform
      const float2 e0 = cbuf[qq * (kFusedCap + 1) + l], e1 = cbuf[qq * (kFusedCap + 1) + l + 64];
      float s0 = e0.x, s1 = e1.x;
      int32_t i0 = __float_as_int(e0.y), i1 = __float_as_int(e1.y);
      bitonic_sort_desc<64>(s0, i0);
      bitonic_sort_desc<64>(s1, i1);
      merge_lists<64>(s0, i0, s1, i1);   // the best 64 of the 128, sorted
      const float ns = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s0), K - 1));
      const int32_t ni = __builtin_amdgcn_readlane(i0, K - 1);
      if (l == 0) {
        thr_s[qq] = ns;
        thr_i[qq] = ni;
        cnt[qq] = -1;   // marks: filter this query again
      }
    }
    __syncthreads();
    // queries not overflowed keep their lists: their lanes add nothing
    const bool redo = cnt[j] < 0;
    __syncthreads();
    if (threadIdx.x == 0) again = 0;
    if (threadIdx.x < kQPerWave && cnt[threadIdx.x] < 0) cnt[threadIdx.x] = 0;
    if (!redo) {
      thr_s[j] = __builtin_huge_valf();   // (written by both lanes of j: same value)
      thr_i[j] = -1;
    }
    __syncthreads();
  }

  HHFM_TMARK(5);
  // ---- 4. sort the survivors, write the top K ----
  const int64_t ob = split * ostride_s;
  {
    // this wave's query pairs p = wv + NW u: each query in a 32-lane half;
    // when every pair's lists fit 32 lanes (the common case: ~24 survivors)
    // the pairs' networks run side by side
    constexpr int PW = kQPerWave / 2 / NW;
    bool small = true;
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const int pp = wv + NW * u;
      small = small && cnt[2 * pp] <= 32 && cnt[2 * pp + 1] <= 32;
    }
    if (small) {
      float sv[PW];
      int32_t iv[PW];
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int qq = 2 * (wv + NW * u) + h, nq = cnt[qq];
        const float2 e = cbuf[qq * (kFusedCap + 1) + (j < nq ? j : 0)];
        sv[u] = j < nq ? e.x : kNegInf;
        iv[u] = j < nq ? __float_as_int(e.y) : kNoIdx;
      }
      bitonic_sort_desc_n<32, PW>(sv, iv);
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int qq = 2 * (wv + NW * u) + h;
        const int64_t b = q0 + qq;
        if (b < B && j < K) {
          out_s[b * ostride_b + ob + j] = sv[u];
          out_i[b * ostride_b + ob + j] = iv[u] == kNoIdx ? kNoIdx : iv[u] + gbase;
        }
      }
    } else {
#pragma unroll 1
      for (int qi = 0; qi < 2 * PW; ++qi) {
        const int qq = 2 * (wv + NW * (qi >> 1)) + (qi & 1), nq = cnt[qq];
        // per pair: a pair whose lists both fit 32 lanes takes the 32-lane
        // network (its second query is done with the first); a list of at
        // most 64 one 64-lane sort
        const int qo = qq ^ 1, no = cnt[qo];
        if (nq <= 32 && no <= 32) {
          if (qi & 1) continue;   // done with its pair
          const int qh = qq + h, nh = h ? no : nq;
          const float2 e = cbuf[qh * (kFusedCap + 1) + (j < nh ? j : 0)];
          float sv[1] = {j < nh ? e.x : kNegInf};
          int32_t iv[1] = {j < nh ? __float_as_int(e.y) : kNoIdx};
          bitonic_sort_desc_n<32, 1>(sv, iv);
          const int64_t b = q0 + qh;
          if (b < B && j < K) {
            out_s[b * ostride_b + ob + j] = sv[0];
            out_i[b * ostride_b + ob + j] = iv[0] == kNoIdx ? kNoIdx : iv[0] + gbase;
          }
          continue;
        }
        if (nq <= 64) {
          const float2 e = cbuf[qq * (kFusedCap + 1) + (l < nq ? l : 0)];
          float s1 = l < nq ? e.x : kNegInf;
          int32_t i1 = l < nq ? __float_as_int(e.y) : kNoIdx;
          bitonic_sort_desc<64>(s1, i1);
          const int64_t b = q0 + qq;
          if (b < B && l < K) {
            out_s[b * ostride_b + ob + l] = s1;
            out_i[b * ostride_b + ob + l] = i1 == kNoIdx ? kNoIdx : i1 + gbase;
          }
          continue;
        }
        float ls = kNegInf;
        int32_t li = kNoIdx;
#pragma unroll 1
        for (int c = 0; c < nq; c += 64) {
          const float2 e = cbuf[qq * (kFusedCap + 1) + (c + l < nq ? c + l : 0)];
          float s = c + l < nq ? e.x : kNegInf;
          int32_t i = c + l < nq ? __float_as_int(e.y) : kNoIdx;
          bitonic_sort_desc<64>(s, i);
          merge_lists<32>(ls, li, s, i);
          if (l >= 32) {
            ls = kNegInf;
            li = kNoIdx;
          }
        }
        const int64_t b = q0 + qq;
        if (b < B && l < K) {
          out_s[b * ostride_b + ob + l] = ls;
          out_i[b * ostride_b + ob + l] = li == kNoIdx ? kNoIdx : li + gbase;
        }
      }
    }
  }
#if HHFM_FUSED_TIMING
  HHFM_TMARK(6);
  if (l == 0) {
    atomicAdd(&g_fused_t[0], tmk[1] - tmk[0]);
    atomicAdd(&g_fused_t[1], tmk[2] - tmk[1]);
    atomicAdd(&g_fused_t[2], tmk[3] - tmk[2]);
    atomicAdd(&g_fused_t[3], tmk[4] - tmk[3]);
    atomicAdd(&g_fused_t[4], tmk[5] - tmk[4]);
    atomicAdd(&g_fused_t[5], tmk[6] - tmk[5]);
    atomicAdd(&g_fused_t[6], 1ull);
  }
#endif
}

}  // namespace hhfm
