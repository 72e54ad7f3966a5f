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
// diagnostic knock-outs of the in-kernel merge (wrong results; timing only):
// 1 the last arriver merges zero keys instead of loading the S lists, 2 it
// does not merge at all, 4 it merges but writes no output
#ifndef HHFM_FUSED_KO
#define HHFM_FUSED_KO 0
#endif
#if HHFM_FUSED_KO && !defined(HHFM_DIAG_BUILD)
#error "HHFM_FUSED_KO: diagnostic builds only (-DHHFM_DIAG_BUILD)"
#endif
#if HHFM_FUSED_TIMING
// per workgroup, wave 0's s_memtime at kFusedMarks points (plain stores: no
// atomics that would queue beside the hand-off); host side: differences
constexpr int kFusedTimingWG = 16384, kFusedMarks = 24;
__device__ unsigned long long g_fused_t[kFusedTimingWG][kFusedMarks];
#define HHFM_MARK(i) tmk[i] = __builtin_amdgcn_s_memtime()
#else
#define HHFM_MARK(i) (void)0
#endif

constexpr int kFusedCap = 128;    // list entries held per query
// arrival counters (one per 32 queries) at the workspace's start
constexpr int kFusedMaxGroups = HHFM_CATALOG_WS_ZERO / 4;
constexpr int kFusedMaxS = 16;    // item ranges (workgroups) per 32 queries (merge: 4 unrolled)
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

// ---- rolled networks -------------------------------------------------------
// The kernel runs once per workgroup on a CU whose instruction cache the
// dispatch has just emptied: every executed line is fetched from L2 (~290
// fetches per workgroup, ~100 cycles per 64-B line measured), so an unrolled
// network costs more in instruction fetch than in execution.  These loops
// fetch one body; the partner exchange picks its DPP / swizzle / permlane
// form behind a wave-uniform branch on d.
HHFM_DEV void xor_lane2_rt(int32_t& a, int32_t& b, int d) {
  if (d == 1) { a = xor_lane(a, 1); b = xor_lane(b, 1); }
  else if (d == 2) { a = xor_lane(a, 2); b = xor_lane(b, 2); }
  else if (d == 4) { a = xor_lane(a, 4); b = xor_lane(b, 4); }
  else if (d == 8) { a = xor_lane(a, 8); b = xor_lane(b, 8); }
  else if (d == 16) { a = xor_lane(a, 16); b = xor_lane(b, 16); }
  else { a = xor_lane(a, 32); b = xor_lane(b, 32); }
}
HHFM_DEV uint64_t xor_lane64_rt(uint64_t v, int d) {
  int32_t lo = (int32_t)(uint32_t)v, hi = (int32_t)(uint32_t)(v >> 32);
  xor_lane2_rt(lo, hi, d);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
// bitonic sort of keys, descending, in aligned groups of N lanes (rolled)
template <int N>
HHFM_DEV void sort_keys_rt(uint64_t& k) {
  const int l = lane_id() & (N - 1);
#pragma unroll 1
  for (int size = 2; size <= N; size <<= 1) {
    const bool desc = (l & size) == 0 || size == N;
#pragma unroll 1
    for (int d = size >> 1; d >= 1; d >>= 1) {
      const uint64_t p = xor_lane64_rt(k, d);
      const bool keep_max = ((l & d) == 0) == desc;
      k = ((p > k) == keep_max) ? p : k;
    }
  }
}
// the best N of the union of two descending key lists (rolled merge_keys)
template <int N>
HHFM_DEV void merge_keys_rt(uint64_t& a, uint64_t b) {
  const int l = lane_id();
  const int src = (l & ~(N - 1)) | (N - 1 - (l & (N - 1)));
  const uint32_t blo = (uint32_t)__shfl((int32_t)(uint32_t)b, src, kWave);
  const uint32_t bhi = (uint32_t)__shfl((int32_t)(uint32_t)(b >> 32), src, kWave);
  const uint64_t r = ((uint64_t)bhi << 32) | blo;
  a = r > a ? r : a;
  const int lg = l & (N - 1);
#pragma unroll 1
  for (int d = N >> 1; d >= 1; d >>= 1) {
    const uint64_t p = xor_lane64_rt(a, d);
    a = ((p > a) == ((lg & d) == 0)) ? p : a;
  }
}
// two independent score sorts (descending, aligned groups of 32), rolled
HHFM_DEV void sort_scores2_rt(float& s0, float& s1) {
  const int l = lane_id() & 31;
#pragma unroll 1
  for (int size = 2; size <= 32; size <<= 1) {
    const bool desc = (l & size) == 0 || size == 32;
#pragma unroll 1
    for (int d = size >> 1; d >= 1; d >>= 1) {
      int32_t a = __float_as_int(s0), b = __float_as_int(s1);
      xor_lane2_rt(a, b, d);
      const bool keep_max = ((l & d) == 0) == desc;
      const float p0 = __int_as_float(a), p1 = __int_as_float(b);
      s0 = keep_max ? fmaxf(s0, p0) : fminf(s0, p0);
      s1 = keep_max ? fmaxf(s1, p1) : fminf(s1, p1);
    }
  }
}

// network form (A/B knobs, default: unrolled DPP networks; rolled loops
// measured slower — every stage's uniform branch chain and DPP hazard waits
// cost more than the instruction fetch they save)
#ifndef HHFM_FUSED_ROLLED
#define HHFM_FUSED_ROLLED 0
#endif
template <int N>
HHFM_DEV void sort_keys(uint64_t& k) {
  if constexpr (HHFM_FUSED_ROLLED) sort_keys_rt<N>(k);
  else sort_keys_desc<N>(k);
}
template <int N>
HHFM_DEV void merge_keys_sel(uint64_t& a, uint64_t b) {
  if constexpr (HHFM_FUSED_ROLLED) merge_keys_rt<N>(a, b);
  else merge_keys<N>(a, b);
}
HHFM_DEV void sort_scores2(float& s0, float& s1) {
  if constexpr (HHFM_FUSED_ROLLED) {
    sort_scores2_rt(s0, s1);
  } else {
    float m[2] = {s0, s1};
    sort_desc_scores_n<32, 2>(m);
    s0 = m[0];
    s1 = m[1];
  }
}

// QL: the split query pieces in LDS (116 instead of 140 registers at C3: two
// workgroups per CU, for grids past one workgroup per CU: 3,000 queries 33.0
// -> 28.2 us) or in registers (one workgroup per CU: 300 queries 17.3 us
// against 19.5 with QL)
template <bool BF16, int KT, bool FM, bool SPLIT, int T, bool QL>
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
  __shared__ bf16x8 qps[SPLIT && QL ? 3 : 1][SPLIT && QL ? NU : 1][kWave];
  __shared__ int32_t qid[kQPerWave][1 + 2 * kFusedMaxCtx];   // the queries' field ids
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
  uint64_t tmk[kFusedMarks] = {};
#endif
  HHFM_MARK(0);
  // the query rows' raw ids first (8 threads per query; only the first 256
  // threads form queries): thread tp of a query loads its fields tp, tp + 8,
  // tp + 16 (field 0 the user, then the context and the time columns).  These
  // are the oldest loads, so waiting for them leaves the tile loads below in
  // flight (vmcnt counts in order)
  const int pq_q = threadIdx.x >> 3, pq_t = threadIdx.x & 7;
  const int64_t pq_b = q0 + pq_q;
  const bool pq_on = threadIdx.x < 8 * kQPerWave && pq_b < B;
  const int nc = c1 - c0, nt = t1 - t0, nf = 1 + nc + nt;
  int32_t rid[3];
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    const int f = pq_t + 8 * x;
    const int col = f == 0 ? ucol : (f <= nc ? c0 + f - 1 : t0 + f - 1 - nc);
    rid[x] = (pq_on && f < nf) ? qidx[pq_b * ncols + col] : 0;
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
  // the first PD tiles: at once in the waves that form no query (4..7);
  // behind the query row loads in the others (0..3), whose wait for those
  // rows would otherwise drain 8 KB of tile loads per wave first (vmcnt
  // counts in order: 5.3K -> ~2K cycles measured for the row phase)
  auto issue_tiles = [&]() {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      wr[d] = 0.f;
      load_tile(tile_of(d), ar[d], wr[d]);
    }
  };
  const bool qwave = wv * kWave < 8 * kQPerWave;   // this wave forms queries
  if (!qwave) issue_tiles();

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
    const int qq = pq_q, tp = pq_t;
    const int64_t b = q0 + qq;
    if (threadIdx.x < 8 * kQPerWave) {
      // the query's (clamped) field ids through LDS: the 8 threads of a query
      // are lanes of one wave, and a wave's LDS accesses complete in order
#pragma unroll
      for (int x = 0; x < 3; ++x)
        if (tp + 8 * x < nf) qid[qq][tp + 8 * x] = clamp_id(rid[x], M);
      HHFM_MARK(1);   // the ids arrived
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
#pragma unroll
      for (int cc = 0; cc < CPT; ++cc) {
        const int ch = tp + 8 * cc;
        if (ch < CPR) {
          auto ld = [&](int f) {
            return *reinterpret_cast<const uint4*>(E + (int64_t)qid[qq][f] * ROWB + 16 * ch);
          };
          // the user row, then the context and the time fields in field order,
          // four rows in flight per step (rolled: one body fetched)
          float uu[EPC], cx[EPC], tm[EPC], r[EPC];
          const uint4 ru = ld(0);
#pragma unroll
          for (int v = 0; v < EPC; ++v) cx[v] = tm[v] = 0.f;
#pragma unroll 1
          for (int f0 = 1; f0 < nf; f0 += 4) {
            uint4 rr[4];
#pragma unroll
            for (int x = 0; x < 4; ++x) rr[x] = ld(f0 + x < nf ? f0 + x : 0);
#pragma unroll
            for (int x = 0; x < 4; ++x) {
              const int f = f0 + x;   // wave-uniform
              if (f >= nf) break;
              cvt(rr[x], r);
              if (f <= nc) {
#pragma unroll
                for (int v = 0; v < EPC; ++v) cx[v] += r[v];
              } else {
#pragma unroll
                for (int v = 0; v < EPC; ++v) tm[v] += r[v];
              }
            }
          }
          cvt(ru, uu);
#pragma unroll
          for (int v = 0; v < EPC; ++v) {
            float hv = 0.f;
            if (b < B) {
              if constexpr (FM) {
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
      if constexpr (FM) {
#pragma unroll
        for (int c = 0; c < LPT; ++c) {
          const int ch = tp + 8 * c;
          if (ch < CPR && EPC * ch < 64)
#pragma unroll
            for (int v = 0; v < EPC; ++v) pq[qq][EPC * ch + v] = part[c][v];
        }
      }
    }
    HHFM_MARK(2);   // rows loaded, hq written
    if (qwave) issue_tiles();
    if (threadIdx.x < kQPerWave) {
      cnt[threadIdx.x] = 0;
      // the lowest finite score: items past N (held as -inf) never pass
      thr_k[threadIdx.x] = (uint64_t)ukey(-__FLT_MAX__) << 32;
    }
    if (threadIdx.x < 2) ovf[threadIdx.x] = 0;
    lds_barrier();
    HHFM_MARK(3);
    if constexpr (FM) {
      for (int q2 = wv; q2 < kQPerWave; q2 += NW) {
        float x = l < k ? pq[q2][l] : 0.f;
        x = group_sum<kWave>(x);
        if (l == 0) cq_l[q2] = x;
      }
      lds_barrier();
    }
  }

  // B operand (catalog_main): this lane's query j, k slices {EPC(2t+h) ..}.
  // Split-bf16: the three pieces are the same for every wave, so wave u
  // splits k slice u once for the workgroup into LDS and every wave reads
  // them per tile (48 fewer registers per lane: two workgroups fit a CU)
  float bq[KT][EPC];
  bf16x8 qp[3][QL ? 1 : NU];
  if constexpr (!SPLIT) {
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int e = 0; e < EPC; ++e) bq[t][e] = hq[j][(2 * t + h) * EPC + e];
  } else if constexpr (!QL) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int t = BF16 ? u : 2 * u + (e >> 2), ee = BF16 ? e : (e & 3);
        x[e] = hq[j][(2 * t + h) * EPC + ee];
      }
      split3x8(x, qp[0][u], qp[1][u], qp[2][u]);
    }
  } else {
#pragma unroll 1
    for (int u = wv; u < NU; u += NW) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int t = BF16 ? u : 2 * u + (e >> 2), ee = BF16 ? e : (e & 3);
        x[e] = hq[j][(2 * t + h) * EPC + ee];
      }
      bf16x8 a0, a1, a2;
      split3x8(x, a0, a1, a2);
      qps[0][u][l] = a0;
      qps[1][u][l] = a1;
      qps[2][u][l] = a2;
    }
    lds_barrier();
  }
  const float cq = FM ? cq_l[j] : 0.f;
  HHFM_MARK(4);   // B operands ready

  {
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
      // this tile's view of the piece array (laundered: the reads stay per
      // tile instead of being hoisted into 48 live registers)
      const bf16x8* qv = &qps[0][0][l];
      if constexpr (QL) asm volatile("" : "+v"(qv));
      auto QP = [&](int pc, int u) {
        if constexpr (QL) return qv[(pc * NU + u) * kWave];
        else return qp[pc][u];
      };
      if constexpr (SPLIT && BF16) {
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const bf16x8 ai = __builtin_bit_cast(bf16x8, ar_[t]);
          ar_[t] = *reinterpret_cast<const uint4*>(nrow + 32 * t);
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
          ar_[2 * u] = *reinterpret_cast<const uint4*>(nrow + 32 * (2 * u));
          ar_[2 * u + 1] = *reinterpret_cast<const uint4*>(nrow + 32 * (2 * u + 1));
          bf16x8 i0, i1, i2;
          split3x8(x, i0, i1, i2);
          const bf16x8 p0 = QP(0, u), p1 = QP(1, u), p2 = QP(2, u);
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
    HHFM_MARK(5);   // scores in registers

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
    HHFM_MARK(6);
    lds_barrier();
    HHFM_MARK(7);
    {   // wave wv: queries QW wv + 2u + h, one per 32-lane half
      constexpr int QW = kQPerWave / NW, U = QW / 2;
      float m[U];
#pragma unroll
      for (int u = 0; u < U; ++u) m[u] = gmx[wv * QW + 2 * u + h][j];
      static_assert(U == 2, "two queries per lane half");
      sort_scores2(m[0], m[1]);
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
    HHFM_MARK(8);
    lds_barrier();
    HHFM_MARK(9);   // threshold set

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
        // per row its bit (v_cmp + v_cndmask with the bit as a literal), then
        // a 3-input OR tree: depth 4 instead of a 16-long dependent chain
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
          uint32_t bb[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) bb[r] = sc[tt][r] >= ts ? (1u << r) : 0u;
          const uint32_t o0 = bb[0] | bb[1] | bb[2], o1 = bb[3] | bb[4] | bb[5];
          const uint32_t o2 = bb[6] | bb[7] | bb[8], o3 = bb[9] | bb[10] | bb[11];
          const uint32_t o4 = bb[12] | bb[13] | bb[14];
          pm[tt] = (o0 | o1 | o2) | (o3 | o4 | bb[15]);
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
      if (first) HHFM_MARK(10);
      int pos = atomicAdd(&cnt[j], n);
      if (first) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        HHFM_MARK(11);
      }
      asm volatile("" : "+v"(ib));   // recompute the indices below (no 16 T live values)
      // per step one survivor of every tile per lane (lowest row first; the
      // four extractions independent of each other); a lane without one
      // writes the query's spare slot (no exec-mask branches)
      uint32_t mt[T];
#pragma unroll
      for (int tt = 0; tt < T; ++tt) mt[tt] = pm[tt];
      uint32_t any = 0;
#pragma unroll
      for (int tt = 0; tt < T; ++tt) any |= mt[tt];
#pragma unroll 1
      while (__ballot(any != 0) != 0) {
        any = 0;
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
          const uint32_t m = mt[tt];
          const int r = __builtin_ctz(m | 0x10000u) & 15;
          const float x = select16(sc[tt], r);
          const int32_t it = ib + tt * kTile + (r & 3) + 8 * (r >> 2);
          const int slot = m ? (pos < kFusedCap ? pos : kFusedCap) : kFusedCap;
          cbuf[qbase + slot] = ekey(x, it);
          pos += m ? 1 : 0;
          mt[tt] = m & (m - 1);
          any |= mt[tt];
        }
      }
      // a lane whose last slot lies past the cap flags the overflow in this
      // round's flag word (two words alternate, so the reset of the next
      // round's word never races with this round's writers)
      if (pos > kFusedCap) ovf[rnd & 1] = 1;
      if (first) HHFM_MARK(12);
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
        sort_keys<64>(k0);
        sort_keys<64>(k1);
        merge_keys_sel<64>(k0, k1);   // the best 64 of the 128, sorted
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
    HHFM_MARK(13);   // survivors listed
  }

  // ---- 4. per query: the range's entries at or above the final threshold,
  // sorted (its exact top K) ----
  // Two queries per pass, one per 32-lane half: a half's lanes load its
  // query's entries 32 at a time, the passing ones are compacted into the
  // wave's LDS scratch and one 32-lane key network sorts them (typically
  // ~K·1.2 pass).  A query with more than 32 passing takes the 64-lane
  // network (+ merges past 64), one query at a time.
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
      if (u == 0) HHFM_MARK(14);
      if (__ballot(nv > 32) == 0) {
        uint64_t key = j < nv ? fscr[wv][(h << 5) + j] : 0ull;
        sort_keys<32>(key);
        if (u == 0) HHFM_MARK(15);
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
            sort_keys<64>(key);
            if (c == 0) top = key;
            else merge_keys_sel<32>(top, key);
            if (l >= 32) top = 0;
          }
          if (l < 32) emit(q2, l, top);
        }
      }
    }
  }
  HHFM_MARK(16);   // range lists emitted

  // ---- 5. S > 1: hand-off, the last arriving workgroup merges ----
  bool merged = false;
  if (S > 1) {
    // every storing wave drains its sc1 stores, then the barrier, then ONE
    // lane's agent-scope add for the whole workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    HHFM_MARK(17);
    lds_barrier();
    HHFM_MARK(18);
    if (threadIdx.x == 0) {
      const uint32_t old = __hip_atomic_fetch_add((gu32*)(arrive + g), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      last_sh = old == (uint32_t)(S - 1);
    }
    HHFM_MARK(19);
    lds_barrier();
    HHFM_MARK(20);
    merged = last_sh != 0 && !(HHFM_FUSED_KO & 2);   // uniform
    if (merged) {
      // no instruction: keeps the sc1 loads below the barrier
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      constexpr int QW = kQPerWave / NW;
      // lane (h, j) holds rank j of the lists h, h + 2, ... of the wave's QW
      // queries; up to 4 lists per query every load is issued before any
      // merge (one memory latency; merged from registers — a rolled merge
      // staged through LDS measured 60 % slower), more take a rolled loop
      // (src: lane j's rank of list sl of the wave's query u)
      auto src = [&](int u, int sl) {
        return (const gu64*)(part + ((((int64_t)g * S + (sl < S ? sl : 0)) * kQPerWave +
                                      wv * QW + u) << 5) + j);
      };
      auto store = [&](int u, uint64_t a) {
        const int64_t b = q0 + wv * QW + u;
        if (b < B && l < K && !((HHFM_FUSED_KO & 4) && a != 1ull)) {
          out_s[b * K + l] = ukey_inv((uint32_t)(a >> 32));
          const int32_t it = ~(int32_t)(uint32_t)a;
          out_i[b * K + l] = it == kNoIdx ? kNoIdx : it + gbase;
        }
      };
      if (S <= 4) {
        // half h merges lists h and h + 2: the second loaded reversed (lane
        // j takes rank 31 - j), so max(first, second) is bitonic without a
        // lane permutation; half 0 sorts it descending, half 1 ascending, so
        // the final max(half 0, half 1 swapped) is bitonic too.  The QW
        // queries' networks run stage by stage (their chains interleave).
        uint64_t a[QW];
#pragma unroll
        for (int u = 0; u < QW; ++u) {
          uint64_t v[2];
#pragma unroll
          for (int x = 0; x < 2; ++x) {
            const int sl = 2 * x + h;
            const gu64* q = src(u, sl) + (x == 1 ? 31 - 2 * j : 0);
            v[x] = (HHFM_FUSED_KO & 1) ? 0ull
                   : __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[x] = sl < S ? v[x] : 0ull;
          }
          a[u] = v[1] > v[0] ? v[1] : v[0];
        }
        const bool asc = h != 0;
#pragma unroll
        for (int d = 16; d >= 1; d >>= 1) {
          const bool keep_max = ((j & d) == 0) != asc;
          uint64_t p[QW];
#pragma unroll
          for (int u = 0; u < QW; ++u) p[u] = xor_lane64(a[u], d);
#pragma unroll
          for (int u = 0; u < QW; ++u) a[u] = ((p[u] > a[u]) == keep_max) ? p[u] : a[u];
        }
        // half 0: max with half 1's ascending list, then a descending cleanup
        {
          uint64_t p[QW];
#pragma unroll
          for (int u = 0; u < QW; ++u) p[u] = xor_lane64(a[u], 32);
#pragma unroll
          for (int u = 0; u < QW; ++u) a[u] = p[u] > a[u] ? p[u] : a[u];
        }
#pragma unroll
        for (int d = 16; d >= 1; d >>= 1) {
          const bool keep_max = (j & d) == 0;
          uint64_t p[QW];
#pragma unroll
          for (int u = 0; u < QW; ++u) p[u] = xor_lane64(a[u], d);
#pragma unroll
          for (int u = 0; u < QW; ++u) a[u] = ((p[u] > a[u]) == keep_max) ? p[u] : a[u];
        }
#pragma unroll
        for (int u = 0; u < QW; ++u) store(u, a[u]);
      } else {
#pragma unroll 1
        for (int u = 0; u < QW; ++u) {
          uint64_t a = 0;
#pragma unroll 1
          for (int x = 0; 2 * x < S; ++x) {
            const int sl = 2 * x + h;
            const uint64_t t =
                __hip_atomic_load(src(u, sl), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            merge_keys_sel<32>(a, sl < S ? t : 0ull);
          }
          merge_keys<32>(a, xor_lane64(a, 32));   // the odd lists' half into the even's
          store(u, a);
        }
      }
      // re-arm the counter for the next call (stream order publishes it)
      if (threadIdx.x == 0)
        __hip_atomic_store((gu32*)(arrive + g), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  HHFM_MARK(21);
#if HHFM_FUSED_TIMING
  if (threadIdx.x == 0 && blockIdx.x < kFusedTimingWG) {
    tmk[22] = merged ? 1ull : 0ull;
    tmk[23] = 1ull;
#pragma unroll
    for (int p = 0; p < kFusedMarks; ++p) g_fused_t[blockIdx.x][p] = tmk[p];
  }
#endif
  (void)merged;
}

}  // namespace hhfm
