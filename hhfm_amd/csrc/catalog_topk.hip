// K2 — full-catalog scoring + fused top-K on gfx950.
//
//   hhfm_catalog_topk replaces FM.topk       (Newcode/FM.py:172-198)
//                     and      OUR.topk      (Newcode/OurModel7.py:229-307)
// Both reference graphs broadcast-multiply [B,1,k] x [1,N,k], reduce over k
// and call tf.nn.top_k(score, 20).  Here the [B,N] score matrix never exists:
//
//  1. catalog_queries: one fp32 query vector per row (HHFM h = u+Σctx[+Σtime];
//     FM q = u+f with f = Σctx and the item-independent term q·f).
//  2. catalog_main: a workgroup = 4 waves = 128 queries x one item split.
//     Each wave owns 32 queries; their fp32 vectors stay in VGPRs as the
//     MFMA B operand for the whole split.  Item tiles of 32 rows stream
//     through the A operand (one 16-B load per lane per 8 (fp32) / 16 (bf16)
//     k, next tile prefetched while this one is multiplied) and
//     v_mfma_f32_32x32x2_f32 — exact fp32 (each MFMA is a k-ordered fmaf
//     chain), same 157 TF peak as the fp32 VALU — yields a 32x32 score tile.
//     For FM one extra MFMA adds w_item + q·f.  The VALU then filters the
//     tile against each query's current K-th score; survivors enter a
//     per-query sorted list in LDS (single insertions when sparse, a
//     bitonic sort + merge when dense — the first tiles of a split).
//  3. topk_merge: per query, merge the S split lists (and, multi-GPU, the R
//     rank lists gathered over RCCL) into the final top-K.
// Order everywhere: score descending, item index ascending (tf.nn.top_k).
#include "gemm_mfma.h"

#include <algorithm>

namespace hhfm {

typedef float f32x16 __attribute__((ext_vector_type(16)));

#ifndef HHFM_MAIN_KO
#define HHFM_MAIN_KO 0
#endif
#ifndef HHFM_MAIN_PRIO
#define HHFM_MAIN_PRIO 1   // s_setprio(1) around the MFMA chain (C4 bf16 1.66 -> 1.48 ms)
#endif
#ifndef HHFM_STORE_WG
#define HHFM_STORE_WG 2048   // STORE launch size (C3: 512-2048 equal, 4096 +15 %)
#endif
#ifndef HHFM_MAIN_TARGET_WG
#define HHFM_MAIN_TARGET_WG 512   // workgroups the item splits aim for (256: 2.16, 512: 1.64, 768: 1.78, 1024: 1.72, 2048: 1.87 ms, C4 shard bf16)
#endif
// threshold seed, at most (fp32 / bf16 tables): its items are scored by a
// GMAX pass (per query and 32-item tile the largest score, no score matrix);
// C4 shard, 1,024 queries: fp32 24 / 32 / 48 / 64 K items 1.726 / 1.70 /
// 1.683 / 1.688 ms, bf16 32 / 48 / 64 / 72 K 0.910 / 0.861 / 0.857 / 0.849 ms
// (profiles/r05_k2_seed_ab.txt)
#ifndef HHFM_SEED_F32
#define HHFM_SEED_F32 49152
#endif
#ifndef HHFM_SEED_BF16
#define HHFM_SEED_BF16 73728
#endif
constexpr int64_t kSeedMax[2] = {HHFM_SEED_F32, HHFM_SEED_BF16};
// scored query-item pairs of the seed, at most: the full seed up to 1,024 queries
constexpr int64_t kSeedBudget[2] = {kSeedMax[0] * 1024, kSeedMax[1] * 1024};
#ifndef HHFM_RING_PAIR
#define HHFM_RING_PAIR 0   // 1: catalog_ring bf16 with one s_barrier per two tiles (6-slot ring; measured neutral at C4, 1.20 vs 1.21 ms)
#endif
#ifndef HHFM_RING_SLOTS
// catalog_ring bf16 tile slots: R-1 tiles of DMA lead, or (pairs) R-2
#define HHFM_RING_SLOTS (HHFM_RING_PAIR ? 6 : 4)
#endif
#ifndef HHFM_FUSED_T2
#define HHFM_FUSED_T2 0   // fused kernel: 2-tile ranges at few queries (A/B knob)
#endif
#ifndef HHFM_MAIN_PF
#define HHFM_MAIN_PF 1   // item tiles in flight per wave (1 or 2)
#endif

constexpr int kQPerWave = 32;
constexpr int kQPerBlock = 4 * kQPerWave;
constexpr int kTile = 32;  // items per MFMA tile

// ---------------------------------------------------------------------------
// 1. query vectors
// ---------------------------------------------------------------------------
template <bool BF16>
__global__ __launch_bounds__(256) void catalog_queries(
    const int32_t* __restrict__ qidx, int64_t B, int64_t Bpad, int ncols,
    int mode, int ucol, int c0, int c1, int t0, int t1,
    const char* __restrict__ E, int64_t M, int k, float* __restrict__ H,
    float* __restrict__ cst) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int esz = BF16 ? 2 : 4;
  auto val = [&](int32_t id, int e) -> float {
    const char* r = E + (int64_t)clamp_id(id, M) * k * esz;
    return BF16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(r)[e])
                : reinterpret_cast<const float*>(r)[e];
  };
  for (int64_t b = wave; b < Bpad; b += nwave) {
    float part = 0.f;
    if (b < B) {
      const int32_t* p = qidx + b * (int64_t)ncols;
      for (int e = lane; e < k; e += kWave) {
        const float u = val(p[ucol], e);
        float ctx = 0.f, tim = 0.f;
        for (int c = c0; c < c1; ++c) ctx += val(p[c], e);
        for (int c = t0; c < t1; ++c) tim += val(p[c], e);
        float h;
        if (mode == HHFM_MODE_FM) {
          h = u + ctx;          // UserWithFeature            FM.py:177
          part += h * ctx;      // item-independent (u+f)·f   FM.py:178-183
        } else {
          h = u;                // Σ[user, Σctx, Σtime]        OurModel7.py:270-292
          if (c1 > c0) h = h + ctx;
          if (t1 > t0) h = h + tim;
        }
        H[b * k + e] = h;
      }
    } else {
      for (int e = lane; e < k; e += kWave) H[b * k + e] = 0.f;
    }
    part = group_sum<kWave>(part);
    if (lane == 0) cst[b] = part;
  }
}

// ---------------------------------------------------------------------------
// 2. main kernel
// ---------------------------------------------------------------------------
// XCD-aware bijective remap: consecutive work ids land on one XCD (blocks b
// and b+8 share an XCD), so the workgroups sweeping one item split share L2.
HHFM_DEV int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, slot = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

HHFM_DEV float fkey_inv(int32_t k) { return __int_as_float(k >= 0 ? k : (k ^ 0x7fffffff)); }

template <int KPAD>
HHFM_DEV void insert_one(float* ls, int32_t* li, float s, int32_t it, int K) {
  const int l = lane_id();
  const float es = (l < KPAD) ? ls[l] : kNegInf;
  const int32_t ei = (l < KPAD) ? li[l] : kNoIdx;
  const int pos = __popcll(__ballot(better(es, ei, s, it)));
  if (pos < K) {  // wave-uniform
    const float ps = __shfl_up(es, 1, kWave);
    const int32_t pi = __shfl_up(ei, 1, kWave);
    const float ns = l < pos ? es : (l == pos ? s : ps);
    const int32_t ni = l < pos ? ei : (l == pos ? it : pi);
    if (l < KPAD) {
      ls[l] = ns;
      li[l] = ni;
    }
  }
}

// SPLIT: the dot products on v_mfma_f32_32x32x16_bf16 (16x the fp32 MFMA
// rate) with every fp32 operand split into three bf16 pieces.  bf16 tables:
// item·q = item·q0 + item·q1 + item·q2, every product exact in fp32 (3 MFMAs
// per 16 k instead of 8 fp32 ones).  fp32 tables: the six piece products of
// order >= 2^-16 (the dropped ones are < 2^-24 relative), 6 MFMAs per 16 k
// instead of 8.  The result differs from the k-ordered fmaf chain only in
// fp32 accumulation order (~1e-7 relative; tolerance 1e-5, north_star).
// STORE: no selection — the score tile is written to the score matrix
// out_s [B][ostride_b] (the small-catalog path's scores for topk_dense).  The
// MFMA operands are swapped (queries as A, items as B) so a lane's column is
// an item: each store instruction writes 32 consecutive items of a query row.
// GMAX: no selection — per query and 32-item tile the largest score, out_s
// [B][ostride_b] column = tile (the threshold seed: the K-th largest of K
// disjoint tiles' maxima is a score at least K items reach).  Selecting
// layout, so every maximum is bit for bit a score the main pass computes.
template <bool BF16, int KT, int KPAD, bool FM, bool SPLIT, bool STORE = false, bool GMAX = false>
__global__ __launch_bounds__(256) void catalog_main(
    const float* __restrict__ H, const float* __restrict__ cst, int64_t B,
    const char* __restrict__ E, int64_t item_row_begin, int32_t N,
    const float* __restrict__ w, int K, int S, int tiles_per_split, int nqb,
    float* __restrict__ out_s, int32_t* __restrict__ out_i, int64_t ostride_b,
    int64_t ostride_s, int32_t gbase, int32_t* __restrict__ gthr) {
  constexpr int k = BF16 ? KT * 16 : KT * 8;   // factors
  constexpr int64_t ROWB = (int64_t)KT * 32;   // bytes per embedding row
  constexpr int EPC = BF16 ? 8 : 4;            // k-elements per 16-B chunk
  constexpr int kBulkMin = 128;                // candidates/tile -> bulk merge

  // list stride KPAD + 1: lane j's read of entry LST j + K - 1 (per tile) hits
  // distinct banks (at stride 32 / 64 all 32 lanes fall in 2 / 1 banks)
  constexpr int LST = KPAD + 1;
  __shared__ float lst_s[4][kQPerWave * LST];
  __shared__ int32_t lst_i[4][kQPerWave * LST];
  __shared__ float tb[4][kQPerWave * kTile];

  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wid / nqb;
  const int g = wid - split * nqb;
  const int wv = threadIdx.x / kWave;
  const int l = lane_id();
  const int j = l & 31;   // query column of this lane (MFMA B/C layout)
  const int h = l >> 5;   // k half (A/B layout) / row half (C layout)
  const int64_t q0 = (int64_t)g * kQPerBlock + wv * kQPerWave;
  if (q0 >= B) return;    // whole wave idle; no block-level sync below

  const int ntiles = (N + kTile - 1) / kTile;
  const int tb0 = split * tiles_per_split;
  const int tb1 = min(tb0 + tiles_per_split, ntiles);
  const int item_end = min(tb1 * kTile, N);

  float* ls = lst_s[wv];
  int32_t* li = lst_i[wv];
  float* T = tb[wv];
  for (int x = l; x < kQPerWave * LST && !STORE && !GMAX; x += kWave) {
    ls[x] = kNegInf;
    li[x] = kNoIdx;
  }

  // B operand: this lane's query, k-slices {EPC*(2t+h) .. +EPC} for every t
  const int64_t q = q0 + j;
  float bq[KT][EPC];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const float4* src =
        reinterpret_cast<const float4*>(H + q * k + (2 * t + h) * EPC);
#pragma unroll
    for (int v = 0; v < EPC / 4; ++v) {
      const float4 x = src[v];
      bq[t][4 * v + 0] = x.x; bq[t][4 * v + 1] = x.y;
      bq[t][4 * v + 2] = x.z; bq[t][4 * v + 3] = x.w;
    }
  }
  // split B operand: per 16-k MFMA step u, lane half h holds the query's k
  // values of chunk u (bf16 tables) or of chunks 2u, 2u+1 (fp32 tables) —
  // the same k the A operand's item values carry
  constexpr int NU = SPLIT ? (BF16 ? KT : KT / 2) : 1;
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
  float cq = 0.f;
  if constexpr (FM) cq = cst[q];
  float thr = (q < B) ? kNegInf : __builtin_huge_valf();

  // A operand: a ring of PF item tiles in flight (item row tile*32 + j, 16 B
  // per k-chunk); tile t is consumed from ring slot t % PF and its slot is
  // refilled with tile t + PF while its MFMAs run
  constexpr int PF = HHFM_MAIN_PF;
  uint4 a0[KT], a1[KT];
  float wi0 = 0.f, wi1 = 0.f;
  auto load_tile = [&](int tile, uint4 (&ar)[KT], float& wr) {
    tile = tile < tb1 ? tile : tb1 - 1;
    int item = tile * kTile + j;
    item = item < N ? item : N - 1;
    const char* row = E + (item_row_begin + item) * ROWB + 16 * h;
#pragma unroll
    for (int t = 0; t < KT; ++t) ar[t] = *reinterpret_cast<const uint4*>(row + 32 * t);
    if constexpr (FM) wr = w ? w[item_row_begin + item] : 0.f;
  };
  if (tb0 < tb1) {
    load_tile(tb0, a0, wi0);
    if constexpr (PF == 2) load_tile(tb0 + 1, a1, wi1);
  }

  // A x B on the bf16 MFMA; STORE swaps the roles (queries as A)
  auto mma16 = [&](const bf16x8& x, const bf16x8& y, const f32x16& c) {
    return STORE ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(y, x, c, 0, 0, 0)
                 : __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, c, 0, 0, 0);
  };
  auto tile_step = [&](const int tile, uint4 (&ar)[KT], float& wr) {
    // global threshold hint: load now, consume after the MFMA chain (STORE:
    // no selection, and the small-catalog path leaves gthr unset)
    const int32_t gk = (!STORE && !GMAX && q < B) ? gthr[q] : 0;
    f32x16 acc = {0};
    const int nxt = tile + PF < tb1 ? tile + PF : tile;
    float wcur = wr;
    auto refill = [&](int t) {   // rolling prefetch: chunk t of the next tile
      int item = nxt * kTile + j;
      item = item < N ? item : N - 1;
      ar[t] = *reinterpret_cast<const uint4*>(E + (item_row_begin + item) * ROWB + 16 * h + 32 * t);
    };
    if (HHFM_MAIN_PRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr (SPLIT && BF16) {
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const bf16x8 ai = __builtin_bit_cast(bf16x8, ar[t]);
        refill(t);
        acc = mma16(ai, qp[2][t], acc);
        acc = mma16(ai, qp[1][t], acc);
        acc = mma16(ai, qp[0][t], acc);
      }
    } else if constexpr (SPLIT) {
#pragma unroll
      for (int u = 0; u < KT / 2; ++u) {
        const float x[8] = {__uint_as_float(ar[2 * u].x), __uint_as_float(ar[2 * u].y),
                            __uint_as_float(ar[2 * u].z), __uint_as_float(ar[2 * u].w),
                            __uint_as_float(ar[2 * u + 1].x), __uint_as_float(ar[2 * u + 1].y),
                            __uint_as_float(ar[2 * u + 1].z), __uint_as_float(ar[2 * u + 1].w)};
        refill(2 * u);
        refill(2 * u + 1);
        bf16x8 i0, i1, i2;
        split3x8(x, i0, i1, i2);
        // smallest terms first
        acc = mma16(i2, qp[0][u], acc);
        acc = mma16(i1, qp[1][u], acc);
        acc = mma16(i0, qp[2][u], acc);
        acc = mma16(i1, qp[0][u], acc);
        acc = mma16(i0, qp[1][u], acc);
        acc = mma16(i0, qp[0][u], acc);
      }
    } else
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      float av[EPC];
      if constexpr (BF16) {
        const uint32_t r4[4] = {ar[t].x, ar[t].y, ar[t].z, ar[t].w};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          av[2 * v] = __uint_as_float(r4[v] << 16);
          av[2 * v + 1] = __uint_as_float(r4[v] & 0xffff0000u);
        }
      } else {
        av[0] = __uint_as_float(ar[t].x); av[1] = __uint_as_float(ar[t].y);
        av[2] = __uint_as_float(ar[t].z); av[3] = __uint_as_float(ar[t].w);
      }
      // rolling prefetch: chunk t of the next tile replaces the consumed one
      {
        int item = nxt * kTile + j;
        item = item < N ? item : N - 1;
        ar[t] = *reinterpret_cast<const uint4*>(E + (item_row_begin + item) * ROWB +
                                               16 * h + 32 * t);
      }
#pragma unroll
      for (int e = 0; e < EPC; ++e)
        acc = STORE ? __builtin_amdgcn_mfma_f32_32x32x2f32(bq[t][e], av[e], acc, 0, 0, 0)
                    : __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bq[t][e], acc, 0, 0, 0);
    }
    if (HHFM_MAIN_PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (FM) {
      // D[i][j] += w_i * 1 + 1 * (q_j·f_j)   (bias row/col folded into one MFMA)
      // STORE: D[q][i] += 1 * w_i + (q_q·f_q) * 1 — the same products at the
      // same k positions as the selecting kernel, so both give the same bits
      if constexpr (STORE)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h == 0 ? 1.f : cq,
                                                   h == 0 ? wcur : 1.f, acc, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h == 0 ? wcur : 1.f,
                                                   h == 0 ? 1.f : cq, acc, 0, 0, 0);
      int item = nxt * kTile + j;
      item = item < N ? item : N - 1;
      wr = w ? w[item_row_begin + item] : 0.f;
    }

    if constexpr (STORE) {   // rows = queries q0 + ..., column = item tile*32 + j
      const int32_t item = tile * kTile + j;
      if (item < item_end) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t qr = q0 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (qr < B) out_s[qr * ostride_b + item] = acc[r];
        }
      }
      return;
    }
    if constexpr (GMAX) {   // lane (j, h): query q, items rows (r&3)+8(r>>2)+4h
      const int ib = tile * kTile;
      float m = kNegInf;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        m = ib + row < item_end ? fmaxf(m, acc[r]) : m;
      }
      m = fmaxf(m, shfl_f(m, l ^ 32));
      if (h == 0 && q < B) out_s[q * ostride_b + tile] = m;
      return;
    }
    // ---- filter against the per-query K-th score ----
    // The threshold is the better of this split's K-th score and the best
    // K-th score any split has published for the query (gthr: monotone
    // atomicMax hint; a stale value only admits extra candidates).
    if (q < B) thr = fmaxf(thr, fkey_inv(gk));
    const int ibase = tile * kTile;
#if HHFM_MAIN_KO & 1   // diagnostic knock-out: no selection (scores still consumed)
    {
      float sx = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) sx += acc[r];
      if (sx == 1234.5f) out_s[0] = sx;
      return;
    }
#endif
    // survivors as wave ballots (SGPRs; a lane reads its own bit back where
    // needed), and the item_end mask only on the split's partial last tile
    uint64_t pm[16];
    if (ibase + kTile <= item_end) {
#pragma unroll
      for (int r = 0; r < 16; ++r) pm[r] = __ballot(acc[r] >= thr);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        pm[r] = __ballot(acc[r] >= thr && ibase + row < item_end);
      }
    }
    int count = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) count += __popcll(pm[r]);
    if (count == 0) return;
    const uint64_t lbit = 1ull << l;
#define HHFM_PASS(r) ((pm[r] & lbit) != 0)
#define HHFM_PASSMASK(r) (pm[r])

    if (count <= kBulkMin) {
      // sparse: one wave-wide sorted insertion per surviving score
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        uint64_t m = HHFM_PASSMASK(r);
        while (m) {
          const int L = __builtin_ctzll(m);
          m &= m - 1;
          const float s = __int_as_float(
              __builtin_amdgcn_readlane(__float_as_int(acc[r]), L));
          const int row = (r & 3) + 8 * (r >> 2) + 4 * (L >> 5);
          const int qq = L & 31;
          insert_one<KPAD>(ls + qq * LST, li + qq * LST, s, ibase + row, K);
        }
      }
    } else {
      // dense: transpose the masked tile to LDS (XOR-swizzled, conflict
      // free), bitonic-sort each query's 32 scores, merge into its list
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        T[j * kTile + (row ^ j)] = HHFM_PASS(r) ? acc[r] : kNegInf;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): tile visible to the wave
      __builtin_amdgcn_wave_barrier();
      for (int p = 0; p < kQPerWave / 2; ++p) {
        const int qh = 2 * p + h;
        float s = T[qh * kTile + (j ^ qh)];
        int32_t it = s == kNegInf ? kNoIdx : ibase + j;
        bitonic_sort_desc<32>(s, it);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int qq = 2 * p + hh;
          float bs = shfl_f(s, 32 * hh + j);
          int32_t bi = shfl_i(it, 32 * hh + j);
          if (l >= 32) { bs = kNegInf; bi = kNoIdx; }
          float as = l < KPAD ? ls[qq * LST + l] : kNegInf;
          int32_t ai = l < KPAD ? li[qq * LST + l] : kNoIdx;
          merge_lists<KPAD>(as, ai, bs, bi);
          if (l < KPAD) {
            ls[qq * LST + l] = as;
            li[qq * LST + l] = ai;
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if (q < B) {
      const float kth = ls[j * LST + (K - 1)];
      if (kth > thr) {
        thr = kth;
        if (h == 0) atomicMax(gthr + q, fkey(kth));   // publish for other splits
      }
    }
  };
  if constexpr (PF == 2) {
    for (int tile = tb0; tile < tb1; tile += 2) {
      tile_step(tile, a0, wi0);
      if (tile + 1 < tb1) tile_step(tile + 1, a1, wi1);
    }
  } else {
    for (int tile = tb0; tile < tb1; ++tile) tile_step(tile, a0, wi0);
  }

#undef HHFM_PASS
#undef HHFM_PASSMASK
  if constexpr (STORE || GMAX) return;
  // ---- emit this split's sorted list per query ----
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  for (int qq = 0; qq < kQPerWave; ++qq) {
    const int64_t b = q0 + qq;
    if (b >= B) break;
    if (l < K) {
      const int32_t ii = li[qq * LST + l];
      out_s[b * ostride_b + split * ostride_s + l] = ls[qq * LST + l];
      out_i[b * ostride_b + split * ostride_s + l] = ii == kNoIdx ? kNoIdx : ii + gbase;
    }
  }
}

// ---------------------------------------------------------------------------
// 2a'. catalog_ring — the streaming kernel with the item tiles staged in LDS
//
// catalog_main streams every item tile into each wave's registers one tile
// ahead: at the C4 shape that leaves the SIMDs parked on memory half the time
// (bf16 tables: SQ_WAIT_ANY 50 % of wave cycles, MFMA busy 35 %) and, for
// fp32 tables, every wave splits the same tile into its three bf16 pieces (4
// copies of ~320 VALU per tile).  Here a workgroup is 4 waves = 128 queries x
// one item split (two workgroups per CU, two waves per SIMD), and the tile is
// fetched ONCE per workgroup:
//   * bf16 tables: a ring of R tile slots, filled R-1 tiles ahead by LDS-DMA
//     (global_load_lds_dwordx4) with per-lane source addresses chosen so the
//     image is [k16 step][half][item] x 16 B — every A-operand ds_read_b128
//     reads 16 consecutive 16-B slots (conflict-free);
//   * fp32 tables: each lane loads NU/NW (item, 16-k step, half) units of the
//     tile one tile ahead into registers, splits them into their three bf16
//     pieces (exact, split3x8) and stores them into a double-buffered piece
//     image [piece][step][half][item]: 1/256 of the split work per lane.
// One s_barrier per tile (4 waves; the other workgroup on the CU is not
// coupled to it).  The MFMA products, their k order and the selection are
// catalog_main's (SPLIT path), so scores are bit-identical to it and to the
// GMAX seed.  Candidates are inserted one by one (the dense sort + merge
// path and its LDS transpose buffer are dropped): the kernel runs only behind
// the threshold seed, which leaves a few insertions per query and split.
// Used for K <= 32, bf16 k = 128 and fp32 k in {64, 128}.
// ---------------------------------------------------------------------------
#ifndef HHFM_RING_KO
// diagnostic knock-outs (wrong results; timing only): 1 no selection (scores
// still consumed), 2 no per-tile s_barrier, 4 no MFMA chain
#define HHFM_RING_KO 0
#endif
#ifndef HHFM_RING_TIMING
#define HHFM_RING_TIMING 0   // diagnostic build: per-phase s_memtime sums (hhfm_debug_ring_timing)
#endif
#if (HHFM_MAIN_KO || HHFM_RING_KO || HHFM_RING_TIMING) && !defined(HHFM_DIAG_BUILD)
#error "K2 knock-out / timing macros give wrong results: diagnostic builds only (-DHHFM_DIAG_BUILD)"
#endif
#if HHFM_RING_TIMING
// [0] publish (vmcnt + barrier + staging issue), [1] MFMA chain to ballots,
// [2] selection, [3] wave-tiles, [4] whole kernel per wave, [5] waves
__device__ unsigned long long g_ring_t[8];
#endif

template <bool BF16, int KT, int NW>
struct RingCfg {
  static constexpr int kRingWaves = NW;                      // waves (x 32 queries) per workgroup
  static constexpr int kRowB = KT * 32;                      // bytes per item row
  static constexpr int kTileB = kTile * kRowB;               // one raw tile
  static constexpr int kNU = BF16 ? KT : KT / 2;             // 16-k MFMA steps per tile
  static constexpr int kSlots = BF16 ? HHFM_RING_SLOTS : 2;
  static constexpr int kStageB = BF16 ? kSlots * kTileB : 2 * 3 * kNU * 1024;
  // per-query lists of KPAD 32 at a stride of 33 entries: the per-tile read
  // of every query's K-th entry (lane j: entry 33 j + K - 1) then hits 32
  // banks, not 2 (a 16-way conflict per wave and tile at stride 32)
  static constexpr int kLStride = 33;
  static constexpr int kListB = kRingWaves * kQPerWave * kLStride * 8;
  static constexpr int kSmem = kStageB + kListB;
  static constexpr int kDma = BF16 ? KT / kRingWaves : 0;    // DMA instructions per wave and tile
  static constexpr int kUnits = BF16 ? 0 : (kNU + NW - 1) / NW;   // fp32 split units per lane
};

// GMAX: no selection — per query and tile the largest score into out_s
// [B][ostride_b] (the threshold seed, as catalog_main's GMAX: same products,
// same bits as the selecting pass)
template <bool BF16, int KT, bool FM, int NW, bool GMAX = false>
__global__ __launch_bounds__(NW * 64) void catalog_ring(
    const float* __restrict__ H, const float* __restrict__ cst, int64_t B,
    const char* __restrict__ E, int64_t item_row_begin, int32_t N,
    const float* __restrict__ w, int K, int S, int tiles_per_split, int nqb,
    float* __restrict__ out_s, int32_t* __restrict__ out_i, int64_t ostride_b,
    int64_t ostride_s, int32_t gbase, int32_t* __restrict__ gthr) {
  using Cfg = RingCfg<BF16, KT, NW>;
  constexpr int kRingWaves = NW;
  constexpr int kRingQ = NW * kQPerWave;
  constexpr int KPAD = 32;
  constexpr int k = BF16 ? KT * 16 : KT * 8;
  constexpr int64_t ROWB = Cfg::kRowB;
  constexpr int NU = Cfg::kNU;
  constexpr int R = Cfg::kSlots;
  constexpr bool kPair = BF16 && HHFM_RING_PAIR;   // tiles 2i, 2i+1 behind one barrier
  static_assert(BF16 ? KT % kRingWaves == 0 : true, "ring kernel: bf16 k >= 16 * waves");

  __shared__ __attribute__((aligned(16))) char smem[Cfg::kSmem];
  char* stage = smem;
  float* lst_s = reinterpret_cast<float*>(smem + Cfg::kStageB);
  int32_t* lst_i = reinterpret_cast<int32_t*>(smem + Cfg::kStageB + Cfg::kListB / 2);

  const int wid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wid / nqb;
  const int g = wid - split * nqb;
  const int wv = threadIdx.x / kWave;
  const int l = lane_id();
  const int j = l & 31;   // query column (MFMA B/C layout) / item row (A layout)
  const int h = l >> 5;   // k half (A/B layout) / row half (C layout)
  const int64_t q0 = (int64_t)g * kRingQ + wv * kQPerWave;
  const bool wave_live = q0 < B;   // idle waves still take part in barriers and staging

  const int ntiles = (N + kTile - 1) / kTile;
  const int tb0 = split * tiles_per_split;
  const int tb1 = min(tb0 + tiles_per_split, ntiles);
  const int item_end = min(tb1 * kTile, N);

  constexpr int LST = Cfg::kLStride;
  float* ls = lst_s + wv * (kQPerWave * LST);
  int32_t* li = lst_i + wv * (kQPerWave * LST);
  for (int x = l; x < kQPerWave * LST && !GMAX; x += kWave) {
    ls[x] = kNegInf;
    li[x] = kNoIdx;
  }

  // B operand: the wave's 32 queries split into three bf16 pieces (catalog_main)
  const int64_t q = q0 + j;
  constexpr int EPC = BF16 ? 8 : 4;
  bf16x8 qp[3][NU];
  {
    const int64_t qs = q < B ? q : 0;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      float x[8];
      if constexpr (BF16) {
        const float4* src = reinterpret_cast<const float4*>(H + qs * k + (2 * u + h) * EPC);
        const float4 a = src[0], b = src[1];
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
        x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      } else {   // chunks 2u and 2u+1 of the lane half: k {16u+4h..+3, 16u+8+4h..+3}
        const float4 a = *reinterpret_cast<const float4*>(H + qs * k + (4 * u + h) * EPC);
        const float4 b = *reinterpret_cast<const float4*>(H + qs * k + (4 * u + 2 + h) * EPC);
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
        x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      }
      split3x8(x, qp[0][u], qp[1][u], qp[2][u]);
    }
  }
  float cq = 0.f;
  if constexpr (FM) cq = q < B ? cst[q] : 0.f;
  // the threshold seed (and any K-th an earlier split published): read once —
  // behind the seed the per-split lists rarely beat it, so a per-tile reload
  // of the hint would only put a global load on every tile's critical path
  float thr = (!GMAX && q < B) ? fkey_inv(gthr[q]) : __builtin_huge_valf();

  auto item_row = [&](int tile, int jj) -> const char* {
    tile = tile < tb1 ? tile : tb1 - 1;
    int item = tile * kTile + jj;
    item = item < N ? item : N - 1;
    return E + (item_row_begin + item) * ROWB;
  };

  // ---- staging ----
  // bf16: DMA instruction d of wave wv moves LDS units [64(wv + 4d), +64):
  // unit P = (t*2 + h)*32 + j  <-  item j, bytes [32t + 16h, +16) of its row
  auto dma_tile = [&](int tile, int slot) {
    if constexpr (BF16) {
#pragma unroll
      for (int d = 0; d < Cfg::kDma; ++d) {
        const int t = wv + kRingWaves * d;
        const char* src = item_row(tile, j) + 32 * t + 16 * h;
        char* dst = stage + slot * Cfg::kTileB + t * 1024;
        __builtin_amdgcn_global_load_lds((const void*)src, (void*)dst, 16, 0, 0);
      }
    }
  };
  // fp32: lane units (item j, step u = wv + 4r, half h); raw = their 8 floats
  constexpr int NUL = Cfg::kUnits > 0 ? Cfg::kUnits : 1;
  auto load_unit = [&](int tile, uint4 (&raw)[NUL][2]) {
    if constexpr (!BF16) {
      const char* row = item_row(tile, j) + 16 * h;
#pragma unroll
      for (int r = 0; r < NUL; ++r) {
        const int u = wv + kRingWaves * r;
        // (compile-time true when the waves divide the steps: no branch, so
        // the compiler counts these loads exactly in its vmcnt waits)
        if (NU % kRingWaves == 0 || u < NU) {
          raw[r][0] = *reinterpret_cast<const uint4*>(row + 64 * u);
          raw[r][1] = *reinterpret_cast<const uint4*>(row + 64 * u + 32);
        }
      }
    }
  };
  auto store_pieces = [&](const uint4 (&raw)[NUL][2], int buf) {
    if constexpr (!BF16) {
#pragma unroll
      for (int r = 0; r < NUL; ++r) {
        const int u = wv + kRingWaves * r;
        if (NU % kRingWaves != 0 && u >= NU) continue;
        const float x[8] = {__uint_as_float(raw[r][0].x), __uint_as_float(raw[r][0].y),
                            __uint_as_float(raw[r][0].z), __uint_as_float(raw[r][0].w),
                            __uint_as_float(raw[r][1].x), __uint_as_float(raw[r][1].y),
                            __uint_as_float(raw[r][1].z), __uint_as_float(raw[r][1].w)};
        bf16x8 pcs[3];
        split3x8(x, pcs[0], pcs[1], pcs[2]);
        char* base = stage + buf * (3 * NU * 1024) + (u * 2 + h) * 512 + j * 16;
#pragma unroll
        for (int pc = 0; pc < 3; ++pc)
          *reinterpret_cast<bf16x8*>(base + pc * NU * 1024) = pcs[pc];
      }
    }
  };
  // A fragment: bf16 slot/step t, or fp32 piece pc of step u
  auto a_bf16 = [&](int slot, int t) {
    return *reinterpret_cast<const bf16x8*>(stage + slot * Cfg::kTileB + (t * 2 + h) * 512 +
                                            j * 16);
  };
  auto a_piece = [&](int buf, int pc, int u) {
    return *reinterpret_cast<const bf16x8*>(stage + buf * (3 * NU * 1024) + pc * NU * 1024 +
                                            (u * 2 + h) * 512 + j * 16);
  };
  // vmcnt(n): wait until at most n of this wave's vector-memory ops are in flight
  // (n a compile-time constant; lgkmcnt/expcnt untouched)
#define HHFM_VMCNT(n) \
  __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

  uint4 raw[NUL][2];
  float wnext = 0.f;
  if (tb0 < tb1) {
    if constexpr (BF16) {
      for (int s = 0; s < (kPair ? R - 2 : R - 1); ++s) dma_tile(tb0 + s, s);
    } else {
      load_unit(tb0, raw);
      store_pieces(raw, 0);
      load_unit(tb0 + 1, raw);
    }
    if constexpr (FM) {
      const int item = min(tb0 * kTile + j, N - 1);
      wnext = w ? w[item_row_begin + item] : 0.f;
    }
  }

  auto mma16 = [&](const bf16x8& x, const bf16x8& y, const f32x16& c) {
#if HHFM_RING_KO & 4   // knock-out: the operands still read, no MFMA
    f32x16 r = c;
    r[0] += __builtin_bit_cast(float, __builtin_bit_cast(uint4, x).x) * 1e-30f;
    (void)y;
    return r;
#else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, c, 0, 0, 0);
#endif
  };

  // sync: publish the stage (every fp32 tile; bf16 pairs: the first tile of
  // each pair, whose barrier also covers the second)
#if HHFM_RING_TIMING
  uint64_t tm_k0 = __builtin_amdgcn_s_memtime(), tm1 = 0, sum_pub = 0, sum_mma = 0,
           sum_sel = 0, ntl = 0;
#endif
  // one tile = publish (sync: the stage is complete and the previous one
  // free), score (the MFMA chain; acc = this wave's 32 items x 32 queries),
  // select (filter + insert into the per-query lists)
  auto publish = [&](const int tile, const bool sync) {
    const int it = tile - tb0;
    (void)it;
    // ---- publish: tile's stage complete and the previous tile's stage free ----
    if (sync) {
      // bf16: every step issues its DMAs unconditionally (tiles past the split
      // re-read its last tile into a free slot), so the count of tiles issued
      // after this one is exact up to the split's end: R-2, or (pairs) the
      // next pair's 2
      if constexpr (kPair)
        HHFM_VMCNT(2 * Cfg::kDma);
      else if constexpr (BF16)
        HHFM_VMCNT((R - 2) * Cfg::kDma);
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's piece stores landed
      if (!(HHFM_RING_KO & 2)) __builtin_amdgcn_s_barrier();
      if constexpr (kPair) {   // into the previous pair's slots
        dma_tile(tile + 4, (it + 4) % R);
        dma_tile(tile + 5, (it + 5) % R);
      } else if constexpr (BF16) {
        dma_tile(tile + R - 1, (it + R - 1) % R);
      } else {
        // split tile+1 into the other piece buffer, then fetch the unit of
        // tile+2 into the same registers (one tile of lead), unconditionally:
        // past the split's end load_unit re-reads its last tile
        store_pieces(raw, (it + 1) & 1);
        load_unit(tile + 2, raw);
      }
    }
  };
  auto score = [&](const int tile) -> f32x16 {
    const int it = tile - tb0;
    float wcur = wnext;
    if constexpr (FM) {
      const int item = min((tile + 1 < tb1 ? tile + 1 : tile) * kTile + j, N - 1);
      wnext = w ? w[item_row_begin + item] : 0.f;
    }
    f32x16 acc = {0};
    if (HHFM_MAIN_PRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr (BF16) {
      const int slot = it % R;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const bf16x8 ai = a_bf16(slot, t);
        acc = mma16(ai, qp[2][t], acc);
        acc = mma16(ai, qp[1][t], acc);
        acc = mma16(ai, qp[0][t], acc);
      }
    } else {
      const int buf = it & 1;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const bf16x8 i0 = a_piece(buf, 0, u), i1 = a_piece(buf, 1, u), i2 = a_piece(buf, 2, u);
        acc = mma16(i2, qp[0][u], acc);   // smallest terms first (catalog_main order)
        acc = mma16(i1, qp[1][u], acc);
        acc = mma16(i0, qp[2][u], acc);
        acc = mma16(i1, qp[0][u], acc);
        acc = mma16(i0, qp[1][u], acc);
        acc = mma16(i0, qp[0][u], acc);
      }
    }
    if (HHFM_MAIN_PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (FM)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h == 0 ? wcur : 1.f, h == 0 ? 1.f : cq, acc,
                                                 0, 0, 0);
    return acc;
  };
  auto select = [&](const int tile, const f32x16& acc) {
    if (!wave_live) return;
#if HHFM_RING_KO & 1
    {
      float sx = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) sx += acc[r];
      if (sx == 1234.5f) out_s[0] = sx;
      return;
    }
#endif
    if constexpr (GMAX) {
      const int ib = tile * kTile;
      float m = kNegInf;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        m = ib + row < item_end ? fmaxf(m, acc[r]) : m;
      }
      m = fmaxf(m, shfl_f(m, l ^ 32));
      if (h == 0 && q < B && tile < tb1) out_s[q * ostride_b + tile] = m;
      return;
    }
    // ---- filter + insert: catalog_main's selection ----
    const int ibase = tile * kTile;
    uint64_t pm[16];
    if (ibase + kTile <= item_end) {
#pragma unroll
      for (int r = 0; r < 16; ++r) pm[r] = __ballot(acc[r] >= thr);
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        pm[r] = __ballot(acc[r] >= thr && ibase + row < item_end);
      }
    }
    int count = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) count += __popcll(pm[r]);
    if (count == 0) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      uint64_t m = pm[r];
      while (m) {
        const int L = __builtin_ctzll(m);
        m &= m - 1;
        const float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc[r]), L));
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (L >> 5);
        const int qq = L & 31;
        insert_one<KPAD>(ls + qq * LST, li + qq * LST, s, ibase + row, K);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    if (q < B) {
      const float kth = ls[j * LST + (K - 1)];
      if (kth > thr) {
        thr = kth;
        if (h == 0) atomicMax(gthr + q, fkey(kth));
      }
    }
  };
#if HHFM_RING_TIMING
#define HHFM_RING_T(x) x
#else
#define HHFM_RING_T(x)
#endif
  auto step = [&](const int tile, const bool sync) {
    HHFM_RING_T(const uint64_t t0 = __builtin_amdgcn_s_memtime();)
    publish(tile, sync);
    HHFM_RING_T(tm1 = __builtin_amdgcn_s_memtime();)
    select(tile, score(tile));
    HHFM_RING_T(sum_pub += tm1 - t0; sum_mma += __builtin_amdgcn_s_memtime() - tm1; ++ntl;)
  };
  // one raw register set, loaded one tile ahead (fp32).  Two sets
  // alternating over an unrolled pair of steps (two tiles of lead) ran the
  // same with unconditional loads (1.572 vs 1.571 ms) and 1.66 ms with the
  // old conditional ones, whose registers the compiler rotated through copies
  // behind a vmcnt(0) every second tile (profiles/r05_k2_c4.txt)
  for (int tile = tb0; tile < tb1; ++tile) step(tile, !kPair || !((tile - tb0) & 1));
#undef HHFM_RING_T
#undef HHFM_VMCNT
#if HHFM_RING_TIMING
  if (wave_live && l == 0) {
    atomicAdd(&g_ring_t[0], sum_pub);
    atomicAdd(&g_ring_t[1], sum_mma);
    atomicAdd(&g_ring_t[2], sum_sel);
    atomicAdd(&g_ring_t[3], ntl);
    atomicAdd(&g_ring_t[4], __builtin_amdgcn_s_memtime() - tm_k0);
    atomicAdd(&g_ring_t[5], 1ull);
  }
#endif
  if (!wave_live || GMAX) return;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  for (int qq = 0; qq < kQPerWave; ++qq) {
    const int64_t b = q0 + qq;
    if (b >= B) break;
    if (l < K) {
      const int32_t ii = li[qq * LST + l];
      out_s[b * ostride_b + split * ostride_s + l] = ls[qq * LST + l];
      out_i[b * ostride_b + split * ostride_s + l] = ii == kNoIdx ? kNoIdx : ii + gbase;
    }
  }
}

// ---------------------------------------------------------------------------
// 3. merge of R sorted lists per query
// ---------------------------------------------------------------------------
template <int KPAD>
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const float* __restrict__ in_s, const int32_t* __restrict__ in_i, int R,
    int64_t B, int K, int64_t stride_r, int64_t stride_b,
    float* __restrict__ out_s, int32_t* __restrict__ out_i) {
  const int l = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t b = wave; b < B; b += nwave) {
    float as = kNegInf;
    int32_t ai = kNoIdx;
    // lists in groups of kPF: a group's loads are all in flight before its
    // merges (one load latency per group instead of per list).  KPAD = 32:
    // the two 32-lane halves merge the even and the odd lists side by side,
    // then the odd half's list is merged into the even half's.  Every merge
    // keeps the top KPAD of a union under the strict (score desc, id asc)
    // order, so the result is the sequential merge's; lists past R are empty
    // (-inf, no index) and merge as no-ops.
    constexpr int kPF = 8;
    constexpr int kHalves = KPAD == 32 ? 2 : 1;
    const int h = kHalves == 2 ? l >> 5 : 0;
    const int lh = l & (KPAD - 1);
    for (int r0 = 0; r0 < R; r0 += kPF * kHalves) {
      float bs[kPF];
      int32_t bi[kPF];
#pragma unroll
      for (int u = 0; u < kPF; ++u) {
        const int r = r0 + u * kHalves + h;
        const bool ok = r < R && lh < K;
        const int64_t off = (int64_t)(r < R ? r : 0) * stride_r + b * stride_b;
        bs[u] = ok ? in_s[off + lh] : kNegInf;
        bi[u] = ok ? in_i[off + lh] : kNoIdx;
      }
#pragma unroll
      for (int u = 0; u < kPF; ++u) {
        if constexpr (kHalves == 2) {
          const int src = (h << 5) + (31 - lh);   // reverse within the half
          const float rs = shfl_f(bs[u], src);
          const int32_t ri = shfl_i(bi[u], src);
          if (better(rs, ri, as, ai)) {
            as = rs;
            ai = ri;
          }
          bitonic_merge_desc<32>(as, ai);
        } else {
          merge_lists<KPAD>(as, ai, bs[u], bi[u]);
        }
      }
    }
    if constexpr (kHalves == 2) {   // the odd half's list into the even half's
      const float rs = shfl_f(as, 32 + (31 - lh));
      const int32_t ri = shfl_i(ai, 32 + (31 - lh));
      if (h == 0 && better(rs, ri, as, ai)) {
        as = rs;
        ai = ri;
      }
      bitonic_merge_desc<32>(as, ai);
    }
    if (l < K) {
      out_s[b * K + l] = as;
      out_i[b * K + l] = ai;
    }
  }
}

}  // namespace hhfm

#include "catalog_fused.h"

namespace hhfm {

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct Plan {
  int64_t Bpad;
  int nqb, S, tiles_per_split;
  bool dense;            // small catalog: score matrix + dense top-K
  int64_t ldsc;
  int seed_n;            // streaming path: items of the threshold seed (0 = none)
  int rnqb[2], rS[2], rtps[2];   // catalog_ring with 4 / 8 waves: query groups, splits, tiles
  int sS[2], stps[2];            // the same over the seed's items (its GMAX pass)
  int fS, fT;            // fused small-catalog kernel: workgroups (item ranges) per 32 queries, tiles per wave
  size_t off_H, off_cst, off_thr, off_ps, off_pi, off_sc, off_seed_sc, off_seed_s,
      off_seed_i, total;
};

// Small catalogs (evaluate_TopK over Frappe's 4,082 items is the case): the
// fused kernel's per-split top-K warm-up dominates when every split holds only
// a few tiles, so score the whole [B, N] matrix with the MFMA GEMM (fp32
// 16x16x4, bf16 tables widened on load) and select with one wave per query
// (hhfm_topk_dense).  Chosen by size alone, so the workspace query agrees.
static bool dense_catalog(int64_t B, int32_t N) {
  return N <= 16384 && (int64_t)B * N <= (int64_t)64 << 20;
}

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// catalog_ring item splits: ~2 x 4-wave (v = 0) or 1 x 8-wave (v = 1)
// workgroups per CU over nqb query groups, >= 16 tiles per split
static void ring_splits(int nqb, int v, int ntiles, int& S, int& tps) {
  const int smax = ntiles / 16 > 1 ? ntiles / 16 : 1;
  int rs = ((512 >> v) + nqb - 1) / nqb;
  rs = rs > smax ? smax : (rs < 1 ? 1 : rs);
  tps = (ntiles + rs - 1) / rs;
  S = (ntiles + tps - 1) / tps;
}

// Threshold seed of the streaming path (default on; HHFM_PLAN_NO_SEED off):
// the first seed_n items are scored by the main pass's own kernel in its GMAX
// form (per query and 32-item tile only the tile's maximum), and the dense
// top-K over those seed_n / 32 maxima writes every query's K-th one, t, as
// its threshold hint before the main pass.  K distinct catalog items score
// >= t, so the global K-th is >= t and items below t can be dropped; without
// it every item split warms its lists up from -inf and the per-split
// thresholds (and their atomicMax hint, a max of per-split K-ths) stay near
// the K-th of one split, which costs ~K·ln(items per split / K) list
// insertions per query and split.  The GMAX pass computes every score with
// the main pass's products in the same k order, so t is bit-exactly a score
// the main pass reproduces (tests/test_gpu_kernels.py: seeded == unseeded).
static Plan make_plan(int64_t B, int32_t N, int32_t k, int32_t K, int32_t plan, bool bf16) {
  Plan p{};
  p.nqb = (int)((B + kQPerBlock - 1) / kQPerBlock);
  p.Bpad = (int64_t)p.nqb * kQPerBlock;
  const int ntiles = (N + kTile - 1) / kTile;
  // ~2 resident workgroups per CU, but >= 16 tiles per split so
  // the per-split warm-up of the top-K lists stays amortised
  const int target = HHFM_MAIN_TARGET_WG;
  int S = (target + p.nqb - 1) / p.nqb;
  const int smax = ntiles / 16 > 1 ? ntiles / 16 : 1;
  if (S > smax) S = smax;
  if (S < 1) S = 1;
  p.tiles_per_split = (ntiles + S - 1) / S;
  p.S = (ntiles + p.tiles_per_split - 1) / p.tiles_per_split;
  p.dense = dense_catalog(B, N);
  for (int v = 0; v < 2; ++v) {   // catalog_ring: 2 x 4-wave or 1 x 8-wave workgroups per CU
    const int nq = 128 << v;
    p.rnqb[v] = (int)((B + nq - 1) / nq);
    ring_splits(p.rnqb[v], v, ntiles, p.rS[v], p.rtps[v]);
  }
  const int nsplit = std::max(p.S, std::max(p.rS[0], p.rS[1]));
  // [0, HHFM_CATALOG_WS_ZERO): the fused kernel's arrival counters, zero
  // before the first call and re-armed by every call; no plan writes there
  size_t off = HHFM_CATALOG_WS_ZERO;
  p.off_H = off;   off += align256((size_t)p.Bpad * k * sizeof(float));
  p.off_cst = off; off += align256((size_t)p.Bpad * sizeof(float));
  p.off_thr = off; off += align256((size_t)p.Bpad * sizeof(int32_t));
  p.off_ps = off;
  if (nsplit > 1) {
    off += align256((size_t)B * nsplit * K * sizeof(float));
    p.off_pi = off;
    off += align256((size_t)B * nsplit * K * sizeof(int32_t));
  } else {
    p.off_pi = off;
  }
  p.ldsc = (N + 3) & ~3;
  p.off_sc = off;
  // the fused kernel's range lists [groups][S][32 queries][32] keys share the
  // score matrix's region (never both in one call)
  // ranges of 8 x 2 tiles (512 items) while the grid stays within one
  // workgroup per CU, else 8 x 4 tiles: more CUs per query group at few
  // queries (the per-workgroup latency chain is the cost there)
  {
    const int nqb = (int)((B + kQPerWave - 1) / kQPerWave);
    const int s2 = (ntiles + kFusedWaves * 2 - 1) / (kFusedWaves * 2);
    // (2-tile ranges measured slower at 300 queries: 22.5 vs 17.4 us — the
    // merge of 8 lists per query outweighs the shorter ranges; kept off)
    p.fT = HHFM_FUSED_T2 && (int64_t)nqb * s2 <= 256 && s2 <= kFusedMaxS ? 2 : kFusedTiles;
    p.fS = (ntiles + kFusedWaves * p.fT - 1) / (kFusedWaves * p.fT);
  }
  if (p.dense) {
    const size_t sc_bytes = (size_t)B * p.ldsc * sizeof(float);
    const size_t fl_bytes = p.fS > 1 ? (size_t)((B + kQPerWave - 1) / kQPerWave) * p.fS *
                                           kQPerWave * 32 * sizeof(uint64_t)
                                     : 0;
    off += align256(sc_bytes > fl_bytes ? sc_bytes : fl_bytes);
  }
  // seed: up to kSeedMax items, kSeedBudget query-item pairs and 1/16 of the
  // catalog (the seed pass then costs <= ~6 % of the MFMA work); none below
  // 4,096 items (catalogs under 65,536 items)
  p.seed_n = 0;
  if (!p.dense && !(plan & HHFM_PLAN_NO_SEED)) {
    int64_t sn = kSeedBudget[bf16] / p.Bpad;
    sn = sn > kSeedMax[bf16] ? kSeedMax[bf16] : sn;
    sn = sn > (int64_t)N / 16 ? (int64_t)N / 16 : sn;
    sn &= ~int64_t(31);
    if (sn >= 4096) p.seed_n = (int)sn;
  }
  for (int v = 0; v < 2; ++v) {
    p.sS[v] = p.stps[v] = 0;
    if (p.seed_n) ring_splits(p.rnqb[v], v, p.seed_n / kTile, p.sS[v], p.stps[v]);
  }
  p.off_seed_sc = off;
  if (p.seed_n) {   // the seed's tile maxima [B][seed_n / 32], their top-K lists
    off += align256((size_t)B * (p.seed_n / kTile) * sizeof(float));
    p.off_seed_s = off;
    off += align256((size_t)B * K * sizeof(float));
    p.off_seed_i = off;
    off += align256((size_t)B * K * sizeof(int32_t));
  } else {
    p.off_seed_s = p.off_seed_i = off;
  }
  p.total = off;
  return p;
}

template <bool BF16, int KT, int KPAD, bool FM>
static void launch_main(const Plan& p, const float* H, const float* cst, int64_t B,
                        const char* E, int64_t item_row_begin, int32_t N,
                        const float* w, int K, float* os, int32_t* oi,
                        int64_t sb, int64_t ss, int32_t gbase, int32_t* gthr,
                        int32_t plan, hipStream_t st) {
  constexpr bool kCanSplit = BF16 || KT >= 2;   // fp32 split steps pair two chunks
  if (kCanSplit && !(plan & HHFM_PLAN_EXACT_FP32))
    hipLaunchKernelGGL((catalog_main<BF16, KT, KPAD, FM, kCanSplit>), dim3(p.nqb * p.S),
                       dim3(256), 0, st, H, cst, B, E, item_row_begin, N, w, K,
                       p.S, p.tiles_per_split, p.nqb, os, oi, sb, ss, gbase, gthr);
  else
    hipLaunchKernelGGL((catalog_main<BF16, KT, KPAD, FM, false>), dim3(p.nqb * p.S),
                       dim3(256), 0, st, H, cst, B, E, item_row_begin, N, w, K,
                       p.S, p.tiles_per_split, p.nqb, os, oi, sb, ss, gbase, gthr);
}

// catalog_ring (K <= 32, bf16 k >= 128 / fp32 k >= 64, split-bf16 MFMA):
// waves per workgroup 4 for bf16 tables, 8 for fp32 (HHFM_PLAN_RING_ALT swaps)
static int ring_waves(bool bf16, int32_t plan) {
  return (bf16 != ((plan & HHFM_PLAN_RING_ALT) != 0)) ? 4 : 8;
}

template <bool BF16, int KT, bool FM>
static void launch_ring(const Plan& p, const float* H, const float* cst, int64_t B,
                        const char* E, int64_t item_row_begin, int32_t N, const float* w,
                        int K, float* os, int32_t* oi, int64_t sb, int64_t ss, int32_t gbase,
                        int32_t* gthr, int32_t plan, hipStream_t st) {
  if (ring_waves(BF16, plan) == 8)
    hipLaunchKernelGGL((catalog_ring<BF16, KT, FM, 8>), dim3(p.rnqb[1] * p.rS[1]), dim3(512), 0,
                       st, H, cst, B, E, item_row_begin, N, w, K, p.rS[1], p.rtps[1], p.rnqb[1],
                       os, oi, sb, ss, gbase, gthr);
  else
    hipLaunchKernelGGL((catalog_ring<BF16, KT, FM, 4>), dim3(p.rnqb[0] * p.rS[0]), dim3(256), 0,
                       st, H, cst, B, E, item_row_begin, N, w, K, p.rS[0], p.rtps[0], p.rnqb[0],
                       os, oi, sb, ss, gbase, gthr);
}

template <bool BF16, bool FM>
static bool dispatch_ring(int KT, const Plan& p, const float* H, const float* cst, int64_t B,
                          const char* E, int64_t irb, int32_t N, const float* w, int K,
                          float* os, int32_t* oi, int64_t sb, int64_t ss, int32_t gbase,
                          int32_t* gthr, int32_t plan, hipStream_t st) {
  switch (KT) {
    case 8: launch_ring<BF16, 8, FM>(p, H, cst, B, E, irb, N, w, K, os, oi, sb, ss, gbase, gthr, plan, st); break;
    case 16:
      if constexpr (BF16) return false;
      else launch_ring<BF16, 16, FM>(p, H, cst, B, E, irb, N, w, K, os, oi, sb, ss, gbase, gthr, plan, st);
      break;
    default: return false;
  }
  return true;
}

// the threshold seed's tile maxima on catalog_ring (GMAX) over the first
// seed_n items, when the main pass runs on the ring too
template <bool BF16, int KT, bool FM>
static void launch_ring_gmax(const Plan& p, const float* H, const float* cst, int64_t B,
                             const char* E, int64_t irb, const float* w, float* gm, int64_t ldg,
                             int32_t plan, hipStream_t st) {
  if (ring_waves(BF16, plan) == 8)
    hipLaunchKernelGGL((catalog_ring<BF16, KT, FM, 8, true>), dim3(p.rnqb[1] * p.sS[1]), dim3(512),
                       0, st, H, cst, B, E, irb, p.seed_n, w, 1, p.sS[1], p.stps[1], p.rnqb[1], gm,
                       nullptr, ldg, 0, 0, nullptr);
  else
    hipLaunchKernelGGL((catalog_ring<BF16, KT, FM, 4, true>), dim3(p.rnqb[0] * p.sS[0]), dim3(256),
                       0, st, H, cst, B, E, irb, p.seed_n, w, 1, p.sS[0], p.stps[0], p.rnqb[0], gm,
                       nullptr, ldg, 0, 0, nullptr);
}

template <bool BF16, bool FM>
static bool dispatch_ring_gmax(int KT, const Plan& p, const float* H, const float* cst, int64_t B,
                               const char* E, int64_t irb, const float* w, float* gm, int64_t ldg,
                               int32_t plan, hipStream_t st) {
  switch (KT) {
    case 8: launch_ring_gmax<BF16, 8, FM>(p, H, cst, B, E, irb, w, gm, ldg, plan, st); break;
    case 16:
      if constexpr (BF16) return false;
      else launch_ring_gmax<BF16, 16, FM>(p, H, cst, B, E, irb, w, gm, ldg, plan, st);
      break;
    default: return false;
  }
  return true;
}

template <bool BF16, int KPAD, bool FM>
static bool dispatch_kt(int KT, const Plan& p, const float* H, const float* cst,
                        int64_t B, const char* E, int64_t irb, int32_t N,
                        const float* w, int K, float* os, int32_t* oi, int64_t sb,
                        int64_t ss, int32_t gbase, int32_t* gthr, int32_t plan, hipStream_t st) {
  switch (KT) {
    case 1: launch_main<BF16, 1, KPAD, FM>(p, H, cst, B, E, irb, N, w, K, os, oi, sb, ss, gbase, gthr, plan, st); break;
    case 2: launch_main<BF16, 2, KPAD, FM>(p, H, cst, B, E, irb, N, w, K, os, oi, sb, ss, gbase, gthr, plan, st); break;
    case 4: launch_main<BF16, 4, KPAD, FM>(p, H, cst, B, E, irb, N, w, K, os, oi, sb, ss, gbase, gthr, plan, st); break;
    case 8: launch_main<BF16, 8, KPAD, FM>(p, H, cst, B, E, irb, N, w, K, os, oi, sb, ss, gbase, gthr, plan, st); break;
    case 16: launch_main<BF16, 16, KPAD, FM>(p, H, cst, B, E, irb, N, w, K, os, oi, sb, ss, gbase, gthr, plan, st); break;
    default: return false;
  }
  return true;
}

// small-catalog score matrix on the catalog kernel (STORE): any number of
// item tiles per split (no top-K lists to warm up), ~2,048 workgroups
template <bool BF16, int KT, bool FM>
static void launch_store(int64_t B, int nqb, int32_t N, const float* H, const float* cst,
                         const char* E, int64_t irb, const float* w, float* sc, int64_t ldsc,
                         int32_t* gthr, int32_t plan, hipStream_t st) {
  const int ntiles = (N + kTile - 1) / kTile;
  int S = (HHFM_STORE_WG + nqb - 1) / nqb;
  S = S > ntiles ? ntiles : (S < 1 ? 1 : S);
  const int tps = (ntiles + S - 1) / S;
  S = (ntiles + tps - 1) / tps;
  constexpr bool kCanSplit = BF16 || KT >= 2;
  if (kCanSplit && !(plan & HHFM_PLAN_EXACT_FP32))
    hipLaunchKernelGGL((catalog_main<BF16, KT, 32, FM, kCanSplit, true>), dim3(nqb * S),
                       dim3(256), 0, st, H, cst, B, E, irb, N, w, 1, S, tps, nqb, sc, nullptr,
                       ldsc, 0, 0, gthr);
  else
    hipLaunchKernelGGL((catalog_main<BF16, KT, 32, FM, false, true>), dim3(nqb * S),
                       dim3(256), 0, st, H, cst, B, E, irb, N, w, 1, S, tps, nqb, sc, nullptr,
                       ldsc, 0, 0, gthr);
}

// the fused small-catalog kernel (catalog_fused.h): S 8-wave workgroups per
// 32 queries, each over one range of 8 x kFusedTiles item tiles; the last to
// finish merges the S range lists
template <bool BF16, int KT, bool FM, int T>
static void launch_fused_t(int64_t B, int S, const int32_t* qidx, int ncols, int mode, int ucol,
                         int c0, int c1, int t0, int t1, const char* E, int64_t M, int64_t irb,
                         int32_t N, const float* w, int K, float* os, int32_t* oi, int32_t gbase,
                         uint32_t* arrive, uint64_t* part, int32_t plan, hipStream_t st) {
  constexpr bool kCanSplit = BF16 || KT >= 2;
  const int nqb = (int)((B + kQPerWave - 1) / kQPerWave);
  // past one workgroup per CU the split query pieces move to LDS (two
  // workgroups per CU); below it they stay in registers
  const bool ql = (int64_t)nqb * S > 256;
#define HHFM_FL(SP, QL_)                                                                       \
  hipLaunchKernelGGL((catalog_fused<BF16, KT, FM, SP, T, QL_>), dim3(nqb * S),                 \
                     dim3(kFusedWaves * 64), 0, st, qidx, B, ncols, mode, ucol, c0, c1, t0, t1, \
                     E, M, irb, N, w, K, os, oi, gbase, S, arrive, part)
  if (kCanSplit && !(plan & HHFM_PLAN_EXACT_FP32)) {
    if (ql) HHFM_FL(kCanSplit, true);
    else HHFM_FL(kCanSplit, false);
  } else {
    HHFM_FL(false, false);
  }
#undef HHFM_FL
}

template <bool BF16, int KT, bool FM>
static void launch_fused(int64_t B, int S, int T, const int32_t* qidx, int ncols, int mode,
                         int ucol, int c0, int c1, int t0, int t1, const char* E, int64_t M,
                         int64_t irb, int32_t N, const float* w, int K, float* os, int32_t* oi,
                         int32_t gbase, uint32_t* arrive, uint64_t* part, int32_t plan,
                         hipStream_t st) {
  if (T == 2)
    launch_fused_t<BF16, KT, FM, 2>(B, S, qidx, ncols, mode, ucol, c0, c1, t0, t1, E, M, irb, N,
                                    w, K, os, oi, gbase, arrive, part, plan, st);
  else
    launch_fused_t<BF16, KT, FM, kFusedTiles>(B, S, qidx, ncols, mode, ucol, c0, c1, t0, t1, E,
                                              M, irb, N, w, K, os, oi, gbase, arrive, part, plan,
                                              st);
}

template <bool BF16, bool FM>
static bool dispatch_fused(int KT, int64_t B, int S, int T, const int32_t* qidx, int ncols, int mode,
                           int ucol, int c0, int c1, int t0, int t1, const char* E, int64_t M,
                           int64_t irb, int32_t N, const float* w, int K, float* os, int32_t* oi,
                           int32_t gbase, uint32_t* arrive, uint64_t* part, int32_t plan,
                           hipStream_t st) {
#define HHFM_FUSED(KT_) \
  launch_fused<BF16, KT_, FM>(B, S, T, qidx, ncols, mode, ucol, c0, c1, t0, t1, E, M, irb, N, w, K, \
                              os, oi, gbase, arrive, part, plan, st)
  switch (KT) {
    case 1: HHFM_FUSED(1); break;
    case 2: HHFM_FUSED(2); break;
    case 4: HHFM_FUSED(4); break;
    case 8: HHFM_FUSED(8); break;
    default: return false;
  }
#undef HHFM_FUSED
  return true;
}

// threshold seed on the catalog kernel (GMAX): per query and 32-item tile
// the largest score into gm [B][ldg], ~2,048 workgroups like STORE
template <bool BF16, int KT, bool FM>
static void launch_gmax(int64_t B, int nqb, int32_t N, const float* H, const float* cst,
                        const char* E, int64_t irb, const float* w, float* gm, int64_t ldg,
                        int32_t plan, hipStream_t st) {
  const int ntiles = (N + kTile - 1) / kTile;
  int S = (HHFM_STORE_WG + nqb - 1) / nqb;
  S = S > ntiles ? ntiles : (S < 1 ? 1 : S);
  const int tps = (ntiles + S - 1) / S;
  S = (ntiles + tps - 1) / tps;
  constexpr bool kCanSplit = BF16 || KT >= 2;
  if (kCanSplit && !(plan & HHFM_PLAN_EXACT_FP32))
    hipLaunchKernelGGL((catalog_main<BF16, KT, 32, FM, kCanSplit, false, true>), dim3(nqb * S),
                       dim3(256), 0, st, H, cst, B, E, irb, N, w, 1, S, tps, nqb, gm, nullptr,
                       ldg, 0, 0, nullptr);
  else
    hipLaunchKernelGGL((catalog_main<BF16, KT, 32, FM, false, false, true>), dim3(nqb * S),
                       dim3(256), 0, st, H, cst, B, E, irb, N, w, 1, S, tps, nqb, gm, nullptr,
                       ldg, 0, 0, nullptr);
}

template <bool BF16, bool FM>
static bool dispatch_gmax(int KT, int64_t B, int nqb, int32_t N, const float* H, const float* cst,
                          const char* E, int64_t irb, const float* w, float* gm, int64_t ldg,
                          int32_t plan, hipStream_t st) {
  switch (KT) {
    case 1: launch_gmax<BF16, 1, FM>(B, nqb, N, H, cst, E, irb, w, gm, ldg, plan, st); break;
    case 2: launch_gmax<BF16, 2, FM>(B, nqb, N, H, cst, E, irb, w, gm, ldg, plan, st); break;
    case 4: launch_gmax<BF16, 4, FM>(B, nqb, N, H, cst, E, irb, w, gm, ldg, plan, st); break;
    case 8: launch_gmax<BF16, 8, FM>(B, nqb, N, H, cst, E, irb, w, gm, ldg, plan, st); break;
    case 16: launch_gmax<BF16, 16, FM>(B, nqb, N, H, cst, E, irb, w, gm, ldg, plan, st); break;
    default: return false;
  }
  return true;
}

template <bool BF16, bool FM>
static bool dispatch_store(int KT, int64_t B, int nqb, int32_t N, const float* H,
                           const float* cst, const char* E, int64_t irb, const float* w,
                           float* sc, int64_t ldsc, int32_t* gthr, int32_t plan, hipStream_t st) {
  switch (KT) {
    case 1: launch_store<BF16, 1, FM>(B, nqb, N, H, cst, E, irb, w, sc, ldsc, gthr, plan, st); break;
    case 2: launch_store<BF16, 2, FM>(B, nqb, N, H, cst, E, irb, w, sc, ldsc, gthr, plan, st); break;
    case 4: launch_store<BF16, 4, FM>(B, nqb, N, H, cst, E, irb, w, sc, ldsc, gthr, plan, st); break;
    case 8: launch_store<BF16, 8, FM>(B, nqb, N, H, cst, E, irb, w, sc, ldsc, gthr, plan, st); break;
    case 16: launch_store<BF16, 16, FM>(B, nqb, N, H, cst, E, irb, w, sc, ldsc, gthr, plan, st); break;
    default: return false;
  }
  return true;
}

static void launch_merge(const float* in_s, const int32_t* in_i, int R, int64_t B,
                         int K, int64_t stride_r, int64_t stride_b, float* os,
                         int32_t* oi, hipStream_t st) {
  int64_t blocks = (B + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (K <= 32)
    hipLaunchKernelGGL(topk_merge_kernel<32>, dim3((int)blocks), dim3(256), 0, st,
                       in_s, in_i, R, B, K, stride_r, stride_b, os, oi);
  else
    hipLaunchKernelGGL(topk_merge_kernel<64>, dim3((int)blocks), dim3(256), 0, st,
                       in_s, in_i, R, B, K, stride_r, stride_b, os, oi);
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_catalog_topk_workspace(int64_t B, int32_t item_count,
                                           int32_t k, int32_t K,
                                           size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || item_count < 1 || k < 1 || K < 1 || K > 64)
    return HHFM_EINVAL;
  // the largest plan of either table dtype
  const size_t a = make_plan(B, item_count, k, K, HHFM_PLAN_DEFAULT, false).total;
  const size_t b = make_plan(B, item_count, k, K, HHFM_PLAN_DEFAULT, true).total;
  *ws_bytes = a > b ? a : b;
  return HHFM_OK;
}

extern "C" int hhfm_catalog_topk(
    const int32_t* qidx, int64_t B, int32_t ncols, int32_t mode,
    int32_t user_col, int32_t ctx_begin, int32_t ctx_end, int32_t time_begin,
    int32_t time_end, const void* E, int64_t features_M, int32_t k,
    int32_t dtype, const float* w, int32_t item_row_begin, int32_t item_count,
    int32_t global_item_base, int32_t K, float* top_score, int32_t* top_idx,
    void* workspace, size_t ws_bytes, void* stream) {
  return hhfm_catalog_topk_ex(qidx, B, ncols, mode, user_col, ctx_begin, ctx_end, time_begin,
                              time_end, E, features_M, k, dtype, w, item_row_begin, item_count,
                              global_item_base, K, top_score, top_idx, workspace, ws_bytes,
                              HHFM_PLAN_DEFAULT, nullptr, stream);
}

extern "C" int hhfm_catalog_topk_ex(
    const int32_t* qidx, int64_t B, int32_t ncols, int32_t mode,
    int32_t user_col, int32_t ctx_begin, int32_t ctx_end, int32_t time_begin,
    int32_t time_end, const void* E, int64_t features_M, int32_t k,
    int32_t dtype, const float* w, int32_t item_row_begin, int32_t item_count,
    int32_t global_item_base, int32_t K, float* top_score, int32_t* top_idx,
    void* workspace, size_t ws_bytes, int32_t plan, int32_t* status, void* stream) {
  if (B < 0 || ncols < 1 || ncols > 64 || k < 1 || features_M < 1) return HHFM_EINVAL;
  if (plan & ~HHFM_PLAN_ALL) return HHFM_EINVAL;
  if (dtype != HHFM_F32 && dtype != HHFM_BF16) return HHFM_EINVAL;
  if (mode != HHFM_MODE_FM && mode != HHFM_MODE_HHFM) return HHFM_EINVAL;
  if (user_col < 0 || user_col >= ncols) return HHFM_EINVAL;
  if (ctx_begin > ctx_end || time_begin > time_end) return HHFM_EINVAL;
  if (ctx_end > ctx_begin && (ctx_begin < 0 || ctx_end > ncols)) return HHFM_EINVAL;
  if (time_end > time_begin && (time_begin < 0 || time_end > ncols)) return HHFM_EINVAL;
  if (item_count < 1 || item_row_begin < 0 ||
      (int64_t)item_row_begin + item_count > features_M)
    return HHFM_EINVAL;
  if (K < 1 || K > item_count) return HHFM_EINVAL;
  if (K > 64) return HHFM_EUNSUPPORTED;
  const bool bf16 = dtype == HHFM_BF16;
  const int epc2 = bf16 ? 16 : 8;  // k per 16-B chunk pair (two lane halves)
  if (k % epc2) return HHFM_EUNSUPPORTED;
  const int KT = k / epc2;
  if (KT > 16 || (KT & (KT - 1))) return HHFM_EUNSUPPORTED;
  if (B == 0) return HHFM_OK;
  if (!qidx || !E || !top_score || !top_idx) return HHFM_EINVAL;
  if ((reinterpret_cast<uintptr_t>(E) & 15) != 0) return HHFM_EUNSUPPORTED;

  const Plan p = make_plan(B, item_count, k, K, plan, bf16);
  if (!workspace || ws_bytes < p.total) return HHFM_EWORKSPACE;
  char* ws = reinterpret_cast<char*>(workspace);
  float* H = reinterpret_cast<float*>(ws + p.off_H);
  float* cst = reinterpret_cast<float*>(ws + p.off_cst);
  int32_t* gthr = reinterpret_cast<int32_t*>(ws + p.off_thr);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const char* Eb = reinterpret_cast<const char*>(E);
  {
    const int rc = launch_check_query_ids(qidx, B, ncols, user_col, ctx_begin, ctx_end,
                                          time_begin, time_end, features_M, status, st);
    if (rc != HHFM_OK) return rc;
  }

  // small catalogs: scores and top-K in one kernel launch (catalog_fused.h):
  // the default up to 8,192 items (one workgroup walks the whole catalog for
  // its 32 queries); HHFM_PLAN_STORE forces the score-matrix path,
  // HHFM_PLAN_FUSED the fused kernel up to the dense limit
  const bool fused_size = item_count <= 8192 || (plan & HHFM_PLAN_FUSED);
  if (p.dense && fused_size && K <= 32 && KT <= 8 && p.fS <= kFusedMaxS &&
      (B + kQPerWave - 1) / kQPerWave <= kFusedMaxGroups &&
      ctx_end - ctx_begin <= kFusedMaxCtx && time_end - time_begin <= kFusedMaxCtx &&
      !(plan & (HHFM_PLAN_GEMM | HHFM_PLAN_STORE))) {
    const bool fmm = mode == HHFM_MODE_FM;
    const float* wv = (fmm && w) ? w : nullptr;
    uint32_t* arrive = reinterpret_cast<uint32_t*>(ws);
    uint64_t* part = reinterpret_cast<uint64_t*>(ws + p.off_sc);
#define HHFM_FARGS KT, B, p.fS, p.fT, qidx, ncols, mode, user_col, ctx_begin, ctx_end, time_begin, \
    time_end, Eb, features_M, (int64_t)item_row_begin, item_count, wv, K, top_score, top_idx, \
    global_item_base, arrive, part, plan, st
    const bool ok = bf16 ? (fmm ? dispatch_fused<true, true>(HHFM_FARGS)
                                : dispatch_fused<true, false>(HHFM_FARGS))
                         : (fmm ? dispatch_fused<false, true>(HHFM_FARGS)
                                : dispatch_fused<false, false>(HHFM_FARGS));
#undef HHFM_FARGS
    if (ok) return (int)hipGetLastError();
  }

  {
    int64_t blocks = (p.Bpad + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    if (bf16)
      hipLaunchKernelGGL(catalog_queries<true>, dim3((int)blocks), dim3(256), 0, st,
                         qidx, B, p.Bpad, ncols, mode, user_col, ctx_begin,
                         ctx_end, time_begin, time_end, Eb, features_M, k, H, cst);
    else
      hipLaunchKernelGGL(catalog_queries<false>, dim3((int)blocks), dim3(256), 0, st,
                         qidx, B, p.Bpad, ncols, mode, user_col, ctx_begin,
                         ctx_end, time_begin, time_end, Eb, features_M, k, H, cst);
  }

  if (p.dense) {
    float* sc = reinterpret_cast<float*>(ws + p.off_sc);
    const bool one = (plan & HHFM_PLAN_ONE_WAVE) != 0;
    if (!(plan & HHFM_PLAN_GEMM)) {   // the score matrix from the catalog kernel (STORE)
      const bool fmm = mode == HHFM_MODE_FM;
      const float* wv = (fmm && w) ? w : nullptr;
      bool ok;
      if (bf16) ok = fmm ? dispatch_store<true, true>(KT, B, p.nqb, item_count, H, cst, Eb, item_row_begin, wv, sc, p.ldsc, gthr, plan, st)
                         : dispatch_store<true, false>(KT, B, p.nqb, item_count, H, cst, Eb, item_row_begin, wv, sc, p.ldsc, gthr, plan, st);
      else ok = fmm ? dispatch_store<false, true>(KT, B, p.nqb, item_count, H, cst, Eb, item_row_begin, wv, sc, p.ldsc, gthr, plan, st)
                    : dispatch_store<false, false>(KT, B, p.nqb, item_count, H, cst, Eb, item_row_begin, wv, sc, p.ldsc, gthr, plan, st);
      if (ok) {
        launch_topk_dense(sc, B, item_count, p.ldsc, K, global_item_base, top_score, top_idx, st,
                          one);
        return (int)hipGetLastError();
      }
    }
    GemmArgs g{};
    g.M = B;
    g.N = item_count;
    g.K = k;
    g.A = H;
    g.lda = k;
    g.Bt = Eb + (int64_t)item_row_begin * k * (bf16 ? 2 : 4);
    g.ldb = k;
    g.b_src_bf16 = bf16;
    const bool fmm = mode == HHFM_MODE_FM;
    g.bias = (fmm && w) ? w + item_row_begin : nullptr;   // w_item   FM.py:184
    g.rowbias = fmm ? cst : nullptr;                      // (u+f)·f  FM.py:178-183
    g.C = sc;
    g.ldc = p.ldsc;
    launch_gemm(g, false, 0, st);
    launch_topk_dense(sc, B, item_count, p.ldsc, K, global_item_base, top_score, top_idx, st, one);
    return (int)hipGetLastError();
  }

  if (!p.seed_n) {   // streaming path without a seed: the per-query threshold
    // hints start below every score (0x80808080 decodes to ~-3.4e38); the
    // seed writes every b < B, the only hints the kernels read
    const hipError_t me = hipMemsetAsync(gthr, 0x80, (size_t)p.Bpad * sizeof(int32_t), st);
    if (me != hipSuccess) return (int)me;
  }
  // (bf16 k = 256 would spill at two waves per SIMD: catalog_main keeps it)
  const bool ring = K <= 32 && p.seed_n > 0 && (bf16 ? KT == 8 : (KT == 8 || KT == 16)) &&
                    !(plan & (HHFM_PLAN_EXACT_FP32 | HHFM_PLAN_NO_RING));
  const int S_used = ring ? p.rS[ring_waves(bf16, plan) == 8 ? 1 : 0] : p.S;
  float* os;
  int32_t* oi;
  int64_t sb, ss;
  if (S_used > 1) {
    os = reinterpret_cast<float*>(ws + p.off_ps);
    oi = reinterpret_cast<int32_t*>(ws + p.off_pi);
    sb = (int64_t)S_used * K;
    ss = K;
  } else {
    os = top_score;
    oi = top_idx;
    sb = K;
    ss = 0;
  }
  const int32_t gbase = global_item_base;  // order-preserving shift
  const bool fm = mode == HHFM_MODE_FM;
  bool ok;
  if (p.seed_n) {   // threshold seed (make_plan)
    float* ssc = reinterpret_cast<float*>(ws + p.off_seed_sc);
    float* sds = reinterpret_cast<float*>(ws + p.off_seed_s);
    int32_t* sdi = reinterpret_cast<int32_t*>(ws + p.off_seed_i);
    const float* wv = (fm && w) ? w : nullptr;
    const int64_t irb = item_row_begin;
    const int32_t G = p.seed_n / kTile;   // tiles of the seed (>= 128 >= K)
    // the tile maxima on the kernel the main pass runs on (bit-identical scores)
    if (ring) {
      if (bf16) ok = fm ? dispatch_ring_gmax<true, true>(KT, p, H, cst, B, Eb, irb, wv, ssc, G, plan, st)
                        : dispatch_ring_gmax<true, false>(KT, p, H, cst, B, Eb, irb, wv, ssc, G, plan, st);
      else ok = fm ? dispatch_ring_gmax<false, true>(KT, p, H, cst, B, Eb, irb, wv, ssc, G, plan, st)
                   : dispatch_ring_gmax<false, false>(KT, p, H, cst, B, Eb, irb, wv, ssc, G, plan, st);
    } else if (bf16) {
      ok = fm ? dispatch_gmax<true, true>(KT, B, p.nqb, p.seed_n, H, cst, Eb, irb, wv, ssc, G, plan, st)
              : dispatch_gmax<true, false>(KT, B, p.nqb, p.seed_n, H, cst, Eb, irb, wv, ssc, G, plan, st);
    } else {
      ok = fm ? dispatch_gmax<false, true>(KT, B, p.nqb, p.seed_n, H, cst, Eb, irb, wv, ssc, G, plan, st)
              : dispatch_gmax<false, false>(KT, B, p.nqb, p.seed_n, H, cst, Eb, irb, wv, ssc, G, plan, st);
    }
    if (!ok) return HHFM_EUNSUPPORTED;
    // gthr[b] = key of the K-th largest tile maximum
    launch_topk_dense(ssc, B, G, G, K, 0, sds, sdi, st, false, gthr);
  }
#define HHFM_MAIN_ARGS KT, p, H, cst, B, Eb, (int64_t)item_row_begin, item_count, w, K, os, oi, sb, ss, gbase, gthr, plan, st
  if (ring) {
    if (bf16) ok = fm ? dispatch_ring<true, true>(HHFM_MAIN_ARGS) : dispatch_ring<true, false>(HHFM_MAIN_ARGS);
    else ok = fm ? dispatch_ring<false, true>(HHFM_MAIN_ARGS) : dispatch_ring<false, false>(HHFM_MAIN_ARGS);
  } else if (K <= 32) {
    if (bf16) ok = fm ? dispatch_kt<true, 32, true>(HHFM_MAIN_ARGS) : dispatch_kt<true, 32, false>(HHFM_MAIN_ARGS);
    else ok = fm ? dispatch_kt<false, 32, true>(HHFM_MAIN_ARGS) : dispatch_kt<false, 32, false>(HHFM_MAIN_ARGS);
  } else {
    if (bf16) ok = fm ? dispatch_kt<true, 64, true>(HHFM_MAIN_ARGS) : dispatch_kt<true, 64, false>(HHFM_MAIN_ARGS);
    else ok = fm ? dispatch_kt<false, 64, true>(HHFM_MAIN_ARGS) : dispatch_kt<false, 64, false>(HHFM_MAIN_ARGS);
  }
#undef HHFM_MAIN_ARGS
  if (!ok) return HHFM_EUNSUPPORTED;
  if (S_used > 1) {
    launch_merge(os, oi, S_used, B, K, /*stride_r=*/K, /*stride_b=*/(int64_t)S_used * K,
                 top_score, top_idx, st);
  }
  return (int)hipGetLastError();
}

#if HHFM_FUSED_TIMING
// diagnostic builds only: read and clear the fused kernel's per-workgroup
// phase stamps (out: kFusedTimingWG x kFusedMarks)
extern "C" int hhfm_debug_fused_timing(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fused_t), sizeof(g_fused_t)) != hipSuccess) return -1;
  return 0;
}
extern "C" int hhfm_debug_fused_timing_clear(void) {
  static unsigned long long zero[kFusedTimingWG][kFusedMarks];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fused_t), zero, sizeof(zero));
}
#endif

#if HHFM_RING_TIMING
// diagnostic builds only: read and clear the ring kernel's phase sums
extern "C" int hhfm_debug_ring_timing(unsigned long long* out) {
  hipDeviceSynchronize();
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ring_t), sizeof(g_ring_t)) != hipSuccess) return -1;
  static const unsigned long long zero[8] = {0};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ring_t), zero, sizeof(zero));
}
#endif

extern "C" int hhfm_topk_merge(const float* in_score, const int32_t* in_idx,
                               int32_t R, int64_t B, int32_t K, float* out_score,
                               int32_t* out_idx, void* stream) {
  if (R < 1 || B < 0 || K < 1) return HHFM_EINVAL;
  if (K > 64) return HHFM_EUNSUPPORTED;
  if (B == 0) return HHFM_OK;
  if (!in_score || !in_idx || !out_score || !out_idx) return HHFM_EINVAL;
  launch_merge(in_score, in_idx, R, B, K, /*stride_r=*/B * K, /*stride_b=*/K,
               out_score, out_idx, reinterpret_cast<hipStream_t>(stream));
  return (int)hipGetLastError();
}
