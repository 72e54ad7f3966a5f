// K4 — AFM (attentional FM) on gfx950, on top of the shared MFMA GEMM.
//
//   hhfm_afm_forward       replaces AFM.out  (Newcode/AFM.py:103-142)
//   hhfm_afm_catalog_topk  replaces AFM.topk (Newcode/AFM.py:209-246)
//
// A1 (per row): the attention pre-activations of all F(F-1)/2 pair products
// are one GEMM [B·P, k] x [k, A] whose A operand is formed on the fly as
// E[x_i] ⊙ E[x_j] (f32 MFMA, exact fp32) and whose epilogue applies
// relu(· + b)·p and sums over A -> one logit per pair; afm_rows_finish does
// the pair softmax, Σ att·(e_i ⊙ e_j), the projection P, Σw and w0.
// A2 (catalog): the item-side pre-activation (uf_f ⊙ item)·W equals
// item·(diag(uf_f)·W), so for every (query, field) f it is ONE GEMM
// items [N, k] x W'' [k, B·u_f·A] (W'' built per query by afm_cat_prep) with a
// grouped epilogue (relu(·+b)·p summed per A-column group) -> logits [N, B·u_f];
// afm_cat_finish forms the exp-weighted score of AFM.py:232-243 and
// hhfm_topk_dense selects.  The reference's raw exp (no max subtraction,
// AFM.py:223,230) is kept.
#include <cstdlib>

#include <atomic>

#include "gemm_mfma.h"

namespace hhfm {

static size_t a256(size_t x) { return (x + 255) & ~size_t(255); }

HHFM_DEV float tab(const void* E, int bf16, int64_t id, int k, int c) {
  return bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(E)[id * k + c])
              : reinterpret_cast<const float*>(E)[id * k + c];
}

// ---- A1 finish: wave per row --------------------------------------------------
__global__ __launch_bounds__(256) void afm_rows_finish(
    const int32_t* __restrict__ idx, int64_t B, int F, const void* __restrict__ E, int t_bf16,
    int64_t M, int k, const float* __restrict__ w, float w0, const float* __restrict__ P,
    const float* __restrict__ logit_part, int ntl, float* __restrict__ out) {
  const int l = lane_id();
  const int np = F * (F - 1) / 2;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t m = wave; m < B; m += nwave) {
    const int32_t* x = idx + m * F;
    // logits of this row's pairs: lane l holds pairs l and l + 64 (np <= 120)
    float lg0 = kNegInf, lg1 = kNegInf;
    if (l < np) {
      lg0 = 0.f;
      for (int t = 0; t < ntl; ++t) lg0 += logit_part[((m * np) + l) * ntl + t];
    }
    if (l + kWave < np) {
      lg1 = 0.f;
      for (int t = 0; t < ntl; ++t) lg1 += logit_part[((m * np) + l + kWave) * ntl + t];
    }
    float mx = fmaxf(lg0, lg1);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mx = fmaxf(mx, __shfl_xor(mx, d, kWave));
    const float e0 = l < np ? expf(lg0 - mx) : 0.f;
    const float e1 = l + kWave < np ? expf(lg1 - mx) : 0.f;
    const float s = group_sum<kWave>(e0 + e1);
    const float att0 = e0 / s, att1 = e1 / s;     // tf.nn.softmax(axis=1), AFM.py:125
    float bil = 0.f;
    // uniform loop: every lane takes part in the shuffles (att of pair p
    // lives in lane p, which may lie beyond k)
    for (int c0 = 0; c0 < k; c0 += kWave) {
      const int c = c0 + l;
      const bool in = c < k;
      float afm = 0.f;
      for (int p = 0; p < np; ++p) {
        int i, j;
        pair_ij(p, F, i, j);
        const float ap = p < kWave ? __shfl(att0, p, kWave) : __shfl(att1, p - kWave, kWave);
        if (in)
          afm += ap * (tab(E, t_bf16, clamp_id(x[i], M), k, c) *
                       tab(E, t_bf16, clamp_id(x[j], M), k, c));
      }
      if (in) bil += afm * P[c];                  // AFM·P (AFM.py:138-139)
    }
    bil = group_sum<kWave>(bil);
    if (l == 0) {
      float fb = 0.f;
      for (int f = 0; f < F; ++f) fb += w[clamp_id(x[f], M)];
      out[m] = (bil + fb) + w0;                   // add_n, AFM.py:142
    }
  }
}

// ---- A1 fused: one wave scores floor(32/np) rows per step --------------------
// Every (row, pair) "combo" of R = floor(32/np) rows is one MFMA column: the
// attention pre-activations are computed TRANSPOSED, D[unit][combo] =
// Σ_k Wᵀ[unit][k]·(e_i⊙e_j)[combo][k], with v_mfma_f32_32x32x2_f32 (exact
// fp32 products, fp32 accumulation): A = Wᵀ rows from an XOR-swizzled LDS
// image, B = the combo's pair product formed in registers from two 16-B
// gathers per 8 k.  A lane then holds one combo and 16 attention units per
// tile, so relu(·+b)·p sums in-lane; the same products dotted with P give
// s = (e_i⊙e_j)·P, and out = Σ_p softmax(logit)_p·s_p + Σw + w0 — the
// AFM.py:118-142 value with Σ_p att_p Σ_c(...) re-associated per pair.  Pair
// products, logits and attention weights never leave registers.
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kAfmMaxK = 256;
constexpr int kAfmFusedMaxF = 8;     // F(F-1)/2 <= 28 combos of one row fit 32 columns

// LDS of the fused AFM kernels is sized per call (dynamic); above the default
// 64 KB a launch must raise the kernel's limit (gfx950: 160 KB per workgroup).
static void allow_lds(const void* fn, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
static size_t afm_rows_fused_lds(int k, int A, bool split) {
  const int NA = (A + 31) / 32 * 32;
  const size_t img = split ? (size_t)NA * k * 3 / 2 : (size_t)NA * k;   // 3 bf16 pieces or fp32
  return 4 * (img + k + 2 * NA + 4 * 32 * 4);   // + 4 waves x 32 combos x float4
}

// SPLIT (k % 16 == 0): the attention GEMM on v_mfma_f32_32x32x16_bf16 with
// both fp32 operands split into three bf16 pieces (split3x8): Wᵀ once into
// three bf16 LDS images, the pair products in registers per 16 k; the six
// piece products of order >= 2^-16, 6 MFMAs per 16 k instead of 8
// 32x32x2_f32 ones (512 -> 192 cycles).  A 16-k step's lane half h holds k
// {16t+4h .. +3} and {16t+8+4h .. +3}: two of the exact kernel's 8-k steps.
// KS > 0 (SPLIT only): k = 16·KS known at compile time, so the k loop unrolls
// (no register rotation moves, constant gather offsets); KS = 0: any k.
// XOR key of Wᵀ unit row u in a [unit][U2] image of 16-B chunks that the
// MFMA loops read with ds_read_b128, lane l <-> unit 32n + (l & 31).  Each
// 16-lane b128 group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and the same
// +32) must land on 16 distinct 16-B slots of the 256-B bank row
// (MI355X_MICROARCH.md §LDS).  U2 a power of two: 16/U2 rows share a bank
// row, so the key is a row's index among those at the same slot offset,
// (u·U2/16) mod U2 (u mod 16 once U2 >= 16) — keying on u & (U2−1) instead
// left every pair of lanes j, j+8 on one slot at U2 = 8 (k = 64: 31 % of
// the A1 kernel's LDS cycles were conflicts).  Other U2: u & SW2, SW2 + 1
// the largest power of two dividing U2 (<= 16), inside the row.
HHFM_DEV int afm_img_key(int u, int U2, int SW2) {
  if ((U2 & (U2 - 1)) == 0) return U2 >= 16 ? (u & 15) : (((u * U2) >> 4) & (U2 - 1));
  return u & SW2;
}

template <bool TBF, int NT, bool SPLIT, int KS = 0>
__global__ __launch_bounds__(256, NT <= 2 ? 3 : NT == 3 ? 2 : 1) void afm_rows_fused(
    const int32_t* __restrict__ idx, int64_t B, int F, const void* __restrict__ E, int64_t M,
    int k_arg, const float* __restrict__ w, float w0, const float* __restrict__ Wt,
    const float* __restrict__ att_b, const float* __restrict__ att_p, int A,
    const float* __restrict__ P, float* __restrict__ out) {
  constexpr int NA = NT * 32;
  const int k = KS > 0 ? 16 * KS : k_arg;
  extern __shared__ __attribute__((aligned(16))) float smem[];   // afm_rows_fused_lds()
  float4* img = reinterpret_cast<float4*>(smem);
  uint4* imgb = reinterpret_cast<uint4*>(smem);   // SPLIT: 3 piece images [NA][k/8] x 16 B
  float* Pl = smem + (SPLIT ? NA * k * 3 / 2 : NA * k);
  float* bl = Pl + k;
  float* apl = bl + NA;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int j = l & 31, h = l >> 5;
  const int U = k / 4;                       // 16-B units per Wᵀ row
  int sw = 1;                                // XOR group: largest power of 2 dividing U, <= 16
  while (sw < 16 && U % (2 * sw) == 0) sw *= 2;
  const int SW = sw - 1;
  const int U2 = k / 8;                      // SPLIT: 16-B bf16 units per Wᵀ row
  int sw2 = 1;
  while (sw2 < 16 && U2 % (2 * sw2) == 0) sw2 *= 2;
  const int SW2 = sw2 - 1;
  if constexpr (SPLIT) {
    for (int x = tid; x < NA * U2; x += 256) {
      const int u = x / U2, c = x - u * U2;
      const int kb = 16 * (c >> 1) + 4 * (c & 1);
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = u < A ? Wt[(int64_t)u * k + kb + e] : 0.f;
        v[4 + e] = u < A ? Wt[(int64_t)u * k + kb + 8 + e] : 0.f;
      }
      bf16x8 q0, q1, q2;
      split3x8(v, q0, q1, q2);
      const int o = u * U2 + (c ^ afm_img_key(u, U2, SW2));
      imgb[o] = __builtin_bit_cast(uint4, q0);
      imgb[NA * U2 + o] = __builtin_bit_cast(uint4, q1);
      imgb[2 * NA * U2 + o] = __builtin_bit_cast(uint4, q2);
    }
  } else {
    for (int x = tid; x < NA * U; x += 256) {
      const int u = x / U, c = x - u * U;
      const float4 v = u < A ? *reinterpret_cast<const float4*>(Wt + (int64_t)u * k + 4 * c)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
      img[u * U + (c ^ (u & SW))] = v;
    }
  }
  for (int x = tid; x < k; x += 256) Pl[x] = P[x];
  for (int x = tid; x < NA; x += 256) {
    bl[x] = x < A ? att_b[x] : 0.f;
    apl[x] = x < A ? att_p[x] : 0.f;
  }
  __syncthreads();

  const int np = F * (F - 1) / 2, R = 32 / np;
  const int r = j / np, p = j - r * np;
  int pi, pj;
  pair_ij(p, F, pi, pj);                     // (only read when this lane's combo is live)
  const bool live = r < R;
  const int64_t nblk = (B + R - 1) / R;
  const int64_t wstride = (int64_t)gridDim.x * 4;
  const int KQ = k / 8;
  // the lane combo's two table rows in block blk
  auto ids_of = [&](int64_t blk, int64_t& ia, int64_t& ib) {
    const int64_t row = blk * R + r;
    const int64_t rr = (live && row < B) ? row : 0;
    ia = clamp_id(idx[rr * F + (live ? pi : 0)], M);
    ib = clamp_id(idx[rr * F + (live ? pj : 1)], M);
  };
  // this lane's 4 k of 8-k step t, one step of gathers in flight ahead
  auto gather = [&](int64_t ia, int64_t ib, int t, float4& x, float4& y) {
    const int c0 = 8 * t + 4 * h;
    if constexpr (TBF) {
      const uint2 u = *reinterpret_cast<const uint2*>(
          reinterpret_cast<const uint16_t*>(E) + ia * k + c0);
      const uint2 v = *reinterpret_cast<const uint2*>(
          reinterpret_cast<const uint16_t*>(E) + ib * k + c0);
      x = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                      __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      y = make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                      __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u));
    } else {
      x = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(E) + ia * k + c0);
      y = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(E) + ib * k + c0);
    }
  };
  // The next block's ids are read at the start of this block and its first
  // step is gathered during this block's last one: the idx -> row dependent
  // chain never stalls a block start.
  int64_t blk = (int64_t)blockIdx.x * 4 + wv;
  int64_t ia = 0, ib = 0;
  float4 xa = make_float4(0.f, 0.f, 0.f, 0.f), ya = xa, xb = xa, yb = xa;
  if (blk < nblk) {
    ids_of(blk, ia, ib);
    gather(ia, ib, 0, xa, ya);
    if constexpr (SPLIT) gather(ia, ib, 1, xb, yb);
  }
  for (; blk < nblk; blk += wstride) {
    const int64_t row = blk * R + r;
    const bool ok = live && row < B;
    const bool has_next = blk + wstride < nblk;
    int64_t na = 0, nb = 0;
    if (has_next) ids_of(blk + wstride, na, nb);
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int x = 0; x < 16; ++x) acc[n][x] = 0.f;
    float sP = 0.f;
    // Σw of the row: lanes p < F of the row's group fetch one field each
    const float wf = (ok && p < F) ? w[clamp_id(idx[row * F + p], M)] : 0.f;
    if constexpr (SPLIT) {
      auto step2 = [&](int t2) {
        // steps 2t2, 2t2+1 are in (xa, ya), (xb, yb); fetch the next pair
        float4 xn = xa, yn = ya, xm = xb, ym = yb;
        if (2 * t2 + 2 < KQ) {
          gather(ia, ib, 2 * t2 + 2, xn, yn);
          gather(ia, ib, 2 * t2 + 3, xm, ym);
        } else if (has_next) {
          gather(na, nb, 0, xn, yn);
          gather(na, nb, 1, xm, ym);
        }
        const int c0 = 16 * t2 + 4 * h;
        const float ea[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
        const float eb[8] = {ya.x, ya.y, ya.z, ya.w, yb.x, yb.y, yb.z, yb.w};
        float pe[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          pe[e] = ea[e] * eb[e];
          sP = fmaf(pe[e], Pl[c0 + (e < 4 ? e : e + 4)], sP);
        }
        bf16x8 b0, b1, b2;                   // bf16 table: two pieces (split2x8)
        if constexpr (TBF)
          split2x8(pe, b0, b1);
        else
          split3x8(pe, b0, b1, b2);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int u = 32 * n + j;          // A-operand row = attention unit
          const int o = u * U2 + ((2 * t2 + h) ^ afm_img_key(u, U2, SW2));
          const bf16x8 a0 = __builtin_bit_cast(bf16x8, imgb[o]);
          const bf16x8 a1 = __builtin_bit_cast(bf16x8, imgb[NA * U2 + o]);
          const bf16x8 a2 = __builtin_bit_cast(bf16x8, imgb[2 * NA * U2 + o]);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[n], 0, 0, 0);
          if constexpr (!TBF)
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[n], 0, 0, 0);
        }
        xa = xn;
        ya = yn;
        xb = xm;
        yb = ym;
      };
      if constexpr (KS > 0) {
#pragma unroll
        for (int t2 = 0; t2 < KS; ++t2) step2(t2);
      } else {
        for (int t2 = 0; t2 < KQ / 2; ++t2) step2(t2);
      }
    } else
    for (int t = 0; t < KQ; ++t) {
      float4 xn = xa, yn = ya;
      if (t + 1 < KQ) gather(ia, ib, t + 1, xn, yn);
      else if (has_next) gather(na, nb, 0, xn, yn);
      const int c0 = 8 * t + 4 * h;
      const float ea[4] = {xa.x, xa.y, xa.z, xa.w}, eb[4] = {ya.x, ya.y, ya.z, ya.w};
      float pe[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pe[e] = ea[e] * eb[e];
        sP = fmaf(pe[e], Pl[c0 + e], sP);
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int u = 32 * n + j;            // A-operand row = attention unit
        const float4 wa = img[u * U + ((2 * t + h) ^ (u & SW))];
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.x, pe[0], acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.y, pe[1], acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.z, pe[2], acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.w, pe[3], acc[n], 0, 0, 0);
      }
      xa = xn;
      ya = yn;
    }
    ia = na;
    ib = nb;
    // logit of this lane's combo: Σ_units p·relu(acc + b)  (AFM.py:112-117)
    float lg = 0.f;
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int u = 32 * n + 8 * g4 + 4 * h;
        const float4 bq = *reinterpret_cast<const float4*>(bl + u);
        const float4 pq = *reinterpret_cast<const float4*>(apl + u);
        lg = fmaf(fmaxf(acc[n][4 * g4 + 0] + bq.x, 0.f), pq.x, lg);
        lg = fmaf(fmaxf(acc[n][4 * g4 + 1] + bq.y, 0.f), pq.y, lg);
        lg = fmaf(fmaxf(acc[n][4 * g4 + 2] + bq.z, 0.f), pq.z, lg);
        lg = fmaf(fmaxf(acc[n][4 * g4 + 3] + bq.w, 0.f), pq.w, lg);
      }
    lg += __shfl_xor(lg, 32, kWave);
    sP += __shfl_xor(sP, 32, kWave);
    // softmax over the row's np pairs (tf.nn.softmax, AFM.py:125) and the
    // attention-weighted sum of the pair scores, by the row's first lane from
    // the combos' (logit, pair score, Σw share) parked in LDS — independent
    // reads instead of a serial chain of cross-lane shuffles.  (One wave's LDS
    // accesses complete in order, so no barrier.)
    float4* ep = reinterpret_cast<float4*>(apl + NA) + 32 * wv;
    if (h == 0) ep[j] = make_float4(lg, sP, wf, 0.f);
    // every combo's lane takes its own exp (the row's max read back from the
    // parked logits) — one lane per row taking all np exps in turn was 15 % of
    // the kernel — then the row's first lane sums in the reference's order
    if (h == 0 && live) {
      const float4* e = ep + r * np;
      float mx = kNegInf;
      for (int q = 0; q < np; ++q) mx = fmaxf(mx, e[q].x);
      ep[j].w = expf(lg - mx);
    }
    if (ok && p == 0 && h == 0) {
      const float4* e = ep + r * np;
      float se = 0.f, num = 0.f;
      for (int q = 0; q < np; ++q) {
        const float4 eq = e[q];
        se += eq.w;
        num = fmaf(eq.w, eq.y, num);
      }
      float fb = 0.f;
      if (np >= F) {   // the row's lanes fetched one field each
        for (int f = 0; f < F; ++f) fb += e[f].z;
      } else {         // F = 2: one lane per row
        for (int f = 0; f < F; ++f) fb += w[clamp_id(idx[row * F + f], M)];
      }
      out[row] = (num / se + fb) + w0;   // add_n, AFM.py:142
    }
  }
}

// ---- A1 pair-major: one wave = 32 rows, one MFMA tile column per row ---------
// The transposed pre-activations D[unit][row] = Σ_k Wᵀ[unit][k]·(e_i⊙e_j)[row][k]
// are computed for ONE pair (i, j) of 32 rows at a time (split-bf16 MFMA as
// afm_rows_fused: Wᵀ as three bf16 LDS images, the pair product split in
// registers per 16 k, the six piece products of order >= 2^-16), so lane j
// (both halves) ends up holding row j's logit of that pair: relu(· + b)·p
// summed over its 16 units per tile and the two lane halves, the bias the
// accumulators' initial value.  The row's pair logits and pair scores
// s = (e_i⊙e_j)·P are parked in a lane-private LDS slot per pair, and the
// pair softmax (tf.nn.softmax, AFM.py:125) + Σ_p att_p·s_p runs in-lane for
// the 32 rows at once — no per-row serial epilogue, all 32 columns live
// (afm_rows_fused packs floor(32/np) rows of np pairs: 30 of 32 at F = 5,
// and its softmax runs one lane per row).  F <= 8.
// One 16-k step of gathers in flight at three workgroups per CU: against a
// whole pair's gathers in flight at two, 0.556-0.572 vs 0.638-0.654 ms (bf16
// table) and 0.619-0.634 vs 0.638-0.642 (fp32) per 1 M Frappe rows
// (profiles/r04_afm_pairs_pf_occ_ab.txt; four per CU: 0.68 / 0.70 ms).

// LDS: the three Wᵀ piece images, P, b, p, then per wave the rows' ids
// [F][32] and the pair slots [np][32] (sized per call: F = 5 needs 40 KB at
// k = A = 64, so four workgroups fit a CU)
static size_t afm_rows_pairs_lds(int NA, int K, int F) {
  const int np = F * (F - 1) / 2;
  return (size_t)3 * NA * K * 2 + 4 * (K + 2 * NA) + (size_t)4 * F * 32 * 4 +
         (size_t)4 * np * 32 * 8;
}

template <bool TBF, int NT, int KS>
__global__ __launch_bounds__(256, 3) void afm_rows_pairs(
    const int32_t* __restrict__ idx, int64_t B, int F, const void* __restrict__ E, int64_t M,
    const float* __restrict__ w, float w0, const float* __restrict__ Wt,
    const float* __restrict__ att_b, const float* __restrict__ att_p, int A,
    const float* __restrict__ P, float* __restrict__ out) {
  constexpr int NA = NT * 32, K = 16 * KS, U2 = K / 8;
  constexpr int SW2 = ((U2 & -U2) < 16 ? (U2 & -U2) : 16) - 1;   // largest pow2 | U2, <= 16
  extern __shared__ __attribute__((aligned(16))) float smem[];   // afm_rows_pairs_lds()
  uint4* imgb = reinterpret_cast<uint4*>(smem);                   // [piece][unit][chunk]
  float* Pl = smem + 3 * NA * U2 * 4;
  float* bl = Pl + K;
  float* apl = bl + NA;
  int32_t* idl = reinterpret_cast<int32_t*>(apl + NA);            // [wave][f][32]
  float2* slots = reinterpret_cast<float2*>(idl + 4 * F * 32);     // [wave][pair][32]
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int j = l & 31, h = l >> 5;
  for (int x = tid; x < NA * U2; x += 256) {
    const int u = x / U2, c = x - u * U2;
    const int kb = 16 * (c >> 1) + 4 * (c & 1);
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = u < A ? Wt[(int64_t)u * K + kb + e] : 0.f;
      v[4 + e] = u < A ? Wt[(int64_t)u * K + kb + 8 + e] : 0.f;
    }
    bf16x8 q0, q1, q2;
    split3x8(v, q0, q1, q2);
    const int o = u * U2 + (c ^ afm_img_key(u, U2, SW2));
    imgb[o] = __builtin_bit_cast(uint4, q0);
    imgb[NA * U2 + o] = __builtin_bit_cast(uint4, q1);
    imgb[2 * NA * U2 + o] = __builtin_bit_cast(uint4, q2);
  }
  for (int x = tid; x < K; x += 256) Pl[x] = P[x];
  for (int x = tid; x < NA; x += 256) {
    bl[x] = x < A ? att_b[x] : 0.f;
    apl[x] = x < A ? att_p[x] : 0.f;
  }
  __syncthreads();

  const int np = F * (F - 1) / 2;
  float2* sl = slots + wv * np * 32;
  int32_t* il = idl + wv * F * 32;
  const int64_t nblk = (B + 31) / 32;
  for (int64_t blk = (int64_t)blockIdx.x * 4 + wv; blk < nblk; blk += (int64_t)gridDim.x * 4) {
    const int64_t row = blk * 32 + j;
    const bool ok = row < B;
    const int64_t rr = ok ? row : B - 1;
    float fb = 0.f;
    if (h == 0)
      for (int f = 0; f < F; ++f) {
        const int32_t id = clamp_id(idx[rr * F + f], M);
        il[f * 32 + j] = id;
        fb += w[id];                                  // Σ_f w[x_f]   AFM.py:140
      }
    // (one wave's LDS accesses complete in order: the ids are read back below)
    // this lane's 8 k of 16-k step t of table row `id`: {16t + 4h .. +3, 16t + 8 + 4h .. +3}
    auto gather = [&](int32_t id, int t, float (&x)[8]) {
      const int c0 = 16 * t + 4 * h;
      if constexpr (TBF) {
        const uint16_t* r = reinterpret_cast<const uint16_t*>(E) + (int64_t)id * K + c0;
        const uint2 lo = *reinterpret_cast<const uint2*>(r), hi = *reinterpret_cast<const uint2*>(r + 8);
        const uint32_t u4[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[2 * e] = __uint_as_float(u4[e] << 16);
          x[2 * e + 1] = __uint_as_float(u4[e] & 0xffff0000u);
        }
      } else {
        const float* r = reinterpret_cast<const float*>(E) + (int64_t)id * K + c0;
        const float4 lo = *reinterpret_cast<const float4*>(r), hi = *reinterpret_cast<const float4*>(r + 8);
        x[0] = lo.x; x[1] = lo.y; x[2] = lo.z; x[3] = lo.w;
        x[4] = hi.x; x[5] = hi.y; x[6] = hi.z; x[7] = hi.w;
      }
    };
    int pi = 0, pj = 1;
    int32_t ia = il[j], ib = il[32 + j];
    // pairs run i-major, (i, i+1) .. (i, F−1): row i's k slice is gathered
    // once per run (all KS steps held), row j's one 16-k step ahead
    // (row i held across its run: 0.627 -> 0.548 ms per 1 M rows, fp32 table;
    // row j two steps ahead, or two workgroups per CU: slower,
    // profiles/r04_afm_xrun_ab.txt, r04_afm_ypf_occ_ab.txt)
    float xh[KS][8], ya[1][8];
#pragma unroll
    for (int t = 0; t < KS; ++t) gather(ia, t, xh[t]);
    gather(ib, 0, ya[0]);
    for (int p = 0; p < np; ++p) {
      // the next pair's rows (read now, gathered during this pair's MFMAs)
      int ni = pi, nj = pj + 1;
      if (nj == F) {
        ++ni;
        nj = ni + 1;
      }
      const bool more = p + 1 < np;
      int32_t na = 0, nb = 0;
      if (more) {
        na = il[ni * 32 + j];
        nb = il[nj * 32 + j];
      }
      // the accumulators' initial value: unit 32n + 8g4 + 4h + e's bias
      f32x16 acc[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 b4 = *reinterpret_cast<const float4*>(bl + 32 * n + 8 * g4 + 4 * h);
          acc[n][4 * g4 + 0] = b4.x;
          acc[n][4 * g4 + 1] = b4.y;
          acc[n][4 * g4 + 2] = b4.z;
          acc[n][4 * g4 + 3] = b4.w;
        }
      float sP = 0.f;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        float pe[8];
        const int c0 = 16 * t + 4 * h;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          pe[e] = xh[t][e] * ya[0][e];
          sP = fmaf(pe[e], Pl[c0 + (e < 4 ? e : e + 4)], sP);
        }
        if (t + 1 < KS)                               // the next step of row j
          gather(ib, t + 1, ya[0]);
        else if (more)                                // the next pair's first step
          gather(nb, 0, ya[0]);
        if (more && ni != pi) gather(na, t, xh[t]);   // a new run: step t of row i
        // bf16 table: the pair product has <= 16 significant bits, two pieces
        // (the third is +0, its MFMA skipped: the same sums)
        bf16x8 b0, b1, b2;
        if constexpr (TBF)
          split2x8(pe, b0, b1);
        else
          split3x8(pe, b0, b1, b2);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int u = 32 * n + j;                   // A-operand row = attention unit
          const int o = u * U2 + ((2 * t + h) ^ afm_img_key(u, U2, SW2));
          const bf16x8 a0 = __builtin_bit_cast(bf16x8, imgb[o]);
          const bf16x8 a1 = __builtin_bit_cast(bf16x8, imgb[NA * U2 + o]);
          const bf16x8 a2 = __builtin_bit_cast(bf16x8, imgb[2 * NA * U2 + o]);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[n], 0, 0, 0);
          if constexpr (!TBF)
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[n], 0, 0, 0);
        }
      }
      // the row's logit of this pair: Σ_units p·relu(acc)  (AFM.py:112-117)
      float lg = 0.f;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 pq = *reinterpret_cast<const float4*>(apl + 32 * n + 8 * g4 + 4 * h);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 0], 0.f), pq.x, lg);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 1], 0.f), pq.y, lg);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 2], 0.f), pq.z, lg);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 3], 0.f), pq.w, lg);
        }
      lg += __shfl_xor(lg, 32, kWave);
      sP += __shfl_xor(sP, 32, kWave);
      if (h == 0) sl[p * 32 + j] = make_float2(lg, sP);
      pi = ni;
      pj = nj;
      ia = na;
      ib = nb;
    }
    // softmax over the row's pairs + Σ_p att_p·s_p, in-lane (lane j = row j)
    if (h == 0 && ok) {
      float mx = kNegInf;
      for (int p = 0; p < np; ++p) mx = fmaxf(mx, sl[p * 32 + j].x);
      float se = 0.f, num = 0.f;
      for (int p = 0; p < np; ++p) {
        const float2 q = sl[p * 32 + j];
        const float e = expf(q.x - mx);
        se += e;
        num = fmaf(e, q.y, num);
      }
      out[row] = (num / se + fb) + w0;                // add_n, AFM.py:142
    }
  }
}

// ---- A2 prep: one 64-thread block per query ------------------------------------
// uf = [E[q0], E[q2], ..., E[q_{F-1}]] (u_f = F-1 fields, AFM.py:210-212)
constexpr int kAfmMaxUF = 15;

__global__ __launch_bounds__(64) void afm_cat_prep(
    const int32_t* __restrict__ q, int64_t B, int F, const void* __restrict__ E, int t_bf16,
    int64_t M, int k, const float* __restrict__ Wt, const float* __restrict__ ab,
    const float* __restrict__ ap, int A, const float* __restrict__ P,
    float* __restrict__ W2, float* __restrict__ D, float* __restrict__ ufdot,
    float* __restrict__ suma, int emit_w2) {
  __shared__ float uf[kAfmMaxUF][kAfmMaxK];
  __shared__ float pr[kAfmMaxK];
  const int l = threadIdx.x;
  const int uF = F - 1;
  const int64_t b = blockIdx.x;
  if (b >= B) return;
  const int32_t* x = q + b * F;
  for (int f = 0; f < uF; ++f) {
    const int col = f == 0 ? 0 : f + 1;
    const int64_t id = clamp_id(x[col], M);
    for (int c = l; c < k; c += 64) uf[f][c] = tab(E, t_bf16, id, k, c);
  }
  __syncthreads();
  float uw[kAfmMaxK / 64];
#pragma unroll
  for (int r = 0; r < kAfmMaxK / 64; ++r) uw[r] = 0.f;
  float sa = 0.f;
  for (int i = 0; i < uF; ++i)
    for (int j = i + 1; j < uF; ++j) {
      for (int c = l; c < k; c += 64) pr[c] = uf[i][c] * uf[j][c];
      __syncthreads();
      float lg = 0.f;
      for (int a = l; a < A; a += 64) {
        float acc = 0.f;
        for (int c = 0; c < k; ++c) acc += pr[c] * Wt[(int64_t)a * k + c];
        lg += ap[a] * fmaxf(acc + ab[a], 0.f);
      }
      lg = group_sum<kWave>(lg);
      const float aij = expf(lg);                 // raw exp, AFM.py:223
      sa += aij;
#pragma unroll
      for (int r = 0; r < kAfmMaxK / 64; ++r) {
        const int c = l + 64 * r;
        if (c < k) uw[r] += aij * pr[c];           // UFwise, AFM.py:232
      }
      __syncthreads();
    }
  float ud = 0.f;
#pragma unroll
  for (int r = 0; r < kAfmMaxK / 64; ++r) {
    const int c = l + 64 * r;
    if (c < k) ud += P[c] * uw[r];
  }
  ud = group_sum<kWave>(ud);
  if (l == 0) {
    ufdot[b] = ud;
    suma[b] = sa;
  }
  // W''[(b*uF+f)*A + a][c] = uf_f[c] * W[c][a];  D[b*uF+f][c] = P[c]*uf_f[c]
  if (!emit_w2) return;
  for (int f = 0; f < uF; ++f) {
    for (int a = 0; a < A; ++a) {
      float* dst = W2 + ((b * uF + f) * (int64_t)A + a) * k;
      for (int c = l; c < k; c += 64) dst[c] = uf[f][c] * Wt[(int64_t)a * k + c];
    }
    for (int c = l; c < k; c += 64) D[(b * uF + f) * (int64_t)k + c] = P[c] * uf[f][c];
  }
}

// The fused paths need only ufdot / suma: the same sums as afm_cat_prep, 4
// waves per query, Wᵀ transposed into LDS once ([c][a]: lane a reads
// consecutive words), the query pairs spread over the waves, each pair's
// logits summed over c in afm_cat_prep's order; the per-wave Σ aij and
// aij·pr terms are added in pair order by wave 0 (the same order as the
// single-wave loop).
constexpr int kAfmQsMaxPairs = 28;   // uF <= 8
__global__ __launch_bounds__(256) void afm_cat_qside(
    const int32_t* __restrict__ q, int64_t B, int F, const void* __restrict__ E, int t_bf16,
    int64_t M, int k, const float* __restrict__ Wt, const float* __restrict__ ab,
    const float* __restrict__ ap, int A, const float* __restrict__ P,
    float* __restrict__ ufdot, float* __restrict__ suma) {
  extern __shared__ __attribute__((aligned(16))) float qs[];   // afm_cat_qside_lds()
  const int NA = (A + 63) / 64 * 64;
  float* wt = qs;                        // [k][NA]
  float* uf = wt + k * NA;               // [uF][k]
  float* aij = uf + (F - 1) * k;         // [pairs]
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int uF = F - 1, np = uF * (uF - 1) / 2;
  const int64_t b = blockIdx.x;
  const int32_t* x = q + b * F;
  for (int i = tid; i < uF * k; i += 256) {
    const int f = i / k, c = i - f * k;
    uf[i] = tab(E, t_bf16, clamp_id(x[f == 0 ? 0 : f + 1], M), k, c);
  }
  for (int i = tid; i < k * NA; i += 256) {
    const int a = i / k, c = i - a * k;   // coalesced read of Wt[a][c]
    wt[c * NA + a] = a < A ? Wt[(int64_t)a * k + c] : 0.f;
  }
  __syncthreads();
  for (int pidx = wv; pidx < np; pidx += 4) {
    int i = 0, rem = pidx;
    while (rem >= uF - 1 - i) { rem -= uF - 1 - i; ++i; }
    const int j = i + 1 + rem;
    const float* ui = uf + i * k;
    const float* uj = uf + j * k;
    float lg = 0.f;
    for (int a = l; a < A; a += 64) {
      float acc = 0.f;
      for (int c = 0; c < k; ++c) acc += (ui[c] * uj[c]) * wt[c * NA + a];
      lg += ap[a] * fmaxf(acc + ab[a], 0.f);
    }
    lg = group_sum<kWave>(lg);
    if (l == 0) aij[pidx] = expf(lg);     // raw exp, AFM.py:223
  }
  __syncthreads();
  if (wv == 0) {
    float uw[kAfmMaxK / 64];
#pragma unroll
    for (int r = 0; r < kAfmMaxK / 64; ++r) uw[r] = 0.f;
    float sa = 0.f;
    for (int pidx = 0, i = 0; i < uF; ++i)
      for (int j = i + 1; j < uF; ++j, ++pidx) {
        const float a = aij[pidx];
        sa += a;
#pragma unroll
        for (int r = 0; r < kAfmMaxK / 64; ++r) {
          const int c = l + 64 * r;
          if (c < k) uw[r] += a * (uf[i * k + c] * uf[j * k + c]);   // UFwise, AFM.py:232
        }
      }
    float ud = 0.f;
#pragma unroll
    for (int r = 0; r < kAfmMaxK / 64; ++r) {
      const int c = l + 64 * r;
      if (c < k) ud += P[c] * uw[r];
    }
    ud = group_sum<kWave>(ud);
    if (l == 0) {
      ufdot[b] = ud;
      suma[b] = sa;
    }
  }
}

static size_t afm_cat_qside_lds(int F, int k, int A) {
  const int NA = (A + 63) / 64 * 64;
  return 4 * ((size_t)k * NA + (size_t)(F - 1) * k + kAfmQsMaxPairs);
}

// ---- A2 finish: wave per (query, 64-item block), lane = item -------------------
__global__ __launch_bounds__(256) void afm_cat_finish(
    int64_t nq, int uF, int A, int G, const float* __restrict__ part, int64_t ldp,
    const float* __restrict__ D, const float* __restrict__ ufdot, const float* __restrict__ suma,
    const void* __restrict__ E, int t_bf16, int k, int64_t item_row_begin, int32_t N,
    const float* __restrict__ w, float* __restrict__ scores) {
  const int l = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nblk = (N + kWave - 1) / kWave;
  if (wave >= nq * nblk) return;
  const int64_t b = wave / nblk;
  const int32_t i = (int32_t)((wave - b * nblk) * kWave + l);
  if (i >= N) return;
  const int gpa = A / G;
  const int64_t id = item_row_begin + i;
  float num = ufdot[b], den = suma[b];
  float extra_num = 0.f, extra_den = 0.f;
  for (int f = 0; f < uF; ++f) {
    float lg = 0.f;
    for (int t = 0; t < gpa; ++t) lg += part[(int64_t)i * ldp + (b * uF + f) * gpa + t];
    const float a = expf(lg);                      // raw exp, AFM.py:230
    const float* d = D + (b * uF + f) * (int64_t)k;
    float dot = 0.f;
    for (int c = 0; c < k; ++c) dot += d[c] * tab(E, t_bf16, id, k, c);
    extra_num += a * dot;
    extra_den += a;
  }
  num += extra_num;
  den += extra_den;
  scores[b * N + i] = num / den + w[id];           // score3 + bias, AFM.py:239-243
}

// ---- A2 fused: wave = one query x 32-item tiles, lane column = item ----------
// The item-side logit of (query, item, field f) is Σ_a p_a·relu((uf_f ⊙ item)·W
// + b)_a (AFM.py:227-230): the A1 kernel's transposed product with the pair
// product uf_f ⊙ item formed in registers (uf_f broadcast from LDS, the item
// row streamed from HBM one 8-k step ahead), the shared Wᵀ image as the A
// operand.  Per field the lane also forms P·(uf_f ⊙ item); the score
// (P·ufw + Σ_f e^lg_f P·(uf_f ⊙ item)) / (Σa_uf + Σ_f e^lg_f) + w_item
// (AFM.py:232-243) is written once per (query, item) for hhfm_topk_dense.
constexpr int kAfmCatFusedMaxUF = 7;

// SPLIT (k % 16 == 0): as afm_rows_fused — Wᵀ as three bf16 LDS images, the
// pair product uf_f ⊙ item split in registers per 16 k, 6 bf16 MFMAs per
// 16 k instead of 8 fp32 ones.
template <bool TBF, int NT, bool SPLIT>
__global__ __launch_bounds__(256) void afm_cat_fused(
    const int32_t* __restrict__ q, int64_t nq, int F, const void* __restrict__ E, int64_t M,
    int k, const float* __restrict__ Wt, const float* __restrict__ att_b,
    const float* __restrict__ att_p, int A, const float* __restrict__ P,
    const float* __restrict__ ufdot, const float* __restrict__ suma, int64_t item_row_begin,
    int32_t N, int tiles_per_block, int nchunk, const float* __restrict__ w,
    float* __restrict__ scores) {
  constexpr int NA = NT * 32;
  extern __shared__ __attribute__((aligned(16))) float smem[];   // afm_cat_fused_lds()
  float4* img = reinterpret_cast<float4*>(smem);
  uint4* imgb = reinterpret_cast<uint4*>(smem);   // SPLIT: 3 piece images [NA][k/8] x 16 B
  float* Pl = smem + (SPLIT ? NA * k * 3 / 2 : NA * k);
  float* bl = Pl + kAfmMaxK;
  float* apl = bl + NA;
  float* ufl = apl + NA;                     // [4 waves][uF][k]
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int j = l & 31, h = l >> 5;
  const int uF = F - 1;
  const int U = k / 4;
  int sw = 1;
  while (sw < 16 && U % (2 * sw) == 0) sw *= 2;
  const int SW = sw - 1;
  const int64_t qg = blockIdx.x / nchunk;
  const int chunk = (int)(blockIdx.x - qg * nchunk);
  const int U2 = k / 8;
  int sw2 = 1;
  while (sw2 < 16 && U2 % (2 * sw2) == 0) sw2 *= 2;
  const int SW2 = sw2 - 1;
  if constexpr (SPLIT) {
    for (int x = tid; x < NA * U2; x += 256) {
      const int u = x / U2, c = x - u * U2;
      const int kb = 16 * (c >> 1) + 4 * (c & 1);
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = u < A ? Wt[(int64_t)u * k + kb + e] : 0.f;
        v[4 + e] = u < A ? Wt[(int64_t)u * k + kb + 8 + e] : 0.f;
      }
      bf16x8 q0, q1, q2;
      split3x8(v, q0, q1, q2);
      const int o = u * U2 + (c ^ afm_img_key(u, U2, SW2));
      imgb[o] = __builtin_bit_cast(uint4, q0);
      imgb[NA * U2 + o] = __builtin_bit_cast(uint4, q1);
      imgb[2 * NA * U2 + o] = __builtin_bit_cast(uint4, q2);
    }
  } else {
    for (int x = tid; x < NA * U; x += 256) {
      const int u = x / U, c = x - u * U;
      const float4 v = u < A ? *reinterpret_cast<const float4*>(Wt + (int64_t)u * k + 4 * c)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
      img[u * U + (c ^ (u & SW))] = v;
    }
  }
  for (int x = tid; x < k; x += 256) Pl[x] = P[x];
  for (int x = tid; x < NA; x += 256) {
    bl[x] = x < A ? att_b[x] : 0.f;
    apl[x] = x < A ? att_p[x] : 0.f;
  }
  // uf of the 4 queries: [E[q0], E[q2], ..., E[q_{F-1}]]  (AFM.py:210-212)
  for (int x = tid; x < 4 * uF * k; x += 256) {
    const int qq = x / (uF * k), r = x - qq * uF * k, f = r / k, c = r - f * k;
    const int64_t b = qg * 4 + qq;
    float v = 0.f;
    if (b < nq) v = tab(E, TBF, clamp_id(q[b * F + (f == 0 ? 0 : f + 1)], M), k, c);
    ufl[x] = v;
  }
  __syncthreads();

  const int64_t b = qg * 4 + wv;
  if (b >= nq) return;
  const float* uq = ufl + wv * uF * k;
  const float ud = ufdot[b], sa = suma[b];
  const int KQ = k / 8;
  const int S = uF * KQ;
  const int ntile = (N + 31) / 32;
  const int t0 = chunk * tiles_per_block;
  const int t1 = min(t0 + tiles_per_block, ntile);
  for (int tile = t0; tile < t1; ++tile) {
    const int32_t item = tile * 32 + j;
    const bool ok = item < N;
    const int64_t id = item_row_begin + (ok ? item : 0);
    auto gather = [&](int t) -> float4 {
      const int c0 = 8 * t + 4 * h;
      if constexpr (TBF) {
        const uint2 u = *reinterpret_cast<const uint2*>(
            reinterpret_cast<const uint16_t*>(E) + id * k + c0);
        return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                           __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      } else {
        return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(E) + id * k + c0);
      }
    };
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int x = 0; x < 16; ++x) acc[n][x] = 0.f;
    float sP = 0.f, num = 0.f, den = 0.f;
    float4 xa = gather(0);
    // field f done: its logit from the accumulators, raw exp (AFM.py:230)
    auto finish_field = [&]() {
      float lg = 0.f;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int u = 32 * n + 8 * g4 + 4 * h;
          const float4 bq = *reinterpret_cast<const float4*>(bl + u);
          const float4 pq = *reinterpret_cast<const float4*>(apl + u);
          const float bv[4] = {bq.x, bq.y, bq.z, bq.w}, pv[4] = {pq.x, pq.y, pq.z, pq.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            lg = fmaf(fmaxf(acc[n][4 * g4 + e] + bv[e], 0.f), pv[e], lg);
            acc[n][4 * g4 + e] = 0.f;
          }
        }
      lg += __shfl_xor(lg, 32, kWave);
      sP += __shfl_xor(sP, 32, kWave);
      const float a = expf(lg);
      num = fmaf(a, sP, num);
      den += a;
      sP = 0.f;
    };
    if constexpr (SPLIT) {
      float4 xb = gather(1);
      const int K2 = KQ / 2;
      for (int s = 0, f = 0, t2 = 0; s < uF * K2; ++s) {
        // the item's steps 2t2, 2t2+1 are in xa, xb; fetch the next pair
        // (the item row again from step 0 when the field wraps)
        const bool last = s + 1 == uF * K2;
        const int nt = t2 + 1 < K2 ? t2 + 1 : 0;
        const float4 xn = last ? xa : gather(2 * nt), xm = last ? xb : gather(2 * nt + 1);
        const int c0 = 16 * t2 + 4 * h;
        const float4 ua = *reinterpret_cast<const float4*>(uq + f * k + c0);
        const float4 ub = *reinterpret_cast<const float4*>(uq + f * k + c0 + 8);
        float pe[8] = {xa.x * ua.x, xa.y * ua.y, xa.z * ua.z, xa.w * ua.w,
                       xb.x * ub.x, xb.y * ub.y, xb.z * ub.z, xb.w * ub.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) sP = fmaf(pe[e], Pl[c0 + (e < 4 ? e : e + 4)], sP);
        bf16x8 b0, b1, b2;                   // bf16 table: two pieces (split2x8)
        if constexpr (TBF)
          split2x8(pe, b0, b1);
        else
          split3x8(pe, b0, b1, b2);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int u = 32 * n + j;
          const int o = u * U2 + ((2 * t2 + h) ^ afm_img_key(u, U2, SW2));
          const bf16x8 a0 = __builtin_bit_cast(bf16x8, imgb[o]);
          const bf16x8 a1 = __builtin_bit_cast(bf16x8, imgb[NA * U2 + o]);
          const bf16x8 a2 = __builtin_bit_cast(bf16x8, imgb[2 * NA * U2 + o]);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[n], 0, 0, 0);
          if constexpr (!TBF)
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[n], 0, 0, 0);
        }
        xa = xn;
        xb = xm;
        if (++t2 == K2) {
          finish_field();
          t2 = 0;
          ++f;
        }
      }
      if (ok && h == 0) scores[b * N + item] = (ud + num) / (sa + den) + w[id];
      continue;
    }
    for (int s = 0, f = 0, t = 0; s < S; ++s) {
      const float4 xn = (s + 1 < S) ? gather(t + 1 < KQ ? t + 1 : 0) : xa;
      const int c0 = 8 * t + 4 * h;
      const float4 ua = *reinterpret_cast<const float4*>(uq + f * k + c0);
      const float pe[4] = {xa.x * ua.x, xa.y * ua.y, xa.z * ua.z, xa.w * ua.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) sP = fmaf(pe[e], Pl[c0 + e], sP);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int u = 32 * n + j;
        const float4 wa = img[u * U + ((2 * t + h) ^ (u & SW))];
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.x, pe[0], acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.y, pe[1], acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.z, pe[2], acc[n], 0, 0, 0);
        acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.w, pe[3], acc[n], 0, 0, 0);
      }
      xa = xn;
      if (++t == KQ) {   // field f done
        finish_field();
        t = 0;
        ++f;
      }
    }
    if (ok && h == 0) scores[b * N + item] = (ud + num) / (sa + den) + w[id];
  }
}

// ---- A2 per query: the query field folded into the attention weights -------
// (uf_f ⊙ item)·W = item·(uf_f ⊙ W): a workgroup takes ONE query and a chunk of
// item tiles, builds W''_f = uf_f ⊙ W (fp32, rounded once) for each of its
// query fields and splits it into three bf16 LDS images once, so the item row
// — the MFMA B operand — is split once per 16-k step for ALL fields (bf16
// tables: it is its own single piece, 3 MFMAs per 16 k instead of 6), where
// afm_cat_fused splits the pair product uf_f ⊙ item per field.  Likewise
// P·(uf_f ⊙ item) = (P ⊙ uf_f)·item.  The products and the softmax / score
// are AFM.py:227-243's; each term is rounded at a different place than
// forming uf_f ⊙ item first (~1e-7 relative; tolerance 1e-5).
template <int KS>
static size_t afm_cat_w_lds(int F, int A) {
  const int NA = (A + 31) / 32 * 32, uF = F - 1;
  return (size_t)uF * 3 * NA * KS * 32 + (size_t)2 * uF * KS * 16 * 4 + 2 * NA * 4;
}

template <bool TBF, int NT, int KS>
__global__ __launch_bounds__(512) void afm_cat_w(
    const int32_t* __restrict__ q, int64_t nq, int F, const void* __restrict__ E, int64_t M,
    const float* __restrict__ Wt, const float* __restrict__ att_b,
    const float* __restrict__ att_p, int A, const float* __restrict__ P,
    const float* __restrict__ ufdot, const float* __restrict__ suma, int64_t item_row_begin,
    int32_t N, const float* __restrict__ w, float* __restrict__ scores) {
  constexpr int NA = NT * 32, K = 16 * KS, U2 = K / 8;   // 16-B chunks per unit row
  // swizzle mask: the largest power of two (<= 16) that DIVIDES U2, so the
  // XOR stays inside the unit's row (U2 = 6 at k = 48: mask 1, not 3)
  constexpr int SW2 = ((U2 & -U2) < 16 ? (U2 & -U2) : 16) - 1;
  constexpr int NP = TBF ? 1 : 3;                        // item pieces
  extern __shared__ __attribute__((aligned(16))) float smem[];   // afm_cat_w_lds()
  const int uF = F - 1;
  uint4* imgb = reinterpret_cast<uint4*>(smem);          // [f][piece][unit][chunk]
  float* Ql = smem + (size_t)uF * 3 * NA * U2 * 4;       // [f][K]: P ⊙ uf_f
  float* ufs = Ql + uF * K;                              // [f][K]: uf_f
  float* bl = ufs + uF * K;
  float* apl = bl + NA;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int j = l & 31, h = l >> 5;
  for (int x = tid; x < NA; x += 512) {
    bl[x] = x < A ? att_b[x] : 0.f;
    apl[x] = x < A ? att_p[x] : 0.f;
  }
  // persistent (one block per CU, the images take 98 KB at k = A = 64): this
  // block's equal share [g0, g1) of the query-major (query b, item tile t)
  // order; the W'' images are rebuilt once per query the share touches
  // (one (query, chunk) per block rebuilt them for every 4 tiles per wave and
  // left a partial last round of blocks: 300-query call 0.29 -> 0.26 ms,
  // profiles/r04_afm_cat_persist_ab.txt)
  const int ntile = (N + 31) / 32;
  const int64_t T = nq * ntile;
  int64_t g0 = T * blockIdx.x / gridDim.x;
  const int64_t g1 = T * (blockIdx.x + 1) / gridDim.x;
  while (g0 < g1) {
  const int64_t b = g0 / ntile;
  const int t0 = (int)(g0 - b * ntile);
  const int t1 = (int)min<int64_t>(ntile, t0 + (g1 - g0));
  g0 += t1 - t0;
  __syncthreads();                   // the previous query's images are no longer read
  // uf of the query: [E[q0], E[q2], ..., E[q_{F-1}]]  (AFM.py:210-212)
  for (int x = tid; x < uF * K; x += 512) {
    const int f = x / K, c = x - f * K;
    const float v = tab(E, TBF, clamp_id(q[b * F + (f == 0 ? 0 : f + 1)], M), K, c);
    ufs[x] = v;
    Ql[x] = P[c] * v;
  }
  __syncthreads();
  for (int x = tid; x < uF * NA * U2; x += 512) {
    const int f = x / (NA * U2), r = x - f * NA * U2, u = r / U2, c = r - u * U2;
    const int kb = 16 * (c >> 1) + 4 * (c & 1);
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = u < A ? Wt[(int64_t)u * K + kb + e] * ufs[f * K + kb + e] : 0.f;
      v[4 + e] = u < A ? Wt[(int64_t)u * K + kb + 8 + e] * ufs[f * K + kb + 8 + e] : 0.f;
    }
    bf16x8 p0, p1, p2;
    split3x8(v, p0, p1, p2);
    const int o = u * U2 + (c ^ afm_img_key(u, U2, SW2));
    imgb[(f * 3 + 0) * NA * U2 + o] = __builtin_bit_cast(uint4, p0);
    imgb[(f * 3 + 1) * NA * U2 + o] = __builtin_bit_cast(uint4, p1);
    imgb[(f * 3 + 2) * NA * U2 + o] = __builtin_bit_cast(uint4, p2);
  }
  __syncthreads();

  const float ud = ufdot[b], sa = suma[b];
  // this lane's k of 16-k step t: {16t + 4h .. +3, 16t + 8 + 4h .. +3}
  auto gather = [&](int tile, float (&x)[KS][8]) {
    int32_t item = tile * 32 + j;
    item = item < N ? item : 0;
    const int64_t id = item_row_begin + item;
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const int c0 = 16 * t + 4 * h;
      if constexpr (TBF) {
        const uint16_t* r = reinterpret_cast<const uint16_t*>(E) + id * K + c0;
        const uint2 lo = *reinterpret_cast<const uint2*>(r), hi = *reinterpret_cast<const uint2*>(r + 8);
        const uint32_t u4[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[t][2 * e] = __uint_as_float(u4[e] << 16);
          x[t][2 * e + 1] = __uint_as_float(u4[e] & 0xffff0000u);
        }
      } else {
        const float* r = reinterpret_cast<const float*>(E) + id * K + c0;
        const float4 lo = *reinterpret_cast<const float4*>(r), hi = *reinterpret_cast<const float4*>(r + 8);
        x[t][0] = lo.x; x[t][1] = lo.y; x[t][2] = lo.z; x[t][3] = lo.w;
        x[t][4] = hi.x; x[t][5] = hi.y; x[t][6] = hi.z; x[t][7] = hi.w;
      }
    }
  };
  // 8 waves, two per SIMD: a wave's gather and LDS waits overlap its
  // partner's MFMAs (a register prefetch of the next row would cost the
  // second wave)
  for (int tile = t0 + wv; tile < t1; tile += 8) {
    float xc[KS][8];
    gather(tile, xc);
    const int32_t item = tile * 32 + j;
    // the item's pieces, once for every field
    bf16x8 ip[NP][KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      if constexpr (TBF) {
        u32x4_t u;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          u[e] = (__float_as_uint(xc[t][2 * e]) >> 16) | (__float_as_uint(xc[t][2 * e + 1]) & 0xffff0000u);
        ip[0][t] = __builtin_bit_cast(bf16x8, u);
      } else {
        split3x8(xc[t], ip[0][t], ip[1][t], ip[2][t]);
      }
    }
    float num = 0.f, den = 0.f;
    for (int f = 0; f < uF; ++f) {
      f32x16 acc[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int x = 0; x < 16; ++x) acc[n][x] = 0.f;
      float sP = 0.f;
      const uint4* fi = imgb + f * 3 * NA * U2;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        const int c0 = 16 * t + 4 * h;
#pragma unroll
        for (int e = 0; e < 8; ++e) sP = fmaf(xc[t][e], Ql[f * K + c0 + (e < 4 ? e : e + 4)], sP);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int u = 32 * n + j;
          const int o = u * U2 + ((2 * t + h) ^ afm_img_key(u, U2, SW2));
          const bf16x8 a0 = __builtin_bit_cast(bf16x8, fi[o]);
          const bf16x8 a1 = __builtin_bit_cast(bf16x8, fi[NA * U2 + o]);
          const bf16x8 a2 = __builtin_bit_cast(bf16x8, fi[2 * NA * U2 + o]);
          // smallest terms first (bf16 tables: the item is one piece)
          if constexpr (!TBF) {
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, ip[2][t], acc[n], 0, 0, 0);
            acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, ip[1][t], acc[n], 0, 0, 0);
          }
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, ip[0][t], acc[n], 0, 0, 0);
          if constexpr (!TBF) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, ip[1][t], acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, ip[0][t], acc[n], 0, 0, 0);
          acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, ip[0][t], acc[n], 0, 0, 0);
        }
      }
      // field f: logit Σ_a p_a·relu(· + b_a), raw exp (AFM.py:227-230)
      float lg = 0.f;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int u = 32 * n + 8 * g4 + 4 * h;
          const float4 bq = *reinterpret_cast<const float4*>(bl + u);
          const float4 pq = *reinterpret_cast<const float4*>(apl + u);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 0] + bq.x, 0.f), pq.x, lg);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 1] + bq.y, 0.f), pq.y, lg);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 2] + bq.z, 0.f), pq.z, lg);
          lg = fmaf(fmaxf(acc[n][4 * g4 + 3] + bq.w, 0.f), pq.w, lg);
        }
      lg += __shfl_xor(lg, 32, kWave);
      sP += __shfl_xor(sP, 32, kWave);
      const float a = expf(lg);
      num = fmaf(a, sP, num);
      den += a;
    }
    if (item < N && h == 0)
      scores[b * N + item] = (ud + num) / (sa + den) + w[item_row_begin + item];
  }
  }
}

static size_t afm_cat_fused_lds(int F, int k, int A, bool split) {
  const int NA = (A + 31) / 32 * 32;
  const size_t img = split ? (size_t)NA * k * 3 / 2 : (size_t)NA * k;
  return 4 * (img + kAfmMaxK + 2 * NA + 4 * (size_t)(F - 1) * k);
}

// fused A2 envelope: Wᵀ padded to NT*32 <= 128 rows, <= 7 query fields, the
// Wᵀ image and the 4 queries' fields in LDS; HHFM_PLAN_GEMM forces the GEMM path.
static bool afm_cat_fused_ok(int F, int k, int A, int32_t plan) {
  const int NT = (A + 31) / 32;
  return !(plan & HHFM_PLAN_GEMM) && F - 1 <= kAfmCatFusedMaxUF && k % 8 == 0 && k <= kAfmMaxK && NT <= 4 &&
         afm_cat_fused_lds(F, k, A, false) <= 160 * 1024;
}

// split-bf16 variant of the fused kernels: k % 16 == 0, its LDS images fit,
// and no HHFM_PLAN_EXACT_FP32
static bool afm_split(int F, int k, int A, int32_t plan) {
  return k % 16 == 0 && !(plan & HHFM_PLAN_EXACT_FP32) &&
         afm_cat_fused_lds(F, k, A, true) <= 160 * 1024;
}

struct AfmCatPlan {
  int64_t qc;
  int G;
  bool fused;
  size_t off_W2, off_D, off_ud, off_sa, off_part, off_sc, total;
};

static AfmCatPlan afm_cat_plan(int64_t B, int F, int k, int A, int N, int64_t max_cols,
                               int32_t plan) {
  AfmCatPlan p{};
  const int uF = F - 1;
  p.fused = afm_cat_fused_ok(F, k, A, plan);
  if (p.fused) {   // only Σa_uf, P·ufw and the [qc, N] score block
    int64_t qc = max_cols / ((int64_t)uF * A);
    if (qc < 1) qc = 1;
    if (qc > B) qc = B;
    p.qc = qc;
    size_t off = 0;
    p.off_W2 = p.off_D = p.off_part = 0;
    p.off_ud = off; off += a256((size_t)qc * 4);
    p.off_sa = off; off += a256((size_t)qc * 4);
    p.off_sc = off; off += a256((size_t)qc * N * 4);
    p.total = off;
    return p;
  }
  // logit groups of the grouped-dot epilogue: 16, 32 or 64 columns that
  // divide A (a group never straddles two (query, field) column blocks)
  p.G = A % 64 == 0 ? 64 : (A % 32 == 0 ? 32 : 16);
  int64_t qc = max_cols / ((int64_t)uF * A);
  if (qc < 1) qc = 1;
  if (qc > B) qc = B;
  p.qc = qc;
  const int64_t cols = qc * uF * A;
  size_t off = 0;
  p.off_W2 = off; off += a256((size_t)cols * k * 4);
  p.off_D = off; off += a256((size_t)qc * uF * k * 4);
  p.off_ud = off; off += a256((size_t)qc * 4);
  p.off_sa = off; off += a256((size_t)qc * 4);
  p.off_part = off; off += a256((size_t)N * (cols / p.G) * 4);
  p.off_sc = off; off += a256((size_t)qc * N * 4);
  p.total = off;
  return p;
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_afm_forward_workspace(int64_t B, int32_t F, int32_t A, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || F < 2 || A < 1) return HHFM_EINVAL;
  const int64_t np = (int64_t)F * (F - 1) / 2;
  const int ntl = (A + GBN - 1) / GBN;
  *ws_bytes = a256((size_t)B * np * ntl * 4);
  return HHFM_OK;
}

extern "C" int hhfm_afm_forward(const int32_t* idx, int64_t B, int32_t F, const void* E,
                                int64_t features_M, int32_t k, int32_t dtype, const float* w,
                                float w0, const float* Wt, const float* att_b,
                                const float* att_p, int32_t A, const float* P, float* out,
                                void* workspace, size_t ws_bytes, void* stream) {
  return hhfm_afm_forward_ex(idx, B, F, E, features_M, k, dtype, w, w0, Wt, att_b, att_p, A, P,
                             out, HHFM_PLAN_DEFAULT, workspace, ws_bytes, stream);
}

extern "C" int hhfm_afm_forward_ex(const int32_t* idx, int64_t B, int32_t F, const void* E,
                                   int64_t features_M, int32_t k, int32_t dtype, const float* w,
                                   float w0, const float* Wt, const float* att_b,
                                   const float* att_p, int32_t A, const float* P, float* out,
                                   int32_t plan, void* workspace, size_t ws_bytes,
                                   void* stream) {
  if (plan & ~HHFM_PLAN_ALL) return HHFM_EINVAL;
  if (B < 0 || F < 2 || F > 16 || k < 1 || A < 1 || features_M < 1) return HHFM_EINVAL;
  if (dtype != HHFM_F32 && dtype != HHFM_BF16) return HHFM_EINVAL;
  if (k % 4) return HHFM_EUNSUPPORTED;
  if (B == 0) return HHFM_OK;
  if (!idx || !E || !w || !Wt || !att_b || !att_p || !P || !out) return HHFM_EINVAL;
  size_t need = 0;
  hhfm_afm_forward_workspace(B, F, A, &need);
  if (!workspace || ws_bytes < need) return HHFM_EWORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int np = F * (F - 1) / 2;
  {  // fused path: F <= 8, k % 8 == 0, A <= 128, (A padded to 32) x k <= 32 x 512
    const int NT = (A + 31) / 32;
    if (F <= kAfmFusedMaxF && k % 8 == 0 && k <= kAfmMaxK && NT <= 4 && NT * k <= 512) {
      const int R = 32 / np;
      const int64_t nblk = (B + R - 1) / R;
      int64_t blocks = (nblk + 3) / 4;
      if (blocks > 2048) blocks = 2048;
      const bool tb = dtype == HHFM_BF16;
      const bool split = k % 16 == 0 && !(plan & HHFM_PLAN_EXACT_FP32) &&
                         afm_rows_fused_lds(k, A, true) <= 160 * 1024;
      // pair-major kernel (32 rows per wave tile): split arithmetic, k = 16·KS
      // for KS in {2, 3, 4} (a whole pair's gathers in flight), A <= 96,
      // F <= 8 (default; HHFM_PLAN_PER_FIELD keeps the combo-packed
      // afm_rows_fused)
      const int KSp = k / 16;
      const size_t lp = afm_rows_pairs_lds(NT * 32, k, F);
      if (split && !(plan & HHFM_PLAN_PER_FIELD) && KSp >= 2 && KSp <= 4 && NT <= 3 &&
          lp <= 160 * 1024) {
        const int64_t nb32 = (B + 31) / 32;
        int64_t pblocks = (nb32 + 3) / 4;
        if (pblocks > 2048) pblocks = 2048;
#define HHFM_AFM_PAIRS_L(N, TB, KS)                                                          \
  {                                                                                        \
    allow_lds((const void*)afm_rows_pairs<TB, N, KS>, lp);                                  \
    hipLaunchKernelGGL((afm_rows_pairs<TB, N, KS>), dim3((unsigned)pblocks), dim3(256), lp, \
                       st, idx, B, F, E, features_M, w, w0, Wt, att_b, att_p, A, P, out);  \
  }
#define HHFM_AFM_PAIRS_K(N, TB)                      \
  switch (KSp) {                                     \
    case 2: HHFM_AFM_PAIRS_L(N, TB, 2) break;        \
    case 3: HHFM_AFM_PAIRS_L(N, TB, 3) break;        \
    default: HHFM_AFM_PAIRS_L(N, TB, 4) break;       \
  }
#define HHFM_AFM_PAIRS(N)                                                   \
  if (NT == N) {                                                           \
    if (tb) { HHFM_AFM_PAIRS_K(N, true) } else { HHFM_AFM_PAIRS_K(N, false) } \
    return (int)hipGetLastError();                                         \
  }
        HHFM_AFM_PAIRS(1)
        HHFM_AFM_PAIRS(2)
        HHFM_AFM_PAIRS(3)
#undef HHFM_AFM_PAIRS
#undef HHFM_AFM_PAIRS_K
#undef HHFM_AFM_PAIRS_L
      }
      const size_t lds = afm_rows_fused_lds(k, A, split);
#define HHFM_AFM_FUSED_K(N, TB, SP, KS)                                                      \
  {                                                                                        \
    allow_lds((const void*)afm_rows_fused<TB, N, SP, KS>, lds);                             \
    hipLaunchKernelGGL((afm_rows_fused<TB, N, SP, KS>), dim3((unsigned)blocks), dim3(256),  \
                       lds, st, idx, B, F, E, features_M, k, w, w0, Wt, att_b, att_p, A, P, \
                       out);                                                                \
  }
#define HHFM_AFM_FUSED_L(N, TB, SP)                                                         \
  if (SP && k == 64) HHFM_AFM_FUSED_K(N, TB, SP, 4)                                          \
  else if (SP && k == 128) HHFM_AFM_FUSED_K(N, TB, SP, 8)                                    \
  else HHFM_AFM_FUSED_K(N, TB, SP, 0)
#define HHFM_AFM_FUSED(N)                                                                   \
  if (NT == N) {                                                                           \
    if (tb) {                                                                              \
      if (split) HHFM_AFM_FUSED_L(N, true, true) else HHFM_AFM_FUSED_L(N, true, false)     \
    } else {                                                                               \
      if (split) HHFM_AFM_FUSED_L(N, false, true) else HHFM_AFM_FUSED_L(N, false, false)   \
    }                                                                                      \
    return (int)hipGetLastError();                                                         \
  }
      HHFM_AFM_FUSED(1)
      HHFM_AFM_FUSED(2)
      HHFM_AFM_FUSED(3)
      HHFM_AFM_FUSED(4)
#undef HHFM_AFM_FUSED
#undef HHFM_AFM_FUSED_L
#undef HHFM_AFM_FUSED_K
    }
  }
  const int ntl = (A + GBN - 1) / GBN;
  float* part = reinterpret_cast<float*>(workspace);
  GemmArgs g{};
  g.M = B * np;
  g.N = A;
  g.K = k;
  g.pair_mode = 1;
  g.P = np;
  g.gidx = idx;
  g.T = E;
  g.Mtab = features_M;
  g.F = F;
  g.kf = k;
  g.t_bf16 = dtype == HHFM_BF16;
  g.Bt = Wt;
  g.ldb = k;
  g.bias = att_b;
  g.relu = 1;
  g.dotv = att_p;
  g.partial = part;
  launch_gemm(g, false, 1, st);
  int64_t blocks = (B + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(afm_rows_finish, dim3((unsigned)blocks), dim3(256), 0, st, idx, B, F, E,
                     (int)(dtype == HHFM_BF16), features_M, k, w, w0, P, part, ntl, out);
  return (int)hipGetLastError();
}

extern "C" int hhfm_afm_catalog_topk_workspace(int64_t B, int32_t F, int32_t k, int32_t A,
                                               int32_t item_count, int64_t max_cols,
                                               size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || F < 3 || k < 1 || A < 1 || item_count < 1 || max_cols < 1)
    return HHFM_EINVAL;
  *ws_bytes = afm_cat_plan(B, F, k, A, item_count, max_cols, HHFM_PLAN_DEFAULT).total;
  return HHFM_OK;
}

extern "C" int hhfm_afm_catalog_topk_workspace_ex(int64_t B, int32_t F, int32_t k, int32_t A,
                                                  int32_t item_count, int64_t max_cols,
                                                  int32_t plan, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || F < 3 || k < 1 || A < 1 || item_count < 1 || max_cols < 1 ||
      (plan & ~HHFM_PLAN_ALL))
    return HHFM_EINVAL;
  *ws_bytes = afm_cat_plan(B, F, k, A, item_count, max_cols, plan).total;
  return HHFM_OK;
}

extern "C" int hhfm_afm_catalog_topk(const int32_t* qidx, int64_t B, int32_t F, const void* E,
                                     int64_t features_M, int32_t k, int32_t dtype,
                                     const float* w, const float* Wt, const float* att_b,
                                     const float* att_p, int32_t A, const float* P,
                                     int32_t item_row_begin, int32_t item_count,
                                     int32_t global_item_base, int32_t K, int64_t max_cols,
                                     float* top_score, int32_t* top_idx, void* workspace,
                                     size_t ws_bytes, void* stream) {
  return hhfm_afm_catalog_topk_ex(qidx, B, F, E, features_M, k, dtype, w, Wt, att_b, att_p, A,
                                  P, item_row_begin, item_count, global_item_base, K, max_cols,
                                  top_score, top_idx, HHFM_PLAN_DEFAULT, workspace, ws_bytes,
                                  stream);
}

extern "C" int hhfm_afm_catalog_topk_ex(const int32_t* qidx, int64_t B, int32_t F,
                                        const void* E, int64_t features_M, int32_t k,
                                        int32_t dtype, const float* w, const float* Wt,
                                        const float* att_b, const float* att_p, int32_t A,
                                        const float* P, int32_t item_row_begin,
                                        int32_t item_count, int32_t global_item_base, int32_t K,
                                        int64_t max_cols, float* top_score, int32_t* top_idx,
                                        int32_t plan, void* workspace, size_t ws_bytes,
                                        void* stream) {
  if (plan & ~HHFM_PLAN_ALL) return HHFM_EINVAL;
  if (B < 0 || F < 3 || F - 1 > kAfmMaxUF || k < 1 || k > kAfmMaxK || A < 1 ||
      features_M < 1 || max_cols < 1)
    return HHFM_EINVAL;
  if (dtype != HHFM_F32 && dtype != HHFM_BF16) return HHFM_EINVAL;
  if (item_count < 1 || item_row_begin < 0 || (int64_t)item_row_begin + item_count > features_M)
    return HHFM_EINVAL;
  if (K < 1 || K > item_count) return HHFM_EINVAL;
  if (K > 64) return HHFM_EUNSUPPORTED;
  if (!afm_cat_fused_ok(F, k, A, plan) && (k % 4 || A % 16))
    return HHFM_EUNSUPPORTED;
  if (B == 0) return HHFM_OK;
  if (!qidx || !E || !w || !Wt || !att_b || !att_p || !P || !top_score || !top_idx)
    return HHFM_EINVAL;
  const AfmCatPlan p = afm_cat_plan(B, F, k, A, item_count, max_cols, plan);
  if (!workspace || ws_bytes < p.total) return HHFM_EWORKSPACE;
  char* ws = reinterpret_cast<char*>(workspace);
  float* W2 = reinterpret_cast<float*>(ws + p.off_W2);
  float* D = reinterpret_cast<float*>(ws + p.off_D);
  float* ud = reinterpret_cast<float*>(ws + p.off_ud);
  float* sa = reinterpret_cast<float*>(ws + p.off_sa);
  float* part = reinterpret_cast<float*>(ws + p.off_part);
  float* sc = reinterpret_cast<float*>(ws + p.off_sc);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int uF = F - 1;
  const int tb = dtype == HHFM_BF16;
  for (int64_t b0 = 0; b0 < B; b0 += p.qc) {
    const int64_t nq = (B - b0) < p.qc ? (B - b0) : p.qc;
    const size_t qsl = afm_cat_qside_lds(F, k, A);
    if (p.fused && uF * (uF - 1) / 2 <= kAfmQsMaxPairs &&
        qsl <= 64 * 1024) {
      hipLaunchKernelGGL(afm_cat_qside, dim3((unsigned)nq), dim3(256), qsl, st, qidx + b0 * F, nq,
                         F, E, tb, features_M, k, Wt, att_b, att_p, A, P, ud, sa);
    } else {
      hipLaunchKernelGGL(afm_cat_prep, dim3((unsigned)nq), dim3(64), 0, st, qidx + b0 * F, nq, F,
                         E, tb, features_M, k, Wt, att_b, att_p, A, P, W2, D, ud, sa,
                         (int)!p.fused);
    }
    if (p.fused) {
      const int64_t qgroups = (nq + 3) / 4;
      const int ntile = (item_count + 31) / 32;
      int64_t nchunk = (2048 + qgroups - 1) / qgroups;
      if (nchunk > ntile) nchunk = ntile;
      const int tpb = (int)((ntile + nchunk - 1) / nchunk);
      nchunk = (ntile + tpb - 1) / tpb;
      const dim3 grid((unsigned)(qgroups * nchunk));
      const int NT = (A + 31) / 32;
      const bool split = afm_split(F, k, A, plan);
      // per-query kernel: its W'' images fit (k <= 64), split arithmetic
      const int KSw = k / 16;
      bool wdone = false;
      if (split && !(plan & HHFM_PLAN_PER_FIELD) && k % 16 == 0 && KSw >= 1 && KSw <= 4) {
        size_t wl = 0;
        switch (KSw) {
          case 1: wl = afm_cat_w_lds<1>(F, A); break;
          case 2: wl = afm_cat_w_lds<2>(F, A); break;
          case 3: wl = afm_cat_w_lds<3>(F, A); break;
          default: wl = afm_cat_w_lds<4>(F, A); break;
        }
        if (wl <= 160 * 1024) {
          // one block per CU walks an equal share of the query-major tiles
          const int cus = stream_cu_count(st);
          const int64_t T = nq * (int64_t)ntile;
          const dim3 wgrid((unsigned)(T < cus ? T : cus));
#define HHFM_AFM_CAT_W_L(N, TB, KS)                                                              \
  {                                                                                             \
    allow_lds((const void*)afm_cat_w<TB, N, KS>, wl);                                            \
    hipLaunchKernelGGL((afm_cat_w<TB, N, KS>), wgrid, dim3(512), wl, st, qidx + b0 * F, nq, F,   \
                       E, features_M, Wt, att_b, att_p, A, P, ud, sa, (int64_t)item_row_begin,   \
                       item_count, w, sc);                                                       \
    wdone = true;                                                                               \
  }
#define HHFM_AFM_CAT_W_K(N, TB)                                                                  \
  switch (KSw) {                                                                                \
    case 1: HHFM_AFM_CAT_W_L(N, TB, 1) break;                                                   \
    case 2: HHFM_AFM_CAT_W_L(N, TB, 2) break;                                                   \
    case 3: HHFM_AFM_CAT_W_L(N, TB, 3) break;                                                   \
    default: HHFM_AFM_CAT_W_L(N, TB, 4) break;                                                  \
  }
#define HHFM_AFM_CAT_W(N)                                                                        \
  if (NT == N) {                                                                                \
    if (tb) { HHFM_AFM_CAT_W_K(N, true) } else { HHFM_AFM_CAT_W_K(N, false) }                   \
  }
          HHFM_AFM_CAT_W(1)
          HHFM_AFM_CAT_W(2)
          HHFM_AFM_CAT_W(3)
          HHFM_AFM_CAT_W(4)
#undef HHFM_AFM_CAT_W
#undef HHFM_AFM_CAT_W_K
#undef HHFM_AFM_CAT_W_L
        }
      }
      const size_t lds = afm_cat_fused_lds(F, k, A, split);
#define HHFM_AFM_CAT_FUSED_L(N, TB, SP)                                                       \
  {                                                                                          \
    allow_lds((const void*)afm_cat_fused<TB, N, SP>, lds);                                    \
    hipLaunchKernelGGL((afm_cat_fused<TB, N, SP>), grid, dim3(256), lds, st, qidx + b0 * F,   \
                       nq, F, E, features_M, k, Wt, att_b, att_p, A, P, ud, sa,                \
                       (int64_t)item_row_begin, item_count, tpb, (int)nchunk, w, sc);          \
  }
#define HHFM_AFM_CAT_FUSED(N)                                                                 \
  if (NT == N && !wdone) {                                                                   \
    if (tb) {                                                                                \
      if (split) HHFM_AFM_CAT_FUSED_L(N, true, true) else HHFM_AFM_CAT_FUSED_L(N, true, false) \
    } else {                                                                                 \
      if (split) HHFM_AFM_CAT_FUSED_L(N, false, true)                                        \
      else HHFM_AFM_CAT_FUSED_L(N, false, false)                                             \
    }                                                                                        \
  }
      HHFM_AFM_CAT_FUSED(1)
      HHFM_AFM_CAT_FUSED(2)
      HHFM_AFM_CAT_FUSED(3)
      HHFM_AFM_CAT_FUSED(4)
#undef HHFM_AFM_CAT_FUSED
#undef HHFM_AFM_CAT_FUSED_L
    } else {
      GemmArgs g{};
      g.M = item_count;
      g.N = (int)(nq * uF * A);
      g.K = k;
      g.A = reinterpret_cast<const char*>(E) + (int64_t)item_row_begin * k * (tb ? 2 : 4);
      g.lda = k;
      g.a_src_bf16 = tb;
      g.Bt = W2;
      g.ldb = k;
      g.bias = att_b;
      g.relu = 1;
      g.dotv = att_p;
      g.partial = part;
      g.G = p.G;
      g.mod = A;
      g.ldp = nq * uF * A / p.G;
      launch_gemm(g, false, 2, st);
      const int64_t nblk = (item_count + kWave - 1) / kWave;
      const int64_t waves = nq * nblk;
      hipLaunchKernelGGL(afm_cat_finish, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, nq,
                         uF, A, p.G, part, g.ldp, D, ud, sa, E, tb, k, (int64_t)item_row_begin,
                         item_count, w, sc);
    }
    int64_t tblocks = (nq + 3) / 4;
    if (tblocks > 4096) tblocks = 4096;
    if (K <= 32)
      hipLaunchKernelGGL((topk_dense_kernel<32, 32>), dim3((unsigned)tblocks), dim3(256), 0, st, sc, nq,
                         item_count, (int64_t)item_count, K, global_item_base,
                         top_score + b0 * K, top_idx + b0 * K, nullptr);
    else
      hipLaunchKernelGGL((topk_dense_kernel<64, 32>), dim3((unsigned)tblocks), dim3(256), 0, st, sc, nq,
                         item_count, (int64_t)item_count, K, global_item_base,
                         top_score + b0 * K, top_idx + b0 * K, nullptr);
  }
  return (int)hipGetLastError();
}
