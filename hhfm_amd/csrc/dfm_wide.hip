// K3w — DeepFM forward, bf16 MLP, ITEM plan, 256 rows per workgroup.
// Replaces DeepFM.out (Newcode/DFM.py:104-137) like dfm_fused.hip's kernels;
// planned by hhfm_dfm_forward_workspace_ex / hhfm_dfm_catalog_topk
// (mlp_gemm.hip) through dfm_fused_launch.
#include <utility>

#include "dfm_fused.h"

namespace hhfm {

// ---------------------------------------------------------------------------
// K3w — the bf16-MLP DeepFM forward at 256 rows per workgroup (the ITEM plan:
// layer 0 of the item field on MFMA, every other field from P, rows grouped
// by user).  dfm_fused keeps 32 rows x all output units per wave in
// accumulators (208 registers), so its workgroup holds 128 rows and streams
// every weight once per 128 rows: ≈32 B/clk of L2 -> LDS per CU at the MFMA
// rate, what one CU pulls — the C5 kernel ran at that stream, MFMA busy 35 %.
// Here a wave owns RT 16-row tiles (v_mfma_f32_16x16x32_bf16; RT = 2 at two
// waves per SIMD, 8 waves = 256 rows, by default; RT = 3 at one, 192 rows) and
// walks the output units 32 at a time: per pass, the full-K MFMA chain of
// 2 unit tiles x 3 row tiles (24 accumulator registers), then bias + ReLU +
// bf16 straight into the next layer's B operand — the 16x16 result puts
// units 4kq..+3 of a tile on lane group kq, exactly the k a lane group
// supplies next (k order {32s + 4kq .. +3, 32s + 16 + 4kq .. +3}), so no
// lane movement.  Live: the layer input (104 registers for 32 rows x 416
// units) + the output being built (104) + 16 (RT = 2), within the 256 two
// waves per SIMD leave: no scratch since the unstaged body moved to its own
// launch (profiles/r06_kernel_resources.txt); the
// weight stream per row falls to 2/3 (≈21 B/clk per CU), each 1-KB A
// fragment feeds three MFMAs.
//   * weights: dfm_pack_weights_w lays each (layer, 32-unit pass) out as S
//     k32 steps of 2 KB, [unit tile j][kq][unit r] x 16 B (lane-linear, no
//     bank conflicts); a 3-slot LDS ring filled two passes ahead by
//     lane-linear LDS-DMA, one counted vmcnt + barrier per pass, the DMAs
//     issued one per MFMA step;
//   * layer 0 = Σ_f P_f[x_f] (projected fields, staged in LDS when the
//     block's id spans fit) + the item field's k32 steps on MFMA, B = the
//     gathered item rows (k order 32s + 8kq .. +7);
//   * the FM part from the item's B operand registers and the other fields'
//     table rows, before layer 0.
// Instantiated per shape (TM 32-unit passes in every layer, S0 = k/32 item
// steps, NF projected fields); other shapes take dfm_fused.
// ---------------------------------------------------------------------------

// diagnostic knock-outs (timing only, wrong results; default 0): 1 FM part,
// 2 P sums, 4 per-pass barriers, 8 weight DMA after the first two passes,
// 16 MFMAs, 32 staging copies
#ifndef HHFM_WKO
#define HHFM_WKO 0
#endif
#if HHFM_WKO && !defined(HHFM_DIAG_BUILD)
#error "HHFM_WKO knock-outs give wrong results: diagnostic builds only (-DHHFM_DIAG_BUILD)"
#endif
// 16-row tiles per wave and waves per workgroup: 2 x 8 = 256 rows, two waves
// per SIMD (C5 bf16 10.0-10.3 ms, bit-identical), against 3 x 4 = 192 rows at
// one wave per SIMD (12.9-13.0 ms; profiles/r04_k3w_two_waves_ab.txt): the
// second wave's MFMAs cover the first's DMA issue, epilogue and barrier waits,
// and each weight byte streamed feeds 256 rows instead of 192.  The template
// admits RT in 1..3 at 4 waves and RT <= 2 at 8 (at most 16 row tiles); the
// plan bits HHFM_PLAN_WIDE_* run the alternates at the test shape, and every
// admitted shape was measured bit-identical to the default at C5 as well
// (profiles/r05_wide_shapes.txt).  (The wrong results of round-4 scratch logs
// gpurun_out/wide_r{1,2}w4.log came from a working tree before commit
// 5f4698f, which sized the per-wave vmcnt wait from the DMA units each wave
// issues; the committed template was never wrong at those shapes.)
#ifndef HHFM_WIDE_RT
#define HHFM_WIDE_RT 2
#endif
#ifndef HHFM_WIDE_NWV
#define HHFM_WIDE_NWV 8
#endif
// FM part of staged blocks: 1 = the fields' Σ_k Wp_k·e_k² from per-row sums g
// computed once per staged table row; 0 = per row and k, as the overflow
// launch does.  0: with 1 a row's bits depended on whether its block fitted
// LDS (the sums are ordered differently), which a batch of mostly grouped rows
// with a few wide-span blocks showed (tests/test_gpu_dfm.py "mixed").  C5
// takes its FM part from the pair table (PAIRS) and is not affected.
#ifndef HHFM_WFM
#define HHFM_WFM 0
#endif
// staged blocks: P sums of layer-0 pass t+1 among pass t's MFMA steps (0: at
// the pass start)
#ifndef HHFM_WPI
#define HHFM_WPI 1
#endif
// PAIRS: 1 = each row's base (Σ_f w·Wp + Σ_{f<g} C[x_f][x_g]) + bp formed in
// the prologue from the pair table, in dfm_fm_base_pairs' order (the same
// bits, tested); 0 = that launch's output read in the epilogue.  C5 bf16
// 9.85 -> 9.74-9.76 ms per pass (profiles/r06_wfb_ab.txt): the 0.28-ms launch
// and its round trip of the bases through HBM gone, its gathers now under
// the other workgroup's MFMAs
#ifndef HHFM_WFB
#define HHFM_WFB 1
#endif

template <int B_, int E_, class Fn>
HHFM_DEV void static_for(Fn&& fn) {
  if constexpr (B_ < E_) {
    fn(std::integral_constant<int, B_>{});
    static_for<B_ + 1, E_>(fn);
  }
}

// the wave's DMAs older than its N most recent have landed, every wave's LDS
// reads have returned, then the block barrier
template <int N>
HHFM_DEV void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// materialise a value here: the compiler sinks pure arithmetic towards its
// last use (the store after the last layer), keeping its inputs live
HHFM_DEV void pin(float& v) { asm volatile("" : "+v"(v)); }
HHFM_DEV void pin(uint4& v) {
  u32x4_t t = __builtin_bit_cast(u32x4_t, v);
  asm volatile("" : "+v"(t));
  v = __builtin_bit_cast(uint4, t);
}

// ReLU of two packed bf16 values: v_pk_max_i16 against 0
// (asm: the compiler otherwise splits the pair and converts each half alone)
HHFM_DEV uint32_t relu_bf16x2(uint32_t v) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(v));
  return r;
}

// one lane-linear 16-B-per-lane LDS-DMA to the LDS byte offset lds_off from
// the uniform base + the lane's 32-bit byte offset (SGPR base: no 64-bit
// per-lane address registers, which the staged kernel has none spare for)
HHFM_DEV void dma16_at(const void* base, uint32_t voff, uint32_t lds_off) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :
               : "v"(voff), "s"(base), "s"(__builtin_amdgcn_readfirstlane(lds_off))
               : "memory");
}

// pass (layer i, t), k32 step s, unit tile j, lane (r, kq): 16 B of
//   layer 0: W0[32t + 16j + r][fe0·k + 32s + 8kq .. +7]
//   layer i: W_i[32t + 16j + r][32s + 4kq .. +3] ++ W_i[..][32s + 16 + 4kq .. +3]
// zero outside the layer's rows / columns
__global__ __launch_bounds__(256) void dfm_pack_weights_w(FusedDfmArgs a, int TM, int S0,
                                                          uint4* __restrict__ out,
                                                          uint32_t* __restrict__ ovf) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *ovf = 0;   // the overflow count (dfm_fused_w)
  const int64_t n0 = (int64_t)TM * S0 * 2;            // layer-0 1-KB units
  const int64_t total = (n0 + 2 * (int64_t)TM * TM * 2) * 64;
  const int fe0 = (int)(a.perm & 15);   // caller field of internal field 0 (the item)
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t unit = x >> 6;
    const int lane = (int)(x & 63), r = lane & 15, kq = lane >> 4;
    int i, t, sj;
    if (unit < n0) {
      i = 0;
      t = (int)(unit / (2 * S0));
      sj = (int)(unit % (2 * S0));
    } else {
      const int64_t rel = unit - n0;
      i = 1 + (int)(rel / (2 * (int64_t)TM * TM));
      const int rr = (int)(rel % (2 * (int64_t)TM * TM));
      t = rr / (2 * TM);
      sj = rr % (2 * TM);
    }
    const int s = sj >> 1, j = sj & 1;
    const int n = 32 * t + 16 * j + r;
    const uint16_t* row = a.Wt[i] + (int64_t)n * a.ldb[i];
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n < a.dims[i]) {
      if (i == 0) {
        v = *reinterpret_cast<const uint4*>(row + fe0 * a.k + 32 * s + 8 * kq);
      } else {
        const int c0 = 32 * s + 4 * kq, c1 = c0 + 16;
        if (c0 < a.ldb[i]) {
          const uint2 lo = *reinterpret_cast<const uint2*>(row + c0);
          v.x = lo.x;
          v.y = lo.y;
        }
        if (c1 < a.ldb[i]) {
          const uint2 hi = *reinterpret_cast<const uint2*>(row + c1);
          v.z = hi.x;
          v.w = hi.y;
        }
      }
    }
    out[x] = v;
  }
}

// Overflow list, in the packed-weight workspace past the weights: the count
// in a 256-B head, then row-unit indices (units of the overflow launch's rows)
constexpr int kOvfHead = 64;

// One block of kWideRows rows from row m0.  RT row tiles (16 rows) per wave,
// NWV waves: 3 x 4 (one wave per SIMD, 192 rows) or 2 x 8 (two waves per
// SIMD, 256 rows).  OVF false: the staged body only — a block whose id spans
// do not fit LDS appends its ovf_rows-row units to the overflow list and
// ends; OVF true: the unstaged body (P and table rows read from memory), for
// the listed units.  Each kernel then holds one body: the staged kernel at
// two waves per SIMD has no registers left for the unstaged one's state
// (224 B of scratch per lane when both were compiled together).
template <int TM, int S0, int NF, bool PAIRS, int RT, int NWV, bool OVF>
HHFM_DEV void wide_rows(const FusedDfmArgs& a, const int64_t m0, uint32_t* ovf, int ovf_rows) {
  constexpr int kWideRows = NWV * 16 * RT;
  constexpr int NTH = NWV * 64;
  // PAIRS: a.fmbase[m] = (Σ_f w·Wp + FM part) + bp from the pair table
  // (dfm_fm_pairs), so no table rows are staged and no FM part runs here
  static_assert(NF >= 1 && NF < kFusedMaxF, "wide DeepFM kernel: fields");
  static_assert((NWV == 4 || NWV == 8) && RT >= 1 && RT <= 3 && RT * NWV <= 16,
                "wide DeepFM kernel: 1-3 row tiles at 4 waves, 1-2 at 8");
  constexpr int F = NF + 1;
  constexpr int NR = TM * 32;
  constexpr int NCH = 3 * TM;                          // passes: (layer, 32 units)
  constexpr int kUnits = 2 * (TM > S0 ? TM : S0);      // 1-KB units per ring slot
  constexpr int kSlotB = kUnits * 1024;
  constexpr int kIds = 3 * kSlotB;
  constexpr int kBl = kIds + kWideRows * kFusedMaxF * 4;
  constexpr int kVl = kBl + 3 * NR * 4;
  constexpr int kWp = kVl + NR * 4;
  constexpr int kPlo = kWp + (kFusedMaxF + kFusedMaxK) * 4;
  constexpr int kYl = kPlo + 6 * kFusedMaxF * 4;
  constexpr int kPst = kYl + kWideRows * 4;
  constexpr int kPsLd = NR + 4;                        // staged P row stride (floats)
  constexpr int kPsFloats = (kLdsBytes - kPst) / 4;
  static_assert(kPst + 4 * 1024 <= kLdsBytes, "wide DeepFM kernel: LDS");
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];   // ONE LDS object
  int32_t* ids = reinterpret_cast<int32_t*>(smem + kIds);
  float* blv = reinterpret_cast<float*>(smem + kBl);
  float* vl = reinterpret_cast<float*>(smem + kVl);
  float* wpl = reinterpret_cast<float*>(smem + kWp);
  int32_t* plo = reinterpret_cast<int32_t*>(smem + kPlo);   // lo | hi | P | E | g base | perm⁻¹
  float* ylds = reinterpret_cast<float*>(smem + kYl);
  float* pst = reinterpret_cast<float*>(smem + kPst);

  const int tid = threadIdx.x, l = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = l & 15, kq = l >> 4;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int k = a.k;
  const float* P = reinterpret_cast<const float*>(a.proj);
  const uint16_t* E = reinterpret_cast<const uint16_t*>(a.E);

  // rows past B repeat row B-1 (never stored), so the id spans stay tight
  for (int x = tid; x < kWideRows * F; x += NTH) {
    int64_t m = m0 + x / F;
    m = m < a.B ? m : a.B - 1;
    const int fe = (int)((a.perm >> (4 * (x % F))) & 15);
    ids[x] = clamp_id(a.idx[m * F + fe], a.M);
  }
  for (int i = 0; i < 3; ++i)
    for (int n = tid; n < NR; n += NTH) blv[i * NR + n] = n < a.dims[i] ? a.bias[i][n] : 0.f;
  for (int n = tid; n < NR; n += NTH) vl[n] = n < a.dims[2] ? a.Wp[F + k + n] : 0.f;
  for (int x = tid; x < F + k; x += NTH)
    wpl[x < F ? x : x - F + kFusedMaxF] = a.Wp[x < F ? (int)((a.perm >> (4 * x)) & 15) : x];
  if (tid < kFusedMaxF) {
    plo[tid] = 0x7fffffff;
    plo[kFusedMaxF + tid] = -1;
    if (tid < F) plo[5 * kFusedMaxF + (int)((a.perm >> (4 * tid)) & 15)] = tid;
  }
  __syncthreads();

  // pass c: 2·S k32-step halves of 1 KB at unit cbase(c) -> ring slot c % 3
  auto cunits = [](int c) { return c < TM ? 2 * S0 : 2 * TM; };
  auto cbase = [](int c) { return c < TM ? c * 2 * S0 : TM * 2 * S0 + (c - TM) * 2 * TM; };
  auto dma_unit = [&](int c, int u) {
    dma16_at(a.packed + (int64_t)(cbase(c) + u) * 64, 16 * l, lds0 + (c % 3) * kSlotB + u * 1024);
  };
  for (int c = 0; c < 2; ++c)
    for (int u = wv; u < cunits(c); u += NWV) dma_unit(c, u);

  // layer 0's B operand: the item rows of this lane's three rows (k32 step
  // s: columns 32s + 8kq .. +7), in flight with the weight passes
  const int row0 = 16 * RT * wv + r;       // row tile rt: row0 + 16·rt
  uint4 E0[RT][S0];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int64_t id = ids[(row0 + 16 * rt) * F];
#pragma unroll
    for (int s = 0; s < S0; ++s)
      E0[rt][s] = *reinterpret_cast<const uint4*>(E + id * k + 32 * s + 8 * kq);
  }
  if (!PAIRS && tid < kWideRows) {   // Σ_f w[x_f]·Wp[f], one row per thread (dfm_fused's order)
    float wv8[kFusedMaxF];
#pragma unroll
    for (int f = 0; f < kFusedMaxF; ++f) wv8[f] = f < F ? a.w[ids[tid * F + f]] : 0.f;
    float y1 = 0.f;
#pragma unroll
    for (int f = 0; f < kFusedMaxF; ++f)
      if (f < F) y1 += wv8[f] * wpl[f];
    ylds[tid] = y1;
  }
  if (PAIRS && HHFM_WFB && tid < kWideRows) {   // the caller's field order, as dfm_fm_base_pairs
    const float* C = reinterpret_cast<const float*>(a.scratch);
    int32_t x[F];
#pragma unroll
    for (int c = 0; c < F; ++c) x[c] = ids[tid * F + plo[5 * kFusedMaxF + c]];
    float y2 = 0.f;
#pragma unroll
    for (int f = 0; f < F; ++f)
#pragma unroll
      for (int g = f + 1; g < F; ++g) y2 += C[(int64_t)x[f] * a.M + x[g]];
    float y1 = 0.f;
#pragma unroll
    for (int f = 0; f < F; ++f) y1 = __fmaf_rn(a.w[x[f]], a.Wp[f], y1);
    ylds[tid] = (y1 + y2) + a.bp;
  }
  for (int x = tid; x < (OVF ? 0 : kWideRows * NF); x += NTH) {
    const int row = x / NF, f = 1 + x % NF;
    atomicMin(&plo[f], ids[row * F + f]);
    atomicMax(&plo[kFusedMaxF + f], ids[row * F + f]);
  }
  __syncthreads();
  // all projected fields' P rows and table rows lo..hi staged in LDS when
  // they fit (rows grouped by user: the user's and the contexts' few rows);
  // otherwise the block's units go to the overflow launch, which reads them
  // from memory.  (One kernel with both bodies behind a uniform branch per
  // field between LDS and memory reads was merged by the compiler into flat
  // loads, and one with both bodies behind one branch spilled.)
  const int ek = k / 2;   // bf16 table row in floats
  // staged table rows 16 B apart in bank space (a row is 0 mod 64 banks), so
  // the FM part's reads of different rows by one lane group do not conflict
  const int ekp = PAIRS ? 0 : ek + 4;
  if constexpr (!OVF) {
    int used = 0;
    for (int f = 1; f < F; ++f) {
      const int span = plo[kFusedMaxF + f] - plo[f] + 1;
      if (tid == 0) {
        plo[2 * kFusedMaxF + f] = used;
        plo[3 * kFusedMaxF + f] = used + span * kPsLd;
        plo[4 * kFusedMaxF + f] = used + span * (kPsLd + ekp);
      }
      used += span * (kPsLd + ekp) + (PAIRS ? 0 : ((span + 3) & ~3));
    }
    if (used > kPsFloats || (HHFM_WKO & 32)) {   // uniform: every thread read the same plo
      if (tid == 0) {
        const int64_t u0 = m0 / ovf_rows;
        int n = 0;
        for (int64_t r = m0; r < m0 + kWideRows && r < a.B; r += ovf_rows) ++n;
        const uint32_t at = atomicAdd(ovf, (uint32_t)n);
        for (int j = 0; j < n; ++j) ovf[kOvfHead + at + j] = (uint32_t)(u0 + j);
      }
      dma_wait();   // passes 0 and 1 landed before the workgroup's LDS is released
      return;
    }
  }
  if constexpr (!OVF) {
    int used = 0;
    for (int f = 1; f < F; ++f) {
      const int lo = plo[f], span = plo[kFusedMaxF + f] - lo + 1;
      for (int x = tid; x < span * (NR / 4); x += NTH) {
        const int row = x / (NR / 4), c4 = x % (NR / 4);
        *reinterpret_cast<float4*>(pst + used + row * kPsLd + 4 * c4) =
            *reinterpret_cast<const float4*>(P + (f - 1) * a.proj_fstride +
                                             (int64_t)(lo + row) * a.proj_ld + 4 * c4);
      }
      const float4* Ef = reinterpret_cast<const float4*>(
          reinterpret_cast<const float*>(a.E) + (int64_t)lo * ek);
      float4* dst = reinterpret_cast<float4*>(pst + used + span * kPsLd);
      // the copy also forms g[id] = Σ_k Wp_k·E[id][k]² of each staged row (the
      // FM part's Σ_f e_f² term per table row): a row's 4·S0 chunks are
      // consecutive lanes of one wave, summed by a butterfly
      constexpr int CPR = 4 * S0;   // 16-B chunks per bf16 row (k = 32·S0)
      static_assert((CPR & (CPR - 1)) == 0 && CPR <= kWave, "wide DeepFM kernel: k");
      for (int x = tid; x < (PAIRS ? 0 : span * CPR); x += NTH) {
        const int row = x / CPR, c = x % CPR;
        const float4 v = Ef[x];
        dst[row * (ekp / 4) + c] = v;
#if HHFM_WFM
        const uint32_t u4[4] = {__float_as_uint(v.x), __float_as_uint(v.y),
                                __float_as_uint(v.z), __float_as_uint(v.w)};
        const float* wc = wpl + kFusedMaxF + 8 * c;
        float g = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float e0 = __uint_as_float(u4[q] << 16), e1 = __uint_as_float(u4[q] & 0xffff0000u);
          g += e0 * e0 * wc[2 * q];
          g += e1 * e1 * wc[2 * q + 1];
        }
#pragma unroll
        for (int o = CPR / 2; o >= 1; o >>= 1) g += __shfl_xor(g, o, kWave);
        if (c == 0) pst[used + span * (kPsLd + ekp) + row] = g;
#endif
      }
      used += span * (kPsLd + ekp) + (PAIRS ? 0 : ((span + 3) & ~3));
    }
  }
  dma_wait();
  __syncthreads();   // passes 0 and 1, the item rows, the staged rows, the plan

  auto body = [&](auto stc) {
    constexpr bool ST = decltype(stc)::value;
    // layer inputs in B-operand form, one uint4 per (row tile, k32 step)
    uint4 X[RT][TM], Y[RT][TM];
    float y2[RT] = {}, part[RT] = {};
    int pid[RT][F];   // this lane's rows' ids (projected fields)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int f = 1; f < F; ++f) pid[rt][f] = ids[(row0 + 16 * rt) * F + f];
    // staged blocks: LDS float offsets of the rows' P and table rows, and
    // ½ Σ_f g[x_f] of the rows (lane group 0 adds it at the end)
    // (offsets < 40,960 floats: two 16-bit offsets per register, unpacked
    // at each use by volatile asm so the unpacked values are not kept live —
    // the staged kernel runs layer 0 at its 256-register limit)
    static_assert(kPsFloats < 65536, "wide DeepFM kernel: 16-bit LDS offsets");
    uint32_t pbw[(RT + 1) / 2][F] = {}, ebw[(RT + 1) / 2][F] = {};
    float gh[RT] = {};
    if constexpr (ST) {
#pragma unroll
      for (int f = 1; f < F; ++f) {
        const int lo = plo[f], pofs = plo[2 * kFusedMaxF + f], eofs = plo[3 * kFusedMaxF + f];
        const int gofs = plo[4 * kFusedMaxF + f];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          pbw[rt >> 1][f] |= (uint32_t)(pofs + (pid[rt][f] - lo) * kPsLd) << (16 * (rt & 1));
          ebw[rt >> 1][f] |= (uint32_t)(eofs + (pid[rt][f] - lo) * ekp) << (16 * (rt & 1));
          if constexpr (HHFM_WFM && !PAIRS) gh[rt] += pst[gofs + pid[rt][f] - lo];
        }
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) pin(gh[rt]);   // summed here, not at the store
    }
    auto half16 = [](uint32_t w, int hi) -> int {
      uint32_t o;
      if (hi) asm volatile("v_lshrrev_b32 %0, 16, %1" : "=v"(o) : "v"(w));
      else asm volatile("v_and_b32 %0, 0xffff, %1" : "=v"(o) : "v"(w));
      return (int)o;
    };
    auto pbo = [&](int rt, int f) { return half16(pbw[rt >> 1][f], rt & 1); };
    auto ebo = [&](int rt, int f) { return half16(ebw[rt >> 1][f], rt & 1); };

    // FM second-order part (DFM.py:114-122) before layer 0: per k32 step,
    // the item's 8 columns 32s + 8kq .. +7 from its B operand, the other
    // fields' from their rows; lane groups summed at the end
#pragma unroll
    for (int s = 0; s < ((HHFM_WKO & 1) || PAIRS ? 0 : S0); ++s) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const uint4 ex = E0[rt][s];
        const uint32_t x4[4] = {ex.x, ex.y, ex.z, ex.w};
        float fs[8], fq[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v0 = __uint_as_float(x4[q] << 16), v1 = __uint_as_float(x4[q] & 0xffff0000u);
          fs[2 * q] = v0;
          fq[2 * q] = v0 * v0;
          fs[2 * q + 1] = v1;
          fq[2 * q + 1] = v1 * v1;
        }
#pragma unroll
        for (int f2 = 1; f2 < F; ++f2) {
          uint4 u;
          if constexpr (ST)
            u = *reinterpret_cast<const uint4*>(
                reinterpret_cast<const uint16_t*>(pst + ebo(rt, f2)) + 32 * s + 8 * kq);
          else
            u = *reinterpret_cast<const uint4*>(E + (int64_t)pid[rt][f2] * k + 32 * s + 8 * kq);
          const uint32_t u4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float u0 = __uint_as_float(u4[q] << 16), u1 = __uint_as_float(u4[q] & 0xffff0000u);
            fs[2 * q] += u0;
            fs[2 * q + 1] += u1;
            if constexpr (!(ST && HHFM_WFM)) {   // staged rows: Σ_k Wp_k·e_k² from g
              fq[2 * q] += u0 * u0;
              fq[2 * q + 1] += u1 * u1;
            }
          }
        }
        const float4* wc = reinterpret_cast<const float4*>(wpl + kFusedMaxF + 32 * s + 8 * kq);
        const float4 w0 = wc[0], w1 = wc[1];
        const float wq[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        float d = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) d += 0.5f * (fs[q] * fs[q] - fq[q]) * wq[q];
        y2[rt] += d;
        // one step at a time: the fence keeps the loads of later steps below,
        // the pin keeps this step's arithmetic here (otherwise the compiler
        // sinks it to the store at the end and keeps every loaded row live)
        pin(y2[rt]);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // P_f rows of this lane's three rows, units 32t + 16j + 4kq .. +3 (at
    // dfm_proj_pos of the first: 4 contiguous floats), summed into acc
    auto psum = [&](int t, f32x4 (&acc)[RT][2]) {
      const int pos0 = 32 * t + 16 * (kq & 1) + 4 * (kq >> 1);   // j = 0; j = 1: +8
#pragma unroll
      for (int f = 1; f < F; ++f) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const float* pp;
          if constexpr (ST)
            pp = pst + pbo(rt, f) + pos0;
          else
            pp = P + (f - 1) * a.proj_fstride + (int64_t)pid[rt][f] * a.proj_ld + pos0;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float4 x = *reinterpret_cast<const float4*>(pp + 8 * j);
            acc[rt][j][0] += x.x;
            acc[rt][j][1] += x.y;
            acc[rt][j][2] += x.z;
            acc[rt][j][3] += x.w;
          }
        }
      }
    };

    // staged blocks: the P sums of layer-0 pass t+1 are formed during pass t's
    // MFMA steps, unit (field f, row tile rt) in f-major order spread over the
    // steps — per accumulator the same order of additions as psum
    constexpr int kPU = NF * RT;
    auto psum_part = [&](int t, int s, f32x4 (&acc)[RT][2]) {
      const int pos0 = 32 * t + 16 * (kq & 1) + 4 * (kq >> 1);
#pragma unroll
      for (int u = 0; u < kPU; ++u) {
        if (u < s * kPU / S0 || u >= (s + 1) * kPU / S0) continue;
        const int f = 1 + u / RT, rt = u % RT;
        const float* pp = pst + pbo(rt, f) + pos0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float4 x = *reinterpret_cast<const float4*>(pp + 8 * j);
          acc[rt][j][0] += x.x;
          acc[rt][j][1] += x.y;
          acc[rt][j][2] += x.z;
          acc[rt][j][3] += x.w;
        }
      }
    };
    f32x4 accN[RT][2];

    static_for<0, NCH>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      constexpr int layer = p / TM, t = p % TM;
      constexpr int S = layer == 0 ? S0 : TM;
      constexpr int Unext = p + 1 < NCH ? (p + 1 < TM ? 2 * S0 : 2 * TM) : 0;
      if constexpr (p > 0 && !(HHFM_WKO & 4)) vm_barrier<Unext / NWV>();   // pass p landed; slot (p+2)%3 free
      const uint4* wsl = reinterpret_cast<const uint4*>(smem + (p % 3) * kSlotB) + l;
      // this wave's DMAs of pass p+2: units wv, wv+4, ..., one per MFMA step
      const int Udma = p + 2 < NCH && !(HHFM_WKO & 8) ? cunits(p + 2) : 0;
      int dq = wv;
      // the layer's bias (DFM.py:127) is the accumulators' initial value:
      // units 32t + 16j + 4kq .. +3, the same for the three row tiles
      const float* bl = blv + layer * NR + 32 * t + 4 * kq;
      const f32x4 binit[2] = {*reinterpret_cast<const f32x4*>(bl),
                              *reinterpret_cast<const f32x4*>(bl + 16)};
      constexpr bool PI = ST && HHFM_WPI && !(HHFM_WKO & 2);   // interleaved P sums
      f32x4 acc[RT][2];
      if constexpr (layer == 0 && PI && t > 0) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[rt][j] = accN[rt][j];
      } else {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[rt][j] = binit[j];
        if constexpr (layer == 0 && !(HHFM_WKO & 2)) psum(t, acc);
      }
      constexpr bool PN = layer == 0 && PI && t + 1 < TM;   // this pass forms pass t+1's
      if constexpr (PN) {
        const float* bn = blv + 32 * (t + 1) + 4 * kq;
        const f32x4 bnext[2] = {*reinterpret_cast<const f32x4*>(bn),
                                *reinterpret_cast<const f32x4*>(bn + 16)};
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int j = 0; j < 2; ++j) accN[rt][j] = bnext[j];
      }
      // A fragments read from the weight ring two k32 steps ahead (one step
      // ahead: 12.87-12.93 vs 12.80-12.83 ms at C5, profiles/r04_k3w_wpf_ab.txt)
      uint4 fa0 = wsl[0], fa1 = wsl[64];
      uint4 fb0 = fa0, fb1 = fa1;
#ifdef HHFM_WIDE_PF2
      constexpr bool PF2 = HHFM_WIDE_PF2;
#else
      constexpr bool PF2 = RT == 3;   // two waves per SIMD: the other wave covers the LDS latency
#endif
      if (PF2 && S > 1) {
        fb0 = wsl[128];
        fb1 = wsl[192];
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const bf16x8 a0 = __builtin_bit_cast(bf16x8, fa0), a1 = __builtin_bit_cast(bf16x8, fa1);
        if constexpr (PF2) {
          fa0 = fb0;
          fa1 = fb1;
          if (s + 2 < S) {
            fb0 = wsl[128 * (s + 2)];
            fb1 = wsl[128 * (s + 2) + 64];
          }
        } else if (s + 1 < S) {
          fa0 = wsl[128 * (s + 1)];
          fa1 = wsl[128 * (s + 1) + 64];
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          uint4 bx;
          if constexpr (layer == 0)
            bx = E0[rt][s];
          else if constexpr (layer == 1)
            bx = X[rt][s];
          else
            bx = Y[rt][s];
          const bf16x8 b = __builtin_bit_cast(bf16x8, bx);
#if HHFM_WKO & 16
          acc[rt][0][0] += (float)b[0] * (float)a0[0];
          acc[rt][1][0] += (float)b[1] * (float)a1[0];
#else
          acc[rt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b, acc[rt][0], 0, 0, 0);
          acc[rt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b, acc[rt][1], 0, 0, 0);
#endif
        }
        if constexpr (PN) psum_part(t + 1, s, accN);
        if (dq < Udma) {
          dma_unit(p + 2, dq);
          dq += NWV;
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the next fragment reads behind this step
      }
      while (dq < Udma) {
        dma_unit(p + 2, dq);
        dq += NWV;
      }
      if constexpr (layer < 2) {
        // ReLU (DFM.py:128) + bf16: units 32t + 4kq .. +3 and 32t + 16 + 4kq
        // .. +3 are lane group kq's k of step t next layer.  RNE first, then
        // the ReLU on the packed pair as int16 max with 0 (a negative bf16 is
        // a negative int16, and RNE keeps the sign): the same bits as
        // rounding max(x, 0)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const f32x4 c0 = acc[rt][0], c1 = acc[rt][1];
          const uint4 o = make_uint4(relu_bf16x2(pack_bf16x2(c0[0], c0[1])),
                                     relu_bf16x2(pack_bf16x2(c0[2], c0[3])),
                                     relu_bf16x2(pack_bf16x2(c1[0], c1[1])),
                                     relu_bf16x2(pack_bf16x2(c1[2], c1[3])));
          if constexpr (layer == 0)
            X[rt][t] = o;
          else
            Y[rt][t] = o;
          pin(layer == 0 ? X[rt][t] : Y[rt][t]);
        }
      } else {
        const float* vv = vl + 32 * t + 4 * kq;
        const float4 v0 = *reinterpret_cast<const float4*>(vv);
        const float4 v1 = *reinterpret_cast<const float4*>(vv + 16);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const f32x4 c0 = acc[rt][0], c1 = acc[rt][1];
          part[rt] += fmaxf(c0[0], 0.f) * v0.x;
          part[rt] += fmaxf(c0[1], 0.f) * v0.y;
          part[rt] += fmaxf(c0[2], 0.f) * v0.z;
          part[rt] += fmaxf(c0[3], 0.f) * v0.w;
          part[rt] += fmaxf(c1[0], 0.f) * v1.x;
          part[rt] += fmaxf(c1[1], 0.f) * v1.y;
          part[rt] += fmaxf(c1[2], 0.f) * v1.z;
          part[rt] += fmaxf(c1[3], 0.f) * v1.w;
          pin(part[rt]);
        }
      }
    });

    // the lane index formed again here (volatile: not kept live from the
    // prologue — at two waves per SIMD the staged kernel has no register for it)
    int le;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(le));
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float pt = part[rt], yy = y2[rt];
      pt += __shfl_xor(pt, 16, kWave);
      pt += __shfl_xor(pt, 32, kWave);
      yy += __shfl_xor(yy, 16, kWave);
      yy += __shfl_xor(yy, 32, kWave);
      const int row = 16 * RT * wv + (le & 15) + 16 * rt;
      const int64_t m = m0 + row;
      if constexpr (ST && HHFM_WFM && !PAIRS) yy -= 0.5f * gh[rt];   // − ½ Σ_f g[x_f], staged fields
      if (le < 16 && m < a.B) {
        if constexpr (PAIRS) a.out[a.order ? a.order[m] : m] = (HHFM_WFB ? ylds[row] : a.fmbase[m]) + pt;
        else a.out[a.order ? a.order[m] : m] = ((ylds[row] + yy) + a.bp) + pt;
      }
    }
  };
  body(BoolC<!OVF>{});
}

template <int TM, int S0, int NF, bool PAIRS, int RT = 3, int NWV = 4, bool OVF = false>
__global__ __launch_bounds__(NWV * 64, 1) void dfm_fused_w(FusedDfmArgs a, uint32_t* ovf,
                                                           int ovf_rows) {
  constexpr int kWideRows = NWV * 16 * RT;
  if constexpr (!OVF) {
    wide_rows<TM, S0, NF, PAIRS, RT, NWV, false>(a, (int64_t)blockIdx.x * kWideRows, ovf,
                                                 ovf_rows);
  } else {   // grid-stride over the listed units (kWideRows == ovf_rows)
    const uint32_t n = ovf[0];
    for (uint32_t u = blockIdx.x; u < n; u += gridDim.x) {
      __syncthreads();   // the previous unit's LDS reads are done before it is refilled
      wide_rows<TM, S0, NF, PAIRS, RT, NWV, true>(a, (int64_t)ovf[kOvfHead + u] * kWideRows,
                                                  ovf, ovf_rows);
    }
  }
}

// the staged launch, then the overflow launch over the units it listed:
// 4 waves x ORT row tiles (one wave per SIMD), a unit a divisor of the
// staged block; at most one workgroup per CU (the LDS), grid-stride
template <int T, int A, int N, bool PAIRS, int RT, int NWV>
static void wide_launch_rows(const FusedDfmArgs& c, uint32_t* ovf, bool first, hipStream_t st) {
  constexpr int kRowsWG = NWV * 16 * RT;
  constexpr int ORT = kRowsWG % 128 == 0 ? 2 : 1, kRowsOvf = 64 * ORT;
  const int64_t g1 = (c.B + kRowsWG - 1) / kRowsWG, g2 = (c.B + kRowsOvf - 1) / kRowsOvf;
  if (!first) (void)hipMemsetAsync(ovf, 0, sizeof(uint32_t), st);   // (the packing zeroed it)
  hipLaunchKernelGGL((dfm_fused_w<T, A, N, PAIRS, RT, NWV, false>), dim3((unsigned)g1),
                     dim3(NWV * 64), 0, st, c, ovf, kRowsOvf);
  hipLaunchKernelGGL((dfm_fused_w<T, A, N, PAIRS, ORT, 4, true>),
                     dim3((unsigned)(g2 < 256 ? g2 : 256)), dim3(256), 0, st, c, ovf, kRowsOvf);
}

template <int T, int A, int N, int RT, int NWV>
static void wide_launch_shape(const FusedDfmArgs& a, hipStream_t st) {
  constexpr int kRowsWG = NWV * 16 * RT;
  const int64_t units = ((int64_t)T * A * 2 + 2 * (int64_t)T * T * 2) * 64;
  const int pblocks = (int)((units + 255) / 256 < 2048 ? (units + 255) / 256 : 2048);
  // the overflow list after the packed weights, in the rest of the packed
  // workspace (dfm_fused_pack_bytes: ~6.6 MB at C5); rows in chunks whose
  // units always fit it (one chunk below ~200 M rows)
  const size_t wbytes = ((size_t)units * 16 + 255) & ~size_t(255);
  uint32_t* ovf = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(const_cast<uint4*>(a.packed)) +
                                              wbytes);
  hipLaunchKernelGGL(dfm_pack_weights_w, dim3(pblocks), dim3(256), 0, st, a, T, A,
                     const_cast<uint4*>(a.packed), ovf);
  const int64_t cap = ((int64_t)dfm_fused_pack_bytes(a.L, a.dims, true) - (int64_t)wbytes) / 4 -
                      kOvfHead;
  const int64_t chunk = cap / (kRowsWG / 64) * kRowsWG;   // units of >= 64 rows
  const bool pairs = dfm_fm_pairs(a, true, st, !HHFM_WFB);
  for (int64_t r0 = 0; r0 < a.B; r0 += chunk) {
    FusedDfmArgs c = a;
    c.B = a.B - r0 < chunk ? a.B - r0 : chunk;
    c.idx += r0 * a.F;
    if (c.order) c.order += r0;   // out[order[m]]: order holds the caller's rows
    else c.out += r0;
    if (pairs) {
      c.fmbase = a.fm_out + r0;
      wide_launch_rows<T, A, N, true, RT, NWV>(c, ovf, r0 == 0, st);
    } else {
      wide_launch_rows<T, A, N, false, RT, NWV>(c, ovf, r0 == 0, st);
    }
  }
}

bool dfm_wide_launch(const FusedDfmArgs& a, int TM, int32_t plan, hipStream_t st) {
  bool ok = a.L == 3 && a.Fd == 1 && a.k % 32 == 0;
  for (int i = 0; i < 3; ++i) ok = ok && (a.dims[i] + 31) / 32 == TM;
  if (!ok) return false;
  const int S0 = a.k / 32;
  constexpr int kRT = HHFM_WIDE_RT, kNWV = HHFM_WIDE_NWV;
  const int shape = plan & HHFM_PLAN_WIDE_MASK;
  if (TM == 13 && S0 == 8 && a.F == 5) {   // C5: F = 5, k = 256, 3 x 400
    wide_launch_shape<13, 8, 4, kRT, kNWV>(a, st);
    return true;
  }
  if (TM == 5 && S0 == 2 && a.F == 5) {    // tests: F = 5, k = 64, 3 x 150
    if (shape == HHFM_PLAN_WIDE_3X4) wide_launch_shape<5, 2, 4, 3, 4>(a, st);
    else if (shape == HHFM_PLAN_WIDE_2X4) wide_launch_shape<5, 2, 4, 2, 4>(a, st);
    else if (shape == HHFM_PLAN_WIDE_1X4) wide_launch_shape<5, 2, 4, 1, 4>(a, st);
    else wide_launch_shape<5, 2, 4, kRT, kNWV>(a, st);
    return true;
  }
  return false;
}

}  // namespace hhfm
