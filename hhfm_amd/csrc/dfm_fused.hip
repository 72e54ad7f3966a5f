// K3' — DeepFM forward as ONE kernel per 128-row block (bf16 MLP).
//
//   Used by hhfm_dfm_forward / hhfm_dfm_catalog_topk (mlp_gemm.hip) when the
//   MLP runs in bf16, k % 16 == 0, k <= 512, F <= 16, at most 4 layers and
//   every layer at most 416 wide; otherwise the layer-by-layer GEMM path runs.
//   Replaces DeepFM.out (Newcode/DFM.py:104-137) end to end.
//
// Why: the layered path re-gathers the [B, F·k] operand once per 128-column
// tile and round-trips every activation through HBM.  Here a wave owns 32
// rows for the whole network and keeps them in registers:
//
//   * every layer computes the TRANSPOSED product  Yᵀ[n][m] = W[n][:]·Xᵀ[:][m]
//     with v_mfma_f32_32x32x16_bf16 (A = weight rows from LDS, B = the
//     wave's activations), so a result tile has the row m on the lane and
//     the output features n in its 16 registers;
//   * the epilogue (bias, ReLU, bf16 RNE) packs those registers pairwise and
//     one v_permlane32_swap per pair puts them in the next layer's B-operand
//     order (k = 8·half + j) — activations never touch LDS or HBM;
//   * layer 0's B operand is gathered straight from the embedding table into
//     registers one K-chunk ahead, in c-major order (all F fields of one
//     16-column slice in a row), so the same values also give the FM part
//     ½((Σe)²−Σe²)·Wp and the output needs no second pass over E;
//   * dfm_pack_weights first lays all weights out as a sequence of 64-deep
//     K-chunks, each [32·TM rows][8 × 16 B] zero-padded, in the layer-0 step
//     order and already XOR-swizzled, so a chunk is ONE contiguous block:
//     the main kernel streams chunk g+1 into the other half of a double
//     buffer by LDS-DMA (global_load_lds_dwordx4, lane-linear) while the
//     block's 4 waves run chunk g's MFMAs (one barrier a chunk).
//
// All LDS is one __shared__ object: a second object beside the LDS-DMA
// target makes hipcc drain the DMA (vmcnt(0)) before LDS reads.
//
// Projected layer 0 (PROJ = true).  Layer 0 is linear before its ReLU and
// row m's input is the concat of F table rows, so
//   h_0[m] = Σ_f W0[:, f·k:(f+1)·k] · E[x_f]  =  Σ_f P_f[x_f]
// with P_f[id] = W0_f · E[id] computed ONCE per call for every table row
// (dfm_project_layer0: F MFMA GEMMs [M, k] x [k, N0] over the same operands
// as the direct kernel — bf16-rounded for the bf16 MLP, exact fp32 for the
// fp32 MLP — fp32 results; a bf16 P was measured: 7 % faster, and its extra
// rounding moved bf16-MLP catalog rankings past the 5e-3 test bound).  When
// the rows outnumber the table rows (rows >= 2·M; C5 scores 12.5 M rows
// against 5,051 table rows) this removes layer 0's MFMA work (61 % of C5's
// FLOPs) and its weight stream: the kernel gathers F rows of P per row
// straight into the accumulator layout and runs the hidden layers as before.
//
// out[m] = ((Σ_f w[x_f]·Wp[f] + Σ_c y2_c·Wp[F+c]) + bp) + Σ_n relu(h_L)·Wp[F+k+n]
#include <hipcub/hipcub.hpp>

#include "dfm_fused.h"


#if (defined(HHFM_KO_PROJP) || defined(HHFM_KO_PROJFM)) && !defined(HHFM_DIAG_BUILD)
#error "HHFM_KO_PROJP / HHFM_KO_PROJFM give wrong results: diagnostic builds only (-DHHFM_DIAG_BUILD)"
#endif

namespace hhfm {

#ifndef HHFM_F32S_TIMING
#define HHFM_F32S_TIMING 0   // diagnostic build: dfm_fused_f32s per-phase s_memtime sums
#endif
#if HHFM_F32S_TIMING && !defined(HHFM_DIAG_BUILD)
#error "HHFM_F32S_TIMING: diagnostic builds only (-DHHFM_DIAG_BUILD)"
#endif
#if HHFM_F32S_TIMING
// per wave and block: [0] ids + plan loads, [1] item gather issue + spans +
// staging, [2] layer-0 adds, [3] hidden layers, [4] epilogue, [5] blocks x waves
// (scripts/diag/f32s_phases.py)
__device__ unsigned long long g_f32s_t[8];
#define HHFM_F32S_T(x) x
#else
#define HHFM_F32S_T(x)
#endif


constexpr int kFusedRows = 128;   // rows per workgroup (4 waves x 32)

// Chunk g, row n, slot u' holds 8 bf16 of source unit u = u' ^ ((n>>1)&7):
//   layer 0, chunk c:  step S = 4c + u/2 -> W0[n][(S%F)·k + 16(S/F) + 8(u&1) ..]
//   layer i, chunk c:  Wi[n][64c + 8u ..]
// zero outside the layer's rows / columns / steps.
__global__ __launch_bounds__(256) void dfm_pack_weights(FusedDfmArgs a, int TM, int nc0, int NC,
                                                        uint4* __restrict__ out) {
  const int NR = 32 * TM;
  const int Fd = a.Fd;                        // layer-0 K covers the direct fields only
  const int nS = Fd * (a.k / 16);
  const int64_t total = (int64_t)(nc0 + (a.L - 1) * NC) * NR * 8;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(x / (NR * 8));
    const int rem = (int)(x - (int64_t)g * NR * 8);
    const int n = rem >> 3, u = (rem & 7) ^ ((n >> 1) & 7);
    int i, kk;
    bool ok;
    if (g < nc0) {
      i = 0;
      const int S = 4 * g + (u >> 1);
      ok = S < nS;
      kk = (int)((a.perm >> (4 * (S % Fd))) & 15) * a.k + 16 * (S / Fd) + 8 * (u & 1);
    } else {
      i = 1 + (g - nc0) / NC;
      kk = 64 * ((g - nc0) % NC) + 8 * u;
      ok = kk < a.ldb[i];
    }
    ok = ok && n < a.dims[i];
    out[x] = ok ? *reinterpret_cast<const uint4*>(a.Wt[i] + (int64_t)n * a.ldb[i] + kk)
                : make_uint4(0, 0, 0, 0);
  }
}


template <bool TBF, int TM, bool PROJ>
__global__ __launch_bounds__(256, 1) void dfm_fused(FusedDfmArgs a) {
  constexpr int NR = TM * 32;                // weight rows per chunk
  constexpr int CU = NR * 8;                 // 16-B units per chunk
  constexpr int NC = (TM + 1) / 2;           // chunks per hidden layer
  constexpr int kW = 2 * CU * 16;
  constexpr int kIds = kW, kBl = kIds + kFusedRows * kFusedMaxF * 4;
  constexpr int kVl = kBl + kFusedMaxLayers * NR * 4, kWp = kVl + NR * 4;
  constexpr int kPlo = kWp + (kFusedMaxF + kFusedMaxK) * 4;   // PROJ: per-field id span
  // PROJ: the rest of the LDS stages P rows of projected fields whose ids in
  // this block span few table rows (row stride NR + 4 floats: rows of distinct
  // ids start 4 banks apart)
  constexpr int kYl = kPlo + 4 * kFusedMaxF * 4;   // per-row Σ_f w[x_f]·Wp[f]
  constexpr int kPst = kYl + kFusedRows * 4;
  constexpr int kPsLd = NR + 4;
  constexpr int kPsFloats = PROJ ? (kLdsBytes - kPst) / 4 : 0;
  constexpr int kSmem = kPst + kPsFloats * 4;
  static_assert(kSmem <= kLdsBytes, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[kSmem];
  uint4* wbuf0 = reinterpret_cast<uint4*>(smem);   // [2][NR rows][8 slots]
  int32_t* ids = reinterpret_cast<int32_t*>(smem + kIds);
  float* blv = reinterpret_cast<float*>(smem + kBl);  // [layer][NR]
  float* vl = reinterpret_cast<float*>(smem + kVl);
  float* wpl = reinterpret_cast<float*>(smem + kWp);

  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int r = l & 31, h = l >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * kFusedRows;
  const int F = a.F, k = a.k, L = a.L;
  // layer 0 on MFMA over the direct fields [0, Fd); fields [Fd, F) come from P
  const int Fd = PROJ ? a.Fd : F;
  const int nS = Fd * (k / 16);              // layer-0 k16 steps
  const int nc0 = (nS + 3) / 4;              // layer-0 K-chunks (none when all projected)
  const int nchunks = nc0 + (L - 1) * NC;

  for (int x = tid; x < kFusedRows * F; x += 256) {
    const int64_t m = m0 + x / F;
    const int fe = (int)((a.perm >> (4 * (x % F))) & 15);
    ids[x] = m < a.B ? clamp_id(a.idx[m * F + fe], a.M) : 0;
  }
  for (int i = 0; i < L; ++i)
    for (int n = tid; n < NR; n += 256) blv[i * NR + n] = n < a.dims[i] ? a.bias[i][n] : 0.f;
  for (int n = tid; n < NR; n += 256) vl[n] = n < a.dims[L - 1] ? a.Wp[F + k + n] : 0.f;
  // Wp: [0, F) the Σw weights, [kFusedMaxF, +k) the FM columns (16-B aligned)
  for (int x = tid; x < F + k; x += 256)
    wpl[x < F ? x : x - F + kFusedMaxF] = a.Wp[x < F ? (int)((a.perm >> (4 * x)) & 15) : x];
  int* plo = reinterpret_cast<int*>(smem + kPlo);   // [0,16) lo, [16,32) hi, [32,48) LDS base
  if (PROJ && tid < kFusedMaxF) {
    plo[tid] = 0x7fffffff;
    plo[kFusedMaxF + tid] = -1;
  }
  // layer-0 K order is c-major: step S covers field S%F, columns 16(S/F)..+15.
  // Padding steps (S >= nS) multiply zero weights and skip the FM part.

  // chunk g -> LDS buffer b: TM lane-linear 1-KB DMAs per wave
  auto dma = [&](int g, int b) {
    const uint4* src = a.packed + (int64_t)g * CU + 64 * wv + l;
    uint4* dst = wbuf0 + b * CU + 64 * wv;
    // (the asm form pays off where the projected kernels' staged P reads sit
    // between the DMAs and the MFMAs: -1 % there, +1.5 % on the direct kernel)
#pragma unroll
    for (int q = 0; q < TM; ++q) {
      if constexpr (PROJ)
        lds_dma16(src + 256 * q, dst + 256 * q);
      else
        __builtin_amdgcn_global_load_lds((const void*)(src + 256 * q), (void*)(dst + 256 * q),
                                         16, 0, 0);
    }
  };
  // A fragment of tile t, k16 step s of a chunk: row 32t + r, unit 2s + h
  const int swz = (r >> 1) & 7;
  auto wfrag = [&](int b, int t, int s) {
    return __builtin_bit_cast(bf16x8, wbuf0[b * CU + (32 * t + r) * 8 + ((2 * s + h) ^ swz)]);
  };

  // ---- layer-0 operand: gathered embeddings, one chunk ahead in registers ----
  struct EChunk {
    uint4 v[TBF ? 4 : 8];
  };
  const int myrow = 32 * wv + r;
  // layer-0 step cursor (step S: field f = S % F, columns col = 16·(S / F)),
  // advanced incrementally: wave-uniform, so it lives in SGPRs without a
  // division per step
  struct Cur {
    int S, f, col;
  };
  auto adv = [&](Cur& u) {
    ++u.S;
    if (++u.f == Fd) {
      u.f = 0;
      u.col += 16;
    }
  };
  auto eload = [&](EChunk& e, Cur& u) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bool real = u.S < nS;                // padding steps: zero weights
      const int64_t id = ids[myrow * F + (real ? u.f : 0)];
      const int col = (real ? u.col : 0) + 8 * h;
      if constexpr (TBF) {
        e.v[s] = *reinterpret_cast<const uint4*>(
            reinterpret_cast<const uint16_t*>(a.E) + id * k + col);
      } else {
        const uint4* p = reinterpret_cast<const uint4*>(
            reinterpret_cast<const float*>(a.E) + id * k + col);
        e.v[2 * s] = p[0];
        e.v[2 * s + 1] = p[1];
      }
      adv(u);
    }
  };

  __syncthreads();   // ids, step tables visible

  // Projected fields whose ids in this block span few table rows (Frappe's
  // context fields: 7, 2, 3 rows) are staged in LDS, P rows and table rows:
  // the block's id span per field by LDS atomics over its 128 rows (tail rows
  // hold id 0); the body is instantiated twice (staged / HBM) and the block
  // picks one — a runtime select between LDS and HBM addresses would compile
  // to flat loads inside the MFMA loop.
  const int ek = TBF ? k / 2 : k;   // table row in floats
  bool allfit = false;
  if constexpr (PROJ) {
    for (int x = tid; x < kFusedRows * (F - Fd); x += 256) {
      const int row = x / (F - Fd), f = Fd + x % (F - Fd);
      atomicMin(&plo[f], ids[row * F + f]);
      atomicMax(&plo[kFusedMaxF + f], ids[row * F + f]);
    }
    __syncthreads();
    int64_t need = 0;
    for (int f = Fd; f < F; ++f)
      need += (int64_t)(plo[kFusedMaxF + f] - plo[f] + 1) * (kPsLd + ek);
    allfit = need <= kPsFloats;
  }

  auto body = [&](auto stc) {
    constexpr bool ST = decltype(stc)::value;
    // (the projected kernels' first P field initialises the accumulators)
    f32x16 acc[TM];
  #ifndef HHFM_KO_PROJP
    if constexpr (!PROJ)
  #endif
  #pragma unroll
      for (int t = 0; t < TM; ++t)
  #pragma unroll
        for (int x = 0; x < 16; ++x) acc[t][x] = 0.f;
    float fs[8], fq[8];
    float y2 = 0.f;

    // Per K-chunk g (buffer g&1): DMA chunk g+1 into the other buffer (read in
    // chunk g-1, released by its barrier), load the next embedding chunk into
    // the other register set, run chunk g's MFMAs, then vmcnt(0) + barrier
    // (__syncthreads) publishes chunk g+1.

    // One 64-deep chunk from LDS buffer b: the TM weight fragments of step
    // j+1 are read right behind step j's MFMAs (software pipelined; one wave
    // per SIMD has no other wave to hide LDS latency), bop(j) supplies the B
    // operand of step j and side(j) runs beside it.
    auto run_chunk = [&](int b, auto&& bop, auto&& side) {
      bf16x8 fa[TM];
  #pragma unroll
      for (int t = 0; t < TM; ++t) fa[t] = wfrag(b, t, 0);
  #pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 bb = bop(j);
  #pragma unroll
        for (int t = 0; t < TM; ++t) {
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[t], bb, acc[t], 0, 0, 0);
          if (j < 3) fa[t] = wfrag(b, t, j + 1);
          __builtin_amdgcn_sched_barrier(0);   // keep the read right behind its MFMA
        }
        side(j);
      }
    };

    // Everything the block's first MFMA chunk waits for is issued together and
    // met by ONE barrier: layer-0 chunk 0 (weights + gathered embeddings; with
    // every field projected, hidden chunk 0), the staged rows, and the Σw
    // term of the output (one row per thread, all F loads in flight).
    EChunk e0, e1;
    Cur cg{0, 0, 0}, cs{0, 0, 0};   // next gather step, next FM-side step
    const bool direct0 = !PROJ || Fd > 0;
    if (direct0) {
      eload(e0, cg);
      dma(0, 0);
    } else if (nchunks > 0) {
      dma(0, 0);
    }
    float* ylds = reinterpret_cast<float*>(smem + kYl);
    if (tid < kFusedRows) {
      float wv8[kFusedMaxF];
  #pragma unroll
      for (int f = 0; f < kFusedMaxF; ++f) wv8[f] = f < F ? a.w[ids[tid * F + f]] : 0.f;
      float y1 = 0.f;
  #pragma unroll
      for (int f = 0; f < kFusedMaxF; ++f)
        if (f < F) y1 += wv8[f] * wpl[f];
      ylds[tid] = y1;
    }
    if constexpr (PROJ) {
      // ----- ST: the block's projected fields' P rows and table rows, rows
      // lo..hi of each, staged in LDS (read below instead of HBM) -----
      float* pst = reinterpret_cast<float*>(smem + kPst);
      const float* P = reinterpret_cast<const float*>(a.proj);
      if constexpr (ST) {
        int used = 0;
        for (int f = Fd; f < F; ++f) {
          const int lo = plo[f], span = plo[kFusedMaxF + f] - lo + 1;
          for (int x = tid; x < span * (NR / 4); x += 256) {
            const int row = x / (NR / 4), c4 = x % (NR / 4);
            *reinterpret_cast<float4*>(pst + used + row * kPsLd + 4 * c4) =
                *reinterpret_cast<const float4*>(P + (f - Fd) * a.proj_fstride +
                                                 (int64_t)(lo + row) * a.proj_ld + 4 * c4);
          }
          const float4* Ef = reinterpret_cast<const float4*>(
              reinterpret_cast<const float*>(a.E) + (int64_t)lo * ek);
          float4* dst = reinterpret_cast<float4*>(pst + used + span * kPsLd);
          for (int x = tid; x < span * ek / 4; x += 256) dst[x] = Ef[x];
          if (tid == 0) {
            plo[2 * kFusedMaxF + f] = used;                  // P rows
            plo[3 * kFusedMaxF + f] = used + span * kPsLd;   // table rows
          }
          used += span * (kPsLd + ek);
        }
      }
    }
    dma_wait();
    __syncthreads();   // chunk 0, the staged rows and the Σw terms landed
    if constexpr (PROJ) {
      float* pst = reinterpret_cast<float*>(smem + kPst);
      const float* P = reinterpret_cast<const float*>(a.proj);
      // ----- projected layer 0: acc = Σ_{f >= Fd} P_f[x_f]; with Fd == 0 also
      // the FM part from the table (otherwise the direct loop below adds the
      // MFMA part of fields < Fd and the FM part) -----
      // lane (r, h) holds units 32t + 8g + 4h + e of its row (32x32 C/D map):
      // one float4 of P per (field, tile, g); all 4·TM of a field in flight.
      // (Diagnostic knock-outs, never in the product build: HHFM_KO_PROJP /
      // HHFM_KO_PROJFM skip the P / FM loads — scripts/build_variants.sh.)
  #ifndef HHFM_KO_PROJP
      // P in accumulator order: positions 32t + 16h .. +15 are this lane's
      // units of tile t (64 contiguous bytes), from LDS when staged; all 4·TM
      // reads of a field in flight (a tile-outer order, each tile's fields
      // summed in registers first, ran 6 % slower).  The first field is
      // written, the others added (an accumulator add is a read-modify-write
      // of an AGPR).
      auto addp = [&](const float4* pp, auto first) {
  #pragma unroll
        for (int t = 0; t < TM; ++t)
  #pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float4 x = pp[8 * t + g4];
            if constexpr (decltype(first)::value) {
              acc[t][4 * g4 + 0] = x.x;
              acc[t][4 * g4 + 1] = x.y;
              acc[t][4 * g4 + 2] = x.z;
              acc[t][4 * g4 + 3] = x.w;
            } else {
              acc[t][4 * g4 + 0] += x.x;
              acc[t][4 * g4 + 1] += x.y;
              acc[t][4 * g4 + 2] += x.z;
              acc[t][4 * g4 + 3] += x.w;
            }
          }
      };
      auto prow = [&](int f) {
        if constexpr (ST)
          return reinterpret_cast<const float4*>(pst + plo[2 * kFusedMaxF + f] +
                                                 (ids[myrow * F + f] - plo[f]) * kPsLd) +
                 4 * h;
        else
          return reinterpret_cast<const float4*>(P + (f - Fd) * a.proj_fstride +
                                                 (int64_t)ids[myrow * F + f] * a.proj_ld) +
                 4 * h;
      };
      addp(prow(Fd), BoolC<true>{});   // Fd < F whenever P is planned
      for (int f = Fd + 1; f < F; ++f) addp(prow(f), BoolC<false>{});
  #endif
      // FM second-order part (DFM.py:114-122): the lane half h takes columns
      // 16j + 8h .. +7 of every 16-column block j, as the direct kernel's side()
      for (int j = 0; j < (Fd == 0 ? k / 16 : 0); ++j) {
  #ifndef HHFM_KO_PROJFM
        float s8[8], q8[8];
  #pragma unroll
        for (int q = 0; q < 8; ++q) { s8[q] = 0.f; q8[q] = 0.f; }
        for (int f = 0; f < F; ++f) {
          const int64_t id = ids[myrow * F + f];
          float v[8];
          if constexpr (TBF) {
            const uint4 x = *reinterpret_cast<const uint4*>(
                reinterpret_cast<const uint16_t*>(a.E) + id * k + 16 * j + 8 * h);
            const uint32_t x4[4] = {x.x, x.y, x.z, x.w};
  #pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[2 * q] = __uint_as_float(x4[q] << 16);
              v[2 * q + 1] = __uint_as_float(x4[q] & 0xffff0000u);
            }
          } else {
            const float4* p = reinterpret_cast<const float4*>(
                reinterpret_cast<const float*>(a.E) + id * k + 16 * j + 8 * h);
            const float4 p0 = p[0], p1 = p[1];
            v[0] = p0.x; v[1] = p0.y; v[2] = p0.z; v[3] = p0.w;
            v[4] = p1.x; v[5] = p1.y; v[6] = p1.z; v[7] = p1.w;
          }
  #pragma unroll
          for (int q = 0; q < 8; ++q) {
            s8[q] += v[q];
            q8[q] += v[q] * v[q];
          }
        }
        const float4* wc = reinterpret_cast<const float4*>(wpl + kFusedMaxF + 16 * j + 8 * h);
        const float4 w0 = wc[0], w1 = wc[1];
        const float wq[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        float d = 0.f;
  #pragma unroll
        for (int q = 0; q < 8; ++q) d += 0.5f * (s8[q] * s8[q] - q8[q]) * wq[q];
        y2 += d;
  #endif
      }
    }
    if (direct0) {

    // ----- layer 0: B operand = gathered embeddings; FM part on the side -----
    // Chunk c first turns the embeddings gathered during chunk c-1 into its 4
    // B operands (and the fp32 values of the FM part), THEN issues chunk c+1's
    // weight DMA and gathers into the freed registers: the compiler's wait on
    // the gathered registers (it cannot count loads across the loop's back
    // edge, so it is a vmcnt(0)) then lands before the new loads, not after.
    auto chunk0 = [&](int c, EChunk& e, EChunk& en) {
      const int b = c & 1;
      float v[4][8];
      uint4 bxs[4];
  #pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (TBF) {
          bxs[j] = e.v[j];   // already the B operand; fp32 values made per step
        } else {
          const uint4 p = e.v[2 * j], q = e.v[2 * j + 1];
          v[j][0] = __uint_as_float(p.x); v[j][1] = __uint_as_float(p.y);
          v[j][2] = __uint_as_float(p.z); v[j][3] = __uint_as_float(p.w);
          v[j][4] = __uint_as_float(q.x); v[j][5] = __uint_as_float(q.y);
          v[j][6] = __uint_as_float(q.z); v[j][7] = __uint_as_float(q.w);
          bxs[j] = make_uint4(pack_bf16x2(v[j][0], v[j][1]), pack_bf16x2(v[j][2], v[j][3]),
                              pack_bf16x2(v[j][4], v[j][5]), pack_bf16x2(v[j][6], v[j][7]));
        }
      }
      // then the next chunk's weight DMA and gathers, in one burst
      // (measured: placing them one per MFMA gap instead ran 6-7 % slower)
      if (c + 1 < nchunks) dma(c + 1, b ^ 1);
      if (c + 1 < nc0) eload(en, cg);
      auto bop = [&](int j) {
        if constexpr (TBF) {
          const uint32_t x4[4] = {bxs[j].x, bxs[j].y, bxs[j].z, bxs[j].w};
  #pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[j][2 * q] = __uint_as_float(x4[q] << 16);
            v[j][2 * q + 1] = __uint_as_float(x4[q] & 0xffff0000u);
          }
        }
        return __builtin_bit_cast(bf16x8, bxs[j]);
      };
      // FM second-order part over the same values (DFM.py:114-122)
      auto side = [&](int j) {
        const int f = cs.S < nS ? cs.f : -1;
        if (f == 0) {
  #pragma unroll
          for (int q = 0; q < 8; ++q) { fs[q] = 0.f; fq[q] = 0.f; }
        }
  #pragma unroll
        for (int q = 0; q < 8; ++q) {
          fs[q] += v[j][q];
          fq[q] += v[j][q] * v[j][q];
        }
        if (f == Fd - 1) {   // (a branch-free form, evaluated every step, ran 11 % slower)
          if constexpr (PROJ) {
            // the projected fields' values of these 8 columns (their rows are
            // few and cache-resident: Frappe's contexts)
            for (int f2 = Fd; f2 < F; ++f2) {
              const int64_t id2 = ids[myrow * F + f2];
              const int eb = plo[3 * kFusedMaxF + f2];   // ST: staged, no HBM round trip
              float u8[8];
              if constexpr (TBF) {
                uint4 x;
                if constexpr (ST)
                  x = *reinterpret_cast<const uint4*>(
                      reinterpret_cast<const uint16_t*>(smem + kPst + 4 * eb) +
                      (id2 - plo[f2]) * k + cs.col + 8 * h);
                else
                  x = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(a.E) +
                                                      id2 * k + cs.col + 8 * h);
                const uint32_t x4[4] = {x.x, x.y, x.z, x.w};
  #pragma unroll
                for (int qq = 0; qq < 4; ++qq) {
                  u8[2 * qq] = __uint_as_float(x4[qq] << 16);
                  u8[2 * qq + 1] = __uint_as_float(x4[qq] & 0xffff0000u);
                }
              } else {
                float4 p0, p1;
                if constexpr (ST) {
                  const float4* p2 = reinterpret_cast<const float4*>(
                      reinterpret_cast<const float*>(smem + kPst + 4 * eb) + (id2 - plo[f2]) * k +
                      cs.col + 8 * h);
                  p0 = p2[0];
                  p1 = p2[1];
                } else {
                  const float4* p2 = reinterpret_cast<const float4*>(
                      reinterpret_cast<const float*>(a.E) + id2 * k + cs.col + 8 * h);
                  p0 = p2[0];
                  p1 = p2[1];
                }
                u8[0] = p0.x; u8[1] = p0.y; u8[2] = p0.z; u8[3] = p0.w;
                u8[4] = p1.x; u8[5] = p1.y; u8[6] = p1.z; u8[7] = p1.w;
              }
  #pragma unroll
              for (int qq = 0; qq < 8; ++qq) {
                fs[qq] += u8[qq];
                fq[qq] += u8[qq] * u8[qq];
              }
            }
          }
          const float4* wc =
              reinterpret_cast<const float4*>(wpl + kFusedMaxF + cs.col + 8 * h);
          const float4 w0 = wc[0], w1 = wc[1];
          const float wq[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
          float d = 0.f;
  #pragma unroll
          for (int q = 0; q < 8; ++q) d += 0.5f * (fs[q] * fs[q] - fq[q]) * wq[q];
          y2 += d;
        }
        adv(cs);
      };
      run_chunk(b, bop, side);
      dma_wait();
      __syncthreads();   // chunk c+1's weights and embeddings landed
    };
    // (two register sets alternate, so no copy of the gathered chunk is needed
    // on the loop's back edge)
    for (int c = 0; c < nc0; c += 2) {
      chunk0(c, e0, e1);
      if (c + 1 < nc0) chunk0(c + 1, e1, e0);
    }
    }   // direct layer 0

    // ----- layers 1..L-1: B operand = the previous layer's output, in registers -----
    uint32_t X[TM][8];
    int g = nc0;
    for (int i = 1; i < L; ++i) {
      // epilogue of layer i-1: bias + ReLU (DFM.py:127-128, every layer), bf16,
      // then into B-operand order (k = 8*half + j) with one swap per pair
      const float* bli = blv + (i - 1) * NR;
  #pragma unroll
      for (int t = 0; t < TM; ++t) {
        float v[16];
  #pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 bq = *reinterpret_cast<const float4*>(bli + 32 * t + 8 * g4 + 4 * h);
          const float bv[4] = {bq.x, bq.y, bq.z, bq.w};
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[4 * g4 + e] = fmaxf(acc[t][4 * g4 + e] + bv[e], 0.f);
            acc[t][4 * g4 + e] = 0.f;
          }
        }
  #pragma unroll
        for (int q = 0; q < 8; ++q) X[t][q] = pack_bf16x2(v[2 * q], v[2 * q + 1]);
        swap_halves(X[t][0], X[t][2]);
        swap_halves(X[t][1], X[t][3]);
        swap_halves(X[t][4], X[t][6]);
        swap_halves(X[t][5], X[t][7]);
      }
  #pragma unroll
      for (int c = 0; c < NC; ++c, ++g) {
        const int b = g & 1;
        if (g + 1 < nchunks) dma(g + 1, b ^ 1);
        auto bop = [&](int j) {   // step j = input tile 2c + j/2, k16 half j%2
          const int tin = 2 * c + (j >> 1), s2 = 4 * (j & 1);
          const uint4 bx = tin < TM ? make_uint4(X[tin][s2], X[tin][s2 + 1], X[tin][s2 + 2],
                                                 X[tin][s2 + 3])
                                    : make_uint4(0, 0, 0, 0);
          return __builtin_bit_cast(bf16x8, bx);
        };
        run_chunk(b, bop, [](int) {});
        dma_wait();
        __syncthreads();
      }
    }

    // ---- last layer: relu(acc + b) · Wp_deep, FM part, bias terms ----
    const float* blL = blv + (L - 1) * NR;
    float part = 0.f;
  #pragma unroll
    for (int t = 0; t < TM; ++t)
  #pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int n = 32 * t + 8 * g4 + 4 * h;
        const float4 bq = *reinterpret_cast<const float4*>(blL + n);
        const float4 vq = *reinterpret_cast<const float4*>(vl + n);
        part += fmaxf(acc[t][4 * g4 + 0] + bq.x, 0.f) * vq.x;
        part += fmaxf(acc[t][4 * g4 + 1] + bq.y, 0.f) * vq.y;
        part += fmaxf(acc[t][4 * g4 + 2] + bq.z, 0.f) * vq.z;
        part += fmaxf(acc[t][4 * g4 + 3] + bq.w, 0.f) * vq.w;
      }
    part += __shfl_xor(part, 32, kWave);
    y2 += __shfl_xor(y2, 32, kWave);
    const int64_t m = m0 + myrow;
    if (h == 0 && m < a.B) a.out[a.order ? a.order[m] : m] = ((ylds[myrow] + y2) + a.bp) + part;
  };
  if constexpr (PROJ) {
    if (allfit) body(BoolC<true>{});
    else body(BoolC<false>{});
  } else {
    body(BoolC<false>{});
  }
}

// ---------------------------------------------------------------------------
// fp32 MLP (the reference numerics): v_mfma_f32_16x16x4_f32 (exact fp32
// products, fp32 accumulation), 4 waves x 16 rows per workgroup (16-row
// tiles: 32x32 ones would need 208 accumulator + 208 activation registers
// per lane at 416 units, beyond one wave's 512).  Each lane group kq = lane/16 supplies
// 4 consecutive k of every 16-k step (one 16-B gather / weight unit feeds 4
// MFMAs), and a 16x16 result tile holds, per lane group q, units 4q..4q+3 —
// exactly the k a lane group supplies in the next layer, so a layer's fp32
// output IS the next layer's B operand in registers, no reordering.  Chunks
// are 32 k deep; layer 0 runs its 16-column blocks field-minor (c-major).
// ---------------------------------------------------------------------------
constexpr int kF32Waves = 4;
constexpr int kF32Rows = kF32Waves * 16;   // rows per workgroup

__global__ __launch_bounds__(256) void dfm_pack_weights_f32(FusedDfmArgs a, int TM, int nc0,
                                                            uint4* __restrict__ out) {
  const int NR = 32 * TM;
  const int nB = a.F * (a.k / 16);            // layer-0 16-column blocks
  const int64_t total = (int64_t)(nc0 + (a.L - 1) * TM) * NR * 8;
  const float* const* Wf = reinterpret_cast<const float* const*>(a.Wt);
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(x / (NR * 8));
    const int rem = (int)(x - (int64_t)g * NR * 8);
    const int n = rem >> 3, u = (rem & 7) ^ ((n >> 1) & 7);
    int i, kk;
    bool ok;
    if (g < nc0) {   // chunk = 2 blocks of 16 columns, unit u = (block u/4, quarter u%4)
      i = 0;
      const int b = 2 * g + (u >> 2);
      ok = b < nB;
      kk = (b % a.F) * a.k + 16 * (b / a.F) + 4 * (u & 3);
    } else {
      i = 1 + (g - nc0) / TM;
      kk = 32 * ((g - nc0) % TM) + 4 * u;
      ok = kk < a.ldb[i];
    }
    ok = ok && n < a.dims[i];
    out[x] = ok ? *reinterpret_cast<const uint4*>(Wf[i] + (int64_t)n * a.ldb[i] + kk)
                : make_uint4(0, 0, 0, 0);
  }
}

template <bool TBF, int TM, bool PROJ>
__global__ __launch_bounds__(256, 1) void dfm_fused_f32(FusedDfmArgs a) {
  constexpr int NR = TM * 32;
  constexpr int T16 = 2 * TM;                // 16-unit output tiles
  constexpr int CU = NR * 8;
  constexpr int kMaxBlocks = kFusedMaxF * kFusedMaxK / 16 + 2;
  constexpr int kW = 2 * CU * 16;
  constexpr int kIds = kW, kBl = kIds + kF32Rows * kFusedMaxF * 4;
  constexpr int kVl = kBl + kFusedMaxLayers * NR * 4, kWp = kVl + NR * 4;
  constexpr int kSf = kWp + (kFusedMaxF + kFusedMaxK) * 4, kSc = kSf + kMaxBlocks * 4;
  constexpr int kSmem = kSc + kMaxBlocks * 4;
  __shared__ __attribute__((aligned(16))) char smem[kSmem];   // ONE LDS object
  uint4* wbuf0 = reinterpret_cast<uint4*>(smem);
  int32_t* ids = reinterpret_cast<int32_t*>(smem + kIds);
  float* blv = reinterpret_cast<float*>(smem + kBl);
  float* vl = reinterpret_cast<float*>(smem + kVl);
  float* wpl = reinterpret_cast<float*>(smem + kWp);
  int32_t* blk_f = reinterpret_cast<int32_t*>(smem + kSf);
  int32_t* blk_col = reinterpret_cast<int32_t*>(smem + kSc);

  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int r = l & 15, kq = l >> 4;         // row in the wave's 16 / k quarter
  const int64_t m0 = (int64_t)blockIdx.x * kF32Rows;
  const int F = a.F, k = a.k, L = a.L;
  const int nB = F * (k / 16);
  const int nc0 = PROJ ? 0 : (nB + 1) / 2;
  const int nchunks = nc0 + (L - 1) * TM;

  for (int x = tid; x < kF32Rows * F; x += 256) {
    const int64_t m = m0 + x / F;
    ids[x] = m < a.B ? clamp_id(a.idx[m * F + x % F], a.M) : 0;
  }
  for (int i = 0; i < L; ++i)
    for (int n = tid; n < NR; n += 256) blv[i * NR + n] = n < a.dims[i] ? a.bias[i][n] : 0.f;
  for (int n = tid; n < NR; n += 256) vl[n] = n < a.dims[L - 1] ? a.Wp[F + k + n] : 0.f;
  for (int x = tid; x < F + k; x += 256) wpl[x] = a.Wp[x];
  for (int b = tid; b < 2 * nc0; b += 256) {
    blk_f[b] = b < nB ? b % F : -1;
    blk_col[b] = b < nB ? 16 * (b / F) : 0;
  }

  // chunk g -> buffer b: CU/64 lane-linear 1-KB DMAs spread over 8 waves
  auto dma = [&](int g, int b) {
    const uint4* src = a.packed + (int64_t)g * CU;
    uint4* dst = wbuf0 + b * CU;
#pragma unroll
    for (int q = 0; q < (TM * 4 + kF32Waves - 1) / kF32Waves; ++q) {
      const int ins = wv + kF32Waves * q;      // 1-KB piece (TM*4 of them)
      if (ins < TM * 4)
        __builtin_amdgcn_global_load_lds((const void*)(src + 64 * ins + l),
                                         (void*)(dst + 64 * ins), 16, 0, 0);
    }
  };
  // A fragment: output unit 16*t + r, 16-B weight unit u of the chunk
  auto wfrag = [&](int b, int t, int u) {
    const int row = 16 * t + r;
    return __builtin_bit_cast(float4, wbuf0[b * CU + row * 8 + (u ^ ((row >> 1) & 7))]);
  };

  struct EChunk {
    float4 v[2];
  };
  const int myrow = 16 * wv + r;
  auto eload = [&](EChunk& e, int c) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int b = 2 * c + q;
      const int f = blk_f[b];
      const int64_t id = ids[myrow * F + (f >= 0 ? f : 0)];
      const int col = blk_col[b] + 4 * kq;
      if constexpr (TBF) {
        const uint2 x = *reinterpret_cast<const uint2*>(
            reinterpret_cast<const uint16_t*>(a.E) + id * k + col);
        e.v[q] = make_float4(__uint_as_float(x.x << 16), __uint_as_float(x.x & 0xffff0000u),
                             __uint_as_float(x.y << 16), __uint_as_float(x.y & 0xffff0000u));
      } else {
        e.v[q] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.E) + id * k +
                                                  col);
      }
    }
  };

  f32x4 acc[T16];
#pragma unroll
  for (int t = 0; t < T16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float fs[4], fq[4];
  float y2 = 0.f;

  __syncthreads();

  // one 16-k step (weight units 4s..4s+3 of the chunk; lane group kq takes
  // unit 4s+kq): 4 MFMAs per output tile, next tile's fragment read ahead
  auto step = [&](int b, int s, const float (&bv)[4]) {
    float4 fa = wfrag(b, 0, 4 * s + kq);
#pragma unroll
    for (int t = 0; t < T16; ++t) {
      const float4 cur = fa;
      if (t + 1 < T16) fa = wfrag(b, t + 1, 4 * s + kq);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x, bv[0], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.y, bv[1], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.z, bv[2], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.w, bv[3], acc[t], 0, 0, 0);
    }
  };

  if constexpr (PROJ) {
    // ----- projected layer 0: acc = Σ_f P_f[x_f] (16x16 C/D map: lane group
    // kq holds units 16t + 4kq .. +3 of its row), FM part from the table -----
    if (nchunks > 0) dma(0, 0);
    for (int f = 0; f < F; ++f) {
      const float4* pp = reinterpret_cast<const float4*>(
                             reinterpret_cast<const float*>(a.proj) + f * a.proj_fstride +
                             (int64_t)ids[myrow * F + f] * a.proj_ld) + kq;
#pragma unroll
      for (int t = 0; t < T16; ++t) {
        const float4 x = pp[4 * t];
        acc[t][0] += x.x;
        acc[t][1] += x.y;
        acc[t][2] += x.z;
        acc[t][3] += x.w;
      }
    }
    // FM second-order part (DFM.py:114-122), columns 16j + 4kq .. +3 of every
    // 16-column block j, summed as the direct kernel does
    for (int j = 0; j < k / 16; ++j) {
#pragma unroll
      for (int x = 0; x < 4; ++x) { fs[x] = 0.f; fq[x] = 0.f; }
      for (int f = 0; f < F; ++f) {
        const int64_t id = ids[myrow * F + f];
        float bv[4];
        if constexpr (TBF) {
          const uint2 x = *reinterpret_cast<const uint2*>(
              reinterpret_cast<const uint16_t*>(a.E) + id * k + 16 * j + 4 * kq);
          bv[0] = __uint_as_float(x.x << 16); bv[1] = __uint_as_float(x.x & 0xffff0000u);
          bv[2] = __uint_as_float(x.y << 16); bv[3] = __uint_as_float(x.y & 0xffff0000u);
        } else {
          const float4 x = *reinterpret_cast<const float4*>(
              reinterpret_cast<const float*>(a.E) + id * k + 16 * j + 4 * kq);
          bv[0] = x.x; bv[1] = x.y; bv[2] = x.z; bv[3] = x.w;
        }
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          fs[x] += bv[x];
          fq[x] += bv[x] * bv[x];
        }
      }
      const float* wc = wpl + F + 16 * j + 4 * kq;
#pragma unroll
      for (int x = 0; x < 4; ++x) y2 += 0.5f * (fs[x] * fs[x] - fq[x]) * wc[x];
    }
    __syncthreads();   // vmcnt(0): hidden chunk 0 landed
  } else {
  EChunk ea, eb;
  eload(ea, 0);
  dma(0, 0);
  __syncthreads();

  // ----- layer 0 -----
  auto chunk0 = [&](int c, EChunk& e, EChunk& en) {
    const int b = c & 1;
    if (c + 1 < nchunks) dma(c + 1, b ^ 1);
    if (c + 1 < nc0) eload(en, c + 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float bv[4] = {e.v[q].x, e.v[q].y, e.v[q].z, e.v[q].w};
      step(b, q, bv);
      // FM second-order part (DFM.py:114-122) over the same fp32 values
      const int B = 2 * c + q;
      const int f = blk_f[B];
      if (f == 0) {
#pragma unroll
        for (int x = 0; x < 4; ++x) { fs[x] = 0.f; fq[x] = 0.f; }
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        fs[x] += bv[x];
        fq[x] += bv[x] * bv[x];
      }
      if (f == F - 1) {
        const float* wc = wpl + F + blk_col[B] + 4 * kq;
#pragma unroll
        for (int x = 0; x < 4; ++x) y2 += 0.5f * (fs[x] * fs[x] - fq[x]) * wc[x];
      }
    }
    __syncthreads();
  };
  for (int c = 0; c < nc0; c += 2) {
    chunk0(c, ea, eb);
    if (c + 1 < nc0) chunk0(c + 1, eb, ea);
  }
  }   // direct layer 0

  // ----- layers 1..L-1: the previous layer's fp32 output is the B operand -----
  f32x4 X[T16];
  int g = nc0;
  for (int i = 1; i < L; ++i) {
    const float* bli = blv + (i - 1) * NR;
#pragma unroll
    for (int t = 0; t < T16; ++t) {
#pragma unroll
      for (int x = 0; x < 4; ++x)   // relu after every layer (DFM.py:128)
        X[t][x] = fmaxf(acc[t][x] + bli[16 * t + 4 * kq + x], 0.f);
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int c = 0; c < TM; ++c, ++g) {   // chunk c = input tiles 2c, 2c+1
      const int b = g & 1;
      if (g + 1 < nchunks) dma(g + 1, b ^ 1);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float bv[4] = {X[2 * c + s][0], X[2 * c + s][1], X[2 * c + s][2], X[2 * c + s][3]};
        step(b, s, bv);
      }
      __syncthreads();
    }
  }

  const float* blL = blv + (L - 1) * NR;
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < T16; ++t)
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int n = 16 * t + 4 * kq + x;
      part += fmaxf(acc[t][x] + blL[n], 0.f) * vl[n];
    }
  part += __shfl_xor(part, 16, kWave);
  part += __shfl_xor(part, 32, kWave);
  const int64_t m = m0 + myrow;
  y2 += __shfl_xor(y2, 16, kWave);
  y2 += __shfl_xor(y2, 32, kWave);
  if (kq == 0 && m < a.B) {
    float y1 = 0.f;
    for (int f = 0; f < F; ++f) y1 += a.w[ids[myrow * F + f]] * wpl[f];
    a.out[m] = ((y1 + y2) + a.bp) + part;
  }
}

// ---------------------------------------------------------------------------
// fp32 MLP with the hidden layers on split-bf16 MFMA (PROJ only: layer 0 is
// the fp32 P gather above).  Every fp32 operand is split into three bf16
// pieces, x = x0 + x1 + x2 exactly (split3x8), and each 32-k step of a
// 16-unit output tile runs the six piece products of order >= 2^-16 on
// v_mfma_f32_16x16x32_bf16, smallest first (w2x0, w1x1, w0x2, w1x0, w0x1,
// w0x0): products exact in fp32, fp32 accumulation, the dropped products
// below 2^-24 relative — fp32-faithful, the same contract as K2's split
// kernels.  6 x 16 cycles per 32 k instead of 8 x 32 for 16x16x4_f32.
//   * B operand: the layer input X stays fp32 in registers in the 16x16
//     C/D layout (lane group kq holds units 16t + 4kq .. +3); a 32-k step c
//     takes lane group kq's 8 k as {32c + 4kq .. +3, 32c + 16 + 4kq .. +3} —
//     the k order inside a step is free as long as A uses the same — and
//     splits them once per step for all 2·TM output tiles;
//   * A operand: dfm_pack_weights_f32s pre-splits the weights once per call
//     into half-chunks [piece][tile][kq][16 rows][8 bf16] (one 32-k step,
//     half the output units; a tile's fragment read is 1 KB contiguous and
//     each 16-lane group reads 256 consecutive bytes), padded to
//     a multiple of 4 KB so every wave issues the same number of LDS-DMAs;
//   * a 3-slot LDS ring, filled two half-chunks ahead by lane-linear LDS-DMA;
//     one counted vmcnt + s_barrier per half-chunk.
// ---------------------------------------------------------------------------
template <int TM, int NW>
struct F32sCfg {
  static constexpr int HR = 16 * TM;                          // rows of a half-chunk
  static constexpr int PlaneB = HR * 64;                      // one piece plane
  static constexpr int SlotB = (3 * PlaneB + 8191) / 8192 * 8192;
  static constexpr int kDmaW = SlotB / (1024 * NW);           // DMA instructions per wave
  static constexpr int kRows = 16 * NW;                       // rows per workgroup
};

__host__ __device__ static inline int f32s_slot_bytes(int TM) {
  return (3 * 16 * TM * 64 + 8191) / 8192 * 8192;
}

__global__ __launch_bounds__(256) void dfm_pack_weights_f32s(FusedDfmArgs a, int TM,
                                                             char* __restrict__ out) {
  const int HR = 16 * TM, PlaneB = HR * 64, SlotB = f32s_slot_bytes(TM);
  const int64_t total = (int64_t)(a.L - 1) * TM * 2 * HR * 4;
  const float* const* Wf = reinterpret_cast<const float* const*>(a.Wt);
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int blk = (int)(x / (HR * 4));
    const int rem = (int)(x - (int64_t)blk * HR * 4);
    const int nl = rem >> 2, kq = rem & 3;
    const int i = 1 + blk / (2 * TM), c = (blk >> 1) % TM, hh = blk & 1;
    const int n = HR * hh + nl;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = 32 * c + (j < 4 ? 4 * kq + j : 16 + 4 * kq + j - 4);
      v[j] = (n < a.dims[i] && kk < a.ldb[i]) ? Wf[i][(int64_t)n * a.ldb[i] + kk] : 0.f;
    }
    bf16x8 p0, p1, p2;
    split3x8(v, p0, p1, p2);
    // [piece][tile][kq][row in tile] x 16 B: the 16 lanes of one kq read 256
    // consecutive bytes (conflict-free ds_read_b128)
    char* base = out + (int64_t)blk * SlotB + (nl >> 4) * 1024 + kq * 256 + (nl & 15) * 16;
    *reinterpret_cast<bf16x8*>(base) = p0;
    *reinterpret_cast<bf16x8*>(base + PlaneB) = p1;
    *reinterpret_cast<bf16x8*>(base + 2 * PlaneB) = p2;
  }
}

// NW waves x 16 rows per workgroup: 8 waves (two per SIMD, 128 rows) halve
// the weight bytes per row against 4 and let one wave's LDS-DMA issue and
// barrier wait overlap the other's MFMAs; each wave keeps acc (104) + X (104)
// within the 256 registers two waves per SIMD leave it.
template <bool TBF, int TM, int NW>
__global__ __launch_bounds__(NW * 64, 1) void dfm_fused_f32s(FusedDfmArgs a) {
  using Cfg = F32sCfg<TM, NW>;
  constexpr int NR = TM * 32;
  constexpr int T16 = 2 * TM;                // 16-unit output tiles
  constexpr int NT = NW * 64;
  constexpr int kIds = 3 * Cfg::SlotB, kBl = kIds + Cfg::kRows * kFusedMaxF * 4;
  constexpr int kVl = kBl + kFusedMaxLayers * NR * 4;
  constexpr int kSpan = kVl + NR * 4;        // [F] lo, [F] hi, [F] staged row base
  constexpr int kSmem = kSpan + 3 * kFusedMaxF * 4;
  static_assert(kSmem <= kLdsBytes, "split fp32 DeepFM kernel: LDS");
  // P rows staged in ring slot 2 (free until the first hidden half-chunk),
  // padded by one 16-B chunk per row against bank conflicts
  constexpr int kPRowB = NR * 4 + 16;
  constexpr int kStageRows = Cfg::SlotB / kPRowB;
  __shared__ __attribute__((aligned(16))) char smem[kSmem];   // ONE LDS object
  int32_t* ids = reinterpret_cast<int32_t*>(smem + kIds);
  float* blv = reinterpret_cast<float*>(smem + kBl);
  float* vl = reinterpret_cast<float*>(smem + kVl);
  int32_t* plo = reinterpret_cast<int32_t*>(smem + kSpan);
  int32_t* phi = plo + kFusedMaxF;
  int32_t* psb = phi + kFusedMaxF;

  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int r = l & 15, kq = l >> 4;
  const int64_t m0 = (int64_t)blockIdx.x * Cfg::kRows;
  const int F = a.F, k = a.k, L = a.L;
  const int H = (L - 1) * TM * 2;            // hidden half-chunks
  HHFM_F32S_T(uint64_t tq[6]; tq[0] = __builtin_amdgcn_s_memtime();)

  for (int x = tid; x < Cfg::kRows * F; x += NT) {
    const int64_t m = m0 + x / F;
    ids[x] = m < a.B ? clamp_id(a.idx[m * F + x % F], a.M) : 0;
  }
  for (int i = 0; i < L; ++i)
    for (int n = tid; n < NR; n += NT) blv[i * NR + n] = n < a.dims[i] ? a.bias[i][n] : 0.f;
  for (int n = tid; n < NR; n += NT) vl[n] = n < a.dims[L - 1] ? a.Wp[F + k + n] : 0.f;
  if (tid < F) {
    plo[tid] = 0x7fffffff;
    phi[tid] = -1;
  }
  __syncthreads();
  HHFM_F32S_T(tq[1] = __builtin_amdgcn_s_memtime();)
  const int myrow = 16 * wv + r;
  f32x4 X[T16];
  // field 1 (the item: its ids span the whole catalog, it is never staged)
  // is gathered into X now, in flight through the span / staging prologue;
  // X = P_1 + P_0 + P_2 + ... equals the in-order sum bit for bit (IEEE
  // addition commutes, and 0 + P_0 = P_0); C5 fp32 38.84 -> 38.70 ms
  // (profiles/r04_k3_f32_pre_ab.txt)
  constexpr int kPre = 1;
  const bool pre = F > kPre;
  if (pre) {
    const int id = ids[myrow * F + kPre];
    const float4* pp = reinterpret_cast<const float4*>(
                           reinterpret_cast<const float*>(a.proj) + kPre * a.proj_fstride +
                           (int64_t)id * a.proj_ld) + kq;
#pragma unroll
    for (int t = 0; t < T16; ++t) {
      const float4 x = pp[4 * t];
      X[t] = f32x4{x.x, x.y, x.z, x.w};
    }
  } else {
#pragma unroll
    for (int t = 0; t < T16; ++t) X[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // each field's id span over the block (rows grouped by user: the user and
  // the context fields span a few table rows)
  for (int x = tid; x < Cfg::kRows * F; x += NT) {
    const int64_t m = m0 + x / F;
    if (m < a.B) {
      atomicMin(&plo[x % F], ids[x]);
      atomicMax(&phi[x % F], ids[x]);
    }
  }
  __syncthreads();
  // staging plan (every thread computes the same): fields in order, while
  // their spans fit the slot's kStageRows rows
  int staged = 0;
  for (int f = 0; f < F; ++f) {
    const int span = phi[f] - plo[f] + 1;
    const bool st = a.stage && f != kPre && span > 0 && staged + span <= kStageRows;
    if (tid == 0) psb[f] = st ? staged : -1;
    staged += st ? span : 0;
  }
  __syncthreads();
  char* pstage = smem + 2 * Cfg::SlotB;
  if (staged > 0) {
    // lane-linear LDS-DMA: chunk c of the image = row c / CPR, 16-B part
    // c % CPR (the last part of a row is padding: it re-reads part 0)
    constexpr int CPR = kPRowB / 16;
    const int nins = (staged * CPR + 63) / 64;
    for (int ins = wv; ins < nins; ins += NW) {
      const int c = ins * 64 + l;
      const int row = c / CPR < staged ? c / CPR : 0;
      const int part = c % CPR < CPR - 1 ? c % CPR : 0;
      int f = 0;
      for (int g = 0; g < F; ++g)
        if (psb[g] >= 0 && row >= psb[g] && row <= psb[g] + phi[g] - plo[g]) f = g;
      const int64_t id = plo[f] + (row - psb[f]);
      const char* src = reinterpret_cast<const char*>(a.proj) +
                        ((int64_t)f * a.proj_fstride + id * a.proj_ld) * 4 + part * 16;
      lds_dma16(src, pstage + ins * 1024);
    }
    dma_wait();
  }
  __syncthreads();

  // half-chunk hc -> ring slot: kDmaW lane-linear 1-KB DMAs per wave; past the
  // last half-chunk the last one is re-read into the free slot, so every
  // step issues the same count and the vmcnt wait below stays exact
  auto dma_half = [&](int hc, int slot) {
    const int blk = hc < H ? hc : H - 1;
    const char* src = reinterpret_cast<const char*>(a.packed) + (int64_t)blk * Cfg::SlotB;
    char* dst = smem + slot * Cfg::SlotB;
#pragma unroll
    for (int d = 0; d < Cfg::kDmaW; ++d) {
      const int piece = wv + NW * d;
      lds_dma16(src + piece * 1024 + l * 16, dst + piece * 1024);
    }
  };
  if (H > 0) {
    dma_half(0, 0);
    dma_half(1, 1);
  }
  HHFM_F32S_T(tq[2] = __builtin_amdgcn_s_memtime();)

  // ----- layer 0 from P: X = Σ_f P_f[x_f] (lane group kq: units 16t+4kq..+3),
  // straight into the registers of layer 1's input -----
  for (int f = 0; f < F; ++f) {
    if (f == kPre) continue;   // already in X
    const int id = ids[myrow * F + f];
    const int sb = psb[f];   // uniform: this field's rows staged in LDS
    if (sb >= 0) {
      const float4* pp = reinterpret_cast<const float4*>(
                             pstage + (sb + id - plo[f]) * kPRowB) + kq;
#pragma unroll
      for (int t = 0; t < T16; ++t) {
        const float4 x = pp[4 * t];
        X[t][0] += x.x;
        X[t][1] += x.y;
        X[t][2] += x.z;
        X[t][3] += x.w;
      }
    } else {
      const float4* pp = reinterpret_cast<const float4*>(
                             reinterpret_cast<const float*>(a.proj) + f * a.proj_fstride +
                             (int64_t)id * a.proj_ld) + kq;
#pragma unroll
      for (int t = 0; t < T16; ++t) {
        const float4 x = pp[4 * t];
        X[t][0] += x.x;
        X[t][1] += x.y;
        X[t][2] += x.z;
        X[t][3] += x.w;
      }
    }
  }
  // ----- hidden layers: 6 split-bf16 MFMAs per tile and 32-k step -----
  HHFM_F32S_T(asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); tq[3] = __builtin_amdgcn_s_memtime();)
  auto mma = [](const bf16x8& w, const bf16x8& x, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x, c, 0, 0, 0);
  };
  f32x4 acc[T16];
  int hc = 0;
  for (int i = 1; i < L; ++i) {
    const float* bli = blv + (i - 1) * NR;
#pragma unroll
    for (int t = 0; t < T16; ++t)
#pragma unroll
      for (int x = 0; x < 4; ++x)   // relu after every layer (DFM.py:128)
        X[t][x] = fmaxf((i == 1 ? X[t][x] : acc[t][x]) + bli[16 * t + 4 * kq + x], 0.f);
#pragma unroll
    for (int c = 0; c < TM; ++c) {
      bf16x8 xb0, xb1, xb2;
      {
        const float v[8] = {X[2 * c][0],     X[2 * c][1],     X[2 * c][2],     X[2 * c][3],
                            X[2 * c + 1][0], X[2 * c + 1][1], X[2 * c + 1][2], X[2 * c + 1][3]};
        split3x8(v, xb0, xb1, xb2);
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh, ++hc) {
        // this wave's DMA of half-chunk hc landed (hc+1's may still fly), every
        // wave's reads of hc-1's slot are done: publish hc, refill hc-1's slot
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(Cfg::kDmaW)
                     : "memory");
        // half-chunk hc+2 into the slot hc-1 used: one DMA after each of the
        // first kDmaW tiles (an LDS-DMA issue costs ~60 cycles; a burst of
        // them would idle the MFMA pipe)
        const int nb = hc + 2 < H ? hc + 2 : H - 1;
        const char* dsrc = reinterpret_cast<const char*>(a.packed) + (int64_t)nb * Cfg::SlotB +
                           wv * 1024 + l * 16;
        char* ddst = smem + ((hc + 2) % 3) * Cfg::SlotB + wv * 1024;
        const char* slot = smem + (hc % 3) * Cfg::SlotB + kq * 256 + r * 16;
        auto frag = [&](int tl, int pc) {
          return *reinterpret_cast<const bf16x8*>(slot + pc * Cfg::PlaneB + tl * 1024);
        };
        // fragments one tile ahead at one wave per SIMD; at two the other
        // wave covers the LDS latency and the registers go to acc + X
        constexpr bool kAhead = NW == 4;
        bf16x8 w0, w1, w2;
        if constexpr (kAhead) {
          w0 = frag(0, 0);
          w1 = frag(0, 1);
          w2 = frag(0, 2);
        }
#pragma unroll
        for (int tl = 0; tl < TM; ++tl) {
          bf16x8 c0, c1, c2;
          if constexpr (kAhead) {
            c0 = w0; c1 = w1; c2 = w2;
            if (tl + 1 < TM) {
              w0 = frag(tl + 1, 0);
              w1 = frag(tl + 1, 1);
              w2 = frag(tl + 1, 2);
            }
          } else {
            c0 = frag(tl, 0);
            c1 = frag(tl, 1);
            c2 = frag(tl, 2);
          }
          f32x4& ac = acc[TM * hh + tl];
          // smallest terms first; a layer's first step starts from zero
          ac = mma(c2, xb0, c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : ac);
          ac = mma(c1, xb1, ac);
          ac = mma(c0, xb2, ac);
          ac = mma(c1, xb0, ac);
          ac = mma(c0, xb1, ac);
          ac = mma(c0, xb0, ac);
          if (tl < Cfg::kDmaW) lds_dma16(dsrc + tl * NW * 1024, ddst + tl * NW * 1024);
        }
#pragma unroll
        for (int d = TM; d < Cfg::kDmaW; ++d)
          lds_dma16(dsrc + d * NW * 1024, ddst + d * NW * 1024);
      }
    }
  }
  dma_wait();   // the trailing (re-read) DMAs
  HHFM_F32S_T(tq[4] = __builtin_amdgcn_s_memtime();)

  const float* blL = blv + (L - 1) * NR;
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < T16; ++t)
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int n = 16 * t + 4 * kq + x;
      part += fmaxf(acc[t][x] + blL[n], 0.f) * vl[n];
    }
  part += __shfl_xor(part, 16, kWave);
  part += __shfl_xor(part, 32, kWave);
  const int64_t m = m0 + myrow;
  if (kq == 0 && m < a.B) a.out[a.order ? a.order[m] : m] = a.fmbase[m] + part;
#if HHFM_F32S_TIMING
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  tq[5] = __builtin_amdgcn_s_memtime();
  if (l == 0) {
    for (int q = 0; q < 5; ++q) atomicAdd(&g_f32s_t[q], tq[q + 1] - tq[q]);
    atomicAdd(&g_f32s_t[5], 1ull);
  }
#endif
}

// the FM part's per-element steps, spelled out (fused or not) so the two
// kernels below round identically
HHFM_DEV void fmb_acc(float& s, float& q, float v) {
  s += v;
  q = __fmaf_rn(v, v, q);
}
HHFM_DEV float fmb_term(float y, float s, float q, float wp) {
  return __fmaf_rn(0.5f * __fmaf_rn(s, s, -q), wp, y);
}

// base[m] = ((Σ_f w[x_f]·Wp[f] + Σ_c ½((Σ_f e_fc)² − Σ_f e_fc²)·Wp[F+c]) + bp)
// (DFM.py:109-122, 132-137 without the deep part): 16 lanes per row, 16-B
// column chunks, at full occupancy — the FM part's table reads are latency-
// bound inside the one-wave-per-SIMD MFMA kernel.
template <bool TBF, int KJ>
__global__ __launch_bounds__(256) void dfm_fm_base(const int32_t* __restrict__ idx, int64_t B,
                                                   int F, const void* __restrict__ E, int64_t M,
                                                   int k, const float* __restrict__ w,
                                                   const float* __restrict__ Wp, float bp,
                                                   float* __restrict__ base) {
  const int l = threadIdx.x & 63, sub = l & 15;
  const int64_t row0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / 16;
  const int64_t nrow = ((int64_t)gridDim.x * blockDim.x) / 16;
  // lane `sub` owns columns 64j + 4sub .. +3: KJ = k / 64 independent 16-B
  // loads per field (KJ = 0: any k % 4 == 0, one column block at a time)
  constexpr int J = KJ > 0 ? KJ : 1;
  for (int64_t m = row0; m < B; m += nrow) {   // a row's 16 lanes stay together
    const int32_t* p = idx + m * F;
    float y2 = 0.f;
    for (int c00 = 0; c00 < k; c00 += 64 * J) {
      float s4[J][4], q4[J][4];
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int x = 0; x < 4; ++x) { s4[j][x] = 0.f; q4[j][x] = 0.f; }
      const bool live = KJ > 0 || c00 + 4 * sub < k;
#pragma unroll 4
      for (int f = 0; f < F; ++f) {
        const int64_t id = clamp_id(p[f], M);
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const int c0 = c00 + 64 * j + 4 * sub;
          float v[4] = {0.f, 0.f, 0.f, 0.f};
          if (live) {
            if constexpr (TBF) {
              const uint2 x = *reinterpret_cast<const uint2*>(
                  reinterpret_cast<const uint16_t*>(E) + id * k + c0);
              v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
              v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
            } else {
              const float4 x = *reinterpret_cast<const float4*>(
                  reinterpret_cast<const float*>(E) + id * k + c0);
              v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
            }
          }
#pragma unroll
          for (int x = 0; x < 4; ++x) fmb_acc(s4[j][x], q4[j][x], v[x]);
        }
      }
      if (live)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
          for (int x = 0; x < 4; ++x)
            y2 = fmb_term(y2, s4[j][x], q4[j][x], Wp[F + c00 + 64 * j + 4 * sub + x]);
    }
    y2 = group_sum<16>(y2);
    if (sub == 0) {
      float y1 = 0.f;
      for (int f = 0; f < F; ++f) y1 = __fmaf_rn(w[clamp_id(p[f], M)], Wp[f], y1);
      base[m] = (y1 + y2) + bp;
    }
  }
}

// dfm_fm_base over blocks of kFmbRows consecutive rows (rows grouped by user):
// every field whose ids span few table rows in the block (the user and the
// contexts) has those rows copied to LDS once, so only the item's row of each
// row is read from the cache hierarchy (the grid-stride kernel above read all
// F rows of every row through L1/L2: L1-bandwidth-bound).  Same arithmetic in
// the same order per row — the same bits.
constexpr int kFmbRows = 256;
constexpr int kFmbStageB = 32 * 1024;
template <bool TBF, int KJ>
__global__ __launch_bounds__(256) void dfm_fm_base_st(const int32_t* __restrict__ idx, int64_t B,
                                                      int F, const void* __restrict__ E,
                                                      int64_t M, int k,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ Wp, float bp,
                                                      float* __restrict__ base) {
  static_assert(KJ > 0, "staged FM part: k % 64 == 0");
  constexpr int ES = TBF ? 2 : 4;
  __shared__ __attribute__((aligned(16))) char stage[kFmbStageB];
  __shared__ int32_t sid[kFmbRows * kFusedMaxF];
  __shared__ int32_t slo[kFusedMaxF], shi[kFusedMaxF], sbase[kFusedMaxF];
  const int tid = threadIdx.x, sub = tid & 15;
  const int64_t m0 = (int64_t)blockIdx.x * kFmbRows;
  const int nr = (int)(B - m0 < kFmbRows ? B - m0 : kFmbRows);
  if (tid < F) {
    slo[tid] = 0x7fffffff;
    shi[tid] = -1;
  }
  for (int x = tid; x < nr * F; x += 256) sid[x] = clamp_id(idx[m0 * F + x], M);
  __syncthreads();
  for (int x = tid; x < nr * F; x += 256) {
    atomicMin(&slo[x % F], sid[x]);
    atomicMax(&shi[x % F], sid[x]);
  }
  __syncthreads();
  // staging plan (every thread computes the same): fields in order while
  // their spans fit
  const int rowb = k * ES, cap = kFmbStageB / rowb;
  int used = 0;
  for (int f = 0; f < F; ++f) {
    const int span = shi[f] - slo[f] + 1;
    const bool st = used + span <= cap;
    if (tid == 0) sbase[f] = st ? used : -1;
    used += st ? span : 0;
  }
  __syncthreads();
  for (int f = 0; f < F; ++f) {
    if (sbase[f] < 0) continue;
    const int span = shi[f] - slo[f] + 1, c16 = rowb / 16;
    const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(E) +
                                                      (int64_t)slo[f] * rowb);
    uint4* dst = reinterpret_cast<uint4*>(stage + sbase[f] * rowb);
    for (int x = tid; x < span * c16; x += 256) dst[x] = src[x];
  }
  __syncthreads();
  for (int rr = tid / 16; rr < nr; rr += 16) {   // a row's 16 lanes stay together
    const int32_t* p = sid + rr * F;
    float y2 = 0.f;
    float s4[KJ][4], q4[KJ][4];
#pragma unroll
    for (int j = 0; j < KJ; ++j)
#pragma unroll
      for (int x = 0; x < 4; ++x) { s4[j][x] = 0.f; q4[j][x] = 0.f; }
#pragma unroll 4
    for (int f = 0; f < F; ++f) {
      const int id = p[f], sb = sbase[f];
      const char* rowp = sb >= 0 ? stage + (sb + id - slo[f]) * rowb
                                 : reinterpret_cast<const char*>(E) + (int64_t)id * rowb;
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        const int c0 = 64 * j + 4 * sub;
        float v[4];
        if constexpr (TBF) {
          uint2 x;
          if (sb >= 0) x = *reinterpret_cast<const uint2*>(stage + (sb + id - slo[f]) * rowb + c0 * 2);
          else x = *reinterpret_cast<const uint2*>(rowp + c0 * 2);
          v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
          v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
        } else {
          float4 x;
          if (sb >= 0) x = *reinterpret_cast<const float4*>(stage + (sb + id - slo[f]) * rowb + c0 * 4);
          else x = *reinterpret_cast<const float4*>(rowp + c0 * 4);
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        }
#pragma unroll
        for (int x = 0; x < 4; ++x) fmb_acc(s4[j][x], q4[j][x], v[x]);
      }
    }
#pragma unroll
    for (int j = 0; j < KJ; ++j)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        y2 = fmb_term(y2, s4[j][x], q4[j][x], Wp[F + 64 * j + 4 * sub + x]);
    y2 = group_sum<16>(y2);
    if (sub == 0) {
      float y1 = 0.f;
      for (int f = 0; f < F; ++f) y1 = __fmaf_rn(w[p[f]], Wp[f], y1);
      base[m0 + rr] = (y1 + y2) + bp;
    }
  }
}

// ---- the FM part from pair tables -------------------------------------------
// Σ_k Wp_k·½((Σ_f e_fk)² − Σ_f e_fk²) = Σ_{f<g} Σ_k Wp_k·e_fk·e_gk
// = Σ_{f<g} C[x_f][x_g] with C = (E ⊙ Wp)·Eᵀ over the table (DFM.py:114-122
// re-associated): one exact-fp32 MFMA GEMM per call (2·M²·k flops) instead of
// reading every row's F table rows.  Rows grouped by user: a block's entries
// of its user's row of C stay in L1/L2; the item's are one line per row.
__global__ __launch_bounds__(256) void dfm_scale_rows(const void* __restrict__ E, int tbf,
                                                      int64_t M, int k,
                                                      const float* __restrict__ wk,
                                                      float* __restrict__ out) {
  const int64_t n = M * k;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(x % k);
    const float e = tbf ? __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(E)[x] << 16)
                        : reinterpret_cast<const float*>(E)[x];
    out[x] = e * wk[c];
  }
}

__global__ __launch_bounds__(256) void dfm_fm_base_pairs(const int32_t* __restrict__ idx,
                                                         int64_t B, int F, int64_t M,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ Wp, float bp,
                                                         const float* __restrict__ C,
                                                         float* __restrict__ base) {
  // a row's F(F-1)/2 entries of C are gathered through L1/L2 (a block's rows
  // share one or two users after grouping; copying their whole rows of C to
  // LDS first measured slower)
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= B) return;
  int32_t x[kFusedMaxF];
  for (int f = 0; f < F; ++f) x[f] = clamp_id(idx[m * F + f], M);
  float y2 = 0.f;
  for (int f = 0; f < F; ++f)
    for (int g = f + 1; g < F; ++g) y2 += C[(int64_t)x[f] * M + x[g]];
  float y1 = 0.f;
  for (int f = 0; f < F; ++f) y1 = __fmaf_rn(w[x[f]], Wp[f], y1);
  base[m] = (y1 + y2) + bp;
}

// the pair table built only in the tiles the call's field ranges read
// (HHFM_PAIRS_ALL_TILES=1: every tile — the same bits, A/B)
#ifndef HHFM_PAIRS_ALL_TILES
#define HHFM_PAIRS_ALL_TILES 0
#endif
bool dfm_fm_pairs(const FusedDfmArgs& a, bool tbf, hipStream_t st, bool base) {
  const int64_t M = a.M, B = a.B;
  const int k = a.k;
  const size_t cbytes = (size_t)M * M * 4, sbytes = (size_t)M * k * 4;
  const bool ready = a.pairs_ready && *a.pairs_ready;
  if ((a.plan & HHFM_PLAN_ROW_FM) || !a.scratch || !a.fm_out || M > 32768 ||
      (!ready && M * 16 > B) || k % 4 || cbytes + sbytes + 512 > a.scratch_bytes)
    return false;
  float* Cp = reinterpret_cast<float*>(a.scratch);
  if (!ready) {
  float* Es = reinterpret_cast<float*>(reinterpret_cast<char*>(a.scratch) +
                                       ((cbytes + 255) & ~size_t(255)));
  hipLaunchKernelGGL(dfm_scale_rows, dim3(1024), dim3(256), 0, st, a.E, (int)tbf, M, k,
                     a.Wp + a.F, Es);
  GemmArgs g{};
  g.M = M;
  g.N = (int)M;
  g.K = k;
  g.A = Es;
  g.lda = k;
  g.Bt = a.E;
  g.ldb = k;
  g.b_src_bf16 = tbf;
  g.C = Cp;
  g.ldc = M;
  if (a.franges && !a.pairs_ready && !(HHFM_PAIRS_ALL_TILES)) {   // this call's rows only
    g.tile_ranges = a.franges;
    g.tr_F = a.F;
  }
  launch_gemm(g, false, 0, st);
  if (a.pairs_ready) *a.pairs_ready = true;
  }
  if (base)
    hipLaunchKernelGGL(dfm_fm_base_pairs, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st,
                       a.idx, B, a.F, M, a.w, a.Wp, a.bp, Cp, a.fm_out);
  return true;
}

static int fused_tm(int maxT) {
  const int tms[] = {2, 4, 5, 7, 8, 10, 13};
  for (int t : tms)
    if (maxT <= t) return t;
  return 0;
}

static int fused_max_tiles(int L, const int32_t* dims) {
  int maxT = 0;
  for (int i = 0; i < L; ++i) {
    const int T = (dims[i] + 31) / 32;
    maxT = T > maxT ? T : maxT;
  }
  return maxT;
}

bool dfm_fused_eligible(int L, const int32_t* dims) {
  return L >= 1 && L <= kFusedMaxLayers && fused_tm(fused_max_tiles(L, dims)) > 0;
}

// workspace for the packed weights; an upper bound over F·k <= 16·512 so the
// size is known from (nlayers, dims) alone
size_t dfm_fused_pack_bytes(int L, const int32_t* dims, bool mlp_bf16) {
  const int TM = fused_tm(fused_max_tiles(L, dims));
  const int nc0 = mlp_bf16 ? (kFusedMaxF * kFusedMaxK / 16 + 3) / 4
                           : (kFusedMaxF * kFusedMaxK / 16 + 1) / 2;
  const int nch = mlp_bf16 ? (TM + 1) / 2 : TM;
  const size_t direct = (size_t)(nc0 + (L - 1) * nch) * 32 * TM * 8 * 16;
  const size_t split = (size_t)(L - 1) * TM * 2 * f32s_slot_bytes(TM);   // dfm_fused_f32s
  return mlp_bf16 || direct >= split ? direct : split;
}

// ---------------------------------------------------------------------------
// Projected layer 0: P_f[id] = W0[:, f·k:(f+1)·k] · E[id] for every table row
// id and field f, fp32, row stride 32·TM (columns >= dims[0] zero).  F MFMA
// GEMMs [M, k] x [k, N0] on the shared tile kernel, A = the table through an
// identity gather (fp32 tables rounded to bf16 exactly like the direct
// kernel's B operand; bf16 MFMA with fp32 accumulation, or exact fp32 MFMA for
// the fp32 MLP).  Workspace: [P: F·M·ld floats][identity ids: M int32].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dfm_iota(int32_t* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)i;
}

bool dfm_proj_eligible(int F, int k, int L, const int32_t* dims) {
  return dfm_fused_eligible(L, dims) && F >= 1 && F <= kFusedMaxF && k % 16 == 0 &&
         k <= kFusedMaxK;
}

int dfm_proj_ld(int L, const int32_t* dims) { return 32 * fused_tm(fused_max_tiles(L, dims)); }

// P for the projected (internal) fields j in [proj_from, F): P_j = W0
// restricted to the caller's field perm(j), laid out [id][j][NR] (one row of
// all projected fields per table row), computed by ONE GEMM against the
// stacked weights Wc[(j, n)][k] = W0[n][perm(j)·k ..] (zero for n >= N0).
static size_t proj_al(size_t x) { return (x + 255) & ~size_t(255); }

size_t dfm_proj_bytes(int F, int proj_from, int64_t M, int L, const int32_t* dims) {
  const size_t ld = (size_t)dfm_proj_ld(L, dims), nf = (size_t)(F - proj_from);
  return proj_al(nf * (size_t)M * ld * 4) + proj_al((size_t)M * 4) +
         proj_al(nf * ld * kFusedMaxK * 4);
}

// Wc rows (j, n), 16-B units: W0 (esz-byte elements, row stride ldb0)
__global__ __launch_bounds__(256) void dfm_proj_weights(const char* __restrict__ W0, int esz,
                                                        int ldb0, int N0, int NR, int nf,
                                                        int proj_from, uint64_t perm, int k,
                                                        uint4* __restrict__ Wc) {
  const int upr = k * esz / 16;   // units per row
  const int64_t total = (int64_t)nf * NR * upr;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = x / upr;
    const int u = (int)(x - row * upr);
    const int j = (int)(row / NR), n = (int)(row - (int64_t)j * NR);
    const int fe = (int)((perm >> (4 * (proj_from + j))) & 15);
    Wc[x] = n < N0 ? *reinterpret_cast<const uint4*>(W0 + ((size_t)n * ldb0 + (size_t)fe * k) * esz +
                                                    16 * u)
                   : make_uint4(0, 0, 0, 0);
  }
}

void dfm_project_layer0(const void* E, int64_t M, int k, bool tbf, bool mlp_bf16, int F,
                        int proj_from, uint64_t perm, const void* Wt0, int N0, int L,
                        const int32_t* dims, void* ws, hipStream_t st) {
  const int ld = dfm_proj_ld(L, dims), nf = F - proj_from;
  const int esz = mlp_bf16 ? 2 : 4;   // weight element size
  char* base = reinterpret_cast<char*>(ws);
  const size_t pbytes = proj_al((size_t)nf * M * ld * 4);
  int32_t* iota = reinterpret_cast<int32_t*>(base + pbytes);
  uint4* Wc = reinterpret_cast<uint4*>(base + pbytes + proj_al((size_t)M * 4));
  const int64_t ib = (M + 255) / 256 < 4096 ? (M + 255) / 256 : 4096;
  hipLaunchKernelGGL(dfm_iota, dim3((unsigned)ib), dim3(256), 0, st, iota, M);
  const int64_t wu = (int64_t)nf * ld * (k * esz / 16);
  hipLaunchKernelGGL(dfm_proj_weights, dim3((unsigned)((wu + 255) / 256 < 2048 ? (wu + 255) / 256
                                                                               : 2048)),
                     dim3(256), 0, st, reinterpret_cast<const char*>(Wt0), esz,
                     (F * k + 7) & ~7, N0, ld, nf, proj_from, perm, k, Wc);
  GemmArgs g{};
  g.M = M;
  g.N = nf * ld;
  g.K = k;
  g.gidx = iota; g.T = E; g.Mtab = M; g.F = 1; g.kf = k; g.t_bf16 = tbf;
  g.Bt = Wc;
  g.ldb = k;
  g.relu = 0;
  g.C = reinterpret_cast<float*>(ws);
  g.ldc = nf * ld;
  g.c_perm32 = mlp_bf16;   // the bf16 kernel's accumulator order (ld % 32 == 0)
  launch_gemm(g, mlp_bf16, 0, st);
}

// returns false when the shape is outside the fused kernel's envelope.
// proj != nullptr: the layer-0 products of fields [proj_from, F) come from
// dfm_project_layer0's workspace (PROJ kernels; the fp32 MLP projects all
// fields, proj_from = 0).
bool dfm_fused_launch(const int32_t* idx, int64_t B, int F, const void* E, int64_t M, int k,
                      bool tbf, bool mlp_bf16, const float* w, int L, const int32_t* dims,
                      const void* const* Wt, const float* const* bias, const float* Wp, float bp,
                      float* out, void* pack_ws, const void* proj, int proj_from,
                      uint64_t perm, const int32_t* order, float* fm_base, void* scratch,
                      size_t scratch_bytes, int32_t plan, bool* pairs_ready, hipStream_t st,
                      const int32_t* franges) {
  if (!dfm_fused_eligible(L, dims) || F > kFusedMaxF || k > kFusedMaxK) return false;
  if (k % 16) return false;
  for (int i = 0; i < L; ++i)
    if (reinterpret_cast<uintptr_t>(Wt[i]) & 15) return false;
  const int TM = fused_tm(fused_max_tiles(L, dims));
  FusedDfmArgs a{};
  a.idx = idx; a.B = B; a.F = F; a.k = k; a.E = E; a.M = M; a.w = w; a.L = L;
  int kin = F * k;
  for (int i = 0; i < L; ++i) {
    a.dims[i] = dims[i];
    a.ldb[i] = (kin + 7) & ~7;
    a.Wt[i] = reinterpret_cast<const uint16_t*>(Wt[i]);
    a.bias[i] = bias[i];
    kin = dims[i];
  }
  a.Wp = Wp; a.bp = bp; a.out = out;
  a.packed = reinterpret_cast<const uint4*>(pack_ws);
  a.proj = proj;
  a.proj_fstride = 32 * TM;   // [id][projected field][32·TM] (dfm_project_layer0)
  a.proj_ld = (proj ? F - proj_from : 1) * 32 * TM;
  const bool pj = proj != nullptr;
  a.Fd = pj ? proj_from : F;
  a.perm = perm;
  a.order = order;
  a.scratch = scratch;
  a.scratch_bytes = scratch_bytes;
  a.fm_out = fm_base;
  a.plan = plan;
  a.pairs_ready = pairs_ready;
  a.franges = franges;
  if (pj && (proj_from < 0 || proj_from >= F)) return false;
  if (!mlp_bf16) {
    // the fp32 kernel projects all fields, in the caller's order
    const bool split = pj && L > 1 && dfm_f32_split(plan);
    // (the split kernel also takes rows grouped by user: out[order[m]])
    if ((pj && proj_from != 0) || perm != kDfmIdentityPerm || (order && !split)) return false;
    const dim3 grid((unsigned)((B + kF32Rows - 1) / kF32Rows));
    if (split) {
      if (!fm_base) return false;
      // FM part from the pair table C = (E ⊙ Wp)·Eᵀ (dfm_fm_pairs) when it fits
      // and pays; otherwise from the rows
      if (dfm_fm_pairs(a, tbf, st)) {
      } else {
        const int64_t rows_per_block = 256 / 16;
        int64_t fb = (B + rows_per_block - 1) / rows_per_block;
        if (fb > 8192) fb = 8192;
#define HHFM_FMB(KJ)                                                                       \
  if (tbf)                                                                                 \
    hipLaunchKernelGGL((dfm_fm_base<true, KJ>), dim3((unsigned)fb), dim3(256), 0, st, idx, B, \
                       F, E, M, k, w, Wp, bp, fm_base);                                    \
  else                                                                                     \
    hipLaunchKernelGGL((dfm_fm_base<false, KJ>), dim3((unsigned)fb), dim3(256), 0, st, idx,   \
                       B, F, E, M, k, w, Wp, bp, fm_base);
        const int kj = k % 64 ? 0 : k / 64;
        const unsigned sblocks = (unsigned)((B + kFmbRows - 1) / kFmbRows);
#define HHFM_FMBS(KJ)                                                                      \
  if (tbf)                                                                                 \
    hipLaunchKernelGGL((dfm_fm_base_st<true, KJ>), dim3(sblocks), dim3(256), 0, st, idx, B, \
                       F, E, M, k, w, Wp, bp, fm_base);                                    \
  else                                                                                     \
    hipLaunchKernelGGL((dfm_fm_base_st<false, KJ>), dim3(sblocks), dim3(256), 0, st, idx,   \
                       B, F, E, M, k, w, Wp, bp, fm_base);
        if (!(plan & HHFM_PLAN_UNSTAGED) && kj > 0 && k * (tbf ? 2 : 4) <= kFmbStageB) {
          switch (kj) {
            case 1: HHFM_FMBS(1) break;
            case 2: HHFM_FMBS(2) break;
            case 4: HHFM_FMBS(4) break;
            default: HHFM_FMBS(8) break;
          }
        } else
        switch (kj) {
          case 1: HHFM_FMB(1) break;
          case 2: HHFM_FMB(2) break;
          case 4: HHFM_FMB(4) break;
          case 8: HHFM_FMB(8) break;
          default: HHFM_FMB(0) break;
        }
#undef HHFM_FMB
#undef HHFM_FMBS
      }
      a.fmbase = fm_base;
      a.stage = !(plan & HHFM_PLAN_UNSTAGED);
      const int64_t units = (int64_t)(L - 1) * TM * 2 * 16 * TM * 4;
      const int pblocks = (int)((units + 255) / 256 < 2048 ? (units + 255) / 256 : 2048);
      hipLaunchKernelGGL(dfm_pack_weights_f32s, dim3(pblocks), dim3(256), 0, st, a, TM,
                         reinterpret_cast<char*>(pack_ws));
      // 8 waves x 16 rows (two waves per SIMD; one wave per SIMD measured
      // slower)
      const dim3 g8((unsigned)((B + 127) / 128));
#define HHFM_FUSED32S(T)                                                                   \
  case T:                                                                                  \
    if (tbf) hipLaunchKernelGGL((dfm_fused_f32s<true, T, 8>), g8, dim3(512), 0, st, a);     \
    else hipLaunchKernelGGL((dfm_fused_f32s<false, T, 8>), g8, dim3(512), 0, st, a);        \
    break;
      switch (TM) {
        HHFM_FUSED32S(2)
        HHFM_FUSED32S(4)
        HHFM_FUSED32S(5)
        HHFM_FUSED32S(7)
        HHFM_FUSED32S(8)
        HHFM_FUSED32S(10)
        HHFM_FUSED32S(13)
        default: return false;
      }
#undef HHFM_FUSED32S
      return true;
    }
    const int nc0 = pj ? 0 : (F * (k / 16) + 1) / 2;
    const int64_t units = (int64_t)(nc0 + (L - 1) * TM) * 32 * TM * 8;
    const int pblocks = (int)((units + 255) / 256 < 2048 ? (units + 255) / 256 : 2048);
    if (units > 0)
      hipLaunchKernelGGL(dfm_pack_weights_f32, dim3(pblocks), dim3(256), 0, st, a, TM, nc0,
                         reinterpret_cast<uint4*>(pack_ws));
#define HHFM_FUSED32(T)                                                                    \
  case T:                                                                                  \
    if (pj) {                                                                              \
      if (tbf) hipLaunchKernelGGL((dfm_fused_f32<true, T, true>), grid, dim3(256), 0, st, a); \
      else hipLaunchKernelGGL((dfm_fused_f32<false, T, true>), grid, dim3(256), 0, st, a);    \
    } else {                                                                               \
      if (tbf) hipLaunchKernelGGL((dfm_fused_f32<true, T, false>), grid, dim3(256), 0, st, a);\
      else hipLaunchKernelGGL((dfm_fused_f32<false, T, false>), grid, dim3(256), 0, st, a);   \
    }                                                                                      \
    break;
    switch (TM) {
      HHFM_FUSED32(2)
      HHFM_FUSED32(4)
      HHFM_FUSED32(5)
      HHFM_FUSED32(7)
      HHFM_FUSED32(8)
      HHFM_FUSED32(10)
      HHFM_FUSED32(13)
      default: return false;
    }
#undef HHFM_FUSED32
    return true;
  }
  // the ITEM plan at an instantiated shape: 256 rows per workgroup (dfm_wide.hip)
  if (pj && tbf && a.Fd == 1 && L == 3 && !(plan & HHFM_PLAN_NARROW) &&
      dfm_wide_launch(a, TM, plan, st))
    return true;
  const dim3 grid((unsigned)((B + kFusedRows - 1) / kFusedRows));
  const int nS = a.Fd * (k / 16), nc0 = (nS + 3) / 4, NC = (TM + 1) / 2;
  const int64_t units = (int64_t)(nc0 + (L - 1) * NC) * 32 * TM * 8;
  const int pblocks = (int)((units + 255) / 256 < 2048 ? (units + 255) / 256 : 2048);
  if (units > 0)
    hipLaunchKernelGGL(dfm_pack_weights, dim3(pblocks), dim3(256), 0, st, a, TM, nc0, NC,
                       reinterpret_cast<uint4*>(pack_ws));
#define HHFM_FUSED(T)                                                                      \
  case T:                                                                                  \
    if (pj) {                                                                              \
      if (tbf) hipLaunchKernelGGL((dfm_fused<true, T, true>), grid, dim3(256), 0, st, a);     \
      else hipLaunchKernelGGL((dfm_fused<false, T, true>), grid, dim3(256), 0, st, a);        \
    } else {                                                                               \
      if (tbf) hipLaunchKernelGGL((dfm_fused<true, T, false>), grid, dim3(256), 0, st, a);    \
      else hipLaunchKernelGGL((dfm_fused<false, T, false>), grid, dim3(256), 0, st, a);       \
    }                                                                                      \
    break;
  switch (TM) {
    HHFM_FUSED(2)
    HHFM_FUSED(4)
    HHFM_FUSED(5)
    HHFM_FUSED(7)
    HHFM_FUSED(8)
    HHFM_FUSED(10)
    HHFM_FUSED(13)
    default: return false;
  }
#undef HHFM_FUSED
  return true;
}

// ---------------------------------------------------------------------------
// Row grouping for the projected kernel: the row indices ordered by one
// field's id (counting sort below, or hipCUB's radix sort), so a 128-row block sees few distinct
// ids of that field and its P rows stage in LDS.  Scores are written back to
// the caller's row positions; every row's arithmetic is unchanged.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dfm_order_keys(const int32_t* __restrict__ idx,
                                                      int64_t B, int F, int key_field, int64_t M,
                                                      uint32_t* __restrict__ keys,
                                                      int32_t* __restrict__ vals) {
  for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < B;
       m += (int64_t)gridDim.x * blockDim.x) {
    keys[m] = (uint32_t)clamp_id(idx[m * F + key_field], M);
    vals[m] = (int32_t)m;
  }
}

static int dfm_key_bits(int64_t M) {
  int b = 1;
  while (b < 31 && (int64_t(1) << b) < M) ++b;
  return b;
}

static size_t dfm_al256(size_t x) { return (x + 255) & ~size_t(255); }

// rows[m] = idx[order[m]]: the fused kernel then reads a block's rows as one
// contiguous slab
__global__ __launch_bounds__(256) void dfm_gather_rows(const int32_t* __restrict__ idx,
                                                       const int32_t* __restrict__ order,
                                                       int64_t B, int F,
                                                       int32_t* __restrict__ rows) {
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < B * F;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = x / F;
    rows[x] = idx[(int64_t)order[m] * F + (x - m * F)];
  }
}

// Counting-sort grouping for key ranges up to kGroupBins ids (Frappe's users:
// 957 of 5,051 table rows).  dfm_group_hist: every 1024-thread block
// histograms an 8 K-row slice in LDS and adds it to the global counts;
// dfm_group_scan turns them into group starts.  dfm_group_scatter then sorts
// its 4 K-row slice by key in LDS (a local counting sort: per-row rank from
// the LDS atomic, a block scan, one global reservation per (slice, id)) and
// writes the grouped copy dword by dword in sorted order, so consecutive
// lanes store consecutive words of one id's run (a per-row scatter of 4-B
// words to random runs cost 3.4x as much at 12.5 M rows:
// scripts/diag/groupbench.hip).  Positions inside one id's group depend on
// atomic timing — every row's arithmetic does not, so the scores are
// identical either way.  Larger key ranges take hipCUB's radix sort.
constexpr int kGroupBins = 8192;
constexpr int kGroupRows = 8192;      // rows per histogram block
// (8 K / 16 K rows per block: C5 bf16 +0.00-0.07 ms, profiles/r06_scatter_rows_ab.txt)
#ifndef HHFM_SCATTER_ROWS
#define HHFM_SCATTER_ROWS 4096
#endif
constexpr int kScatterRows = HHFM_SCATTER_ROWS;   // rows per scatter block (<= 65536: 16-bit local index)

// franges (or null, F <= kFusedMaxF): every field's id range over the rows
// (FusedDfmArgs::franges encoding, global atomicMax onto zeros) — the same
// lines the key column's reads fetch
__global__ __launch_bounds__(1024) void dfm_group_hist(const int32_t* __restrict__ idx, int64_t B,
                                                      int F, int key_field, int64_t M,
                                                      uint32_t* __restrict__ count,
                                                      int32_t* __restrict__ franges) {
  __shared__ uint32_t hcnt[kGroupBins];
  __shared__ int32_t fr[2 * kFusedMaxF];
  const int nb = (int)M;
  for (int b = threadIdx.x; b < nb; b += 1024) hcnt[b] = 0;
  if (threadIdx.x < 2 * kFusedMaxF) fr[threadIdx.x] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kGroupRows;
  const int64_t r1 = r0 + kGroupRows < B ? r0 + kGroupRows : B;
  int32_t rl[kFusedMaxF], rh[kFusedMaxF];
#pragma unroll
  for (int f = 0; f < kFusedMaxF; ++f) rl[f] = rh[f] = 0;
  for (int64_t m = r0 + threadIdx.x; m < r1; m += 1024) {
    atomicAdd(&hcnt[clamp_id(idx[m * F + key_field], M)], 1u);
    if (franges) {
#pragma unroll
      for (int f = 0; f < kFusedMaxF; ++f)
        if (f < F) {
          const int32_t v = clamp_id(idx[m * F + f], M);
          rl[f] = max(rl[f], 0x7fffffff - v);
          rh[f] = max(rh[f], v);
        }
    }
  }
  if (franges) {
#pragma unroll
    for (int f = 0; f < kFusedMaxF; ++f) {
      if (f < F) {
        for (int o = 32; o; o >>= 1) {
          rl[f] = max(rl[f], __shfl_xor(rl[f], o, 64));
          rh[f] = max(rh[f], __shfl_xor(rh[f], o, 64));
        }
        if ((threadIdx.x & 63) == 0) {
          atomicMax(&fr[2 * f], rl[f]);
          atomicMax(&fr[2 * f + 1], rh[f]);
        }
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += 1024)
    if (hcnt[b]) atomicAdd(&count[b], hcnt[b]);
  if (franges && threadIdx.x < 2 * F) atomicMax(&franges[threadIdx.x], fr[threadIdx.x]);
}

// exclusive scan of count[0, M) into start (one block)
__global__ __launch_bounds__(1024) void dfm_group_scan(const uint32_t* __restrict__ count,
                                                       int64_t M, uint32_t* __restrict__ start) {
  __shared__ uint32_t part[1024];
  const int per = (int)((M + 1023) / 1024);
  const int b0 = threadIdx.x * per;
  uint32_t s = 0;
  for (int b = b0; b < b0 + per && b < M; ++b) s += count[b];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {   // Hillis-Steele inclusive scan
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;   // exclusive prefix of this thread's bins
  for (int b = b0; b < b0 + per && b < M; ++b) {
    start[b] = run;
    run += count[b];
  }
}

__global__ __launch_bounds__(1024) void dfm_group_scatter(const int32_t* __restrict__ idx,
                                                          int64_t B, int F, int key_field,
                                                          int64_t M,
                                                          const uint32_t* __restrict__ start,
                                                          uint32_t* __restrict__ cursor,
                                                          int32_t* __restrict__ rows,
                                                          int32_t* __restrict__ order) {
  constexpr int kPer = kScatterRows / 1024;
  __shared__ uint32_t lstart[kGroupBins];   // slice count, then local group start
  __shared__ int32_t delta[kGroupBins];     // global group position - local start
  __shared__ uint32_t lrow[kScatterRows];   // sorted slot -> (key - lo) << 16 | local row
  __shared__ uint32_t wsum[16];
  __shared__ int krange[2];                 // the slice's key range [lo, hi]
  if (threadIdx.x == 0) { krange[0] = (int)M; krange[1] = -1; }
  const int64_t r0 = (int64_t)blockIdx.x * kScatterRows;
  const int n = (int)(r0 + kScatterRows < B ? kScatterRows : B - r0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int key[kPer];
  int klo = (int)M, khi = -1;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int j = threadIdx.x + i * 1024;
    key[i] = j < n ? clamp_id(idx[(r0 + j) * F + key_field], M) : 0;
    if (j < n) { klo = min(klo, key[i]); khi = max(khi, key[i]); }
  }
  for (int off = 32; off; off >>= 1) {
    klo = min(klo, __shfl_xor(klo, off, 64));
    khi = max(khi, __shfl_xor(khi, off, 64));
  }
  __syncthreads();
  if (lane == 0) { atomicMin(&krange[0], klo); atomicMax(&krange[1], khi); }
  __syncthreads();
  // only the slice's key range is counted and scanned (the key field spans
  // a fraction of the table: Frappe's users are 957 of its 5,051 rows)
  const int lo = krange[0], nb = krange[1] - lo + 1;
  for (int b = threadIdx.x; b < nb; b += 1024) lstart[b] = 0;
  __syncthreads();
  uint32_t rank[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i)
    if (threadIdx.x + i * 1024 < n) rank[i] = atomicAdd(&lstart[key[i] - lo], 1u);
  __syncthreads();
  // exclusive block scan of the slice counts: a chunk of bins per thread,
  // wave-level inclusive scan of the chunk sums, then the waves' totals
  const int per = (nb + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  uint32_t s = 0;
  for (int b = b0; b < b0 + per && b < nb; ++b) s += lstart[b];
  uint32_t inc = s;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(inc, off, 64);
    if (lane >= off) inc += v;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t run = inc - s;
  for (int i = 0; i < w; ++i) run += wsum[i];
  for (int b = b0; b < b0 + per && b < nb; ++b) {
    const uint32_t c = lstart[b];
    lstart[b] = run;
    delta[b] = c ? (int32_t)(start[lo + b] + atomicAdd(&cursor[lo + b], c)) - (int32_t)run : 0;
    run += c;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int j = threadIdx.x + i * 1024;
    if (j < n) lrow[lstart[key[i] - lo] + rank[i]] = ((uint32_t)(key[i] - lo) << 16) | (uint32_t)j;
  }
  __syncthreads();
  // word f of sorted slot j; j = x / F by a multiply-high (exact for
  // x < 2^32 / F, here x < kScatterRows * F)
  const uint32_t inv_f = 0xffffffffu / (uint32_t)F + 1u;
  for (int x = threadIdx.x; x < n * F; x += 1024) {
    const int j = (int)__umulhi((uint32_t)x, inv_f), f = x - j * F;
    const uint32_t e = lrow[j];
    const int jl = (int)(e & 0xffff);
    const int64_t pos = (int64_t)delta[e >> 16] + j;
    rows[pos * F + f] = idx[(r0 + jl) * F + f];
    if (f == 0) order[pos] = (int32_t)(r0 + jl);
  }
}

size_t dfm_order_bytes(int64_t B, int F, int64_t M) {
  size_t tmp = 0;
  if (M > kGroupBins)
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (const int32_t*)nullptr,
                                             (int32_t*)nullptr, (int)B, 0, dfm_key_bits(M));
  else
    tmp = 3 * dfm_al256((size_t)M * 4) + dfm_al256(2 * kFusedMaxF * 4);
  return 4 * dfm_al256((size_t)B * 4) + dfm_al256((size_t)B * F * 4) + dfm_al256(tmp);
}

// Groups the rows by field key_field: returns the order (in ws) and the
// regrouped rows in *rows_out, or null when B does not fit the sort's int.
// franges_out (or null): the fields' id ranges when the counting sort ran
// (FusedDfmArgs::franges), else null.
const int32_t* dfm_order_rows(const int32_t* idx, int64_t B, int F, int key_field, int64_t M,
                              void* ws, const int32_t** rows_out, hipStream_t st,
                              const int32_t** franges_out) {
  if (franges_out) *franges_out = nullptr;
  if (B < 1 || B > 0x7fffffff) return nullptr;
  char* p = reinterpret_cast<char*>(ws);
  const size_t col = dfm_al256((size_t)B * 4);
  int32_t* rows = reinterpret_cast<int32_t*>(p + 4 * col);
  char* tmp_ws = p + 4 * col + dfm_al256((size_t)B * F * 4);
  int32_t* vout = reinterpret_cast<int32_t*>(p + 3 * col);
  if (M <= kGroupBins) {
    const size_t mb = dfm_al256((size_t)M * 4);
    uint32_t* count = reinterpret_cast<uint32_t*>(tmp_ws);
    uint32_t* cursor = reinterpret_cast<uint32_t*>(tmp_ws + mb);
    uint32_t* start = reinterpret_cast<uint32_t*>(tmp_ws + 2 * mb);
    int32_t* fr = franges_out && F <= kFusedMaxF
                      ? reinterpret_cast<int32_t*>(tmp_ws + 3 * mb) : nullptr;
    if (hipMemsetAsync(count, 0, 2 * mb, st) != hipSuccess) return nullptr;
    if (fr && hipMemsetAsync(fr, 0, 2 * kFusedMaxF * 4, st) != hipSuccess) return nullptr;
    const unsigned nblk = (unsigned)((B + kGroupRows - 1) / kGroupRows);
    hipLaunchKernelGGL(dfm_group_hist, dim3(nblk), dim3(1024), 0, st, idx, B, F, key_field, M,
                       count, fr);
    if (fr) *franges_out = fr;
    hipLaunchKernelGGL(dfm_group_scan, dim3(1), dim3(1024), 0, st, count, M, start);
    const unsigned sblk = (unsigned)((B + kScatterRows - 1) / kScatterRows);
    hipLaunchKernelGGL(dfm_group_scatter, dim3(sblk), dim3(1024), 0, st, idx, B, F, key_field,
                       M, start, cursor, rows, vout);
    *rows_out = rows;
    return vout;
  }
  uint32_t* kin = reinterpret_cast<uint32_t*>(p);
  uint32_t* kout = reinterpret_cast<uint32_t*>(p + col);
  int32_t* vin = reinterpret_cast<int32_t*>(p + 2 * col);
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kin, kout, vin, vout, (int)B, 0,
                                           dfm_key_bits(M), st);
  const int64_t nb = (B + 255) / 256 < 8192 ? (B + 255) / 256 : 8192;
  hipLaunchKernelGGL(dfm_order_keys, dim3((unsigned)nb), dim3(256), 0, st, idx, B, F, key_field,
                     M, kin, vin);
  if (hipcub::DeviceRadixSort::SortPairs(tmp_ws, tmp, kin, kout, vin, vout, (int)B, 0,
                                         dfm_key_bits(M), st) != hipSuccess)
    return nullptr;
  const int64_t gb = (B * F + 255) / 256 < 8192 ? (B * F + 255) / 256 : 8192;
  hipLaunchKernelGGL(dfm_gather_rows, dim3((unsigned)gb), dim3(256), 0, st, idx, vout, B, F, rows);
  *rows_out = rows;
  return vout;
}

}  // namespace hhfm

#if HHFM_F32S_TIMING
extern "C" int hhfm_debug_f32s_timing(unsigned long long* out) {
  hipDeviceSynchronize();
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hhfm::g_f32s_t), sizeof(hhfm::g_f32s_t)) != hipSuccess)
    return -1;
  static const unsigned long long zero[8] = {0};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(hhfm::g_f32s_t), zero, sizeof(zero));
}
#endif
