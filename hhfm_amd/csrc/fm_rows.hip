// K1 — per-row FM / HHFM scoring on gfx950 (HBM-bound sparse gather + reduce).
//
//   hhfm_fm_score_rows     replaces the FM.out graph        (Newcode/FM.py:99-120)
//   hhfm_hybrid_score_rows replaces OUR.PositiveFeadback    (Newcode/OurModel7.py:105-171)
//
// Layout / mapping:
//   * one embedding row = RV 16-byte chunks (RV = k*elem_size/16); a row is
//     owned by an aligned group of LPR = RV lanes, each lane issuing ONE
//     16-B load per field (global_load_dwordx4), so a wave-instruction moves
//     64 lanes x 16 B = 1 KiB of whole rows;
//   * every lane keeps U rows x F fields of loads in flight (~20 x 16 B) and
//     the index rows of the NEXT iteration are fetched before this
//     iteration's gathers are consumed (hides the idx->gather dependency);
//   * the ½((Σv)²−Σv²) interaction is reduced first inside the lane (4 or 8
//     elements), then across the LPR lanes with a DPP/ds_swizzle butterfly —
//     no LDS allocation, no atomics, one fp32 store per row.
#include "hhfm_common.h"

namespace hhfm {

// blocks per CU the grid is capped at (grid-stride beyond): at configs[1]
// 16 / 32 / 64 / 256 / 2048 ran 3.98 / 3.95 / 3.94 / 4.11 / 4.51 ms
// (profiles/r04_k1_grid_cap_ab.txt)
#ifndef HHFM_K1_CAP
#define HHFM_K1_CAP 64
#endif
// diagnostic (timing only, wrong results; default 0): where the `w` gathers
// are served from — 1: every w index folded into a 1 MB window (L2-resident),
// 2: w index x 32 (every gather its own 128-B line of a 2 GB array: no reuse
// in L2 or the Infinity Cache); scripts/diag/k1_wmap.sh
#ifndef HHFM_K1_WMAP
#define HHFM_K1_WMAP 0
#endif
// diagnostic (timing only, wrong results; default 0): 1 — fields 2.. (the
// context columns at configs[1]) keep their ids and `w` gathers but their
// embedding rows are not loaded (zeros); scripts/diag/k1_ctx_ko.sh
#ifndef HHFM_K1_CTXKO
#define HHFM_K1_CTXKO 0
#endif
#if (HHFM_K1_WMAP || HHFM_K1_CTXKO) && !defined(HHFM_DIAG_BUILD)
#error "K1 knock-out macros give wrong results: diagnostic builds only (-DHHFM_DIAG_BUILD)"
#endif
#ifndef HHFM_K1_U5
#define HHFM_K1_U5 5   // rows per lane in flight at F = 5
#endif
// F = 5 (configs[1]): 5 rows in flight per lane 3.98 ms against 4 4.11, 3
// 4.07, 6 5.05 (profiles/r04_k1_rows_in_flight_ab.txt); the HHFM rows and
// the bf16 tables gain or hold too (profiles/r04_k1_u5_microbench.txt)
template <int F>
struct RowsPerLane {
  static constexpr int value =
      F <= 3 ? 6 : (F == 4 ? 4 : (F == 5 ? HHFM_K1_U5 : (F <= 8 ? 3 : 2)));
};

// Raw (unclamped) index rows: nothing may consume them until the gathers
// issued before them are consumed, or the in-order vmcnt would serialise.
template <int F, int U, bool NT = false>
HHFM_DEV void load_ids(int32_t (&id)[U][F], const int32_t* __restrict__ idx,
                       int64_t base, int64_t B, int g, int RPW, int ncols) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    int64_t row = base + (int64_t)u * RPW + g;
    const int32_t* p = idx + (row < B ? row : 0) * (int64_t)ncols;
#pragma unroll
    for (int f = 0; f < F; ++f) id[u][f] = load_i32<NT>(p + f);
  }
}

// ---------------------------------------------------------------------------
// FM row kernel: out = Σ_k ½[(Σ_f e)² − Σ_f e²] + Σ_f w + w0
// ---------------------------------------------------------------------------
// NTM: 0 every load default, 1 every load non-temporal (HHFM_FLAG_STREAM_TABLE),
// 2 only the user and item rows (fields 0, 1) non-temporal — planned for
// tables far beyond the caches, where those rows are read once and the
// default policy lets them evict the re-read `w` lines and context rows from
// the Infinity Cache: 4.21 -> 4.11 ms at configs[1] (ids and output
// non-temporal as well: 4.53 ms; profiles/r04_k1_nt_ab.txt)
template <int F, int LPR, bool BF16, bool HAS_W, int NTM>
__global__ __launch_bounds__(256) void fm_rows_fast(
    const int32_t* __restrict__ idx, int64_t B, const char* __restrict__ E,
    int64_t M, const float* __restrict__ w, float w0, float* __restrict__ out,
    int32_t* __restrict__ status) {
  constexpr int U = RowsPerLane<F>::value;
  constexpr int RPW = kWave / LPR;  // rows per wave per unroll slot
  constexpr int RPI = RPW * U;      // rows per wave-iteration
  constexpr int64_t ROW_BYTES = (int64_t)LPR * 16;
  constexpr bool NT = NTM == 1;
  using C = Chunk<BF16>;

  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane & (LPR - 1);
  const int g = lane / LPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int64_t stride = nwave * RPI;

  int64_t base = wave * RPI;
  int32_t raw[U][F];
  bool bad = false;
  if (base < B) load_ids<F, U, NT>(raw, idx, base, B, g, RPW, F);

  for (; base < B; base += stride) {
    C c[U][F];
    int32_t id[U][F];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int f = 0; f < F; ++f) {
        id[u][f] = clamp_id(raw[u][f], M);
        bad |= id[u][f] != raw[u][f];
        if (HHFM_K1_CTXKO && f >= 2) {
#pragma unroll
          for (int e = 0; e < C::kElems; ++e) c[u][f].v[e] = 0.f;
        } else if (NTM == 2 && f < 2)
          c[u][f].template load<true>(E + (int64_t)id[u][f] * ROW_BYTES + sub * 16);
        else
          c[u][f].template load<NT>(E + (int64_t)id[u][f] * ROW_BYTES + sub * 16);
      }

    // Σ_f w[x_f]: lane `sub` gathers fields f ≡ sub (mod LPR); loads are
    // unconditional (clamped ids) so the vmcnt counting stays exact
    float wv[U];
    if constexpr (HAS_W) {
      constexpr int WPL = (F + LPR - 1) / LPR;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        wv[u] = 0.f;
#pragma unroll
        for (int r = 0; r < WPL; ++r) {
          const int fsel = r * LPR + sub;
          int32_t my = id[u][0];
#pragma unroll
          for (int f = 1; f < F; ++f) my = (fsel == f) ? id[u][f] : my;
          const float wl = HHFM_K1_WMAP == 1   ? w[my & 0x3ffff]
                           : HHFM_K1_WMAP == 2 ? w[(int64_t)my * 32]
                                               : w[my];
          wv[u] += (fsel < F) ? wl : 0.f;
        }
      }
    }

    // prefetch next iteration's index rows before consuming the gathers
    // (unconditional: rows past B read row 0, which keeps vmcnt counting exact)
    load_ids<F, U, NT>(raw, idx, base + stride, B, g, RPW, F);

#pragma unroll
    for (int u = 0; u < U; ++u) {
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < C::kElems; ++e) {
        float s = c[u][0].v[e];
        float q = c[u][0].v[e] * c[u][0].v[e];
#pragma unroll
        for (int f = 1; f < F; ++f) {
          s += c[u][f].v[e];
          q += c[u][f].v[e] * c[u][f].v[e];
        }
        t += 0.5f * (s * s - q);
      }
      t = group_sum<LPR>(t);
      float fb = 0.f;
      if constexpr (HAS_W) fb = group_sum<LPR>(wv[u]);
      const int64_t row = base + (int64_t)u * RPW + g;
      if (sub == 0 && row < B) {
        if constexpr (NT) __builtin_nontemporal_store((t + fb) + w0, out + row);
        else out[row] = (t + fb) + w0;
      }
    }
  }
  report_bad_id(status, bad);
}

// Generic fallback (any k, any F <= 64): one wave per row, lanes stride over k.
template <bool BF16>
__global__ __launch_bounds__(256) void fm_rows_generic(
    const int32_t* __restrict__ idx, int64_t B, int F, const char* __restrict__ E,
    int64_t M, int k, const float* __restrict__ w, float w0,
    float* __restrict__ out, int32_t* __restrict__ status) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int esz = BF16 ? 2 : 4;
  bool bad = false;
  for (int64_t row = wave; row < B; row += nwave) {
    const int32_t* p = idx + row * (int64_t)F;
    for (int f = lane; f < F; f += kWave) bad |= clamp_id(p[f], M) != p[f];
    float t = 0.f;
    for (int e = lane; e < k; e += kWave) {
      float s = 0.f, q = 0.f;
      for (int f = 0; f < F; ++f) {
        const char* r = E + (int64_t)clamp_id(p[f], M) * k * esz;
        float v = BF16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(r)[e])
                       : reinterpret_cast<const float*>(r)[e];
        s += v;
        q += v * v;
      }
      t += 0.5f * (s * s - q);
    }
    t = group_sum<kWave>(t);
    float fb = 0.f;
    if (w != nullptr)
      for (int f = 0; f < F; ++f) fb += w[clamp_id(p[f], M)];
    if (lane == 0) out[row] = (t + fb) + w0;
  }
  report_bad_id(status, bad);
}

// ---------------------------------------------------------------------------
// HHFM row kernel, canonical column layout [user, item, ctx x NC, time x rest]
//   h = (u + Σctx) + Σtime ; out = Σ_k h·item
// ---------------------------------------------------------------------------
template <int F, int LPR, bool BF16>
__global__ __launch_bounds__(256) void hybrid_rows_fast(
    const int32_t* __restrict__ idx, int64_t B, int nctx,
    const char* __restrict__ E, int64_t M, float* __restrict__ out,
    int32_t* __restrict__ status) {
  constexpr int U = RowsPerLane<F>::value;
  constexpr int RPW = kWave / LPR;
  constexpr int RPI = RPW * U;
  constexpr int64_t ROW_BYTES = (int64_t)LPR * 16;
  using C = Chunk<BF16>;

  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane & (LPR - 1);
  const int g = lane / LPR;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int64_t stride = nwave * RPI;
  const int ctx_end = 2 + nctx;

  int64_t base = wave * RPI;
  int32_t raw[U][F];
  bool bad = false;
  if (base < B) load_ids<F, U>(raw, idx, base, B, g, RPW, F);

  for (; base < B; base += stride) {
    C c[U][F];
    int32_t id[U][F];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int f = 0; f < F; ++f) {
        id[u][f] = clamp_id(raw[u][f], M);
        bad |= id[u][f] != raw[u][f];
        c[u][f].load(E + (int64_t)id[u][f] * ROW_BYTES + sub * 16);
      }

    // (unconditional: rows past B read row 0, which keeps vmcnt counting exact)
    load_ids<F, U>(raw, idx, base + stride, B, g, RPW, F);

#pragma unroll
    for (int u = 0; u < U; ++u) {
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < C::kElems; ++e) {
        float ctx = 0.f, tim = 0.f;
#pragma unroll
        for (int f = 2; f < F; ++f) {
          if (f < ctx_end) ctx += c[u][f].v[e];
          else tim += c[u][f].v[e];
        }
        float h = c[u][0].v[e];
        if (nctx > 0) h = h + ctx;
        if (ctx_end < F) h = h + tim;
        t += h * c[u][1].v[e];
      }
      t = group_sum<LPR>(t);
      const int64_t row = base + (int64_t)u * RPW + g;
      if (sub == 0 && row < B) out[row] = t;
    }
  }
  report_bad_id(status, bad);
}

template <bool BF16>
__global__ __launch_bounds__(256) void hybrid_rows_generic(
    const int32_t* __restrict__ idx, int64_t B, int ncols, int ucol, int icol,
    int c0, int c1, int t0, int t1, const char* __restrict__ E, int64_t M,
    int k, float* __restrict__ out, int32_t* __restrict__ status) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int esz = BF16 ? 2 : 4;
  auto val = [&](int32_t id, int e) -> float {
    const char* r = E + (int64_t)clamp_id(id, M) * k * esz;
    return BF16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(r)[e])
                : reinterpret_cast<const float*>(r)[e];
  };
  bool bad = false;
  for (int64_t row = wave; row < B; row += nwave) {
    const int32_t* p = idx + row * (int64_t)ncols;
    // only the columns the score reads (user, item, ctx, time), like
    // check_query_ids_kernel: an unused column never raises
    for (int c = lane; c < ncols; c += kWave)
      if (c == ucol || c == icol || (c >= c0 && c < c1) || (c >= t0 && c < t1))
        bad |= clamp_id(p[c], M) != p[c];
    float t = 0.f;
    for (int e = lane; e < k; e += kWave) {
      float h = val(p[ucol], e);
      if (c1 > c0) {
        float s = 0.f;
        for (int c = c0; c < c1; ++c) s += val(p[c], e);
        h = h + s;
      }
      if (t1 > t0) {
        float s = 0.f;
        for (int c = t0; c < t1; ++c) s += val(p[c], e);
        h = h + s;
      }
      t += h * val(p[icol], e);
    }
    t = group_sum<kWave>(t);
    if (lane == 0) out[row] = t;
  }
  report_bad_id(status, bad);
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------
static int grid_for(int64_t rows, int64_t rows_per_block) {
  int64_t g = (rows + rows_per_block - 1) / rows_per_block;
  const int64_t cap = 256 * HHFM_K1_CAP;  // 256 CUs x HHFM_K1_CAP blocks; grid-stride the rest
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

template <int F, int LPR, bool BF16>
static void launch_fm_fast(const int32_t* idx, int64_t B, const char* E,
                           int64_t M, const float* w, float w0, float* out,
                           bool nt, int32_t* status, hipStream_t s) {
  constexpr int RPB = 4 * (kWave / LPR) * RowsPerLane<F>::value;
  const int grid = grid_for(B, RPB);
  // rows far beyond the caches: the user / item rows streamed (NTM 2)
  const bool big = M * (int64_t)LPR * 16 >= ((int64_t)1 << 30);
  if (w && nt)
    hipLaunchKernelGGL((fm_rows_fast<F, LPR, BF16, true, 1>), dim3(grid),
                       dim3(256), 0, s, idx, B, E, M, w, w0, out, status);
  else if (w && big && F >= 2)
    hipLaunchKernelGGL((fm_rows_fast<F, LPR, BF16, true, 2>), dim3(grid),
                       dim3(256), 0, s, idx, B, E, M, w, w0, out, status);
  else if (w)
    hipLaunchKernelGGL((fm_rows_fast<F, LPR, BF16, true, 0>), dim3(grid),
                       dim3(256), 0, s, idx, B, E, M, w, w0, out, status);
  else
    hipLaunchKernelGGL((fm_rows_fast<F, LPR, BF16, false, 0>), dim3(grid),
                       dim3(256), 0, s, idx, B, E, M, w, w0, out, status);
}

template <int F, int LPR, bool BF16>
static void launch_hybrid_fast(const int32_t* idx, int64_t B, int nctx,
                               const char* E, int64_t M, float* out,
                               int32_t* status, hipStream_t s) {
  constexpr int RPB = 4 * (kWave / LPR) * RowsPerLane<F>::value;
  const int grid = grid_for(B, RPB);
  hipLaunchKernelGGL((hybrid_rows_fast<F, LPR, BF16>), dim3(grid), dim3(256), 0,
                     s, idx, B, nctx, E, M, out, status);
}

// dispatch on LPR (16-byte chunks per row) for a fixed F and dtype
#define HHFM_LPR_SWITCH(LAUNCH, F, BF16, ...)            \
  switch (lpr) {                                         \
    case 4: LAUNCH<F, 4, BF16>(__VA_ARGS__); break;      \
    case 8: LAUNCH<F, 8, BF16>(__VA_ARGS__); break;      \
    case 16: LAUNCH<F, 16, BF16>(__VA_ARGS__); break;    \
    case 32: LAUNCH<F, 32, BF16>(__VA_ARGS__); break;    \
    case 64: LAUNCH<F, 64, BF16>(__VA_ARGS__); break;    \
    default: return false;                               \
  }

#define HHFM_F_SWITCH(LAUNCH, BF16, ...)                          \
  switch (F) {                                                    \
    case 2: HHFM_LPR_SWITCH(LAUNCH, 2, BF16, __VA_ARGS__) break;   \
    case 3: HHFM_LPR_SWITCH(LAUNCH, 3, BF16, __VA_ARGS__) break;   \
    case 4: HHFM_LPR_SWITCH(LAUNCH, 4, BF16, __VA_ARGS__) break;   \
    case 5: HHFM_LPR_SWITCH(LAUNCH, 5, BF16, __VA_ARGS__) break;   \
    case 6: HHFM_LPR_SWITCH(LAUNCH, 6, BF16, __VA_ARGS__) break;   \
    case 7: HHFM_LPR_SWITCH(LAUNCH, 7, BF16, __VA_ARGS__) break;   \
    case 8: HHFM_LPR_SWITCH(LAUNCH, 8, BF16, __VA_ARGS__) break;   \
    case 10: HHFM_LPR_SWITCH(LAUNCH, 10, BF16, __VA_ARGS__) break; \
    case 12: HHFM_LPR_SWITCH(LAUNCH, 12, BF16, __VA_ARGS__) break; \
    default: return false;                                        \
  }

static bool try_fm_fast(const int32_t* idx, int64_t B, int F, const char* E,
                        int64_t M, int lpr, bool bf16, const float* w, float w0,
                        float* out, bool nt, int32_t* status, hipStream_t s) {
  if (bf16) {
    HHFM_F_SWITCH(launch_fm_fast, true, idx, B, E, M, w, w0, out, nt, status, s)
  } else {
    HHFM_F_SWITCH(launch_fm_fast, false, idx, B, E, M, w, w0, out, nt, status, s)
  }
  return true;
}

static bool try_hybrid_fast(const int32_t* idx, int64_t B, int F, int nctx,
                            const char* E, int64_t M, int lpr, bool bf16,
                            float* out, int32_t* status, hipStream_t s) {
  if (bf16) {
    HHFM_F_SWITCH(launch_hybrid_fast, true, idx, B, nctx, E, M, out, status, s)
  } else {
    HHFM_F_SWITCH(launch_hybrid_fast, false, idx, B, nctx, E, M, out, status, s)
  }
  return true;
}

static int lpr_for(int64_t k, int dtype) {
  const int64_t row_bytes = k * (dtype == HHFM_BF16 ? 2 : 4);
  if (row_bytes % 16) return 0;
  return (int)(row_bytes / 16);
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_fm_score_rows_ex(const int32_t* idx, int64_t B, int32_t F,
                                     const void* E, int64_t features_M, int32_t k,
                                     int32_t dtype, const float* w, float w0,
                                     float* out, int32_t flags, int32_t* status,
                                     void* stream) {
  if (B < 0 || F < 1 || F > 64 || k < 1 || features_M < 1) return HHFM_EINVAL;
  if (dtype != HHFM_F32 && dtype != HHFM_BF16) return HHFM_EINVAL;
  if (flags & ~HHFM_FLAG_STREAM_TABLE) return HHFM_EINVAL;
  if (B == 0) return HHFM_OK;
  if (!idx || !E || !out) return HHFM_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool bf16 = dtype == HHFM_BF16;
  const int lpr = lpr_for(k, dtype);
  const bool aligned = (reinterpret_cast<uintptr_t>(E) & 15) == 0;
  if (!(lpr && aligned &&
        try_fm_fast(idx, B, F, reinterpret_cast<const char*>(E), features_M,
                    lpr, bf16, w, w0, out, (flags & HHFM_FLAG_STREAM_TABLE) != 0, status,
                    s))) {
    const int grid = grid_for(B, 4);
    if (bf16)
      hipLaunchKernelGGL(fm_rows_generic<true>, dim3(grid), dim3(256), 0, s, idx,
                         B, F, reinterpret_cast<const char*>(E), features_M, k,
                         w, w0, out, status);
    else
      hipLaunchKernelGGL(fm_rows_generic<false>, dim3(grid), dim3(256), 0, s,
                         idx, B, F, reinterpret_cast<const char*>(E),
                         features_M, k, w, w0, out, status);
  }
  return (int)hipGetLastError();
}

extern "C" int hhfm_fm_score_rows(const int32_t* idx, int64_t B, int32_t F,
                                  const void* E, int64_t features_M, int32_t k,
                                  int32_t dtype, const float* w, float w0,
                                  float* out, void* stream) {
  return hhfm_fm_score_rows_ex(idx, B, F, E, features_M, k, dtype, w, w0, out,
                               HHFM_FM_ROWS_DEFAULT_FLAGS, nullptr, stream);
}

extern "C" int hhfm_hybrid_score_rows_ex(const int32_t* idx, int64_t B,
                                         int32_t ncols, int32_t user_col,
                                         int32_t item_col, int32_t ctx_begin,
                                         int32_t ctx_end, int32_t time_begin,
                                         int32_t time_end, const void* E,
                                         int64_t features_M, int32_t k,
                                         int32_t dtype, float* out, int32_t* status,
                                         void* stream) {
  if (B < 0 || ncols < 2 || ncols > 64 || k < 1 || features_M < 1)
    return HHFM_EINVAL;
  if (dtype != HHFM_F32 && dtype != HHFM_BF16) return HHFM_EINVAL;
  auto in_range = [&](int c) { return c >= 0 && c < ncols; };
  if (!in_range(user_col) || !in_range(item_col)) return HHFM_EINVAL;
  if (ctx_begin > ctx_end || time_begin > time_end) return HHFM_EINVAL;
  if (ctx_end > ctx_begin && (!in_range(ctx_begin) || ctx_end > ncols))
    return HHFM_EINVAL;
  if (time_end > time_begin && (!in_range(time_begin) || time_end > ncols))
    return HHFM_EINVAL;
  if (B == 0) return HHFM_OK;
  if (!idx || !E || !out) return HHFM_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool bf16 = dtype == HHFM_BF16;
  const int lpr = lpr_for(k, dtype);
  const bool aligned = (reinterpret_cast<uintptr_t>(E) & 15) == 0;
  const int nctx = ctx_end - ctx_begin;
  const int ntime = time_end - time_begin;
  // canonical layout: [user, item, ctx..., time...] spanning every column
  const bool canonical = user_col == 0 && item_col == 1 &&
                         (nctx == 0 || ctx_begin == 2) &&
                         (ntime == 0 || time_begin == 2 + nctx) &&
                         2 + nctx + ntime == ncols;
  if (!(canonical && lpr && aligned &&
        try_hybrid_fast(idx, B, ncols, nctx,
                        reinterpret_cast<const char*>(E), features_M, lpr,
                        bf16, out, status, s))) {
    const int grid = grid_for(B, 4);
    if (bf16)
      hipLaunchKernelGGL(hybrid_rows_generic<true>, dim3(grid), dim3(256), 0, s,
                         idx, B, ncols, user_col, item_col, ctx_begin, ctx_end,
                         time_begin, time_end,
                         reinterpret_cast<const char*>(E), features_M, k, out, status);
    else
      hipLaunchKernelGGL(hybrid_rows_generic<false>, dim3(grid), dim3(256), 0,
                         s, idx, B, ncols, user_col, item_col, ctx_begin,
                         ctx_end, time_begin, time_end,
                         reinterpret_cast<const char*>(E), features_M, k, out, status);
  }
  return (int)hipGetLastError();
}

extern "C" int hhfm_hybrid_score_rows(const int32_t* idx, int64_t B,
                                      int32_t ncols, int32_t user_col,
                                      int32_t item_col, int32_t ctx_begin,
                                      int32_t ctx_end, int32_t time_begin,
                                      int32_t time_end, const void* E,
                                      int64_t features_M, int32_t k,
                                      int32_t dtype, float* out, void* stream) {
  return hhfm_hybrid_score_rows_ex(idx, B, ncols, user_col, item_col, ctx_begin, ctx_end,
                                   time_begin, time_end, E, features_M, k, dtype, out,
                                   nullptr, stream);
}

extern "C" const char* hhfm_error_string(int code) {
  switch (code) {
    case HHFM_OK: return "ok";
    case HHFM_EINVAL: return "invalid argument";
    case HHFM_EUNSUPPORTED: return "unsupported shape";
    case HHFM_EWORKSPACE: return "workspace too small";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
  }
}

extern "C" int hhfm_abi_version(void) { return HHFM_ABI_VERSION; }
