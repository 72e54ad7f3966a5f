// K3 — DeepFM on gfx950: LDS-tiled MFMA GEMM with a row-gathered A operand
// and fused epilogues, plus the small kernels around it.
//
//   hhfm_dfm_forward        replaces DeepFM.out   (Newcode/DFM.py:104-137)
//   hhfm_dfm_catalog_topk   replaces DeepFM.topk  (Newcode/DFM.py:219-231)
//   hhfm_topk_dense         replaces tf.nn.top_k on a materialised [B,N]
//                           score matrix (DFM.py:230, AFM.py:245)
//
// GEMM tile: 128 x 128 per 256-thread workgroup (4 waves, 2x2, 64x64 per
// wave); K staged through double-buffered LDS with one barrier per K-step.
//   bf16 mode: v_mfma_f32_16x16x32_bf16, BK = 32, fp32 accumulate;
//   f32  mode: v_mfma_f32_16x16x4_f32  (exact fp32 fmaf chains), BK = 16,
//              each lane reads 4 consecutive k with one ds_read_b128 and
//              feeds them to 4 MFMAs (k-permuted identically for A and B).
// A modes: dense [M][lda] (hidden activations) or gathered — row m is the
// concatenation of the F field embeddings E[idx[m][f]] (DFM.py:104,125), read
// straight from the table (no [B, F*k] staging buffer in HBM).
// Epilogues: (a) relu(acc + bias) stored as bf16 / f32 (DFM.py:127-128);
// (b) relu(acc + bias) · v summed over the tile's columns into per-row
// partials (last hidden layer fused with the concat projection, DFM.py:137).
#include <cstdlib>

#include "gemm_mfma.h"

namespace hhfm {

bool dfm_fused_eligible(int L, const int32_t* dims);
size_t dfm_fused_pack_bytes(int L, const int32_t* dims, bool mlp_bf16);
bool dfm_fused_launch(const int32_t* idx, int64_t B, int F, const void* E, int64_t M, int k,
                      bool tbf, bool mlp_bf16, const float* w, int L, const int32_t* dims,
                      const void* const* Wt, const float* const* bias, const float* Wp, float bp,
                      float* out, void* pack_ws, const void* proj, int proj_from,
                      uint64_t perm, const int32_t* order, float* fm_base, void* scratch,
                      size_t scratch_bytes, int32_t plan, bool* pairs_ready, hipStream_t st,
                      const int32_t* franges);
bool dfm_proj_eligible(int F, int k, int L, const int32_t* dims);
size_t dfm_proj_bytes(int F, int proj_from, int64_t M, int L, const int32_t* dims);
void dfm_project_layer0(const void* E, int64_t M, int k, bool tbf, bool mlp_bf16, int F,
                        int proj_from, uint64_t perm, const void* Wt0, int N0, int L,
                        const int32_t* dims, void* ws, hipStream_t st);
size_t dfm_order_bytes(int64_t B, int F, int64_t M);
inline bool dfm_f32_split(int32_t plan) { return !(plan & HHFM_PLAN_EXACT_FP32); }
const int32_t* dfm_order_rows(const int32_t* idx, int64_t B, int F, int key_field, int64_t M,
                              void* ws, const int32_t** rows_out, hipStream_t st,
                              const int32_t** franges_out);
constexpr uint64_t kDfmIdentityPerm = 0xFEDCBA9876543210ull;

// ---------------------------------------------------------------------------
// FM part of DeepFM and the final reduce
//   base[m] = Σ_f w[x_f]·Wp[f] + Σ_c y2_c·Wp[F+c] + bp        (DFM.py:109-122,132,137)
//   out[m]  = base[m] + Σ_t partial[m][t]
// ---------------------------------------------------------------------------
template <bool TBF>
__global__ __launch_bounds__(256) void dfm_fm_part(const int32_t* __restrict__ idx,
                                                   int64_t B, int F, const void* __restrict__ E,
                                                   int64_t M, int k, const float* __restrict__ w,
                                                   const float* __restrict__ Wp, float bp,
                                                   float* __restrict__ base) {
  const int l = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t m = wave; m < B; m += nwave) {
    const int32_t* p = idx + m * F;
    float acc = 0.f;
    for (int c = l; c < k; c += kWave) {
      float s = 0.f, q = 0.f;
      for (int f = 0; f < F; ++f) {
        const int64_t id = clamp_id(p[f], M);
        const float v = TBF ? bf16_to_f32(reinterpret_cast<const uint16_t*>(E)[id * k + c])
                            : reinterpret_cast<const float*>(E)[id * k + c];
        s += v;
        q += v * v;
      }
      acc += 0.5f * (s * s - q) * Wp[F + c];
    }
    acc = group_sum<kWave>(acc);
    if (l == 0) {
      float y1 = 0.f;
      for (int f = 0; f < F; ++f) y1 += w[clamp_id(p[f], M)] * Wp[f];
      base[m] = (y1 + acc) + bp;
    }
  }
}

__global__ __launch_bounds__(256) void dfm_reduce(const float* __restrict__ base,
                                                  const float* __restrict__ partial, int nt,
                                                  int64_t B, float* __restrict__ out) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B) return;
  float s = 0.f;
  for (int t = 0; t < nt; ++t) s += partial[m * nt + t];
  out[m] = base[m] + s;
}

// rows[b*N + i] = qidx[b] with column item_col replaced by item_row_begin + i
__global__ __launch_bounds__(256) void dfm_build_rows(const int32_t* __restrict__ q, int64_t B,
                                                      int F, int item_col, int32_t item_row_begin,
                                                      int32_t N, int32_t* __restrict__ rows) {
  const int64_t total = B * (int64_t)N * F;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(x % F);
    const int64_t r = x / F;
    const int64_t b = r / N;
    const int32_t i = (int32_t)(r - b * N);
    rows[x] = f == item_col ? item_row_begin + i : q[b * F + f];
  }
}


// workspace: [base B][partial B*ntiles][h0 B*maxL][h1 B*maxL][packed weights of
// the fused kernels, when their envelope admits the layer widths][projected
// layer 0 (dfm_fused.hip), when planned][row order, when planned]
struct DfmPlan {
  size_t off_base, off_part, off_h0, off_h1, off_pack, off_proj, off_order, total;
  int maxL, ntl;
  bool proj;
  int proj_from;   // internal fields [proj_from, F) come from P
  uint64_t perm;   // internal field j = caller's field (perm >> 4j) & 15
  bool group;      // rows grouped by the caller's field perm(proj_from) (forward)
};

static size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
// activations / weights keep their K dimension padded to 8 (16-B rows)
static int pad8(int x) { return (x + 7) & ~7; }

// Projected layer 0 (dfm_fused.hip): at most this much workspace for P.
constexpr size_t kProjMaxBytes = size_t(1) << 30;

// proj_mode (include/hhfm.h hhfm_dfm_proj): OFF plans no projection (F, k,
// M unused); ON projects every field; CTX the fields >= 2 (LoadData's
// contexts after user and item; bf16 MLP); ITEM every field but the item
// (bf16 MLP; the item is field 1 of a forward row, item_col of a catalog row)
// with the forward's rows grouped by field 0, so a block's user P rows stage
// in LDS like the contexts' (a catalog block is one query already) — each
// whenever the fused kernels admit the shape and P fits kProjMaxBytes.
// AUTO: nothing below rows_total = 2·M (P costs one layer-0 row per table
// row and projected field); ON for the fp32 MLP; for the bf16 MLP ITEM in
// the catalog, and in the forward once rows_total >= 64·M (grouping pays
// when a user has many rows), CTX below that.  Projecting the user and item
// fields straight from HBM is not a win with the bf16 MLP: their P rows are
// table-random fp32 rows, more bytes per row than the weight stream they
// replace (profiles/r02_dfm_ctx_phases.json).
static DfmPlan dfm_plan(int64_t B, int nlayers, const int32_t* dims, int mlp_dtype, int F = 0,
                        int k = 0, int64_t M = 0, int64_t rows_total = 0,
                        int proj_mode = HHFM_DFM_PROJ_OFF, int item_field = 1,
                        bool forward = true, int32_t plan = HHFM_PLAN_DEFAULT) {
  DfmPlan p{};
  p.maxL = 0;
  for (int i = 0; i < nlayers; ++i) p.maxL = pad8(dims[i]) > p.maxL ? pad8(dims[i]) : p.maxL;
  p.ntl = (dims[nlayers - 1] + GBN - 1) / GBN;
  const size_t esz = mlp_dtype == HHFM_BF16 ? 2 : 4;
  size_t off = 0;
  p.off_base = off; off += al256((size_t)B * 4);
  p.off_part = off; off += al256((size_t)B * p.ntl * 4);
  p.off_h0 = off; off += al256((size_t)B * p.maxL * esz);
  p.off_h1 = off; off += al256((size_t)B * p.maxL * esz);
  p.off_pack = off;
  if (dfm_fused_eligible(nlayers, dims))
    off += al256(dfm_fused_pack_bytes(nlayers, dims, mlp_dtype == HHFM_BF16));
  p.off_proj = off;
  p.proj_from = -1;
  p.perm = kDfmIdentityPerm;
  const bool bf = mlp_dtype == HHFM_BF16;
  int mode = proj_mode;
  if (mode == HHFM_DFM_PROJ_AUTO)
    mode = rows_total < 2 * M ? HHFM_DFM_PROJ_OFF
           : !bf ? HHFM_DFM_PROJ_ON
           : (!forward || rows_total >= 64 * M) ? HHFM_DFM_PROJ_ITEM
           : HHFM_DFM_PROJ_CTX;
  int from = -1;
  uint64_t perm = kDfmIdentityPerm;
  if (mode == HHFM_DFM_PROJ_ON) from = 0;
  if (mode == HHFM_DFM_PROJ_CTX && bf && F >= 3) from = 2;
  if (mode == HHFM_DFM_PROJ_ITEM && bf && F >= 2 && item_field >= 0 && item_field < F) {
    from = 1;
    perm = (uint64_t)item_field;   // the item first, then the others in order
    for (int f = 0, j = 1; f < F; ++f)
      if (f != item_field) perm |= (uint64_t)f << (4 * j++);
    for (int j = F; j < 16; ++j) perm |= (uint64_t)j << (4 * j);
  }
  if (from >= 0 && M > 0 && dfm_proj_eligible(F, k, nlayers, dims)) {
    const size_t pb = dfm_proj_bytes(F, from, M, nlayers, dims);
    if (pb <= kProjMaxBytes) {
      p.proj = true;
      p.proj_from = from;
      p.perm = perm;
      off += al256(pb);
      p.off_order = off;
      // fp32 MLP on the split kernel: rows grouped by user too (a block then
      // reads one or two users' P rows: L1/L2 hits instead of Infinity-Cache
      // reads); HHFM_PLAN_UNGROUPED turns it off
      const bool f32_group = !bf && mode == HHFM_DFM_PROJ_ON && forward && nlayers > 1 &&
                             rows_total >= 64 * M && !(plan & HHFM_PLAN_UNGROUPED) &&
                             dfm_f32_split(plan);
      if (((mode == HHFM_DFM_PROJ_ITEM) || f32_group) && forward && B <= 0x7fffffff) {
        p.group = true;
        off += al256(dfm_order_bytes(B, F, M));
      }
    }
  }
  if (!p.group) p.off_order = off;
  p.total = off;
  return p;
}

// The fused kernels stream Wt by 16-B LDS-DMA (dfm_fused_launch declines a
// misaligned view); a projected plan needs them, so a misaligned Wt plans
// the direct path instead of failing after P was put on the stream.
static bool wt_aligned(int32_t nlayers, const void* const* Wt) {
  for (int i = 0; i < nlayers; ++i)
    if (reinterpret_cast<uintptr_t>(Wt[i]) & 15) return false;
  return true;
}

static bool proj_mode_ok(int m) {
  return m == HHFM_DFM_PROJ_OFF || m == HHFM_DFM_PROJ_ON || m == HHFM_DFM_PROJ_AUTO ||
         m == HHFM_DFM_PROJ_CTX || m == HHFM_DFM_PROJ_ITEM;
}

static int dfm_check(int64_t B, int32_t F, int32_t k, int32_t dtype, int32_t nlayers,
                     const int32_t* dims, int32_t mlp_dtype) {
  if (B < 0 || F < 1 || k < 1 || nlayers < 1 || nlayers > 16 || !dims) return HHFM_EINVAL;
  if ((dtype != HHFM_F32 && dtype != HHFM_BF16) ||
      (mlp_dtype != HHFM_F32 && mlp_dtype != HHFM_BF16))
    return HHFM_EINVAL;
  const int el = mlp_dtype == HHFM_BF16 ? 8 : 4;
  if (k % el) return HHFM_EUNSUPPORTED;  // gathered A chunks never straddle fields
  for (int i = 0; i < nlayers; ++i)
    if (dims[i] < 1) return HHFM_EINVAL;
  return HHFM_OK;
}

// proj: P from dfm_project_layer0 (the fused PROJ kernels then run), or null
static int dfm_forward_impl(const int32_t* idx, int64_t B, int32_t F, const void* E,
                            int64_t M, int32_t k, int32_t dtype, const float* w,
                            int32_t nlayers, const int32_t* dims, const void* const* Wt,
                            const float* const* bias, int32_t mlp_dtype, const float* Wp,
                            float bp, float* out, char* ws, const DfmPlan& p, const void* proj,
                            const int32_t* order, int32_t plan, bool* pairs_ready,
                            hipStream_t st, const int32_t* franges = nullptr) {
  const bool bf = mlp_dtype == HHFM_BF16;
  // One fused kernel per row block when the shape fits (dfm_fused.hip /
  // dfm_wide.hip, bf16 or fp32 MLP); the layer-by-layer GEMMs otherwise.
  if (p.off_proj > p.off_pack &&
      dfm_fused_launch(idx, B, F, E, M, k, dtype == HHFM_BF16, bf, w, nlayers, dims, Wt, bias,
                       Wp, bp, out, ws + p.off_pack, proj, p.proj_from, p.perm, order,
                       reinterpret_cast<float*>(ws + p.off_base), ws + p.off_h0,
                       p.off_pack - p.off_h0, plan, pairs_ready, st, franges))
    return (int)hipGetLastError();
  if (proj) return HHFM_EUNSUPPORTED;   // planned only inside the fused envelope
  float* base = reinterpret_cast<float*>(ws + p.off_base);
  float* part = reinterpret_cast<float*>(ws + p.off_part);
  void* h[2] = {ws + p.off_h0, ws + p.off_h1};
  {
    int64_t blocks = (B + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    if (dtype == HHFM_BF16)
      hipLaunchKernelGGL(dfm_fm_part<true>, dim3((int)blocks), dim3(256), 0, st, idx, B, F, E, M,
                         k, w, Wp, bp, base);
    else
      hipLaunchKernelGGL(dfm_fm_part<false>, dim3((int)blocks), dim3(256), 0, st, idx, B, F, E,
                         M, k, w, Wp, bp, base);
  }
  int Kin = F * k;  // layer 0: gathered rows, K = F*k (k % 8 checked)
  for (int i = 0; i < nlayers; ++i) {
    GemmArgs g{};
    g.M = B;
    g.N = dims[i];
    g.K = Kin;
    if (i == 0) {
      g.gidx = idx; g.T = E; g.Mtab = M; g.F = F; g.kf = k; g.t_bf16 = dtype == HHFM_BF16;
    } else {
      g.A = h[(i - 1) & 1]; g.lda = Kin;
    }
    g.Bt = Wt[i];
    g.ldb = Kin;
    g.bias = bias[i];
    g.relu = 1;  // DFM.py:128 applies the activation after EVERY layer
    const bool last = i == nlayers - 1;
    if (!last) {
      g.C = h[i & 1]; g.ldc = pad8(dims[i]); g.c_bf16 = bf;
    } else {
      g.dotv = Wp + F + k; g.partial = part;
    }
    launch_gemm(g, bf, last ? 1 : 0, st);
    Kin = pad8(dims[i]);
  }
  hipLaunchKernelGGL(dfm_reduce, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, base, part,
                     p.ntl, B, out);
  return (int)hipGetLastError();
}

}  // namespace hhfm

using namespace hhfm;

extern "C" int hhfm_dfm_forward_workspace(int64_t B, int32_t nlayers, const int32_t* layer_dims,
                                          int32_t mlp_dtype, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || nlayers < 1 || !layer_dims) return HHFM_EINVAL;
  *ws_bytes = dfm_plan(B, nlayers, layer_dims, mlp_dtype).total;
  return HHFM_OK;
}

static bool plan_ok(int32_t plan) { return !(plan & ~HHFM_PLAN_ALL); }

extern "C" int hhfm_dfm_forward_workspace_ex(int64_t B, int32_t F, int32_t k,
                                             int64_t features_M, int32_t nlayers,
                                             const int32_t* layer_dims, int32_t mlp_dtype,
                                             int32_t proj_mode, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || F < 1 || k < 1 || features_M < 1 || nlayers < 1 || !layer_dims)
    return HHFM_EINVAL;
  if (!proj_mode_ok(proj_mode)) return HHFM_EINVAL;
  *ws_bytes = dfm_plan(B, nlayers, layer_dims, mlp_dtype, F, k, features_M, B, proj_mode).total;
  return HHFM_OK;
}

static int dfm_forward_planned(const int32_t* idx, int64_t B, int32_t F, const void* E,
                               int64_t features_M, int32_t k, int32_t dtype, const float* w,
                               int32_t nlayers, const int32_t* layer_dims,
                               const void* const* Wt, const float* const* bias,
                               int32_t mlp_dtype, const float* Wp, float bp, float* out,
                               char* ws, const DfmPlan& p, int32_t plan, hipStream_t st) {
  const void* proj = nullptr;
  const int32_t* order = nullptr;
  const int32_t* franges = nullptr;
  if (p.proj) {
    dfm_project_layer0(E, features_M, k, dtype == HHFM_BF16, mlp_dtype == HHFM_BF16, F,
                       p.proj_from, p.perm, Wt[0], layer_dims[0], nlayers, layer_dims,
                       ws + p.off_proj, st);
    proj = ws + p.off_proj;
    const int32_t* grouped = nullptr;
    if (p.group)
      order = dfm_order_rows(idx, B, F, (int)((p.perm >> (4 * p.proj_from)) & 15), features_M,
                             ws + p.off_order, &grouped, st, &franges);
    if (order) idx = grouped;
  }
  return dfm_forward_impl(idx, B, F, E, features_M, k, dtype, w, nlayers, layer_dims, Wt, bias,
                          mlp_dtype, Wp, bp, out, ws, p, proj, order, plan, nullptr, st,
                          franges);
}

static int dfm_forward_args(const int32_t* idx, int64_t B, int32_t F, const void* E,
                            int64_t features_M, int32_t k, int32_t dtype, const float* w,
                            int32_t nlayers, const int32_t* layer_dims, const void* const* Wt,
                            const float* const* bias, int32_t mlp_dtype, const float* Wp,
                            float* out) {
  int rc = dfm_check(B, F, k, dtype, nlayers, layer_dims, mlp_dtype);
  if (rc) return rc;
  if (features_M < 1) return HHFM_EINVAL;
  if (B == 0) return HHFM_OK;
  if (!idx || !E || !w || !Wt || !bias || !Wp || !out) return HHFM_EINVAL;
  for (int i = 0; i < nlayers; ++i)
    if (!Wt[i] || !bias[i]) return HHFM_EINVAL;
  return 1;   // proceed
}

extern "C" int hhfm_dfm_forward(const int32_t* idx, int64_t B, int32_t F, const void* E,
                                int64_t features_M, int32_t k, int32_t dtype, const float* w,
                                int32_t nlayers, const int32_t* layer_dims,
                                const void* const* Wt, const float* const* bias,
                                int32_t mlp_dtype, const float* Wp, float bp, float* out,
                                void* workspace, size_t ws_bytes, void* stream) {
  const int rc = dfm_forward_args(idx, B, F, E, features_M, k, dtype, w, nlayers, layer_dims, Wt,
                                  bias, mlp_dtype, Wp, out);
  if (rc != 1) return rc;
  // AUTO (rows_total = B) when the workspace holds that plan, else direct
  DfmPlan p = dfm_plan(B, nlayers, layer_dims, mlp_dtype, F, k, features_M, B,
                       wt_aligned(nlayers, Wt) ? HHFM_DFM_PROJ_AUTO : HHFM_DFM_PROJ_OFF);
  if (!p.proj || !workspace || ws_bytes < p.total) p = dfm_plan(B, nlayers, layer_dims, mlp_dtype);
  if (!workspace || ws_bytes < p.total) return HHFM_EWORKSPACE;
  return dfm_forward_planned(idx, B, F, E, features_M, k, dtype, w, nlayers, layer_dims, Wt,
                             bias, mlp_dtype, Wp, bp, out, reinterpret_cast<char*>(workspace), p,
                             HHFM_PLAN_DEFAULT, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int hhfm_dfm_forward_ex(const int32_t* idx, int64_t B, int32_t F, const void* E,
                                   int64_t features_M, int32_t k, int32_t dtype, const float* w,
                                   int32_t nlayers, const int32_t* layer_dims,
                                   const void* const* Wt, const float* const* bias,
                                   int32_t mlp_dtype, const float* Wp, float bp, float* out,
                                   int32_t proj_mode, int32_t plan, void* workspace,
                                   size_t ws_bytes, void* stream) {
  if (!proj_mode_ok(proj_mode) || !plan_ok(plan)) return HHFM_EINVAL;
  const int rc = dfm_forward_args(idx, B, F, E, features_M, k, dtype, w, nlayers, layer_dims, Wt,
                                  bias, mlp_dtype, Wp, out);
  if (rc != 1) return rc;
  if (!wt_aligned(nlayers, Wt)) proj_mode = HHFM_DFM_PROJ_OFF;
  const DfmPlan p = dfm_plan(B, nlayers, layer_dims, mlp_dtype, F, k, features_M, B, proj_mode,
                             1, true, plan);
  if (!workspace || ws_bytes < p.total) return HHFM_EWORKSPACE;
  return dfm_forward_planned(idx, B, F, E, features_M, k, dtype, w, nlayers, layer_dims, Wt,
                             bias, mlp_dtype, Wp, bp, out, reinterpret_cast<char*>(workspace), p,
                             plan, reinterpret_cast<hipStream_t>(stream));
}

// D2: chunk_rows bounds the rows (queries x items) scored per forward pass.
static int64_t dfm_cat_qchunk(int64_t B, int32_t N, int64_t chunk_rows) {
  int64_t qc = chunk_rows / N;
  if (qc < 1) qc = 1;
  if (qc > B) qc = B;
  return qc;
}

static size_t dfm_cat_bytes(const DfmPlan& p, int64_t rows, int F) {
  return p.total + al256((size_t)rows * F * 4) + al256((size_t)rows * 4);
}

extern "C" int hhfm_dfm_catalog_topk_workspace(int64_t B, int32_t F, int32_t item_count,
                                               int32_t nlayers, const int32_t* layer_dims,
                                               int32_t mlp_dtype, int64_t chunk_rows,
                                               size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || F < 1 || item_count < 1 || chunk_rows < 1) return HHFM_EINVAL;
  const int64_t qc = dfm_cat_qchunk(B, item_count, chunk_rows);
  const int64_t rows = qc * item_count;
  *ws_bytes = dfm_cat_bytes(dfm_plan(rows, nlayers, layer_dims, mlp_dtype), rows, F);
  return HHFM_OK;
}

extern "C" int hhfm_dfm_catalog_topk_workspace_ex(int64_t B, int32_t F, int32_t k,
                                                  int64_t features_M, int32_t item_count,
                                                  int32_t nlayers, const int32_t* layer_dims,
                                                  int32_t mlp_dtype, int64_t chunk_rows,
                                                  int32_t proj_mode, size_t* ws_bytes) {
  if (!ws_bytes || B < 0 || F < 1 || k < 1 || features_M < 1 || item_count < 1 ||
      chunk_rows < 1 || nlayers < 1 || !layer_dims)
    return HHFM_EINVAL;
  if (!proj_mode_ok(proj_mode)) return HHFM_EINVAL;
  const int64_t qc = dfm_cat_qchunk(B, item_count, chunk_rows);
  const int64_t rows = qc * item_count;
  // (the item column moves no workspace: any column gives the catalog's size)
  const DfmPlan p = dfm_plan(rows, nlayers, layer_dims, mlp_dtype, F, k, features_M,
                             B * (int64_t)item_count, proj_mode, 1, false);
  *ws_bytes = dfm_cat_bytes(p, rows, F);
  return HHFM_OK;
}

static int dfm_catalog_run(const int32_t* qidx, int64_t B, int32_t F, int32_t item_col,
                           const void* E, int64_t features_M, int32_t k, int32_t dtype,
                           const float* w, int32_t nlayers, const int32_t* layer_dims,
                           const void* const* Wt, const float* const* bias, int32_t mlp_dtype,
                           const float* Wp, float bp, int32_t item_row_begin,
                           int32_t item_count, int32_t global_item_base, int32_t K,
                           int64_t chunk_rows, float* top_score, int32_t* top_idx,
                           void* workspace, size_t ws_bytes, int proj_mode, int32_t plan,
                           void* stream) {
  int rc = dfm_check(B, F, k, dtype, nlayers, layer_dims, mlp_dtype);
  if (rc) return rc;
  if (item_col < 0 || item_col >= F || item_count < 1 || item_row_begin < 0 ||
      (int64_t)item_row_begin + item_count > features_M || chunk_rows < 1)
    return HHFM_EINVAL;
  if (K < 1 || K > item_count) return HHFM_EINVAL;
  if (K > 64) return HHFM_EUNSUPPORTED;
  if (B == 0) return HHFM_OK;
  if (!qidx || !E || !w || !Wt || !bias || !Wp || !top_score || !top_idx) return HHFM_EINVAL;
  const int64_t qc = dfm_cat_qchunk(B, item_count, chunk_rows);
  const int64_t rows = qc * item_count;
  DfmPlan p;
  if (!wt_aligned(nlayers, Wt)) proj_mode = HHFM_DFM_PROJ_OFF;
  if (proj_mode < 0) {   // legacy entry point: AUTO when the workspace holds that plan
    p = dfm_plan(rows, nlayers, layer_dims, mlp_dtype, F, k, features_M,
                 B * (int64_t)item_count, HHFM_DFM_PROJ_AUTO, item_col, false);
    if (!p.proj || !workspace || ws_bytes < dfm_cat_bytes(p, rows, F))
      p = dfm_plan(rows, nlayers, layer_dims, mlp_dtype);
  } else {
    p = dfm_plan(rows, nlayers, layer_dims, mlp_dtype, F, k, features_M,
                 B * (int64_t)item_count, proj_mode, item_col, false, plan);
  }
  if (!workspace || ws_bytes < dfm_cat_bytes(p, rows, F)) return HHFM_EWORKSPACE;
  char* ws = reinterpret_cast<char*>(workspace);
  int32_t* rbuf = reinterpret_cast<int32_t*>(ws + p.total);
  float* sc = reinterpret_cast<float*>(ws + p.total + al256((size_t)rows * F * 4));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const void* proj = nullptr;
  if (p.proj) {   // once per call: every query chunk reuses it
    dfm_project_layer0(E, features_M, k, dtype == HHFM_BF16, mlp_dtype == HHFM_BF16, F,
                       p.proj_from, p.perm, Wt[0], layer_dims[0], nlayers, layer_dims,
                       ws + p.off_proj, st);
    proj = ws + p.off_proj;
  }
  // the FM pair table C depends on E and Wp only: built by the first chunk,
  // reused by the others
  bool pairs_ready = false;
  for (int64_t b0 = 0; b0 < B; b0 += qc) {
    const int64_t nb = (B - b0) < qc ? (B - b0) : qc;
    const int64_t nrows = nb * item_count;
    int64_t blocks = (nrows * F + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(dfm_build_rows, dim3((unsigned)blocks), dim3(256), 0, st, qidx + b0 * F,
                       nb, F, item_col, item_row_begin, item_count, rbuf);
    rc = dfm_forward_impl(rbuf, nrows, F, E, features_M, k, dtype, w, nlayers, layer_dims, Wt,
                          bias, mlp_dtype, Wp, bp, sc, ws, p, proj, nullptr, plan, &pairs_ready,
                          st);
    if (rc) return rc;
    launch_topk_dense(sc, nb, item_count, item_count, K, global_item_base, top_score + b0 * K,
                      top_idx + b0 * K, st, (plan & HHFM_PLAN_ONE_WAVE) != 0);
  }
  return (int)hipGetLastError();
}

extern "C" int hhfm_dfm_catalog_topk(const int32_t* qidx, int64_t B, int32_t F, int32_t item_col,
                                     const void* E, int64_t features_M, int32_t k, int32_t dtype,
                                     const float* w, int32_t nlayers, const int32_t* layer_dims,
                                     const void* const* Wt, const float* const* bias,
                                     int32_t mlp_dtype, const float* Wp, float bp,
                                     int32_t item_row_begin, int32_t item_count,
                                     int32_t global_item_base, int32_t K, int64_t chunk_rows,
                                     float* top_score, int32_t* top_idx, void* workspace,
                                     size_t ws_bytes, void* stream) {
  return dfm_catalog_run(qidx, B, F, item_col, E, features_M, k, dtype, w, nlayers, layer_dims,
                         Wt, bias, mlp_dtype, Wp, bp, item_row_begin, item_count,
                         global_item_base, K, chunk_rows, top_score, top_idx, workspace,
                         ws_bytes, -1, HHFM_PLAN_DEFAULT, stream);
}

extern "C" int hhfm_dfm_catalog_topk_ex(const int32_t* qidx, int64_t B, int32_t F,
                                        int32_t item_col, const void* E, int64_t features_M,
                                        int32_t k, int32_t dtype, const float* w,
                                        int32_t nlayers, const int32_t* layer_dims,
                                        const void* const* Wt, const float* const* bias,
                                        int32_t mlp_dtype, const float* Wp, float bp,
                                        int32_t item_row_begin, int32_t item_count,
                                        int32_t global_item_base, int32_t K, int64_t chunk_rows,
                                        float* top_score, int32_t* top_idx, int32_t proj_mode,
                                        int32_t plan, void* workspace, size_t ws_bytes,
                                        void* stream) {
  if (!proj_mode_ok(proj_mode) || !plan_ok(plan)) return HHFM_EINVAL;
  return dfm_catalog_run(qidx, B, F, item_col, E, features_M, k, dtype, w, nlayers, layer_dims,
                         Wt, bias, mlp_dtype, Wp, bp, item_row_begin, item_count,
                         global_item_base, K, chunk_rows, top_score, top_idx, workspace,
                         ws_bytes, proj_mode, plan, stream);
}

extern "C" int hhfm_topk_dense(const float* scores, int64_t B, int32_t N, int64_t ld, int32_t K,
                               int32_t global_item_base, float* top_score, int32_t* top_idx,
                               void* stream) {
  if (B < 0 || N < 1 || ld < N || K < 1 || K > N) return HHFM_EINVAL;
  if (K > 64) return HHFM_EUNSUPPORTED;
  if (B == 0) return HHFM_OK;
  if (!scores || !top_score || !top_idx) return HHFM_EINVAL;
  launch_topk_dense(scores, B, N, ld, K, global_item_base, top_score, top_idx,
                    reinterpret_cast<hipStream_t>(stream));
  return (int)hipGetLastError();
}

extern "C" int hhfm_topk_dense_ex(const float* scores, int64_t B, int32_t N, int64_t ld,
                                  int32_t K, int32_t global_item_base, float* top_score,
                                  int32_t* top_idx, int32_t plan, void* stream) {
  if (!plan_ok(plan) || B < 0 || N < 1 || ld < N || K < 1 || K > N) return HHFM_EINVAL;
  if (K > 64) return HHFM_EUNSUPPORTED;
  if (B == 0) return HHFM_OK;
  if (!scores || !top_score || !top_idx) return HHFM_EINVAL;
  launch_topk_dense(scores, B, N, ld, K, global_item_base, top_score, top_idx,
                    reinterpret_cast<hipStream_t>(stream), (plan & HHFM_PLAN_ONE_WAVE) != 0);
  return (int)hipGetLastError();
}
