/*
 * hhfm.h — C ABI of the MI355X (gfx950) factorization-machine scoring backend.
 *
 * The reference (data-man-34/HHFM, Newcode/{FM,OurModel7,AFM,DFM}.py) has no native code and no FFI:
 * its hot path is a chain of TensorFlow-1.x graph ops run through
 * `model.sess.run(...)`.  Each entry point below replaces one such op chain
 * (reference file:line cited per function).  The Python host package
 * `hhfm_amd` binds these through the thin pybind11 module `_hhfm`; the ctypes
 * stub a maintainer would add instead is in INTEGRATION.md.
 *
 * Conventions (every function):
 *   - all array pointers are DEVICE memory owned by the caller; the library
 *     allocates nothing and keeps no global mutable state (reentrant);
 *   - `stream` is a hipStream_t (NULL = default stream); every call is
 *     asynchronous on it;
 *   - index arrays are row-major int32 [rows][ncols] (the reference feeds
 *     int32 placeholders, FM.py:89);
 *   - embedding tables are row-major [features_M][k] in `dtype`
 *     (HHFM_F32 or HHFM_BF16; compute is always fp32);
 *   - return 0 on success, a positive hipError_t on a launch error, or a
 *     negative HHFM_E* code for invalid arguments (see hhfm_error_string).
 */
#ifndef HHFM_H_
#define HHFM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HHFM_ABI_VERSION 6
/* leading workspace bytes of hhfm_catalog_topk(_ex) that must start zero */
#define HHFM_CATALOG_WS_ZERO 16384

enum hhfm_dtype { HHFM_F32 = 0, HHFM_BF16 = 1 };

/* Plan flags (ABI v4).  Which kernel runs is chosen from the shapes and these
 * per-call flags only — the library reads no environment variable.  0 is the
 * default plan.  HHFM_PLAN_EXACT_FP32 is the one NUMERICS choice: the dot
 * products run as k-ordered fp32 fmaf chains on fp32 MFMA instead of on bf16
 * MFMA over an exact three-piece bf16 split of every fp32 operand (both within
 * 1e-5 relative of the reference).  Every other bit forces an
 * alternative kernel that other shapes take anyway (same products; bit-
 * identical, or the same terms summed in another order) so the tests can
 * compare both paths on one shape.  Bits an entry point does not use are
 * ignored; bits outside HHFM_PLAN_ALL are rejected with HHFM_EINVAL. */
#define HHFM_PLAN_DEFAULT 0
#define HHFM_PLAN_EXACT_FP32 (1 << 0) /* catalog, AFM, DeepFM fp32 hidden layers */
#define HHFM_PLAN_NO_SEED (1 << 1)    /* catalog streaming path: no threshold-seed pass */
#define HHFM_PLAN_NO_RING (1 << 2)    /* catalog streaming path: catalog_main, not the ring */
#define HHFM_PLAN_RING_ALT (1 << 3)   /* catalog ring: 8 waves per workgroup for bf16
                                         tables, 4 for fp32 (default: the other way) */
#define HHFM_PLAN_GEMM (1 << 4)       /* small catalog and AFM catalog: the score matrix
                                         from the shared LDS-tiled fp32 GEMM */
#define HHFM_PLAN_ROW_FM (1 << 5)     /* DeepFM fp32 MLP: FM part from the table rows,
                                         not from the pair table C = (E*Wp)E^T */
#define HHFM_PLAN_UNSTAGED (1 << 6)   /* DeepFM fp32 MLP: P rows and table rows read
                                         through the caches, not staged in LDS */
#define HHFM_PLAN_UNGROUPED (1 << 7)  /* DeepFM fp32 MLP: rows not grouped by user */
#define HHFM_PLAN_NARROW (1 << 8)     /* DeepFM bf16 ITEM plan: 128-row kernel, not the 256-row one */
#define HHFM_PLAN_PER_FIELD (1 << 9)  /* AFM catalog: pair product split per query field
                                         (afm_cat_fused), not the folded weights */
#define HHFM_PLAN_ONE_WAVE (1 << 10)  /* dense top-K: one wave per query at every size */
/* DeepFM bf16 ITEM plan, 256-row kernel: its workgroup shape (16-row tiles per
 * wave x waves) — 0 the default 2 x 8; these alternates are instantiated for
 * the k = 64, 3 x 150 test shape only (ABI v5), so every shape the kernel
 * template admits runs in the parity tests (bit-identical by construction) */
#define HHFM_PLAN_WIDE_3X4 (1 << 11)
#define HHFM_PLAN_WIDE_2X4 (2 << 11)
#define HHFM_PLAN_WIDE_1X4 (3 << 11)
#define HHFM_PLAN_WIDE_MASK (3 << 11)
#define HHFM_PLAN_STORE (1 << 13)     /* small catalog: the score matrix materialised by the
                                         catalog kernel + dense top-K, not the fused
                                         score-and-select kernel (ABI v5) */
#define HHFM_PLAN_FUSED (1 << 14)     /* small catalog: the fused kernel at any query count
                                         (default: from 1,024 queries) (ABI v5) */
#define HHFM_PLAN_ALL ((1 << 15) - 1)

/* catalog scoring modes */
enum hhfm_catalog_mode {
  HHFM_MODE_FM = 0,   /* FM.topk:  (u+f)·(i+f) + w_i        FM.py:174-185      */
  HHFM_MODE_HHFM = 1  /* OUR.topk: (u+Σctx[+Σtime])·i        OurModel7.py:232-295 */
};

enum hhfm_status {
  HHFM_OK = 0,
  HHFM_EINVAL = -1,       /* bad size / pointer / column range            */
  HHFM_EUNSUPPORTED = -2, /* shape outside what the kernels implement     */
  HHFM_EWORKSPACE = -3    /* workspace smaller than *_workspace() reports */
};

const char* hhfm_error_string(int code);
int hhfm_abi_version(void);

/* ------------------------------------------------------------------------
 * M1 — FM per-row score (replaces the `FM.out` graph, FM.py:99-120)
 *   out[b] = Σ_k ½[(Σ_f E[x_bf,k])² − Σ_f E[x_bf,k]²] + Σ_f w[x_bf] + w0
 * idx: int32 [B][F]; w may be NULL (then Σw = 0, the DeepFM-interaction use).
 * out: float [B].
 * ---------------------------------------------------------------------- */
int hhfm_fm_score_rows(const int32_t* idx, int64_t B, int32_t F,
                       const void* E, int64_t features_M, int32_t k,
                       int32_t dtype, const float* w, float w0, float* out,
                       void* stream);

/* Same, with tuning flags and an optional id status word:
 *   HHFM_FLAG_STREAM_TABLE — read embedding rows / ids and write `out` with
 *   non-temporal accesses (measured 10 % slower at configs[1]).
 *   Any other bit is rejected with HHFM_EINVAL.
 *   Without the flag, a table of 1 GiB or more (far beyond the caches) loads
 *   the first two columns' rows — the user and item, read once per launch —
 *   non-temporal and everything else with the default policy (the same
 *   arithmetic and bits; 2.4 % faster at configs[1]).
 * status: NULL, or a device int32 the kernel ORs HHFM_STATUS_BAD_ID into when
 *   it meets an id outside [0, features_M) (such ids are read as row 0 so the
 *   kernel cannot fault).  hhfm_status_read() turns it into HHFM_EINVAL —
 *   the InvalidArgumentError tf.nn.embedding_lookup raises (FM.py:99). */
#define HHFM_FLAG_STREAM_TABLE 1
#define HHFM_FM_ROWS_DEFAULT_FLAGS 0
#define HHFM_STATUS_BAD_ID 1
int hhfm_fm_score_rows_ex(const int32_t* idx, int64_t B, int32_t F,
                          const void* E, int64_t features_M, int32_t k,
                          int32_t dtype, const float* w, float w0, float* out,
                          int32_t flags, int32_t* status, void* stream);

/* ------------------------------------------------------------------------
 * H1 — HHFM per-row score (replaces `OUR.PositiveFeadback`,
 * OurModel7.py:105-171 with sum pooling, :14-19)
 *   h_b = E[x_b,user_col] + Σ_{c∈[ctx_begin,ctx_end)} E[x_bc]
 *                         (+ Σ_{t∈[time_begin,time_end)} E[x_bt])
 *   out[b] = Σ_k h_b,k · E[x_b,item_col],k
 * An empty range (begin == end) disables that term. idx: int32 [B][ncols].
 * ---------------------------------------------------------------------- */
int hhfm_hybrid_score_rows(const int32_t* idx, int64_t B, int32_t ncols,
                           int32_t user_col, int32_t item_col,
                           int32_t ctx_begin, int32_t ctx_end,
                           int32_t time_begin, int32_t time_end,
                           const void* E, int64_t features_M, int32_t k,
                           int32_t dtype, float* out, void* stream);
/* Same, with the optional id status word of hhfm_fm_score_rows_ex. */
int hhfm_hybrid_score_rows_ex(const int32_t* idx, int64_t B, int32_t ncols,
                              int32_t user_col, int32_t item_col,
                              int32_t ctx_begin, int32_t ctx_end,
                              int32_t time_begin, int32_t time_end,
                              const void* E, int64_t features_M, int32_t k,
                              int32_t dtype, float* out, int32_t* status,
                              void* stream);

/* ------------------------------------------------------------------------
 * M2/H2 — full-catalog score + fused top-K (replaces FM.topk, FM.py:172-198,
 * and OUR.topk, OurModel7.py:229-307: broadcast multiply [B,N,k] +
 * reduce_sum + tf.nn.top_k), without materialising the [B,N] score matrix.
 *
 *   query columns (qidx int32 [B][ncols]):
 *     HHFM_MODE_HHFM: h = E[user] + Σ ctx cols (+ Σ time cols); score = h·E[item]
 *     HHFM_MODE_FM:   f = Σ ctx cols, q = E[user]+f;
 *                     score = q·(E[item]+f) + w[item]   (w may be NULL)
 *   catalog: items are rows [item_row_begin, item_row_begin+item_count) of E.
 *   output:  top_score/top_idx [B][K], sorted by (score desc, index asc) —
 *            tf.nn.top_k order; top_idx = global_item_base + offset in range.
 *   K must be in [1, 64] and <= item_count.
 *   arithmetic: the h·item products run on bf16 MFMA with every fp32
 *            operand split exactly into three bf16 pieces (products of
 *            order >= 2^-16 kept, fp32 accumulation: ~1e-7 relative to a
 *            k-ordered fp32 chain); plan HHFM_PLAN_EXACT_FP32 (the _ex form)
 *            selects the fp32-MFMA kernels (the k-ordered fmaf chain).
 * Workspace: query `hhfm_catalog_topk_workspace` with the same sizes (it
 * covers every plan).  Its first HHFM_CATALOG_WS_ZERO bytes must be zero
 * before the first call (the small-catalog kernel's per-call arrival
 * counters: every call leaves them zero again); a buffer used by other
 * entry points in between must be re-zeroed there (ABI v6).
 * ---------------------------------------------------------------------- */
int hhfm_catalog_topk_workspace(int64_t B, int32_t item_count, int32_t k,
                                int32_t K, size_t* ws_bytes);

int hhfm_catalog_topk(const int32_t* qidx, int64_t B, int32_t ncols,
                      int32_t mode, int32_t user_col, int32_t ctx_begin,
                      int32_t ctx_end, int32_t time_begin, int32_t time_end,
                      const void* E, int64_t features_M, int32_t k,
                      int32_t dtype, const float* w, int32_t item_row_begin,
                      int32_t item_count, int32_t global_item_base, int32_t K,
                      float* top_score, int32_t* top_idx, void* workspace,
                      size_t ws_bytes, void* stream);
/* Same, with plan flags (HHFM_PLAN_EXACT_FP32, _NO_SEED, _NO_RING,
 * _RING_ALT, _GEMM, _ONE_WAVE) and the optional id status word (query ids
 * are checked on the stream before scoring; the item range on the host). */
int hhfm_catalog_topk_ex(const int32_t* qidx, int64_t B, int32_t ncols,
                         int32_t mode, int32_t user_col, int32_t ctx_begin,
                         int32_t ctx_end, int32_t time_begin, int32_t time_end,
                         const void* E, int64_t features_M, int32_t k,
                         int32_t dtype, const float* w, int32_t item_row_begin,
                         int32_t item_count, int32_t global_item_base, int32_t K,
                         float* top_score, int32_t* top_idx, void* workspace,
                         size_t ws_bytes, int32_t plan, int32_t* status, void* stream);

/* ------------------------------------------------------------------------
 * Top-K merge of R sorted partial lists per query (the item-sharded
 * multi-GPU path: RCCL all-gather output, rank-major).  Replaces the single
 * tf.nn.top_k over the full catalog (FM.py:185, OurModel7.py:295).
 *   in_score/in_idx: [R][B][K]; out_*: [B][K]; same (score desc, idx asc) order.
 * hhfm_topk_merge_host is the same merge on host memory (no GPU needed).
 * ---------------------------------------------------------------------- */
int hhfm_topk_merge(const float* in_score, const int32_t* in_idx, int32_t R,
                    int64_t B, int32_t K, float* out_score, int32_t* out_idx,
                    void* stream);
int hhfm_topk_merge_host(const float* in_score, const int32_t* in_idx,
                         int32_t R, int64_t B, int32_t K, float* out_score,
                         int32_t* out_idx);

/* ------------------------------------------------------------------------
 * D1 — DeepFM per-row score (replaces `DeepFM.out`, DFM.py:104-137)
 *   y1 = w[x] (F), y2 = ½((Σe)² − Σe²) (k), h_0 = concat_f E[x_f] (F·k),
 *   h_{i+1} = relu(h_i · W_i + b_i) for every layer (ReLU after the last one
 *   too, DFM.py:128), out = [y1, y2, h_L] · Wp + bp.
 * Wt[i] are DEVICE pointers to the layer weights TRANSPOSED, [dims[i]][K_i]
 * with K_0 = F·k and K_i = dims[i-1] rounded up to a multiple of 8 (pad
 * columns zero), in mlp_dtype; bias[i] device float [dims[i]];
 * the Wt/bias/layer_dims arrays themselves are host arrays.  mlp_dtype
 * HHFM_F32 runs exact-fp32 MFMA (v_mfma_f32_16x16x4_f32), HHFM_BF16 runs
 * bf16 MFMA with fp32 accumulation (activations rounded to bf16).
 * Wp: device float [F + k + dims[L-1]].  k must be a multiple of 4 (f32) /
 * 8 (bf16); layer widths are arbitrary.
 * ---------------------------------------------------------------------- */
int hhfm_dfm_forward_workspace(int64_t B, int32_t nlayers, const int32_t* layer_dims,
                               int32_t mlp_dtype, size_t* ws_bytes);

/* Projected layer 0 (ABI v3).  Layer 0 is linear before its ReLU, so
 * h_0 = Σ_f P_f[x_f] with P_f[id] = W0[:, f·k:(f+1)·k] · E[id]: the forward
 * computes P for every table row of the projected fields once per call (MFMA
 * GEMMs, the direct kernel's operand rounding, fp32 results) and the fused
 * kernel gathers it instead of streaming those fields' layer-0 weights — a
 * saving when rows >= 2·features_M (DFM.py:125-128 computed by the same
 * products, summed per field first).
 * The *_ex entry points take proj_mode explicitly; hhfm_dfm_forward /
 * hhfm_dfm_catalog_topk follow HHFM_DFM_PROJ_AUTO when ws_bytes covers that
 * plan (the *_workspace_ex size with HHFM_DFM_PROJ_AUTO) and run direct
 * otherwise.  The plan (direct, projected, which fields) changes the
 * summation order of layer 0, so scores may differ between plans within the
 * tested tolerances (fp32 MLP 2e-5, bf16 MLP 5e-3 of the output magnitude).
 * Projection needs the fused envelope (k % 16 == 0, k <= 512, F <= 16,
 * <= 4 layers of <= 416 units) and 16-B aligned Wt[i]; otherwise every mode
 * runs direct.
 * P needs (F - first projected field)·features_M·32·⌈max width/32⌉ floats
 * (at most 1 GiB planned). */
enum hhfm_dfm_proj {
  HHFM_DFM_PROJ_OFF = 0,  /* plan the direct path only                       */
  HHFM_DFM_PROJ_ON = 1,   /* project every field                             */
  HHFM_DFM_PROJ_AUTO = 2, /* below rows (B, or B·item_count) = 2·M: OFF;
                             fp32 MLP: ON; bf16 MLP: ITEM in the catalog,
                             ITEM in the forward from rows >= 64·M, CTX
                             below that                                      */
  HHFM_DFM_PROJ_CTX = 3,  /* bf16 MLP, F >= 3: project the context fields
                             2..F-1 (LoadData's layout: user, item,
                             contexts), fields 0 and 1 stay on MFMA; other
                             shapes run direct                               */
  HHFM_DFM_PROJ_ITEM = 4  /* bf16 MLP, F >= 2: project every field but the
                             item (field 1 of a forward row, item_col of a
                             catalog row), which stays on MFMA; the forward
                             processes its rows grouped by field 0 (a device
                             radix sort; scores land at the caller's row
                             positions); other shapes run direct             */
};
int hhfm_dfm_forward_workspace_ex(int64_t B, int32_t F, int32_t k, int64_t features_M,
                                  int32_t nlayers, const int32_t* layer_dims,
                                  int32_t mlp_dtype, int32_t proj_mode, size_t* ws_bytes);
int hhfm_dfm_forward(const int32_t* idx, int64_t B, int32_t F, const void* E,
                     int64_t features_M, int32_t k, int32_t dtype, const float* w,
                     int32_t nlayers, const int32_t* layer_dims, const void* const* Wt,
                     const float* const* bias, int32_t mlp_dtype, const float* Wp,
                     float bp, float* out, void* workspace, size_t ws_bytes,
                     void* stream);
/* Same, with the projection mode and the plan flags explicit (fp32 MLP:
 * HHFM_PLAN_EXACT_FP32 keeps the hidden layers on exact-fp32 MFMA, _ROW_FM,
 * _UNSTAGED, _UNGROUPED; bf16 MLP: _NARROW; the catalog also _ONE_WAVE);
 * ws_bytes must cover hhfm_dfm_forward_workspace_ex(..., proj_mode). */
int hhfm_dfm_forward_ex(const int32_t* idx, int64_t B, int32_t F, const void* E,
                        int64_t features_M, int32_t k, int32_t dtype, const float* w,
                        int32_t nlayers, const int32_t* layer_dims, const void* const* Wt,
                        const float* const* bias, int32_t mlp_dtype, const float* Wp,
                        float bp, float* out, int32_t proj_mode, int32_t plan,
                        void* workspace, size_t ws_bytes, void* stream);

/* D2 — DeepFM.topk (DFM.py:219-231): every query row is tiled over the
 * catalog with column item_col replaced by each item id, scored by D1 and
 * top-K selected; at most chunk_rows (query x item) rows per pass. */
int hhfm_dfm_catalog_topk_workspace(int64_t B, int32_t F, int32_t item_count,
                                    int32_t nlayers, const int32_t* layer_dims,
                                    int32_t mlp_dtype, int64_t chunk_rows,
                                    size_t* ws_bytes);
int hhfm_dfm_catalog_topk_workspace_ex(int64_t B, int32_t F, int32_t k,
                                       int64_t features_M, int32_t item_count,
                                       int32_t nlayers, const int32_t* layer_dims,
                                       int32_t mlp_dtype, int64_t chunk_rows,
                                       int32_t proj_mode, size_t* ws_bytes);
int hhfm_dfm_catalog_topk(const int32_t* qidx, int64_t B, int32_t F, int32_t item_col,
                          const void* E, int64_t features_M, int32_t k, int32_t dtype,
                          const float* w, int32_t nlayers, const int32_t* layer_dims,
                          const void* const* Wt, const float* const* bias,
                          int32_t mlp_dtype, const float* Wp, float bp,
                          int32_t item_row_begin, int32_t item_count,
                          int32_t global_item_base, int32_t K, int64_t chunk_rows,
                          float* top_score, int32_t* top_idx, void* workspace,
                          size_t ws_bytes, void* stream);
/* Same, with the projection mode and plan flags explicit (see
 * hhfm_dfm_forward_ex). */
int hhfm_dfm_catalog_topk_ex(const int32_t* qidx, int64_t B, int32_t F, int32_t item_col,
                             const void* E, int64_t features_M, int32_t k, int32_t dtype,
                             const float* w, int32_t nlayers, const int32_t* layer_dims,
                             const void* const* Wt, const float* const* bias,
                             int32_t mlp_dtype, const float* Wp, float bp,
                             int32_t item_row_begin, int32_t item_count,
                             int32_t global_item_base, int32_t K, int64_t chunk_rows,
                             float* top_score, int32_t* top_idx, int32_t proj_mode,
                             int32_t plan, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * A1 — AFM per-row score (replaces `AFM.out`, AFM.py:103-142), attention on,
 * keep = [1,1]: pairs i<j of the F fields, logit = Σ_a p_a·relu(((e_i⊙e_j)·W)_a
 * + b_a), att = softmax over pairs, out = (Σ att·(e_i⊙e_j))·P + Σ w + w0.
 * Wt: device float [A][k] = attention_W TRANSPOSED; att_b [A], att_p [A],
 * P [k] (the prediction vector).  F <= 16, k % 4 == 0.
 * ---------------------------------------------------------------------- */
int hhfm_afm_forward_workspace(int64_t B, int32_t F, int32_t A, size_t* ws_bytes);
int hhfm_afm_forward(const int32_t* idx, int64_t B, int32_t F, const void* E,
                     int64_t features_M, int32_t k, int32_t dtype, const float* w, float w0,
                     const float* Wt, const float* att_b, const float* att_p, int32_t A,
                     const float* P, float* out, void* workspace, size_t ws_bytes,
                     void* stream);
/* Same, with plan flags: HHFM_PLAN_EXACT_FP32 runs the attention contraction
 * on exact-fp32 MFMA instead of split-bf16 (k % 16 == 0 shapes). */
int hhfm_afm_forward_ex(const int32_t* idx, int64_t B, int32_t F, const void* E,
                        int64_t features_M, int32_t k, int32_t dtype, const float* w,
                        float w0, const float* Wt, const float* att_b, const float* att_p,
                        int32_t A, const float* P, float* out, int32_t plan,
                        void* workspace, size_t ws_bytes, void* stream);

/* A2 — AFM.topk (AFM.py:209-246): uf = [E[col 0], E[cols 2..F-1]], exp-weighted
 * pair attention over uf pairs and uf x item pairs (raw exp, as the
 * reference), score = (Σ_c P_c·score1_c) / weight + w_item, then top-K.
 * At most max_cols = (queries per pass)·(F-1)·A GEMM columns per pass.
 * k <= 256, k % 4 == 0, A % 16 == 0 (or inside the fused envelope), F <= 16. */
int hhfm_afm_catalog_topk_workspace(int64_t B, int32_t F, int32_t k, int32_t A,
                                    int32_t item_count, int64_t max_cols,
                                    size_t* ws_bytes);
int hhfm_afm_catalog_topk(const int32_t* qidx, int64_t B, int32_t F, const void* E,
                          int64_t features_M, int32_t k, int32_t dtype, const float* w,
                          const float* Wt, const float* att_b, const float* att_p,
                          int32_t A, const float* P, int32_t item_row_begin,
                          int32_t item_count, int32_t global_item_base, int32_t K,
                          int64_t max_cols, float* top_score, int32_t* top_idx,
                          void* workspace, size_t ws_bytes, void* stream);
/* Same, with plan flags: HHFM_PLAN_EXACT_FP32, _PER_FIELD, _GEMM (the
 * workspace for _GEMM is hhfm_afm_catalog_topk_workspace_ex's). */
int hhfm_afm_catalog_topk_workspace_ex(int64_t B, int32_t F, int32_t k, int32_t A,
                                       int32_t item_count, int64_t max_cols, int32_t plan,
                                       size_t* ws_bytes);
int hhfm_afm_catalog_topk_ex(const int32_t* qidx, int64_t B, int32_t F, const void* E,
                             int64_t features_M, int32_t k, int32_t dtype, const float* w,
                             const float* Wt, const float* att_b, const float* att_p,
                             int32_t A, const float* P, int32_t item_row_begin,
                             int32_t item_count, int32_t global_item_base, int32_t K,
                             int64_t max_cols, float* top_score, int32_t* top_idx,
                             int32_t plan, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * H6 — one training step (`partial_fit`, sess.run((loss, optimizer))).
 *   FM   (FM.py:123-136):        loss = Σ (y − out)²/2 + λ·Σ E²/2
 *   HHFM (OurModel7.py:172-193): loss = −Σ log σ(pos − max_j neg_j) + λ·Σ E²/2
 * optimizer (TF-1.x semantics, FM.py:129-136; `acc` slots per variable):
 *   0 = AdagradOptimizer  accum += g², var -= lr·g·rsqrt(accum); n floats
 *       initialised to 0.1 (TF's initial_accumulator_value);
 *   1 = GradientDescentOptimizer (no slots);
 *   2 = MomentumOptimizer(momentum = 0.95)  accum = accum·0.95 + g,
 *       var -= accum·lr; n floats initialised to 0;
 *   3 = AdamOptimizer(β1 0.9, β2 0.999, ε 1e-8)  2n floats (m, then v)
 *       initialised to 0; β1^t, β2^t and a started flag live in the
 *       workspace (zero-filled once = step 1; a power that underflows to 0
 *       stays 0, as TF's does).
 * Variables whose TF gradient is an IndexedSlices (an embedding_lookup with
 * no dense l2 term on the same variable: w of FM; the table of FM / HHFM at
 * λ = 0, of DeepFM and of AFM; w of DeepFM and AFM) follow TF's sparse
 * rules: Momentum updates only the rows the batch touched, Adam decays m
 * and v of every row (AdamOptimizer._apply_sparse_shared).
 * E, w are fp32 and updated in place; *loss (device float) receives the loss
 * of the pre-update parameters.  The workspace (hhfm_train_workspace bytes)
 * must be zero-filled once; the step leaves it zeroed except Adam's β powers.  HHFM: X [B][ncols]
 * full rows [user, item, ctx..., time...], Neg [B][NG] negative item ids,
 * NG <= 16.
 * ---------------------------------------------------------------------- */
size_t hhfm_train_workspace(int64_t features_M, int32_t k);
int hhfm_fm_train_step(const int32_t* idx, const float* y, int64_t B, int32_t F, float* E,
                       float* w, float* w0, int64_t features_M, int32_t k, float lr,
                       float lambda_l2, int32_t optimizer, float* accE, float* accw,
                       float* accw0, void* workspace, size_t ws_bytes, float* loss,
                       void* stream);
int hhfm_hhfm_train_step(const int32_t* X, const int32_t* Neg, int64_t B, int32_t ncols,
                         int32_t ctx_begin, int32_t ctx_end, int32_t time_begin,
                         int32_t time_end, int32_t NG, float* E, int64_t features_M,
                         int32_t k, float lr, float lambda_l2, int32_t optimizer, float* accE,
                         void* workspace, size_t ws_bytes, float* loss, void* stream);

/* DeepFM (DFM.py:139-155, 214-217; use_fm = use_deep = True, loss "mse"):
 *   loss = Σ (y − out)²/2 + λ·(‖Wp‖² + Σ_l ‖W_l‖²)/2
 * one step of the optimizer (codes as above) on every variable, in place.
 * W[l] is layer l row-major [d_{l-1}][d_l] (d_{-1} = F·k), bias[l] [d_l], Wp
 * the concat projection [F + k + d_{L-1}], bp a device float.  acc (every
 * optimizer but 1): 2L+4 device slot arrays in the order E, w, W_0..W_{L-1},
 * b_0..b_{L-1}, Wp, bp, sized and initialised as above.
 * The workspace (hhfm_dfm_train_workspace bytes for batches of at most B rows)
 * must be zero-filled once; the step keeps its gradient regions zeroed.  Its
 * persistent part (gradients, Adam's β powers) leads at offsets independent
 * of B: a workspace grown for a larger batch keeps the state when that
 * prefix (hhfm_dfm_train_state_bytes) is copied into the new zero-filled one.
 * Requires k % 4 == 0, L <= 4, F + k + d_{L-1} <= 1024. */
int hhfm_dfm_train_workspace(int64_t B, int32_t F, int32_t k, int64_t features_M,
                             int32_t nlayers, const int32_t* layer_dims, size_t* ws_bytes);
/* The size of that persistent prefix (ABI v5): copy exactly these bytes of an
 * old workspace into a new zero-filled one; everything after it is per-batch
 * scratch. */
int hhfm_dfm_train_state_bytes(int32_t F, int32_t k, int64_t features_M, int32_t nlayers,
                               const int32_t* layer_dims, size_t* state_bytes);
int hhfm_dfm_train_step(const int32_t* idx, const float* y, int64_t B, int32_t F, float* E,
                        float* w, int64_t features_M, int32_t k, int32_t nlayers,
                        const int32_t* layer_dims, float* const* W, float* const* bias,
                        float* Wp, float* bp, float lr, float lambda_l2, int32_t optimizer,
                        float* const* acc, void* workspace, size_t ws_bytes, float* loss,
                        void* stream);

/* AFM (AFM.py:103-156, 205-207; attention = 1, keep = [1, 1]):
 *   loss = Σ (y − out)²/2 + λ·‖attention_W‖²/2
 * one step of the optimizer (codes as above) on every variable, in place:
 * E [M][k], w [M], w0 (device float), W = attention_W [k][A] row-major,
 * b = attention_b [A], pvec = attention_p [A], P = prediction [k].  acc
 * (every optimizer but 1): 7 device slot arrays in the order E, w, w0, W, b,
 * pvec, P, sized and initialised as above.  The workspace
 * (hhfm_afm_train_workspace bytes for batches of at most B rows) must be
 * zero-filled once; the step keeps its gradient regions zeroed; grown as for
 * DeepFM (the hhfm_afm_train_state_bytes prefix copied into the new one).
 * Requires 2 <= F <= 16, k and A multiples of 4 and <= 256.  Replaces
 * sess.run((loss, optimizer)) of AFM.partial_fit (AFM.py:205-207). */
int hhfm_afm_train_workspace(int64_t B, int32_t F, int32_t k, int32_t A,
                             int64_t features_M, size_t* ws_bytes);
int hhfm_afm_train_state_bytes(int32_t F, int32_t k, int32_t A, int64_t features_M,
                               size_t* state_bytes);
int hhfm_afm_train_step(const int32_t* idx, const float* y, int64_t B, int32_t F, float* E,
                        float* w, float* w0, int64_t features_M, int32_t k, int32_t A,
                        float* W, float* b, float* pvec, float* P, float lr,
                        float lambda_att, int32_t optimizer, float* const* acc,
                        void* workspace, size_t ws_bytes, float* loss, void* stream);

/* tf.nn.top_k(scores, K) over a materialised score matrix [B][ld] (first N
 * columns), K <= 64; ids reported as global_item_base + column. */
int hhfm_topk_dense(const float* scores, int64_t B, int32_t N, int64_t ld, int32_t K,
                    int32_t global_item_base, float* top_score, int32_t* top_idx,
                    void* stream);
/* Same, with plan flags: HHFM_PLAN_ONE_WAVE keeps one wave per query where
 * the default splits a query over 4 waves (B <= 1,024, N >= 1,024). */
int hhfm_topk_dense_ex(const float* scores, int64_t B, int32_t N, int64_t ld, int32_t K,
                       int32_t global_item_base, float* top_score, int32_t* top_idx,
                       int32_t plan, void* stream);

/* ------------------------------------------------------------------------
 * H5 / H3 — harness membership test and metric walk
 *
 * positive_feedback (NewLoadData.py:49-56: key = every column but the item
 * -> set of items) as two sorted device arrays: keys [nkeys][key_cols]
 * int32, distinct, lexicographically sorted (key_cols = ncols - 1); codes
 * [ncodes] int64 = (rank of the key in `keys`) << 32 | item, sorted.
 *
 * hhfm_pf_contains: out[b][j] = 1 iff cand[b][j] is in positive_feedback
 * of row b's key — the rejection test of Train.sample_negative
 * (FM.py:291-293).  cand == NULL (num = 1): the row's own item (column
 * item_col) — evaluate_TopK's `item in positive_feedback[key]`
 * (FM.py:343-355).  rows: int32 [B][ncols]; out: uint8 [B][num].
 *
 * hhfm_topk_walk: evaluate_TopK's walk over P predictions (FM.py:344-357)
 * per row: outcome = n >= 0 (target at walk position n < TopK), -1 (walk
 * passed TopK-1: the reference appends 0, 0, 0), -2 (predictions
 * exhausted: it appends nothing).  pred: int32 [B][P] global item ids,
 * target int32 [B], positive uint8 [B] (from hhfm_pf_contains).
 * ---------------------------------------------------------------------- */
int hhfm_pf_contains(const int32_t* keys, int64_t nkeys, int32_t key_cols,
                     const int64_t* codes, int64_t ncodes, const int32_t* rows,
                     int64_t B, int32_t ncols, int32_t item_col,
                     const int32_t* cand, int32_t num, uint8_t* out, void* stream);
int hhfm_topk_walk(const int32_t* pred, int64_t B, int32_t P, const int32_t* target,
                   const uint8_t* positive, int32_t TopK, int32_t* outcome, void* stream);

/* hhfm_sample_negative (ABI v5) — all of Train.sample_negative
 * (FM.py:284-294) on the device, on numpy's own random stream:
 *   samples = np.random.randint(lo, hi, size=(B, num)), then in row-major
 *   order each sample that is in positive_feedback[key of its row] re-drawn
 *   with np.random.randint(lo, hi) until it is not.
 * mt_state: device uint32 [625] = the legacy RandomState's MT19937 key[624]
 * followed by pos (np.random.get_state()[1:3]); on return it holds the state
 * after the last word the call read, for np.random.set_state — the samples
 * and the state equal the reference's bit for bit (numpy's masked bounded
 * draw: 32-bit outputs AND the smallest covering mask, rejected while > hi -
 * 1 - lo).  rows int32 [B][ncols] (key = every column but item_col), keys /
 * codes as for hhfm_pf_contains; samples: device int64 [B][num].  Requires
 * 0 <= lo < hi <= 2^31, B·num < 2^30.  A row whose positives cover all of
 * [lo, hi) (where the reference loops forever) returns HHFM_EINVAL.  Unlike
 * the other entry points this call synchronises `stream` (a few small
 * device-to-host reads steer the generation rounds); the workspace is
 * hhfm_sample_negative_workspace(B, num) bytes, no initialisation needed.
 * Replaces FM.py:284-294 (and OurModel7.py, AFM.py, DFM.py's copies). */
int hhfm_sample_negative_workspace(int64_t B, int32_t num, size_t* ws_bytes);
/* The same, sized for the faster re-draw test: per-key bitmaps of the
 * positives over [lo, hi) (nkeys x ceil((hi - lo) / 32) words, used when at
 * most 256 MB); hhfm_sample_negative takes the bitmap path whenever ws_bytes
 * covers it.  Results are identical either way. */
int hhfm_sample_negative_workspace_ex(int64_t B, int32_t num, int64_t lo, int64_t hi,
                                      int64_t nkeys, size_t* ws_bytes);
int hhfm_sample_negative(uint32_t* mt_state, int64_t lo, int64_t hi, const int32_t* rows,
                         int64_t B, int32_t ncols, int32_t item_col, int32_t num,
                         const int32_t* keys, int64_t nkeys, const int64_t* codes,
                         int64_t ncodes, int64_t* samples, void* workspace, size_t ws_bytes,
                         void* stream);

/* ------------------------------------------------------------------------
 * L1 — the libfm loader's per-cell work (NewLoadData.py:16-58), HOST code:
 * every pointer below is host memory, nothing touches the GPU.
 *
 * hhfm_libfm_encode: parse `len` bytes of "label tok ... tok" lines
 * (ncols fields separated by single spaces, blank lines skipped, at most
 * max_rows rows) into labels [rows] (double) and ids [rows][ncols-1]
 * (int64): the column-major first-occurrence token -> id map over columns
 * 1.. (NewLoadData.py:29-34; identical tokens share an id across columns).
 * distinct[ncols-1] = distinct tokens per column (n_user, n_item, ...:
 * NewLoadData.py:22-23); *features_M = distinct tokens overall.
 *
 * hhfm_loader_split: over the shuffled rows data [rows][ncols] (label,
 * user, item, ctx...), is_test[r] = 1 iff row r's key (every column but 0
 * and item_col) is unseen and fewer than test_size rows went to Test so
 * far (NewLoadData.py:46-58).
 * ---------------------------------------------------------------------- */
int hhfm_libfm_encode(const char* buf, int64_t len, int32_t ncols, int64_t max_rows,
                      double* labels, int64_t* ids, int64_t* rows_out, int64_t* features_M,
                      int64_t* distinct);
int hhfm_loader_split(const int64_t* data, int64_t rows, int32_t ncols, int32_t item_col,
                      int64_t test_size, uint8_t* is_test);

/* ------------------------------------------------------------------------
 * Id validation (tf.nn.embedding_lookup raises InvalidArgumentError on an id
 * outside [0, features_M): FM.py:99, OurModel7.py:105, AFM.py:104, DFM.py:105).
 * Every kernel reads such an id as row 0 so it can never fault; callers that
 * want TF's error pass a device status word:
 *   hhfm_check_ids   — async: ORs HHFM_STATUS_BAD_ID into *status (device
 *                      int32) if any of idx[0..n) is outside [0, features_M);
 *                      covers every entry point without an _ex status form
 *                      (AFM, DeepFM, training, harness).
 *   hhfm_status_read — synchronises `stream`, reads and clears *status;
 *                      returns HHFM_EINVAL if a bad id was seen, else HHFM_OK.
 * ---------------------------------------------------------------------- */
int hhfm_check_ids(const int32_t* idx, int64_t n, int64_t features_M, int32_t* status,
                   void* stream);
int hhfm_status_read(int32_t* status, void* stream);

/* ------------------------------------------------------------------------
 * Measurement probe (not a scoring entry point): streams `bytes` (a multiple
 * of 16, 16-B aligned) of device memory once with 16-B loads, so bench.py
 * can report K1's HBM fraction against the box's measured read ceiling as
 * well as the 8 TB/s spec.  mode 0: grid-stride; 1: one contiguous chunk per
 * workgroup, 8 loads in flight per lane; 2: as 1 with non-temporal loads.
 * `sink`: one device float (written only on an impossible data value, so the
 * loads cannot be elided).
 * ---------------------------------------------------------------------- */
int hhfm_probe_stream_read(const void* buf, int64_t bytes, int32_t mode, float* sink,
                           void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HHFM_H_ */
