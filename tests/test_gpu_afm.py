"""AFM (K4) on the GPU vs the reference graph (golden afm.npz) and vs the
oracle at Frappe shape.  fp32 numerics (exact-fp32 MFMA, or split-bf16 MFMA
for the fused kernels when k % 16 == 0 — PLAN_EXACT_FP32 forces the former).
Rows: 1e-5 relative of the float64 value of AFM.py:103-142, elementwise on
every row whose condition number Σ|terms| / |out| is at most 100, normwise
on the rest (tests/helpers.kappa_check; κ counts in the parity report).
Catalog: top-K positions exact except fp32 ties within 1e-5 of the query's
score scale."""
import os

import numpy as np
import pytest
import torch

from oracle import fm_oracle as orc
from oracle import parity
from tests.helpers import kappa_check

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _afm(nu, ni, M, k, A=None, F=5, table_dtype=torch.float32):
    from hhfm_amd.AFM import AFM
    return AFM(nu, ni, M, 1, [A or k, k], None, 0.1, 100.0, [1, 1], "AdagradOptimizer", 0.999, F,
               table_dtype=table_dtype)


def test_afm_vs_reference_graph():
    d = dict(np.load(os.path.join(G, "afm.npz")))
    nu, ni = int(d["n_user"]), int(d["n_item"])
    M, k = d["E"].shape
    m = _afm(nu, ni, M, k)
    m.set_weights(feature_embeddings=d["E"], feature_bias=d["w"][:, None], bias=d["w0"],
                  attention_W=d["attention_W"], attention_b=d["attention_b"],
                  attention_p=d["attention_p"], prediction=d["prediction"])
    out = m.score_rows(d["X"])[:, 0]
    ex, mag = parity.afm_rows_exact(d["X"], d["E"], d["w"], d["w0"], d["attention_W"],
                                    d["attention_b"], d["attention_p"], d["prediction"])
    kappa_check("afm_rows_kappa", out, d["out"], ex, mag)
    out2 = m.sess.run(m.out, feed_dict={m.train_features: d["X"], m.train_labels: None,
                                         m.dropout_keep: [1.0, 1.0], m.train_phase: False})
    assert np.array_equal(out2[:, 0], out)
    pred = m.topk(d["A"], 20)
    # bit-exact against the reference graph's golden top-20
    assert np.array_equal(pred, d["topk_idx"]), int((pred != d["topk_idx"]).sum())


@pytest.mark.parametrize("exact", ["0", "1"])
@pytest.mark.parametrize("k,A", [(64, 64), (32, 16), (128, 128), (64, 32), (24, 32), (48, 48)])
def test_afm_frappe_shape(k, A, exact):
    from hhfm_amd import ops
    plan = ops.PLAN_EXACT_FP32 if exact == "1" else 0
    rng = np.random.default_rng(k + A)
    nu, ni = 957, 4082
    M = nu + ni + 12
    m = _afm(nu, ni, M, k, A)
    W = m.get_weights()
    W["feature_bias"] = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    m.set_weights(feature_bias=W["feature_bias"])
    X = np.stack([rng.integers(0, nu, 700), rng.integers(nu, nu + ni, 700),
                  rng.integers(nu + ni, nu + ni + 7, 700), rng.integers(nu + ni + 7, nu + ni + 9, 700),
                  rng.integers(nu + ni + 9, M, 700)], 1).astype(np.int32)
    args = (W["attention_W"], W["attention_b"], W["attention_p"], W["prediction"])
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    ref = orc.afm_out(X, E, w, 0.0, *args)[:, 0]
    Wt, b, p, P = m._att()
    Xd = torch.from_numpy(X).cuda()
    got = ops.afm_forward(Xd, m.table, m.weights["feature_bias"].reshape(-1), 0.0, Wt, b, p, P,
                          plan=plan).cpu().numpy()
    ex, mag = parity.afm_rows_exact(X, E, w, 0.0, *args)
    kappa_check("afm_rows_kappa", got, ref, ex, mag)
    A_ = X[:40]
    sc = orc.afm_catalog_scores(A_, E, w, *args, nu, ni)
    rs, ri = orc.top_k(sc, 20)
    # the default per-query kernel (folded weights) and the per-field one
    for cplan in (plan, plan | ops.PLAN_PER_FIELD):
        s_, pred = ops.afm_catalog_topk(torch.from_numpy(A_).cuda(), m.table,
                                        m.weights["feature_bias"].reshape(-1), Wt, b, p, P, nu,
                                        ni, 20, 0, plan=cplan)
        pred = pred.cpu().numpy()
        bad, swaps = orc.topk_swaps(sc, ri, pred, 1e-5 * np.abs(sc).max(1, keepdims=True))
        assert bad == 0 and swaps == 0, (cplan, bad, swaps)
        # returned scores: 1e-5 relative of the oracle's score of that item
        picked = np.take_along_axis(sc, pred.astype(np.int64), 1)
        rel = np.abs(s_.cpu().numpy() - picked) / np.maximum(np.abs(picked), 1e-30)
        assert rel.max() <= 1e-5, (cplan, float(rel.max()))


def test_afm_catalog_query_chunks():
    """max_cols forcing several query passes == one pass."""
    from hhfm_amd import ops
    rng = np.random.default_rng(1)
    nu, ni, k = 100, 900, 32
    M = nu + ni + 12
    m = _afm(nu, ni, M, k)
    A_ = np.stack([rng.integers(0, nu, 33), rng.integers(nu, nu + ni, 33),
                   rng.integers(nu + ni, nu + ni + 7, 33), rng.integers(nu + ni + 7, nu + ni + 9, 33),
                   rng.integers(nu + ni + 9, M, 33)], 1).astype(np.int32)
    q = torch.from_numpy(A_).cuda()
    Wt, b, p, P = m._att()
    res = [ops.afm_catalog_topk(q, m.table, m.weights["feature_bias"].reshape(-1), Wt, b, p, P,
                                nu, ni, 20, 0, mc)[1].cpu().numpy() for mc in (1 << 17, 4 * 32 * 5)]
    assert np.array_equal(res[0], res[1])


@pytest.mark.parametrize("F,k,A,tdt,B", [
    (2, 16, 8, "f32", 1),        # fused: one pair per row, 32 rows per MFMA block
    (3, 48, 40, "bf16", 257),    # fused: NT=2, bf16 table, ragged rows
    (7, 32, 96, "f32", 1001),    # fused: 21 pairs, NT=3
    (8, 64, 64, "bf16", 130),    # fused: 28 pairs (largest that fits 32 columns)
    (9, 32, 32, "f32", 300),     # GEMM path: 36 pairs > 32
    (5, 20, 16, "f32", 77),      # GEMM path: k % 8 != 0
    (12, 64, 64, "f32", 203),    # GEMM path: 66 pairs (resturant / ml width, F = 12)
    (16, 32, 48, "bf16", 65),    # GEMM path: 120 pairs, the largest F
])
def test_afm_rows_envelope(F, k, A, tdt, B):
    """A1 across the fused kernel's envelope (F <= 8, k % 8 == 0) and the
    GEMM path beyond it, fp32 and bf16 tables, against the oracle."""
    from tests.helpers import bf16_round
    rng = np.random.default_rng(F * 100 + k)
    M = 811
    tdtype = torch.bfloat16 if tdt == "bf16" else torch.float32
    m = _afm(50, 700, M, k, A, F=F, table_dtype=tdtype)
    W = m.get_weights()
    W["feature_bias"] = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    m.set_weights(feature_bias=W["feature_bias"])
    X = rng.integers(0, M, size=(B, F)).astype(np.int32)
    E = W["feature_embeddings"]
    if tdt == "bf16":
        E = bf16_round(E)
    args = (W["attention_W"], W["attention_b"], W["attention_p"], W["prediction"])
    ref = orc.afm_out(X, E, W["feature_bias"][:, 0], 0.0, *args)[:, 0]
    got = m.score_rows(X)[:, 0]
    ex, mag = parity.afm_rows_exact(X, E, W["feature_bias"][:, 0], 0.0, *args)
    kappa_check("afm_rows_kappa", got, ref, ex, mag)


@pytest.mark.parametrize("F,k,A,tdt,nq,ni,K", [
    (5, 64, 64, "f32", 37, 1001, 20),     # fused (Frappe shape), ragged last item tile
    (3, 48, 40, "bf16", 9, 700, 1),       # fused: A padded to 64, bf16 table
    (8, 32, 96, "f32", 5, 333, 64),       # fused: 7 query fields, NT = 3
    (4, 16, 8, "bf16", 70, 64, 5),        # fused: one tile pair per query group
    (9, 32, 32, "f32", 11, 500, 20),      # GEMM path: 8 query fields
    (5, 20, 16, "f32", 13, 400, 20),      # GEMM path: k % 8 != 0
    (5, 128, 128, "f32", 6, 300, 20),     # fused: 75 KB of LDS (raised dynamic limit)
    (12, 64, 64, "f32", 7, 250, 20),      # GEMM path: 11 query fields (F = 12 datasets)
    (5, 48, 48, "f32", 17, 901, 20),      # per-query kernel at k = 48 (U2 = 6 swizzle)
    (3, 48, 40, "f32", 33, 777, 20),      # ... A padded to 64, two query fields
    (5, 32, 96, "f32", 9, 555, 20),       # A = 96: 32-column logit groups on the GEMM path
    (5, 64, 64, "f32", 1, 100, 10),       # persistent per-query kernel: 4 tiles, grid of 4
    (5, 32, 32, "bf16", 3, 70, 5),        # ... 3 queries x 3 tiles: shares cross queries
])
def test_afm_catalog_envelope(F, k, A, tdt, nq, ni, K):
    """A2 across the fused kernels' envelope (the per-query kernel with the
    folded weights by default, the per-field kernel with PLAN_PER_FIELD) and
    the GEMM path (PLAN_GEMM, and every shape beyond the fused envelope)."""
    from hhfm_amd import ops
    from tests.helpers import bf16_round
    rng = np.random.default_rng(F * 1000 + k + A)
    nu = 60
    M = nu + ni + 40
    tdtype = torch.bfloat16 if tdt == "bf16" else torch.float32
    m = _afm(nu, ni, M, k, A, F=F, table_dtype=tdtype)
    W = m.get_weights()
    W["feature_bias"] = rng.normal(0, 0.01, (M, 1)).astype(np.float32)
    m.set_weights(feature_bias=W["feature_bias"])
    A_ = np.concatenate([rng.integers(0, nu, (nq, 1)), rng.integers(nu, nu + ni, (nq, 1)),
                         rng.integers(nu + ni, M, (nq, F - 2))], 1).astype(np.int32)
    E = W["feature_embeddings"]
    if tdt == "bf16":
        E = bf16_round(E)
    args = (W["attention_W"], W["attention_b"], W["attention_p"], W["prediction"])
    sc = orc.afm_catalog_scores(A_, E, W["feature_bias"][:, 0], *args, nu, ni)
    rs, ri = orc.top_k(sc, K)
    pred = m.topk(A_, K)
    bad, swaps = orc.topk_swaps(sc, ri, pred, 1e-5 * np.abs(sc).max(1, keepdims=True))
    assert bad == 0 and swaps == 0, (bad, swaps)
    Wt, b, p, P = m._att()
    q = torch.from_numpy(A_).cuda()
    gemm_ok = A % 16 == 0   # the GEMM path's envelope
    for plan in (ops.PLAN_PER_FIELD,) + ((ops.PLAN_GEMM,) if gemm_ok else ()):
        s_, i_ = ops.afm_catalog_topk(q, m.table, m.weights["feature_bias"].reshape(-1), Wt, b, p,
                                      P, nu, ni, K, 0, plan=plan)
        i_ = i_.cpu().numpy()
        bad, swaps = orc.topk_swaps(sc, ri, i_, 1e-5 * np.abs(sc).max(1, keepdims=True))
        assert bad == 0 and swaps == 0, (plan, bad, swaps)
        picked = np.take_along_axis(sc, i_.astype(np.int64), 1)
        rel = np.abs(s_.cpu().numpy() - picked) / np.maximum(np.abs(picked), 1e-30)
        assert rel.max() <= 1e-5, (plan, float(rel.max()))
