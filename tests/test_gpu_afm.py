"""AFM (K4) on the GPU vs the reference graph (golden afm.npz) and vs the
oracle at Frappe shape.  fp32 numerics (exact-fp32 MFMA, or split-bf16 MFMA
for the fused rows kernel when k % 16 == 0 — HHFM_AFM_EXACT=1 forces the
former); tolerance 1e-5 of the natural magnitude of each reduction."""
import os

import numpy as np
import pytest
import torch

from oracle import fm_oracle as orc

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
    scale = np.abs(d["out"]).max()
    assert np.allclose(out, d["out"], rtol=1e-5, atol=1e-5 * scale)
    out2 = m.sess.run(m.out, feed_dict={m.train_features: d["X"], m.train_labels: None,
                                         m.dropout_keep: [1.0, 1.0], m.train_phase: False})
    assert np.array_equal(out2[:, 0], out)
    pred = m.topk(d["A"], 20)
    # bit-exact against the reference graph's golden top-20
    assert np.array_equal(pred, d["topk_idx"]), int((pred != d["topk_idx"]).sum())


@pytest.mark.parametrize("exact", ["0", "1"])
@pytest.mark.parametrize("k,A", [(64, 64), (32, 16), (128, 128), (64, 32), (24, 32)])
def test_afm_frappe_shape(k, A, exact, monkeypatch):
    monkeypatch.setenv("HHFM_AFM_EXACT", exact)
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
    ref = orc.afm_out(X, W["feature_embeddings"], W["feature_bias"][:, 0], 0.0, *args)[:, 0]
    got = m.score_rows(X)[:, 0]
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())
    A_ = X[:40]
    sc = orc.afm_catalog_scores(A_, W["feature_embeddings"], W["feature_bias"][:, 0], *args, nu, ni)
    pred = m.topk(A_, 20)
    rs, ri = orc.top_k(sc, 20)
    bad, swaps = orc.topk_swaps(sc, ri, pred, 1e-5 * np.abs(sc).max(1, keepdims=True))
    assert bad == 0 and swaps == 0, (bad, swaps)


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
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max())


@pytest.mark.parametrize("F,k,A,tdt,nq,ni,K", [
    (5, 64, 64, "f32", 37, 1001, 20),     # fused (Frappe shape), ragged last item tile
    (3, 48, 40, "bf16", 9, 700, 1),       # fused: A padded to 64, bf16 table
    (8, 32, 96, "f32", 5, 333, 64),       # fused: 7 query fields, NT = 3
    (4, 16, 8, "bf16", 70, 64, 5),        # fused: one tile pair per query group
    (9, 32, 32, "f32", 11, 500, 20),      # GEMM path: 8 query fields
    (5, 20, 16, "f32", 13, 400, 20),      # GEMM path: k % 8 != 0
    (5, 128, 128, "f32", 6, 300, 20),     # fused: 75 KB of LDS (raised dynamic limit)
    (12, 64, 64, "f32", 7, 250, 20),      # GEMM path: 11 query fields (F = 12 datasets)
])
def test_afm_catalog_envelope(F, k, A, tdt, nq, ni, K):
    """A2 across the fused kernel's envelope and the GEMM path beyond it."""
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
    pred = m.topk(A_, K)
    rs, ri = orc.top_k(sc, K)
    bad, swaps = orc.topk_swaps(sc, ri, pred,
                                         1e-5 * np.abs(sc).max(1, keepdims=True))
    assert bad == 0 and swaps == 0, (bad, swaps)
