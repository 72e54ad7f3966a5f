"""GPU end-to-end parity of the drop-in model classes against the golden
vectors that the REFERENCE's own graphs produced (tests/golden/*.npz), and
HR@10 identity through the harness on Frappe-shape synthetic data."""
import os

import numpy as np
import pytest
import torch

from oracle import fm_oracle as orc
from tests.helpers import bf16_round

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
RTOL = 1e-5


def load(name):
    return dict(np.load(os.path.join(G, name)))


def _assert_topk(ref_scores, got_idx, K=20, rtol=RTOL):
    rs, ri = orc.top_k(ref_scores, K + 1)
    scale = np.abs(ref_scores).max(1, keepdims=True)
    mism, amb = orc.topk_index_agreement(rs, ri[:, :K], got_idx, rtol * scale)
    assert mism == 0, (mism, amb)
    return amb


def test_fm_model_vs_reference_graph():
    from hhfm_amd.FM import FM
    d = load("fm.npz")
    nu, ni = int(d["n_user"]), int(d["n_item"])
    M, k = d["E"].shape
    m = FM(5, M, nu, ni, k, 0.1, 0.1, 1, "AdagradOptimizer", 0, 0)
    m.set_weights(feature_embeddings=d["E"], feature_bias=d["w"][:, None], bias=d["w0"])
    out = m.score_rows(d["X"])[:, 0]
    assert np.allclose(out, d["out"], rtol=RTOL, atol=1e-7)
    # the reference call form: sess.run(model.out, feed_dict=...)
    out2 = m.sess.run(m.out, feed_dict={m.train_features: d["X"], m.train_labels: None,
                                         m.dropout_keep: 1.0, m.train_phase: False})
    assert np.array_equal(out2[:, 0], out)
    pred = m.topk(d["A"], 20)
    assert pred.dtype == np.int32 and pred.shape == (len(d["A"]), 20)
    amb = _assert_topk(d["topk_scores"], pred)
    dec = pred[:, :5] == d["topk_idx"][:, :5]
    assert dec.mean() > 0.95 or amb > 0


@pytest.mark.parametrize("tag", ["frappe", "jiaju", "resturant"])
def test_hhfm_model_vs_reference_graph(tag):
    from hhfm_amd.OurModel7 import OUR
    d = load(f"hhfm_{tag}.npz")
    fd, td = int(d["feature_dimension"]), int(d["time_dimension"])
    nu, ni = int(d["n_user"]), int(d["n_item"])
    M, k = d["E"].shape
    m = OUR(fd, td, M, nu, ni, k, 0.1, 0.01, "AdagradOptimizer", True, td > 0)
    m.set_weights(feature_embeddings=d["E"])
    out = m.score_rows(d["X"])[:, 0]
    assert np.allclose(out, d["out"], rtol=RTOL, atol=1e-8)
    feed = {m.Pos: d["X"][:, :2], m.Fea: d["X"][:, 2:2 + fd]}
    if td:
        feed[m.Tim] = d["X"][:, 2 + fd:]
    assert np.array_equal(m.sess.run(m.PositiveFeadback, feed_dict=feed)[:, 0], out)
    pred = m.topk(d["A"], 20)
    _assert_topk(d["topk_scores"], pred)
    assert (pred == d["topk_idx"]).mean() > 0.95


def test_hhfm_bf16_table_parity():
    from hhfm_amd.OurModel7 import OUR
    d = load("hhfm_frappe.npz")
    nu, ni = int(d["n_user"]), int(d["n_item"])
    M, k = d["E"].shape
    m = OUR(3, 0, M, nu, ni, k, 0.1, 0.01, "AdagradOptimizer", True, False,
            table_dtype=torch.bfloat16)
    m.set_weights(feature_embeddings=d["E"])
    Eb = bf16_round(d["E"])
    ref = orc.hhfm_positive_feedback(d["X"], Eb, 3, 0)[:, 0]
    assert np.allclose(m.score_rows(d["X"])[:, 0], ref, rtol=RTOL, atol=1e-8)
    _assert_topk(orc.hhfm_catalog_scores(d["A"], Eb, nu, ni, 3, 0), m.topk(d["A"], 20))


def test_out_of_range_ids_raise_like_tf():
    from hhfm_amd.FM import FM
    m = FM(5, 100, 10, 50, 16, 0.1, 0.1, 1, "AdagradOptimizer", 0, 0)
    with pytest.raises(ValueError):
        m.score_rows(np.array([[0, 10, 99, 100, 1]]))


def test_hr_at_10_identical_to_oracle_through_harness():
    """Same loader split, same sampled rows, same top-20 lists => identical
    HR/NDCG/PRE@10 (GPU model vs the oracle model) on Frappe-shape data."""
    from hhfm_amd.harness import Train
    from hhfm_amd.NewLoadData import LoadData
    from hhfm_amd.OurModel7 import OUR
    from tests.test_harness import OracleModel
    np.random.seed(2016)
    data = LoadData(G + "/", "synth_frappe")
    E = np.random.default_rng(7).normal(0, 0.01, (data.features_M, 64)).astype(np.float32)
    gpu = OUR(3, 0, data.features_M, data.n_user, data.n_item, 64, 0.1, 0.01,
              "AdagradOptimizer", True, False)
    gpu.set_weights(feature_embeddings=E)
    ref = OracleModel(E, None, data.n_user, data.n_item, fm_scores=False)
    for topk in (5, 10):
        res = []
        for model in (gpu, ref):
            t = Train(data=data, model=model)
            t.TopK = topk
            np.random.seed(99)
            res.append(t.evaluate_TopK(data.Test_data))
        assert res[0] == res[1], res
    aucs = []
    for model in (gpu, ref):
        t = Train(data=data, model=model)
        np.random.seed(5)
        aucs.append(t.evaluate_AUC(data.Test_data))
    # strict pos > neg on fp32 scores: allow a flip of at most 2 near-ties
    assert abs(aucs[0] - aucs[1]) <= 2.0 / (50 * len(data.Test_data))


def test_sharded_catalog_on_one_device_matches_full():
    """The multi-GPU decomposition (shard scorers + merge) on one device."""
    from hhfm_amd import distributed as hd
    from hhfm_amd import ops
    from hhfm_amd.OurModel7 import OUR
    d = load("hhfm_frappe.npz")
    nu, ni = int(d["n_user"]), int(d["n_item"])
    M, k = d["E"].shape
    m = OUR(3, 0, M, nu, ni, k, 0.1, 0.01, "AdagradOptimizer", True, False)
    m.set_weights(feature_embeddings=d["E"])
    sc = hd.model_scorer(m)
    parts = [sc(d["A"], *hd.shard_range(ni, 8, r)[:1], np.diff(hd.shard_range(ni, 8, r))[0], 20)
             for r in range(8)]
    gs = torch.stack([p[0] for p in parts])
    gi = torch.stack([p[1] for p in parts])
    s, i = ops.topk_merge(gs, gi)
    assert np.array_equal(i.cpu().numpy(), m.topk(d["A"], 20))
