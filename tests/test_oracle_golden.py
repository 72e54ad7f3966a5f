"""Pin the CPU oracle to golden vectors produced by the reference's own model
classes (tests/golden/make_golden.py: Newcode/{FM,OurModel7,AFM,DFM}.py run
on a numpy restatement of the TF-1.x ops)."""
import os

import numpy as np
import pytest

from oracle import cpu as ocpu
from oracle import fm_oracle as orc

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(os.path.join(G, name)))


def close(a, b, rtol=1e-5, atol=1e-7):
    return np.allclose(a, b, rtol=rtol, atol=atol)


def test_fm_out_and_topk():
    d = load("fm.npz")
    assert close(orc.fm_out(d["X"], d["E"], d["w"], d["w0"])[:, 0], d["out"])
    assert close(ocpu.fm_out(d["X"], d["E"], d["w"], float(d["w0"])), d["out"])
    sc = orc.fm_catalog_scores(d["A"], d["E"], d["w"], int(d["n_user"]), int(d["n_item"]))
    assert close(sc, d["topk_scores"])
    _, idx = orc.top_k(sc, 20)
    assert np.array_equal(idx, d["topk_idx"])
    s, i = ocpu.catalog_topk(d["A"], d["E"], 0, 20, int(d["n_user"]), int(d["n_item"]),
                             w=d["w"], ctx=(2, 5))
    assert np.array_equal(i, d["topk_idx"])


@pytest.mark.parametrize("tag", ["frappe", "jiaju", "resturant"])
def test_hhfm_out_and_topk(tag):
    d = load(f"hhfm_{tag}.npz")
    fd, td = int(d["feature_dimension"]), int(d["time_dimension"])
    nu, ni = int(d["n_user"]), int(d["n_item"])
    out = orc.hhfm_positive_feedback(d["X"], d["E"], fd, td, True, td > 0)[:, 0]
    assert close(out, d["out"])
    c, t = (2, 2 + fd), ((2 + fd, 2 + fd + td) if td else (0, 0))
    assert close(ocpu.hhfm_rows(d["X"], d["E"], c, t), d["out"])
    sc = orc.hhfm_catalog_scores(d["A"], d["E"], nu, ni, fd, td, True, td > 0)
    assert close(sc, d["topk_scores"])
    assert np.array_equal(orc.top_k(sc, 20)[1], d["topk_idx"])
    s, i = ocpu.catalog_topk(d["A"], d["E"], 1, 20, nu, ni, ctx=c, time=t)
    assert np.array_equal(i, d["topk_idx"])


def test_afm_out_and_topk():
    d = load("afm.npz")
    args = (d["attention_W"], d["attention_b"], d["attention_p"], d["prediction"])
    assert close(orc.afm_out(d["X"], d["E"], d["w"], d["w0"], *args)[:, 0], d["out"])
    sc = orc.afm_catalog_scores(d["A"], d["E"], d["w"], *args, int(d["n_user"]), int(d["n_item"]))
    assert close(sc, d["topk_scores"], rtol=1e-5, atol=1e-6)
    assert np.array_equal(orc.top_k(sc, 20)[1], d["topk_idx"])


def test_dfm_out_and_topk():
    d = load("dfm.npz")
    layers = [d[f"layer_{i}"] for i in range(3)]
    biases = [d[f"bias_{i}"] for i in range(3)]
    out = orc.dfm_out(d["X"], d["E"], d["w"], layers, biases, d["concat_projection"],
                      d["concat_bias"])[:, 0]
    assert close(out, d["out"])
    sc = orc.dfm_catalog_scores(d["A"], d["E"], d["w"], layers, biases, d["concat_projection"],
                                d["concat_bias"], int(d["n_user"]), int(d["n_item"]))
    assert close(sc, d["topk_scores"])
    assert np.array_equal(orc.top_k(sc, 20)[1], d["topk_idx"])


def test_known_answers():
    """Hand-computable cases: F=2,k=1 -> ½((a+b)²−a²−b²) = ab."""
    E = np.array([[3.0], [5.0], [0.0]], np.float32)
    w = np.array([0.5, 0.25, 0.0], np.float32)
    out = orc.fm_out(np.array([[0, 1]]), E, w, 1.0)
    assert out[0, 0] == np.float32(15.0 + 0.75 + 1.0)
    # HHFM: (u + c) · i
    E = np.array([[1.0, 2.0], [3.0, 4.0], [0.5, 0.5]], np.float32)
    assert orc.hhfm_positive_feedback(np.array([[0, 1, 2]]), E, 1, 0)[0, 0] == np.float32(1.5 * 3 + 2.5 * 4)
    # top_k ties: lower index first
    v, i = orc.top_k(np.array([[1.0, 2.0, 2.0, 0.0, 2.0]]), 3)
    assert i.tolist() == [[1, 2, 4]]


def test_c_oracle_matches_numpy_at_scale():
    from tests.helpers import synth_rows, table
    rng = np.random.default_rng(9)
    X, M = synth_rows(rng, 20000, 957, 4082, (7, 2, 3))
    E = table(rng, M, 64)
    w = rng.normal(0, 0.01, M).astype(np.float32)
    assert close(ocpu.fm_out(X, E, w, 0.2), orc.fm_out(X, E, w, 0.2)[:, 0])
