"""hhfm_amd.NewLoadData.LoadData vs the reference LoadData's outputs
(tests/golden/make_golden.py ran Newcode/NewLoadData.py with seed 2016)."""
import hashlib
import json
import os

import numpy as np
import pytest

from hhfm_amd.NewLoadData import LoadData

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("encoder", ["native", "python"])
@pytest.mark.parametrize("tag", ["frappe", "jiaju"])
def test_loaddata_matches_reference(tag, encoder):
    """encoder="native": C++ tokenizer / id map / split walk (libhhfm.so host
    code, hhfm_libfm_encode + hhfm_loader_split); "python": pandas."""
    ref = np.load(os.path.join(G, f"loaddata_{tag}.npz"))
    np.random.seed(2016)
    d = LoadData(G + "/", f"synth_{tag}", encoder=encoder)
    assert d.n_user == int(ref["n_user"]) and d.n_item == int(ref["n_item"])
    assert d.features_M == int(ref["features_M"])
    assert list(d.Train_data.columns) == list(ref["columns"])
    assert np.array_equal(d.Train_data.values, ref["train"])
    assert np.array_equal(d.Test_data.values, ref["test"])
    keys, items = [], []
    for k in sorted(d.positive_feedback):
        for it in sorted(d.positive_feedback[k]):
            keys.append(k)
            items.append(it)
    assert np.array_equal(np.array(keys), ref["pf_keys"])
    assert np.array_equal(np.array(items), ref["pf_items"])


def test_loaddata_shared_token_ids():
    """Quirk 1: identical tokens in different columns share one id."""
    np.random.seed(0)
    d = LoadData(G + "/", "synth_frappe")
    import pandas as pd
    raw = pd.read_csv(os.path.join(G, "synth_frappe", "synth_frappe.libfm"), sep=" ", header=None)
    tokens = raw.values[:, 1:].T.reshape(-1)
    first = {}
    for t in tokens:
        first.setdefault(t, len(first))
    assert d.features_M == len(first)
    # "night" appears as daytime and as homework value -> one id
    assert "night" in set(raw[3]) and "night" in set(raw[5])


REAL = "/root/reference/data/positive/"


@pytest.mark.parametrize("encoder", ["native", "python"])
@pytest.mark.skipif(not os.path.exists(REAL + "frappe/frappe.libfm"),
                    reason="real Frappe only exists in the builder container")
def test_loaddata_real_frappe_hashes(encoder):
    with open(os.path.join(G, "frappe_real.json")) as f:
        ref = json.load(f)
    np.random.seed(2016)
    d = LoadData(REAL, "frappe", encoder=encoder)
    assert [d.n_user, d.n_item, d.features_M] == ref["sizes"]
    assert hashlib.sha256(np.ascontiguousarray(d.Train_data.values, np.int64)).hexdigest() == ref["train_sha256"]
    assert hashlib.sha256(np.ascontiguousarray(d.Test_data.values, np.int64)).hexdigest() == ref["test_sha256"]


@pytest.mark.skipif(not os.path.exists(REAL + "frappe/frappe.libfm"),
                    reason="real Frappe only exists in the builder container")
def test_hr_at_k_real_frappe_matches_reference_harness():
    """Same loader split + same sampled rows + same top-20 lists => the same
    HR/NDCG/PRE@K as the reference harness on real Frappe (model: seeded
    random-weight HHFM scored by the oracle; trained reference weights do
    not exist)."""
    from hhfm_amd.OurModel7 import Train as M7Train
    from tests.test_harness import OracleModel
    with open(os.path.join(G, "frappe_real.json")) as f:
        ref = json.load(f)
    np.random.seed(2016)
    d = LoadData(REAL, "frappe")
    E = np.random.default_rng(606).normal(0, 0.01, (d.features_M, 64)).astype(np.float32)
    m = OracleModel(E, None, d.n_user, d.n_item, fm_scores=False)
    for topk in (5, 10):
        t = M7Train.__new__(M7Train)
        import hhfm_amd.harness as H
        H.Train.__init__(t, data=d, model=m)
        t.TopK = topk
        np.random.seed(31)
        assert t.evaluate_TopK(d.Test_data) == ref[f"hhfm_random_w_topk{topk}"]


def test_loaddata_native_equals_python_frappe_shape(tmp_path):
    """Frappe-shape synthetic libfm (96k rows of string tokens): the C++
    encoder + split walk give the pandas path's fields exactly, and consume
    the same numpy RNG draws."""
    import bench
    path = bench.frappe_shape_dataset(str(tmp_path))
    out, nxt = {}, {}
    for enc in ("native", "python"):
        np.random.seed(2016)
        out[enc] = LoadData(path, "frappe_shape", encoder=enc)
        nxt[enc] = np.random.randint(1 << 30)
    a, b = out["native"], out["python"]
    assert (a.n_user, a.n_item, a.features_M) == (b.n_user, b.n_item, b.features_M)
    assert np.array_equal(a.Train_data.values, b.Train_data.values)
    assert np.array_equal(a.Test_data.values, b.Test_data.values)
    assert a.positive_feedback == b.positive_feedback and a.train_set == b.train_set
    assert nxt["native"] == nxt["python"]


def test_libfm_encode_rejects_ragged_rows(tmp_path):
    (tmp_path / "bad").mkdir()
    (tmp_path / "bad" / "bad.libfm").write_text("1 a b c\n1 a b\n")
    with pytest.raises(ValueError):
        LoadData(str(tmp_path) + "/", "bad", encoder="native")


def test_libfm_encode_crlf_and_blank_lines(tmp_path):
    """Windows line ends and blank lines: the C++ tokenizer gives the pandas
    path's ids, labels and split (read_csv skips blank lines)."""
    d = tmp_path / "crlf"
    d.mkdir()
    rng = np.random.default_rng(3)
    lines = []
    for r in range(400):
        lines.append(f"{rng.choice([1, -1])} u{rng.integers(0, 30)} i{rng.integers(0, 50)} "
                     f"c{rng.integers(0, 4)} d{rng.integers(0, 3)}")
        if r % 97 == 0:
            lines.append("")
    (d / "crlf.libfm").write_bytes(("\r\n".join(lines) + "\r\n\r\n").encode())
    out = {}
    for enc in ("native", "python"):
        np.random.seed(5)
        out[enc] = LoadData(str(tmp_path) + "/", "crlf", encoder=enc)
    a, b = out["native"], out["python"]
    assert (a.n_user, a.n_item, a.features_M) == (b.n_user, b.n_item, b.features_M)
    assert np.array_equal(a.Train_data.values, b.Train_data.values)
    assert np.array_equal(a.Test_data.values, b.Test_data.values)
    assert a.positive_feedback == b.positive_feedback
