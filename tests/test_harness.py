"""hhfm_amd.harness vs the reference's own Train.sample_negative /
evaluate_TopK / evaluate_AUC (fixtures from tests/golden/make_golden.py),
driven by oracle-backed stand-in models: identical RNG streams and metric
walks (including the FM.py:354 quirk) give identical numbers."""
import json
import os

import numpy as np
import pytest

from hhfm_amd import harness
from hhfm_amd.NewLoadData import LoadData
from oracle import fm_oracle as orc

G = os.path.join(os.path.dirname(__file__), "golden")


def planted_topk(A, n_user, n_item, tp):
    """Identical to make_golden.planted_topk (target planted at rank (7u+c1)%24)."""
    out = np.empty((A.shape[0], tp), dtype=np.int32)
    for r, line in enumerate(A):
        tgt = int(line[1]) - n_user
        fill = [(tgt + 1 + 3 * j) % n_item for j in range(tp)]
        pos = (7 * int(line[0]) + int(line[2])) % 24
        if pos < tp:
            fill[pos] = tgt
        out[r] = fill
    return out


class OracleModel:
    def __init__(self, E, w, nu, ni, fm_scores=True, planted=False):
        self.E, self.w, self.nu, self.ni = E, w, nu, ni
        self.fm_scores, self.planted = fm_scores, planted

    def score_rows(self, X):
        if self.fm_scores:
            return orc.fm_out(X, self.E, self.w)
        return orc.hhfm_positive_feedback(X, self.E, 3, 0)

    def topk(self, A, tp):
        if self.planted:
            return planted_topk(np.asarray(A), self.nu, self.ni, tp)
        return orc.hhfm_topk(A, self.E, self.nu, self.ni, 3, 0, tp=tp)[1]


@pytest.fixture(scope="module")
def setup():
    np.random.seed(2016)
    d = LoadData(G + "/", "synth_frappe")
    arr = np.load(os.path.join(G, "harness.npz"))
    with open(os.path.join(G, "harness.json")) as f:
        ref = json.load(f)
    return d, arr, ref


def make(d, model, TopK=10, cls=harness.Train, **attrs):
    t = cls(data=d, model=model)
    t.TopK = TopK
    for k, v in attrs.items():
        setattr(t, k, v)
    return t


def test_sample_negative_same_stream(setup):
    d, arr, _ = setup
    t = make(d, None)
    np.random.seed(7)
    got = t.sample_negative(arr["neg_in"], 10)
    assert np.array_equal(got, arr["neg_out"])
    # no sampled negative is a positive of its key
    keys = harness.row_keys(arr["neg_in"])
    for k, row in zip(keys, got):
        assert not (set(row.tolist()) & d.positive_feedback.get(k, set()))


@pytest.mark.parametrize("topk", [5, 10])
@pytest.mark.parametrize("variant", ["fm", "dfm"])
def test_evaluate_topk_oracle_model(setup, topk, variant):
    d, arr, ref = setup
    m = OracleModel(arr["E"], arr["w"], d.n_user, d.n_item)
    t = make(d, m, topk, eval_num=300 if variant == "fm" else 60)
    np.random.seed(11)
    assert t.evaluate_TopK(d.Test_data) == pytest.approx(ref[f"{variant}_topk{topk}"], abs=0, rel=0)


@pytest.mark.parametrize("topk", [1, 5, 10, 20])
@pytest.mark.parametrize("variant,seed", [("fm", 23), ("dfm", 29)])
def test_evaluate_topk_planted(setup, topk, variant, seed):
    d, arr, ref = setup
    m = OracleModel(arr["E"], arr["w"], d.n_user, d.n_item, planted=True)
    t = make(d, m, topk, eval_num=300 if variant == "fm" else 60)
    np.random.seed(seed)
    got = t.evaluate_TopK(d.Test_data)
    assert got == ref[f"planted_{variant}_topk{topk}"]


def test_evaluate_auc_fm_and_hhfm_variants(setup):
    d, arr, ref = setup
    m = OracleModel(arr["E"], arr["w"], d.n_user, d.n_item)
    np.random.seed(13)
    assert make(d, m).evaluate_AUC(d.Test_data) == ref["fm_auc_test"]
    np.random.seed(19)
    assert make(d, m).evaluate_AUC(d.Train_data) == ref["fm_auc_train"]
    mh = OracleModel(arr["E"], arr["w"], d.n_user, d.n_item, fm_scores=False)
    np.random.seed(17)
    t = make(d, mh, auc_first_chunk_only=True, auc_label_filter=False)
    assert t.evaluate_AUC(d.Train_data) == ref["hhfm_auc_train"]
