"""Device harness (hhfm_pf_contains, hhfm_topk_walk) against the reference's
own Train.sample_negative / evaluate_TopK / evaluate_AUC outputs (the golden
fixtures of tests/test_harness.py, made by tests/golden/make_golden.py from
the reference harness) and against the host harness: identical samples,
identical HR / NDCG / PRE / AUC, bit for bit."""
import numpy as np
import pytest
import torch

from hhfm_amd import harness, ops
from tests.test_harness import OracleModel, make, setup  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


class DeviceOracleModel(OracleModel):
    """The oracle-backed stand-in with a cuda `device`: the Train harness
    then runs membership and the metric walk on the GPU."""
    device = torch.device("cuda", 0)


def test_sample_negative_device_golden(setup):  # noqa: F811
    d, arr, _ = setup
    t = make(d, DeviceOracleModel(arr["E"], arr["w"], d.n_user, d.n_item))
    assert t._device() is not None
    np.random.seed(7)
    got = t.sample_negative(arr["neg_in"], 10)
    assert np.array_equal(got, arr["neg_out"])


@pytest.mark.parametrize("topk", [5, 10])
@pytest.mark.parametrize("variant", ["fm", "dfm"])
def test_evaluate_topk_device_golden(setup, topk, variant):  # noqa: F811
    d, arr, ref = setup
    m = DeviceOracleModel(arr["E"], arr["w"], d.n_user, d.n_item)
    t = make(d, m, topk, eval_num=300 if variant == "fm" else 60)
    np.random.seed(11)
    assert t.evaluate_TopK(d.Test_data) == ref[f"{variant}_topk{topk}"]


@pytest.mark.parametrize("topk", [1, 5, 10, 20])
@pytest.mark.parametrize("variant,seed", [("fm", 23), ("dfm", 29)])
def test_evaluate_topk_planted_device_golden(setup, topk, variant, seed):  # noqa: F811
    """Planted targets hit every walk position 0..23 (and miss), including
    rows whose target is a train positive of its key (FM.py:354 quirk)."""
    d, arr, ref = setup
    m = DeviceOracleModel(arr["E"], arr["w"], d.n_user, d.n_item, planted=True)
    t = make(d, m, topk, eval_num=300 if variant == "fm" else 60)
    np.random.seed(seed)
    assert t.evaluate_TopK(d.Test_data) == ref[f"planted_{variant}_topk{topk}"]


def test_evaluate_auc_device_golden(setup):  # noqa: F811
    d, arr, ref = setup
    m = DeviceOracleModel(arr["E"], arr["w"], d.n_user, d.n_item)
    np.random.seed(13)
    assert make(d, m).evaluate_AUC(d.Test_data) == ref["fm_auc_test"]
    np.random.seed(19)
    assert make(d, m).evaluate_AUC(d.Train_data) == ref["fm_auc_train"]
    mh = DeviceOracleModel(arr["E"], arr["w"], d.n_user, d.n_item, fm_scores=False)
    np.random.seed(17)
    t = make(d, mh, auc_first_chunk_only=True, auc_label_filter=False)
    assert t.evaluate_AUC(d.Train_data) == ref["hhfm_auc_train"]


def test_pf_contains_matches_host_membership(setup):  # noqa: F811
    """Random rows (known and unknown keys) x candidates, the rows' own
    items, dense collisions: the device test equals the host set lookup."""
    d, _, _ = setup
    pf = d.positive_feedback
    rng = np.random.default_rng(5)
    X = np.asarray(d.Train_data.values[:, 1:], dtype=np.int64)
    rows = X[rng.integers(0, len(X), 3000)].copy()
    rows[::7, 0] = d.features_M + 5            # keys absent from positive_feedback
    # candidates: half drawn from the key's own positives (hits), half random
    cand = rng.integers(d.n_user, d.n_user + d.n_item, (3000, 17))
    keys = harness.row_keys(rows)
    for r, k in enumerate(keys):
        its = sorted(pf.get(k, ()))
        if its:
            cand[r, ::2] = rng.choice(its, size=cand[r, ::2].shape)
    dp = harness.DevicePairSet(pf, rows.shape[1] - 1, torch.device("cuda", 0))
    got = dp.contains(rows, cand)
    ref = np.array([[int(c) in pf.get(k, ()) for c in row] for k, row in zip(keys, cand)])
    assert got.shape == ref.shape and np.array_equal(got, ref)
    assert ref.sum() > 1000 and (~ref).sum() > 1000
    own = dp.contains(rows)
    assert np.array_equal(own, np.array([int(r[1]) in pf.get(k, ()) for k, r in zip(keys, rows)]))
    # empty positive_feedback: nothing is a member
    empty = harness.DevicePairSet({}, rows.shape[1] - 1, torch.device("cuda", 0))
    assert not empty.contains(rows, cand).any()


@pytest.mark.parametrize("TopK", [1, 5, 10, 20, 25])
def test_topk_walk_matches_host_walk(TopK):
    rng = np.random.default_rng(TopK)
    B, P = 4000, 20
    pred = np.stack([rng.permutation(60)[:P] for _ in range(B)]).astype(np.int32)
    target = rng.integers(0, 60, B).astype(np.int32)
    positive = (rng.random(B) < 0.45).astype(np.uint8)
    dev = torch.device("cuda", 0)
    got = ops.topk_walk(torch.from_numpy(pred).to(dev), torch.from_numpy(target).to(dev),
                        torch.from_numpy(positive).to(dev), TopK).cpu().numpy()
    host = harness.hr_ndcg_pre_at(pred, target, TopK, positive.astype(bool))
    for n, h in zip(got.tolist(), host):
        if h is None:
            assert n == -2
        elif h[0] == 0:
            assert n == -1
        else:
            assert n >= 0 and h[2] == 1 / (n + 1)
    assert {-2, -1}.issubset(set(got.tolist())) or TopK >= 20


def test_sample_negative_device_equals_host_at_frappe_shape(tmp_path):
    """A 30k-row Frappe-shape loader split, 50 negatives per row (evaluate_AUC):
    the device rejection test gives the host's samples exactly."""
    import bench
    from hhfm_amd.NewLoadData import LoadData
    np.random.seed(2016)
    d = LoadData(bench.frappe_shape_dataset(str(tmp_path), rows=30000), "frappe_shape")
    X = np.asarray(d.Train_data.values[:, 1:], dtype=np.int64)
    host = harness.Train(data=d, model=None)
    devt = harness.Train(data=d, model=DeviceOracleModel(None, None, d.n_user, d.n_item))
    np.random.seed(99)
    a = host.sample_negative(X, 50)
    np.random.seed(99)
    b = devt.sample_negative(X, 50)
    assert np.array_equal(a, b)
    nxt_dev = np.random.randint(1 << 30)      # same RNG consumption as the host path
    np.random.seed(99)
    host.sample_negative(X, 50)
    assert np.random.randint(1 << 30) == nxt_dev
