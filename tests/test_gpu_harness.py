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


def _state_eq(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2] and a[3:] == b[3:]


def _both(t_host, t_dev, X, num, prime):
    """host and device sample_negative from the same RandomState: samples
    and the state after the call (np.random.get_state) must be equal."""
    prime()
    s0 = np.random.get_state()
    a = t_host.sample_negative(X, num)
    sa = np.random.get_state()
    np.random.set_state(s0)
    b = t_dev.sample_negative(X, num)
    sb = np.random.get_state()
    assert a.dtype == b.dtype and a.shape == b.shape
    assert np.array_equal(a, b), int((a != b).sum())
    assert _state_eq(sa, sb), (sa[2], sb[2])
    return a


def test_sample_negative_on_device_frappe_shape_state(tmp_path):
    """The whole sampler on the device (hhfm_sample_negative: MT19937 words,
    masked bounded draws, membership, row-major re-draws) at the row-table
    shape — every Frappe-shape train row, 50 negatives (evaluate_AUC's draw):
    the samples AND numpy's generator state afterwards equal the host
    harness's (the reference's stream), from a fresh seed (pos 624), from
    mid-block positions, and from pos = 624 after a full block."""
    import bench
    from hhfm_amd.NewLoadData import LoadData
    np.random.seed(2016)
    d = LoadData(bench.frappe_shape_dataset(str(tmp_path)), "frappe_shape")
    X = np.asarray(d.Train_data.values[:, 1:], dtype=np.int64)
    host = harness.Train(data=d, model=None)
    devt = harness.Train(data=d, model=DeviceOracleModel(None, None, d.n_user, d.n_item))
    _both(host, devt, X, 50, lambda: np.random.seed(99))
    _both(host, devt, X[:1000], 2, lambda: (np.random.seed(5), np.random.randint(0, 7, 333)))
    _both(host, devt, X[:777], 10,
          lambda: (np.random.seed(6), np.random.randint(0, 1 << 32, 624, dtype=np.uint64)))
    # a second call continues the stream like the reference's
    np.random.seed(3)
    a1, a2 = host.sample_negative(X[:5000], 10), host.sample_negative(X[5000:9000], 50)
    np.random.seed(3)
    b1, b2 = devt.sample_negative(X[:5000], 10), devt.sample_negative(X[5000:9000], 50)
    assert np.array_equal(a1, b1) and np.array_equal(a2, b2)


class _PF:
    def __init__(self, pf, n_user, n_item):
        self.positive_feedback, self.n_user, self.n_item = pf, n_user, n_item


@pytest.mark.parametrize("bitmaps", [True, False])
@pytest.mark.parametrize("n_item,cover", [(5, 0.8), (2, 0.5), (64, 0.9), (65, 0.5),
                                          (1000, 0.97), (1, 0.0)])
def test_sample_negative_on_device_heavy_rejection(n_item, cover, bitmaps, monkeypatch):
    """Keys whose positives cover most of the catalog force long re-draw
    chains (several rounds of 256 entries, values running out, generation
    rounds that slide the MT window); catalogs of 2^k and 2^k + 1 items set
    the mask's rejection rate to 0 and ~1/2; one item draws nothing
    (randint(lo, lo + 1)).  Device == host harness, samples and state, with
    the re-draw test on key bitmaps and on the binary searches."""
    monkeypatch.setattr(harness, "SAMPLER_BITMAPS", bitmaps)
    rng = np.random.default_rng(n_item)
    n_user, ncols = 40, 4
    keys = [tuple(int(v) for v in rng.integers(0, 50, ncols - 1)) for _ in range(60)]
    pf = {}
    for k in keys:
        n_pos = min(int(cover * n_item), n_item - 1)
        pf[k] = set(int(n_user + i) for i in rng.choice(n_item, n_pos, replace=False))
    rows = []
    for _ in range(3000):
        k = keys[rng.integers(0, len(keys))] if rng.random() < 0.9 else (99, 99, 99)
        rows.append([k[0], n_user, k[1], k[2]])
    X = np.asarray(rows, dtype=np.int64)
    data = _PF(pf, n_user, n_item)
    host = harness.Train(data=data, model=None)
    devt = harness.Train(data=data, model=DeviceOracleModel(None, None, n_user, n_item))
    for seed, num in ((1, 10), (2, 1), (3, 50)):
        _both(host, devt, X, num, lambda: np.random.seed(seed))


def test_sample_negative_on_device_refuses_a_hang():
    """A key whose positives are the whole catalog makes the reference loop
    forever (FM.py:291-293); the device sampler reports it instead."""
    n_user, n_item = 10, 4
    pf = {(1, 2, 3): set(range(n_user, n_user + n_item))}
    X = np.asarray([[1, n_user, 2, 3]] * 5, dtype=np.int64)
    devt = harness.Train(data=_PF(pf, n_user, n_item),
                         model=DeviceOracleModel(None, None, n_user, n_item))
    with pytest.raises(ValueError):
        devt.sample_negative(X, 3)


def test_sample_negative_on_device_one_free_item_in_50k():
    """Keys whose positives cover all but ONE item of a 50,000-item catalog:
    every entry of such a row re-draws ~50,000 times (the reference finishes,
    slowly), far past the old guard of 64 + count/1024 generation rounds.
    Device == host harness, samples and state."""
    n_user, n_item = 10, 50_000
    rng = np.random.default_rng(50_000)
    pf = {}
    for key in ((1, 2, 3), (4, 5, 6)):
        free = int(rng.integers(0, n_item))
        pf[key] = set(n_user + i for i in range(n_item) if i != free)
    rows = [[1, n_user, 2, 3]] * 6 + [[4, n_user, 5, 6]] * 6 + [[7, n_user, 8, 9]] * 4
    X = np.asarray(rows, dtype=np.int64)
    data = _PF(pf, n_user, n_item)
    host = harness.Train(data=data, model=None)
    devt = harness.Train(data=data, model=DeviceOracleModel(None, None, n_user, n_item))
    a = _both(host, devt, X, 2, lambda: np.random.seed(11))
    for key, r in ((1, a[:6]), (4, a[6:12])):
        k = (key, key + 1, key + 2)
        assert not any(int(v) in pf[k] for v in r.ravel())
