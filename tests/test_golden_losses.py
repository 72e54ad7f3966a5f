"""H6 training objectives pinned by the REFERENCE's own loss graphs.

tests/golden/losses.npz holds `self.loss` of FM.py:123-126, OurModel7.py:
172-184, AFM.py:144-148 and DFM.py:139-152, evaluated by the unmodified
reference modules (tests/golden/make_golden.py, TF ops restated by
tf1_numpy.py) at seeded weights on a seeded batch with negatives.  The
oracle's training steps (CPU, here) and the GPU partial_fit kernels
(-m gpu) must return those values: partial_fit reports the loss of the
parameters BEFORE its update, as sess.run((loss, optimizer)) does."""
import os

import numpy as np
import pytest

from oracle import fm_oracle as orc

G = os.path.join(os.path.dirname(__file__), "golden")
RTOL = 1e-5


def load():
    return dict(np.load(os.path.join(G, "losses.npz")))


def _acc(*arrays):
    return [np.full_like(np.asarray(a, np.float32), 0.1) for a in arrays]


def test_oracle_fm_loss():
    d = load()
    accE, accw = _acc(d["fm_E"], d["fm_w"])
    loss = orc.fm_train_step(d["fm_X"], d["fm_Y"], d["fm_E"], d["fm_w"], d["fm_w0"], accE, accw,
                             np.float32(0.1), 0.1, float(d["fm_lamda"]))[0]
    assert np.isclose(loss, d["fm_loss"], rtol=RTOL), (loss, d["fm_loss"])


def test_oracle_hhfm_loss():
    d = load()
    (accE,) = _acc(d["hhfm_E"])
    loss = orc.hhfm_train_step(d["hhfm_X"], d["hhfm_Neg"], d["hhfm_E"], accE, 0.1,
                               float(d["hhfm_lamda"]), 3, 0)[0]
    assert np.isclose(loss, d["hhfm_loss"], rtol=RTOL), (loss, d["hhfm_loss"])


def _afm_args(d):
    names = ("E", "w", "w0", "W", "b", "p", "P")
    vals = (d["afm_E"], d["afm_w"], d["afm_w0"], d["afm_attention_W"], d["afm_attention_b"],
            d["afm_attention_p"], d["afm_prediction"])
    acc = {n: np.full_like(np.asarray(v, np.float32), 0.1) for n, v in zip(names, vals)}
    return vals, acc


def test_oracle_afm_loss():
    d = load()
    vals, acc = _afm_args(d)
    loss = orc.afm_train_step(d["afm_X"], d["afm_Y"], *vals, acc, 0.1, float(d["afm_lamda"]))[0]
    assert np.isclose(loss, d["afm_loss"], rtol=RTOL), (loss, d["afm_loss"])


def _dfm_parts(d):
    layers = [d["dfm_layer_0"], d["dfm_layer_1"]]
    biases = [d["dfm_bias_0"], d["dfm_bias_1"]]
    acc = {"E": d["dfm_E"], "w": d["dfm_w"], "Wp": d["dfm_concat_projection"],
           "bp": np.float32(d["dfm_concat_bias"])}
    for i in range(2):
        acc[f"W{i}"] = layers[i]
        acc[f"b{i}"] = biases[i]
    acc = {n: np.full_like(np.asarray(v, np.float32), 0.1) for n, v in acc.items()}
    return layers, biases, acc


def test_oracle_dfm_loss():
    d = load()
    layers, biases, acc = _dfm_parts(d)
    loss = orc.dfm_train_step(d["dfm_X"], d["dfm_Y"], d["dfm_E"], d["dfm_w"], layers, biases,
                              d["dfm_concat_projection"], d["dfm_concat_bias"], acc, 0.01,
                              float(d["dfm_l2"]))[0]
    assert np.isclose(loss, d["dfm_loss"], rtol=RTOL), (loss, d["dfm_loss"])


# ---------------------------------------------------------------------------
# GPU partial_fit (csrc/train.hip) against the same reference-graph values
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("opt", ["AdagradOptimizer", "GradientDescentOptimizer"])
def test_gpu_fm_partial_fit_returns_reference_loss(opt):
    from hhfm_amd.FM import FM
    d = load()
    M, k = d["fm_E"].shape
    m = FM(5, M, int(d["n_user"]), int(d["n_item"]), k, 0.1, float(d["fm_lamda"]), 1, opt, 0, 0)
    m.set_weights(feature_embeddings=d["fm_E"], feature_bias=d["fm_w"][:, None],
                  bias=d["fm_w0"])
    loss = m.partial_fit({"X": d["fm_X"], "Y": d["fm_Y"][:, None]})
    assert np.isclose(loss, d["fm_loss"], rtol=RTOL), (loss, d["fm_loss"])


@pytest.mark.gpu
def test_gpu_hhfm_partial_fit_returns_reference_loss():
    from hhfm_amd.OurModel7 import OUR
    d = load()
    M, k = d["hhfm_E"].shape
    m = OUR(3, 0, M, int(d["n_user"]), int(d["n_item"]), k, 0.1, float(d["hhfm_lamda"]),
            "AdagradOptimizer", True, False)
    m.set_weights(feature_embeddings=d["hhfm_E"])
    X = d["hhfm_X"]
    loss = m.partial_fit({"X": X[:, :2], "F1": X[:, 2:], "Y": d["hhfm_Neg"]})
    assert np.isclose(loss, d["hhfm_loss"], rtol=RTOL), (loss, d["hhfm_loss"])


@pytest.mark.gpu
def test_gpu_afm_partial_fit_returns_reference_loss():
    from hhfm_amd.AFM import AFM
    d = load()
    M, k = d["afm_E"].shape
    m = AFM(int(d["n_user"]), int(d["n_item"]), M, 1, [k, k], None, 0.1, float(d["afm_lamda"]),
            [1, 1], "AdagradOptimizer", 0.999, 5)
    m.set_weights(feature_embeddings=d["afm_E"], feature_bias=d["afm_w"][:, None],
                  bias=d["afm_w0"], attention_W=d["afm_attention_W"],
                  attention_b=d["afm_attention_b"], attention_p=d["afm_attention_p"],
                  prediction=d["afm_prediction"])
    loss = m.partial_fit({"X": d["afm_X"], "Y": d["afm_Y"][:, None]})
    assert np.isclose(loss, d["afm_loss"], rtol=RTOL), (loss, d["afm_loss"])


@pytest.mark.gpu
def test_gpu_dfm_partial_fit_returns_reference_loss():
    from hhfm_amd.DFM import DeepFM
    d = load()
    M, k = d["dfm_E"].shape
    m = DeepFM(int(d["n_user"]), int(d["n_item"]), M, 5, k, [32, 24], None, 0.01, 0,
               float(d["dfm_l2"]))
    m.set_weights(feature_embeddings=d["dfm_E"], feature_bias=d["dfm_w"][:, None],
                  concat_projection=d["dfm_concat_projection"],
                  concat_bias=d["dfm_concat_bias"],
                  **{f"layer_{i}": d[f"dfm_layer_{i}"] for i in range(2)},
                  **{f"bias_{i}": d[f"dfm_bias_{i}"] for i in range(2)})
    loss = m.partial_fit({"X": d["dfm_X"], "Y": d["dfm_Y"][:, None]})
    assert np.isclose(loss, d["dfm_loss"], rtol=RTOL), (loss, d["dfm_loss"])

