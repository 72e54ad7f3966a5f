"""AFM — drop-in for Newcode/AFM.py (AFM, Train, AFM_main).

Scoring runs on the gfx950 kernels of afm.hip (exact-fp32 MFMA):
  * ``score_rows`` / ``sess.run(model.out)`` -> hhfm_afm_forward (AFM.py:103-142)
  * ``topk(A, tp)`` -> hhfm_afm_catalog_topk (AFM.py:209-246)
  * ``partial_fit(data)`` -> hhfm_afm_train_step (AFM.py:144-156, 205-207)
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from . import NewLoadData as DATA
from . import harness, ops
from ._model import Fetch, Placeholder, ScoringModel

method = "AFM"


def parse_args(dataname, factor, TopK, argv=None):
    """Same flags and defaults as the reference (AFM.py:27-61)."""
    p = argparse.ArgumentParser(description="Run DeepFM.")
    p.add_argument("--path", nargs="?", default="../data/positive/")
    p.add_argument("--dataset", nargs="?", default=dataname)
    p.add_argument("--epoch", type=int, default=60)
    p.add_argument("--batch_size", type=int, default=5000)
    p.add_argument("--attention", type=int, default=1)
    p.add_argument("--hidden_factor", nargs="?", default="[%d,%d]" % (factor, factor))
    p.add_argument("--lamda_attention", type=float, default=100.0)
    p.add_argument("--keep", nargs="?", default="[1,1]")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--optimizer", nargs="?", default="AdagradOptimizer")
    p.add_argument("--verbose", type=int, default=10)
    p.add_argument("--batch_norm", type=int, default=0)
    p.add_argument("--decay", type=float, default=0.999)
    p.add_argument("--activation", nargs="?", default="relu")
    p.add_argument("--TopK", type=int, default=TopK)
    p.add_argument("--Result", type=int, default=0)
    p.add_argument("--result_file", default="../result.txt")
    return p.parse_args(argv)


class AFM(ScoringModel):
    def __init__(self, n_user, n_item, features_M, attention, hidden_factor,
                 activation_function, learning_rate, lamda_attention, keep, optimizer_type,
                 decay, valid_dimension, random_seed=2016, device=None,
                 table_dtype=torch.float32):
        self.n_user = n_user
        self.n_item = n_item
        self.learning_rate = learning_rate
        self.attention = attention
        self.hidden_factor = list(hidden_factor)
        self.activation_function = activation_function
        self.features_M = features_M
        self.valid_dimension = valid_dimension
        self.lamda_attention = lamda_attention
        self.keep = keep
        self.random_seed = random_seed
        self.optimizer_type = optimizer_type
        self.decay = decay
        self.u_f = valid_dimension - 1
        if not attention:
            raise NotImplementedError("the kernels implement attention=1 (the reference default)")
        self._setup_device(device, table_dtype)
        self._init_graph()

    def _init_graph(self):
        self.train_features = Placeholder("train_features_afm")
        self.train_labels = Placeholder("train_labels_afm")
        self.dropout_keep = Placeholder("dropout_keep_afm")
        self.train_phase = Placeholder("train_phase_afm")
        self.out = Fetch("out_afm")
        self.weights = self._initialize_weights()

    def _initialize_weights(self):
        """AFM.py:173-201 (attention weights glorot-normal from a seeded RNG)."""
        rng = np.random.default_rng(self.random_seed)
        A, k = self.hidden_factor
        glorot = np.sqrt(2.0 / (A + k))
        t = lambda a: torch.from_numpy(np.asarray(a, np.float32)).to(self.device)  # noqa: E731
        return {
            "feature_embeddings": self._normal((self.features_M, k), 0.01, self.random_seed),
            "feature_bias": torch.zeros(self.features_M, 1, device=self.device),
            "bias": torch.zeros((), device=self.device),
            "attention_W": t(rng.normal(0, glorot, (k, A))),
            "attention_b": t(rng.normal(0, glorot, (1, A))),
            "attention_p": t(rng.normal(0, 1, A)),
            "prediction": torch.ones(k, 1, device=self.device),
        }

    def _att(self):
        W = self.weights
        return (W["attention_W"].t().contiguous(), W["attention_b"].reshape(-1).contiguous(),
                W["attention_p"].reshape(-1).contiguous(), W["prediction"].reshape(-1).contiguous())

    def score_rows(self, X) -> np.ndarray:
        idx = self._idx(X)
        Wt, b, p, P = self._att()
        out = ops.afm_forward(idx, self.table, self.weights["feature_bias"].reshape(-1),
                              float(self.weights["bias"]), Wt, b, p, P)
        return self._np_out(out)

    def catalog_topk(self, q, begin, count, K):
        """Top-K of items [begin, begin+count) by the attention score of
        AFM.py:209-246 -> (scores, global item offsets) device tensors [B, K]."""
        Wt, b, p, P = self._att()
        return ops.afm_catalog_topk(q, self.table, self.weights["feature_bias"].reshape(-1),
                                    Wt, b, p, P, self.n_user + begin, count, int(K), begin)

    def topk(self, A, tp):
        _, ids = self.catalog_topk(self._idx(A), 0, self.n_item, tp)
        return ids.cpu().numpy()

    def _run_fetch(self, fetch, feed):
        if fetch is self.out:
            return self.score_rows(feed[self.train_features])
        return super()._run_fetch(fetch, feed)

    def partial_fit(self, data):
        """AFM.py:205-207 -> hhfm_afm_train_step (loss, then the update)."""
        from .training import afm_partial_fit
        return afm_partial_fit(self, data)


class Train(harness.Train):
    method = "AFM"

    def __init__(self, args, data=None, model=None):
        data = data if data is not None else DATA.LoadData(args.path, args.dataset)
        super().__init__(args, data=data)
        self.valid_dimension = self.data.Train_data.shape[1] - 1
        hf = [int(x) for x in args.hidden_factor.strip("[]").split(",")]
        keep = [float(x) for x in args.keep.strip("[]").split(",")]
        if args.verbose > 0:
            print("AFM: dataset=%s, factors=%s, #epoch=%d, batch=%d, lr=%.4f, "
                  "lamda_attention=%.1e, keep=%s, optimizer=%s, batch_norm=%d"
                  % (args.dataset, args.hidden_factor, args.epoch, args.batch_size, args.lr,
                     args.lamda_attention, args.keep, args.optimizer, args.batch_norm))
        self.model = model if model is not None else AFM(
            self.n_user, self.n_item, self.data.features_M, args.attention, hf, None, args.lr,
            args.lamda_attention, keep, args.optimizer, args.decay, self.valid_dimension)

    def train(self):
        from .training import run_training
        return run_training(self, negatives=2, neg_label=-1, plateau=-0.01, epoch_cap=None)


def AFM_main(dataname, factor, Topk, argv=None):
    args = parse_args(dataname, factor, Topk, argv)
    session = Train(args)
    session.train()
    return session
