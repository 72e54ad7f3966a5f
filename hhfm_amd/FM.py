"""FM — drop-in for Newcode/FM.py (model class, Train harness, FM_main).

Scoring runs on the gfx950 kernels:
  * ``score_rows`` / ``sess.run(model.out)`` -> hhfm_fm_score_rows (FM.py:99-120)
  * ``topk(A, tp)`` -> hhfm_catalog_topk, HHFM_MODE_FM (FM.py:172-198)
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from . import NewLoadData as DATA
from . import harness, ops
from ._model import Fetch, Placeholder, ScoringModel

method = "FM"


def parse_args(dataname, factor, TopK, argv=None):
    """Same flags and defaults as the reference (FM.py:24-57)."""
    p = argparse.ArgumentParser(description="Run FM.")
    p.add_argument("--process", nargs="?", default="train")
    p.add_argument("--mla", type=int, default=0)
    p.add_argument("--path", nargs="?", default="../data/positive/")
    p.add_argument("--dataset", nargs="?", default=dataname)
    p.add_argument("--epoch", type=int, default=60)
    p.add_argument("--batch_size", type=int, default=5000)
    p.add_argument("--hidden_factor", type=int, default=factor)
    p.add_argument("--lamda", type=float, default=0.1)
    p.add_argument("--keep", type=float, default=1)
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--optimizer", nargs="?", default="AdagradOptimizer")
    p.add_argument("--verbose", type=int, default=10)
    p.add_argument("--batch_norm", type=int, default=0)
    p.add_argument("--TopK", type=int, default=TopK)
    p.add_argument("--Result", type=int, default=0)
    p.add_argument("--result_file", default="../result.txt")
    return p.parse_args(argv)


class FM(ScoringModel):
    def __init__(self, valid_dimension, features_M, n_user, n_item, hidden_factor,
                 learning_rate, lamda_bilinear, keep, optimizer_type, batch_norm,
                 verbose, random_seed=2016, device=None, table_dtype=torch.float32):
        self.valid_dimension = valid_dimension
        self.n_user = n_user
        self.n_item = n_item
        self.learning_rate = learning_rate
        self.hidden_factor = hidden_factor
        self.features_M = features_M
        self.lamda_bilinear = lamda_bilinear
        self.keep = keep
        self.random_seed = random_seed
        self.optimizer_type = optimizer_type
        self.batch_norm = batch_norm
        self.verbose = verbose
        self.train_rmse, self.valid_rmse, self.test_rmse = [], [], []
        if batch_norm:
            raise NotImplementedError("batch_norm=1 is not part of the scoring path "
                                      "(the reference runs with batch_norm=0, FM.py:50)")
        self._setup_device(device, table_dtype)
        self._init_graph()

    def _init_graph(self):
        # placeholders / fetches a reference caller may use (FM.py:89-120)
        self.train_features = Placeholder("train_features_fm")
        self.train_labels = Placeholder("train_labels_fm")
        self.dropout_keep = Placeholder("dropout_keep_fm")
        self.train_phase = Placeholder("train_phase_fm")
        self.out = Fetch("out")
        self.weights = self._initialize_weights()

    def _initialize_weights(self):
        """FM.py:150-158: E ~ N(0, 0.01), feature_bias = 0, bias = 0."""
        return {
            "feature_embeddings": self._normal((self.features_M, self.hidden_factor), 0.01,
                                               self.random_seed),
            "feature_bias": torch.zeros(self.features_M, 1, device=self.device),
            "bias": torch.zeros((), device=self.device),
        }

    # -- scoring ------------------------------------------------------------------
    def score_rows(self, X) -> np.ndarray:
        """FM.out for full rows [user, item, ctx...] -> float32 [B, 1]."""
        idx = self._idx(X)
        w = self.weights["feature_bias"].reshape(-1)
        out = ops.fm_score_rows(idx, self.table, w, float(self.weights["bias"]))
        return self._np_out(out)

    def catalog_topk(self, q, begin, count, K):
        """Top-K of items [begin, begin+count) by (u+f)·(i+f) + w_i (FM.py:172-185)
        -> (scores, global item offsets) device tensors [B, K]."""
        ncols = q.shape[1]
        return ops.catalog_topk(q, self.table, ops.MODE_FM, int(K), self.n_user + begin, count,
                                begin, self.weights["feature_bias"].reshape(-1), 0,
                                (2, ncols) if ncols > 2 else (0, 0), (0, 0))

    def topk(self, A, tp):
        """Top-``tp`` item offsets in [0, n_item) by (u+f)·(i+f) + w_i."""
        _, ids = self.catalog_topk(self._idx(A), 0, self.n_item, tp)
        return ids.cpu().numpy()

    def _run_fetch(self, fetch, feed):
        if fetch is self.out:
            return self.score_rows(feed[self.train_features])
        return super()._run_fetch(fetch, feed)

    def partial_fit(self, data):
        from .training import fm_partial_fit
        return fm_partial_fit(self, data)


class Train(harness.Train):
    method = "FM"

    def __init__(self, args, data=None, model=None):
        data = data if data is not None else DATA.LoadData(args.path, args.dataset)
        super().__init__(args, data=data)
        self.valid_dimension = self.data.Train_data.shape[1] - 1
        if args.verbose > 0:
            print("FM: dataset=%s, factors=%d, #epoch=%d, batch=%d, lr=%.4f, lambda=%.1e, "
                  "keep=%.2f, optimizer=%s, batch_norm=%d"
                  % (args.dataset, args.hidden_factor, args.epoch, args.batch_size, args.lr,
                     args.lamda, args.keep, args.optimizer, args.batch_norm))
        self.model = model if model is not None else FM(
            self.valid_dimension, self.data.features_M, self.n_user, self.n_item,
            args.hidden_factor, args.lr, args.lamda, args.keep, args.optimizer,
            args.batch_norm, args.verbose)

    def train(self):
        from .training import run_training
        return run_training(self, negatives=2, neg_label=0)


def FM_main(dataname, factor, Topk, argv=None):
    args = parse_args(dataname, factor, Topk, argv)
    session = Train(args)
    session.train()
    return session
