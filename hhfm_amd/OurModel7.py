"""HHFM (OurModel7) — drop-in for Newcode/OurModel7.py (OUR, Train, M7_main).

Sum pooling everywhere (the committed setting, OurModel7.py:14-19), so the
pairwise-product branches of the reference graph are dead code and
  h = E[user] + Σ E[ctx] (+ Σ E[time]),   score = h · E[item]   (no bias).
Scoring runs on the gfx950 kernels:
  * ``score_rows`` / ``sess.run(model.PositiveFeadback)`` -> hhfm_hybrid_score_rows
    (OurModel7.py:105-171)
  * ``topk(A, tp)`` -> hhfm_catalog_topk, HHFM_MODE_HHFM (OurModel7.py:229-307)
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from . import NewLoadData as DATA
from . import harness, ops
from ._model import Fetch, Placeholder, ScoringModel, rows_from

method = "M7"


def parse_args(dataname, factor, Topk, argv=None):
    """Same flags and defaults as the reference (OurModel7.py:23-49)."""
    p = argparse.ArgumentParser(description="Run .")
    p.add_argument("--path", nargs="?", default="../data/positive/")
    p.add_argument("--dataset", nargs="?", default=dataname)
    p.add_argument("--epoch", type=int, default=60)
    p.add_argument("--batch_size", type=int, default=5000)
    p.add_argument("--hidden_factor", type=int, default=factor)
    p.add_argument("--lamda", type=float, default=0.01)
    p.add_argument("--keep", type=float, default=1)
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--optimizer", nargs="?", default="AdagradOptimizer")
    p.add_argument("--batch_norm", type=int, default=0)
    p.add_argument("--TopK", type=int, default=Topk)
    p.add_argument("--Result", type=int, default=0)
    p.add_argument("--result_file", default="../result.txt")
    return p.parse_args(argv)


class OUR(ScoringModel):
    def __init__(self, feature_dimension, time_dimension, features_M, n_user, n_item,
                 hidden_factor, learning_rate, lamda_bilinear, optimizer_type, context, time,
                 random_seed=2016, device=None, table_dtype=torch.float32):
        self.feature_dimension = feature_dimension
        self.time_dimension = time_dimension
        self.n_user = n_user
        self.n_item = n_item
        self.learning_rate = learning_rate
        self.hidden_factor = hidden_factor
        self.features_M = features_M
        self.lamda_bilinear = lamda_bilinear
        self.optimizer_type = optimizer_type
        self.context = context
        self.time = time
        self.random_seed = random_seed
        if not context and time:
            # the reference never sets self.num on this branch (OurModel7.py:96-99)
            # and its graph construction fails at :159
            raise AttributeError("'OUR' object has no attribute 'num'")
        if not context and not time:
            raise UnboundLocalError("OUR needs context and/or time fields")
        self.num = 3 if (context and time) else 2
        self._setup_device(device, table_dtype)
        self._init_graph()

    def _init_graph(self):
        self.Pos = Placeholder("Pos")
        self.Fea = Placeholder("Fea") if self.context else None
        self.Tim = Placeholder("Tim") if self.time else None
        self.Neg = Placeholder("Neg")
        self.PositiveFeadback = Fetch("PositiveFeadback")
        self.weights = self._initialize_weights()

    def _initialize_weights(self):
        """OurModel7.py:207-216 (feature_bias/wgt are unused by the score)."""
        return {
            "feature_embeddings": self._normal((self.features_M, self.hidden_factor), 0.01,
                                               self.random_seed),
            "feature_bias": torch.zeros(self.features_M, 1, device=self.device),
        }

    def _ranges(self, ncols):
        """Column split of a full row (OurModel7.py:236-242, 374-385)."""
        td = self.time_dimension if self.time else 0
        ctx = (2, ncols - td) if self.context else (0, 0)
        tim = (ncols - td, ncols) if self.time else (0, 0)
        if ctx[1] <= ctx[0]:
            ctx = (0, 0)
        return ctx, tim

    def score_rows(self, X) -> np.ndarray:
        """PositiveFeadback for full rows [user, item, ctx..., time...] -> [B,1]."""
        idx = self._idx(X)
        ctx, tim = self._ranges(idx.shape[1])
        out = ops.hybrid_score_rows(idx, self.table, 0, 1, ctx, tim)
        return self._np_out(out)

    def catalog_topk(self, q, begin, count, K):
        """Top-K of items [begin, begin+count) by h·item (OurModel7.py:229-295)
        -> (scores, global item offsets) device tensors [B, K]."""
        ctx, tim = self._ranges(q.shape[1])
        return ops.catalog_topk(q, self.table, ops.MODE_HHFM, int(K), self.n_user + begin,
                                count, begin, None, 0, ctx, tim)

    def topk(self, A, tp):
        _, ids = self.catalog_topk(self._idx(A), 0, self.n_item, tp)
        return ids.cpu().numpy()

    def _run_fetch(self, fetch, feed):
        if fetch is self.PositiveFeadback:
            return self.score_rows(rows_from(feed, self.Pos, self.Fea, self.Tim))
        return super()._run_fetch(fetch, feed)

    def partial_fit(self, data):
        from .training import hhfm_partial_fit
        return hhfm_partial_fit(self, data)


class Train(harness.Train):
    method = "M7"
    auc_first_chunk_only = True      # OurModel7.py:461 (returns inside the loop)
    auc_label_filter = False         # OurModel7.py:431

    def __init__(self, args, data=None, model=None):
        data = data if data is not None else DATA.LoadData(args.path, args.dataset)
        super().__init__(args, data=data)
        self.features_M = self.data.features_M
        self.valid_dimension = self.data.Train_data.shape[1] - 1
        print("OurModel: dataset=%s, factors=%d, #epoch=%d, batch=%d, lr=%.4f, lambda=%.1e, "
              "keep=%.2f, optimizer=%s, batch_norm=%d"
              % (args.dataset, args.hidden_factor, args.epoch, args.batch_size, args.lr,
                 args.lamda, args.keep, args.optimizer, args.batch_norm))
        # dataset switch, OurModel7.py:326-346
        self.context, self.time, self.time_dimension = True, False, 0
        if args.dataset == "resturant":
            self.time, self.time_dimension = True, 5
        elif args.dataset == "jiaju":
            self.time, self.time_dimension = True, 3
        self.feature_dimension = self.valid_dimension - 2 - self.time_dimension
        self.model = model if model is not None else OUR(
            self.feature_dimension, self.time_dimension, self.features_M, self.n_user,
            self.n_item, args.hidden_factor, args.lr, args.lamda, args.optimizer,
            self.context, self.time)

    def train(self):
        from .training import run_training_hhfm
        return run_training_hhfm(self)


def M7_main(dataname, factor, Topk, argv=None):
    args = parse_args(dataname, factor, Topk, argv)
    session = Train(args)
    session.train()
    return session
