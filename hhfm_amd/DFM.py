"""DeepFM — drop-in for Newcode/DFM.py (DeepFM, Train, DFM_main).

Scoring runs on the gfx950 kernels of mlp_gemm.hip:
  * ``score_rows`` / ``sess.run(model.out)`` -> hhfm_dfm_forward (DFM.py:104-137):
    FM part + an LDS-tiled MFMA GEMM chain whose first layer gathers the
    field embeddings straight from the table;
  * ``topk(A, tp)`` -> hhfm_dfm_catalog_topk (DFM.py:219-231).
``mlp_dtype=torch.float32`` (default, reference numerics: exact-fp32 MFMA)
or ``torch.bfloat16`` (bf16 MFMA, fp32 accumulation).
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from . import NewLoadData as DATA
from . import harness, ops
from ._model import Fetch, Placeholder, ScoringModel

method = "DFM"


def parse_args(dataname, factor, Topk, argv=None):
    """Same flags and defaults as the reference (DFM.py:19-47)."""
    p = argparse.ArgumentParser(description="Run .")
    p.add_argument("--path", nargs="?", default="../data/positive/")
    p.add_argument("--dataset", nargs="?", default=dataname)
    p.add_argument("--epoch", type=int, default=60)
    p.add_argument("--batch_size", type=int, default=5000)
    p.add_argument("--hidden_factor", type=int, default=factor)
    p.add_argument("--lamda", type=float, default=0.01)
    p.add_argument("--keep", type=float, default=1)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--optimizer", nargs="?", default="AdagradOptimizer")
    p.add_argument("--verbose", type=int, default=10)
    p.add_argument("--batch_norm", type=int, default=0)
    p.add_argument("--TopK", type=int, default=Topk)
    p.add_argument("--Result", type=int, default=0)
    p.add_argument("--result_file", default="../result.txt")
    return p.parse_args(argv)


class DeepFM(ScoringModel):
    def __init__(self, n_user, n_item, feature_size, field_size, embedding_size, deep_layers,
                 deep_layers_activation=None, learning_rate=0.01, verbose=True, l2_reg=0.0,
                 random_seed=2016, use_fm=True, use_deep=True, loss_type="mse", device=None,
                 table_dtype=torch.float32, mlp_dtype=torch.float32):
        assert use_fm or use_deep
        assert loss_type in ["logloss", "mse"], \
            "loss_type can be either 'logloss' for classification task or 'mse' for regression task"
        if not (use_fm and use_deep and loss_type == "mse"):
            raise NotImplementedError("the scoring kernels implement the reference setting "
                                      "use_fm=use_deep=True, loss_type='mse' (DFM.py:255-257)")
        self.n_user = n_user
        self.n_item = n_item
        self.feature_size = feature_size
        self.features_M = feature_size
        self.field_size = field_size
        self.embedding_size = embedding_size
        self.deep_layers = list(deep_layers)
        self.deep_layers_activation = deep_layers_activation
        self.use_fm, self.use_deep = use_fm, use_deep
        self.l2_reg = l2_reg
        self.learning_rate = learning_rate
        self.verbose = verbose
        self.random_seed = random_seed
        self.loss_type = loss_type
        if mlp_dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("mlp_dtype must be torch.float32 or torch.bfloat16")
        self.mlp_dtype = mlp_dtype
        self._setup_device(device, table_dtype)
        self._init_graph()

    def _init_graph(self):
        self.feat_index = Placeholder("feat_index")
        self.label = Placeholder("label")
        self.dropout_keep_fm = Placeholder("dropout_keep_fm")
        self.dropout_keep_deep = Placeholder("dropout_keep_deep")
        self.train_phase = Placeholder("train_phase")
        self.out = Fetch("out")
        self.weights = self._initialize_weights()
        self._prep = None

    def _initialize_weights(self):
        """DFM.py:171-211 (glorot-normal layers from a seeded numpy RNG)."""
        rng = np.random.default_rng(self.random_seed)
        M, k, F = self.feature_size, self.embedding_size, self.field_size
        W = {"feature_embeddings": self._normal((M, k), 0.01, self.random_seed),
             "feature_bias": torch.rand(M, 1, generator=self._gen(self.random_seed + 1),
                                        device=self.device)}
        fan_in = F * k
        for i, n in enumerate(self.deep_layers):
            glorot = np.sqrt(2.0 / (fan_in + n))
            W[f"layer_{i}"] = torch.from_numpy(
                rng.normal(0, glorot, (fan_in, n)).astype(np.float32)).to(self.device)
            W[f"bias_{i}"] = torch.from_numpy(
                rng.normal(0, glorot, (1, n)).astype(np.float32)).to(self.device)
            fan_in = n
        inp = F + k + self.deep_layers[-1]
        glorot = np.sqrt(2.0 / (inp + 1))
        W["concat_projection"] = torch.from_numpy(
            rng.normal(0, glorot, (inp, 1)).astype(np.float32)).to(self.device)
        W["concat_bias"] = torch.tensor(0.01, device=self.device)
        return W

    def set_weights(self, **arrays):
        super().set_weights(**arrays)
        self._prep = None

    def _prepared(self):
        key = tuple(id(self.weights[f"layer_{i}"]) for i in range(len(self.deep_layers)))
        if self._prep is None or self._prep[0] != key:
            L = len(self.deep_layers)
            Wt, bs, dims = ops.dfm_prepare_weights(
                [self.weights[f"layer_{i}"] for i in range(L)],
                [self.weights[f"bias_{i}"] for i in range(L)], self.mlp_dtype,
                self.field_size, self.embedding_size)
            Wp = self.weights["concat_projection"].reshape(-1).float().contiguous()
            self._prep = (key, Wt, bs, dims, Wp, float(self.weights["concat_bias"]))
        return self._prep[1:]

    def score_rows(self, X) -> np.ndarray:
        idx = self._idx(X)
        Wt, bs, dims, Wp, bp = self._prepared()
        out = ops.dfm_forward(idx, self.table, self.weights["feature_bias"].reshape(-1), Wt, bs,
                              dims, self.mlp_dtype, Wp, bp)
        return self._np_out(out)

    def catalog_topk(self, q, begin, count, K):
        """Top-K of items [begin, begin+count) by the DeepFM score of
        DFM.py:219-231 -> (scores, global item offsets) device tensors [B, K]."""
        Wt, bs, dims, Wp, bp = self._prepared()
        return ops.dfm_catalog_topk(q, self.table, self.weights["feature_bias"].reshape(-1),
                                    Wt, bs, dims, Wp, bp, 1, self.n_user + begin, count, int(K),
                                    begin)

    def topk(self, A, tp):
        _, ids = self.catalog_topk(self._idx(A), 0, self.n_item, tp)
        return ids.cpu().numpy()

    def _run_fetch(self, fetch, feed):
        if fetch is self.out:
            return self.score_rows(feed[self.feat_index])
        return super()._run_fetch(fetch, feed)

    def partial_fit(self, data):
        """DFM.py:214-217 on the gfx950 train-step kernels (fp32)."""
        from .training import dfm_partial_fit
        return dfm_partial_fit(self, data)


class Train(harness.Train):
    method = "DFM"
    eval_num = 60        # DFM.py:369

    def __init__(self, args, data=None, model=None):
        data = data if data is not None else DATA.LoadData(args.path, args.dataset)
        super().__init__(args, data=data)
        if args.verbose > 0:
            print("DFM: dataset=%s, factors=%d, #epoch=%d, batch=%d, lr=%.4f, lambda=%.1e, "
                  "keep=%.2f, optimizer=%s, batch_norm=%d"
                  % (args.dataset, args.hidden_factor, args.epoch, args.batch_size, args.lr,
                     args.lamda, args.keep, args.optimizer, args.batch_norm))
        self.model = model if model is not None else DeepFM(
            self.n_user, self.n_item, self.data.features_M, self.data.Train_data.shape[1] - 1,
            args.hidden_factor, [150, 200, 150], None, args.lr, args.verbose, args.lamda)

    def train(self):
        from .training import run_training
        return run_training(self, negatives=2, neg_label=-1, epoch_cap=None)


def DFM_main(dataname, factor, Topk, argv=None):
    args = parse_args(dataname, factor, Topk, argv)
    session = Train(args)
    session.train()
    return session
