"""LoadData — the libfm loader of the reference (Newcode/NewLoadData.py:6-62),
restated with the same public surface and the same results for the same
``np.random`` state.

Behaviour kept:
  * every token of columns 1.. is mapped to ONE global id, assigned in
    column-major first-occurrence order (all user tokens, then items, then
    each context column; NewLoadData.py:29-34) — identical tokens in
    different columns share one id;
  * ``n_user``/``n_item`` = distinct user / item tokens (:22-23);
  * rows are shuffled with ``np.random.shuffle`` (:39); a row goes to Test iff
    its (user, ctx...) key is unseen and fewer than int(0.1*rows) rows went to
    Test so far (:48-54), otherwise to Train and ``positive_feedback[key]``
    (:55-58).
The per-cell ``applymap`` is replaced by one vectorised dictionary pass.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import pandas as pd


class LoadData(object):
    def __init__(self, path, dataset, ratio=0.9):
        self.path = path + dataset + "/"
        self.trainfile = self.path + dataset + ".libfm"
        self.Total_data = pd.read_csv(self.trainfile, sep=" ", header=None)
        ncol = self.Total_data.shape[1]
        self.Total_data.columns = ["label", "user", "item"] + \
            ["feature" + str(i - 2) for i in range(3, ncol)]
        self.n_user = len(self.Total_data["user"].value_counts())
        self.n_item = len(self.Total_data["item"].value_counts())

        # column-major first-occurrence id assignment over columns 1..
        tokens = self.Total_data.values[:, 1:].T.reshape([-1])
        ids = {}
        for tok in tokens:
            if tok not in ids:
                ids[tok] = len(ids)
        mapped = np.fromiter((ids[t] for t in tokens), dtype=np.int64, count=len(tokens))
        mapped = mapped.reshape(ncol - 1, -1).T
        for c, col in enumerate(self.Total_data.columns[1:]):
            self.Total_data[col] = mapped[:, c]
        self.features_M = len(ids)

        data = self.Total_data.values
        np.random.shuffle(data)
        test_size = int(len(data) * (1 - ratio))
        self.positive_feedback = defaultdict(set)
        self.train_set = defaultdict(set)
        key_cols = [i for i in range(1, ncol) if i != 2]
        keys = [tuple(r) for r in data[:, key_cols].tolist()]
        items = data[:, 2].tolist()
        users = data[:, 1].tolist()
        seen = set()
        is_test = np.zeros(len(data), dtype=bool)
        n_test = 0
        for r, key in enumerate(keys):
            if key not in seen and n_test < test_size:
                seen.add(key)
                is_test[r] = True
                n_test += 1
            else:
                self.positive_feedback[key].add(items[r])
                self.train_set[users[r]].add(items[r])
        self.Train_data = pd.DataFrame(data[~is_test])
        self.Test_data = pd.DataFrame(data[is_test])
        self.Train_data.columns = self.Total_data.columns
        self.Test_data.columns = self.Total_data.columns
