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

encoder="native" (default): the tokenizer, the id map and the split walk run
in C++ (``hhfm_libfm_encode``, ``hhfm_loader_split`` in libhhfm.so — host
code); encoder="python": pandas + one vectorised
dictionary pass.  Both reproduce the reference's fields on its fixtures
(tests/test_loaddata.py).  The shuffle stays numpy's (same stream).
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import pandas as pd


class LoadData(object):
    def __init__(self, path, dataset, ratio=0.9, encoder="native"):
        self.path = path + dataset + "/"
        self.trainfile = self.path + dataset + ".libfm"
        if encoder == "native":
            self._encode_native()
        elif encoder == "python":
            self._encode_python()
        else:
            raise ValueError("encoder must be 'native' or 'python'")
        ncol = self.Total_data.shape[1]

        data = self.Total_data.values
        np.random.shuffle(data)
        test_size = int(len(data) * (1 - ratio))
        self.positive_feedback = defaultdict(set)
        self.train_set = defaultdict(set)
        key_cols = [i for i in range(1, ncol) if i != 2]
        if encoder == "native":
            from ._native import native
            d64 = np.ascontiguousarray(data, dtype=np.int64)
            is_test = np.zeros(len(data), dtype=np.uint8)
            native().loader_split(d64.ctypes.data, len(d64), ncol, 2, test_size,
                                  is_test.ctypes.data)
            is_test = is_test.astype(bool)
            train_rows = np.flatnonzero(~is_test)
            keys = [tuple(r) for r in data[train_rows][:, key_cols].tolist()]
            items = data[train_rows, 2].tolist()
            users = data[train_rows, 1].tolist()
            for key, it, u in zip(keys, items, users):
                self.positive_feedback[key].add(it)
                self.train_set[u].add(it)
        else:
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

    @staticmethod
    def _columns(ncol):
        return ["label", "user", "item"] + ["feature" + str(i - 2) for i in range(3, ncol)]

    def _encode_python(self):
        self.Total_data = pd.read_csv(self.trainfile, sep=" ", header=None)
        ncol = self.Total_data.shape[1]
        self.Total_data.columns = self._columns(ncol)
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

    def _encode_native(self):
        from ._native import native
        with open(self.trainfile, "rb") as f:
            raw = f.read()
        first = next((ln for ln in raw.split(b"\n", 64) if ln.strip(b"\r")), b"")
        ncol = len(first.rstrip(b"\r").split(b" "))
        cap = raw.count(b"\n") + 1
        labels = np.empty(cap, dtype=np.float64)
        ids = np.empty((cap, max(ncol - 1, 1)), dtype=np.int64)
        distinct = np.empty(max(ncol - 1, 1), dtype=np.int64)
        rows, fm = native().libfm_encode(raw, ncol, cap, labels.ctypes.data, ids.ctypes.data,
                                         distinct.ctypes.data)
        lab = labels[:rows]
        # read_csv's dtype for the label column: int64 when every value is integral
        if np.all(np.isfinite(lab)) and np.array_equal(lab, np.round(lab)):
            lab = lab.astype(np.int64)
        cols = self._columns(ncol)
        self.Total_data = pd.DataFrame(ids[:rows], columns=cols[1:])
        self.Total_data.insert(0, "label", lab)
        self.n_user = int(distinct[0])
        self.n_item = int(distinct[1])
        self.features_M = int(fm)
