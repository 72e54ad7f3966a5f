"""The train / evaluate harness of the reference (the ``Train`` class copied
into every Newcode model file, e.g. FM.py:199-359), restated once.

Semantics kept exactly, including the reference's quirks (SURVEY.md §8a
H3-H5, Appendix 3-4, 6), because HR parity depends on them:
  * ``sample_negative`` (FM.py:284-294): one ``np.random.randint`` draw of
    the whole [rows, num] block, then row-major rejection re-draws (one
    scalar ``randint`` per retry) while the negative is in
    ``positive_feedback[(user, ctx...)]`` — same RNG stream as the reference;
    the membership test is vectorised, the re-draw order is not changed;
  * ``evaluate_TopK`` (FM.py:325-359): ``int(min(3000,len)/num)`` batches of
    ``num`` rows drawn WITH replacement, ``model.topk(rows, 20)`` and the
    metric walk over the 20 predictions in which a target that is a train
    positive of its key makes every non-hit a ``continue`` (:354-355) and a
    row whose walk runs out appends nothing;  "PRE" is 1/(rank+1) (:351);
  * ``evaluate_AUC`` (FM.py:296-324): label>0 rows, chunks of 600, 50
    negatives each, mean of strict ``pos > neg``; the HHFM variant
    (OurModel7.py:430-461) keeps all rows and returns after the first chunk.
The model is duck-typed: ``model.score_rows(X) -> float32 [B,1]`` (replaces
``sess.run(model.out | model.PositiveFeadback)``) and
``model.topk(A, tp) -> int [B,tp]`` item offsets.
"""
from __future__ import annotations

import math

import numpy as np


def partition_all(n, seq):
    """toolz.partition_all (the reference's batching helper)."""
    seq = list(seq)
    return [seq[i:i + n] for i in range(0, len(seq), n)]


class _PairSet:
    """Vectorised membership of (key, item) in positive_feedback."""

    def __init__(self, positive_feedback):
        self.pf = positive_feedback
        self.key_id = {}
        pairs = []
        for kid, (key, items) in enumerate(positive_feedback.items()):
            self.key_id[key] = kid
            for it in items:
                pairs.append((kid << 32) | int(it))
        self.pairs = np.unique(np.asarray(pairs, dtype=np.int64))

    def contains(self, keys, items):
        kid = np.fromiter((self.key_id.get(k, -1) for k in keys), dtype=np.int64, count=len(keys))
        code = (kid[:, None] << 32) | np.asarray(items, dtype=np.int64)
        hit = np.isin(code, self.pairs)
        hit &= kid[:, None] >= 0
        return hit


def row_keys(data):
    """tuple(user[[i for i in range(len(user)) if i != 1]]) per row
    (FM.py:291): every column except the item."""
    data = np.asarray(data)
    cols = [i for i in range(data.shape[1]) if i != 1]
    return [tuple(r) for r in data[:, cols].tolist()]


class Train(object):
    """Harness core; model-specific subclasses live next to each model."""

    eval_num = 300          # rows per topk call (DFM: 60, DFM.py:369)
    auc_first_chunk_only = False   # HHFM/CARS2 quirk (OurModel7.py:461)
    auc_label_filter = True        # FM/AFM/DFM keep label>0 rows (FM.py:298)
    method = "FM"

    def __init__(self, args=None, data=None, model=None):
        self.args = args
        if args is not None:
            self.batch_size = args.batch_size
            self.epoch = args.epoch
            self.verbose = getattr(args, "verbose", 0)
            self.keep = getattr(args, "keep", 1)
            self.TopK = args.TopK
        if data is not None:
            self.data = data
            self.n_user = data.n_user
            self.n_item = data.n_item
        self.model = model
        self._pairs = None
        self._pairs_src = None

    # -- H5 -----------------------------------------------------------------
    def _pair_index(self):
        pf = self.data.positive_feedback
        if self._pairs is None or self._pairs_src is not pf or \
                sum(len(v) for v in pf.values()) != self._pairs_n:
            self._pairs = _PairSet(pf)
            self._pairs_src = pf
            self._pairs_n = sum(len(v) for v in pf.values())
        return self._pairs

    def sample_negative(self, data, num=10):
        """FM.py:284-294 with the same np.random stream."""
        lo, hi = self.n_user, self.n_user + self.n_item
        samples = np.random.randint(lo, hi, size=(len(data), num))
        if len(data) == 0:
            return samples
        keys = row_keys(data)
        pf = self.data.positive_feedback
        bad = self._pair_index().contains(keys, samples)
        for i, j in np.argwhere(bad):      # row-major, like the nested loop
            key = keys[i]
            neg = samples[i, j]
            while neg in pf[key]:
                samples[i, j] = neg = np.random.randint(lo, hi)
        return samples

    # -- H4 -----------------------------------------------------------------
    def evaluate_AUC(self, data1):
        dat = data1.values
        if self.auc_label_filter:
            dat = dat[dat[:, 0] > 0]
        X = np.array(dat[:, 1:], dtype=np.int64)
        score = []
        for chunk in partition_all(600, range(len(X))):
            pos = X[chunk]
            negs = self.sample_negative(pos, 50)
            neg = np.repeat(pos[:, None, :], 50, axis=1).reshape(-1, pos.shape[1])
            neg[:, 1] = negs.reshape(-1)
            neg_score = np.asarray(self.model.score_rows(neg)).reshape(-1, 1)
            pos_out = np.asarray(self.model.score_rows(pos)).reshape(-1, 1)
            pos_score = np.repeat(pos_out, 50, axis=0)
            score.extend((pos_score > neg_score).reshape(-1).tolist())
            if self.auc_first_chunk_only:
                return np.mean(score)
        return np.mean(score)

    # -- H3 -----------------------------------------------------------------
    def evaluate_TopK(self, data1):
        size = np.min([3000, len(data1)])
        hits, ndcg, pre = [], [], []
        dat = data1.values
        num = self.eval_num
        pf = self.data.positive_feedback
        for _ in range(int(size / num)):
            feed = np.array(dat[:, 1:][np.random.randint(0, len(dat), num)], dtype=np.int64)
            prediction = np.asarray(self.model.topk(feed, 20)) + self.n_user
            for i, line in enumerate(feed):
                item = line[1]
                key = tuple(line[[c for c in range(len(line)) if c != 1]])
                positive = item in pf.get(key, ())
                n = 0
                for it in prediction[i]:
                    if n > self.TopK - 1:
                        hits.append(0); ndcg.append(0); pre.append(0)
                        break
                    elif it == item:
                        hits.append(1)
                        ndcg.append(np.log(2) / np.log(n + 2))
                        pre.append(1 / (n + 1))
                        break
                    elif positive:
                        continue
                    else:
                        n = n + 1
        return [np.average(hits), np.average(ndcg), np.average(pre)]

    def _log(self, line):
        print(line)


def hr_ndcg_pre_at(topk_items, targets, TopK, positive_mask):
    """Vector form of the evaluate_TopK walk for one batch (used to check the
    GPU top-K lists end to end): returns per-row (hit, ndcg, pre) or None for
    rows that append nothing."""
    out = []
    for pred, item, positive in zip(topk_items, targets, positive_mask):
        n = 0
        res = None
        for it in pred:
            if n > TopK - 1:
                res = (0, 0.0, 0.0)
                break
            elif it == item:
                res = (1, math.log(2) / math.log(n + 2), 1 / (n + 1))
                break
            elif positive:
                continue
            else:
                n += 1
        out.append(res)
    return out
