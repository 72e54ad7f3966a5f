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

With a model on the GPU (``model.device`` a cuda device) the per-element
work runs on the device: ``sample_negative`` as a
whole through ``hhfm_sample_negative`` (numpy's MT19937 stream generated on
the device, masked bounded draws, membership and the row-major re-draws;
the host's RandomState resumes from the state it returns),
evaluate_TopK's target test through ``hhfm_pf_contains`` (positive_feedback
as sorted key / (key, item) code arrays, ``DevicePairSet``) and the metric
walk through ``hhfm_topk_walk``.  The walk's ranks are turned into the
reference's float64 values on the host, so the results are identical to
the host path (tests/test_gpu_harness.py).
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


# the device sampler's re-draw membership test: per-key bitmaps (True) or the
# binary searches over the sorted codes (False: the workspace without bitmaps);
# identical results — the switch exists for tests
SAMPLER_BITMAPS = True


class DevicePairSet:
    """positive_feedback as the two sorted device arrays hhfm_pf_contains
    searches: distinct keys [nkeys, key_cols] int32 in lexicographic order,
    and (key rank << 32 | item) int64 codes, sorted."""

    def __init__(self, positive_feedback, key_cols, device):
        import torch
        keys = list(positive_feedback.keys())
        K = np.asarray(keys, dtype=np.int64).reshape(len(keys), key_cols)
        order = np.lexsort(K.T[::-1]) if len(keys) else np.zeros(0, np.int64)
        lens = np.fromiter((len(positive_feedback[keys[i]]) for i in order), dtype=np.int64,
                           count=len(order))
        items = np.fromiter((it for i in order for it in positive_feedback[keys[i]]),
                            dtype=np.int64, count=int(lens.sum()))
        codes = np.sort((np.repeat(np.arange(len(order), dtype=np.int64), lens) << 32) | items)
        self.key_cols = key_cols
        self.n = len(keys)
        self.keys = torch.from_numpy(np.ascontiguousarray(K[order], dtype=np.int32)).to(device)
        self.codes = torch.from_numpy(codes).to(device)
        self.device = device

    def contains(self, rows, cand=None):
        """rows int [B, key_cols+1] (item in column 1); cand int [B, num] or
        None (the rows' own items) -> numpy bool [B, num] / [B]."""
        import torch
        from . import ops
        B = len(rows)
        if self.n == 0 or B == 0:
            return np.zeros((B,) if cand is None else (B, np.shape(cand)[1]), dtype=bool)
        r = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.int32)).to(self.device)
        c = None if cand is None else \
            torch.from_numpy(np.ascontiguousarray(cand, dtype=np.int32)).to(self.device)
        return ops.pf_contains(self.keys, self.codes, r, 1, c).cpu().numpy().astype(bool)


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
        self._dpairs = None

    # -- H5 -----------------------------------------------------------------
    def _pair_index(self):
        pf = self.data.positive_feedback
        if self._pairs is None or self._pairs_src is not pf or \
                sum(len(v) for v in pf.values()) != self._pairs_n:
            self._pairs = _PairSet(pf)
            self._pairs_src = pf
            self._pairs_n = sum(len(v) for v in pf.values())
        return self._pairs

    def _device(self):
        """The model's cuda device, or None (host harness)."""
        dev = getattr(self.model, "device", None)
        if dev is None:
            return None
        import torch
        dev = torch.device(dev)
        return dev if dev.type == "cuda" else None

    def _device_pairs(self, dev, key_cols):
        pf = self.data.positive_feedback
        n = sum(len(v) for v in pf.values())
        d = self._dpairs
        if d is None or d[0] is not pf or d[1] != n or d[2].device != dev or \
                d[2].key_cols != key_cols:
            self._dpairs = d = (pf, n, DevicePairSet(pf, key_cols, dev))
        return d[2]

    def sample_negative(self, data, num=10):
        """FM.py:284-294 with the same np.random stream.  With a GPU model the
        whole call — block draw, membership, re-draws — runs on the device
        on numpy's own MT19937 stream (hhfm_sample_negative), and the global
        RandomState continues exactly where the reference's would."""
        lo, hi = self.n_user, self.n_user + self.n_item
        dev = self._device()
        if dev is not None and len(data) > 0:
            return self._device_sample_negative(dev, np.asarray(data), num, lo, hi)
        samples = np.random.randint(lo, hi, size=(len(data), num))
        if len(data) == 0:
            return samples
        pf = self.data.positive_feedback
        keys = row_keys(data)
        bad = self._pair_index().contains(keys, samples)
        for i, j in np.argwhere(bad):      # row-major, like the nested loop
            key = keys[i]
            neg = samples[i, j]
            while neg in pf[key]:
                samples[i, j] = neg = np.random.randint(lo, hi)
        return samples

    def _device_sample_negative(self, dev, data, num, lo, hi):
        """hhfm_sample_negative: the legacy RandomState's (key, pos) in, the
        samples and the state after the call's last word out."""
        import torch
        from . import ops
        from ._native import native
        st = np.random.get_state()
        if st[0] != "MT19937":
            raise ValueError(f"np.random state {st[0]!r}: the device sampler follows MT19937")
        state = np.empty(625, np.uint32)
        state[:624] = st[1]
        state[624] = st[2]
        B, ncols = data.shape
        pairs = self._device_pairs(dev, ncols - 1)
        nat = native()
        nbytes = (nat.sample_negative_workspace_ex(B, num, lo, hi, pairs.n) if SAMPLER_BITMAPS
                  else nat.sample_negative_workspace(B, num))
        cache = getattr(self, "_sampler_bufs", None)
        if cache is None or cache["dev"] != dev or cache["ws"].numel() < nbytes:
            cache = self._sampler_bufs = {
                "dev": dev, "ws": torch.empty(nbytes, dtype=torch.uint8, device=dev),
                "state": torch.empty(625, dtype=torch.int32, pin_memory=True)}
        sd = torch.from_numpy(state.view(np.int32)).to(dev)
        rows = torch.from_numpy(np.ascontiguousarray(data, dtype=np.int32)).to(dev)
        out = torch.empty(B * num, dtype=torch.int64, device=dev)
        nat.sample_negative(sd.data_ptr(), lo, hi, rows.data_ptr(), B, ncols, 1, num,
                            pairs.keys.data_ptr() if pairs.n else 0, pairs.n,
                            pairs.codes.data_ptr() if pairs.n else 0, pairs.codes.numel(),
                            out.data_ptr(), cache["ws"].data_ptr(), nbytes,
                            ops._stream(dev))
        # the samples land in a pinned block of torch's caching host allocator
        # that the returned array owns (no second host copy of B x num int64)
        host, hstate = torch.empty(B * num, dtype=torch.int64, pin_memory=True), cache["state"]
        host.copy_(out, non_blocking=True)
        hstate.copy_(sd, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        new = hstate.numpy().view(np.uint32)
        np.random.set_state((st[0], new[:624].copy(), int(new[624]), st[3], st[4]))
        return host.numpy().reshape(B, num)

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
        dev = self._device()
        for _ in range(int(size / num)):
            feed = np.array(dat[:, 1:][np.random.randint(0, len(dat), num)], dtype=np.int64)
            prediction = np.asarray(self.model.topk(feed, 20)) + self.n_user
            if dev is not None:
                for n in self._device_walk(dev, feed, prediction).tolist():
                    if n >= 0:
                        hits.append(1)
                        ndcg.append(np.log(2) / np.log(n + 2))
                        pre.append(1 / (n + 1))
                    elif n == -1:
                        hits.append(0); ndcg.append(0); pre.append(0)
                continue
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

    def _device_walk(self, dev, feed, prediction):
        """hhfm_pf_contains (target test) + hhfm_topk_walk for one batch ->
        numpy int32 outcomes (see ops.topk_walk)."""
        import torch
        from . import ops
        pairs = self._device_pairs(dev, feed.shape[1] - 1)
        rows = torch.from_numpy(np.ascontiguousarray(feed, dtype=np.int32)).to(dev)
        if pairs.n:
            positive = ops.pf_contains(pairs.keys, pairs.codes, rows, 1)
        else:
            positive = torch.zeros(len(feed), dtype=torch.uint8, device=dev)
        pred = torch.from_numpy(np.ascontiguousarray(prediction, dtype=np.int32)).to(dev)
        target = rows[:, 1].contiguous()
        return ops.topk_walk(pred, target, positive, self.TopK).cpu().numpy()

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
