"""Item-sharded full-catalog top-K across the GPUs of a node,
and row-sharded per-row scoring / metrics.

The reference ranks the whole catalog on one device with one tf.nn.top_k
(FM.py:185, OurModel7.py:295).  Here, one process per GPU:
  1. rank r owns the contiguous item range [begin_r, end_r) of the catalog
     (tables are replicated: users + ctx are tiny, items are read only in
     the rank's range);
  2. it computes its local top-K with hhfm_catalog_topk (scores fp32, ids
     already global item offsets);
  3. one all-gather of the packed (score bits, id) int32 [B, K, 2] per rank —
     RCCL over xGMI when the process group is ``nccl``, gloo on CPU;
  4. hhfm_topk_merge (device) / hhfm_topk_merge_host merges the R sorted
     lists with the same (score desc, id asc) order, which reproduces the
     single-device ranking because ranges are contiguous and ordered.
Payload per rank: B*K*8 bytes (160 KB at B=1024, K=20) — latency-bound.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import ops

NEG_INF = float("-inf")
NO_IDX = 0x7FFFFFFF


def shard_range(n_item: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous near-equal split (first n_item % world ranks get one more)."""
    base, extra = divmod(n_item, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def _pad(scores: torch.Tensor, ids: torch.Tensor, K: int):
    if scores.shape[1] == K:
        return scores, ids
    B = scores.shape[0]
    ps = torch.full((B, K), NEG_INF, dtype=torch.float32, device=scores.device)
    pi = torch.full((B, K), NO_IDX, dtype=torch.int32, device=ids.device)
    ps[:, :scores.shape[1]] = scores
    pi[:, :ids.shape[1]] = ids
    return ps, pi


def comm_device(group=None) -> torch.device:
    """Where this rank's collective payloads live: its GPU for RCCL
    (backend ``nccl``), host memory for gloo (the CPU tests).  The
    collective calls themselves are the same for every backend."""
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_topk(scores: torch.Tensor, ids: torch.Tensor, group=None):
    """All-gather each rank's [B,K] lists -> [R,B,K] (rank-major).

    One collective: (score bits, id) are packed as an int32 [B,K,2] payload
    (8 B per entry), so the latency-bound exchange is a single all-gather
    into one dim-0-concatenated [R·B, K, 2] tensor — the same call for RCCL
    and for gloo, so the gloo tests run exactly the code path RCCL runs."""
    world = dist.get_world_size(group)
    B, K = scores.shape
    packed = torch.stack([scores.contiguous().view(torch.int32), ids.contiguous()], dim=2)
    out = torch.empty(world * B, K, 2, dtype=torch.int32, device=packed.device)
    dist.all_gather_into_tensor(out, packed, group=group)
    out = out.view(world, B, K, 2)
    return out[..., 0].contiguous().view(torch.float32), out[..., 1].contiguous()


LocalScorer = Callable[[object, int, int, int], Tuple[torch.Tensor, torch.Tensor]]


def sharded_topk(A, K: int, n_item: int, local_scorer: LocalScorer, group=None):
    """Global top-K over an item-sharded catalog.

    ``local_scorer(A, begin, count, K_local)`` returns this rank's sorted
    (scores float32 [B,K_local], global item ids int32 [B,K_local]) for items
    [begin, begin+count); the product scorer is ``model_scorer(model)``.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if K > n_item:
        raise ValueError(f"K={K} exceeds the catalog size {n_item}")
    begin, end = shard_range(n_item, world, rank)
    count = end - begin
    dev = comm_device(group)
    if count > 0:
        s, i = local_scorer(A, begin, count, min(K, count))
        s, i = _pad(s, i, K)
        # the payload where the backend reads it: the GPU for RCCL, host
        # memory for gloo (a device scorer's lists copied once, B·K·8 bytes)
        if world > 1:
            s, i = s.to(dev), i.to(dev)
    else:
        B = len(A)
        s = torch.full((B, K), NEG_INF, dtype=torch.float32, device=dev)
        i = torch.full((B, K), NO_IDX, dtype=torch.int32, device=dev)
    if world == 1:
        return s, i
    gs, gi = gather_topk(s, i, group)
    return ops.topk_merge(gs, gi)


def model_scorer(model) -> LocalScorer:
    """The HIP local scorer of a model for its rank's item range: each model
    class scores items [begin, begin+count) with its own catalog kernel
    (FM.py:172-185, OurModel7.py:229-295, AFM.py:209-246, DFM.py:219-231) and
    reports global item offsets."""
    from .AFM import AFM
    from .DFM import DeepFM
    from .FM import FM
    from .OurModel7 import OUR
    if not isinstance(model, (FM, OUR, AFM, DeepFM)):
        raise TypeError(f"no sharded catalog scorer for {type(model).__name__}; "
                        "expected FM, OUR, AFM or DeepFM")

    def score(A, begin, count, K):
        return model.catalog_topk(model._idx(A), begin, count, K)
    return score


def sharded_model_topk(model, A, tp, group=None) -> np.ndarray:
    """Drop-in for ``model.topk(A, tp)`` with the catalog sharded over the
    ranks of ``group`` (every rank calls it with the same A)."""
    _, ids = sharded_topk(A, int(tp), model.n_item, model_scorer(model), group)
    return ids.cpu().numpy()


# ---------------------------------------------------------------------------
# Row-sharded per-triple metrics ("the only collective is a
# scalar all-reduce of metric sums")
# ---------------------------------------------------------------------------
def sharded_evaluate_auc(tr, data1, group=None) -> float:
    """Train.evaluate_AUC (FM.py:296-324; OurModel7.py:430-461 first-chunk
    variant) with the scoring split over the ranks: every rank draws the
    SAME negatives (identical numpy RNG stream, cheap host work), scores only
    its contiguous slice of each 600-row chunk on its own GPU, and one
    all-reduce of (hits, comparisons) yields exactly the single-device value
    (mean of the same booleans)."""
    from .harness import partition_all
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    dat = data1.values
    if tr.auc_label_filter:
        dat = dat[dat[:, 0] > 0]
    X = np.array(dat[:, 1:], dtype=np.int64)
    hits, total = 0, 0
    for chunk in partition_all(600, range(len(X))):
        pos = X[chunk]
        negs = tr.sample_negative(pos, 50)          # same draw on every rank
        b, e = shard_range(len(pos), world, rank)
        if e > b:
            mine = pos[b:e]
            neg = np.repeat(mine[:, None, :], 50, axis=1).reshape(-1, pos.shape[1])
            neg[:, 1] = negs[b:e].reshape(-1)
            neg_score = np.asarray(tr.model.score_rows(neg)).reshape(-1)
            pos_score = np.repeat(np.asarray(tr.model.score_rows(mine)).reshape(-1), 50)
            hits += int((pos_score > neg_score).sum())
            total += pos_score.size
        if tr.auc_first_chunk_only:
            break
    t = torch.tensor([hits, total], dtype=torch.float64, device=comm_device(group))
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t[0] / t[1])


# ---------------------------------------------------------------------------
# Row-sharded per-row scores (C2 / C5 over N GPUs: rows split, no exchange in
# the data path; one gather only when the caller wants every score on every rank)
# ---------------------------------------------------------------------------
RowScorer = Callable[[object], torch.Tensor]


def sharded_score_rows(X, score_rows: RowScorer, gather: bool = True, group=None):
    """``sess.run(model.out)`` (FM.py:99-120, DFM.py:104-137, AFM.py:103-142)
    over a batch shared by every rank, its rows split across the ranks: rank r
    scores the contiguous rows ``shard_range(len(X), world, r)`` with
    ``score_rows`` (e.g. ``model.score_rows`` — the HIP row kernels on the
    rank's GPU) and, with ``gather``, one all-gather of the per-rank float32
    slices (padded to the longest) returns every row's score in row order on
    every rank — the single-device result, since a row's score never depends
    on the others.  ``gather=False`` returns (this rank's scores, begin)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n = len(X)
    b, e = shard_range(n, world, rank)
    dev = comm_device(group)
    mine = (torch.as_tensor(np.asarray(score_rows(X[b:e])), dtype=torch.float32).reshape(-1)
            if e > b else torch.empty(0, dtype=torch.float32))
    mine = mine.to(dev)
    if not gather:
        return mine, b
    if world == 1:
        return mine
    longest = shard_range(n, world, 0)[1]          # rank 0 holds the longest slice
    pad = torch.zeros(longest, dtype=torch.float32, device=dev)
    pad[:mine.numel()] = mine
    out = torch.empty(world * longest, dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(out, pad, group=group)
    out = out.view(world, longest)
    return torch.cat([out[r, :shard_range(n, world, r)[1] - shard_range(n, world, r)[0]]
                      for r in range(world)])
