"""Tensor-level entry points over the C ABI (include/hhfm.h).

PyTorch-ROCm is plumbing here: it owns device memory and streams.  Every
function launches a hand-written gfx950 kernel from ``libhhfm.so`` on
``torch.cuda.current_stream()``; there is no eager-PyTorch or CPU fallback.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from ._native import native

MODE_FM = 0
MODE_HHFM = 1

# Plan flags (include/hhfm.h, ABI v4): explicit per-call kernel choices; 0 is
# the default plan.  PLAN_EXACT_FP32 selects k-ordered fp32-MFMA arithmetic
# instead of split-bf16; the others force a fallback kernel on the same
# scores (tests compare both paths on one shape).
PLAN_EXACT_FP32 = 1 << 0
PLAN_NO_SEED = 1 << 1
PLAN_NO_RING = 1 << 2
PLAN_RING_ALT = 1 << 3
PLAN_GEMM = 1 << 4
PLAN_ROW_FM = 1 << 5
PLAN_UNSTAGED = 1 << 6
PLAN_UNGROUPED = 1 << 7
PLAN_NARROW = 1 << 8
PLAN_PER_FIELD = 1 << 9
PLAN_ONE_WAVE = 1 << 10
PLAN_WIDE_3X4 = 1 << 11   # DeepFM 256-row kernel shapes (test shape only)
PLAN_WIDE_2X4 = 2 << 11
PLAN_WIDE_1X4 = 3 << 11
PLAN_STORE = 1 << 13      # small catalog: score matrix + dense top-K (not the fused kernel)
PLAN_FUSED = 1 << 14      # small catalog: the fused score-and-select kernel at any query count


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    raise TypeError(f"embedding table must be float32 or bfloat16, got {t.dtype}")


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _need_cuda(*ts: Optional[torch.Tensor]) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("hhfm_amd kernels take device (cuda/HIP) tensors")
        if not t.is_contiguous():
            raise ValueError("hhfm_amd kernels take contiguous tensors")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError("all tensors must be on the same device")
    return dev


def _idx(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.int32:
        raise TypeError(f"{name} must be int32 (the reference feeds int32 placeholders)")
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D [rows, cols]")
    return t


_STATUS = {}


def status_word(dev: torch.device) -> torch.Tensor:
    """This device's id status word (include/hhfm.h HHFM_STATUS_BAD_ID)."""
    t = _STATUS.get(dev.index)
    if t is None:
        t = torch.zeros(1, dtype=torch.int32, device=dev)
        _STATUS[dev.index] = t
    return t


def check_status(dev: torch.device, features_M: int) -> None:
    """Synchronise and raise like tf.nn.embedding_lookup (InvalidArgumentError,
    FM.py:99) if a kernel on this stream met an id outside [0, features_M)."""
    if native().status_read(status_word(dev).data_ptr(), _stream(dev)) != 0:
        raise ValueError(f"indices must be in [0, {features_M})")


def validate_ids(idx: torch.Tensor, features_M: int) -> None:
    """Raise like tf.nn.embedding_lookup does for ids outside [0, M): one
    hhfm_check_ids kernel + a 4-byte status read (the kernels themselves read
    such ids as row 0, so they can never fault)."""
    if idx.numel() == 0:
        return
    dev = _need_cuda(idx)
    native().check_ids(idx.data_ptr(), idx.numel(), int(features_M),
                       status_word(dev).data_ptr(), _stream(dev))
    check_status(dev, features_M)


def _status_ptr(status: Optional[torch.Tensor]) -> int:
    if status is None:
        return 0
    if status.dtype != torch.int32 or status.numel() < 1 or not status.is_cuda:
        raise TypeError("status must be a device int32 tensor")
    return status.data_ptr()


def fm_score_rows(idx: torch.Tensor, E: torch.Tensor, w: Optional[torch.Tensor],
                  w0: float = 0.0, out: Optional[torch.Tensor] = None,
                  status: Optional[torch.Tensor] = None, flags: int = 0) -> torch.Tensor:
    """FM.out (FM.py:99-120) for rows ``idx`` [B, F] -> float32 [B].
    ``status``: optional device int32 word the kernel flags bad ids in."""
    _idx(idx, "idx")
    dev = _need_cuda(idx, E, w, out)
    B, F = idx.shape
    M, k = E.shape
    if w is not None and (w.dtype != torch.float32 or w.numel() != M):
        raise ValueError("w must be float32 with features_M entries")
    if out is None:
        out = torch.empty(B, dtype=torch.float32, device=dev)
    native().fm_score_rows_ex(idx.data_ptr(), B, F, E.data_ptr(), M, k, _dtype_code(E),
                              0 if w is None else w.data_ptr(), float(w0),
                              out.data_ptr(), int(flags), _status_ptr(status), _stream(dev))
    return out


def hybrid_score_rows(idx: torch.Tensor, E: torch.Tensor, user_col: int = 0,
                      item_col: int = 1, ctx: Tuple[int, int] = (0, 0),
                      time: Tuple[int, int] = (0, 0),
                      out: Optional[torch.Tensor] = None,
                      status: Optional[torch.Tensor] = None) -> torch.Tensor:
    """OUR.PositiveFeadback (OurModel7.py:105-171) for rows ``idx`` -> [B]."""
    _idx(idx, "idx")
    dev = _need_cuda(idx, E, out)
    B, ncols = idx.shape
    M, k = E.shape
    if out is None:
        out = torch.empty(B, dtype=torch.float32, device=dev)
    native().hybrid_score_rows(idx.data_ptr(), B, ncols, user_col, item_col,
                               ctx[0], ctx[1], time[0], time[1], E.data_ptr(), M, k,
                               _dtype_code(E), out.data_ptr(), _status_ptr(status),
                               _stream(dev))
    return out


_WS = {}


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=dev)
        _WS[key] = buf
    return buf


_CWS = {}


def _catalog_workspace(dev: torch.device, stream: int, nbytes: int) -> torch.Tensor:
    """hhfm_catalog_topk's own workspace per (device, stream): zero-filled when
    allocated, because its first HHFM_CATALOG_WS_ZERO bytes hold the
    small-catalog kernel's arrival counters (include/hhfm.h, ABI v6: zero
    before the first call, left zero by every call; no other op shares it)."""
    key = (dev.index, stream)
    buf = _CWS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.zeros(max(nbytes, 1 << 16), dtype=torch.uint8, device=dev)
        _CWS[key] = buf
    return buf


def catalog_topk(qidx: torch.Tensor, E: torch.Tensor, mode: int, K: int,
                 item_row_begin: int, item_count: int, global_item_base: int = 0,
                 w: Optional[torch.Tensor] = None, user_col: int = 0,
                 ctx: Tuple[int, int] = (0, 0), time: Tuple[int, int] = (0, 0),
                 status: Optional[torch.Tensor] = None, plan: int = 0
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Full-catalog score + top-K (FM.topk FM.py:172-198, OUR.topk
    OurModel7.py:229-307). Returns (scores float32 [B,K], ids int32 [B,K]).
    ``plan``: PLAN_* flags (PLAN_EXACT_FP32, _NO_SEED, _NO_RING, _RING_ALT,
    _GEMM, _ONE_WAVE)."""
    _idx(qidx, "qidx")
    dev = _need_cuda(qidx, E, w)
    B, ncols = qidx.shape
    M, k = E.shape
    nat = native()
    st = _stream(dev)
    ws = _catalog_workspace(dev, st, nat.catalog_topk_workspace(B, item_count, k, K))
    top_s = torch.empty(B, K, dtype=torch.float32, device=dev)
    top_i = torch.empty(B, K, dtype=torch.int32, device=dev)
    nat.catalog_topk(qidx.data_ptr(), B, ncols, mode, user_col, ctx[0], ctx[1],
                     time[0], time[1], E.data_ptr(), M, k, _dtype_code(E),
                     0 if w is None else w.data_ptr(), item_row_begin, item_count,
                     global_item_base, K, top_s.data_ptr(), top_i.data_ptr(),
                     ws.data_ptr(), ws.numel(), int(plan), _status_ptr(status), st)
    return top_s, top_i


def topk_merge(scores: torch.Tensor, ids: torch.Tensor
               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Merge R sorted [B,K] lists (stacked [R,B,K], rank-major) into [B,K].
    Device tensors use the HIP kernel; host tensors the C++ host merge."""
    if scores.dim() != 3 or scores.shape != ids.shape:
        raise ValueError("expected scores/ids of shape [R, B, K]")
    if scores.dtype != torch.float32 or ids.dtype != torch.int32:
        raise TypeError("scores float32, ids int32")
    scores = scores.contiguous()
    ids = ids.contiguous()
    R, B, K = scores.shape
    out_s = torch.empty(B, K, dtype=torch.float32, device=scores.device)
    out_i = torch.empty(B, K, dtype=torch.int32, device=scores.device)
    nat = native()
    if scores.is_cuda:
        _need_cuda(scores, ids)
        nat.topk_merge(scores.data_ptr(), ids.data_ptr(), R, B, K, out_s.data_ptr(),
                       out_i.data_ptr(), _stream(scores.device))
    else:
        nat.topk_merge_host(scores.data_ptr(), ids.data_ptr(), R, B, K,
                            out_s.data_ptr(), out_i.data_ptr())
    return out_s, out_i


# ---------------------------------------------------------------------------
# DeepFM (K3) and dense top-K
# ---------------------------------------------------------------------------
def _pad8(x: int) -> int:
    return (x + 7) & ~7


def dfm_prepare_weights(layers, biases, mlp_dtype: torch.dtype, F: int, k: int):
    """Transpose (and pad K to a multiple of 8) the MLP weights into the
    [N][K] layout the GEMM kernel streams (include/hhfm.h, D1)."""
    Wt, bs, dims = [], [], []
    Kin = F * k
    for W, b in zip(layers, biases):
        W = torch.as_tensor(W)
        Kreal, N = W.shape
        t = torch.zeros(N, Kin, dtype=torch.float32, device=W.device)
        t[:, :Kreal] = W.t().float()
        Wt.append(t.to(mlp_dtype).contiguous())
        bs.append(torch.as_tensor(b).reshape(-1).float().contiguous())
        dims.append(N)
        Kin = _pad8(N)
    return Wt, bs, dims


# include/hhfm.h hhfm_dfm_proj: off / on / auto / context fields only / every
# field but the item
DFM_PROJ = {False: 0, True: 1, None: 2, "ctx": 3, "item": 4}


def dfm_forward(idx: torch.Tensor, E: torch.Tensor, w: torch.Tensor, Wt, bias, dims,
                mlp_dtype: torch.dtype, Wp: torch.Tensor, bp: float,
                out: Optional[torch.Tensor] = None,
                proj=None, plan: int = 0) -> torch.Tensor:
    """DeepFM.out (DFM.py:104-137) for rows ``idx`` [B, F] -> float32 [B].

    ``proj``: projected layer 0 (include/hhfm.h, ABI v3) — None lets the
    library decide (include/hhfm.h HHFM_DFM_PROJ_AUTO), True / False force it
    on / off, "ctx" projects the context fields 2..F-1 only and "item" every
    field but the item (bf16 MLP).  ``plan``: PLAN_* flags (fp32 MLP:
    PLAN_EXACT_FP32, _ROW_FM, _UNSTAGED, _UNGROUPED; bf16 MLP: _NARROW)."""
    _idx(idx, "idx")
    dev = _need_cuda(idx, E, w, Wp, *Wt, *bias)
    B, F = idx.shape
    M, k = E.shape
    md = _dtype_code(Wt[0])
    if mlp_dtype != Wt[0].dtype:
        raise TypeError("Wt dtype must equal mlp_dtype")
    if out is None:
        out = torch.empty(B, dtype=torch.float32, device=dev)
    nat = native()
    nbytes = nat.dfm_forward_workspace_ex(B, F, k, M, list(dims), md, DFM_PROJ[proj])
    ws = _workspace(dev, nbytes)
    nat.dfm_forward(idx.data_ptr(), B, F, E.data_ptr(), M, k, _dtype_code(E), w.data_ptr(),
                    list(dims), [t.data_ptr() for t in Wt], [t.data_ptr() for t in bias], md,
                    Wp.data_ptr(), float(bp), out.data_ptr(), DFM_PROJ[proj], int(plan),
                    ws.data_ptr(), ws.numel(), _stream(dev))
    return out


def dfm_catalog_topk(qidx: torch.Tensor, E: torch.Tensor, w: torch.Tensor, Wt, bias, dims,
                     Wp: torch.Tensor, bp: float, item_col: int, item_row_begin: int,
                     item_count: int, K: int, global_item_base: int = 0,
                     chunk_rows: int = 1 << 20, proj=None, plan: int = 0):
    """DeepFM.topk (DFM.py:219-231) -> (scores [B,K], ids [B,K]); ``proj`` and
    ``plan`` as in :func:`dfm_forward` (rows = B x item_count)."""
    _idx(qidx, "qidx")
    dev = _need_cuda(qidx, E, w, Wp, *Wt, *bias)
    B, F = qidx.shape
    M, k = E.shape
    md = _dtype_code(Wt[0])
    nat = native()
    nbytes = nat.dfm_catalog_topk_workspace_ex(B, F, k, M, item_count, list(dims), md,
                                               chunk_rows, DFM_PROJ[proj])
    ws = _workspace(dev, nbytes)
    top_s = torch.empty(B, K, dtype=torch.float32, device=dev)
    top_i = torch.empty(B, K, dtype=torch.int32, device=dev)
    nat.dfm_catalog_topk(qidx.data_ptr(), B, F, item_col, E.data_ptr(), M, k, _dtype_code(E),
                         w.data_ptr(), list(dims), [t.data_ptr() for t in Wt],
                         [t.data_ptr() for t in bias], md, Wp.data_ptr(), float(bp),
                         item_row_begin, item_count, global_item_base, K, chunk_rows,
                         top_s.data_ptr(), top_i.data_ptr(), DFM_PROJ[proj], int(plan),
                         ws.data_ptr(), ws.numel(), _stream(dev))
    return top_s, top_i


def topk_dense(scores: torch.Tensor, K: int, global_item_base: int = 0, plan: int = 0):
    """tf.nn.top_k over a device score matrix [B, N] (K <= 64); ``plan``
    PLAN_ONE_WAVE keeps one wave per query."""
    _need_cuda(scores)
    if scores.dtype != torch.float32 or scores.dim() != 2:
        raise TypeError("scores must be float32 [B, N]")
    B, N = scores.shape
    top_s = torch.empty(B, K, dtype=torch.float32, device=scores.device)
    top_i = torch.empty(B, K, dtype=torch.int32, device=scores.device)
    native().topk_dense(scores.data_ptr(), B, N, scores.stride(0), K, global_item_base,
                        top_s.data_ptr(), top_i.data_ptr(), int(plan), _stream(scores.device))
    return top_s, top_i


# ---------------------------------------------------------------------------
# AFM (K4)
# ---------------------------------------------------------------------------
def afm_forward(idx: torch.Tensor, E: torch.Tensor, w: torch.Tensor, w0: float,
                Wt: torch.Tensor, att_b: torch.Tensor, att_p: torch.Tensor, P: torch.Tensor,
                out: Optional[torch.Tensor] = None, plan: int = 0) -> torch.Tensor:
    """AFM.out (AFM.py:103-142) for rows ``idx`` [B, F] -> float32 [B].
    ``Wt`` is attention_W transposed, [A, k] float32; ``plan`` PLAN_EXACT_FP32
    keeps the contraction on exact-fp32 MFMA."""
    _idx(idx, "idx")
    dev = _need_cuda(idx, E, w, Wt, att_b, att_p, P)
    B, F = idx.shape
    M, k = E.shape
    A = Wt.shape[0]
    if out is None:
        out = torch.empty(B, dtype=torch.float32, device=dev)
    nat = native()
    ws = _workspace(dev, nat.afm_forward_workspace(B, F, A))
    nat.afm_forward(idx.data_ptr(), B, F, E.data_ptr(), M, k, _dtype_code(E), w.data_ptr(),
                    float(w0), Wt.data_ptr(), att_b.data_ptr(), att_p.data_ptr(), A, P.data_ptr(),
                    out.data_ptr(), int(plan), ws.data_ptr(), ws.numel(), _stream(dev))
    return out


def afm_catalog_topk(qidx: torch.Tensor, E: torch.Tensor, w: torch.Tensor, Wt: torch.Tensor,
                     att_b: torch.Tensor, att_p: torch.Tensor, P: torch.Tensor,
                     item_row_begin: int, item_count: int, K: int, global_item_base: int = 0,
                     max_cols: int = 1 << 17, plan: int = 0):
    """AFM.topk (AFM.py:209-246) -> (scores [B,K], ids [B,K]); ``plan``:
    PLAN_EXACT_FP32, _PER_FIELD, _GEMM."""
    _idx(qidx, "qidx")
    dev = _need_cuda(qidx, E, w, Wt, att_b, att_p, P)
    B, F = qidx.shape
    M, k = E.shape
    A = Wt.shape[0]
    nat = native()
    ws = _workspace(dev, nat.afm_catalog_topk_workspace(B, F, k, A, item_count, max_cols,
                                                        int(plan)))
    top_s = torch.empty(B, K, dtype=torch.float32, device=dev)
    top_i = torch.empty(B, K, dtype=torch.int32, device=dev)
    nat.afm_catalog_topk(qidx.data_ptr(), B, F, E.data_ptr(), M, k, _dtype_code(E), w.data_ptr(),
                         Wt.data_ptr(), att_b.data_ptr(), att_p.data_ptr(), A, P.data_ptr(),
                         item_row_begin, item_count, global_item_base, K, max_cols,
                         top_s.data_ptr(), top_i.data_ptr(), int(plan), ws.data_ptr(), ws.numel(),
                         _stream(dev))
    return top_s, top_i


# ---- H5 / H3: harness membership test and metric walk ------------------------
def pf_contains(keys: torch.Tensor, codes: torch.Tensor, rows: torch.Tensor, item_col: int,
                cand: Optional[torch.Tensor] = None) -> torch.Tensor:
    """positive_feedback membership on the device (hhfm_pf_contains).

    keys int32 [nkeys, ncols-1] (sorted, distinct), codes int64 (sorted),
    rows int32 [B, ncols]; cand int32 [B, num] -> uint8 [B, num], or the
    rows' own items (cand None) -> uint8 [B]."""
    _need_cuda(keys, codes, rows, cand)
    if keys.dtype != torch.int32 or codes.dtype != torch.int64 or rows.dtype != torch.int32:
        raise TypeError("keys int32, codes int64, rows int32")
    B, ncols = rows.shape
    num = 1 if cand is None else cand.shape[1]
    if cand is not None and (cand.dtype != torch.int32 or cand.shape[0] != B):
        raise ValueError("cand must be int32 [B, num]")
    out = torch.empty(B, num, dtype=torch.uint8, device=rows.device)
    native().pf_contains(keys.data_ptr(), keys.shape[0], ncols - 1, codes.data_ptr(),
                         codes.numel(), rows.data_ptr(), B, ncols, item_col,
                         0 if cand is None else cand.data_ptr(), num, out.data_ptr(),
                         _stream(rows.device))
    return out if cand is not None else out[:, 0]


def topk_walk(pred: torch.Tensor, target: torch.Tensor, positive: torch.Tensor,
              TopK: int) -> torch.Tensor:
    """evaluate_TopK's walk (hhfm_topk_walk): int32 [B] outcomes, n >= 0 hit
    at walk position n, -1 miss (zeros appended), -2 nothing appended."""
    _need_cuda(pred, target, positive)
    if pred.dtype != torch.int32 or target.dtype != torch.int32 or positive.dtype != torch.uint8:
        raise TypeError("pred/target int32, positive uint8")
    B, P = pred.shape
    out = torch.empty(B, dtype=torch.int32, device=pred.device)
    native().topk_walk(pred.data_ptr(), B, P, target.data_ptr(), positive.data_ptr(), TopK,
                       out.data_ptr(), _stream(pred.device))
    return out
