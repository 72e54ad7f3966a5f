"""Shared plumbing of the model classes (FM, OUR, AFM, DeepFM).

Each reference model is a TF-1.x graph plus ``sess.run`` (e.g. FM.py:81-148);
here a model owns its weights as device tensors and scores through the HIP
kernels of ``libhhfm``.  For drop-in use by code written against the
reference, ``model.sess.run(model.out, feed_dict={model.train_features: X})``
(and the HHFM ``Pos``/``Fea``/``Tim`` -> ``PositiveFeadback`` form) are
accepted and routed to ``score_rows``.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from . import ops


class Placeholder:
    """Stand-in for a tf.placeholder handle (a feed_dict key)."""

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"<placeholder {self.name}>"


class Fetch:
    """Stand-in for a graph tensor a caller may ``sess.run``."""

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"<fetch {self.name}>"


class Session:
    def __init__(self, model):
        self._m = model

    def run(self, fetches, feed_dict=None):
        feed = feed_dict or {}
        if isinstance(fetches, (tuple, list)):
            return type(fetches)(self.run(f, feed) for f in fetches)
        return self._m._run_fetch(fetches, feed)


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("hhfm_amd models need a HIP device (MI355X); there is no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


class ScoringModel(object):
    """Weights on device + conversions; subclasses define the graph."""

    def _setup_device(self, device=None, table_dtype=torch.float32):
        self.device = torch.device(device) if device is not None else default_device()
        if table_dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("table_dtype must be torch.float32 or torch.bfloat16")
        self.table_dtype = table_dtype
        self.validate = True
        self.sess = Session(self)

    def _gen(self, seed):
        g = torch.Generator(device=self.device)
        g.manual_seed(int(seed))
        return g

    def _normal(self, shape, std, seed):
        t = torch.empty(shape, dtype=torch.float32, device=self.device)
        t.normal_(0.0, std, generator=self._gen(seed))
        return t

    # -- conversions ----------------------------------------------------------
    def _idx(self, X) -> torch.Tensor:
        """Ids -> device int32.  Wider integer inputs are range-checked BEFORE
        narrowing (a cast would wrap 2**32+5 to 5 and slip past the check)."""
        checked = False
        if isinstance(X, torch.Tensor):
            if X.dtype != torch.int32 and self.validate and X.numel():
                lo, hi = int(X.min()), int(X.max())
                if lo < 0 or hi >= self.features_M:
                    raise ValueError(f"indices must be in [0, {self.features_M}), "
                                     f"got [{lo}, {hi}]")
                checked = True
            t = X.to(device=self.device, dtype=torch.int32)
        else:
            a = np.asarray(X)
            if a.dtype != np.int32 and self.validate and a.size:
                lo, hi = int(a.min()), int(a.max())
                if lo < 0 or hi >= self.features_M:
                    raise ValueError(f"indices must be in [0, {self.features_M}), "
                                     f"got [{lo}, {hi}]")
                checked = True
            t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32))
            t = t.to(self.device, non_blocking=False)
        if t.dim() != 2:
            raise ValueError("expected a 2-D index matrix [rows, columns]")
        t = t.contiguous()
        if self.validate and not checked:
            ops.validate_ids(t, self.features_M)
        return t

    @property
    def table(self) -> torch.Tensor:
        """The embedding table in its storage dtype (what the kernels read)."""
        E = self.weights["feature_embeddings"]
        if self.table_dtype == torch.float32:
            return E
        if getattr(self, "_table_cache_src", None) is not E or self._table_cache_ver != E._version:
            self._table_cache = E.to(self.table_dtype).contiguous()
            self._table_cache_src = E
            self._table_cache_ver = E._version
        return self._table_cache

    # -- weights ---------------------------------------------------------------
    def get_weights(self) -> Dict[str, np.ndarray]:
        return {k: (v.detach().float().cpu().numpy() if isinstance(v, torch.Tensor) else v)
                for k, v in self.weights.items()}

    def set_weights(self, **arrays):
        for k, v in arrays.items():
            if k not in self.weights:
                raise KeyError(f"unknown weight {k!r}; have {sorted(self.weights)}")
            cur = self.weights[k]
            t = torch.as_tensor(np.asarray(v), dtype=torch.float32).to(self.device)
            if isinstance(cur, torch.Tensor) and t.shape != cur.shape:
                t = t.reshape(cur.shape)
            self.weights[k] = t.contiguous()

    def _run_fetch(self, fetch, feed):
        raise TypeError(f"unsupported fetch {fetch!r}")

    @staticmethod
    def _np_out(t: torch.Tensor) -> np.ndarray:
        return t.cpu().numpy().reshape(-1, 1)


def rows_from(feed: dict, *holders: Optional[Placeholder]) -> np.ndarray:
    parts = [np.asarray(feed[h]) for h in holders if h is not None and h in feed]
    return np.concatenate(parts, axis=1)
