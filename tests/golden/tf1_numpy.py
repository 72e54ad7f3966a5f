"""A numpy restatement of the TensorFlow 1.x graph API subset that the
reference's model classes call (data-man-34/HHFM, Newcode/{FM,OurModel7,
AFM,DFM}.py) — used ONLY by tests/golden/make_golden.py, in the builder
container, to execute the reference's own graph-building code and freeze its
outputs as golden vectors.  Nothing from the reference ships or runs on the
GPU box.

TensorFlow itself is absent from the image; the reference
pins no version (TF 1.5–1.15 by its API use).  Each op below restates TF's
published semantics: graph nodes are built lazily, ``Session.run`` evaluates
them in float32 with the feed dict; ``nn.top_k`` sorts descending with ties
to the lower index; ``nn.dropout`` is only accepted with keep_prob == 1 (the
reference's evaluation setting); optimizers are no-ops (training is not
reproduced by the fixtures).
"""
from __future__ import annotations

import contextlib
import types

import numpy as np

float32 = np.float32
int32 = np.int32
int64 = np.int64
bool = np.bool_  # noqa: A001 - mirrors tf.bool

_rng = np.random.default_rng(12345)
LAST_TOPK_INPUT = []   # score matrices handed to nn.top_k (for fixtures)


def set_random_seed(seed):
    global _rng
    _rng = np.random.default_rng(seed)


class Node:
    def __init__(self, fn, inputs=(), name=None):
        self.fn = fn
        self.inputs = list(inputs)
        self.name = name

    def _eval(self, ctx):
        key = id(self)
        if key in ctx:
            return ctx[key]
        vals = [_ev(i, ctx) for i in self.inputs]
        out = self.fn(*vals)
        ctx[key] = out
        return out

    # operators
    def __getitem__(self, k):
        return Node(lambda x: x[k], [self])

    def __add__(self, o): return add(self, o)
    def __radd__(self, o): return add(o, self)
    def __sub__(self, o): return subtract(self, o)
    def __rsub__(self, o): return subtract(o, self)
    def __mul__(self, o): return multiply(self, o)
    def __rmul__(self, o): return multiply(o, self)
    def __truediv__(self, o): return divide(self, o)
    def __neg__(self): return Node(lambda x: -x, [self])


class Placeholder(Node):
    def __init__(self, dtype, shape=None, name=None):
        super().__init__(None, (), name)
        self.dtype = dtype

    def _eval(self, ctx):
        feed = ctx["__feed__"]
        if self not in feed:
            raise KeyError(f"placeholder {self.name} not fed")
        return np.asarray(feed[self], dtype=self.dtype)


class Variable(Node):
    def __init__(self, initial_value=None, name=None, dtype=None, trainable=True):
        super().__init__(None, (), name)
        v = _ev(initial_value, {"__feed__": {}}) if isinstance(initial_value, Node) \
            else np.asarray(initial_value)
        if dtype is not None:
            v = np.asarray(v, dtype=dtype)
        elif v.dtype == np.float64:
            v = v.astype(np.float32)
        self.value = v

    def _eval(self, ctx):
        return self.value


class _NoOp(Node):
    def __init__(self):
        super().__init__(lambda: None, ())


def _ev(x, ctx):
    if isinstance(x, Node):
        return x._eval(ctx)
    if isinstance(x, (list, tuple)):
        return type(x)(_ev(i, ctx) for i in x)
    return x


def _f(x):
    a = np.asarray(x)
    return a.astype(np.float32) if a.dtype == np.float64 else a


def _node(fn, *inputs):
    return Node(fn, inputs)


# ---- constructors ----------------------------------------------------------
def placeholder(dtype, shape=None, name=None):
    return Placeholder(dtype, shape, name)


def constant(value, dtype=None, name=None):
    v = np.asarray(value, dtype=dtype) if dtype is not None else _f(value)
    return Node(lambda: v, (), name)


def random_normal(shape, mean=0.0, stddev=1.0, dtype=np.float32, seed=None):
    v = _rng.normal(mean, stddev, size=shape).astype(np.float32)
    return Node(lambda: v, ())


def random_uniform(shape, minval=0.0, maxval=1.0, dtype=np.float32, seed=None):
    v = _rng.uniform(minval, maxval, size=shape).astype(np.float32)
    return Node(lambda: v, ())


def global_variables_initializer():
    return _NoOp()


# ---- elementwise / reductions -----------------------------------------------
def add(a, b, name=None): return _node(lambda x, y: _f(x) + _f(y), a, b)
def subtract(a, b, name=None): return _node(lambda x, y: _f(x) - _f(y), a, b)
def multiply(a, b, name=None): return _node(lambda x, y: _f(x) * _f(y), a, b)
def divide(a, b, name=None): return _node(lambda x, y: _f(x) / _f(y), a, b)
def square(a, name=None): return _node(lambda x: np.square(_f(x)), a)
def exp(a, name=None): return _node(lambda x: np.exp(_f(x)), a)
def log(a, name=None): return _node(lambda x: np.log(_f(x)), a)
def sigmoid(a, name=None): return _node(lambda x: (1.0 / (1.0 + np.exp(-_f(x)))).astype(np.float32), a)


def add_n(inputs, name=None):
    def fn(*xs):
        out = _f(xs[0])
        for x in xs[1:]:
            out = out + _f(x)
        return out
    return Node(fn, inputs, name)


def _red(op):
    def red(x, axis=None, keep_dims=False, keepdims=None, name=None):
        kd = keep_dims if keepdims is None else keepdims
        return _node(lambda v: op(_f(v), axis=axis, keepdims=kd), x)
    return red


reduce_sum = _red(lambda v, axis, keepdims: np.sum(v, axis=axis, keepdims=keepdims, dtype=v.dtype))
reduce_max = _red(np.max)
reduce_mean = _red(lambda v, axis, keepdims: np.mean(v, axis=axis, keepdims=keepdims, dtype=v.dtype))


def ones_like(x, name=None): return _node(lambda v: np.ones_like(_f(v)), x)
def zeros_like(x, name=None): return _node(lambda v: np.zeros_like(_f(v)), x)


# ---- shape ops ------------------------------------------------------------------
def stack(values, axis=0, name=None): return Node(lambda *xs: np.stack(xs, axis=axis), values)
def concat(values, axis, name=None): return Node(lambda *xs: np.concatenate(xs, axis=axis), values)
def transpose(x, perm=None, name=None): return _node(lambda v: np.transpose(v, perm), x)
def expand_dims(x, axis, name=None): return _node(lambda v: np.expand_dims(v, axis), x)
def reshape(x, shape, name=None): return _node(lambda v: np.reshape(v, shape), x)


def matmul(a, b, name=None):
    return _node(lambda x, y: np.matmul(_f(x), _f(y)).astype(np.float32), a, b)


# ---- nn ------------------------------------------------------------------------
def _embedding_lookup(params, ids, name=None):
    def fn(p, i):
        i = np.asarray(i)
        if i.size and (i.min() < 0 or i.max() >= p.shape[0]):
            raise IndexError("embedding_lookup: id out of range")
        return p[i.astype(np.int64)]
    return _node(fn, params, ids)


def _softmax(x, axis=-1, dim=None, name=None):
    ax = axis if dim is None else dim

    def fn(v):
        v = _f(v)
        e = np.exp(v - v.max(axis=ax, keepdims=True))
        return (e / e.sum(axis=ax, keepdims=True)).astype(np.float32)
    return _node(fn, x)


def _dropout(x, keep_prob, name=None):
    def fn(v, k):
        if float(np.asarray(k)) != 1.0:
            raise NotImplementedError("fixtures are generated with keep_prob == 1")
        return v
    return _node(fn, x, keep_prob)


def _top_k(x, k=1, sorted=True, name=None):   # noqa: A002
    def idx_fn(v):
        v = _f(v)
        LAST_TOPK_INPUT.append(v)
        return np.argsort(-v, axis=-1, kind="stable")[..., :k].astype(np.int32)
    ind = _node(idx_fn, x)
    val = _node(lambda v, i: np.take_along_axis(_f(v), i.astype(np.int64), -1), x, ind)
    return val, ind


def _l2_loss(x, name=None): return _node(lambda v: np.float32(np.sum(np.square(_f(v))) / 2), x)


nn = types.SimpleNamespace(
    embedding_lookup=_embedding_lookup, relu=lambda x, name=None: _node(lambda v: np.maximum(_f(v), 0), x),
    sigmoid=sigmoid, softmax=_softmax, dropout=_dropout, top_k=_top_k, l2_loss=_l2_loss)


# ---- training / session (no-ops for fixtures) ------------------------------------
class _Opt:
    def __init__(self, *a, **k): pass
    def minimize(self, loss): return _NoOp()


train = types.SimpleNamespace(AdamOptimizer=_Opt, AdagradOptimizer=_Opt,
                              GradientDescentOptimizer=_Opt, MomentumOptimizer=_Opt,
                              Saver=lambda *a, **k: None)
losses = types.SimpleNamespace(log_loss=lambda labels, predictions: _NoOp())


def _l2_regularizer(scale):
    return lambda w: _node(lambda v: np.float32(scale * np.sum(np.square(_f(v))) / 2), w)


contrib = types.SimpleNamespace(layers=types.SimpleNamespace(
    l2_regularizer=_l2_regularizer,
    python=types.SimpleNamespace(layers=types.SimpleNamespace(batch_norm=None))))


class ConfigProto:
    def __init__(self, **kw):
        self.gpu_options = types.SimpleNamespace(allow_growth=False)


class Session:
    def __init__(self, config=None, graph=None):
        pass

    def run(self, fetches, feed_dict=None):
        ctx = {"__feed__": dict(feed_dict or {})}
        return _ev(fetches, ctx)


class Graph:
    @contextlib.contextmanager
    def as_default(self):
        yield self


def install(sys_modules):
    """Register this module as ``tensorflow`` (+ the contrib import path the
    reference uses) in ``sys_modules``."""
    import sys
    me = sys.modules[__name__]
    sys_modules["tensorflow"] = me
    for name in ("tensorflow.contrib", "tensorflow.contrib.layers",
                 "tensorflow.contrib.layers.python",
                 "tensorflow.contrib.layers.python.layers"):
        m = types.ModuleType(name)
        m.batch_norm = None
        m.layers = contrib.layers
        sys_modules[name] = m
