"""DeepFM (K3) on the GPU vs the reference graph (golden dfm.npz) and vs the
oracle at larger shapes.

Tolerances: fp32 MLP mode (reference numerics) — the north_star's 1e-5
relative, elementwise against the float64 value of DFM.py:104-137 on every
row whose condition number Σ_j |concat_j·Wp_j| / |out| is at most 100, and
1e-5 of that magnitude on the rest (tests/helpers.kappa_check, κ counts in
the parity report); bf16 MLP mode — compared with an oracle that rounds the
same operands to bf16 (table rows, weights, hidden activations), 5e-3 of the
magnitude (a 1-ulp bf16 flip of a hidden unit, 2^-8 relative, is the expected
discrepancy)."""
import os

import numpy as np
import pytest
import torch

from oracle import fm_oracle as orc
from oracle import parity
from tests.helpers import bf16_round, kappa_check

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def _model(d_or_shapes, mlp_dtype=torch.float32, table_dtype=torch.float32):
    from hhfm_amd.DFM import DeepFM
    nu, ni, M, F, k, layers = d_or_shapes
    return DeepFM(nu, ni, M, F, k, layers, None, 0.01, 0, 0.01, mlp_dtype=mlp_dtype,
                  table_dtype=table_dtype)


_magnitude = parity.dfm_magnitude
_bf16_oracle = parity.dfm_bf16_out


def _f32_check(got, X, E, w, Ls, Bs, Wp, bp, ref32=None):
    """fp32 MLP: 1e-5 relative elementwise on κ <= 100 rows (kappa_check)."""
    ex, mag = parity.dfm_rows_exact(X, E, w, Ls, Bs, Wp, bp)
    if ref32 is None:
        ref32 = orc.dfm_out(X, E, w, Ls, Bs, Wp, bp)[:, 0]
    return kappa_check("dfm_rows_kappa", got, ref32, ex, mag)


def test_dfm_vs_reference_graph():
    d = dict(np.load(os.path.join(G, "dfm.npz")))
    nu, ni = int(d["n_user"]), int(d["n_item"])
    M, k = d["E"].shape
    layers = [d[f"layer_{i}"] for i in range(3)]
    biases = [d[f"bias_{i}"] for i in range(3)]
    m = _model((nu, ni, M, 5, k, [150, 200, 150]))
    m.set_weights(feature_embeddings=d["E"], feature_bias=d["w"][:, None],
                  concat_projection=d["concat_projection"], concat_bias=d["concat_bias"],
                  **{f"layer_{i}": layers[i] for i in range(3)},
                  **{f"bias_{i}": biases[i] for i in range(3)})
    out = m.score_rows(d["X"])[:, 0]
    _f32_check(out, d["X"], d["E"], d["w"], layers, biases, d["concat_projection"],
               d["concat_bias"], ref32=d["out"])
    out2 = m.sess.run(m.out, feed_dict={m.feat_index: d["X"], m.label: None})
    assert np.array_equal(out2[:, 0], out)
    pred = m.topk(d["A"], 20)
    # bit-exact against the reference graph's golden top-20
    assert np.array_equal(pred, d["topk_idx"]), int((pred != d["topk_idx"]).sum())


@pytest.mark.parametrize("mlp", ["f32", "bf16"])
@pytest.mark.parametrize("k,layers", [(64, [400, 400, 400]), (256, [400, 400, 400]),
                                      (32, [150, 200, 150])])
def test_dfm_forward_shapes(mlp, k, layers):
    rng = np.random.default_rng(k + len(layers))
    nu, ni, F = 957, 4082, 5
    M = nu + ni + 12
    B = 3001
    X = np.stack([rng.integers(0, nu, B), rng.integers(nu, nu + ni, B),
                  rng.integers(nu + ni, nu + ni + 7, B), rng.integers(nu + ni + 7, nu + ni + 9, B),
                  rng.integers(nu + ni + 9, M, B)], 1).astype(np.int32)
    mdt = torch.float32 if mlp == "f32" else torch.bfloat16
    m = _model((nu, ni, M, F, k, layers), mlp_dtype=mdt)
    W = m.get_weights()
    Ls = [W[f"layer_{i}"] for i in range(3)]
    Bs = [W[f"bias_{i}"] for i in range(3)]
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    got = m.score_rows(X)[:, 0]
    mag = _magnitude(X, E, w, Ls, Bs, Wp, bp)
    if mlp == "f32":
        _f32_check(got, X, E, w, Ls, Bs, Wp, bp)
    else:
        ref = _bf16_oracle(X, E, w, Ls, Bs, Wp, bp)
        assert np.all(np.abs(got - ref) <= 5e-3 * mag)


@pytest.mark.parametrize("proj", [False, True, "ctx", "item"])
@pytest.mark.parametrize("mlp", ["f32", "bf16"])
def test_dfm_catalog_topk_chunked(mlp, proj):
    """Query chunking (chunk_rows < B*N) gives the same top-K as one pass
    (bf16: the fused kernel scores the chunks; oracle rounds like it)."""
    from hhfm_amd import ops
    rng = np.random.default_rng(8)
    nu, ni, F, k = 50, 700, 5, 32
    M = nu + ni + 12
    mdt = torch.float32 if mlp == "f32" else torch.bfloat16
    m = _model((nu, ni, M, F, k, [64, 48]), mlp_dtype=mdt)
    A = np.stack([rng.integers(0, nu, 37), rng.integers(nu, nu + ni, 37),
                  rng.integers(nu + ni, nu + ni + 7, 37), rng.integers(nu + ni + 7, nu + ni + 9, 37),
                  rng.integers(nu + ni + 9, M, 37)], 1).astype(np.int32)
    W = m.get_weights()
    Ls = [W["layer_0"], W["layer_1"]]
    Bs = [W["bias_0"], W["bias_1"]]
    if mlp == "f32":
        sc = orc.dfm_catalog_scores(A, W["feature_embeddings"], W["feature_bias"][:, 0], Ls, Bs,
                                    W["concat_projection"], float(W["concat_bias"]), nu, ni)
    else:
        rows = np.repeat(A, ni, 0)
        rows[:, 1] = np.tile(np.arange(nu, nu + ni), len(A))
        sc = _bf16_oracle(rows, W["feature_embeddings"], W["feature_bias"][:, 0], Ls, Bs,
                          W["concat_projection"], float(W["concat_bias"])).reshape(len(A), ni)
    Wt, bs, dims, Wp, bp = m._prepared()
    q = torch.from_numpy(A).cuda()
    for chunk in (1 << 20, 1000, 701):
        s, i = ops.dfm_catalog_topk(q, m.table, m.weights["feature_bias"].reshape(-1), Wt, bs,
                                    dims, Wp, bp, 1, nu, ni, 20, 0, chunk, proj=proj)
        rs, ri = orc.top_k(sc, 20)
        tol = (1e-5 if mlp == "f32" else 5e-3) * np.abs(sc).max(1, keepdims=True)
        bad, swaps = orc.topk_swaps(sc, ri, i.cpu().numpy(), tol)
        assert bad == 0 and swaps == 0, (chunk, bad, swaps)


def test_topk_dense_matches_sort():
    from hhfm_amd import ops
    rng = np.random.default_rng(3)
    S = rng.integers(0, 50, size=(77, 3001)).astype(np.float32)   # heavy ties
    for K in (1, 20, 33, 64):
        s, i = ops.topk_dense(torch.from_numpy(S).cuda(), K, 5)
        rs, ri = orc.top_k(S, K)
        assert np.array_equal(i.cpu().numpy(), ri + 5)
        assert np.array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("F,k,layers,tdt,B", [
    (5, 16, [33], "bf16", 129),                 # fused, 1 layer, bf16 table, ragged tail
    (3, 48, [64, 96, 33, 20], "f32", 1000),     # fused, 4 layers, odd widths
    (11, 32, [128, 416], "bf16", 1),            # fused, widest envelope (13 tiles), one row
    (5, 64, [450, 64], "f32", 300),             # layered fallback: 15 tiles
    (5, 64, [64, 64, 64, 64, 64], "f32", 257),  # layered fallback: 5 layers
    (5, 40, [100], "f32", 77),                  # layered fallback: k % 16 != 0
])
@pytest.mark.parametrize("mlp", ["bf16", "f32"])
def test_dfm_fused_envelope(F, k, layers, tdt, B, mlp):
    """The fused per-row-block kernels (dfm_fused.hip, bf16 and fp32 MLP) and
    the layer-by-layer GEMM path outside their envelope, against the oracle
    (bf16: the bf16-rounding oracle, 5e-3; fp32: 1e-5 relative, κ <= 100)."""
    rng = np.random.default_rng(F * 1000 + k)
    M = 997
    tdtype = torch.bfloat16 if tdt == "bf16" else torch.float32
    mdt = torch.bfloat16 if mlp == "bf16" else torch.float32
    m = _model((100, 200, M, F, k, layers), mlp_dtype=mdt, table_dtype=tdtype)
    X = rng.integers(0, M, size=(B, F)).astype(np.int32)
    W = m.get_weights()
    L = len(layers)
    Ls = [W[f"layer_{i}"] for i in range(L)]
    Bs = [W[f"bias_{i}"] for i in range(L)]
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    if tdt == "bf16":
        E = bf16_round(E)
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    got = m.score_rows(X)[:, 0]
    mag = _magnitude(X, E, w, Ls, Bs, Wp, bp)
    if mlp == "bf16":
        ref = _bf16_oracle(X, E, w, Ls, Bs, Wp, bp)
        assert np.all(np.abs(got - ref) <= 5e-3 * mag), np.max(np.abs(got - ref) / mag)
    else:
        _f32_check(got, X, E, w, Ls, Bs, Wp, bp)


@pytest.mark.parametrize("F,k,layers,tdt,B", [
    (5, 256, [400, 400, 400], "f32", 3001),     # C5 shape (TM = 13)
    (5, 64, [150, 200, 150], "bf16", 5000),     # the reference's layers
    (5, 16, [33], "bf16", 129),                 # one layer: no hidden chunks
    (3, 48, [64, 96, 33, 20], "f32", 1000),     # 4 layers, odd widths
    (11, 32, [128, 416], "bf16", 1),            # widest envelope, one row
])
@pytest.mark.parametrize("mlp,proj", [("bf16", True), ("f32", True), ("bf16", "ctx"),
                                      ("bf16", "item")])
def test_dfm_projected_layer0(F, k, layers, tdt, B, mlp, proj):
    """Projected layer 0 (h_0 = Σ_f P_f[x_f], dfm_fused.hip PROJ kernels),
    forced on for every field (True), for the context fields 2..F-1 with
    fields 0, 1 on MFMA ("ctx", bf16 MLP) or for every field but the item
    with the rows grouped by user ("item", bf16 MLP), against the same oracles and
    tolerances as the direct kernels, and against the direct kernel itself
    (bf16: summation order only, so the two differ by at most a bf16 flip of
    a hidden unit)."""
    from hhfm_amd import ops
    rng = np.random.default_rng(F * 7919 + k)
    M = 997
    tdtype = torch.bfloat16 if tdt == "bf16" else torch.float32
    mdt = torch.bfloat16 if mlp == "bf16" else torch.float32
    m = _model((100, 200, M, F, k, layers), mlp_dtype=mdt, table_dtype=tdtype)
    X = rng.integers(0, M, size=(B, F)).astype(np.int32)
    if proj == "item":
        X[:, 0] %= 40   # ~B/40 rows per user: grouped rows stage the user's P rows
    if proj in ("ctx", "item") and F >= 5:
        # narrow context fields; field 4 narrow in the first half of the rows
        # only: those blocks run LDS-staged (PJ = 2), the rest from HBM
        X[:, 2] = 900 + X[:, 2] % 7
        X[:, 3] = 950 + X[:, 3] % 2
        X[:B // 2, 4] = 980 + X[:B // 2, 4] % 3
    W = m.get_weights()
    L = len(layers)
    Ls = [W[f"layer_{i}"] for i in range(L)]
    Bs = [W[f"bias_{i}"] for i in range(L)]
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    if tdt == "bf16":
        E = bf16_round(E)
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    Wt, bs, dims, Wpd, bpd = m._prepared()
    xd = torch.from_numpy(X).cuda()
    wb = m.weights["feature_bias"].reshape(-1)
    got = ops.dfm_forward(xd, m.table, wb, Wt, bs, dims, mdt, Wpd, bpd, proj=proj).cpu().numpy()
    direct = ops.dfm_forward(xd, m.table, wb, Wt, bs, dims, mdt, Wpd, bpd,
                             proj=False).cpu().numpy()
    mag = _magnitude(X, E, w, Ls, Bs, Wp, bp)
    if mlp == "bf16":
        ref = _bf16_oracle(X, E, w, Ls, Bs, Wp, bp)
        assert np.all(np.abs(got - ref) <= 5e-3 * mag), np.max(np.abs(got - ref) / mag)
        assert np.all(np.abs(got - direct) <= 5e-3 * mag), np.max(np.abs(got - direct) / mag)
    else:
        _f32_check(got, X, E, w, Ls, Bs, Wp, bp)
        _f32_check(direct, X, E, w, Ls, Bs, Wp, bp)



@pytest.mark.parametrize("M,users", [(997, 40), (8100, 6000), (20000, 300)])
def test_dfm_item_grouping(M, users):
    """ITEM mode's row grouping (the forward regroups its rows by user: a
    counting sort for tables up to 8 K rows, hipCUB's radix sort above) puts
    every score back at its caller's row: equal to the direct kernel within
    the bf16 tolerance, and to a call on the same rows in another order."""
    from hhfm_amd import ops
    rng = np.random.default_rng(M)
    F, k, B = 5, 64, 6000
    m = _model((users, 400, M, F, k, [150, 200, 150]), mlp_dtype=torch.bfloat16,
               table_dtype=torch.bfloat16)
    X = rng.integers(0, M, size=(B, F)).astype(np.int32)
    X[:, 0] = rng.integers(0, users, B)
    X[:, 2] = M - 7 + X[:, 2] % 7
    X[:, 3] = M - 9 + X[:, 3] % 2
    X[:, 4] = M - 12 + X[:, 4] % 3
    W = m.get_weights()
    Ls = [W[f"layer_{i}"] for i in range(3)]
    Bs = [W[f"bias_{i}"] for i in range(3)]
    E, w = bf16_round(W["feature_embeddings"]), W["feature_bias"][:, 0]
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    Wt, bs, dims, Wpd, bpd = m._prepared()
    wb = m.weights["feature_bias"].reshape(-1)
    xd = torch.from_numpy(X).cuda()
    got = ops.dfm_forward(xd, m.table, wb, Wt, bs, dims, torch.bfloat16, Wpd, bpd,
                          proj="item").cpu().numpy()
    direct = ops.dfm_forward(xd, m.table, wb, Wt, bs, dims, torch.bfloat16, Wpd, bpd,
                             proj=False).cpu().numpy()
    perm = rng.permutation(B)
    again = ops.dfm_forward(xd[torch.from_numpy(perm).cuda()], m.table, wb, Wt, bs, dims,
                            torch.bfloat16, Wpd, bpd, proj="item").cpu().numpy()
    mag = _magnitude(X, E, w, Ls, Bs, Wp, bp)
    ref = _bf16_oracle(X, E, w, Ls, Bs, Wp, bp)
    assert np.all(np.abs(got - ref) <= 5e-3 * mag), np.max(np.abs(got - ref) / mag)
    assert np.all(np.abs(got - direct) <= 5e-3 * mag)
    assert np.array_equal(again, got[perm])   # a row's score never depends on its block


def test_dfm_catalog_item_column_permuted():
    """ITEM mode keeps the catalog's item column on MFMA whichever column it
    is (here 2: the kernel's field order becomes [2, 0, 1, 3, 4] and layer
    0's packed weights, the projection and the Σw weights follow it), against
    the bf16-rounding oracle's top-K."""
    from hhfm_amd import ops
    rng = np.random.default_rng(21)
    nu, ni, F, k = 50, 600, 5, 32
    M = nu + ni + 12
    m = _model((nu, ni, M, F, k, [64, 48]), mlp_dtype=torch.bfloat16)
    A = np.stack([rng.integers(0, nu, 29), rng.integers(nu + ni, nu + ni + 7, 29),
                  rng.integers(nu, nu + ni, 29), rng.integers(nu + ni + 7, nu + ni + 9, 29),
                  rng.integers(nu + ni + 9, M, 29)], 1).astype(np.int32)
    W = m.get_weights()
    Ls = [W["layer_0"], W["layer_1"]]
    Bs = [W["bias_0"], W["bias_1"]]
    rows = np.repeat(A, ni, 0)
    rows[:, 2] = np.tile(np.arange(nu, nu + ni), len(A))
    sc = _bf16_oracle(rows, W["feature_embeddings"], W["feature_bias"][:, 0], Ls, Bs,
                      W["concat_projection"], float(W["concat_bias"])).reshape(len(A), ni)
    Wt, bs, dims, Wp, bp = m._prepared()
    q = torch.from_numpy(A).cuda()
    rs, ri = orc.top_k(sc, 20)
    tol = 5e-3 * np.abs(sc).max(1, keepdims=True)
    for proj in (False, "item"):
        s, i = ops.dfm_catalog_topk(q, m.table, m.weights["feature_bias"].reshape(-1), Wt, bs,
                                    dims, Wp, bp, 2, nu, ni, 20, 0, 1 << 20, proj=proj)
        bad, swaps = orc.topk_swaps(sc, ri, i.cpu().numpy(), tol)
        assert bad == 0 and swaps == 0, (proj, bad, swaps)


def test_dfm_misaligned_weights_plan_direct():
    """A Wt view that is 4-B but not 16-B aligned (the fused kernels' LDS-DMA
    needs 16 B) makes AUTO plan the direct path instead of failing with
    EUNSUPPORTED after P was computed (mlp_gemm.hip wt_aligned): the scores
    equal the aligned call's direct-path scores within the fp32 tolerance."""
    from hhfm_amd import ops
    rng = np.random.default_rng(99)
    nu, ni, F, k = 100, 200, 5, 64
    M = nu + ni + 12
    m = _model((nu, ni, M, F, k, [150, 200, 150]))
    B = 4 * M                                       # AUTO projects (rows >= 2·M)
    X = rng.integers(0, M, size=(B, F)).astype(np.int32)
    W = m.get_weights()
    Ls = [W[f"layer_{i}"] for i in range(3)]
    Bs = [W[f"bias_{i}"] for i in range(3)]
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    Wt, bs, dims, Wpd, bpd = m._prepared()
    shifted = []
    for t in Wt:
        buf = torch.empty(t.numel() + 1, dtype=t.dtype, device=t.device)
        v = buf[1:].view(t.shape)
        v.copy_(t)
        assert v.data_ptr() % 16 != 0
        shifted.append(v)
    xd = torch.from_numpy(X).cuda()
    wb = m.weights["feature_bias"].reshape(-1)
    got = ops.dfm_forward(xd, m.table, wb, shifted, bs, dims, torch.float32, Wpd, bpd,
                          proj=None).cpu().numpy()
    _f32_check(got, X, E, w, Ls, Bs, Wp, bp)
    q = torch.from_numpy(X[:7]).cuda()
    s, i = ops.dfm_catalog_topk(q, m.table, wb, shifted, bs, dims, Wpd, bpd, 1, nu, ni, 20, 0,
                                1 << 20, proj=None)
    s2, i2 = ops.dfm_catalog_topk(q, m.table, wb, Wt, bs, dims, Wpd, bpd, 1, nu, ni, 20, 0,
                                  1 << 20, proj=False)
    assert np.array_equal(i.cpu().numpy(), i2.cpu().numpy())


@pytest.mark.parametrize("tdt", ["f32", "bf16"])
def test_dfm_f32_split_grouped(tdt):
    """fp32 MLP, projected layer 0, hidden layers on split-bf16 MFMA
    (dfm_fused_f32s) with the rows grouped by user (rows >= 64 x table rows):
    1e-5 relative of the float64 reference graph (κ <= 100), a row's score
    independent of its block (a permuted batch gives the permuted scores bit
    for bit).  Every plan alternative is forced by a plan flag and checked
    the same way: P rows read through the caches instead of LDS-staged
    (PLAN_UNSTAGED, same bits), the FM part from the table rows instead of
    the pair table (PLAN_ROW_FM; staged and grid-stride row kernels give the
    same bits), ungrouped rows, exact-fp32 hidden layers."""
    from hhfm_amd import ops
    rng = np.random.default_rng(64)
    F, k, M, users, B = 5, 64, 997, 40, 70000
    tdtype = torch.bfloat16 if tdt == "bf16" else torch.float32
    m = _model((users, 400, M, F, k, [150, 200, 150]), table_dtype=tdtype)
    X = rng.integers(0, M, size=(B, F)).astype(np.int32)
    X[:, 0] = rng.integers(0, users, B)
    W = m.get_weights()
    Ls = [W[f"layer_{i}"] for i in range(3)]
    Bs = [W[f"bias_{i}"] for i in range(3)]
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    if tdt == "bf16":
        E = bf16_round(E)
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    Wt, bs, dims, Wpd, bpd = m._prepared()
    wb = m.weights["feature_bias"].reshape(-1)
    xd = torch.from_numpy(X).cuda()

    def run(x, plan=0):
        return ops.dfm_forward(x, m.table, wb, Wt, bs, dims, torch.float32, Wpd, bpd,
                               proj=True, plan=plan).cpu().numpy()

    got = run(xd)
    perm = rng.permutation(B)
    again = run(xd[torch.from_numpy(perm).cuda()])
    assert np.array_equal(again, got[perm])
    unstaged = run(xd, ops.PLAN_UNSTAGED)                # P rows from HBM/L2 only
    assert np.array_equal(unstaged, got)                 # same values, same order
    rows_fm = run(xd, ops.PLAN_ROW_FM)                   # FM part from the table rows
    fmb = run(xd, ops.PLAN_ROW_FM | ops.PLAN_UNSTAGED)   # ... by the grid-stride kernel
    assert np.array_equal(fmb, rows_fm)
    flat = run(xd, ops.PLAN_UNGROUPED)
    exact = run(xd, ops.PLAN_UNGROUPED | ops.PLAN_EXACT_FP32)
    ref32 = orc.dfm_out(X, E, w, Ls, Bs, Wp, bp)[:, 0]
    for v in (got, flat, exact, rows_fm):
        _f32_check(v, X, E, w, Ls, Bs, Wp, bp, ref32=ref32)


@pytest.mark.parametrize("B,N", [(1, 4082), (300, 4082), (1024, 32768), (3000, 4082),
                                 (77, 1100), (5000, 2048)])
def test_topk_dense_split_waves(B, N):
    """Dense top-K with 4 or 2 waves per query (few queries, N >= 1,024: each
    wave folds a 64-aligned slice, the first merges the lists) equals one wave
    per query bit for bit and np.argsort's (score desc, index asc) order,
    heavy ties included."""
    from hhfm_amd import ops
    rng = np.random.default_rng(B + N)
    S = rng.integers(0, 200, size=(B, N)).astype(np.float32)   # many exact ties
    S[:, ::7] += rng.normal(size=(B, (N + 6) // 7)).astype(np.float32)
    Sd = torch.from_numpy(S).cuda()
    for K in (1, 20, 64):
        s, i = ops.topk_dense(Sd, K, 3)
        s1, i1 = ops.topk_dense(Sd, K, 3, plan=ops.PLAN_ONE_WAVE)
        assert torch.equal(i, i1) and torch.equal(s, s1)
        rs, ri = orc.top_k(S, K)
        assert np.array_equal(i.cpu().numpy(), ri + 3)
        assert np.array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("k,layers,B,grouped", [(256, [400, 400, 400], 50000, True),
                                                (256, [400, 400, 400], 3000, False),
                                                (64, [150, 150, 150], 20000, True),
                                                (64, [150, 150, 150], 777, False),
                                                (64, [150, 150, 150], 90001, True),
                                                (256, [400, 400, 400], 81000, False),
                                                (64, [150, 150, 150], 20000, "mixed"),
                                                (256, [400, 400, 400], 82000, "mixed")])
def test_dfm_wide_item(k, layers, B, grouped):
    """The wide ITEM kernel (dfm_wide.hip, 256 rows per workgroup; shapes it is instantiated for:
    F = 5 with k = 256 / 3 x 400 — C5 — and k = 64 / 3 x 150): against the
    bf16-rounding oracle (5e-3 of the magnitude) and the 128-row kernel
    (PLAN_NARROW), with rows grouped by user (blocks stage their P and table
    rows in LDS) and with random ids (blocks read them from memory, B not a
    multiple of 256) — those blocks run in the overflow launch — and mixed
    (grouped, a few rows with random context ids: most blocks staged, some in
    the overflow launch); a row's score never depends on its block.  B >= 16 x
    the table's 5,051 rows (the last two cases) takes the FM part from the
    pair table (dfm_wide PAIRS, the default C5 kernel), else from the rows;
    the FM-rows variant (PLAN_ROW_FM) is compared there too."""
    from hhfm_amd import ops
    rng = np.random.default_rng(k + B)
    nu, ni, ctx = 957, 4082, (7, 2, 3)
    M = nu + ni + sum(ctx)
    m = _model((nu, ni, M, 5, k, layers), mlp_dtype=torch.bfloat16,
               table_dtype=torch.bfloat16)
    cols = [rng.integers(0, nu if grouped else M, B), rng.integers(nu, nu + ni, B)]
    off = nu + ni
    for c in ctx:
        cols.append(rng.integers(off, off + c, B) if grouped else rng.integers(0, M, B))
        off += c
    X = np.stack(cols, 1).astype(np.int32)
    if grouped == "mixed":
        wild = rng.random(B) < 0.002
        X[wild, 2:] = rng.integers(0, M, (int(wild.sum()), 3))
    W = m.get_weights()
    Ls = [W[f"layer_{i}"] for i in range(3)]
    Bs = [W[f"bias_{i}"] for i in range(3)]
    E, w = bf16_round(W["feature_embeddings"]), W["feature_bias"][:, 0]
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    Wt, bs, dims, Wpd, bpd = m._prepared()
    wb = m.weights["feature_bias"].reshape(-1)
    xd = torch.from_numpy(X).cuda()

    def run(x, plan=0):
        return ops.dfm_forward(x, m.table, wb, Wt, bs, dims, torch.bfloat16, Wpd, bpd,
                               proj="item", plan=plan).cpu().numpy()

    got = run(xd)
    old = run(xd, ops.PLAN_NARROW)
    perm = rng.permutation(B)
    again = run(xd[torch.from_numpy(perm).cuda()])
    mag = _magnitude(X, E, w, Ls, Bs, Wp, bp)
    ref = _bf16_oracle(X, E, w, Ls, Bs, Wp, bp)
    assert np.all(np.abs(got - ref) <= 5e-3 * mag), np.max(np.abs(got - ref) / mag)
    assert np.all(np.abs(got - old) <= 5e-3 * mag), np.max(np.abs(got - old) / mag)
    assert np.array_equal(again, got[perm])
    if B >= 16 * M:
        rows_fm = run(xd, ops.PLAN_ROW_FM)
        assert np.all(np.abs(rows_fm - ref) <= 5e-3 * mag), np.max(np.abs(rows_fm - ref) / mag)
    if k == 64:
        # every workgroup shape the kernel template admits (16-row tiles per
        # wave x waves: 3x4, 2x4, 1x4 besides the default 2x8): bit-identical
        for shape in (ops.PLAN_WIDE_3X4, ops.PLAN_WIDE_2X4, ops.PLAN_WIDE_1X4):
            alt = run(xd, shape)
            assert np.all(np.abs(alt - ref) <= 5e-3 * mag), (shape, np.max(np.abs(alt - ref) / mag))
            assert np.array_equal(alt, got), shape
