"""World-size-2 (and 3) gloo runs of the item-sharded top-K path: shard
split, all-gather, host merge == single-device ranking.  The per-shard scorer
is the C oracle here (no GPU); on the box the same code runs the HIP scorer
and RCCL (tests/test_gpu_models.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hhfm_amd import distributed as hd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cpu as ocpu
    from oracle import fm_oracle as orc
    from tests.helpers import synth_rows, table
    rng = np.random.default_rng(42)
    nu, ni = 300, 5000 if mode != "afm" else 1200
    A, M = synth_rows(rng, 64, nu, ni, (7, 2, 3))
    E = table(rng, M, 32)
    E[nu + 100] = E[nu + 1100]                  # a cross-shard exact tie
    w = rng.normal(0, 0.01, M).astype(np.float32)
    if mode == "afm":                           # AFM.py:209-246 (numpy oracle)
        W = rng.normal(0, 0.2, (32, 16)).astype(np.float32)
        b = rng.normal(0, 0.2, (1, 16)).astype(np.float32)
        pv = rng.normal(0, 1, 16).astype(np.float32)
        P = np.ones((32, 1), np.float32)
        full = orc.afm_catalog_scores(A, E, w, W, b, pv, P, nu, ni)

    def scorer(A_, begin, count, K):
        if mode == "afm":
            s, i = orc.top_k(full[:, begin:begin + count], K)
            return torch.from_numpy(np.ascontiguousarray(s)), \
                torch.from_numpy((i + begin).astype(np.int32))
        s, i = ocpu.catalog_topk(A_, E, 0 if mode == "fm" else 1, K, nu + begin, count,
                                 w=w if mode == "fm" else None, ctx=(2, 5), threads=1)
        return torch.from_numpy(s), torch.from_numpy(i + begin)

    s, i = hd.sharded_topk(A, 20, ni, scorer)
    if rank == 0:
        if mode == "afm":
            rs, ri = orc.top_k(full, 20)
        else:
            rs, ri = ocpu.catalog_topk(A, E, 0 if mode == "fm" else 1, 20, nu, ni,
                                       w=w if mode == "fm" else None, ctx=(2, 5), threads=1)
        q.put((np.array_equal(i.numpy(), ri), float(np.abs(s.numpy() - rs).max())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "hhfm"), (3, "hhfm"), (2, "fm"), (2, "afm")])
def test_sharded_topk_gloo(world, mode):
    """Item-sharded top-K (shard split, one packed all-gather, host merge) ==
    the single-device ranking, HHFM / FM / AFM score modes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    same, err = q.get(timeout=10)
    assert same and err == 0.0


def test_model_scorer_rejects_unknown_models():
    with pytest.raises(TypeError):
        hd.model_scorer(object())


def test_shard_range_partition():
    for n in [1, 7, 4082, 10_000_000]:
        for w in [1, 2, 3, 8]:
            rs = [hd.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(e - b for b, e in rs) - min(e - b for b, e in rs) <= 1


def _auc_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import json
    from hhfm_amd.NewLoadData import LoadData
    from tests.test_harness import G, OracleModel, make
    np.random.seed(2016)
    d = LoadData(G + "/", "synth_frappe")
    arr = np.load(os.path.join(G, "harness.npz"))
    with open(os.path.join(G, "harness.json")) as f:
        ref = json.load(f)
    m = OracleModel(arr["E"], arr["w"], d.n_user, d.n_item)
    np.random.seed(13)
    a_fm = hd.sharded_evaluate_auc(make(d, m), d.Test_data)
    mh = OracleModel(arr["E"], arr["w"], d.n_user, d.n_item, fm_scores=False)
    np.random.seed(17)
    a_h = hd.sharded_evaluate_auc(make(d, mh, auc_first_chunk_only=True, auc_label_filter=False),
                                  d.Train_data)
    if rank == 0:
        q.put((a_fm == ref["fm_auc_test"], a_h == ref["hhfm_auc_train"]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_auc_gloo(world):
    """Row-sharded evaluate_AUC + one scalar all-reduce == the reference
    harness's AUC (fixture), FM and HHFM first-chunk variants."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_auc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    assert q.get(timeout=10) == (True, True)


def _rows_worker(rank, world, port, q, n):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import fm_oracle as orc
    from tests.helpers import synth_rows, table
    rng = np.random.default_rng(7)
    A, M = synth_rows(rng, n, 300, 900, (7, 2, 3))
    E = table(rng, M, 16)
    w = rng.normal(0, 0.01, M).astype(np.float32)
    layers = [rng.normal(0, 0.1, (5 * 16, 24)).astype(np.float32),
              rng.normal(0, 0.1, (24, 12)).astype(np.float32)]
    biases = [rng.normal(0, 0.1, 24).astype(np.float32), rng.normal(0, 0.1, 12).astype(np.float32)]
    Wp = rng.normal(0, 0.1, 5 + 16 + 12).astype(np.float32)
    fm = hd.sharded_score_rows(A, lambda X: orc.fm_out(X, E, w, 0.1))
    dfm = hd.sharded_score_rows(A, lambda X: orc.dfm_out(X, E, w, layers, biases, Wp, 0.2))
    mine, b = hd.sharded_score_rows(A, lambda X: orc.fm_out(X, E, w, 0.1), gather=False)
    if rank == 0:
        q.put((np.array_equal(fm.numpy(), np.asarray(orc.fm_out(A, E, w, 0.1), np.float32).reshape(-1)),
               # (the numpy oracle's BLAS may block a matmul differently per
               # batch size: DeepFM within 1e-6 relative; the GPU kernels'
               # row scores are batch-independent)
               bool(np.allclose(dfm.numpy(), np.asarray(orc.dfm_out(A, E, w, layers, biases, Wp,
                                                                   0.2), np.float32).reshape(-1),
                                rtol=1e-6, atol=1e-7)),
               b == 0 and mine.numel() == hd.shard_range(n, world, 0)[1]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 101), (3, 64), (3, 2)])
def test_sharded_score_rows_gloo(world, n):
    """Row-sharded FM / DeepFM scoring (C2 / C5 over N ranks: contiguous row
    slices, one padded all-gather) == the single-process scores (FM bit for
    bit), including ragged splits and a rank with no rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q, n)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) == (True, True, True)
