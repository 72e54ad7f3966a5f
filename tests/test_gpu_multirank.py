"""Two ranks on one GPU (gloo): the item-sharded top-K and the row-sharded
scoring with the PRODUCT scorers (the HIP catalog and row kernels of every
model class), not the oracle.  Each rank scores its shard on cuda:0; the
lists cross the gloo all-gather in host memory (distributed.comm_device) and
are merged there — the code path RCCL runs with device payloads.  The merged
top-20 must equal the model's own single-process topk and the golden list
the reference graph produced; the gathered row scores must equal the
single-process HIP scores bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hhfm_amd import distributed as hd
    from tests.test_gpu_models import _golden_model
    res = {}
    for name in ("hhfm_frappe", "fm", "afm", "dfm"):
        m, d = _golden_model(name)
        got = hd.sharded_model_topk(m, d["A"], 20)
        one = m.topk(d["A"], 20)
        rows = np.asarray(hd.sharded_score_rows(d["X"], m.score_rows)).reshape(-1)
        ref_rows = np.asarray(m.score_rows(d["X"])).reshape(-1)
        res[name] = (bool(np.array_equal(got, one)), bool(np.array_equal(got, d["topk_idx"])),
                     bool(np.array_equal(rows, ref_rows)))
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


def test_two_ranks_product_scorers():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    res = q.get(timeout=10)
    for name, (same_one, same_golden, rows_equal) in res.items():
        assert same_one, f"{name}: merged top-20 != single-process topk"
        assert same_golden, f"{name}: merged top-20 != golden reference list"
        assert rows_equal, f"{name}: row-sharded scores != single-process scores"
