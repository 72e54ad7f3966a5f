"""bench.py's legs on the device: the C4 catalog is a function of the global
item index (so the top-20 checksum is the same for every rank count), the
sharded C4 step equals the unsharded one, and the probes return sane values."""
import numpy as np
import pytest
import torch

import bench

pytestmark = pytest.mark.gpu


def test_item_rows_depend_on_global_index_only():
    dev = torch.device("cuda", 0)
    full = bench.item_rows(0, 200_000, 16, dev)
    for a, b in [(0, 1), (65_535, 65_537), (70_001, 199_999), (131_072, 200_000)]:
        assert torch.equal(bench.item_rows(a, b, 16, dev), full[a:b])


def test_c4_shards_merge_to_the_unsharded_top20():
    """The bench's C4 decomposition (rank tables [users | ctx | shard items],
    local top-K with global ids, merge) at world 1, 2 and 3 on one device."""
    from hhfm_amd import distributed as hd
    from hhfm_amd import ops
    dev = torch.device("cuda", 0)
    nu, ni, k, B, K = 5000, 300_000, 128, 256, 20
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    users = torch.empty(nu, k, device=dev).normal_(0, 0.01, generator=g)
    ctx = torch.empty(12, k, device=dev).normal_(0, 0.01, generator=g)
    A = torch.stack([torch.randint(0, nu, (B,), generator=g, device=dev),
                     torch.zeros(B, dtype=torch.int64, device=dev),
                     nu + torch.randint(0, 7, (B,), generator=g, device=dev),
                     nu + 7 + torch.randint(0, 2, (B,), generator=g, device=dev),
                     nu + 9 + torch.randint(0, 3, (B,), generator=g, device=dev)],
                    1).to(torch.int32).contiguous()
    res = {}
    for world in (1, 2, 3):
        parts = []
        for r in range(world):
            b0, b1 = hd.shard_range(ni, world, r)
            E = torch.cat([users, ctx, bench.item_rows(b0, b1, k, dev)]).contiguous()
            parts.append(ops.catalog_topk(A, E, ops.MODE_HHFM, K, nu + 12, b1 - b0, b0, None,
                                          0, (2, 5), (0, 0)))
        if world == 1:
            s, i = parts[0]
        else:
            s, i = ops.topk_merge(torch.stack([p[0] for p in parts]),
                                  torch.stack([p[1] for p in parts]))
        res[world] = (bench._sha(i), bench._sha(s))
    assert res[1] == res[2] == res[3], res


def test_stream_read_probe_and_c5_leg_run():
    dev = torch.device("cuda", 0)
    buf = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
    gbs, var = bench.stream_read_peak(buf, reps=3)
    assert 500 < gbs < 20000 and len(var) == 3, (gbs, var)
    r = bench.c5_leg(dev, 1, 0, 100_000, reps=1)
    assert np.isfinite(r["rows_per_s"]) and r["roofline"]["frac"] > 0
    r = bench.c5_leg(dev, 1, 0, 100_000, reps=1, mlp=torch.float32)   # projected layer 0
    assert np.isfinite(r["rows_per_s"]) and 0 < r["roofline"]["frac"] < 1
