#!/usr/bin/env python3
"""Headline benchmark: FM per-row scoring (K1, hhfm_fm_score_rows) on the
BASELINE.json configs[1] workload — "FM k=64 Frappe-shape synthetic,
1xMI355X HIP gather+interaction kernel, fp32" — in its HBM-roofline variant
(SURVEY.md §8d C2(ii)): 8 M users + 8 M items + the 12 Frappe context ids,
table 16.8 M x 64 fp32 (4.3 GB, far beyond the 256 MB Infinity Cache),
2^25 uniformly random Frappe-layout rows [user, item, daytime, isweekend,
homework] per step and GPU, seed 1 (+rank).

A step = one hhfm_fm_score_rows launch over the resident batch (inputs in
HBM before the timed region).  Multi-GPU: one process per GPU, rows sharded
(weak scaling, no data-path collective); value = all ranks' rows / max time.
`--gpus N` without a torch.distributed environment re-launches itself under
torch.distributed.run with N ranks (a child process, started before anything
touches the GPU); the driver's own torchrun launch takes the same path.

Prints ONE JSON line (rank 0).  See DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
if os.environ.get("HHFM_AB_ROOT"):   # diagnostic A/B: another build's package copy first
    sys.path.insert(0, os.environ["HHFM_AB_ROOT"])

METRIC = "scored (user,ctx,item) triples/sec + HR@10, Frappe-shape, 1/2/4/8 MI355X"
BYTES_PER_ROW_F5_K64 = 5 * 64 * 4 + 5 * 4 + 5 * 4 + 4   # 1,324 B
HBM_PEAK_GBS = 8000.0                                   # MI355X_MICROARCH.md (spec)
CTX_CARD = (7, 2, 3)                                    # Frappe daytime/isweekend/homework


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rows", type=int, default=1 << 25)
    p.add_argument("--users", type=int, default=8 << 20)
    p.add_argument("--items", type=int, default=8 << 20)
    p.add_argument("--k", type=int, default=64)
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="CPU-baseline time budget (0 disables)")
    p.add_argument("--cpu-rows", type=int, default=1 << 21)
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_fm_rows.json"),
                   help="calibrated PMC bytes/row, used only when the in-run PMC passes "
                        "cannot run (no rocprofv3, --no-pmc, or a failed pass)")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the in-run rocprofv3 --pmc passes for roofline.traffic")
    p.add_argument("--legs", default="hr,catalog,catalog_bf16,c3,c5",
                   help="extra legs: hr (HR@10 identity after GPU training on Frappe-shape "
                        "data), catalog / catalog_bf16 (C4 item-sharded top-K over an fp32 / "
                        "bf16 table, RCCL all-gather at N>1), c3 (configs[2]: Frappe-catalog "
                        "top-20, rank 0), c5 (configs[4]: DeepFM k=256 3x400 bf16 MLP, "
                        "12.5M rows per GPU)")
    p.add_argument("--hr-epochs", type=int, default=5)
    p.add_argument("--c5-rows", type=int, default=12_500_000)
    p.add_argument("--no-check", action="store_true",
                   help="skip the legs' oracle parity checks (timing only)")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: every rank joins a gloo group and "
                        "rank 0 prints the world it saw")
    return p.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`--gpus N` outside a torch.distributed environment: run this script
    under torch.distributed.run with N ranks, one per GPU, as a CHILD process
    (this process has not touched the GPU), and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dry_run(args):
    """Launcher check (no GPU): each rank joins a gloo group; rank 0 prints
    the ranks it gathered."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    ranks = [rank]
    if world > 1:
        dist.init_process_group("gloo")
        got = [None] * world
        dist.all_gather_object(got, (rank, int(os.environ.get("LOCAL_RANK", "0"))))
        ranks = got
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "gpus_arg": args.gpus, "world": world,
                          "ranks": ranks}), flush=True)


def make_batch(rows, n_user, n_item, k, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    M = n_user + n_item + sum(CTX_CARD)
    E = torch.empty(M, k, dtype=torch.float32, device=dev)
    E.normal_(0.0, 0.01, generator=g)                       # tf.random_normal(0, 0.01), FM.py:153
    w = torch.empty(M, dtype=torch.float32, device=dev).normal_(0.0, 0.01, generator=g)
    cols = [torch.randint(0, n_user, (rows,), generator=g, device=dev, dtype=torch.int32),
            torch.randint(n_user, n_user + n_item, (rows,), generator=g, device=dev,
                          dtype=torch.int32)]
    off = n_user + n_item
    for c in CTX_CARD:
        cols.append(torch.randint(off, off + c, (rows,), generator=g, device=dev,
                                  dtype=torch.int32))
        off += c
    idx = torch.stack(cols, 1).contiguous()
    return idx, E, w, M


def _cpu_quota():
    """Cores the cgroup CPU quota allows (None when unlimited/unreadable)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


def _cpu_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "cpu"


def cpu_baseline(idx, E, w, w0, out_gpu, args):
    """Time the oracle's C restatement of FM.out (oracle/cpu_oracle.c, OpenMP)
    on this box's host cores over a bounded sample of the same workload (same
    4.3 GB table, the batch's first rows): one thread, OMP_NUM_THREADS (the
    box's CPU share), and every core of the affinity mask.  Also the GPU's
    parity on a subset, elementwise and normwise."""
    from oracle import cpu as ocpu
    from oracle import parity
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    n = min(args.cpu_rows, idx.shape[0])
    X = idx[:n].cpu().numpy()
    Eh = E.cpu().numpy()
    wh = w.cpu().numpy()
    ref = ocpu.fm_out(X, Eh, wh, w0, min(share, aff))          # warm (page-in)

    def timed(threads, rows, budget):
        Xs = X[:rows]
        ocpu.fm_out(Xs, Eh, wh, w0, threads)
        reps, t0 = 0, time.perf_counter()
        while True:
            ocpu.fm_out(Xs, Eh, wh, w0, threads)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return reps * rows / el, reps
    budget = args.cpu_seconds / 3
    legs = {}
    r1, reps1 = timed(1, min(n, 1 << 18), budget)
    legs["1"] = {"threads": 1, "triples_per_s": r1, "rows": min(n, 1 << 18), "passes": reps1}
    for t in sorted({min(share, aff), aff}):
        r, reps = timed(t, n, budget)
        legs[str(t)] = {"threads": t, "triples_per_s": r, "rows": n, "passes": reps}
    best = max((v for v in legs.values() if v["threads"] > 1), key=lambda v: v["triples_per_s"],
               default=legs["1"])
    m = min(n, 1 << 16)                                 # parity spot-check subset
    got = out_gpu[:m].cpu().numpy().astype(np.float64)
    rf = ref[:m].astype(np.float64)
    ex, scale = parity.fm_rows_exact(X[:m], Eh, wh, w0)
    err = np.abs(got - rf)
    rel = err / np.maximum(np.abs(rf), 1e-30)
    vs_exact = parity.row_check(got, ex, scale)
    vs_exact["cpu_oracle_max_rel_err_kappa_le_max"] = parity.row_check(
        rf, ex, scale)["max_rel_err_kappa_le_max"]
    return {"value": best["triples_per_s"], "unit": "triples/s", "cores": best["threads"],
            "kind": "port",
            "sample": f"first {n} rows of the same batch (same 4.3 GB table), "
                      f"oracle/cpu_oracle.c (OpenMP) on {_cpu_name()}; single thread on "
                      f"{legs['1']['rows']} rows",
            "single_thread_triples_per_s": r1, "threads_legs": legs,
            "affinity_cores": aff, "cgroup_cpu_quota_cores": _cpu_quota(),
            "gpu_vs_cpu": {"rows": m, "max_rel_err_elementwise": float(rel.max()),
                           "rows_rel_err_gt_1e-5": int((rel > 1e-5).sum()),
                           "max_rel_err_normwise": float((err / scale).max()),
                           "note": "elementwise |gpu-cpu|/|cpu|; rows above 1e-5 are "
                                   "cancellations ((Σv)²≈Σv², |out| << Σ|terms|), bounded "
                                   "by the normwise figure"},
            "gpu_vs_float64": dict(vs_exact, note=(
                "GPU rows vs the float64 value of FM.py:99-120 (oracle/parity.row_check): "
                "rows with κ = Σ|terms|/|out| <= 100 within 1e-5 relative, the rest within "
                "1e-5 of Σ|terms|; the fp32 C oracle's own error on the same rows beside it"))}


def frappe_shape_dataset(path, rows=96203, seed=11):
    """A synthetic libfm file with Frappe's shape: 957 users, 4082 items,
    daytime/isweekend/homework with 7/2/3 values, 96,203 rows, popularity
    skew (no Frappe rows are used or shipped)."""
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(path, "frappe_shape"), exist_ok=True)
    fn = os.path.join(path, "frappe_shape", "frappe_shape.libfm")
    users = rng.zipf(1.3, rows) % 957
    pref = rng.integers(0, 4082, 957)            # each user's taste centre
    items = (pref[users] + (rng.zipf(1.4, rows) % 4082) * rng.choice([-1, 1], rows)) % 4082
    day = rng.integers(0, 7, rows)
    wk = rng.integers(0, 2, rows)
    hw = rng.integers(0, 3, rows)
    with open(fn, "w") as f:
        for u, i, d, w_, h in zip(users, items, day, wk, hw):
            f.write(f"1 u{u} i{i} d{d} w{w_} h{h}\n")
    return path + "/"


def hr_leg(dev, epochs):
    """Load -> train HHFM (k=64, the reference hyper-parameters) on the GPU ->
    evaluate_TopK(TopK=10) with the GPU model and with the oracle model holding
    the same weights and the same sampled rows: HR@10 must be identical."""
    import tempfile
    from hhfm_amd.NewLoadData import LoadData
    from hhfm_amd.OurModel7 import OUR
    from hhfm_amd.harness import Train
    from hhfm_amd import training
    from oracle import fm_oracle as orc

    class _Oracle:
        def __init__(self, E, nu, ni):
            self.E, self.nu, self.ni = E, nu, ni

        def score_rows(self, X):
            return orc.hhfm_positive_feedback(X, self.E, 3, 0)

        def topk(self, A, tp):
            return orc.hhfm_topk(A, self.E, self.nu, self.ni, 3, 0, tp=tp)[1]

    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as tmp:
        np.random.seed(2016)
        data = LoadData(frappe_shape_dataset(tmp), "frappe_shape")
    m = OUR(3, 0, data.features_M, data.n_user, data.n_item, 64, 0.1, 0.01, "AdagradOptimizer",
            True, False, device=dev)
    tr = Train(data=data, model=m)
    tr.batch_size, tr.epoch, tr.TopK = 5000, epochs + 1, 10
    tr.context, tr.time, tr.time_dimension = True, False, 0
    tr.args = argparse.Namespace(Result=-1, result_file=None, dataset="frappe_shape")
    losses = training.run_training_hhfm(tr)
    t_train = time.perf_counter() - t0
    res = {}
    for name, model in (("gpu", m), ("oracle", _Oracle(m.get_weights()["feature_embeddings"],
                                                       data.n_user, data.n_item))):
        tr.model = model
        np.random.seed(2024)
        res[name] = [float(x) for x in tr.evaluate_TopK(data.Test_data)]
    return {"hr10": res["gpu"][0], "ndcg10": res["gpu"][1], "pre10": res["gpu"][2],
            "oracle_hr10": res["oracle"][0], "identical_to_oracle": res["gpu"] == res["oracle"],
            "data": "Frappe-shape synthetic (957 users, 4082 items, ctx 7/2/3, 96,203 rows), "
                    "LoadData split seed 2016",
            "model": f"HHFM k=64 trained {epochs} epochs on the GPU (partial_fit kernels), "
                     "evaluate_TopK TopK=10 (3000 rows)",
            "epoch_loss": losses, "train_s": t_train}


def _oracle_threads():
    aff = len(os.sched_getaffinity(0))
    return min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff, aff)


def _topk_parity(got_s, got_i, ref_i, exact, rel=1e-5):
    """Top-K parity record (oracle/parity.py contract): ids equal to the
    oracle's at every position but float64-verified fp32 ties (counted), every
    returned score within 1e-5 relative of its float64 value, lists sorted."""
    from oracle import parity
    got_s = np.asarray(got_s)
    got_i = np.asarray(got_i)
    bad, swaps, dup = parity.topk_tie_count(got_i, ref_i, exact)
    ex = np.empty(got_s.shape)
    mag = np.empty(got_s.shape)
    for b in range(got_i.shape[0]):
        ex[b], mag[b] = exact(b, got_i[b])
    err = np.abs(got_s - ex)
    relerr = float((err / np.maximum(np.abs(ex), 1e-300)).max())
    normwise = float((err / np.maximum(mag, 1e-300)).max())
    ordered = bool(np.all(np.diff(got_s, axis=1) <= 0))
    return {"queries": int(got_i.shape[0]), "positions": int(got_i.size),
            "ids_equal_to_oracle": bool(np.array_equal(got_i, ref_i)),
            "tie_swaps": swaps, "unexplained": bad, "duplicates": dup,
            "max_rel_err_scores_vs_float64": relerr, "max_normwise_err": normwise,
            "sorted": ordered,
            "parity": bad == 0 and dup == 0 and ordered and normwise <= rel and relerr <= rel}


def catalog_c3_leg(dev, reps=200):
    """configs[2] / C3: HHFM k=64, bf16 table, Frappe vocabulary (957 users,
    4,082 items, ctx 7/2/3), 3,000 queries, top-20 over the full catalog
    (hhfm_catalog_topk: STORE score matrix + dense top-K); beside it the
    reference's own call shape, one topk(A[300], 20) (FM.py:333-334,
    OurModel7.py:471), and the 3,000-query top-20 checked against
    oracle/cpu_oracle.c (same bf16-rounded table)."""
    from hhfm_amd import ops
    from oracle import cpu as ocpu
    from oracle import parity
    nu, ni, ctx, k, B = 957, 4082, (7, 2, 3), 64, 3000
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    M = nu + ni + sum(ctx)
    E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(torch.bfloat16)
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
    off = nu + ni
    for c in ctx:
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()

    def timed(Aq, n):
        def step():
            return ops.catalog_topk(Aq, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5),
                                    (0, 0))
        # back-to-back calls, n of them between two synchronizes: the first
        # launch's latency and the final synchronize are a fixed ~20 us, so n
        # is sized to make them < 0.5 % of the per-call time
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    ms = timed(A, reps)
    A300 = A[:300].contiguous()
    ms300 = timed(A300, 4 * reps)
    s, i = ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0))
    torch.cuda.synchronize()
    Ah = A.cpu().numpy()
    Ef = E.float().cpu().numpy()
    t0 = time.perf_counter()
    rs, ri = ocpu.catalog_topk(Ah, Ef, 1, 20, nu, ni, ctx=(2, 5), threads=_oracle_threads())
    par = _topk_parity(s.cpu().numpy(), i.cpu().numpy(), ri, parity.hhfm_exact(Ah, Ef, nu))
    par["oracle"] = "oracle/cpu_oracle.c oracle_catalog_topk mode 1 (OurModel7.py:294 + " \
                    "tf.nn.top_k order), all 3,000 queries"
    par["oracle_s"] = time.perf_counter() - t0
    pairs = B * ni
    return {"workload": "C3 (configs[2]): HHFM k=64 bf16 table, Frappe vocabulary, 3,000 "
                        "queries x 4,082 items, top-20, one GPU", "ms_per_query_batch": ms,
            "pairs_per_s": pairs / (ms * 1e-3), "TFLOPs": 2.0 * k * pairs / (ms * 1e-3) / 1e12,
            "reference_call_300_queries_us": ms300 * 1e3,
            "reference_call_note": "one topk(A[300], 20) as FM.py:333-334 / OurModel7.py:471 "
                                   "call it (evaluate_TopK's 300-row batches), host-timed "
                                   "back to back",
            "parity": par}


ITEM_BLOCK = 1 << 16


def item_rows(begin, end, k, dev, seed=3_000_000):
    """Rows of catalog items [begin, end) as a function of the GLOBAL item
    index: block j of 65,536 items is drawn from its own seeded generator, so
    every rank count N builds the same catalog and the top-K must match."""
    out = torch.empty(end - begin, k, device=dev)
    j = begin // ITEM_BLOCK
    while j * ITEM_BLOCK < end:
        b0, b1 = j * ITEM_BLOCK, (j + 1) * ITEM_BLOCK
        g = torch.Generator(device=dev)
        g.manual_seed(seed + j)
        blk = torch.empty(ITEM_BLOCK, k, device=dev).normal_(0, 0.01, generator=g)
        lo, hi = max(b0, begin), min(b1, end)
        out[lo - begin:hi - begin] = blk[lo - b0:hi - b0]
        j += 1
    return out


def _sha(t):
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


# top-20 checksums of the C4 legs at N=1 (profiles/r02_bench_full.json, driver
# BENCH_r02.json): the catalog is a function of the global item index, so
# every N must reproduce them (the RCCL all-gather + merge path's check)
C4_N1_SHA = {"fp32": {"ids": "62574e2b64a438f1", "scores": "6cbbc10b494ce2cc"},
             "bf16": {"ids": "c7c4f5f1a9d97ea3", "scores": "502206c7ac910a91"}}
C4_CHECK_QUERIES = 64


def catalog_leg(dev, world, rank, reps=5, table_dtype=torch.float32, check=True):
    """C4: HHFM k=128, 1 M users, 10 M items sharded contiguously over the
    ranks, 1,024 queries, K=20, fp32 (or bf16) table; local
    hhfm_catalog_topk + one packed RCCL all-gather + hhfm_topk_merge per step.
    Table per rank: [users | 12 ctx | this rank's items]; the catalog is a
    function of the global item index (item_rows), so the top-20 checksum is
    the same for every N and is compared with the committed N=1 value.
    Parity (rank 0, every N): the merged top-20 of the first 64 queries
    against oracle/cpu_oracle.c over the FULL 10 M-item catalog."""
    from hhfm_amd import distributed as hd
    from hhfm_amd import ops
    nu, ni, k, B, K = 1 << 20, 10_000_000, 128, 1024, 20
    begin, end = hd.shard_range(ni, world, rank)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    rows_user = torch.empty(nu, k, device=dev).normal_(0, 0.01, generator=g)
    rows_ctx = torch.empty(12, k, device=dev).normal_(0, 0.01, generator=g)
    E = torch.cat([rows_user, rows_ctx, item_rows(begin, end, k, dev)]).to(table_dtype)
    E = E.contiguous()
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.zeros(B, dtype=torch.int64, device=dev)]
    off = nu
    for c in (7, 2, 3):
        cols.append(torch.randint(0, c, (B,), generator=g, device=dev) + off)
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()
    qc = C4_CHECK_QUERIES
    # the checked queries' user rows + the context rows, as the table stores them
    check_rows = torch.cat([rows_user[A[:qc, 0].long()], rows_ctx]).to(table_dtype).float()
    del rows_user
    row0 = nu + 12                       # this rank's first item row

    def scorer(A_, b0, cnt, Kl):
        return ops.catalog_topk(A_, E, ops.MODE_HHFM, Kl, row0 + (b0 - begin), cnt, b0, None,
                                0, (2, 5), (0, 0))

    def step():
        return hd.sharded_topk(A, K, ni, scorer)

    step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        s, i = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    ms = float(el[0]) / reps * 1e3
    pairs = B * ni
    tname = "fp32" if table_dtype == torch.float32 else "bf16"
    sha = {"ids": _sha(i), "scores": _sha(s)}
    res = {"workload": f"C4: HHFM k=128 {tname} table, 10M-item catalog sharded over ranks, "
                       "1,024 queries, top-20 (local split-bf16 MFMA score + select, one "
                       "packed RCCL all-gather, merge)",
           "ms_per_query_batch": ms, "pairs_per_s": pairs / (ms * 1e-3),
           "TFLOPs": 2.0 * k * pairs / (ms * 1e-3) / 1e12, "ranks": world,
           "top20_ids_sha256": sha["ids"], "top20_scores_sha256": sha["scores"],
           "n1_sha256": C4_N1_SHA[tname],
           "matches_n1": sha == C4_N1_SHA[tname],
           "checksum_note": "catalog seeded by global item index: every N must reproduce the "
                            "committed N=1 checksums (bench.py C4_N1_SHA)"}
    if check and rank == 0:
        res["parity"] = _c4_parity(E, check_rows, A[:qc], s[:qc], i[:qc], world, row0, ni, k,
                                   table_dtype, dev)
    del E
    return res


def _c4_parity(E, check_rows, Aq, s, i, world, row0, ni, k, table_dtype, dev):
    """The merged top-20 of the first queries vs oracle/cpu_oracle.c over the
    whole catalog (OurModel7.py:294 as a k-ordered fp32 chain + tf.nn.top_k
    order), on a compact host table [query users | 12 ctx | all items]."""
    from oracle import cpu as ocpu
    from oracle import parity
    qc = Aq.shape[0]
    if world == 1:
        items = E[row0:row0 + ni].float().cpu()
    else:                                   # rank 0 holds one shard: rebuild the catalog
        items = torch.empty(ni, k, dtype=torch.float32)
        step_ = 1 << 20
        for b0 in range(0, ni, step_):
            b1 = min(ni, b0 + step_)
            items[b0:b1] = item_rows(b0, b1, k, dev).to(table_dtype).float().cpu()
    Eh = torch.cat([check_rows.cpu(), items]).numpy()
    del items
    Ah = Aq.cpu().numpy().astype(np.int64)
    nu = 1 << 20
    Ac = np.empty_like(Ah)
    Ac[:, 0] = np.arange(qc)
    Ac[:, 1] = 0
    Ac[:, 2:] = qc + (Ah[:, 2:] - nu)
    Ac = Ac.astype(np.int32)
    base = qc + 12
    t0 = time.perf_counter()
    rs, ri = ocpu.catalog_topk(Ac, Eh, 1, 20, base, ni, ctx=(2, 5), threads=_oracle_threads())
    par = _topk_parity(s.cpu().numpy(), i.cpu().numpy(), ri, parity.hhfm_exact(Ac, Eh, base))
    par["oracle"] = (f"oracle/cpu_oracle.c oracle_catalog_topk mode 1 over all {ni:,} items, "
                     f"first {qc} queries, {_oracle_threads()} threads")
    par["oracle_s"] = time.perf_counter() - t0
    return par


def c5_leg(dev, world, rank, rows, reps=5, warm=3, mlp=torch.bfloat16, check=True):
    """configs[4] / C5: DeepFM F=5, k=256, MLP 3x400 (DFM.py:104-137),
    Frappe vocabulary, `rows` rows per GPU (12.5M = the 100M-row job over 8
    GPUs; weak scaling, rows sharded, no collective).  mlp=bf16: the fused
    bf16-MFMA kernel, the item field of layer 0 on MFMA, the others
    projected (HHFM_DFM_PROJ_ITEM via AUTO: P and the user grouping computed
    inside every step); its roofline prices the reference's FLOPs and states
    the executed ones;
    mlp=fp32 (the reference numerics):
    exact-fp32 MFMA with the projected layer 0 (include/hhfm.h ABI v3: P =
    W0-projection of every table row once per call inside the timed step,
    h0 = Σ_f P_f[x_f]) — its roofline counts the FLOPs it executes."""
    from hhfm_amd import ops
    from hhfm_amd.DFM import DeepFM
    nu, ni, ctx = 957, 4082, (7, 2, 3)
    M = nu + ni + sum(ctx)
    g = torch.Generator(device=dev)
    g.manual_seed(4 + rank)
    cols = [torch.randint(0, nu, (rows,), generator=g, device=dev),
            torch.randint(nu, nu + ni, (rows,), generator=g, device=dev)]
    off = nu + ni
    for c in ctx:
        cols.append(torch.randint(off, off + c, (rows,), generator=g, device=dev))
        off += c
    X = torch.stack(cols, 1).to(torch.int32).contiguous()
    del cols
    # SURVEY §8d C5 prices the gather at bf16 (5·256·2 B per row): the bf16-MLP
    # leg reads a bf16 table; the reference-numerics leg keeps fp32
    m = DeepFM(nu, ni, M, 5, 256, [400, 400, 400], None, 0.01, 0, 0.0, device=dev,
               mlp_dtype=mlp, table_dtype=mlp)
    Wt, bs, dims, Wp, bp = m._prepared()
    out = torch.empty(rows, device=dev)
    wb = m.weights["feature_bias"].reshape(-1)

    def step():
        ops.dfm_forward(X, m.table, wb, Wt, bs, dims, mlp, Wp, bp, out=out)

    # warm steps: the first passes after the lighter legs run 5-15 % slower
    # (clocks ramping: 10.8, 9.9, 9.4, 9.2 ms in one rocprofv3 trace,
    # profiles/r06_dfm_c5_trace.txt)
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    evs = []
    t0 = time.perf_counter()
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        step()
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    ms = float(t[0]) / reps * 1e3
    kern = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    par = _c5_parity(m, X, out, mlp) if check else None
    fl = 2.0 * (5 * 256 * 400 + 2 * 400 * 400) + 2.0 * (5 + 256 + 400)
    if mlp == torch.bfloat16:
        # executed (AUTO = ITEM): the projection of the M table rows for the 4
        # non-item fields, then the item field of layer 0 and the hidden
        # layers per row
        # (+ the FM part's pair table C = (E ⊙ Wp)·Eᵀ, one [M, 256] x [256, M] GEMM)
        ex = (2.0 * 4 * M * 256 * 400 + 2.0 * M * M * 256
              + rows * (2.0 * (256 * 400 + 2 * 400 * 400) + 2.0 * (5 + 256 + 400)))
        return {"workload": "C5 (configs[4]): DeepFM F=5 k=256 + MLP 3x400 (bf16 table as "
                            "SURVEY §8d prices it, bf16 MFMA, fp32 accumulation and FM part; "
                            "layer 0 of every field but the item projected, the FM part from "
                            "the pair table (E*Wp)E^T and the rows grouped by user inside "
                            "every step), "
                            f"Frappe vocabulary, rows sharded {rows:,} per GPU", "ranks": world,
                "rows_per_s": rows * world / (ms * 1e-3), "ms_per_pass": ms, "kernel_ms": kern,
                "executed_TFLOPs": ex / (kern * 1e-3) / 1e12,
                "kernel": "dfm_fused_w<13,8,4,true,2,8> (dfm_wide.hip: 256 rows per workgroup, "
                          "32 per wave, two waves per SIMD) after the user grouping, the "
                          "projection, the FM pair table and the weight packing",
                "roofline": {"bound": "mfma", "executed_flops_per_pass": ex,
                             "achieved_TFLOPs": ex / (kern * 1e-3) / 1e12,
                             "peak_TFLOPs": 2500.0,
                             "frac": ex / (kern * 1e-3) / 1e12 / 2500.0,
                             "reference_flops_per_row": fl,
                             "effective_TFLOPs": fl * rows / (kern * 1e-3) / 1e12,
                             "effective_frac": fl * rows / (kern * 1e-3) / 1e12 / 2500.0,
                             "note": "frac = FLOPs executed (projection + item field of layer "
                                     "0 + hidden layers) / time / bf16 peak; effective_frac "
                                     "prices the reference's 1.665 MFLOP/row"},
                "parity": par}
    # executed fp32 FLOPs of the projected path: the per-call projection of
    # the M table rows (exact-fp32 MFMA GEMM [M,256]x[256,5x400]) + the hidden
    # layers per row (split-bf16: each fp32 product = six bf16 MFMA products,
    # so their ceiling is the bf16 peak / 6) + the FM part and the last dot
    # (+ the FM part's pair table C = (E ⊙ Wp)·Eᵀ, one [M, 256] x [256, M] GEMM)
    ex = (2.0 * 5 * M * 256 * 400 + 2.0 * M * M * 256
          + rows * (2.0 * 2 * 400 * 400 + 2.0 * (5 * 416 + 256 + 400)))
    split_peak = 2500.0 / 6
    return {"workload": "C5 (configs[4]) at the reference numerics: DeepFM F=5 k=256 + MLP "
                        "3x400, fp32-faithful: projected layer 0 (P by exact-fp32 MFMA inside "
                        "every step), hidden layers on split-bf16 MFMA (x = x0+x1+x2 exactly, "
                        "the six piece products of order >= 2^-16, fp32 accumulation), FM part "
                        "from the pair table (E*Wp)E^T (exact-fp32 MFMA inside every step), rows "
                        f"grouped by user, Frappe vocabulary, rows sharded {rows:,} per GPU",
            "ranks": world, "rows_per_s": rows * world / (ms * 1e-3), "ms_per_pass": ms,
            "kernel_ms": kern,
            "reference_flops_TFLOPs": fl * rows / (kern * 1e-3) / 1e12,
            "roofline": {"bound": "mfma (split-bf16: bf16 peak / 6 products)",
                         "executed_flops_per_pass": ex,
                         "achieved_TFLOPs": ex / (kern * 1e-3) / 1e12,
                         "peak_TFLOPs": split_peak,
                         "frac": ex / (kern * 1e-3) / 1e12 / split_peak,
                         "exact_fp32_peak_TFLOPs": 157.3,
                         "vs_exact_fp32_peak": ex / (kern * 1e-3) / 1e12 / 157.3},
            "parity": par}


C5_CHECK_ROWS = 1 << 16


def _c5_parity(m, X, out, mlp):
    """The first 65,536 rows of the timed pass against the oracle: the fp32
    MLP against the float64 value of DFM.py:104-137 (oracle/parity.
    dfm_rows_exact), 1e-5 relative elementwise on every row whose condition
    number Σ|concat_j·Wp_j| / |out| is at most 100 and 1e-5 of that magnitude
    on the rest (oracle/parity.row_check, as K1); the bf16 MLP against the
    oracle that rounds the same operands to bf16 (oracle/parity.dfm_bf16_out),
    5e-3 of the magnitude (tests/test_gpu_dfm.py)."""
    from oracle import fm_oracle as orc
    from oracle import parity
    n = min(C5_CHECK_ROWS, X.shape[0])
    Xh = X[:n].cpu().numpy()
    got = out[:n].cpu().numpy().astype(np.float64)
    W = m.get_weights()
    L = len(m.deep_layers)
    Ls = [W[f"layer_{j}"] for j in range(L)]
    Bs = [W[f"bias_{j}"] for j in range(L)]
    E, w = W["feature_embeddings"], W["feature_bias"][:, 0]
    Wp, bp = W["concat_projection"], float(W["concat_bias"])
    t0 = time.perf_counter()
    if m.table_dtype == torch.bfloat16:
        E = parity.bf16_round(E)
    if mlp != torch.bfloat16:
        ex, mag = parity.dfm_rows_exact(Xh, E, w, Ls, Bs, Wp, bp)
        res = parity.row_check(got, ex, mag)
        ref32 = orc.dfm_out(Xh, E, w, Ls, Bs, Wp, bp)[:, 0]
        res["fp32_oracle"] = {k: v for k, v in parity.row_check(ref32, ex, mag).items()
                              if k.startswith("max_") or k == "rows_failing"}
        res["oracle"] = ("float64 DFM.py:104-137 (oracle/parity.dfm_rows_exact); the fp32 "
                         "restatement oracle/fm_oracle.dfm_out beside it")
        res["oracle_s"] = time.perf_counter() - t0
        return res
    mag = parity.dfm_magnitude(Xh, E, w, Ls, Bs, Wp, bp)
    ref = parity.dfm_bf16_out(Xh, E, w, Ls, Bs, Wp, bp)
    tol, how = 5e-3, "oracle/parity.dfm_bf16_out (bf16-rounded operands)"
    err = np.abs(got - ref) / mag
    return {"rows": n, "oracle": how, "tolerance_of_magnitude": tol,
            "max_err_of_magnitude": float(err.max()),
            "rows_failing": int((err > tol).sum()), "parity": bool((err <= tol).all()),
            "oracle_s": time.perf_counter() - t0}


def _pmc_column(path):
    """Per-dispatch Counter_Value of fm_rows_fast from a rocprofv3 --pmc csv."""
    import csv
    with open(path) as f:
        return [float(r["Counter_Value"]) for r in csv.DictReader(f)
                if "fm_rows_fast" in r["Kernel_Name"]]


def pmc_bytes_per_row(fetch, write, rows, k):
    """HBM bytes per K1 row from the six fm_rows_fast dispatches of
    scripts/pmc_fm_rows.py (calib x2, bench x2, bench-without-w x2):
    FETCH_SIZE is scaled by the calibration launch, whose user/item rows are
    streamed once (known bytes; MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE
    tallies 128-B requests at 64 B); WRITE_SIZE is exact for the output's
    streaming stores.  fetch / write: the two passes' KB values."""
    if len(fetch) != 6 or len(write) != 6:
        raise ValueError(f"expected 6 fm_rows_fast dispatches, got {len(fetch)} / {len(write)}")
    known = rows * (2 * k * 4 + 5 * 4 + 2 * 4)
    calib = 1024.0 * (fetch[0] + fetch[1]) / 2
    factor = known / calib
    rd = 1024.0 * (fetch[2] + fetch[3]) / 2 * factor / rows
    wr = 1024.0 * (write[2] + write[3]) / 2 / rows
    rd_now = 1024.0 * (fetch[4] + fetch[5]) / 2 * factor / rows
    wr_now = 1024.0 * (write[4] + write[5]) / 2 / rows
    return {"hbm_read_bytes_per_row": rd, "hbm_write_bytes_per_row": wr,
            "hbm_bytes_per_row": rd + wr, "no_w_hbm_bytes_per_row": rd_now + wr_now,
            "w_gather_bytes_per_row": rd - rd_now,
            "calibration": {"known_bytes_per_launch": known, "fetch_size_bytes": calib,
                            "factor": factor},
            "fetch_size_kb": fetch, "write_size_kb": write, "pmc_rows": rows}


def pmc_traffic(rows, k, timeout_s=150):
    """K1's HBM bytes per row read from PMC counters in this run: two
    rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: they cannot share a
    pass) over scripts/pmc_fm_rows.py at this bench's row count and table,
    each a child process under its own kill timeout.  Returns (dict, None)
    or (None, reason)."""
    import shutil
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not on PATH"
    if "rocprof" in os.environ.get("LD_PRELOAD", "") or any(
            k.startswith("ROCPROF") for k in os.environ):
        return None, "the bench itself runs under rocprofv3"
    tmp = tempfile.mkdtemp(prefix="hhfm_pmc_")
    env = dict(os.environ, PMC_ROWS=str(rows), PMC_K=str(k))
    vals = {}
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr.lower())
            cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", ctr, "-d", d,
                   "-o", "pmc", "--output-format", "csv", "--", sys.executable,
                   os.path.join(ROOT, "scripts", "pmc_fm_rows.py")]
            r = subprocess.run(cmd, env=env, cwd=tmp, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, text=True)
            if r.returncode != 0:
                return None, f"{ctr} pass exited {r.returncode}: {r.stderr[-300:]}"
            vals[ctr] = _pmc_column(os.path.join(d, "pmc_counter_collection.csv"))
        return pmc_bytes_per_row(vals["FETCH_SIZE"], vals["WRITE_SIZE"], rows, k), None
    except (OSError, ValueError, KeyError) as e:
        return None, f"{type(e).__name__}: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def stream_read_peak(buf, reps=5):
    """The box's measured HBM read ceiling: hhfm_probe_stream_read over
    `buf` (grid-stride, contiguous-chunk and non-temporal chunk variants),
    best launch of `reps` per variant, GB/s -> (best, {variant: GB/s})."""
    from hhfm_amd._native import native
    dev = buf.device
    sink = torch.zeros(1, device=dev)
    nbytes = (buf.numel() * buf.element_size()) & ~15
    st = torch.cuda.current_stream(dev).cuda_stream
    rates = {}
    for mode, name in ((0, "grid_stride"), (1, "chunked"), (2, "chunked_nt")):
        native().probe_stream_read(buf.data_ptr(), nbytes, mode, sink.data_ptr(), st)
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            native().probe_stream_read(buf.data_ptr(), nbytes, mode, sink.data_ptr(), st)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        rates[name] = nbytes / (best * 1e-3) / 1e9
    return max(rates.values()), rates


def gather_rows_peak(idx, E, reps=5):
    """The box's measured ceiling for K1's access pattern: the same row
    kernel over the same user and item columns (two random 256-B table rows
    per row) with the `w` and context loads removed (F=2, w=None), best of
    `reps` launches -> GB/s of its bytes (2 rows + 2 ids + out per row)."""
    from hhfm_amd import ops
    ui = idx[:, :2].contiguous()
    o = torch.empty(ui.shape[0], dtype=torch.float32, device=idx.device)
    ops.fm_score_rows(ui, E, None, 0.0, out=o)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.fm_score_rows(ui, E, None, 0.0, out=o)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    bpr = 2 * E.shape[1] * E.element_size() + 2 * 4 + 4
    del ui, o
    return bpr * idx.shape[0] / (best * 1e-3) / 1e9, best


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))       # before anything touches the GPU
    if args.dry_run:
        dry_run(args)
        return
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rccl_world = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
        rccl_world = dist.get_world_size()
    from hhfm_amd import ops

    idx, E, w, M = make_batch(args.rows, args.users, args.items, args.k, 1 + rank, dev)
    out = torch.empty(args.rows, dtype=torch.float32, device=dev)
    w0 = 0.0
    for _ in range(args.warmup):
        ops.fm_score_rows(idx, E, w, w0, out=out)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        ops.fm_score_rows(idx, E, w, w0, out=out)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    el, kern_ms = float(t[0]), float(t[1])

    rows_total = args.rows * world * args.steps
    value = rows_total / el
    # Compulsory HBM bytes per row: the user and item embedding rows and
    # their w entries, the 5 ids, the output.  The three context rows come
    # from a 12-row vocabulary that stays cache-resident, so SURVEY §8d's
    # 1,324 B (all five rows from HBM) would put `frac` above 1; it is kept
    # as `survey_bytes_per_row` for reference.
    bpr = 2 * args.k * 4 + 5 * 4 + 2 * 4 + 4
    bpr_survey = 5 * args.k * 4 + 5 * 4 + 5 * 4 + 4
    achieved = bpr * args.rows / (kern_ms * 1e-3) / 1e9
    # K1 issues 128-B HBM requests only (TCC_EA0_RDREQ_32B = 0 for every cache
    # policy of the 4-B `w` gathers; profiles/r02_k1_wpolicy.json): the bytes
    # that cross HBM at that granularity are 2 rows x 256 B + 2 w lines x 128 B
    # + ids + out = 792 B/row at k=64.
    bpr_lines = 2 * args.k * 4 + 2 * 128 + 5 * 4 + 4
    peak_meas, peak_variants = stream_read_peak(E)
    gather_peak, gather_ms = gather_rows_peak(idx, E)
    traffic, pmc, why = None, None, "--no-pmc"
    if rank == 0 and world == 1 and not args.no_pmc:
        pmc, why = pmc_traffic(args.rows, args.k)
    if pmc is not None:
        # PMC bytes per row of this run (corrected FETCH_SIZE + WRITE_SIZE) x rows per launch
        traffic = pmc["hbm_bytes_per_row"] * args.rows
        traffic_source = ("measured in this run: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE "
                          "passes (child processes) over scripts/pmc_fm_rows.py at "
                          f"{args.rows} rows, FETCH_SIZE calibrated on a known-byte launch")
    elif os.path.exists(args.traffic_json):
        traffic_source = (f"calibrated, not measured in this run ({why}): PMC bytes/row from "
                          f"{os.path.relpath(args.traffic_json, ROOT)} x rows")
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("k") == args.k and tj.get("fields") == 5:
                traffic = tj["hbm_bytes_per_row"] * args.rows
        except (OSError, ValueError):
            traffic = None
    else:
        traffic_source = f"none ({why})"

    result = {
        "metric": METRIC, "value": value, "unit": "triples/s", "n_gpus": world,
        "world": {"ranks": world, "gpus_arg": args.gpus, "rccl_world_size": rccl_world,
                  "backend": "nccl (RCCL)" if world > 1 else None},
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "FM k=64 Frappe-shape per-row scoring (configs[1], "
                               "HBM-roofline variant: 8M users + 8M items + 12 ctx ids)",
                   "rows_per_gpu": args.rows, "fields": 5, "k": args.k,
                   "table_rows": M, "table_bytes": M * args.k * 4,
                   "parallelism": f"rows sharded x{world}, no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "fm_rows_fast<5,16,f32,w,NTM 2>", "kernel_ms": kern_ms,
                     "traffic_GBps": (traffic / (kern_ms * 1e-3) / 1e9) if traffic else None,
                     "traffic_frac": (traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                                     if traffic else None,
                     "algorithmic_bytes_per_row": bpr,
                     "survey_bytes_per_row": bpr_survey,
                     "survey_rate_GBps": bpr_survey * args.rows / (kern_ms * 1e-3) / 1e9,
                     "peak_measured": peak_meas,
                     "peak_measured_how": "hhfm_probe_stream_read: one 16-B/lane read of the "
                                          "4.3 GB table, best variant and launch of 5, this box",
                     "peak_measured_variants": peak_variants,
                     "frac_vs_measured": (achieved / peak_meas) if peak_meas else None,
                     "peak_gather_measured": gather_peak,
                     "peak_gather_how": "the same row kernel over the same rows' user and item "
                                        "columns only (2 random 256-B rows, no w / context "
                                        f"loads): {gather_ms:.3f} ms, best of 5, this box",
                     "frac_vs_gather": achieved / gather_peak,
                     "line_bytes_per_row": bpr_lines,
                     "line_rate_GBps": bpr_lines * args.rows / (kern_ms * 1e-3) / 1e9,
                     "line_frac_vs_measured": (bpr_lines * args.rows / (kern_ms * 1e-3) / 1e9
                                               / peak_meas) if peak_meas else None,
                     "traffic_source": traffic_source,
                     "traffic_pmc": pmc},
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(idx, E, w, w0, out, args)
    legs = [x for x in args.legs.split(",") if x]
    del idx, E, w, out
    torch.cuda.empty_cache()
    extra = {}
    check = not args.no_check
    # the extra legs never cost the headline line: a failure is recorded, not raised
    if "catalog" in legs:
        try:
            extra["catalog_c4"] = catalog_leg(dev, world, rank, check=check)
        except Exception as e:  # noqa: BLE001
            extra["catalog_c4"] = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
    if "c3" in legs and rank == 0:
        try:
            extra["catalog_c3"] = catalog_c3_leg(dev)
        except Exception as e:  # noqa: BLE001
            extra["catalog_c3"] = {"error": f"{type(e).__name__}: {e}"}
    if "catalog_bf16" in legs:
        try:
            extra["catalog_c4_bf16"] = catalog_leg(dev, world, rank, table_dtype=torch.bfloat16,
                                                   check=check)
        except Exception as e:  # noqa: BLE001
            extra["catalog_c4_bf16"] = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
    if "c5" in legs:
        try:
            extra["dfm_c5"] = c5_leg(dev, world, rank, args.c5_rows, check=check and rank == 0)
        except Exception as e:  # noqa: BLE001
            extra["dfm_c5"] = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
        try:
            extra["dfm_c5_f32"] = c5_leg(dev, world, rank, args.c5_rows, mlp=torch.float32,
                                         check=check and rank == 0)
        except Exception as e:  # noqa: BLE001
            extra["dfm_c5_f32"] = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
    if "hr" in legs and rank == 0:
        try:
            extra["hr_at_10"] = hr_leg(dev, args.hr_epochs)
        except Exception as e:  # noqa: BLE001
            extra["hr_at_10"] = {"error": f"{type(e).__name__}: {e}"}
    if extra:
        result["extra"] = extra
    # one verdict per leg: True / False from the leg's oracle comparison, None
    # when the leg did not run a check (or failed before it)
    summary = {}
    if "cpu_baseline" in result:
        summary["k1_rows"] = result["cpu_baseline"]["gpu_vs_float64"]["parity"]
    for name, leg in extra.items():
        if name == "hr_at_10":
            summary[name] = leg.get("identical_to_oracle")
        elif isinstance(leg.get("parity"), dict):
            summary[name] = leg["parity"]["parity"]
        else:
            summary[name] = None
        if "matches_n1" in leg:
            summary[name + "_matches_n1"] = leg["matches_n1"]
    result["parity"] = summary
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
