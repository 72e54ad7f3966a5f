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

Prints ONE JSON line (rank 0).  See DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

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
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_fm_rows.json"))
    p.add_argument("--legs", default="hr,catalog,catalog_bf16,c3",
                   help="extra legs: hr (HR@10 identity after GPU training on Frappe-shape "
                        "data), catalog / catalog_bf16 (C4 item-sharded top-K over an fp32 / "
                        "bf16 table, RCCL all-gather at N>1), c3 (configs[2]: Frappe-catalog "
                        "top-20, rank 0)")
    p.add_argument("--hr-epochs", type=int, default=5)
    return p.parse_args()


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


def cpu_baseline(idx, E, w, w0, out_gpu, args):
    """Time the oracle's C restatement (OpenMP) on a bounded sample of the same
    workload (same table, first cpu_rows rows) on this box's host cores."""
    from oracle import cpu as ocpu
    threads = min(len(os.sched_getaffinity(0)), 16)
    n = min(args.cpu_rows, idx.shape[0])
    X = idx[:n].cpu().numpy()
    Eh = E.cpu().numpy()
    wh = w.cpu().numpy()
    ref = ocpu.fm_out(X, Eh, wh, w0, threads)          # warm (page-in)
    reps, t0 = 0, time.perf_counter()
    while True:
        ocpu.fm_out(X, Eh, wh, w0, threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    m = min(n, 1 << 16)                                 # parity spot-check subset
    got = out_gpu[:m].cpu().numpy()
    e = Eh[X[:m].astype(np.int64)].astype(np.float64)
    scale = (0.5 * (e.sum(1) ** 2 + (e * e).sum(1))).sum(1) + np.abs(wh[X[:m]]).sum(1) + abs(w0)
    err = float(np.max(np.abs(got - ref[:m]) / scale))
    cpu_name = platform.processor() or "cpu"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": reps * n / el, "unit": "triples/s", "cores": threads, "kind": "port",
            "sample": f"{n} rows of the same workload (same 4.3 GB table) x {reps} passes, "
                      f"oracle/cpu_oracle.c (OpenMP) on {cpu_name}",
            "gpu_vs_cpu_max_rel_err": err}


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


def catalog_c3_leg(dev, reps=50):
    """configs[2] / C3: HHFM k=64, bf16 table, Frappe vocabulary (957 users,
    4,082 items, ctx 7/2/3), 3,000 queries, top-20 over the full catalog
    (hhfm_catalog_topk: score matrix by MFMA GEMM + dense top-K)."""
    from hhfm_amd import ops
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

    def step():
        return ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0))

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    pairs = B * ni
    return {"workload": "C3 (configs[2]): HHFM k=64 bf16 table, Frappe vocabulary, 3,000 "
                        "queries x 4,082 items, top-20, one GPU", "ms_per_query_batch": ms,
            "pairs_per_s": pairs / (ms * 1e-3), "TFLOPs": 2.0 * k * pairs / (ms * 1e-3) / 1e12}


def catalog_leg(dev, world, rank, reps=5, table_dtype=torch.float32):
    """C4: HHFM k=128, 1 M users, 10 M items sharded contiguously over the
    ranks, 1,024 queries, K=20, fp32 (or bf16) table; local
    hhfm_catalog_topk + RCCL all-gather + hhfm_topk_merge per step."""
    from hhfm_amd import distributed as hd
    from hhfm_amd import ops
    nu, ni, k, B, K = 1 << 20, 10_000_000, 128, 1024, 20
    begin, end = hd.shard_range(ni, world, rank)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    # replicated users + ctx, only this rank's item rows are materialised
    rows_user = torch.empty(nu, k, device=dev).normal_(0, 0.01, generator=g)
    rows_ctx = torch.empty(12, k, device=dev).normal_(0, 0.01, generator=g)
    gi = torch.Generator(device=dev)
    gi.manual_seed(1000 + rank)
    rows_item = torch.empty(end - begin, k, device=dev).normal_(0, 0.01, generator=gi)
    E = torch.cat([rows_user, rows_item, rows_ctx]).to(table_dtype).contiguous()
    del rows_user, rows_item
    off = nu + (end - begin)
    cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
            torch.zeros(B, dtype=torch.int64, device=dev)]
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
        off += c
    A = torch.stack(cols, 1).to(torch.int32).contiguous()

    def scorer(A_, b0, cnt, Kl):
        return ops.catalog_topk(A_, E, ops.MODE_HHFM, Kl, nu, cnt, b0, None, 0, (2, 5), (0, 0))

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
    return {"workload": f"C4: HHFM k=128 {tname} table, 10M-item catalog sharded over ranks, "
                        "1,024 queries, top-20 (local split-bf16 MFMA score + select, RCCL "
                        "all-gather, merge)",
            "ms_per_query_batch": ms, "pairs_per_s": pairs / (ms * 1e-3),
            "TFLOPs": 2.0 * k * pairs / (ms * 1e-3) / 1e12, "ranks": world}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
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
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("k") == args.k and tj.get("fields") == 5:
                # PMC bytes per row (calibrated FETCH_SIZE + WRITE_SIZE) x rows per launch
                traffic = tj["hbm_bytes_per_row"] * args.rows
        except (OSError, ValueError):
            traffic = None

    result = {
        "metric": METRIC, "value": value, "unit": "triples/s", "n_gpus": world,
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
                     "kernel": "fm_rows_fast<5,16,f32,w>", "kernel_ms": kern_ms,
                     "traffic_GBps": (traffic / (kern_ms * 1e-3) / 1e9) if traffic else None,
                     "traffic_frac": (traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS)
                                     if traffic else None,
                     "algorithmic_bytes_per_row": bpr,
                     "survey_bytes_per_row": bpr_survey,
                     "survey_rate_GBps": bpr_survey * args.rows / (kern_ms * 1e-3) / 1e9},
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(idx, E, w, w0, out, args)
    legs = [x for x in args.legs.split(",") if x]
    del idx, E, w, out
    torch.cuda.empty_cache()
    extra = {}
    # the extra legs never cost the headline line: a failure is recorded, not raised
    if "catalog" in legs:
        try:
            extra["catalog_c4"] = catalog_leg(dev, world, rank)
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
            extra["catalog_c4_bf16"] = catalog_leg(dev, world, rank, table_dtype=torch.bfloat16)
        except Exception as e:  # noqa: BLE001
            extra["catalog_c4_bf16"] = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
    if "hr" in legs and rank == 0:
        try:
            extra["hr_at_10"] = hr_leg(dev, args.hr_epochs)
        except Exception as e:  # noqa: BLE001
            extra["hr_at_10"] = {"error": f"{type(e).__name__}: {e}"}
    if extra:
        result["extra"] = extra
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
