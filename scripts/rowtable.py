#!/usr/bin/env python3
"""Per-row measurement table for SURVEY §8 (d): every hot-path row at its
configuration on the GPU (HIP events, median of reps, inputs resident), its
roofline (algorithmic bytes or flops per unit from DESIGN.md), and the CPU
restatement timed beside it on a bounded sample of the same workload on this
box's host cores (oracle/cpu_oracle.c with 1 thread and min(cores, 16)
threads where the C restatement exists, the numpy oracle otherwise).

Writes one JSON object to stdout (profiles/r01_rows.json).  Run on the GPU box:
    python scripts/rowtable.py > gpurun_out/rows.json
"""
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("HHFM_AB_ROOT"):   # diagnostic A/B: another build's package copy first
    sys.path.insert(0, os.environ["HHFM_AB_ROOT"])
import bench  # noqa: E402
from hhfm_amd import ops  # noqa: E402
from oracle import cpu as ocpu  # noqa: E402
from oracle import fm_oracle as orc  # noqa: E402

dev = torch.device("cuda", 0)
HBM = 8000.0          # GB/s, MI355X_MICROARCH.md
F32_TF = 157.3        # TF/s fp32 (MFMA 32x32x2 f32 == VALU peak)
BF16_TF = 2500.0      # TF/s bf16 dense MFMA
# split-bf16 kernels (fp32 operands as three bf16 pieces on the bf16 MFMA):
# their own ceiling is the bf16 rate / MFMAs per 16-k product
SPLIT3_TF = BF16_TF / 3   # bf16 table x fp32 query: 3 MFMAs per 16 k (C3, bf16 C4)
SPLIT6_TF = BF16_TF / 6   # fp32 x fp32: 6 MFMAs per 16 k (fp32 C4, AFM fused)
THREADS = min(len(os.sched_getaffinity(0)), 16)
only = os.environ.get("ROWS_ONLY", "")


def gpu_ms(fn, reps=10, warm=2):
    """Median device time per call, calls queued back to back (no host sync
    between them, so a call's host-side set-up overlaps the previous call's
    kernels instead of being timed as idle device time)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t_end = time.perf_counter() + 0.2   # >= 200 ms of the same work first: clocks ramp
    while time.perf_counter() < t_end:
        fn()
        torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def cpu_s(fn, budget=3.0):
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= budget:
            return el / n


def frappe_rows(rng, B, nu=957, ni=4082, ctx=(7, 2, 3)):
    cols = [rng.integers(0, nu, B), rng.integers(nu, nu + ni, B)]
    off = nu + ni
    for c in ctx:
        cols.append(rng.integers(off, off + c, B))
        off += c
    return np.stack(cols, 1).astype(np.int32), off


res = {"host": platform.node(), "cpu_threads": THREADS}
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
try:
    with open("/proc/cpuinfo") as f:
        res["cpu"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
except (OSError, StopIteration):
    pass

# ---- C2 / M1: FM per-row score, roofline variant ------------------------------
if not only or "c2" in only:
    rows = 1 << 25
    idx, E, w, M = bench.make_batch(rows, 8 << 20, 8 << 20, 64, 1, dev)
    out = torch.empty(rows, device=dev)
    ms = gpu_ms(lambda: ops.fm_score_rows(idx, E, w, 0.0, out=out))
    n = 1 << 20
    X, Eh, wh = idx[:n].cpu().numpy(), E.cpu().numpy(), w.cpu().numpy()
    c1 = cpu_s(lambda: ocpu.fm_out(X, Eh, wh, 0.0, 1))
    cN = cpu_s(lambda: ocpu.fm_out(X, Eh, wh, 0.0, THREADS))
    res["C2_M1_fm_rows"] = {
        "config": "FM k=64 fp32, 8M users + 8M items + 12 ctx, 2^25 rows", "unit": "rows/s",
        "gpu_ms": ms, "gpu_rate": rows / (ms * 1e-3),
        "roofline": {"bound": "hbm", "bytes_per_unit": 544,
                     "frac": 544 * rows / (ms * 1e-3) / 1e9 / HBM},
        "cpu_rate_1t": n / c1, "cpu_rate_nt": n / cN, "cpu_sample": f"{n} rows"}
    del idx, E, w, out
    torch.cuda.empty_cache()

# ---- C3 / H2: HHFM catalog top-20, Frappe, k=64 bf16 ---------------------------
if not only or "c3" in only:
    rng = np.random.default_rng(2)
    A, M = frappe_rows(rng, 3000)
    E = rng.normal(0, 0.01, (M, 64)).astype(np.float32)
    Eg = torch.from_numpy(E).to(dev).to(torch.bfloat16)
    Ah = torch.from_numpy(A).to(dev)
    ms = gpu_ms(lambda: ops.catalog_topk(Ah, Eg, ops.MODE_HHFM, 20, 957, 4082, 0, None, 0,
                                         (2, 5), (0, 0)))
    pairs = 3000 * 4082
    Er = Eg.float().cpu().numpy()
    As = A[:300]
    c1 = cpu_s(lambda: ocpu.catalog_topk(As, Er, 1, 20, 957, 4082, ctx=(2, 5), threads=1))
    cN = cpu_s(lambda: ocpu.catalog_topk(As, Er, 1, 20, 957, 4082, ctx=(2, 5), threads=THREADS))
    res["C3_H2_hhfm_catalog"] = {
        "config": "HHFM k=64 bf16 table, 3000 queries x 4082 items, top-20", "unit": "pairs/s",
        "gpu_ms": ms, "gpu_rate": pairs / (ms * 1e-3),
        "roofline": {"bound": "split-bf16 MFMA (3/16k)", "flops_per_unit": 128,
                     "frac": 128 * pairs / (ms * 1e-3) / 1e12 / SPLIT3_TF},
        "cpu_rate_1t": 300 * 4082 / c1, "cpu_rate_nt": 300 * 4082 / cN,
        "cpu_sample": "300 queries x 4082 items (C oracle, same bf16-rounded table)"}

# ---- C4 / H2: HHFM catalog shard, k=128 fp32, 1.25M items ----------------------
if not only or "c4" in only:
    rng = np.random.default_rng(3)
    nu, ni, k = 1 << 20, 1_250_000, 128
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    E = torch.empty(nu + ni + 12, k, device=dev).normal_(0, 0.01, generator=g)
    cols = [torch.randint(0, nu, (1024,), generator=g, device=dev),
            torch.zeros(1024, dtype=torch.int64, device=dev)]
    off = nu + ni
    for c in (7, 2, 3):
        cols.append(torch.randint(off, off + c, (1024,), generator=g, device=dev))
        off += c
    Ah = torch.stack(cols, 1).to(torch.int32).contiguous()
    ms = gpu_ms(lambda: ops.catalog_topk(Ah, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5),
                                         (0, 0)), reps=5)
    pairs = 1024 * ni
    Eh = E.cpu().numpy()
    As = Ah[:16].cpu().numpy()
    c1 = cpu_s(lambda: ocpu.catalog_topk(As, Eh, 1, 20, nu, ni, ctx=(2, 5), threads=1), 2.0)
    cN = cpu_s(lambda: ocpu.catalog_topk(As, Eh, 1, 20, nu, ni, ctx=(2, 5), threads=THREADS), 2.0)
    res["C4_H2_hhfm_catalog_shard"] = {
        "config": "HHFM k=128 fp32, 1,024 queries x 1.25M-item shard (C4 per GPU), top-20",
        "unit": "pairs/s", "gpu_ms": ms, "gpu_rate": pairs / (ms * 1e-3),
        "roofline": {"bound": "split-bf16 MFMA (6/16k)", "flops_per_unit": 256,
                     "frac": 256 * pairs / (ms * 1e-3) / 1e12 / SPLIT6_TF},
        "cpu_rate_1t": 16 * ni / c1, "cpu_rate_nt": 16 * ni / cN,
        "cpu_sample": "16 queries x 1.25M items (C oracle)"}
    del E
    torch.cuda.empty_cache()

# ---- C5 / D1: DeepFM k=256, 3x400 ----------------------------------------------
if not only or "c5" in only:
    from hhfm_amd.DFM import DeepFM
    rng = np.random.default_rng(4)
    B = 12_500_000
    X, M = frappe_rows(rng, B)
    Xg = torch.from_numpy(X).to(dev)
    for mdt, name in ((torch.bfloat16, "C5_D1_dfm_bf16_mlp"), (torch.float32, "C5_D1_dfm_fp32_mlp")):
        # the bf16 MLP reads a bf16 table, as SURVEY §8d prices C5 (and bench.py)
        m = DeepFM(957, 4082, M, 5, 256, [400, 400, 400], None, 0.01, 0, 0.0, device=dev,
                   mlp_dtype=mdt, table_dtype=mdt)
        m.validate = False
        Wt, bs, dims, Wp, bp = m._prepared()
        out = torch.empty(B, device=dev)
        nrows = B if mdt == torch.bfloat16 else 2_000_000
        Xn = Xg[:nrows]
        ms = gpu_ms(lambda: ops.dfm_forward(Xn, m.table, m.weights["feature_bias"].reshape(-1),
                                            Wt, bs, dims, mdt, Wp, bp, out=out[:nrows]), reps=5)
        fl = 2.0 * (5 * 256 * 400 + 2 * 400 * 400) + 2.0 * (5 + 256 + 400)
        W = m.get_weights()
        Ls = [W[f"layer_{i}"] for i in range(3)]
        Bs_ = [W[f"bias_{i}"] for i in range(3)]
        n = 20000
        c = cpu_s(lambda: orc.dfm_out(X[:n], W["feature_embeddings"], W["feature_bias"][:, 0],
                                      Ls, Bs_, W["concat_projection"], float(W["concat_bias"])))
        peak = BF16_TF if mdt == torch.bfloat16 else F32_TF
        if mdt == torch.bfloat16:
            # AUTO = ITEM: fields other than the item projected (rows grouped by
            # user), the item field and the hidden layers on MFMA
            ex = 2.0 * 4 * M * 256 * 400 + nrows * (2.0 * (256 * 400 + 2 * 400 * 400)
                                                    + 2.0 * (5 + 256 + 400))
            roof = {"bound": "MFMA", "flops_per_unit": ex / nrows,
                    "frac": ex / (ms * 1e-3) / 1e12 / peak,
                    "reference_flops_per_unit": fl,
                    "effective_frac": fl * nrows / (ms * 1e-3) / 1e12 / peak}
            cfg = (f"DFM F=5 k=256 MLP 3x400 (bf16 MLP and table; AUTO projection = every "
                   f"field but the item), {nrows:,} rows")
        else:
            # the fp32 MLP runs the projected layer 0 (AUTO: rows >= 2 x table
            # rows): executed FLOPs = the per-call projection of the M table
            # rows + the hidden layers per row
            ex = 2.0 * 5 * M * 256 * 400 + nrows * (2.0 * 2 * 400 * 400 + 2.0 * (5 * 416 + 661))
            # hidden layers on split-bf16 MFMA: their ceiling is the bf16 peak / 6
            roof = {"bound": "split-bf16 MFMA (6/16k)", "flops_per_unit": ex / nrows,
                    "frac": ex / (ms * 1e-3) / 1e12 / SPLIT6_TF,
                    "vs_exact_fp32_peak": ex / (ms * 1e-3) / 1e12 / F32_TF,
                    "reference_flops_per_unit": fl,
                    "reference_flops_TFLOPs": fl * nrows / (ms * 1e-3) / 1e12}
            cfg = (f"DFM F=5 k=256 MLP 3x400 (fp32, projected layer 0), {nrows:,} rows")
        res[name] = {
            "config": cfg, "unit": "rows/s", "gpu_ms": ms,
            "gpu_rate": nrows / (ms * 1e-3),
            "roofline": roof,
            "cpu_rate_numpy": n / c, "cpu_sample": f"{n} rows, numpy oracle (fp32)"}
        del m, out
        torch.cuda.empty_cache()

# ---- A1 / A2: AFM k=64, A=64 ----------------------------------------------------
if not only or "afm" in only:
    from hhfm_amd.AFM import AFM
    rng = np.random.default_rng(5)
    B = 1 << 20
    X, M = frappe_rows(rng, B)
    m = AFM(957, 4082, M, 1, [64, 64], None, 0.1, 100.0, [1, 1], "AdagradOptimizer", 0.999, 5,
            device=dev)
    m.validate = False
    Wt, b, p_, P = m._att()
    Xg = torch.from_numpy(X).to(dev)
    out = torch.empty(B, device=dev)
    ms = gpu_ms(lambda: ops.afm_forward(Xg, m.table, m.weights["feature_bias"].reshape(-1), 0.0,
                                        Wt, b, p_, P, out=out))
    W = m.get_weights()
    args = (W["attention_W"], W["attention_b"], W["attention_p"], W["prediction"])
    n = 20000
    c = cpu_s(lambda: orc.afm_out(X[:n], W["feature_embeddings"], W["feature_bias"][:, 0], 0.0,
                                  *args))
    fl = 2.0 * 10 * 64 * 64
    res["A1_afm_rows"] = {
        "config": "AFM F=5 k=64 A=64, 1M rows", "unit": "rows/s", "gpu_ms": ms,
        "gpu_rate": B / (ms * 1e-3),
        "roofline": {"bound": "split-bf16 MFMA (6/16k)", "flops_per_unit": fl,
                     "frac": fl * B / (ms * 1e-3) / 1e12 / SPLIT6_TF},
        "cpu_rate_numpy": n / c, "cpu_sample": f"{n} rows, numpy oracle"}
    Aq = Xg[:300]
    w1 = m.weights["feature_bias"].reshape(-1)
    ms = gpu_ms(lambda: ops.afm_catalog_topk(Aq, m.table, w1, Wt, b, p_, P, 957, 4082, 20))
    pairs = 300 * 4082
    c = cpu_s(lambda: orc.afm_catalog_scores(X[:10], W["feature_embeddings"],
                                             W["feature_bias"][:, 0], *args, 957, 4082))
    fl = 2.0 * 4 * 64 * 64
    res["A2_afm_catalog"] = {
        "config": "AFM k=64 A=64, 300 queries x 4082 items, top-20", "unit": "pairs/s",
        "gpu_ms": ms, "gpu_rate": pairs / (ms * 1e-3),
        "roofline": {"bound": "split-bf16 MFMA (6/16k)", "flops_per_unit": fl,
                     "frac": fl * pairs / (ms * 1e-3) / 1e12 / SPLIT6_TF},
        "cpu_rate_numpy": 10 * 4082 / c, "cpu_sample": "10 queries x 4082 items, numpy oracle"}
    del m, out
    torch.cuda.empty_cache()

# ---- H6: one HHFM training step (batch 5000, 2 negatives, Frappe vocab) -----------
if not only or "h6" in only:
    from hhfm_amd.OurModel7 import OUR
    from hhfm_amd import training
    rng = np.random.default_rng(6)
    X, M = frappe_rows(rng, 5000)
    m = OUR(3, 0, M, 957, 4082, 64, 0.1, 0.01, "AdagradOptimizer", True, False, device=dev)
    data = {"X": X[:, :2], "F1": X[:, 2:], "Y": rng.integers(957, 957 + 4082, (5000, 2))}
    training.hhfm_partial_fit(m, data)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 50
    for _ in range(reps):
        training.hhfm_partial_fit(m, data)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    E = m.get_weights()["feature_embeddings"]
    acc = np.full_like(E, 0.1)
    Xc = np.concatenate([X[:, :2], X[:, 2:]], 1)
    c = cpu_s(lambda: orc.hhfm_train_step(Xc, data["Y"], E, acc, 0.1, 0.01, 3, 0))
    res["H6_hhfm_train_step"] = {
        "config": "HHFM k=64 partial_fit, batch 5000, 2 negatives, Frappe vocab (5,051 rows)",
        "unit": "steps/s", "gpu_ms_wall": ms, "gpu_rate": 1e3 / ms,
        "cpu_rate_numpy": 1.0 / c, "cpu_sample": "same batch, numpy oracle step"}


# ---- H5 / H3: harness membership + walk on the device (Frappe-shape split) ------
if not only or "h35" in only:
    import tempfile
    from hhfm_amd.NewLoadData import LoadData
    from hhfm_amd.harness import Train

    class _DevModel:
        device = dev

    with tempfile.TemporaryDirectory() as tmp:
        np.random.seed(2016)
        d = LoadData(bench.frappe_shape_dataset(tmp), "frappe_shape")
    X = np.asarray(d.Train_data.values[:, 1:], dtype=np.int64)
    host, devt = Train(data=d, model=None), Train(data=d, model=_DevModel())
    np.random.seed(1)
    devt.sample_negative(X, 50)               # builds the device pair arrays once
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        devt.sample_negative(X, 50)
    t_dev = (time.perf_counter() - t0) / reps
    t_host = cpu_s(lambda: host.sample_negative(X, 50), 3.0)
    n = X.shape[0] * 50
    res["H5_sample_negative"] = {
        "config": f"sample_negative(Train rows, 50) on a Frappe-shape split ({X.shape[0]:,} rows; "
                  "evaluate_AUC's draw), the whole sampler on the device (hhfm_sample_negative: MT19937 stream, masked draws, membership, re-draws)",
        "unit": "samples/s", "gpu_ms_wall": t_dev * 1e3, "gpu_rate": n / t_dev,
        "cpu_rate_numpy": n / t_host,
        "cpu_sample": "same call, host harness (vectorised membership, same stream)"}

def _train_row(step, cpu_step, reps=20):
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    return ms, cpu_s(cpu_step)


# ---- H6: AFM / DeepFM training steps (main.py's factor 128, batch 5000, Frappe) ----
if not only or "h6" in only:
    from hhfm_amd.AFM import AFM
    from hhfm_amd.DFM import DeepFM
    from hhfm_amd import training
    rng = np.random.default_rng(7)
    X, M = frappe_rows(rng, 5000)
    y = rng.choice([1.0, -1.0], 5000).astype(np.float32)[:, None]
    m = AFM(957, 4082, M, 1, [128, 128], None, 0.1, 100.0, [1, 1], "AdagradOptimizer", 0.999, 5,
            device=dev)
    W = m.get_weights()
    names = ["feature_embeddings", "feature_bias", "bias", "attention_W", "attention_b",
             "attention_p", "prediction"]
    cur = [np.asarray(W[n], np.float32) for n in names]
    acc = {kk: np.full_like(v, 0.1) for kk, v in zip(["E", "w", "w0", "W", "b", "p", "P"], cur)}
    ms, c = _train_row(lambda: training.afm_partial_fit(m, {"X": X, "Y": y}),
                       lambda: orc.afm_train_step(X, y, *cur, acc, 0.1, 100.0))
    res["H6_afm_train_step"] = {
        "config": "AFM k=A=128 partial_fit, batch 5000 rows, Frappe vocab (F=5)",
        "unit": "steps/s", "gpu_ms_wall": ms, "gpu_rate": 1e3 / ms,
        "cpu_rate_numpy": 1.0 / c, "cpu_sample": "same batch, numpy oracle step"}
    del m
    m = DeepFM(957, 4082, M, 5, 128, [150, 200, 150], None, 0.01, 0, 0.01, device=dev)
    W = m.get_weights()
    L = 3
    Ls = [W[f"layer_{i}"] for i in range(L)]
    bs = [W[f"bias_{i}"][0] for i in range(L)]
    keys = ["E", "w"] + [f"W{i}" for i in range(L)] + [f"b{i}" for i in range(L)] + ["Wp", "bp"]
    vals = ([W["feature_embeddings"], W["feature_bias"][:, 0]] + Ls + bs
            + [W["concat_projection"][:, 0], np.float32(W["concat_bias"])])
    acc = {kk: np.full_like(np.asarray(v, np.float32), 0.1) for kk, v in zip(keys, vals)}
    ms, c = _train_row(lambda: training.dfm_partial_fit(m, {"X": X, "Y": y}),
                       lambda: orc.dfm_train_step(X, y, vals[0], vals[1], Ls, bs, vals[-2],
                                                  vals[-1], acc, 0.01, 0.01))
    res["H6_dfm_train_step"] = {
        "config": "DeepFM k=128, MLP 150/200/150 partial_fit, batch 5000 rows, Frappe vocab",
        "unit": "steps/s", "gpu_ms_wall": ms, "gpu_rate": 1e3 / ms,
        "cpu_rate_numpy": 1.0 / c, "cpu_sample": "same batch, numpy oracle step"}
    del m
    torch.cuda.empty_cache()

print(json.dumps(res, indent=1))
