import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pytest_terminal_summary(terminalreporter):
    """Per-case parity record: fp32 tie swaps in top-K lists and
    ill-conditioned (κ > 100) row counts, case by case (tests/helpers.py)."""
    try:
        from tests.helpers import PARITY_LOG
    except ImportError:
        return
    if not PARITY_LOG:
        return
    import json
    agg = {}
    for r in PARITY_LOG:
        a = agg.setdefault((r["test"], r["kind"]), {"calls": 0})
        a["calls"] += 1
        for key, v in r.items():
            if key in ("test", "kind"):
                continue
            if key.startswith("max_"):
                a[key] = max(a.get(key, 0.0), v)
            else:
                a[key] = a.get(key, 0) + v
    tr = terminalreporter
    tr.write_sep("-", "parity record (per case)")
    swaps = sum(v.get("swaps", 0) for v in agg.values())
    pos = sum(v.get("positions", 0) for v in agg.values())
    for (test, kind), v in sorted(agg.items()):
        if kind == "topk_tie_swaps":
            tr.write_line(f"{test}: {v['swaps']} fp32 tie swaps of {v['positions']} positions")
        else:
            tr.write_line(f"{test}: {v['rows_kappa_gt_100']} of {v['rows']} rows with κ > 100; "
                          f"max rel err κ<=100 {v['max_rel_err_kappa_le_100']:.3g}, κ>100 gpu "
                          f"{v['max_rel_err_kappa_gt_100']:.3g} / fp32 oracle "
                          f"{v['oracle_max_rel_err_kappa_gt_100']:.3g}")
    tr.write_line(f"total: {swaps} verified fp32 tie swaps of {pos} top-K positions")
    path = os.environ.get("HHFM_PARITY_REPORT")
    if path:
        with open(path, "w") as f:
            json.dump([dict(test=t, kind=kd, **v) for (t, kd), v in sorted(agg.items())], f,
                      indent=1)
