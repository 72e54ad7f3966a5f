#!/usr/bin/env python3
"""Render profiles/r01_rows.json (scripts/rowtable.py) as the DESIGN.md table."""
import json
import sys

ROWS = [("C2_M1_fm_rows", "M1 (C2)"), ("C3_H2_hhfm_catalog", "H2 (C3)"),
        ("C4_H2_hhfm_catalog_shard", "H2 (C4)"), ("C5_D1_dfm_bf16_mlp", "D1 (C5)"),
        ("C5_D1_dfm_fp32_mlp", "D1 (C5)"), ("A1_afm_rows", "A1"), ("A2_afm_catalog", "A2"),
        ("H6_hhfm_train_step", "H6"), ("H6_afm_train_step", "H6"), ("H6_dfm_train_step", "H6"),
        ("H5_sample_negative", "H5")]


def si(x):
    for d, s in ((1e12, " T"), (1e9, " G"), (1e6, " M"), (1e3, " k")):
        if x >= d:
            return f"{x / d:.3g}{s}"
    return f"{x:.3g} "


d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "profiles/r01_rows.json"))
print("| row | workload | GPU | roofline frac | CPU (1 thread / 16 threads, or numpy) |")
print("|---|---|---|---|---|")
for key, name in ROWS:
    v = d.get(key)
    if not v:
        continue
    ms = v.get("gpu_ms", v.get("gpu_ms_wall"))
    rf = v.get("roofline")
    frac = f"{rf['bound']}: {rf['frac']:.2f}" if rf else "—"
    if "cpu_rate_1t" in v:
        cpu = f"{si(v['cpu_rate_1t'])}/ {si(v['cpu_rate_nt'])}{v['unit']}"
    else:
        cpu = f"numpy {si(v['cpu_rate_numpy'])}{v['unit']}"
    print(f"| {name} | {v['config']} | {si(v['gpu_rate'])}{v['unit']} ({ms:.3g} ms) | {frac} | {cpu} |")
