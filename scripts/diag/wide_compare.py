"""Diagnostic: compare wide_probe outputs of several builds against the
shipped build (argv[1]); prints max |diff| / max |ref| per case and which
rows (mod the 16-row tile and per block) differ."""
import sys

import numpy as np

ref = np.load(sys.argv[1])
for path in sys.argv[2:]:
    d = np.load(path)
    print("==", path)
    for key in sorted(d.files):
        a, b = d[key], ref[key]
        bad = np.nonzero(a != b)[0]
        msg = f"  {key}: {len(bad)}/{len(a)} rows differ, max rel {np.abs(a - b).max() / np.abs(b).max():.3g}"
        if len(bad):
            msg += f"; first {bad[:12].tolist()} row%16 hist {np.bincount(bad % 16, minlength=16).tolist()}"
        print(msg)
