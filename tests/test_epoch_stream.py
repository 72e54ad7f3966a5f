"""The epoch loops (H6 harness glue) against the reference's own Train.train.

tests/golden/epoch_stream.json holds, per batch, the sha256 of what the
reference's unmodified Train.train (FM.py:221-282, OurModel7.py:349-413) fed
``partial_fit`` over 2 epochs on synth_frappe (LoadData seeded 2016, loop
seeded 41 / 43, batch 512, Result = 1): the negatives, the label column, the
shuffle and the 512-row partitions.  ``run_training`` / ``run_training_hhfm``
must feed their model the identical stream (tests/golden/make_golden.py,
``gen_epoch_stream``).  Host only: the model is a recording stand-in."""
import argparse
import hashlib
import json
import os

import numpy as np

G = os.path.join(os.path.dirname(__file__), "golden")


class _Recorder:
    def __init__(self):
        self.batches = []

    def partial_fit(self, data):
        h = hashlib.sha256()
        for key in sorted(data):
            a = np.ascontiguousarray(np.asarray(data[key], dtype=np.float64))
            h.update(key.encode())
            h.update(np.asarray(a.shape, np.int64).tobytes())
            h.update(a.tobytes())
        self.batches.append(h.hexdigest())
        return 1.0


def _run(mod, seed, epochs, batch):
    from hhfm_amd.NewLoadData import LoadData
    np.random.seed(2016)
    d = LoadData(G + "/", "synth_frappe")
    from hhfm_amd import harness
    t = object.__new__(mod.Train)        # the model-specific __init__ builds a GPU model
    harness.Train.__init__(t, None, data=d, model=_Recorder())
    t.args = argparse.Namespace(Result=1, dataset="synth_frappe", result_file=None)
    t.epoch, t.batch_size, t.verbose, t.TopK = epochs + 1, batch, 0, 10
    t.context, t.time, t.time_dimension = True, False, 0
    np.random.seed(seed)
    t.train()
    return t.model.batches


def test_fm_epoch_stream_matches_reference():
    from hhfm_amd import FM
    ref = json.load(open(os.path.join(G, "epoch_stream.json")))
    got = _run(FM, ref["seeds"]["fm"], ref["epochs"], ref["batch_size"])
    assert len(got) == len(ref["fm"])
    assert got == ref["fm"]


def test_hhfm_epoch_stream_matches_reference():
    from hhfm_amd import OurModel7
    ref = json.load(open(os.path.join(G, "epoch_stream.json")))
    got = _run(OurModel7, ref["seeds"]["hhfm"], ref["epochs"], ref["batch_size"])
    assert len(got) == len(ref["hhfm"])
    assert got == ref["hhfm"]
