"""Loader for the committed golden fixtures (tests/golden/*.npz|json).

The fixtures were produced by tests/golden/make_golden.py from the reference
implementation itself (see that script's header).  Arrays are loaded with
numpy.load(allow_pickle=False)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def eden():
    arrays = np.load(os.path.join(GOLDEN, "eden_golden.npz"), allow_pickle=False)
    with open(os.path.join(GOLDEN, "eden_golden.json")) as f:
        index = json.load(f)
    return arrays, index


def lossy():
    arrays = np.load(os.path.join(GOLDEN, "lossy_golden.npz"), allow_pickle=False)
    with open(os.path.join(GOLDEN, "lossy_golden.json")) as f:
        index = json.load(f)
    return arrays, index


def metadata_of(case):
    """int_to_float dict of a golden Eden.compress case (eden_pipeline.py:779-785)."""
    md = {0: float(case["seed"]), 1: float(case["total_dim"])}
    k = 2
    for s, d in zip(case["scales"], case["dims"]):
        md[k] = s
        md[k + 1] = float(d)
        k += 2
    return md
