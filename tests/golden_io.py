"""Helpers to read the committed golden fixtures (tests/golden/*.npz)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def tokens_list(arr):
    return [[int(v) for v in row if v >= 0] for row in arr]
