"""NormalizeImage lookup table (ffcv/transforms/normalize.py:42-49).

``table = (arange(256)[:, None] - mean) / std`` in float64, cast to the
target dtype; float16 tables are carried as int16 bits (normalize.py:45-48).
"""
import numpy as np


def make_lut(mean, std, dtype=np.float16):
    table = (np.arange(256)[:, None] - np.asarray(mean)[None, :]) / np.asarray(std)[None, :]
    return table.astype(dtype)
