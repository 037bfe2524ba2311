"""DTW / median filter (oracle/align.py) pinned against transformers' _dynamic_time_warping / _median_filter."""
import numpy as np
import pytest
import torch
from transformers.models.whisper.generation_whisper import _dynamic_time_warping, _median_filter

from oracle.align import dtw, median_filter


@pytest.mark.parametrize("shape", [(1, 1), (3, 7), (12, 40), (40, 12), (25, 300)])
def test_dtw_matches_transformers(shape):
    x = np.random.default_rng(shape[0] * 31 + shape[1]).standard_normal(shape)
    a = dtw(x)
    b = _dynamic_time_warping(x.copy())
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_dtw_ties():
    x = np.zeros((5, 9))
    a = dtw(x)
    b = _dynamic_time_warping(x.copy())
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("width", [1, 3, 7])
def test_median_filter_matches_transformers(width):
    x = np.random.default_rng(width).standard_normal((2, 3, 5, 50)).astype(np.float32)
    ref = _median_filter(torch.from_numpy(x), width).numpy()
    assert np.allclose(median_filter(x, width), ref)
