"""The device-side generator (bench.py's input) is bit-identical to the numpy generator the parity
tests and the CPU baseline use."""
import numpy as np
import pytest

from siddhi_amd import synth


@pytest.mark.parametrize("n,seed,k,e,start", [(100_000, synth.SEEDS[4], 1_000_000, 1000, 0),
                                              (5_000, synth.SEEDS[1], 1000, 1, 12_345_678_901),
                                              (7_777, synth.SEEDS[2], 3, 7, 99)])
def test_torch_generator_matches_numpy(n, seed, k, e, start):
    a = synth.stock_ticks(n, seed, k, e, start)
    b = synth.stock_ticks_torch(n, seed, k, e, start, device="cpu")
    for key in a:
        assert np.array_equal(a[key], b[key].numpy()), key
