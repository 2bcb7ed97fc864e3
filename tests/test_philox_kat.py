"""Philox4x32-10 known-answer tests (Random123 kat_vectors; Salmon et al. SC'11).

These pin the reset-layout RNG of both the oracle and the HIP kernels (the
kernels are checked against the oracle bit for bit in test_gpu_parity.py)."""
import numpy as np
import pytest

from oracle.philox import philox4x32_10, u01_f32

KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_random123_kat(ctr, key, expect):
    out = philox4x32_10(*ctr, *key)
    assert tuple(int(x) for x in out) == expect


def test_vectorised_matches_scalar():
    rng = np.random.default_rng(1)
    c = rng.integers(0, 2**32, size=(4, 100), dtype=np.uint64)
    k = rng.integers(0, 2**32, size=2, dtype=np.uint64)
    vec = philox4x32_10(*c, *k)
    for j in range(0, 100, 17):
        sc = philox4x32_10(*(int(x[j]) for x in c), *(int(x) for x in k))
        assert all(int(vec[w][j]) == int(sc[w]) for w in range(4))


def test_u01_range_and_exactness():
    x = np.array([0, 255, 256, 0xFFFFFFFF], dtype=np.uint32)
    u = u01_f32(x)
    assert u.dtype == np.float32
    assert u[0] == 0 and u[1] == 0 and u[2] == np.float32(2**-24)
    assert u[3] == np.float32(1 - 2**-24) and u[3] < 1
