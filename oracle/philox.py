"""Philox4x32-10 counter-based RNG in NumPy uint64 arithmetic.

TEST INFRASTRUCTURE ONLY. Nothing under ``oracle/`` is imported by the product
path (``gs-marl_amd/``); only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg use it, as the checker.

Why Philox: the reference's ``scenario.reset_world`` draws entity positions from
the global ``np.random`` MT19937 stream (upstream MPE semantics, SURVEY.md
§8(a) row a11 [EXT]); that stream is sequential and cannot be reproduced per env
on a GPU. SURVEY.md Appendix A S14 fixes the [DECISION]: Philox4x32-10 keyed by
(seed) with counter (entity, episode, global env id, stream tag), identical in
this oracle and in ``gs-marl_amd/csrc/gsm_philox.h``.

Pinned against the Random123 published known-answer vectors
(``tests/test_philox_kat.py``) — Salmon et al., "Parallel random numbers: as
easy as 1, 2, 3" (SC'11), Random123 ``kat_vectors``.
"""
from __future__ import annotations

import numpy as np

_MASK = np.uint64(0xFFFFFFFF)
_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint64(0x9E3779B9)
_W1 = np.uint64(0xBB67AE85)

# Stream tags (counter word c3): keep layouts and any future draws disjoint.
TAG_LAYOUT = 0
TAG_ACTIONS = 1


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds.

    All arguments are array-likes of uint32 values (broadcastable). Returns a
    tuple of four uint32 arrays.
    """
    c0 = np.asarray(c0, dtype=np.uint64) & _MASK
    c1 = np.asarray(c1, dtype=np.uint64) & _MASK
    c2 = np.asarray(c2, dtype=np.uint64) & _MASK
    c3 = np.asarray(c3, dtype=np.uint64) & _MASK
    k0 = np.asarray(k0, dtype=np.uint64) & _MASK
    k1 = np.asarray(k1, dtype=np.uint64) & _MASK
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & _MASK
            k1 = (k1 + _W1) & _MASK
        p0 = _M0 * c0  # < 2^64: exact
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK, lo1, (hi0 ^ c3 ^ k1) & _MASK, lo0
    return tuple(x.astype(np.uint32) for x in (c0, c1, c2, c3))


def u01_f32(x):
    """uint32 -> float32 in [0, 1): (x >> 8) * 2^-24 (exact in fp32; Appendix A S14)."""
    x = np.asarray(x, dtype=np.uint32)
    return (x >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)
