"""North_star's state-parity bar, shared by every physics parity test.

Positions and velocities must lie within 1e-6 (absolute) of the fp64 oracle
stepped from the identical fp32 state (BASELINE.json north_star). Only where
|x| >= 8 — one fp32 ulp there is already 9.5e-7, so a correctly rounded fp32
result alone can miss an absolute 1e-6 — a 4-ulp term is added. No BASELINE
config reaches |x| >= 8 (headline half-width sqrt(8) = 2.83); only the
600-agent stress case can.

Every check records the largest error it saw (per test), and conftest prints
the table at the end of the session, so the observed margin is in the log.
"""
import numpy as np

STATE_ATOL = 1e-6
ULP_FROM = 8.0

MAX_ERR: dict = {}


def state_tol(ref):
    a = np.abs(np.asarray(ref, dtype=np.float64))
    ulp = 4 * np.spacing(a.astype(np.float32)).astype(np.float64)
    return np.where(a < ULP_FROM, STATE_ATOL, STATE_ATOL + ulp)


def _test_id():
    import os
    return os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]


def record(what, err):
    key = (_test_id(), what.split(" ")[0].split("(")[0].strip())
    MAX_ERR[key] = max(MAX_ERR.get(key, 0.0), float(err))


def check_state(got, ref, what):
    """|got - ref| <= state_tol(ref) elementwise; records the max error."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    # NaN where MPE gives NaN (App. A S16 strict mode) and nowhere else
    gn, rn = np.isnan(got), np.isnan(ref)
    assert np.array_equal(gn, rn), f"{what}: NaN pattern differs at {np.argwhere(gn != rn)[:5].tolist()}"
    got, ref = np.where(gn, 0.0, got), np.where(rn, 0.0, ref)
    err = np.abs(got - ref)
    m = float(err.max()) if err.size else 0.0
    record(what, m)
    bad = err > state_tol(ref)
    assert not bad.any(), f"{what}: max err {m:.3e} at {np.argwhere(bad)[:5].tolist()}"
    return m
