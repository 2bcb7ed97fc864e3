import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "gs-marl_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def ocfg_factory():
    """Build an oracle config from product EnvConfig kwargs."""
    from oracle import batch_ref as br

    def make(**kw):
        return br.make_cfg(**kw)
    return make


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Largest position/velocity error seen per test against the fp64 oracle
    (bar: 1e-6 absolute, tests/parity_tol.py)."""
    try:
        from parity_tol import MAX_ERR
    except ImportError:
        return
    if not MAX_ERR:
        return
    tr = terminalreporter
    tr.section("state parity: max |got - fp64 oracle| (bar 1e-6)")
    for (test, what), err in sorted(MAX_ERR.items()):
        tr.write_line(f"{err:.3e}  {what:<4} {test}")
    tr.write_line(f"{max(MAX_ERR.values()):.3e}  overall max")
    import json
    import os
    out = os.environ.get("GSM_MAXERR_JSON")
    if out:
        with open(out, "w") as f:
            json.dump({f"{t}::{w}": e for (t, w), e in sorted(MAX_ERR.items())}, f, indent=1)


def pytest_collection_modifyitems(config, items):
    """GPU tests skip (not fail) on a machine without a GPU, unless
    GSM_REQUIRE_GPU=1 demands one (the GPU box runs them with -m gpu)."""
    import os
    if gpu_available() or os.environ.get("GSM_REQUIRE_GPU") == "1":
        return
    skip = pytest.mark.skip(reason="no ROCm GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
