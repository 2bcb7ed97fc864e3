"""The bench line's counter-based roofline figures (bench.counter_bound,
DESIGN.md §5): each is a share of a measured ceiling, so none may exceed 1
(round 3's marginal-cost issue model read 1.23 for C4), and `bound` names the
largest share once it reaches BOUND_AT. Checked on synthetic counters and on
every committed PMC entry with the committed lines' kernel times (CPU only)."""
import json
from pathlib import Path

import pytest

import bench

ROOT = Path(__file__).resolve().parents[1]


def _pmc(valu, salu, hbm_bytes, cycles):
    return dict(hbm_bytes_per_launch=hbm_bytes, grbm_gui_active_per_launch=cycles * bench.N_XCDS,
                valu_insts_per_launch=valu, salu_insts_per_launch=salu, waves=1024,
                wave_quad_cycles_per_launch=1000.0, active_inst_any_quad_cycles_per_launch=300.0)


def test_counter_bound_classifies():
    cyc = 10000.0
    ms = cyc / 2.4e9 * 1e3
    # a VALU stream at 70% of its ceiling binds
    r = bench.counter_bound(_pmc(0.7 * bench.N_SIMDS * cyc * bench.VALU_PEAK, 0.0, 1.0, cyc), ms, 0.1)
    assert r["bound"] == "issue" and r["binding_pipe"] == "valu"
    assert r["valu_frac"] == pytest.approx(0.7, rel=1e-3)
    assert r["wave_issue_frac"] == pytest.approx(0.3)
    # nothing above BOUND_AT: latency-bound
    r = bench.counter_bound(_pmc(0.3 * bench.N_SIMDS * cyc * bench.VALU_PEAK,
                                 0.2 * bench.N_CUS * cyc * bench.SALU_PEAK, 1.0, cyc), ms, 0.1)
    assert r["bound"] == "latency"
    # HBM bytes at 80% of 8 TB/s over the kernel time
    r = bench.counter_bound(_pmc(0.0, 0.0, 0.8 * bench.HBM_PEAK_GBS * 1e9 * ms * 1e-3, cyc), ms, 0.1)
    assert r["bound"] == "hbm" and r["hbm_frac_physical"] == pytest.approx(0.8, rel=1e-3)
    # no counters: every figure null
    assert bench.counter_bound(None, ms, 0.1)["bound"] is None


def test_committed_lines_fractions_at_most_one():
    """Every committed bench line of the round's package: the counter-based
    shares are at most 1 and agree with counter_bound on the committed PMC."""
    import re

    def order(d):   # r5_lines < r5z_lines < r6_lines < r6w_package
        m = re.match(r"r(\d+)(\w*?)_(lines|package)$", d.name)
        return (int(m.group(1)), m.group(2)) if m else (-1, "")
    dirs = [d for d in (ROOT / "profiles").glob("r*_*") if d.is_dir() and order(d)[0] >= 0]
    newest = max(dirs, key=order)
    lines = sorted(newest.glob("bench_*.json"))
    pmc = json.loads((ROOT / "profiles" / "pmc_kernels.json").read_text())
    assert lines and pmc["entries"]
    seen = 0
    for f in lines:
        d = json.loads(f.read_text())
        r = d.get("roofline") or {}
        if r.get("valu_frac") is None:
            continue   # eager / closed-loop lines carry no rollout PMC
        seen += 1
        for k in ("frac", "hbm_frac_physical", "valu_frac", "salu_frac", "wave_issue_frac"):
            assert 0.0 <= r[k] <= 1.0, (f.name, k, r[k])
        key = r["pmc"]["key"]
        again = bench.counter_bound(pmc["entries"][key], r["mean_launch_us"] * 1e-3, r["frac"])
        assert again["bound"] == r["bound"], f.name
        assert again["valu_frac"] == pytest.approx(r["valu_frac"], abs=2e-4), f.name
    assert seen >= 6
