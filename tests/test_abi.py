"""C ABI checks that need no GPU: libgsm.so loads, exports every symbol
include/gsm.h declares with the struct layouts the binding assumes, and the
host-only entry points validate their arguments."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "gsm.h"


def declared_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s+(gsm_\w+)\s*\(", text, re.M)))


@pytest.fixture(scope="module")
def lib():
    from gsmarl_amd import _lib
    if not _lib.LIB_PATH.exists():
        import __graft_entry__ as g
        g.build()
    return _lib.load()


def test_header_declares_expected_api():
    names = declared_functions()
    assert "gsm_step" in names and "gsm_reset" in names and len(names) >= 12


def test_every_declared_symbol_is_exported(lib):
    from gsmarl_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (gsm_\w+)", out))
    for name in declared_functions():
        assert name in exported, name
        assert hasattr(lib, name)
    # the binding types every declared function
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_struct_layouts_match_header(lib, tmp_path):
    """Compile a tiny C probe against gsm.h and compare offsets with ctypes."""
    from gsmarl_amd import _lib
    probe = tmp_path / "probe.c"
    fields_cfg = [f for f, _ in _lib.GsmConfig._fields_]
    fields_buf = [f for f, _ in _lib.GsmBuffers._fields_]
    fields_sz = [f for f, _ in _lib.GsmSizes._fields_]
    fields_out = [f for f, _ in _lib.GsmOutputs._fields_]
    fields_st = [f for f, _ in _lib.GsmState._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gsm.h"', "int main(void){"]
    for s, fs in (("gsm_config", fields_cfg), ("gsm_buffers", fields_buf), ("gsm_sizes", fields_sz),
                  ("gsm_outputs", fields_out), ("gsm_state", fields_st)):
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f in fs:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    probe.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(probe), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.split("\n") if l)
    for s, cls in (("gsm_config", _lib.GsmConfig), ("gsm_buffers", _lib.GsmBuffers), ("gsm_sizes", _lib.GsmSizes),
                   ("gsm_outputs", _lib.GsmOutputs), ("gsm_state", _lib.GsmState)):
        assert int(got[s]) == C.sizeof(cls), s
        for f, _ in cls._fields_:
            assert int(got[f"{s}.{f}"]) == getattr(cls, f).offset, f"{s}.{f}"


def test_query_sizes_and_validation(lib):
    from gsmarl_amd import EnvConfig, _lib
    s = _lib.query_sizes(EnvConfig(n_agents=24, n_envs=8192), lib)
    assert s.n_entities == 72 and s.node_feat_dim == 7 and s.obs_dim == 6
    assert s.max_edges_per_env == 48 * 47 + 48
    assert s.edge_capacity == 8192 * s.max_edges_per_env
    assert s.n_blocks == 8192 // s.envs_per_block
    for bad in (dict(n_envs=0), dict(n_agents=0), dict(dt=0.0), dict(damping=1.5),
                dict(n_agents=24, n_envs=2_000_000)):
        with pytest.raises(_lib.GsmError):
            _lib.query_sizes(EnvConfig(**bad), lib)
    c = _lib.make_config(EnvConfig())
    c.abi_version = 99
    assert lib.gsm_query_sizes(C.byref(c), C.byref(_lib.GsmSizes())) == _lib.GSM_EINVAL
    assert "abi_version" in _lib.last_error(lib)


def test_create_bind_destroy_host_only(lib):
    """gsm_create/gsm_destroy and argument errors touch no GPU."""
    from gsmarl_amd import EnvConfig, _lib
    c = _lib.make_config(EnvConfig(n_agents=3, n_envs=4))
    h = C.c_void_p()
    assert lib.gsm_create(C.byref(c), C.byref(h)) == _lib.GSM_OK and h.value
    # step before bind -> ESTATE, no launch
    assert lib.gsm_step(h, C.c_void_p(1), 1, None) == _lib.GSM_ESTATE
    assert "gsm_bind" in _lib.last_error(lib, h)
    assert lib.gsm_graph_launch(h, 0, None) == _lib.GSM_ESTATE
    assert lib.gsm_graph_launch(h, 9, None) == _lib.GSM_EINVAL
    bufs = _lib.GsmBuffers()
    assert lib.gsm_bind(h, C.byref(bufs)) == _lib.GSM_EINVAL     # NULL pointers
    assert lib.gsm_destroy(h) == _lib.GSM_OK
    assert lib.gsm_destroy(None) == _lib.GSM_OK


def test_capture_into_argument_checks_host_only(lib):
    """gsm_graph_capture_into rejects a NULL handle, an unbound handle and a
    bad slot before it touches a slot, a buffer or the GPU (a navigation bind
    only records the pointers: fake non-NULL ones make no HIP call)."""
    from gsmarl_amd import EnvConfig, _lib
    outs = (_lib.GsmOutputs * 2)()
    a = C.c_void_p(4096)
    assert lib.gsm_graph_capture_into(None, 0, a, 16, 1, 2, 1, outs) == _lib.GSM_EINVAL
    c = _lib.make_config(EnvConfig(n_agents=24, n_envs=4))
    h = C.c_void_p()
    assert lib.gsm_create(C.byref(c), C.byref(h)) == _lib.GSM_OK
    assert lib.gsm_graph_capture_into(h, 0, a, 16, 1, 2, 1, outs) == _lib.GSM_ESTATE   # before bind
    assert lib.gsm_graph_capture(h, 0, a, 16, 1, 2, 1, _lib.GRAPH_ROLL) == _lib.GSM_ESTATE
    fake = {f: 4096 * (i + 1) for i, (f, _) in enumerate(_lib.GsmBuffers._fields_)}
    fake["lsa_v"] = fake["lsa_col"] = fake["lsa_stats"] = fake["env_shape"] = fake["assign"] = None
    bufs = _lib.GsmBuffers(**fake)
    assert lib.gsm_bind(h, C.byref(bufs)) == _lib.GSM_OK
    for bad in (-1, 4, 1 << 20):
        assert lib.gsm_graph_capture_into(h, bad, a, 16, 1, 2, 1, outs) == _lib.GSM_EINVAL, bad
        assert "slot" in _lib.last_error(lib, h)
        assert lib.gsm_graph_capture(h, bad, a, 16, 1, 2, 1, _lib.GRAPH_ROLL) == _lib.GSM_EINVAL, bad
    assert lib.gsm_graph_capture_into(h, 0, a, 16, 1, 2, 1, None) == _lib.GSM_EINVAL   # NULL per_step
    assert lib.gsm_get_state(h, None, None) == _lib.GSM_EINVAL
    assert lib.gsm_set_state(None, C.byref(_lib.GsmState()), None) == _lib.GSM_EINVAL
    assert lib.gsm_destroy(h) == _lib.GSM_OK


def test_product_path_fails_loudly_without_gpu():
    import torch
    from gsmarl_amd import EnvConfig, GpuBatchEnv, _lib
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.GsmError, match="no CPU fallback"):
        GpuBatchEnv(EnvConfig(), "cuda")
    with pytest.raises(_lib.GsmError):
        GpuBatchEnv(EnvConfig(), "cpu")


def test_product_does_not_import_oracle():
    for p in (ROOT / "gs-marl_amd").rglob("*.py"):
        src = p.read_text()
        assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, re.M), p
