"""The C-ABI library loads and exports every function include/*.h declares
(no compute: there may be no GPU here)."""
import ctypes
import os
import re

from hypermerge_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for f in os.listdir(os.path.join(ROOT, "include")):
        if f.endswith(".h"):
            src = open(os.path.join(ROOT, "include", f)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names.update(re.findall(r"\b(hm_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    L = engine.lib()
    decl = declared_functions()
    assert decl, "no declarations parsed"
    assert decl == set(engine.EXPORTS)
    for name in decl:
        assert hasattr(L, name), name


def test_abi_version_and_messages():
    L = engine.lib()
    assert L.hm_abi_version() == 4
    assert L.hm_status_message(1) == b"Inconsistent reuse of sequence number"
    assert L.hm_status_message(2) == b"Modification of unknown object"


def test_struct_layouts_match_header():
    from hypermerge_amd import columnar as C
    assert ctypes.sizeof(C.CBatch) == 12 * 4 + 5 * 8
    assert ctypes.sizeof(C.CResults) == 8 * 8


def test_engine_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        return
    try:
        engine.Engine(0)
    except engine.EngineError as e:
        assert "HIP device error" in str(e)
    else:
        raise AssertionError("Engine() must not silently fall back to the CPU")
