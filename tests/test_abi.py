"""CPU: the C-ABI library builds, loads and exports every symbol include/sda_engine.h declares.

No compute calls here (there is no GPU in the build container); the scheme-size helpers are pure
host functions and are checked against protocol/src/crypto.rs:117-155.
"""
import ctypes as C
import os
import re

import pytest

from sda_amd import engine as E
from sda_amd import schemes as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sda_engine.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(sda_\w+)\s*\(", text, re.M)))


def test_header_symbols_all_bound():
    decl = declared_symbols()
    bound = sorted(name for name, _, _ in E.SIGNATURES)
    assert decl == bound


def test_library_exports_every_symbol():
    lib = E.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_library_is_gfx950_code_object():
    blob = open(E.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_and_status_strings():
    lib = E.load_library()
    assert lib.sda_abi_version() == 1
    ref = {1: "Batch input wrong length", 2: "Sharing failed for packed secret sharing scheme",
           3: "Wrong dimension", 4: "Mismatching dimension", 5: "Inputs must have same length",
           6: "Not enough shares to reconstruct"}
    for code, text in ref.items():
        assert lib.sda_status_string(code).decode() == text


@pytest.mark.parametrize("sch", [S.Additive(3, 433), S.FULL_LOOP_PACKED, S.CONFIG_PACKED])
def test_scheme_sizes(sch):
    lib = E.load_library()
    c = sch.c()
    assert lib.sda_scheme_input_size(C.byref(c)) == sch.input_size()
    assert lib.sda_scheme_output_size(C.byref(c)) == sch.output_size()
    assert lib.sda_scheme_privacy_threshold(C.byref(c)) == sch.privacy_threshold()
    assert lib.sda_scheme_reconstruction_threshold(C.byref(c)) == sch.reconstruction_threshold()
    for d in (0, 1, 7, 8, 9, 1_000_000):
        k = sch.input_size()
        assert lib.sda_share_length(C.byref(c), d) == (d + k - 1) // k


def test_engine_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(E.SdaError) as ei:
        E.Engine(0)
    assert ei.value.status in (E.ERR_DEVICE, E.ERR_INVALID_ARGUMENT)


def test_every_entry_point_opens_a_call_scope():
    """engine.cpp: every sda_status entry point starts with SDA_ENTRY (the RAII CallScope that ends the
    call's stream-ordering scope on every return path), so no entry point can leave a stale
    stream behind for the next call's early fail()."""
    import re
    src = open(os.path.join(ROOT, "sda_amd", "csrc", "engine.cpp")).read()
    defs = list(re.finditer(r"^sda_status (sda_\w+)\([^)]*\)\s*\{\n(.*)\n", src, flags=re.M))
    assert len(defs) >= 30
    missing = [m.group(1) for m in defs if m.group(2).strip() != "SDA_ENTRY;"]
    assert not missing, missing
