"""GPU: the C ABI from a plain C program, with no torch and no Python in its process.

tests/abi_c/full_loop.c links libsda_engine.so and the ROCm runtime it was built against
(/opt/rocm/lib/libamdhip64), which is how the Rust FFI shim of INTEGRATION.md would bind it; every
other GPU test reaches the engine through ctypes inside a torch process (whose bundled HIP runtime
then serves the engine too).  It runs the four integration-tests/tests/full_loop.rs:30-150 variants
with the golden fixture's draws and must reproduce every stage of the golden trace and
`[2, 4, 6, 8]` (full_loop.rs:148).

This module sorts before the other GPU test modules, so the subprocesses start before this pytest
process has touched the GPU.
"""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "abi_c", "full_loop")

KIND_MASK = {"None": 0, "Full": 1, "ChaCha": 2}


def _program_input(v):
    (mk, mp), = v["masking"].items() if isinstance(v["masking"], dict) else (("None", {}),)
    (sk, sp), = v["sharing"].items()
    lines = [f"{KIND_MASK[mk]} {mp.get('modulus', 0)} {mp.get('dimension', 0)} {mp.get('seed_bitsize', 0)}"]
    if sk == "Additive":
        lines.append(f"0 {sp['share_count']} {sp['modulus']} 1 {sp['share_count'] - 1} 0 0")
    else:
        lines.append(f"1 {sp['share_count']} {sp['prime_modulus']} {sp['secret_count']} {sp['privacy_threshold']} "
                     f"{sp['omega_secrets']} {sp['omega_shares']}")
    t = v["trace"]
    D = len(v["inputs"][0])
    lines.append(f"{D} 433 {len(v['inputs'])}")
    for p, secrets in enumerate(v["inputs"]):
        masks = t["masks"][p] if mk != "None" else []
        lines.append(" ".join(map(str, secrets)))
        lines.append(" ".join(map(str, [len(masks)] + masks)))
        lines.append(" ".join(map(str, [len(t["draws"][p])] + t["draws"][p])))
    n = len(t["clerk_results"])
    lines.append(" ".join(map(str, [n] + list(range(n)))))
    return "\n".join(lines) + "\n"


def _parse(out):
    res = {}
    for line in out.splitlines():
        if ":" in line:
            k, v = line.split(":", 1)
            try:
                res[k.strip()] = [int(x) for x in v.split()]
            except ValueError:      # not one of the program's lines (RCCL prints its version banner at init)
                continue
    return res


HBM_BIN = os.path.join(HERE, "abi_c", "hbm_cycle")


def _ensure_built():
    if not (os.path.exists(BIN) and os.path.exists(HBM_BIN)):
        subprocess.run(["make", "-C", os.path.dirname(BIN)], check=True, capture_output=True)


def _hbm_cycle(*args, timeout=300):
    _ensure_built()
    env = {k: val for k, val in os.environ.items() if not k.startswith(("PYTHON", "SDA_HBM"))}
    r = subprocess.run([HBM_BIN, *args], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, (r.stdout, r.stderr)
    return {k.strip(): v.split() for k, v in (l.split(":", 1) for l in r.stdout.splitlines() if ":" in l)}


@pytest.mark.parametrize("devices", ["", "0", "0,0,0"], ids=["handle", "multi1", "multi3"])
@pytest.mark.parametrize("variant", ["simple", "with_fullmask", "with_chachamask", "with_packedshamir"])
def test_c_program_full_loop(variant, devices):
    """One device handle, a one-device multi handle (ChaCha through a one-rank RCCL communicator, RCCL loaded
    from /opt/rocm in a process without torch) and a three-slice handle on one GPU (sda_engine_create_multi)."""
    with open(os.path.join(HERE, "golden", "full_loop_kat.json")) as f:
        v = json.load(f)[variant]
    _ensure_built()
    env = {k: val for k, val in os.environ.items() if not k.startswith("PYTHON")}
    env["SDA_TEST_DEVICES"] = devices
    r = subprocess.run([BIN], input=_program_input(v), capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    got, t = _parse(r.stdout), v["trace"]
    for p in range(len(v["inputs"])):
        assert got[f"masks {p}"] == t["masks"][p]
        assert got[f"masked {p}"] == t["masked"][p]
        for c, row in enumerate(t["shares"][p]):
            assert got[f"shares {p} {c}"] == row
    for c, row in enumerate(t["clerk_results"]):
        assert got[f"clerk {c}"] == row
    if t["combined_mask"] is not None:
        assert got["combined_mask"] == t["combined_mask"]
    assert got["masked_output"] == t["masked_output"]
    assert got["output"] == t["output"]
    assert got["positive"] == [2, 4, 6, 8] == got["fused_reveal"]        # full_loop.rs:148


def test_c_program_does_not_load_torch():
    """The C consumer's process maps /opt/rocm's HIP runtime and no torch library."""
    _ensure_built()
    r = subprocess.run(["ldd", BIN], capture_output=True, text=True, timeout=60)
    assert "libsda_engine.so" in r.stdout and "/opt/rocm" in r.stdout and "torch" not in r.stdout


def test_c_hbm_trim_realloc_sequence():
    """The round-4 corruption's sequence (tests/test_gpu_hbm.py::test_hbm_trim_realloc_sequence_matches_torch) on
    the ROCm runtime the Rust shim would load: three rounds of a filled 2.4 GB buffer freed and released, a
    foreign hipMalloc block, new sda_hbm buffers (none in a retired range) and share-gen into one of them, equal
    to share-gen into a hipMalloc buffer on two reads, the foreign block untouched (tests/abi_c/hbm_cycle.c)."""
    out = _hbm_cycle("seq")
    assert out["seq"][0] == "ok" and int(out["seq"][4]) == 0          # pooled 0 after the final trim
    assert int(out["seq"][6]) > 0                                       # the released ranges were retired


def test_c_configs2_share_gen_matches_fixture():
    """configs[2] (k=8 n=26 t=7, p = 2147482801) at 1M-dim from plain C: the host entry point and the _dev entry
    point into an sda_hbm buffer both give the oracle's tss shares (checksums, tests/golden/abi_c_sharegen.json)."""
    with open(os.path.join(HERE, "golden", "abi_c_sharegen.json")) as f:
        want = [str(x) for x in json.load(f)["checksum"]]
    out = _hbm_cycle("gen")
    assert out["gen_host"] == want and out["gen_dev"] == want


def test_c_hbm_10000_mixed_cycles_retire_nothing():
    """10,000 jobs of 1-3 buffers of 2-192 MiB (2 MiB chunks): size-class reuse keeps the pool bounded and no
    trim happens, so not one byte of address space is retired (the bound this test states: 0 bytes with the
    default SDA_HBM_POOL_MB; the pool's peak stays far below it)."""
    out = _hbm_cycle("cycle", "10000", timeout=600)
    c = dict(zip(out["cycle"][0::2], (int(x) for x in out["cycle"][1::2])))
    assert c["cycles"] == 10000 and c["retired"] == 0 and c["live"] == 0
    assert c["peak_pooled"] < (32768 << 20) // 4
