"""CPU: the shipped code objects' register budgets (no GPU needed).

Rounds 4 and 5 each saw `test_packed_random_schemes[8]` (k = 52, t = 11, n + 1 = 81, p < 2^24) fault on the GPU
after an unrelated edit recompiled the n + 1 = 81 share-gen kernels.  The kernel that scheme ran had 405 of 512
registers (149 AGPRs standing in for VGPRs: this engine has no MFMA work) and 202 SGPR spills; its non-WIDE
sibling had 388 bytes of scratch.  Round 6 removed that class of kernel ("Register budget at
n + 1 = 81"): these tests read every kernel's metadata from sda_amd/libsda_engine.so and fail if it comes back.

The checks are on the library the GPU tests load, parsed in pure Python (scripts/code_objects.py).
"""
import importlib.util
import os
import re
import shutil
import subprocess

import pytest

from sda_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("code_objects", os.path.join(ROOT, "scripts", "code_objects.py"))
CO = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(CO)


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(E.LIB_PATH):
        pytest.fail(f"{E.LIB_PATH} is not built (run __graft_entry__.build())")
    rows = CO.kernels(E.LIB_PATH)
    assert len(rows) > 100, "the fat binary parser found too few kernels"
    return rows


def _gen_args(pretty):
    m = re.match(r"packed_gen_kernel<(\d+), (\d+), (\w+), (\w+), (\w+), (\w+)>", pretty)
    return None if not m else (int(m[1]), int(m[2])) + tuple(x == "true" for x in m.groups()[2:])


def test_share_gen_kernels_have_no_scratch_spills_or_agprs(kernels):
    gen = [k for k in kernels if "packed_gen" in k["pretty"]]
    assert len(gen) >= 70
    bad = [(k["pretty"], k["vgpr"], k["agpr"], k["scratch"], k["vgpr_spill"]) for k in gen
           if k["scratch"] or k["vgpr_spill"] or k["agpr"] or k["vgpr"] > 256]
    assert not bad, f"share-gen kernels past the 256-VGPR budget: {bad}"


def test_share_gen_instantiations_follow_the_register_path_rule(kernels):
    """The non-lazy exact kernels (p < 2^24 or odd B) at n + 1 = 81 exist only for L <= 8; from L = 16 the
    dispatcher sends those schemes to packed_wide.hip (packed_gen.hip gen_register_path)."""
    seen = {_gen_args(k["pretty"]) for k in kernels}
    seen.discard(None)
    expect = set()
    for n3, ls in ((3, (2,)), (9, (2, 4, 8)), (27, (2, 4, 8, 16)), (81, (2, 4, 8, 16, 32, 64))):
        for L in ls:
            expect |= {(L, n3, True, False, True, True), (L, n3, True, False, True, False),
                       (L, n3, True, True, False, False), (L, n3, False, True, False, False)}
            if not (n3 == 81 and L >= 16):
                expect |= {(L, n3, True, False, False, False), (L, n3, False, False, False, False)}
    assert seen == expect, (sorted(seen - expect), sorted(expect - seen))


# Scratch by design: the reveal fix-up's generic path keeps tss' Newton points in a private i64 array (rare:
# raw i64 shares or a trapped batch, DESIGN.md §4.2 "exact reveal, counter-backed"); the opt-in fused codec's
# multi-round variant (elements longer than 5 bytes, SDA_CODEC_PATH=fused) spills 16 VGPRs.
SCRATCH_OK = ("packed_reveal_fixup_kernel<", "varint_decode_combine_kernel<8, false>")


def test_no_kernel_uses_agprs_or_spills_outside_the_listed_paths(kernels):
    agpr = sorted(k["pretty"] for k in kernels if k["agpr"])
    assert not agpr, f"AGPRs used as VGPR overflow (no kernel here issues MFMA): {agpr}"
    scratch = sorted(k["pretty"] for k in kernels
                     if (k["scratch"] or k["vgpr_spill"]) and not k["pretty"].startswith(SCRATCH_OK))
    assert not scratch, f"unexpected scratch / VGPR spills: {scratch}"


def test_hot_path_kernels_fit_their_occupancy(kernels):
    """The benchmarked kernels: no scratch, no spills, and the VGPR counts their DESIGN.md occupancy needs."""
    want = {  # kernel prefix -> max VGPRs (waves per SIMD in DESIGN.md)
        "combine_exact_kernel<long, 2, 8": 64,                 # §4.1: 46 VGPRs, occupancy 8 (SDA_COMBINE_PIPE=0)
        "combine_exact_kernel<long, 2, 4": 64,                 # §4.1: the pipelined default, 54-60 VGPRs, occupancy 8
        "packed_gen_kernel<16, 27, true, true, false, false>": 102,   # canonical, 5 waves
        "packed_gen_kernel<16, 27, true, false, true, true>": 102,    # exact sign-bit, 5 waves
        "packed_reveal_exact_kernel<16, true, 8, true, true>": 64,    # exact reveal, 8 waves
        "packed_reveal_canon_kernel<16, true>": 128,
    }
    for prefix, cap in want.items():
        rows = [k for k in kernels if k["pretty"].startswith(prefix)]
        assert rows, prefix
        for k in rows:
            assert k["vgpr"] <= cap and not k["scratch"] and not k["vgpr_spill"], (k["pretty"], k["vgpr"])


def _objdump():
    for p in ("/opt/rocm/lib/llvm/bin/llvm-objdump", shutil.which("llvm-objdump") or ""):
        if p and os.path.exists(p):
            return p
    return None


def test_lds_dma_stage_issues_every_chunk_before_one_wait(kernels, tmp_path):
    """packed_gen.hip's LDS-DMA stage (both benchmarked share-gen kernels at configs[2]): no s_waitcnt between
    its global_load_lds issues (round 5 had a vmcnt(0) between the secrets and draws loops), and a vmcnt(0) of
    its own before the s_barrier (the barrier does not wait for another wave's DMA writes to LDS)."""
    objdump = _objdump()
    if objdump is None:
        pytest.skip("llvm-objdump not available")
    cos = list(CO.code_objects(E.LIB_PATH))
    hits = 0
    for i, co in enumerate(cos):
        names = [k[".name"] for k in CO.kernel_metadata(co)]
        # <16, 27, WIDE, CANON, LAZY, SIGNBIT>: canonical <1,1,0,0> and exact sign-bit <1,0,1,1>
        targets = [n for n in names if "packed_gen_kernelILi16ELi27ELb1ELb1ELb0ELb0E" in n
                   or "packed_gen_kernelILi16ELi27ELb1ELb0ELb1ELb1E" in n]
        if not targets:
            continue
        path = tmp_path / f"co{i}.o"
        path.write_bytes(co)
        asm = subprocess.run([objdump, "-d", "--no-show-raw-insn", str(path)], capture_output=True, text=True,
                             check=True).stdout
        for name in targets:
            body = asm.split(f"<{name}>:", 1)[1].split("\n\n", 1)[0].split("\n")
            dma = [j for j, l in enumerate(body) if "global_load_lds" in l]
            assert dma, name
            between = [l.strip() for l in body[dma[0]:dma[-1]] if "s_waitcnt" in l]
            assert not between, (name, between)
            bar = next(j for j in range(dma[-1], len(body)) if "s_barrier" in body[j])
            assert any("vmcnt(0)" in l for l in body[dma[-1]:bar]), name
            hits += 1
    assert hits == 2


def test_reveal_kernels_have_no_static_lds(kernels):
    """The staged reveal flush reads its results back from the dynamic LDS base as 16-byte words
    (packed_reveal.hip, reveal_flush): that base is 16-byte aligned only while no static LDS precedes it."""
    rows = [k for k in kernels if k["pretty"].startswith(("packed_reveal_exact_kernel<", "packed_reveal_canon_kernel<"))]
    assert rows
    assert all(k["lds"] == 0 for k in rows), [(k["pretty"], k["lds"]) for k in rows if k["lds"]]
