"""Read the gfx950 code objects inside the engine library and report each kernel's resources.

    python scripts/code_objects.py [sda_amd/libsda_engine.so] [--all]

Pure Python: ELF section table -> `.hip_fatbin` -> every clang offload bundle's gfx950 entry -> the code
object's NT_AMDGPU_METADATA note (msgpack) -> `amdhsa.kernels`.  Used by tests/test_kernel_resources.py, which
fails when a shipped share-gen kernel has scratch, spills or AGPR use ("Register budget at
n + 1 = 81"), and to print the table quoted there.  No GPU and no LLVM tools needed.
"""
import os
import struct
import subprocess
import sys

import msgpack

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = b"hipv4-amdgcn-amd-amdhsa--gfx950"
NT_AMDGPU_METADATA = 32


def _sections(elf: bytes):
    """{name: (offset, size, type)} of a little-endian ELF64 image."""
    assert elf[:4] == b"\x7fELF" and elf[4] == 2, "not an ELF64 image"
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        name, typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        hdrs.append((name, typ, off, size))
    stro = hdrs[shstrndx][2]
    out = {}
    for name, typ, off, size in hdrs:
        end = elf.index(b"\0", stro + name)
        out[elf[stro + name:end].decode()] = (off, size, typ)
    return out


def code_objects(lib_path: str):
    """Every gfx950 code object in the library's fat binary (one per translation unit with device code)."""
    elf = open(lib_path, "rb").read()
    off, size, _ = _sections(elf)[".hip_fatbin"]
    fb = elf[off:off + size]
    pos = fb.find(BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fb, pos + len(BUNDLE_MAGIC))
        p = pos + len(BUNDLE_MAGIC) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24:p + 24 + tlen]
            p += 24 + tlen
            if triple == TARGET and esize:
                yield fb[pos + eoff:pos + eoff + esize]
        pos = fb.find(BUNDLE_MAGIC, pos + 1)


def kernel_metadata(co: bytes):
    """The `amdhsa.kernels` list of one code object."""
    for _name, (off, size, typ) in _sections(co).items():
        if typ != 7:                                    # SHT_NOTE
            continue
        p = off
        while p < off + size:
            namesz, descsz, ntype = struct.unpack_from("<III", co, p)
            name = co[p + 12:p + 12 + namesz].rstrip(b"\0")
            d0 = p + 12 + ((namesz + 3) & ~3)
            if ntype == NT_AMDGPU_METADATA and name == b"AMDGPU":
                return msgpack.unpackb(co[d0:d0 + descsz], raw=False, strict_map_key=False)["amdhsa.kernels"]
            p = d0 + ((descsz + 3) & ~3)
    return []


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        out = r.stdout.split("\n")[:len(names)]
        return [o.replace("sda::(anonymous namespace)::", "").split("(")[0].replace("void ", "") for o in out]
    except (OSError, subprocess.CalledProcessError):
        return list(names)


def kernels(lib_path: str):
    """One dict per kernel: name (mangled), pretty, vgpr, agpr, sgpr, scratch, vgpr_spill, sgpr_spill, lds."""
    rows = []
    for co in code_objects(lib_path):
        for k in kernel_metadata(co):
            rows.append(dict(name=k[".name"], vgpr=k.get(".vgpr_count", 0), agpr=k.get(".agpr_count", 0),
                             sgpr=k.get(".sgpr_count", 0), scratch=k.get(".private_segment_fixed_size", 0),
                             vgpr_spill=k.get(".vgpr_spill_count", 0), sgpr_spill=k.get(".sgpr_spill_count", 0),
                             lds=k.get(".group_segment_fixed_size", 0)))
    for r, pretty in zip(rows, demangle([r["name"] for r in rows])):
        r["pretty"] = pretty
    return rows


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "sda_amd", "libsda_engine.so")
    rows = kernels(lib)
    print(f"{len(rows)} kernels in {lib}")
    print(f"{'kernel':70s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'scratch':>8s} {'vspill':>7s} {'sspill':>7s}")
    for r in sorted(rows, key=lambda r: r["pretty"]):
        if "--all" in sys.argv or r["scratch"] or r["vgpr_spill"] or r["agpr"]:
            print(f"{r['pretty'][:70]:70s} {r['vgpr']:5d} {r['agpr']:5d} {r['sgpr']:5d} {r['scratch']:8d} "
                  f"{r['vgpr_spill']:7d} {r['sgpr_spill']:7d}")


if __name__ == "__main__":
    main()
