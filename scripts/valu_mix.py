#!/usr/bin/env python3
"""VALU issue roofline of the integer kernels: their instruction mix priced at the measured issue
rates of tools/ubench_int, combined with the PMC instruction counts of one round.

    python scripts/valu_mix.py <ubench_int.txt> <kernel_report.json> [more reports] > profiles/valu_roofline.json

1. The device code of each kernel is compiled with the Makefile's flags (--cuda-device-only) and
   disassembled; every VALU instruction is priced by its class's measured rate (T lane-instr/s):
   the mix ceiling = n_valu / sum(n_class / rate_class) is the lane-op rate the kernel would reach if
   it issued VALU back to back with nothing else in its way (its instruction-mix roofline).
2. kernel_report.json (scripts/kernel_report.py) gives SQ_INSTS_VALU per launch at the bench
   configuration (PMC; with several reports, a later one overrides an earlier one's kernels);
   bench.py divides insts x 64 by the live kernel time and by the ceiling.
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output"]

# (bench key, source, -D define or None, mangled-name fragment)
KERNELS = [
    ("gen_exact", "packed_gen.hip", "SDA_GEN_PART=27 -DSDA_GEN_L=16", "packed_gen_kernelILi16ELi27ELb1ELb0ELb1ELb1E"),
    ("gen_canonical", "packed_gen.hip", "SDA_GEN_PART=27 -DSDA_GEN_L=16", "packed_gen_kernelILi16ELi27ELb1ELb1ELb0ELb0E"),
    ("reveal_exact", "packed_reveal.hip", "SDA_REVEAL_PART=16", "packed_reveal_exact_kernelILi16ELb1ELi8ELb1ELb1E"),
    ("reveal_canonical", "packed_reveal.hip", "SDA_REVEAL_PART=16", "packed_reveal_canon_kernelILi16ELb1E"),
    ("chacha_combine", "chacha.hip", None, "chacha_combine_sk_kernelILb1ELb1E"),
]
# the PMC report's short names for the same kernels
PMC_NAMES = {
    "gen_exact": "packed_gen_kernel<16, 27, true, false, true, true>",
    "gen_canonical": "packed_gen_kernel<16, 27, true, true, false, false>",
    "reveal_exact": "packed_reveal_exact_kernel<16, true, 8, true, true>",
    "reveal_canonical": "packed_reveal_canon_kernel<16, true>",
    "chacha_combine": "chacha_combine_sk_kernel<true, true>",
}

# ChaCha20 blocks of the counted launch (bench.py's chacha leg: 256 seeds x 1M-dim, 8 draws per block)
PMC_BLOCKS = {"chacha_combine": 256 * 1_000_000 // 8}

# instruction class -> the ubench_int row(s) that measured it
CLASSES = [
    (r"^v_(add|sub|subrev)_u32$", ["v_add_u32", "v_sub_u32"]),
    (r"^v_(xor|and|or|not)_b32$", ["v_xor_b32", "v_and_b32"]),
    (r"^v_(ashrrev_i32|lshrrev_b32|lshlrev_b32)$", ["v_ashrrev_i32", "v_lshrrev_b32"]),
    (r"^v_bitop3_b32$", ["v_bitop3_b32"]),
    (r"^v_mov_b32$", ["v_add_u32"]),
    (r"^v_(min|max)_(u32|i32)$", ["v_min_u32", "v_max_u32", "v_min_i32"]),
    (r"^v_(min3|max3|med3)_(u32|i32)$", ["v_min3_u32", "v_med3_u32"]),
    (r"^v_add3_u32$", ["v_add3_u32"]),
    (r"^v_(add|sub)_i32$", ["v_sub_i32 clamp"]),
    (r"^v_(alignbit|alignbyte)_b32$", ["v_alignbit_b32", "v_alignbit_b32 (16)"]),
    (r"^v_perm_b32$", ["v_perm_b32"]),
    (r"^v_xad_u32$", ["v_xad_u32"]),
    (r"^v_bfi_b32$", ["v_bfi_b32"]),
    (r"^v_(lshl_or|and_or|or3|lshl_add)_(b32|u32)$", ["v_lshl_or_b32"]),
    (r"^v_mul_lo_u32$", ["v_mul_lo_u32"]),
    (r"^v_mul_hi_u32$", ["v_mul_hi_u32"]),
    (r"^v_mul_u32_u24$", ["v_mul_u32_u24"]),
    (r"^v_mad_(u64_u32|i64_i32)$", ["v_mad_u64_u32", "v_mad_i64_i32"]),
    (r"^v_lshl_add_u64$", ["v_lshl_add_u64"]),
    (r"^v_(add_co|addc_co|sub_co|subb_co|subrev_co)_u32$", ["v_add_co + v_addc_co"]),
    (r"^v_cndmask_b32$", ["v_cmp + v_cndmask"]),
    (r"^v_cmp", ["v_cmp + v_cndmask"]),
    (r"^v_pk_add_u16$", ["v_pk_add_u16 (swap)"]),
]


def rates(path):
    r = {}
    for line in open(path):
        m = re.match(r"^(.*?)\s+([0-9.]+) T lane-instr/s", line)
        if m:
            r.setdefault(m.group(1).strip(), float(m.group(2)))
    return r


def rate_of(op, R):
    base = re.sub(r"_e(32|64)$", "", op)
    for pat, rows in CLASSES:
        if re.match(pat, base):
            vals = [R[x] for x in rows if x in R]
            if vals:
                return sum(vals) / len(vals), base
    return sum(R[x] for x in ("v_min_u32", "v_mul_lo_u32")) / 2, base + " (unclassified: 0.6x rate)"


def disasm(src, define, frag):
    with tempfile.TemporaryDirectory() as d:
        obj = os.path.join(d, "k.o")
        cmd = [HIPCC] + FLAGS + ([f"-D{x}" for x in define.split(" -D")] if define else []) + ["-c", os.path.join(ROOT, "sda_amd", "csrc", src),
                                                                       "-o", obj]
        subprocess.run(cmd, check=True, capture_output=True)
        txt = subprocess.run([OBJDUMP, "-d", obj], check=True, capture_output=True, text=True).stdout
    for f in re.split(r"\n(?=[0-9a-f]+ <[^>]+>:\n)", txt):
        m = re.match(r"[0-9a-f]+ <([^>]+)>:", f)
        if m and frag in m.group(1):
            ops = collections.Counter()
            for line in f.split("\n")[1:]:
                mm = re.match(r"\s+(v_[a-z_0-9]+)\s", line)
                if mm:
                    ops[mm.group(1)] += 1
            return m.group(1), ops
    raise SystemExit(f"kernel {frag} not found in {src}")


# ChaCha's quarter-round chains (4 per wave, add -> xor -> v_alignbit, the combine's 6 waves per SIMD) timed in
# isolation by tools/ubench_bank: the rate the combine's own instruction stream can issue at, which the
# independent per-class prices above overestimate (the QR pattern runs at 38.7 T, its mix prices at 52 T).
PATTERN = {"chacha_combine": ("profiles/r04bank/ubench_bank.txt", "QR chains, different-bank pairs    6 waves/SIMD")}


def pattern_ceiling(path, label):
    try:
        for line in open(os.path.join(ROOT, path)):
            if line.startswith(label):
                return float(line.split()[-3])
    except OSError:
        return None
    return None


def main():
    R = rates(sys.argv[1])
    report, sources = {}, {}
    for path in sys.argv[2:]:
        for k, v in json.load(open(path)).items():
            report[k] = v
            sources[k] = os.path.relpath(path, ROOT)
    out = {"method": __doc__.strip().split("\n\n")[0], "ubench": os.path.relpath(sys.argv[1], ROOT), "kernels": {}}
    for key, src, define, frag in KERNELS:
        name, ops = disasm(src, define, frag)
        n = sum(ops.values())
        t = 0.0
        classes = collections.Counter()
        for op, c in ops.items():
            r, cls = rate_of(op, R)
            t += c / r
            classes[cls] += c
        rec = {"symbol": name, "static_valu": n, "mix_ceiling_T_lane_ops": round(n / t, 3),
               "classes": dict(classes.most_common())}
        hit = next((k for k in report if k.endswith(PMC_NAMES[key])), None)
        c = report[hit].get("counters_max_dispatch", {}) if hit else {}
        if "SQ_INSTS_VALU" in c:
            rec["pmc_valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
            rec["pmc_waves"] = c.get("SQ_WAVES")
            rec["pmc_source"] = sources[hit]
            if key in PMC_BLOCKS:      # work units of the counted launch, to scale to other launch sizes
                rec["pmc_blocks"] = PMC_BLOCKS[key]
        if key in PATTERN:        # the kernel's dependent instruction pattern, measured on its own
            path, label = PATTERN[key]
            pc = pattern_ceiling(path, label)
            if pc:
                rec["pattern_ceiling_T_lane_ops"] = pc
                rec["pattern_source"] = f"{path}: {label}"
        out["kernels"][key] = rec
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
