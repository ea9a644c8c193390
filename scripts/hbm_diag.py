"""The A/B behind DESIGN.md §2's HBM-backing note (the r04y corruption).

Each round: an sda_hbm_alloc buffer A is filled, freed and trimmed (unmapped, released; its virtual range
retired, or returned to the runtime with SDA_HBM_VA_FREE=1); torch then allocates a fresh block T (which
may take A's physical pages) and fills it with a pattern; a new sda_hbm_alloc buffer X (whose range may be
A's again) and a torch buffer `ref` are filled by the same engine kernel.  Printed per round: whether X's
range overlaps a range trimmed earlier, X vs ref mismatches over three reads, X's zero count over two reads,
and how many words of T no longer hold the pattern.  The first line names the HIP runtime the process
mapped (torch's bundled one or /opt/rocm's).  Exit status 1 if any round mismatched.

    SDA_HBM_VA_FREE=0|1 python3 scripts/hbm_diag.py [rounds]
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from sda_amd import Engine  # noqa: E402

PATTERN = 0x5A5A5A5A5A5A5A5A


def mapped_runtime():
    seen = []
    with open("/proc/self/maps") as f:
        for line in f:
            path = line.split()[-1]
            if ("libamdhip64" in path or "libhsa-runtime64" in path) and path not in seen:
                seen.append(path)
    return seen


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    os.environ["SDA_HBM_POOL_MB"] = "0"            # every freed buffer is trimmed at the next allocation
    eng = Engine(0)
    st = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda", 0)
    cols = 1 << 20
    print(f"SDA_HBM_VA_FREE={os.environ.get('SDA_HBM_VA_FREE', '0')} torch.version.hip={torch.version.hip} "
          f"runtime={mapped_runtime()}", flush=True)
    trimmed = []
    bad = 0
    for r in range(rounds):
        rows_a = (300, 130, 40)[r % 3]
        a = eng.hbm_empty((rows_a, cols))
        eng.synth_fill_dev(a.data_ptr(), rows_a, cols, 500 + r, 1, 1 << 40, st)
        torch.cuda.synchronize()
        trimmed.append((a.data_ptr(), a.data_ptr() + a.numel() * 8))
        del a
        eng.hbm_trim(0)
        torch.cuda.empty_cache()
        t = torch.empty((300, cols), dtype=torch.int64, device=dev)
        t.fill_(PATTERN)
        x = eng.hbm_empty((130, cols))
        lo, hi = x.data_ptr(), x.data_ptr() + x.numel() * 8
        reused = any(a0 < hi and lo < a1 for a0, a1 in trimmed)
        ref = torch.empty((130, cols), dtype=torch.int64, device=dev)
        for buf in (x, ref):
            eng.synth_fill_dev(buf.data_ptr(), 130, cols, 600 + r, 1, 1 << 40, st)   # never 0
        torch.cuda.synchronize()
        diffs = [int((x != ref).sum()) for _ in range(3)]
        zeros = [int((x == 0).sum()) for _ in range(2)]
        t_changed = int((t != PATTERN).sum())
        ok = not any(diffs) and not any(zeros) and t_changed == 0
        bad += not ok
        live, pooled, retired = eng.hbm_stats()
        print(f"round {r}: A {rows_a}x{cols} X at {hex(lo)} overlaps-trimmed={reused} diffs={diffs} zeros={zeros} "
              f"torch-block-changed={t_changed} stats(live={live >> 20}M pooled={pooled >> 20}M "
              f"retired={retired >> 20}M)" + ("" if ok else "  MISMATCH"), flush=True)
        del x, ref, t
    print("hbm_diag", "OK" if not bad else f"{bad} BAD ROUNDS", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
