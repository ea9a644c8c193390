"""sda_hbm_alloc buffers across alloc / free cycles: each round allocates a buffer, fills it with an engine
kernel, and checks it three times (at once, after streaming 16 GB through the caches, after a 0.5 s wait)
against a torch buffer filled the same way.  Prints one line per round: the buffer's address, whether that
address was handed out before, and the mismatch / zero counts of each check."""
import sys
import time

import torch

sys.path.insert(0, ".")
from sda_amd import Engine  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    eng = Engine(0)
    st = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda", 0)
    flush = torch.empty(2 * 1024**3, dtype=torch.int64, device=dev)      # 16 GB: evicts L2 and the MALL
    # optional: hold all but `leave` GB of the device in a torch block first (memory pressure)
    leave = float(sys.argv[2]) if len(sys.argv) > 2 else -1
    hold = None
    if leave >= 0:
        free, total = torch.cuda.mem_get_info()
        hold = torch.empty(int((free - leave * 1e9) // 8), dtype=torch.int64, device=dev)
    print(f"free {torch.cuda.mem_get_info()[0] / 1e9:.1f} GB of {torch.cuda.mem_get_info()[1] / 1e9:.1f}", flush=True)
    seen = set()
    bad = 0
    for r in range(rounds):
        rows = (40, 130, 40, 130, 300, 40, 130, 40)[r % 8]
        cols = 1 << 20
        x = eng.hbm_empty((rows, cols))
        ref = torch.empty((rows, cols), dtype=torch.int64, device=dev)
        reused = x.data_ptr() in seen
        seen.add(x.data_ptr())
        for t in (x, ref):
            eng.synth_fill_dev(t.data_ptr(), rows, cols, 100 + r, 1, 1 << 40, st)   # never 0
        torch.cuda.synchronize()
        res = []
        for step in ("now", "flushed", "waited"):
            if step == "flushed":
                flush.add_(1)
                torch.cuda.synchronize()
            if step == "waited":
                time.sleep(0.5)
            res.append((step, int((x != ref).sum()), int((x == 0).sum())))
        ok = all(d == 0 for _, d, _ in res)
        bad += not ok
        print(f"round {r}: {rows} x {cols} at {hex(x.data_ptr())} reused={reused} "
              + " ".join(f"{s}: diff {d} zeros {z}" for s, d, z in res) + ("" if ok else "  MISMATCH"), flush=True)
        del x, ref
    print("hbm_stress", "OK" if not bad else f"{bad} BAD ROUNDS")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
