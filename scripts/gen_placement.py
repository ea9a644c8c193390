"""Does share-gen's time depend on where its buffers sit?  One process, bench.py's 1000 x 1M packed-Shamir
workload: canonical and exact share-gen into each of several freshly allocated share buffers (and from a
second secrets/draws pair), mean of 8 launches each, two rounds.  Prints one line per (buffers, mode).

    python scripts/gen_placement.py [n_share_buffers] [torch|hbm]

hbm: every buffer from Engine.hbm_empty (sda_hbm_alloc, fixed-size physical chunks) instead of torch.empty.
"""
import sys

import torch

sys.path.insert(0, ".")
from sda_amd import Engine, schemes as S  # noqa: E402
from sda_amd import engine as E  # noqa: E402


def main():
    nbuf = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    eng = Engine(0)
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 2 and sys.argv[2] == "hbm":
        empty = lambda shape: eng.hbm_empty(shape, torch.int64)  # noqa: E731
    else:
        empty = lambda shape: torch.empty(shape, dtype=torch.int64, device=dev)  # noqa: E731
    st = torch.cuda.current_stream().cuda_stream
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    V, Dm = 1000, 1_000_000
    B = Dm // k

    def inputs(seed):
        sec = empty((V, Dm))
        eng.synth_fill_dev(sec.data_ptr(), V, Dm, seed, 0, p, st)
        drw = empty((V, B, t))
        eng.synth_fill_dev(drw.data_ptr(), V * B, t, seed + 20, 0, p - 1, st)
        return sec, drw

    pairs = [inputs(0x5DA + 2)]
    shs = [empty((V, n, B)) for _ in range(nbuf)]
    pairs.append(inputs(0x5DA + 3))
    torch.cuda.synchronize()

    def timed(sec, drw, sh, mode, reps=8):
        f = lambda: eng.packed_generate_mode_dev(sch, sec.data_ptr(), Dm, V, drw.data_ptr(), sh.data_ptr(), mode, st)  # noqa
        f()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record()
            f()
            b.record()
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in ev) / reps

    print("secrets/draws pairs:", [(hex(s.data_ptr()), hex(d.data_ptr())) for s, d in pairs], flush=True)
    for rnd in range(2):
        for pi, (sec, drw) in enumerate(pairs):
            for bi, sh in enumerate(shs):
                if pi == 1 and bi > 0:
                    continue
                c = timed(sec, drw, sh, E.REVEAL_CANONICAL)
                x = timed(sec, drw, sh, E.REVEAL_EXACT)
                print(f"round {rnd} inputs {pi} shares {bi} ({hex(sh.data_ptr())}): canonical {c:.3f} ms  "
                      f"exact {x:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
