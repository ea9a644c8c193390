"""In-process A/B of a packed-reveal knob read per launch (SDA_INPROC_KNOB names it): the bench's shamir leg shape
(PackedShamir k=8 n=26 t=7, 1000 x 1M, 15 clerks), the variants interleaved launch block by launch block, HIP events
on the launch stream, so buffer placement and box state are shared by every variant.  Checks every variant reveals
the secrets.
    python scripts/reveal_inproc.py [rounds] [variants ...]
SDA_INPROC_MODE=exact times the exact reveal instead of the canonical one.  Round 6 used it with the flush-store
knob SDA_REVEAL_MEM (bit 0 nontemporal share loads, bit 1 16-byte stores, bit 2 nontemporal stores; profiles/r06ab,
r06ac); variant 6 became the code and the knob was removed.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd import Engine, schemes as S  # noqa: E402
from sda_amd import engine as E  # noqa: E402

knob = os.environ.get("SDA_INPROC_KNOB", "SDA_REVEAL_MEM")
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
variants = sys.argv[2:] or ["0", "1"]
mode = E.REVEAL_EXACT if os.environ.get("SDA_INPROC_MODE") == "exact" else E.REVEAL_CANONICAL
torch.cuda.init()
eng = Engine(0)
st = torch.cuda.current_stream().cuda_stream
sch = S.CONFIG_PACKED
p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
V, D = 1000, 1_000_000
B = D // k
sec = torch.empty((V, D), dtype=torch.int64, device="cuda")
eng.synth_fill_dev(sec.data_ptr(), V, D, 0x5DB2, 0, p, st)
drw = torch.empty((V, B, t), dtype=torch.int64, device="cuda")
eng.synth_fill_dev(drw.data_ptr(), V * B, t, 0x5DB3, 0, p - 1, st)
sh = torch.empty((V, n, B), dtype=torch.int64, device="cuda")
eng.packed_generate_dev(sch, sec.data_ptr(), D, V, drw.data_ptr(), sh.data_ptr(), st)
del drw
idx = list(range(n - (t + k), n))
sub = sh[:, idx, :].contiguous()
del sh
rev = torch.empty((V, D), dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
nbytes = 8.0 * V * (len(idx) * B + D)


def launch():
    eng.packed_reconstruct_dev(sch, D, idx, V, sub.data_ptr(), rev.data_ptr(), mode, st)


res = {v: [] for v in variants}
ok = {}
for r in range(rounds):
    for v in variants:
        os.environ[knob] = v
        launch()                                                                    # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            launch()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[v].append(ms)
        if r == 0:
            ok[v] = torch.equal(torch.remainder(rev, p), sec)
        print(f"round {r} {knob}={v} {ms:.4f} ms  {nbytes / ms / 1e9:.3f} TB/s", flush=True)
for v in variants:
    s = sorted(res[v])
    print(f"{knob}={v}: median {s[len(s) // 2]:.4f} ms, min {s[0]:.4f}, max {s[-1]:.4f}, "
          f"reveals the secrets: {ok[v]}")
