"""In-process A/B of a knob of the clerk's decode -> combine (default SDA_SLOT_CPL, read per call): 1000 x 1M signed
field-share payloads encoded once, the variants interleaved call block by call block, HIP events around 5 calls.
    python scripts/codec_inproc.py [rounds] [variants ...]        (SDA_INPROC_KNOB names the variable)
SDA_INPROC_SHAPE=encode times the encode of the same matrix instead (varint_encode_dev, host wait included);
SDA_INPROC_SHAPE=decode the decode of the payloads back into a 1000 x 1M i64 matrix (varint_decode_dev).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sda_amd import Engine  # noqa: E402

M = 2147482801
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
variants = sys.argv[2:] or ["4", "2"]
knob = os.environ.get("SDA_INPROC_KNOB", "SDA_SLOT_CPL")
torch.cuda.init()
eng = Engine(0)
N, D = 1000, 1_000_000
st = torch.cuda.current_stream().cuda_stream
x = torch.empty((N, D), dtype=torch.int64, device="cuda")
eng.synth_fill_dev(x.data_ptr(), N, D, 0x5DA + 6, -(M - 1), M, st)
cap = N * D * 6 + 32
buf = torch.zeros(cap, dtype=torch.uint8, device="cuda")
ecap = N * D * 10              # the encode shape: room for any i64 (the one-pass encode's condition)
rb = eng.varint_encode_dev(x.data_ptr(), N, D, D, buf.data_ptr(), cap, st)
off = np.concatenate([[0], np.cumsum(rb)]).astype(np.uint64)
enc = os.environ.get("SDA_INPROC_SHAPE") == "encode"
dec = os.environ.get("SDA_INPROC_SHAPE") == "decode"
if dec:
    del x
    mat = torch.empty((N, D), dtype=torch.int64, device="cuda")
    outs = {v: torch.empty(D, dtype=torch.int64, device="cuda") for v in variants}
elif enc:
    del buf
    outs = {v: torch.zeros(ecap, dtype=torch.uint8, device="cuda") for v in variants}
else:
    del x
    outs = {v: torch.empty(D, dtype=torch.int64, device="cuda") for v in variants}


def call(v):
    if dec:
        eng.varint_decode_dev(buf.data_ptr(), off, mat.data_ptr(), D, st)
        outs[v].copy_(mat[N - 1])
    elif enc:
        eng.varint_encode_dev(x.data_ptr(), N, D, D, outs[v].data_ptr(), ecap, st)
    else:
        eng.clerk_decode_combine_dev(M, buf.data_ptr(), off, outs[v].data_ptr(), D, st)



res = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        os.environ[knob] = v
        call(v)                                                                           # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            call(v)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        res[v].append(ms)
        print(f"round {r} {knob}={v} {ms:.4f} ms", flush=True)
for v in variants:
    s = sorted(res[v])
    print(f"{knob}={v}: median {s[len(s) // 2]:.4f} ms, min {s[0]:.4f}, max {s[-1]:.4f}")
print("bit-identical:", all(torch.equal(outs[v], outs[variants[0]]) for v in variants))
