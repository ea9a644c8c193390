import os, sys, torch
sys.path.insert(0, os.getcwd())
from sda_amd import Engine
M = 2147482801
torch.cuda.init(); eng = Engine(0)
N, S = 10_000, 1_048_576
x = torch.empty((N, S), dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
eng.synth_fill_dev(x.data_ptr(), N, S, 0x5DB, 0, M, st)
out = torch.empty(S, dtype=torch.int64, device="cuda")
for r in range(4):
    for D in (1_000_000, 1_048_576, 983_040, 1_015_808):
        eng.combine_dev(M, x.data_ptr(), N, D, S, out.data_ptr(), st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(8):
            eng.combine_dev(M, x.data_ptr(), N, D, S, out.data_ptr(), st)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 8
        waves = (D // 2 + 255) // 256 * 4
        print(f"round {r} D={D} waves={waves} {ms:.4f} ms {8.0*N*D/ms/1e9:.3f} TB/s", flush=True)
