"""Engine.hbm_empty on the GPU: torch ops over an sda_hbm_alloc buffer, an engine kernel writing into one,
and the buffer released with its tensor.  Prints one line per check; exits non-zero on a mismatch."""
import sys

import torch

sys.path.insert(0, ".")
from sda_amd import Engine  # noqa: E402


def main():
    eng = Engine(0)
    st = torch.cuda.current_stream().cuda_stream
    a = eng.hbm_empty((1000, 1 << 20))                      # 8 GB: many chunks
    print("tensor", a.shape, a.dtype, a.device, hex(a.data_ptr()), flush=True)
    a.fill_(3)
    assert int(a.sum()) == 3 * a.numel(), "fill/sum over the hbm tensor"
    eng.synth_fill_dev(a.data_ptr(), 1000, 1 << 20, 7, 0, 1000, st)
    b = torch.empty_like(a)
    eng.synth_fill_dev(b.data_ptr(), 1000, 1 << 20, 7, 0, 1000, st)
    assert torch.equal(a, b), "engine kernel into hbm vs torch buffer"
    print("fill/sum and engine-kernel checks OK", flush=True)
    free0 = torch.cuda.mem_get_info()[0]
    del a
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    print(f"released {(free1 - free0) / 1e9:.2f} GB", flush=True)
    assert free1 - free0 > 7e9, "buffer not released with its tensor"
    print("hbm_check OK")


if __name__ == "__main__":
    main()
