"""sda_hbm_alloc / sda_hbm_free (include/sda_engine.h) and Engine.hbm_empty on the GPU: the buffer is usable
by torch and by the engine's kernels, share-gen into it is bit-identical to share-gen into a torch buffer, it
returns to the pool with its tensor and is handed out again, the pool is bounded and trimmed (physical chunks
released, the virtual range retired), and the error behaviour is the header's."""
import ctypes as C
import os

import pytest

from sda_amd import SdaError, schemes as S
from sda_amd import engine as E

pytestmark = pytest.mark.gpu


def test_hbm_alloc_free_errors(engine):
    lib = E.load_library()
    p = C.c_void_p()
    assert lib.sda_hbm_alloc(engine.device, 0, C.byref(p)) == E.ERR_INVALID_ARGUMENT
    assert lib.sda_hbm_alloc(engine.device, 4096, None) == E.ERR_INVALID_ARGUMENT
    assert lib.sda_hbm_free(None) == E.OK
    assert lib.sda_hbm_alloc(engine.device, 5 << 20, C.byref(p)) == E.OK and p.value
    assert lib.sda_hbm_free(C.c_void_p(p.value + 4096)) == E.ERR_INVALID_ARGUMENT   # not a returned pointer
    assert lib.sda_hbm_free(p) == E.OK
    assert lib.sda_hbm_free(p) == E.ERR_INVALID_ARGUMENT                          # already released
    with pytest.raises(SdaError):
        E._check(lib.sda_hbm_alloc(1 << 20, 4096, C.byref(p)))                    # no such device


def test_hbm_tensor_torch_and_engine(engine):
    import torch
    st = torch.cuda.current_stream().cuda_stream
    rows, cols = 300, 1 << 20                                  # 2.4 GB: many 64 MiB chunks
    a = engine.hbm_empty((rows, cols))
    assert a.is_cuda and a.dtype == torch.int64 and tuple(a.shape) == (rows, cols) and a.is_contiguous()
    a.fill_(3)
    assert int(a.sum()) == 3 * a.numel()
    engine.synth_fill_dev(a.data_ptr(), rows, cols, 11, -5, 1000, st)
    b = torch.empty_like(a)
    engine.synth_fill_dev(b.data_ptr(), rows, cols, 11, -5, 1000, st)
    assert torch.equal(a, b)
    u8 = engine.hbm_empty((12345,), torch.uint8)
    assert u8.dtype == torch.uint8 and u8.numel() == 12345
    u8.zero_()
    assert int(u8.sum()) == 0
    ptr = a.data_ptr()
    del a                                                      # back to the pool with its tensor, still mapped
    a2 = engine.hbm_empty((rows, cols))
    if os.environ.get("SDA_HBM_POOL_MB", "") != "0":          # (the r04y repro runs with the pool disabled)
        assert a2.data_ptr() == ptr                            # the pooled buffer is handed out again
    a2.fill_(-1)
    assert int(a2.min()) == -1 and int(a2.max()) == -1


def test_packed_generate_into_hbm_matches_torch_buffer(engine):
    import torch
    st = torch.cuda.current_stream().cuda_stream
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    V, Dm = 40, 1_000_000
    B = Dm // k
    sec = engine.hbm_empty((V, Dm))
    engine.synth_fill_dev(sec.data_ptr(), V, Dm, 21, 0, p, st)
    drw = engine.hbm_empty((V, B, t))
    engine.synth_fill_dev(drw.data_ptr(), V * B, t, 22, 0, p - 1, st)
    for mode in (E.REVEAL_EXACT, E.REVEAL_CANONICAL):
        sh_h = engine.hbm_empty((V, n, B))
        sh_t = torch.empty((V, n, B), dtype=torch.int64, device=sec.device)
        for sh in (sh_h, sh_t):
            engine.packed_generate_mode_dev(sch, sec.data_ptr(), Dm, V, drw.data_ptr(), sh.data_ptr(), mode, st)
        torch.cuda.synchronize()
        if not torch.equal(sh_h, sh_t):
            diff = (sh_h != sh_t).nonzero()
            raise AssertionError(
                f"mode {mode}: {diff.shape[0]} of {sh_h.numel()} differ, first at {diff[0].tolist()}; zeros: hbm "
                f"{int((sh_h == 0).sum())}, torch {int((sh_t == 0).sum())}; ptrs {hex(sh_h.data_ptr())} "
                f"{hex(sh_t.data_ptr())} {hex(sec.data_ptr())} {hex(drw.data_ptr())}")
        if mode == E.REVEAL_CANONICAL:
            assert int(sh_h.min()) >= 0 and int(sh_h.max()) < p


def test_hbm_trim_realloc_sequence_matches_torch(engine, monkeypatch):
    """The sequence that corrupted data in round 4 (profiles/r04y): a buffer is freed and unmapped, torch takes
    fresh memory, new buffers are allocated and share-gen writes one of them -- now with every free trimmed
    (SDA_HBM_POOL_MB=0).  Share-gen into the new buffer equals share-gen into a torch buffer, repeated reads
    agree, and the torch block allocated in between is untouched (HBM backing)."""
    import torch
    monkeypatch.setenv("SDA_HBM_POOL_MB", "0")
    st = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda", engine.device)
    sch = S.CONFIG_PACKED
    p, k, t, n = sch.prime_modulus, sch.secret_count, sch.privacy_threshold(), sch.share_count
    V, Dm = 40, 1_000_000
    B = Dm // k
    _, _, retired0 = engine.hbm_stats()
    for r in range(3):
        a = engine.hbm_empty((300, 1 << 20))                   # 2.4 GB, as the earlier test's buffer
        engine.synth_fill_dev(a.data_ptr(), 300, 1 << 20, 40 + r, 1, 1 << 40, st)
        torch.cuda.synchronize()
        a_lo, a_hi = a.data_ptr(), a.data_ptr() + a.numel() * 8
        del a
        engine.hbm_trim(0)
        assert engine.hbm_stats()[1] == 0
        torch.cuda.empty_cache()
        blk = torch.full((300, 1 << 20), 0x5A5A5A5A5A5A5A5A, dtype=torch.int64, device=dev)
        sec = engine.hbm_empty((V, Dm))
        engine.synth_fill_dev(sec.data_ptr(), V, Dm, 21 + r, 0, p, st)
        drw = engine.hbm_empty((V, B, t))
        engine.synth_fill_dev(drw.data_ptr(), V * B, t, 22 + r, 0, p - 1, st)
        sh_h = engine.hbm_empty((V, n, B))
        for buf in (sec, drw, sh_h):                           # a retired range is never mapped again
            assert buf.data_ptr() + buf.numel() * 8 <= a_lo or buf.data_ptr() >= a_hi
        sh_t = torch.empty((V, n, B), dtype=torch.int64, device=dev)
        for sh in (sh_h, sh_t):
            engine.packed_generate_mode_dev(sch, sec.data_ptr(), Dm, V, drw.data_ptr(), sh.data_ptr(),
                                            E.REVEAL_EXACT, st)
        torch.cuda.synchronize()
        for _ in range(2):
            assert torch.equal(sh_h, sh_t)
            assert int((sh_h == 0).sum()) == int((sh_t == 0).sum())
        assert int((blk != 0x5A5A5A5A5A5A5A5A).sum()) == 0
        del sec, drw, sh_h, sh_t, blk
    engine.hbm_trim(0)
    live, pooled, retired = engine.hbm_stats()
    assert pooled == 0 and retired > retired0


def test_hbm_pool_is_bounded(engine, monkeypatch):
    """Freed buffers only pool (no wait, no trim).  A request of the same size class takes a pooled buffer back
    without trimming anything; one that needs a new buffer first trims the pool (oldest first) to
    SDA_HBM_POOL_MB; sda_hbm_trim empties the pool."""
    engine.hbm_trim(0)
    monkeypatch.setenv("SDA_HBM_POOL_MB", "256")
    bufs = [engine.hbm_empty((16 << 20,)) for _ in range(4)]    # 4 x 128 MiB (2 chunks, class 2)
    ptrs = [b.data_ptr() for b in bufs]
    for i in range(4):                                         # freed in order: bufs[0] is the oldest
        bufs[i] = None
    live, pooled, retired0 = engine.hbm_stats()
    assert pooled >= 4 * (128 << 20)                           # free only pools (no wait, no trim)
    x = engine.hbm_empty((16 << 20,))                          # same class: a pooled buffer, nothing trimmed
    assert x.data_ptr() in ptrs
    assert engine.hbm_stats()[1] == 3 * (128 << 20) and engine.hbm_stats()[2] == retired0
    y = engine.hbm_empty((48 << 20,))                          # 384 MiB, class 6: new, after a trim to 256 MiB
    live, pooled, retired = engine.hbm_stats()
    assert pooled <= 256 << 20 and retired == retired0 + (128 << 20)
    assert y.data_ptr() not in ptrs
    x.fill_(7)
    y.fill_(-3)
    assert int(x.sum()) == 7 * x.numel() and int(y.sum()) == -3 * y.numel()
    del x, y
    engine.hbm_trim(0)
    assert engine.hbm_stats()[1] == 0
    with pytest.raises(SdaError):
        E._check(engine.lib.sda_hbm_trim(-1, 0))


def test_hbm_size_class_grows_a_pooled_buffer(engine):
    """A pooled buffer serves a larger request of its size class by mapping fresh chunks at its reserved
    range's never-mapped tail: same pointer, more bytes live, the new tail usable by torch and the engine."""
    import torch
    engine.hbm_trim(0)
    chunk = 8 << 20                                            # int64 elements per 64 MiB chunk
    live0 = engine.hbm_stats()[0]
    a = engine.hbm_empty((9 * chunk,))                         # 9 chunks: class 10 (9 mapped)
    pa = a.data_ptr()
    a.fill_(1)
    del a
    b = engine.hbm_empty((9 * chunk - 1000,))                  # same class, fewer bytes: handed back as is
    assert b.data_ptr() == pa and engine.hbm_stats()[0] - live0 == 9 * (64 << 20)
    del b
    c = engine.hbm_empty((11 * chunk,))                        # class 12: a new buffer
    assert c.data_ptr() != pa
    del c
    d = engine.hbm_empty((10 * chunk,))                        # 10 chunks, class 10: the pooled one, grown
    assert d.data_ptr() == pa
    live, _, _ = engine.hbm_stats()
    assert live - live0 == 10 * (64 << 20)
    st = torch.cuda.current_stream().cuda_stream
    engine.synth_fill_dev(d.data_ptr(), 1, d.numel(), 5, -9, 9, st)
    ref = torch.empty_like(d)
    engine.synth_fill_dev(ref.data_ptr(), 1, d.numel(), 5, -9, 9, st)
    assert torch.equal(d, ref)
    d.fill_(4)
    assert int(d[-chunk:].sum()) == 4 * chunk                  # the grown tail
    del d
    engine.hbm_trim(0)
