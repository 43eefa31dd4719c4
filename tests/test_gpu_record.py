"""Frame records (orbgpu_frame_record_pack / _unpack, the unit bench.py broadcasts from rank 0 to the other ranks
at set-up): a record unpacked into a second context reproduces the frame exactly, and a record
that does not fit the receiving context's plan (frame_cap, undistortion) or carries a count above frame_cap is
refused with ORBGPU_ERR_ARG.  The header is checked on the device, so unpack itself never blocks the
host: a refused record leaves count 0 and the next status check (orbgpu_synchronize) returns
ORBGPU_ERR_ARG."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_record_round_trip_and_plan_checks(gpu):
    import torch

    from orbslam2_with_quadrics_amd import _lib, synthetic

    L = _lib.lib()
    f1, _ = synthetic.frame_pair(31, 480, 640)
    a = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    b = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    other = gpu.ORBextractor(1500, 1.2, 8, 20, 7)  # different per-frame capacity
    ka, da = a(f1)
    b(np.roll(f1, 5, axis=1))  # plans b for the same image size, with other contents
    other(f1)
    nbytes = int(L.orbgpu_frame_record_bytes(a.ctx))
    assert nbytes == int(L.orbgpu_frame_record_bytes(b.ctx))
    rec = torch.zeros(nbytes, dtype=torch.uint8, device="cuda:0")
    _lib.check(a.ctx, L.orbgpu_frame_record_pack(a.ctx, 0, C.c_void_p(rec.data_ptr())), "pack")
    a.synchronize()
    _lib.check(b.ctx, L.orbgpu_frame_record_unpack(b.ctx, C.c_void_p(rec.data_ptr())), "unpack")
    b.synchronize()
    kb, db = b.batch_download(0)
    assert kb.tobytes() == ka.tobytes() and np.array_equal(db, da)
    def refused(ctx, ptr):
        assert L.orbgpu_frame_record_unpack(ctx, C.c_void_p(ptr)) == _lib.OK  # stream-ordered: no host wait
        assert L.orbgpu_synchronize(ctx) == _lib.ERR_ARG
        assert b"frame record" in L.orbgpu_last_error(ctx)
        assert L.orbgpu_synchronize(ctx) == _lib.OK  # the status was read and cleared
        n = C.c_int(-1)
        assert L.orbgpu_batch_download(ctx, 0, None, None, 0, C.byref(n)) == _lib.OK and n.value == 0

    # a context planned for another frame_cap refuses the record
    refused(other.ctx, rec.data_ptr())
    # a count above frame_cap is refused
    bad = rec.clone()
    bad[:4] = torch.tensor([0x7fffffff], dtype=torch.int32).view(torch.uint8).to("cuda:0")
    refused(b.ctx, bad.data_ptr())
    # a buffer that is not a record (no magic word) is refused
    zero = torch.zeros_like(rec)
    refused(b.ctx, zero.data_ptr())
    # and the good record still unpacks after a refusal
    _lib.check(b.ctx, L.orbgpu_frame_record_unpack(b.ctx, C.c_void_p(rec.data_ptr())), "unpack")
    b.synchronize()
    kb, db = b.batch_download(0)
    assert kb.tobytes() == ka.tobytes() and np.array_equal(db, da)
