"""Frame records (orbgpu_frame_record_pack / _unpack, the unit bench.py broadcasts from rank 0 to the other ranks
at set-up): a record unpacked into a second context reproduces the frame exactly, and a record
that does not fit the receiving context's plan (frame_cap, undistortion), carries a count above frame_cap or lists
its keypoints out of extraction order is refused with ORBGPU_ERR_ARG.  The header is checked on the device, so unpack itself never blocks the
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
    # keypoints out of extraction order (a level-1 keypoint before a level-0 one) are refused: the batched
    # SearchForInitialization takes F1's octave-0 queries from its first kcap_0 slots
    n = int(np.frombuffer(rec[:4].cpu().numpy().tobytes(), np.int32)[0])
    oct0 = np.where(ka["octave"] == 0)[0]
    assert n > 2 and oct0.size > 0 and oct0.size < n
    swapped = rec.clone()
    kbytes = swapped[16:16 + 28 * n].view(n, 28)
    first, last = kbytes[0].clone(), kbytes[n - 1].clone()  # a level-0 and the last (top-level) keypoint
    kbytes[0], kbytes[n - 1] = last, first
    refused(b.ctx, swapped.data_ptr())
    # and the good record still unpacks after a refusal
    _lib.check(b.ctx, L.orbgpu_frame_record_unpack(b.ctx, C.c_void_p(rec.data_ptr())), "unpack")
    b.synchronize()
    kb, db = b.batch_download(0)
    assert kb.tobytes() == ka.tobytes() and np.array_equal(db, da)


def test_refused_record_is_reported_by_the_cross_context_matcher(gpu):
    """a refused record leaves the receiving context's frame 0 empty; a batched SearchForInitialization on
    another context that matches against it must not pass that off as "zero matches" -- its own next status check
    returns ORBGPU_ERR_ARG too (the refusal bit is folded into the matching context's status)."""
    import torch

    from orbslam2_with_quadrics_amd import _lib, synthetic

    L = _lib.lib()
    f1, f2 = synthetic.frame_pair(32, 480, 640)
    ref = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    cur = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    ref(f1)
    cur(f2)
    cap = int(L.orbgpu_max_keypoints(ref.ctx))
    prev = torch.zeros(2 * cap, dtype=torch.float32, device="cuda:0")
    m12 = torch.zeros(cap, dtype=torch.int32, device="cuda:0")
    nm = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    g = _lib.GridGeom()
    _lib.check(cur.ctx, L.orbgpu_grid_geom_for_image(640, 480, C.byref(g)), "grid")

    def match():
        _lib.check(cur.ctx, L.orbgpu_prev_matched_from_frame(ref.ctx, 0, cur.ctx, C.c_void_p(prev.data_ptr())), "prev")
        _lib.check(cur.ctx, L.orbgpu_search_for_initialization_batch(
            ref.ctx, 0, cur.ctx, g, 0.9, 1, 100, C.c_void_p(prev.data_ptr()), C.c_void_p(m12.data_ptr()),
            C.c_void_p(nm.data_ptr())), "init")

    match()
    assert L.orbgpu_synchronize(cur.ctx) == _lib.OK and int(nm.item()) > 50
    zero = torch.zeros(int(L.orbgpu_frame_record_bytes(ref.ctx)), dtype=torch.uint8, device="cuda:0")
    assert L.orbgpu_frame_record_unpack(ref.ctx, C.c_void_p(zero.data_ptr())) == _lib.OK  # refused on the device
    match()
    assert L.orbgpu_synchronize(cur.ctx) == _lib.ERR_ARG
    assert b"frame record" in L.orbgpu_last_error(cur.ctx)
    assert int(nm.item()) == 0
    assert L.orbgpu_synchronize(ref.ctx) == _lib.ERR_ARG  # the receiving context reports it as well


def test_cross_context_fold_follows_the_frame_now_in_the_slot(gpu):
    """the fold reads a per-frame refusal word that every unpack of frame 0 overwrites and every
    extraction clears (status[1]), not the sticky status bit 128.  A refused unpack followed by a good unpack -- or by a
    fresh extraction -- leaves a valid F1, and a batch match on another context against it returns OK with matches,
    although the reference context's own status still reports the earlier refusal (bit 128, read and cleared once)."""
    import torch

    from orbslam2_with_quadrics_amd import _lib, synthetic

    L = _lib.lib()
    f1, f2 = synthetic.frame_pair(32, 480, 640)
    ref = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    cur = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    ref(f1)
    cur(f2)
    cap = int(L.orbgpu_max_keypoints(ref.ctx))
    prev = torch.zeros(2 * cap, dtype=torch.float32, device="cuda:0")
    m12 = torch.zeros(cap, dtype=torch.int32, device="cuda:0")
    nm = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    g = _lib.GridGeom()
    _lib.check(cur.ctx, L.orbgpu_grid_geom_for_image(640, 480, C.byref(g)), "grid")
    rec = torch.zeros(int(L.orbgpu_frame_record_bytes(ref.ctx)), dtype=torch.uint8, device="cuda:0")
    _lib.check(ref.ctx, L.orbgpu_frame_record_pack(ref.ctx, 0, C.c_void_p(rec.data_ptr())), "pack")
    zero = torch.zeros_like(rec)
    d_f1 = ref.device_alloc(f1.nbytes)
    ref.h2d(d_f1, f1)

    def match():
        _lib.check(cur.ctx, L.orbgpu_prev_matched_from_frame(ref.ctx, 0, cur.ctx, C.c_void_p(prev.data_ptr())), "prev")
        _lib.check(cur.ctx, L.orbgpu_search_for_initialization_batch(
            ref.ctx, 0, cur.ctx, g, 0.9, 1, 100, C.c_void_p(prev.data_ptr()), C.c_void_p(m12.data_ptr()),
            C.c_void_p(nm.data_ptr())), "init")

    try:
        match()
        assert L.orbgpu_synchronize(cur.ctx) == _lib.OK
        n_good = int(nm.item())
        assert n_good > 50
        # refused, then a good record: F1 is valid again
        assert L.orbgpu_frame_record_unpack(ref.ctx, C.c_void_p(zero.data_ptr())) == _lib.OK
        assert L.orbgpu_frame_record_unpack(ref.ctx, C.c_void_p(rec.data_ptr())) == _lib.OK
        match()
        assert L.orbgpu_synchronize(cur.ctx) == _lib.OK, L.orbgpu_last_error(cur.ctx)
        assert int(nm.item()) == n_good
        # refused, then a fresh extraction of frame 0: F1 is valid again
        assert L.orbgpu_frame_record_unpack(ref.ctx, C.c_void_p(zero.data_ptr())) == _lib.OK
        ref.extract_batch_device(d_f1, 1, 640, 480, 640, f1.nbytes)
        match()
        assert L.orbgpu_synchronize(cur.ctx) == _lib.OK, L.orbgpu_last_error(cur.ctx)
        assert int(nm.item()) == n_good
        # the reference context's own check still reports its refusals (read and cleared once)
        assert L.orbgpu_synchronize(ref.ctx) == _lib.ERR_ARG
        assert L.orbgpu_synchronize(ref.ctx) == _lib.OK
        # and a refused record in the slot now is still folded, with the cross-context message
        assert L.orbgpu_frame_record_unpack(ref.ctx, C.c_void_p(zero.data_ptr())) == _lib.OK
        match()
        assert L.orbgpu_synchronize(cur.ctx) == _lib.ERR_ARG
        assert b"reference frame" in L.orbgpu_last_error(cur.ctx)
        assert int(nm.item()) == 0
    finally:
        ref.device_free(d_f1)
