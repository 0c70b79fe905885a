"""GPU: cross-stream ordering of device folds (gs_wait_stream / gs_wait_event /
gs_fold_device_after) and the handle-state reset a pool needs
(gs_reset_config). Edges are written on torch streams behind a GPU-side
sleep and folded with NO torch.cuda.synchronize(): without the ordering the fold
would read the buffer before its writer finished."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rmat(gs, n, scale, seed=0x5EED0026):
    import torch
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, scale, seed, True)
    torch.cuda.synchronize()
    return src, dst


@pytest.mark.parametrize("pipeline", [1, 3])
def test_fold_after_torch_stream_no_sync(gs, oracle_mod, pipeline):
    """Each batch is copied into ONE reused staging buffer on a torch side stream after
    a GPU sleep; the summary waits for that stream (fold_device(after=...)), and the
    torch stream waits for the summary's stream before overwriting the buffer."""
    import torch
    n, B = 1 << 16, 1 << 12
    src, dst = _rmat(gs, n, 14)
    bs = torch.empty(B, dtype=torch.int64, device="cuda")
    bd = torch.empty(B, dtype=torch.int64, device="cuda")
    prod = torch.cuda.Stream()
    with gs.Summary("cc", capacity_hint=1 << 14) as s:
        if pipeline > 1:
            s.set_pipelining(pipeline)
        summ_stream = torch.cuda.ExternalStream(s.stream)
        for o in range(0, n, B):
            with torch.cuda.stream(prod):
                # buffer reuse: wait for every fold queued so far (write-after-read);
                # s.stream joins the pipelining lanes first (gs_get_stream)
                prod.wait_stream(torch.cuda.ExternalStream(s.stream))
                torch.cuda._sleep(200000)  # the writer is still busy when the fold is queued
                bs.copy_(src[o:o + B])
                bd.copy_(dst[o:o + B])
            s.fold_device(bs, bd, n=B, after=prod)
        v, lab = s.labels()
        del summ_stream
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_fold_device_after_event(gs, oracle_mod):
    """gs_fold_device_after with a torch event recorded behind the writer."""
    import ctypes
    import torch
    n = 1 << 15
    src, dst = _rmat(gs, n, 13)
    a = torch.empty(n, dtype=torch.int64, device="cuda")
    b = torch.empty(n, dtype=torch.int64, device="cuda")
    prod = torch.cuda.Stream()
    ev = torch.cuda.Event()
    with torch.cuda.stream(prod):
        torch.cuda._sleep(400000)
        a.copy_(src)
        b.copy_(dst)
        ev.record(prod)
    with gs.Summary("cc", capacity_hint=1 << 13) as s:
        rc = gs.lib().gs_fold_device_after(s.handle, a.data_ptr(), b.data_ptr(), None, n, 1,
                                           ctypes.c_void_p(ev.cuda_event))
        assert rc == 0, gs.lib().gs_last_error()
        v, lab = s.labels()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_group_lanes_follow_handle_stream_every_call(gs, oracle_mod, knobs):
    """a group's own-fold lanes wait for the handle stream at EVERY call, so
    a caller that writes each batch on the summary's stream (gs_get_stream) needs no
    device synchronisation. Batches are generated on the summary stream behind a GPU
    sleep into one reused buffer."""
    import torch
    knobs(group_self_apply=1)
    n, B, scale = 1 << 16, 1 << 12, 14
    with gs.Summary("cc", capacity_hint=1 << scale) as s:
        g = gs.Group(s, gs.group_unique_id(), 1, 0, B)
        bs = torch.empty(B, dtype=torch.int64, device="cuda")
        bd = torch.empty(B, dtype=torch.int64, device="cuda")
        ext = torch.cuda.ExternalStream(s.stream)
        for o in range(0, n, B):
            with torch.cuda.stream(ext):
                torch.cuda._sleep(100000)
            gs.gen_rmat(bs, bd, o, B, scale, 0x5EED0026, True, stream=s.stream)
            g.fold_device(bs, bd, B)
            s.sync()  # the next write reuses the buffer (write-after-read): join the lanes
        g.finish()
        v, lab = s.labels()
        g.close()
    src, dst = _rmat(gs, n, scale)
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_group_lanes_follow_marked_handle_stream(gs, oracle_mod, knobs):
    """gs_group.h ordering contract: a caller that queues its own kernels on the
    handle's stream (a cached gs_get_stream) between group calls, with no other call on
    the handle, marks them with gs_wait_stream(h, that stream); the own folds then run
    behind them. Every batch is generated into its own buffers behind a GPU sleep."""
    import torch
    knobs(group_self_apply=1)
    n, B, scale = 1 << 16, 1 << 12, 14
    with gs.Summary("cc", capacity_hint=1 << scale) as s:
        g = gs.Group(s, gs.group_unique_id(), 1, 0, B)
        st = s.stream
        ext = torch.cuda.ExternalStream(st)
        bufs = []
        for o in range(0, n, B):
            bs = torch.empty(B, dtype=torch.int64, device="cuda")
            bd = torch.empty(B, dtype=torch.int64, device="cuda")
            bufs.append((bs, bd))
            with torch.cuda.stream(ext):
                torch.cuda._sleep(100000)
            gs.gen_rmat(bs, bd, o, B, scale, 0x5EED0026, True, stream=st)
            s.wait_stream(st)  # the mark: the group's lanes start behind the generator
            g.fold_device(bs, bd, B)
        g.finish()
        v, lab = s.labels()
        g.close()
    src, dst = _rmat(gs, n, scale)
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_reset_config_restores_a_fresh_handle(gs, oracle_mod):
    """a pooled handle that had change tracking (and so delta tracking) on,
    released with gs_reset_config, folds more than 2^22 edges between takes like a
    fresh handle (with tracking left on that fails with 'delta list full')."""
    import torch
    n = (1 << 22) + (1 << 20)
    src, dst = _rmat(gs, n, 20)
    with gs.Summary("cc", capacity_hint=1 << 20) as s:
        s.set_change_tracking(True)
        s.fold_device(src[:1 << 16], dst[:1 << 16], n=1 << 16)
        s.take_changes()
        s.set_pipelining(2)
        s.reset_config()
        for o in range(0, n, 1 << 20):
            s.fold_device(src[o:], dst[o:], n=min(1 << 20, n - o))
        v, lab = s.labels()
        ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
        assert np.array_equal(v, ov) and np.array_equal(lab, olab)
        # turning change tracking off also turns off the delta tracking it turned on
        s.reset()
        s.set_change_tracking(True)
        s.set_change_tracking(False)
        for o in range(0, n, 1 << 20):
            s.fold_device(src[o:], dst[o:], n=min(1 << 20, n - o))
        s.sync()
        # a summary that tracked deltas itself keeps them after change tracking goes off
        s.reset()
        s.set_delta_tracking(True)
        s.set_change_tracking(True)
        s.set_change_tracking(False)
        with pytest.raises(gs.GSError):
            for o in range(0, n, 1 << 20):
                s.fold_device(src[o:], dst[o:], n=min(1 << 20, n - o))
            s.sync()
    torch.cuda.synchronize()
