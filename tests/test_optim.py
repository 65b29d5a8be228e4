"""Fused Adam (jabd_amd.optim.Adam, csrc/adam.hip) against torch.optim.Adam.

The reference's optimizer is torch.optim.Adam(lr, weight_decay=5e-4)
(train_mobilenetV3_ecagai.py:564); the oracle for this floating-point step
is torch's own fp32 Adam.  Tolerance: rtol 2e-6 / atol 1e-7 after several
steps (the fused kernel may contract a*b+c into an FMA where torch's
separate foreach kernels round twice).
"""
import copy

import numpy as np
import pytest
import torch


def test_chunk_table_host_side():
    """jabd_adam_num_chunks / jabd_adam_fill_chunks are host code (no GPU)."""
    from jabd_amd import _lib
    numel = np.array([0, 1, 1024, 1025, 3000], dtype=np.int64)
    n = _lib.lib().jabd_adam_num_chunks(numel.ctypes.data, len(numel))
    assert n == 0 + 1 + 1 + 2 + 3
    chunks = np.empty(n, dtype=np.int64)
    _lib.call("jabd_adam_fill_chunks", numel.ctypes.data, len(numel), chunks.ctypes.data)
    pairs = [(int(c) >> 40, int(c) & ((1 << 40) - 1)) for c in chunks]
    assert pairs == [(1, 0), (2, 0), (3, 0), (3, 1024), (4, 0), (4, 1024), (4, 2048)]


def test_unsupported_options_raise():
    from jabd_amd.optim import Adam
    p = torch.nn.Parameter(torch.zeros(4))
    p.grad = torch.zeros(4)
    with pytest.raises(NotImplementedError):
        Adam([p], amsgrad=True).step()
    with pytest.raises(NotImplementedError):
        Adam([p]).step()  # CPU tensors: the HIP path has no CPU fallback


def _params(device, seed=0):
    """Fresh leaf Parameters (same values for the same seed)."""
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 3, 3), (64,), (7,), (1,), (1001,), (320, 160, 1, 1), (5, 5, 37)]
    ps = [torch.nn.Parameter(torch.randn(s, generator=g).to(device)) for s in shapes]
    # a parameter at an odd offset inside a larger buffer (scalar path)
    buf = torch.randn(2051, generator=g).to(device)
    ps.append(torch.nn.Parameter(buf[3:2051]))
    return ps


def _grads(ps, step):
    g = torch.Generator().manual_seed(100 + step)
    return [torch.randn(p.shape, generator=g).to(p.device) * (0.1 * (step + 1)) for p in ps]


@pytest.mark.gpu
@pytest.mark.parametrize("wd", [0.0, 5e-4])
def test_adam_matches_torch(cuda, wd):
    from jabd_amd.optim import Adam
    ref, got = _params(cuda), _params(cuda)
    assert got[-1].data_ptr() % 16 != 0
    o_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=wd)
    o_got = Adam(got, lr=1e-3, weight_decay=wd)
    for step in range(6):
        for ps, opt in ((ref, o_ref), (got, o_got)):
            for p, g in zip(ps, _grads(ps, step)):
                p.grad = g
            if step == 3:  # a parameter without a grad is skipped (its step lags)
                ps[1].grad = None
            opt.step()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(ref, got)):
        torch.testing.assert_close(b.data, a.data, rtol=2e-6, atol=1e-7, msg=f"param {i}")
        sa, sb = o_ref.state[a], o_got.state[b]
        assert float(sa["step"]) == float(sb["step"])
        torch.testing.assert_close(sb["exp_avg"], sa["exp_avg"], rtol=2e-6, atol=1e-8)
        torch.testing.assert_close(sb["exp_avg_sq"], sa["exp_avg_sq"], rtol=2e-6, atol=1e-10)


@pytest.mark.gpu
def test_adam_state_dict_roundtrip(cuda):
    """A torch Adam checkpoint resumes in the fused Adam and vice versa."""
    from jabd_amd.optim import Adam
    ref, got = _params(cuda, 1), _params(cuda, 1)
    o_ref = torch.optim.Adam(ref, lr=2e-3, weight_decay=5e-4)
    for step in range(2):
        for p, g in zip(ref, _grads(ref, step)):
            p.grad = g
        o_ref.step()
    with torch.no_grad():
        for a, b in zip(ref, got):
            b.copy_(a)
    o_got = Adam(got, lr=2e-3, weight_decay=5e-4)
    # deepcopy: torch's state_dict()/load_state_dict() share the `step` tensors
    o_got.load_state_dict(copy.deepcopy(o_ref.state_dict()))
    for step in range(2, 4):
        for ps, opt in ((ref, o_ref), (got, o_got)):
            for p, g in zip(ps, _grads(ps, step)):
                p.grad = g
            opt.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        torch.testing.assert_close(b.data, a.data, rtol=2e-6, atol=1e-7)
    back = torch.optim.Adam(ref, lr=2e-3, weight_decay=5e-4)
    back.load_state_dict(copy.deepcopy(o_got.state_dict()))
    assert float(back.state_dict()["state"][0]["step"]) == 4.0


@pytest.mark.gpu
def test_adam_steps_reach_the_training_convs(cuda):
    """The fused step writes parameters through raw pointers; the training
    convs' packed-weight cache (train._packed, keyed on _version) must see the
    update: three train_steps with jabd Adam match three with torch.optim.Adam."""
    from _util import init_for_parity
    from jabd_amd import parallel, synth
    from jabd_amd.optim import Adam
    from nets.retinaface_r import RetinaFace
    from nets.retinaface_training import MultiBoxLoss
    from utils.anchors import Anchors
    from utils.config import cfg_mnet
    x = synth.images(2, 96, seed=5).to(cuda)
    tg = [torch.from_numpy(t).to(cuda) for t in synth.targets(2, 96, seed=6)]
    pri = Anchors(cfg_mnet, image_size=(96, 96)).get_anchors().to(cuda)
    losses = {}
    for name, mk in (("torch", torch.optim.Adam), ("jabd", Adam)):
        m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=8).to(cuda).train()
        opt = mk(m.parameters(), lr=1e-2, weight_decay=5e-4)
        crit = MultiBoxLoss(2, 0.35, 7, cfg_mnet["variance"], True)
        losses[name] = [float(parallel.train_step(m, crit, opt, x, tg, pri)[0]) for _ in range(3)]
    assert losses["torch"][0] != losses["torch"][2]  # the steps do move the loss
    for a, b in zip(losses["torch"], losses["jabd"]):
        assert abs(a - b) <= 1e-4 * abs(a), losses


@pytest.mark.gpu
@pytest.mark.parametrize("max_jobs", [1024, 16])
def test_batched_repack_equals_fresh_packs(cuda, max_jobs, monkeypatch):
    """After a fused Adam step, every cached training pack of the model is
    rewritten in place by ONE jabd_conv_pack_multi_f32 launch (train.repack;
    max_jobs 16: the same rows split over several launches, as a model with
    more packs than the kernel's 1024-job table takes them):
    each must equal a fresh jabd_conv_pack_f32 pack of the updated weight bit
    for bit (both forms, both layouts), and the cache must be keyed on the new
    version so the next forward reuses it without repacking."""
    from _util import init_for_parity
    from jabd_amd import functional as F
    from jabd_amd import parallel, synth, train
    from jabd_amd.optim import Adam
    from nets.retinaface_r import RetinaFace
    from nets.retinaface_training import MultiBoxLoss
    from utils.anchors import Anchors
    from utils.config import cfg_mnet
    monkeypatch.setattr(train, "REPACK_MAX_JOBS", max_jobs)
    monkeypatch.setattr(train, "_REPACK_TABLES", {})
    x = synth.images(2, 96, seed=5).to(cuda)
    tg = [torch.from_numpy(t).to(cuda) for t in synth.targets(2, 96, seed=6)]
    pri = Anchors(cfg_mnet, image_size=(96, 96)).get_anchors().to(cuda)
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=8).to(cuda).train()
    opt = Adam(m.parameters(), lr=1e-2, weight_decay=5e-4)
    crit = MultiBoxLoss(2, 0.35, 7, cfg_mnet["variance"], True)
    parallel.train_step(m, crit, opt, x, tg, pri)
    torch.cuda.synchronize()
    n = 0
    for p in m.parameters():
        ent = train._PACK.get(id(p))
        if ent is None or ent[0]() is not p:
            continue
        for (ver, ptr, tr), pk in ent[1].items():
            assert ver == p._version and ptr == p.data_ptr()
            ref = F.pack_weight_device(p, tr)
            assert torch.equal(pk.w, ref.w)
            assert (pk.w32 is None) == (ref.w32 is None)
            if pk.w32 is not None:
                assert torch.equal(pk.w32, ref.w32)
            n += 1
    assert n > 50, n
    # the next forward takes the repacked copies: no per-weight pack launch
    # for a parameter (tensors derived per step, e.g. weight slices, are
    # packed per call as before)
    calls = []
    orig = F.pack_weight_device
    F.pack_weight_device = lambda w, *a, **k: calls.append(w) or orig(w, *a, **k)
    try:
        parallel.train_step(m, crit, opt, x, tg, pri)
    finally:
        F.pack_weight_device = orig
    params = {id(p) for p in m.parameters()}
    print("per-call packs of derived tensors:", [tuple(w.shape) for w in calls])
    assert not [w for w in calls if id(w) in params]
