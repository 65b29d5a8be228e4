"""A9/A11 training parity: MultiBoxLoss (values, selection, gradients) and the
full detector backward (every parameter gradient, BN running stats) of the
HIP path against autograd through the oracle restatement (PyTorch-CPU fp32).
Tolerances: losses 1e-5 relative; gradients vs an fp64 oracle run with the
HIP forward's activation masks (tests/_kinks.py), per tensor relative
Frobenius error <= max(2e-3, 4x the mask-matched fp32 oracle's own error)."""
import pytest
import torch

from _kinks import Kinks
from _util import init_for_parity, rel_err
from oracle import box_ref, model_ref


def _targets(B, size, seed):
    from jabd_amd import synth
    return [torch.from_numpy(t) for t in synth.targets(B, size, seed=seed)]


@pytest.mark.gpu
def test_multibox_loss_parity(cuda):
    from nets.retinaface_training import MultiBoxLoss
    cfg = {"min_sizes": [[16, 32], [64, 128], [256, 512]], "steps": [8, 16, 32], "clip": False}
    pri = box_ref.anchors(cfg, (256, 256))
    B, A = 4, pri.shape[0]
    g = torch.Generator().manual_seed(3)
    loc = torch.randn(B, A, 4, generator=g)
    conf = torch.randn(B, A, 2, generator=g) * 2
    landm = torch.randn(B, A, 10, generator=g)
    tg = _targets(B, 256, 9)
    # oracle: match + loss + autograd
    lt, ct, lmt = box_ref.match_batch(tg, pri)
    leaves = [t.clone().requires_grad_(True) for t in (loc, conf, landm)]
    rl, rc, rlm, info = box_ref.multibox_loss(*leaves, lt, ct, lmt)
    (2.0 * rl + rc + rlm).backward()
    # HIP path
    crit = MultiBoxLoss(2, 0.35, 7, [0.1, 0.2], True)
    gl = [t.to(cuda).requires_grad_(True) for t in (loc, conf, landm)]
    l, c, lm = crit(tuple(gl), pri.to(cuda), [t.to(cuda) for t in tg])
    (2.0 * l + c + lm).backward()
    for got, ref in ((l, rl), (c, rc), (lm, rlm)):
        assert abs(float(got) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref))), (got, ref)
    for g_, r_ in zip(gl, leaves):
        assert rel_err(g_.grad, r_.grad) < 1e-5


@pytest.mark.gpu
def test_multibox_diou_loss_parity(cuda):
    """The DIoU variant (nets/retinaface_training_DIOU.py:524-665): values 1e-5
    relative to the fp32 oracle; gradients (analytic DIoU backward in the kernel
    vs autograd through the oracle) relative Frobenius error < 1e-4 against an
    fp64 oracle run."""
    from nets.retinaface_training_DIOU import MultiBoxLoss
    cfg = {"min_sizes": [[16, 32], [64, 128], [256, 512]], "steps": [8, 16, 32], "clip": False}
    pri = box_ref.anchors(cfg, (256, 256))
    B, A = 4, pri.shape[0]
    g = torch.Generator().manual_seed(4)
    loc = torch.randn(B, A, 4, generator=g)
    conf = torch.randn(B, A, 2, generator=g) * 2
    landm = torch.randn(B, A, 10, generator=g)
    tg = _targets(B, 256, 11)
    lt, ct, lmt = box_ref.match_iou_batch(tg, pri)
    refs = {}
    for dt in (torch.float32, torch.float64):
        leaves = [t.clone().to(dt).requires_grad_(True) for t in (loc, conf, landm)]
        out = box_ref.multibox_loss(*leaves, lt.to(dt), ct, lmt.to(dt), diou=(pri, [0.1, 0.2]))
        (2.0 * out[0] + out[1] + out[2]).backward()
        refs[dt] = (out[:3], [t.grad for t in leaves])
    crit = MultiBoxLoss(2, 0.35, 7, [0.1, 0.2], True)
    gl = [t.to(cuda).requires_grad_(True) for t in (loc, conf, landm)]
    l, c, lm = crit(tuple(gl), pri.to(cuda), [t.to(cuda) for t in tg])
    (2.0 * l + c + lm).backward()
    for got, ref in zip((l, c, lm), refs[torch.float32][0]):
        assert abs(float(got) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref))), (got, ref)
    assert float(l) > 0.0
    for g_, r_ in zip(gl, refs[torch.float64][1]):
        assert rel_err(g_.grad, r_) < 1e-4


def _oracle_grads(sd, fn, x, dtype, kk, wseed=5):
    P = {k: (v.clone().to(dtype).requires_grad_(True)
             if v.is_floating_point() and "running" not in k
             else (v.clone().to(dtype) if v.is_floating_point() else v.clone()))
         for k, v in sd.items()}
    g = torch.Generator().manual_seed(wseed)
    with kk.replay():
        ref = fn(P, x.to(dtype), "train", train_bn=True)
    assert not kk.unmatched, f"oracle kinks without a HIP tensor: {kk.unmatched[:5]}"
    wts = [torch.randn(r.shape, generator=g) for r in ref]
    sum(((r * w.to(dtype)).sum() for r, w in zip(ref, wts))).backward()
    grads = {k: p.grad for k, p in P.items()
             if isinstance(p, torch.Tensor) and p.requires_grad and p.grad is not None}
    return [r.detach() for r in ref], grads, P, wts


def _fro(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _train_compare(model, fn, x, cuda, tol=2e-3):
    """Gradients are judged per tensor against an fp64 run of the oracle
    whose activation masks (ReLU / LeakyReLU / Hardswish / Hardsigmoid
    regions, max-pool argmaxes) are the HIP forward's own (tests/_kinks.py):
    relative Frobenius error within max(tol, 4x the error of the equally
    mask-matched fp32 oracle run)."""
    import re
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    kk = Kinks()
    m = model.to(cuda).train()
    with kk.record():
        out = m(x.to(cuda))
    ref64, g64, P64, wts = _oracle_grads(sd, fn, x, torch.float64, kk)
    ref32, g32, _, _ = _oracle_grads(sd, fn, x, torch.float32, kk)
    assert kk.matched > 20
    sum(((o * w.to(cuda)).sum() for o, w in zip(out, wts))).backward()
    for o, r, name in zip(out, ref64, ("loc", "conf", "landm")):
        e = rel_err(o.detach(), r)
        assert e < 1e-3, f"{name} forward rel err {e:.2e}"
    named = dict(m.named_parameters())
    gmax = max(float(g.abs().max()) for g in g64.values())
    # Analytically-zero gradients (rounding noise in every path) are checked
    # for smallness: f_key.bias shifts all logits of a pixel equally
    # (softmax-invariant); a bias feeding conv->BN in training mode is removed
    # by that BN's batch mean.
    zero = re.compile(r"(f_key\.bias|skip\.2\.bias)$")
    rows = []
    for k, rg in g64.items():
        q = named[k]
        assert q.grad is not None, f"no HIP gradient for {k}"
        if zero.search(k) or (k.endswith("skip.1.bias")
                              and k.replace("skip.1.bias", "skip.3.weight") in g64):
            assert float(q.grad.abs().max()) <= 1e-4 * gmax, k
            continue
        rows.append((_fro(q.grad, rg), _fro(g32[k], rg), k))
    assert len(rows) > 50
    bad = [r for r in rows if r[0] > max(tol, 4 * r[1])]
    assert not bad, f"gradients off vs fp64 (hip, oracle-fp32, name): {sorted(bad)[-5:]}"
    for k, v in m.state_dict().items():
        if "running" in k:
            e = rel_err(v, P64[k])
            assert e < 1e-4, f"{k} running stat rel err {e:.2e}"


@pytest.mark.gpu
def test_train_backward_parity_mnv3(cuda):
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=4)
    x = torch.randn(2, 3, 96, 96, generator=torch.Generator().manual_seed(1)) * 50
    _train_compare(m, model_ref.retinaface_mnv3, x, cuda)


@pytest.mark.gpu
def test_train_backward_parity_r50(cuda):
    from nets.retinaface_eca_nonlocal import RetinaFace
    from utils.config import cfg_re50
    m = init_for_parity(RetinaFace(cfg=cfg_re50, mode="train"), seed=6)
    x = torch.randn(2, 3, 128, 128, generator=torch.Generator().manual_seed(2)) * 50
    _train_compare(m, model_ref.retinaface_r50, x, cuda)


@pytest.mark.gpu
def test_train_r50_blocks_parity(cuda):
    """Stem (7x7/2 conv on NCHW input, BN, ReLU, 3x3/2 max-pool) and
    bottlenecks layer1.0 (1x1 downsample), layer2.0 (stride-2 downsample),
    layer2.1 (identity residual) alone: every gradient vs fp64 autograd."""
    from jabd_amd import train as T
    from nets.retinaface_eca_nonlocal import RetinaFace
    from utils.config import cfg_re50
    m = init_for_parity(RetinaFace(cfg=cfg_re50, mode="train"), seed=11)
    x = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(3)) * 50
    blocks = ("layer1.0.", "layer2.0.", "layer2.1.")
    sd = {k[5:]: v.clone() for k, v in m.state_dict().items() if k.startswith("body.")
          and (k.startswith("body.conv1") or k.startswith("body.bn1")
               or any(k.startswith("body." + b) for b in blocks))}

    def ref(dtype):
        P = {k: (v.to(dtype).requires_grad_(True) if v.is_floating_point() and "running" not in k
                 else (v.to(dtype) if v.is_floating_point() else v)) for k, v in sd.items()}
        ctx = model_ref.Ctx(P, True)
        with kk.replay():
            s = model_ref.kink(ctx.bn(ctx.conv(x.to(dtype), "conv1", 2, 3), "bn1"), "relu")
            s = model_ref.maxpool(s)
            for b in blocks:
                st = 2 if b == "layer2.0." else 1
                o = model_ref.kink(ctx.bn(ctx.conv(s, b + "conv1"), b + "bn1"), "relu")
                o = model_ref.kink(ctx.bn(ctx.conv(o, b + "conv2", st, 1), b + "bn2"), "relu")
                o = ctx.bn(ctx.conv(o, b + "conv3"), b + "bn3")
                idn = s if b == "layer2.1." else ctx.bn(ctx.conv(s, b + "downsample.0", st),
                                                         b + "downsample.1")
                s = model_ref.kink(o + idn, "relu")
        assert not kk.unmatched, kk.unmatched
        w = torch.randn(s.shape, generator=torch.Generator().manual_seed(8)).to(dtype)
        (s * w).sum().backward()
        return s.detach(), w, {k: p.grad for k, p in P.items()
                               if isinstance(p, torch.Tensor) and p.grad is not None}

    kk = Kinks()
    body = m.to(cuda).train().body
    with kk.record():
        s = T.bn_act(T.conv(x.to(cuda), body.conv1, 2, 3, nchw_in=True), body.bn1, "relu")
        s = T.MaxPoolFn.apply(s)
        for blk in (body.layer1[0], body.layer2[0], body.layer2[1]):
            s = T._r50_block(blk, s)
    y64, w, g64 = ref(torch.float64)
    _, _, g32 = ref(torch.float32)
    y = s.permute(0, 3, 1, 2)
    assert rel_err(y.detach(), y64) < 1e-4
    (y * w.float().to(cuda)).sum().backward()
    named = dict(body.named_parameters())
    bad = []
    for k, rg in g64.items():
        if k.endswith("conv1.bias"):
            continue
        e, e32 = _fro(named[k].grad, rg), _fro(g32[k], rg)
        if e > max(1e-4, 4 * e32):
            bad.append((e, e32, k))
    assert len(g64) > 30 and not bad, sorted(bad)[-5:]


@pytest.mark.gpu
def test_train_r50_bn3_link(cuda, monkeypatch):
    """bn3's backward taken from the next bottleneck's conv1 data gradient
    (jabd_conv_bn_bwd_sums_res_f32 writes dz = dout * [out > 0] and the
    BatchNorm sums; JABD_R50_BN3_LINK) against the unlinked form
    (jabd_bn_act_bwd_ex_f32 on dout) over layer1.0 (downsample) -> layer1.1
    -> layer1.2 -> layer2.0 (stride-2 downsample): the three links are
    taken, and every gradient and the input gradient agree to fp32
    reassociation."""
    from jabd_amd import train as T
    from nets.retinaface_eca_nonlocal import RetinaFace
    from utils.config import cfg_re50
    m = init_for_parity(RetinaFace(cfg=cfg_re50, mode="train"), seed=5)
    body = m.to(cuda).train().body
    blocks = (body.layer1[0], body.layer1[1], body.layer1[2], body.layer2[0])
    x0 = torch.randn(2, 37, 29, 64, generator=torch.Generator().manual_seed(4)).to(cuda)
    w = None
    calls = []
    real = T._dgrad_1x1_res_bn3

    def spy(*a):
        r = real(*a)
        calls.append(r[1] is not None)
        return r
    monkeypatch.setattr(T, "_dgrad_1x1_res_bn3", spy)
    res = {}
    for link in (True, False):
        monkeypatch.setattr(T, "R50_BN3_LINK", link)
        body.zero_grad()
        x = x0.clone().requires_grad_(True)
        with T._BatchCounts():
            s = x
            for blk in blocks:
                s = T._r50_block(blk, s)
        if w is None:
            w = torch.randn(s.shape, generator=torch.Generator().manual_seed(6)).to(cuda)
        (s * w).sum().backward()
        torch.cuda.synchronize()
        res[link] = (s.detach().clone(), x.grad.clone(),
                     {k: p.grad.clone() for k, p in body.named_parameters() if p.grad is not None})
    assert calls == [True, True, True], calls
    assert torch.equal(res[True][0], res[False][0])
    assert rel_err(res[True][1], res[False][1]) < 1e-5
    g1, g0 = res[True][2], res[False][2]
    assert len(g1) == len(g0) > 30
    bad = [(rel_err(g1[k], g0[k]), k) for k in g0 if rel_err(g1[k], g0[k]) > 1e-5]
    assert not bad, sorted(bad)[-5:]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["mnv3", "r50"])
def test_train_head_parity(cuda, kind):
    """ECA -> FPN(+NLM) -> SSH -> heads sub-graph alone (backbone features as
    leaves), gradients vs the fp64 oracle."""
    from jabd_amd import train as T
    if kind == "mnv3":
        from nets.retinaface_r import RetinaFace
        from utils.config import cfg_mnet as cfg
        chans, names, nlm_name, leaky = (40, 80, 160), ("eca_40", "eca_80", "eca_160"), "fpn.nlm.", 0.1
    else:
        from nets.retinaface_eca_nonlocal import RetinaFace
        from utils.config import cfg_re50 as cfg
        chans, names, nlm_name, leaky = (512, 1024, 2048), ("eca_64", "eca_128", "eca_256"), "fpn.Nlm.", 0.0
    m = init_for_parity(RetinaFace(cfg=cfg, mode="train"), seed=9)
    g = torch.Generator().manual_seed(4)
    feats = [torch.randn(2, c, s, s, generator=g) for c, s in zip(chans, (16, 8, 4))]
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    kk = Kinks()
    mg = m.to(cuda).train()
    fg = [f.permute(0, 2, 3, 1).contiguous().to(cuda).requires_grad_() for f in feats]
    nlm = mg.fpn.nlm if kind == "mnv3" else mg.fpn.Nlm
    with kk.record():
        out = T._head(mg, fg, names, nlm)
    P = {k: (v.double().requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.double() if v.is_floating_point() else v)) for k, v in sd.items()}
    fr = [f.double().requires_grad_() for f in feats]
    ctx = model_ref.Ctx(P, True)
    with kk.replay():
        fe = [model_ref.eca(ctx, f, n, "sigmoid") for f, n in zip(fr, names)]
        f3 = model_ref.fpn(ctx, fe, leaky, nlm_name)
        f3 = [model_ref.ssh(ctx, model_ref.eca(ctx, f3[i], "eca_fpn", "sigmoid"), f"ssh{i + 1}.",
                            leaky) for i in range(3)]
        ref = model_ref.heads(ctx, f3, "train")
    assert not kk.unmatched and kk.matched >= 12, (kk.matched, kk.unmatched)
    wts = [torch.randn(r.shape, generator=g, dtype=torch.float64) for r in ref]
    sum(((r * w).sum() for r, w in zip(ref, wts))).backward()
    sum(((o * w.float().to(cuda)).sum() for o, w in zip(out, wts))).backward()
    for o, r in zip(out, ref):
        assert rel_err(o.detach(), r.detach()) < 1e-3
    errs = [(rel_err(f.grad.permute(0, 3, 1, 2), r.grad), f"feat{i}") for i, (f, r) in
            enumerate(zip(fg, fr))]
    named = dict(mg.named_parameters())
    for k, p in P.items():
        if isinstance(p, torch.Tensor) and p.requires_grad and p.grad is not None:
            if k.endswith("f_key.bias"):
                continue
            errs.append((rel_err(named[k].grad, p.grad), k))
    errs.sort(reverse=True)
    assert errs[0][0] < 2e-3, errs[:6]
