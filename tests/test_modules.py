"""The module surface (jabd_amd/modules.py, nets/*): every module the
reference's callers compose themselves runs libjabd kernels on its own.

Leaf modules (Conv2d, BatchNorm2d/1d, activations, pools, Linear) are checked
against the torch base class's own forward on the CPU in float64 — the plain
PyTorch reference of the same op — forward and (training mode) every
gradient and BN running statistic.  Composites (blocks, SSH, FPN, NLM, ECA,
heads, whole backbones) are checked against the oracle restatement
(oracle/model_ref.py).  Tolerances: forward 1e-4 relative (max-norm) for
single ops, 1e-3 for whole networks (north-star); gradients 1e-4 / 2e-3.
"""
import copy

import pytest
import torch
import torch.nn as nn

from _kinks import Kinks
from _util import init_for_parity, rel_err
from oracle import model_ref

pytestmark = pytest.mark.gpu


def _cl(x):
    return x.contiguous(memory_format=torch.channels_last)


def _leaf_check(cuda, mod, base, x, train=True, fwd_tol=1e-5, grad_tol=1e-5, layout=_cl):
    """mod (HIP subclass) vs base.forward of a float64 CPU copy."""
    ref_m = copy.deepcopy(mod).double().train(train)
    xr = x.double().requires_grad_(train)
    yr = base.forward(ref_m, xr)
    m = mod.to(cuda).train(train)
    xg = layout(x.to(cuda)).requires_grad_(train)
    y = m(xg)
    assert y.shape == yr.shape
    assert rel_err(y.detach(), yr.detach()) <= fwd_tol, rel_err(y.detach(), yr.detach())
    if not train:
        assert not y.requires_grad  # eval mode is inference only
        return
    w = torch.randn(yr.shape, generator=torch.Generator().manual_seed(7), dtype=torch.float64)
    (yr * w).sum().backward()
    (y * w.float().to(cuda)).sum().backward()
    assert rel_err(xg.grad, xr.grad) <= grad_tol, ("input grad", rel_err(xg.grad, xr.grad))
    named = dict(ref_m.named_parameters())
    for k, p in m.named_parameters():
        assert rel_err(p.grad, named[k].grad) <= grad_tol, (k, rel_err(p.grad, named[k].grad))
    ref_b = dict(ref_m.named_buffers())
    for k, b in m.named_buffers():
        if b.is_floating_point():
            assert rel_err(b, ref_b[k]) < 1e-5, k


def _x(shape, seed=0, scale=1.0):
    return torch.randn(shape, generator=torch.Generator().manual_seed(seed)) * scale


# ----------------------------------------------------------------------------- leaves
@pytest.mark.parametrize("cin,cout,k,s,p,groups,bias", [
    (16, 24, 3, 1, 1, 1, False), (16, 24, 3, 2, 1, 1, True), (40, 80, 1, 1, 0, 1, False),
    (32, 32, 3, 2, 1, 32, False), (72, 72, 5, 1, 2, 72, False), (8, 12, 3, 1, 1, 1, False)])
@pytest.mark.parametrize("train", [True, False])
def test_conv2d_leaf(cuda, cin, cout, k, s, p, groups, bias, train):
    from jabd_amd.modules import Conv2d
    torch.manual_seed(cin + k)
    m = init_for_parity(Conv2d(cin, cout, k, s, p, groups=groups, bias=bias), seed=k)
    _leaf_check(cuda, m, nn.Conv2d, _x((2, cin, 19, 23), 1), train, 1e-5, 1e-4)


@pytest.mark.parametrize("train", [True, False])
def test_conv2d_stem_reads_nchw(cuda, train):
    """A 3-channel NCHW network input goes straight into the conv (no layout copy)."""
    from jabd_amd.modules import Conv2d
    m = init_for_parity(Conv2d(3, 16, 3, 2, 1, bias=False), seed=2)
    _leaf_check(cuda, m, nn.Conv2d, _x((2, 3, 33, 40), 3, 50.0), train, 1e-5, 1e-4,
                layout=lambda t: t.contiguous())


@pytest.mark.parametrize("train", [True, False])
def test_batchnorm2d_leaf(cuda, train):
    from jabd_amd.modules import BatchNorm2d
    m = init_for_parity(BatchNorm2d(24), seed=3)
    _leaf_check(cuda, m, nn.BatchNorm2d, _x((4, 24, 9, 11), 4, 3.0) + 1.0, train, 1e-5, 1e-4)


def test_batchnorm2d_eval_odd_channels(cuda):
    from jabd_amd.modules import BatchNorm2d
    m = init_for_parity(BatchNorm2d(10), seed=5)
    _leaf_check(cuda, m, nn.BatchNorm2d, _x((2, 10, 7, 7), 5), False)


@pytest.mark.parametrize("train", [True, False])
def test_batchnorm1d_leaf(cuda, train):
    from jabd_amd.modules import BatchNorm1d
    m = BatchNorm1d(1280)
    with torch.no_grad():
        m.weight.normal_(1, 0.2)
        m.bias.normal_(0, 0.1)
        m.running_var.uniform_(0.5, 1.5)
    _leaf_check(cuda, m, nn.BatchNorm1d, _x((8, 1280), 6), train, 1e-5, 1e-4,
                layout=lambda t: t.contiguous())


@pytest.mark.parametrize("name", ["ReLU", "LeakyReLU", "Hardswish", "Hardsigmoid", "Sigmoid"])
@pytest.mark.parametrize("shape", [(2, 24, 13, 9), (5, 1281)])
def test_activation_leaves(cuda, name, shape):
    from jabd_amd import modules as M
    kw = {"negative_slope": 0.1} if name == "LeakyReLU" else {}
    m = getattr(M, name)(**kw)
    x = _x(shape, 8, 4.0)
    lay = _cl if len(shape) == 4 else (lambda t: t.contiguous())
    _leaf_check(cuda, m, getattr(nn, name), x, True, 2e-6, 2e-6, layout=lay)


@pytest.mark.parametrize("train", [True, False])
def test_maxpool_leaf(cuda, train):
    from jabd_amd.modules import MaxPool2d
    _leaf_check(cuda, MaxPool2d(3, 2, 1), nn.MaxPool2d, _x((2, 64, 17, 20), 9), train, 0.0, 1e-6)


@pytest.mark.parametrize("size", [1, 3, 6, 8])
def test_adaptive_avgpool_leaf(cuda, size):
    from jabd_amd.modules import AdaptiveAvgPool2d
    _leaf_check(cuda, AdaptiveAvgPool2d(size), nn.AdaptiveAvgPool2d, _x((2, 12, 13, 17), 10),
                True, 1e-6, 1e-6)


@pytest.mark.parametrize("train", [True, False])
def test_linear_leaf(cuda, train):
    from jabd_amd.modules import Linear
    torch.manual_seed(3)
    _leaf_check(cuda, Linear(96, 40), nn.Linear, _x((6, 96), 11), train, 1e-5, 1e-4,
                layout=lambda t: t.contiguous())


# ----------------------------------------------------------------------------- composites
def _P(module, dtype=torch.float64, grad=True):
    return {k: (v.detach().cpu().clone().to(dtype).requires_grad_(grad)
                if v.is_floating_point() and "running" not in k
                else (v.detach().cpu().clone().to(dtype) if v.is_floating_point()
                      else v.cpu().clone()))
            for k, v in module.state_dict().items()}


def _composite(cuda, module, ref_fn, inputs, train, fwd_tol=1e-4, grad_tol=2e-3,
               as_list=False, prefix=""):
    """module(*inputs) (or module(list) with as_list) on the GPU vs
    ref_fn(ctx, *inputs) through the oracle, whose parameters are the
    module's state_dict keys under `prefix`.  Training: every input and
    parameter gradient against a float64 oracle run whose activation masks
    are the HIP forward's own (tests/_kinks.py; every oracle kink must find
    its HIP tensor), relative error within max(grad_tol, 4x the error of the
    equally mask-matched float32 oracle run)."""
    snap = {prefix + k: v.detach().cpu().clone() for k, v in module.state_dict().items()}

    def run_ref(dtype):
        P = {k: (v.clone().to(dtype).requires_grad_(train)
                 if v.is_floating_point() and "running" not in k
                 else (v.clone().to(dtype) if v.is_floating_point() else v.clone()))
             for k, v in snap.items()}
        ctx = model_ref.Ctx(P, train)
        xr = [t.to(dtype).requires_grad_(train) for t in inputs]
        ref = ref_fn(ctx, *xr)
        refs = list(ref) if isinstance(ref, (list, tuple)) else [ref]
        return P, xr, refs

    kk = Kinks()
    m = module.to(cuda).train(train)
    xg = [_cl(t.to(cuda)).requires_grad_(train) for t in inputs]
    with kk.record():
        out = m(xg) if as_list else m(*xg)
    outs = list(out) if isinstance(out, (list, tuple)) else [out]
    with kk.replay():
        P, xr, refs = run_ref(torch.float64)
    for o, r in zip(outs, refs):
        assert o.shape == r.shape
        assert rel_err(o.detach(), r.detach()) < fwd_tol, rel_err(o.detach(), r.detach())
    if not train:
        return
    assert not kk.unmatched, kk.unmatched
    with kk.replay():
        P32, xr32, refs32 = run_ref(torch.float32)
    assert not kk.unmatched, kk.unmatched
    g = torch.Generator().manual_seed(12)
    wts = [torch.randn(r.shape, generator=g, dtype=torch.float64) for r in refs]
    sum((r * w).sum() for r, w in zip(refs, wts)).backward()
    sum((r * w.float()).sum() for r, w in zip(refs32, wts)).backward()
    sum((o * w.float().to(cuda)).sum() for o, w in zip(outs, wts)).backward()
    rows = [(rel_err(a.grad, b.grad), rel_err(c.grad, b.grad), f"input{i}")
            for i, (a, b, c) in enumerate(zip(xg, xr, xr32))]
    named = dict(m.named_parameters())
    for k, p in P.items():
        if isinstance(p, torch.Tensor) and p.requires_grad and p.grad is not None:
            if k.endswith("f_key.bias") or k.endswith("skip.2.bias") or \
                    k.endswith("skip.1.bias") and k.replace("skip.1.bias", "skip.3.weight") in P:
                continue  # analytically zero (softmax shift / a BN mean removes it)
            rows.append((rel_err(named[k[len(prefix):]].grad, p.grad),
                         rel_err(P32[k].grad, p.grad), k))
    bad = [r for r in rows if r[0] > max(grad_tol, 4 * r[1])]
    assert not bad, sorted(bad, reverse=True)[:5]
    for k, v in m.state_dict().items():
        if "running" in k:
            assert rel_err(v, P[prefix + k]) < 1e-4, k


BLOCKS = [  # (class name, spec, gate)
    ("Block_eca", (3, 16, 64, 24, "relu", False, 2), "eca"),
    ("Block_eca", (5, 40, 120, 40, "relu", True, 1), "eca"),
    ("Block_eca", (3, 80, 480, 112, "hswish", True, 1), "eca"),
    ("Block", (3, 16, 16, 16, "relu", True, 2), "se"),
    ("Block", (5, 40, 120, 48, "hswish", True, 1), "se"),
    ("Block", (3, 24, 72, 24, "relu", False, 1), "none"),
    ("Block_eca_G", (5, 24, 72, 40, "relu", True, 2), "beca"),
    ("Block_eca_G", (3, 80, 184, 80, "hswish", False, 1), "beca"),
]


@pytest.mark.parametrize("cls,spec,gate", BLOCKS)
@pytest.mark.parametrize("train", [True, False])
def test_mnv3_blocks(cuda, cls, spec, gate, train):
    import nets.mobilenetV3 as mv3
    k, cin, exp, cout, act, se, stride = spec
    act_cls = nn.ReLU if act == "relu" else nn.Hardswish
    m = init_for_parity(getattr(mv3, cls)(k, cin, exp, cout, act_cls, se, stride), seed=cin)
    _composite(cuda, m, lambda ctx, x: model_ref.block(ctx, x, "", spec, gate),
               [_x((4, cin, 20, 24), cin)], train)


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("cin,cout", [(40, 40), (256, 256), (64, 32)])
def test_ssh_module(cuda, train, cin, cout):
    from nets.layers import SSH
    m = init_for_parity(SSH(cin, cout), seed=cout)
    leaky = 0.1 if cout <= 64 else 0.0
    _composite(cuda, m, lambda ctx, x: model_ref.ssh(ctx, x, "", leaky),
               [_x((2, cin, 16, 12), 2)], train)


@pytest.mark.parametrize("kind", ["nlm40", "plain"])
@pytest.mark.parametrize("train", [True, False])
def test_fpn_module(cuda, kind, train):
    if kind == "nlm40":
        from nets.retinaface_r import FPN
        m, nlm = FPN([40, 80, 160], 40), "nlm."
    else:
        from nets.layers import FPN
        m, nlm = FPN([64, 128, 256], 64), None
    m = init_for_parity(m, seed=5)
    chans = [40, 80, 160] if kind == "nlm40" else [64, 128, 256]
    feats = [_x((2, c, s, s + 2), i) for i, (c, s) in enumerate(zip(chans, (24, 12, 6)))]
    _composite(cuda, m, lambda ctx, *f: model_ref.fpn(ctx, list(f), 0.1, nlm, pre=""),
               feats, train, as_list=True)


@pytest.mark.parametrize("train", [True, False])
def test_nlm_module(cuda, train):
    from nets.retinaface_r import NLM
    m = init_for_parity(NLM(40), seed=6)
    _composite(cuda, m, lambda ctx, x: model_ref.nlm(ctx, x, ""), [_x((2, 40, 18, 22), 3)],
               train)


@pytest.mark.parametrize("train", [True, False])
def test_psp_module(cuda, train):
    from nets.retinaface_r import PSPModule
    _composite(cuda, PSPModule((1, 3, 6, 8)),
               lambda ctx, x: model_ref.psp(x, (1, 3, 6, 8)), [_x((2, 12, 21, 19), 4)], train,
               1e-6, 1e-6)


@pytest.mark.parametrize("which", ["retinaface_r", "mobilenetV3"])
@pytest.mark.parametrize("train", [True, False])
def test_eca_block_module(cuda, which, train):
    import importlib
    mod = importlib.import_module(f"nets.{which}")
    m = init_for_parity(mod.eca_block(80), seed=7)
    gate = "sigmoid" if which == "retinaface_r" else "hsigmoid"
    _composite(cuda, m, lambda ctx, x: model_ref.eca(ctx, x, "e", gate),
               [_x((3, 80, 10, 14), 5)], train, 1e-5, 1e-4, prefix="e.")


@pytest.mark.parametrize("train", [True, False])
def test_head_modules(cuda, train):
    from nets.retinaface_r import BboxHead, ClassHead, LandmarkHead
    for cls, k in ((ClassHead, 2), (BboxHead, 4), (LandmarkHead, 10)):
        m = init_for_parity(cls(40, 2), seed=k)

        def ref(ctx, x, k=k):
            o = ctx.conv(x, "conv1x1").permute(0, 2, 3, 1).contiguous()
            return o.view(o.shape[0], -1, k)
        _composite(cuda, m, ref, [_x((2, 40, 12, 10), k)], train, 1e-5, 1e-4)


# ----------------------------------------------------------------------------- backbones
def _stages(model_cls):
    import nets.mobilenetV3 as mv3
    L = [[(s[:4] + ("relu" if s[4] is nn.ReLU else "hswish",) + s[5:]) for s in layer]
         for layer in mv3.LARGE_ECA_LAYERS]
    if model_cls is mv3.MobileNetV3_Small:
        sm = [(s[:4] + ("relu" if s[4] is nn.ReLU else "hswish",) + s[5:])
              for s in mv3.SMALL_LAYERS]
        return [("bneck", [(s, "se" if s[5] else "none") for s in sm])]
    if model_cls is mv3.MobileNetV3_Large_eca:
        return [(f"layer{i + 1}", [(s, "eca") for s in layer]) for i, layer in enumerate(L)]
    if model_cls is mv3.MobileNetV3_Large_change:
        return [(f"layer{i + 1}", [(s, "se" if s[5] else "none") for s in layer])
                for i, layer in enumerate(L)]
    if model_cls is mv3.MobileNetV3_Large_ecaG:
        return [(f"layer{i + 1}", [(s, "beca" if (i, j) in mv3._ECAG_AT else "eca")
                                   for j, s in enumerate(layer)]) for i, layer in enumerate(L)]
    raise KeyError(model_cls)


@pytest.mark.parametrize("name", ["MobileNetV3_Small", "MobileNetV3_Large_eca",
                                  "MobileNetV3_Large_change", "MobileNetV3_Large_ecaG"])
def test_mobilenetv3_classifiers_eval(cuda, name):
    import nets.mobilenetV3 as mv3
    cls = getattr(mv3, name)
    m = init_for_parity(cls(num_classes=100), seed=13).eval()
    with torch.no_grad():
        m.bn3.running_var.uniform_(0.5, 1.5)
        m.linear3.weight.normal_(0, 960 ** -0.5)
        m.linear4.weight.normal_(0, 1280 ** -0.5)
    x = _x((2, 3, 96, 128), 14, 50.0)
    with torch.no_grad():
        ref = model_ref.mobilenetv3(_P(m, torch.float32, False), x, _stages(cls))
        got = m.to(cuda)(x.to(cuda))
    assert rel_err(got, ref) < 1e-3, rel_err(got, ref)


def test_mobilenetv1_stages(cuda):
    from nets.mobilenet025 import MobileNetV1
    m = init_for_parity(MobileNetV1(), seed=15).eval()
    x = _x((2, 3, 64, 96), 16, 50.0)
    P = _P(m, torch.float32, False)
    ctx = model_ref.Ctx(P)
    with torch.no_grad():
        r = x
        mg = m.to(cuda)
        g = x.to(cuda)
        for i, specs in enumerate(model_ref.MNV1_STAGES):
            r = model_ref.mobilenetv1_stage(ctx, r, f"stage{i + 1}", specs)
            g = getattr(mg, f"stage{i + 1}")(g)
            assert rel_err(g, r) < 1e-3, (i, rel_err(g, r))


def test_resnet50_classifier(cuda):
    from nets.resnet_pytorch_r import resnet50
    m = init_for_parity(resnet50(num_classes=10), seed=17).eval()
    with torch.no_grad():
        m.fc.weight.normal_(0, 2048 ** -0.5)
    x = _x((1, 3, 64, 64), 18, 50.0)
    with torch.no_grad():
        ref = model_ref.resnet_classifier(_P(m, torch.float32, False), x)
        got = m.to(cuda)(x.to(cuda))
    assert rel_err(got, ref) < 1e-3


# ----------------------------------------------------------------------------- inline detector
class _InlineRetinaFace(nn.Module):
    """The shape of the detectors the reference's scripts define inline
    (train_mobilenetV3_ecagai.py:319-435, train_50_3_r.py:145-244):
    IntermediateLayerGetter over the exported backbone, then the exported
    ECA / FPN / SSH / head modules composed in forward with plain torch
    glue (list(out.values()), torch.cat, F.softmax)."""

    def __init__(self, cfg, mode="train"):
        super().__init__()
        from nets._getter import IntermediateLayerGetter
        from nets.layers import SSH
        from nets.mobilenetV3 import MobileNetV3_Large_eca
        from nets.retinaface_r import FPN, BboxHead, ClassHead, LandmarkHead, eca_block
        self.body = IntermediateLayerGetter(MobileNetV3_Large_eca(), cfg["return_layers"])
        c, oc = cfg["in_channel"], cfg["out_channel"]
        self.fpn = FPN([c * 2, c * 4, c * 8], oc)
        self.ssh1, self.ssh2, self.ssh3 = SSH(oc, oc), SSH(oc, oc), SSH(oc, oc)
        self.ClassHead = nn.ModuleList([ClassHead(oc, 2) for _ in range(3)])
        self.BboxHead = nn.ModuleList([BboxHead(oc, 2) for _ in range(3)])
        self.LandmarkHead = nn.ModuleList([LandmarkHead(oc, 2) for _ in range(3)])
        self.eca_40, self.eca_80, self.eca_160 = eca_block(40), eca_block(80), eca_block(160)
        self.eca_fpn = eca_block(40)
        self.mode = mode

    def forward(self, inputs):
        out = list(self.body.forward(inputs).values())
        out = [self.eca_40(out[0]), self.eca_80(out[1]), self.eca_160(out[2])]
        fpn = self.fpn.forward(out)
        features = [self.ssh1(self.eca_fpn(fpn[0])), self.ssh2(self.eca_fpn(fpn[1])),
                    self.ssh3(self.eca_fpn(fpn[2]))]
        loc = torch.cat([self.BboxHead[i](f) for i, f in enumerate(features)], dim=1)
        conf = torch.cat([self.ClassHead[i](f) for i, f in enumerate(features)], dim=1)
        landm = torch.cat([self.LandmarkHead[i](f) for i, f in enumerate(features)], dim=1)
        if self.mode == "train":
            return loc, conf, landm
        return loc, torch.softmax(conf, dim=-1), landm


def test_inline_retinaface_forward(cuda):
    from utils.config import cfg_mnet
    m = init_for_parity(_InlineRetinaFace(cfg_mnet, mode="eval"), seed=19).eval()
    x = _x((2, 3, 128, 160), 20, 50.0)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    with torch.no_grad():
        ref = model_ref.retinaface_mnv3(sd, x, "eval")
        got = m.to(cuda)(x.to(cuda))
    for g, r in zip(got, ref):
        assert rel_err(g, r) < 1e-3


def test_inline_retinaface_gradients(cuda):
    """Training mode through the module surface: outputs, every parameter
    gradient and BN running statistic vs the oracle (same bar as the fused
    training path, tests/test_train.py)."""
    from test_train import _train_compare
    from utils.config import cfg_mnet
    m = init_for_parity(_InlineRetinaFace(cfg_mnet, mode="train"), seed=4)
    x = torch.randn(2, 3, 96, 96, generator=torch.Generator().manual_seed(1)) * 50
    _train_compare(m, model_ref.retinaface_mnv3, x, cuda)


# ----------------------------------------------------------------------------- DataParallel
def _replica_state(r, names):
    """state_dict-style view of a replicate()d module (replicas hold their
    parameters as plain attributes, not in _parameters)."""
    out = {}
    for n in names:
        obj = r
        for part in n.split("."):
            obj = getattr(obj, part)
        out[n] = obj.detach().clone().cpu()
    return out


def test_dataparallel_replica_uses_its_own_weights(cuda):
    """nn.DataParallel replicas share the original's __dict__ shallowly; each
    replica must run its own (broadcast) parameters (predict.py:109,
    train_mobilenetV3_ecagai.py:464), not a cached plan of the original."""
    from torch.nn.parallel import replicate
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="eval"), seed=21).eval().to(cuda)
    x = _x((1, 3, 64, 64), 22, 50.0).to(cuda)
    with torch.no_grad():
        base = m(x)                               # caches the original's plan
        r = replicate(m, [cuda])[0]
        for mod in r.modules():                   # the replica gets weights of its own
            for k in list(mod._former_parameters):
                setattr(mod, k, getattr(mod, k) * 1.01)
        out_rep = r(x)
        out_orig = m(x)
    for a, b in zip(out_orig, base):
        assert torch.equal(a, b)  # the original is untouched
    sd = _replica_state(r, list(m.state_dict()))
    ref = model_ref.retinaface_mnv3(sd, x.cpu(), "eval")
    for g, rr in zip(out_rep, ref):
        assert rel_err(g, rr) < 1e-3
    assert rel_err(out_rep[0], base[0]) > 1e-3  # and it really differs from the original's


def test_dataparallel_replica_training_grads_reach_original(cuda):
    """Training through a replicate()d module (DataParallel's path): gradients
    land on the original parameters, equal to running the original itself
    (parameters the forward never uses — the built-but-unused SeModules — get
    DataParallel's zero gradients, and none on the direct path)."""
    from torch.nn.parallel import replicate
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    x = _x((2, 3, 64, 64), 23, 50.0).to(cuda)
    grads = []
    for use_replica in (False, True):
        m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=24).to(cuda).train()
        run = replicate(m, [cuda])[0] if use_replica else m
        out = run(x)
        w = [torch.randn(o.shape, generator=torch.Generator().manual_seed(i)).to(cuda)
             for i, o in enumerate(out)]
        sum((o * ww).sum() for o, ww in zip(out, w)).backward()
        grads.append({k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    assert len(grads[0]) > 100
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k
    for k in set(grads[1]) - set(grads[0]):
        assert ".se." in k and float(grads[1][k].abs().max()) == 0.0, k


@pytest.mark.parametrize("hw", [(32, 48), (20, 24), (16, 16), (32, 32), (8, 8), (16, 24), (40, 40),
                                (32, 64)])
@pytest.mark.parametrize("cls,spec,gate", [b for b in BLOCKS if b[0] == "Block_eca"])
def test_mnv3_block_eca_wgrad_fused(cuda, cls, spec, gate, monkeypatch, hw):
    """Block_eca training (the fused MNv3BlockFn node) over eight map sizes
    (3x40x32x64 is where the 120-channel block has a BN2 output of 9.5e-8):
    the project conv's weight gradient and the ECA gate's sum(da * d) come
    from one GEMM over image-aligned pixel chunks (jabd_conv_wgrad_eca_f32,
    asserted below); every gradient against the mask-matched float64 oracle
    (_composite)."""
    import nets.mobilenetV3 as mv3
    from jabd_amd import train as T
    taken = []
    orig = T._wgrad_eca

    def spy(*a):
        r = orig(*a)
        taken.append(r is not None)
        return r

    monkeypatch.setattr(T, "_wgrad_eca", spy)
    k, cin, exp, cout, act, se, stride = spec
    act_cls = nn.ReLU if act == "relu" else nn.Hardswish
    m = init_for_parity(getattr(mv3, cls)(k, cin, exp, cout, act_cls, se, stride), seed=cin)
    _composite(cuda, m, lambda ctx, x: model_ref.block(ctx, x, "", spec, gate),
               [_x((3, cin) + hw, cin)], True)
    oh, ow = (hw[0] - 1) // stride + 1, (hw[1] - 1) // stride + 1
    # the one-GEMM form serves output maps of whole 64-pixel stages
    # (train.hip wgrad_eca_per); the others take the separate-pass backward
    assert taken and all(taken) == (oh * ow % 64 == 0), (taken, oh, ow)
