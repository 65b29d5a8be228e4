"""JABD-MobileNetV3-BECA (train_mobilenetV3_ecagai.py:161-435, the §8f "next"
variant): BECA gates, bicubic(align_corners) FPN, NLM(40) with ch=40 and
PSP (1, 3, 6, 8).

CPU: the module's state_dict carries the script's keys and the oracle
(oracle/model_ref.retinaface_mnv3_beca) consumes exactly them.
GPU: the ch=40 attention core (nlm_attn.hip) forward and backward, the
standalone NLM / FPN modules, and the whole detector in eval (fused plan)
and training (every parameter gradient) against the oracle — the bars of
test_model.py (logits 1e-3 of max|ref|) and test_train.py (per-tensor
relative Frobenius error <= max(2e-3, 4x the oracle's fp32 error) vs fp64).
"""
import pytest
import torch

from _util import elem_rel_err, init_for_parity, rel_err
from oracle import model_ref

TOL = 1e-3


def _model(mode="eval", seed=21):
    from nets.retinaface_beca import RetinaFace
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode=mode), seed=seed)
    return m.eval() if mode == "eval" else m


def test_beca_state_dict_layout():
    m = _model()
    sd = m.state_dict()
    for k in ("fpn.nlm.f_query.weight", "fpn.nlm.W.bias", "eca_40.conv.weight",
              "eca_fpn.conv.weight", "ssh2.conv5X5_1.1.running_mean", "LandmarkHead.1.conv1x1.bias",
              "body.layer3.4.eca.conv.weight"):
        assert k in sd, k
    assert sd["fpn.nlm.f_query.weight"].shape == (40, 40, 1, 1)
    assert m.fpn.nlm.psp.sizes == (1, 3, 6, 8)
    assert sum(s * s for s in m.fpn.nlm.psp.sizes) == 110
    with torch.no_grad():
        loc, conf, landm = model_ref.retinaface_mnv3_beca(sd, torch.randn(1, 3, 64, 64))
    assert loc.shape == (1, 2 * (8 * 8 + 4 * 4 + 2 * 2), 4)
    assert conf.shape[-1] == 2 and landm.shape[-1] == 10


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 40, 16, 16), (3, 40, 23, 17), (1, 40, 48, 50)])
def test_nlm40_forward_and_gradients(cuda, shape):
    """NLM(40).forward alone (eval: fused pack; training: NlmAttnFn graph) vs the
    oracle's NLM (nets/retinaface_r.py:124-152 = script :208-234)."""
    from nets.retinaface_beca import NLM
    g = torch.Generator().manual_seed(7)
    m = init_for_parity(NLM(40), seed=3)
    x = torch.randn(shape, generator=g)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    # eval forward vs fp32 oracle
    with torch.no_grad():
        ref = model_ref.nlm(model_ref.Ctx(sd), x, "", (1, 3, 6, 8))
    mg = m.to(cuda).eval()
    with torch.no_grad():
        got = mg(x.to(cuda))
    assert rel_err(got, ref) < 1e-5, rel_err(got, ref)
    # gradients vs fp64 autograd through the oracle
    P = {k: v.double().requires_grad_(True) for k, v in sd.items()}
    x64 = x.double().requires_grad_(True)
    w = torch.randn(shape, generator=g)
    (model_ref.nlm(model_ref.Ctx(P), x64, "", (1, 3, 6, 8)) * w.double()).sum().backward()
    mg.train()
    xg = x.to(cuda).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    out = mg(xg)
    (out * w.to(cuda)).sum().backward()
    assert rel_err(out.detach(), ref) < 1e-5
    assert rel_err(xg.grad, x64.grad) < 1e-5, rel_err(xg.grad, x64.grad)
    named = dict(mg.named_parameters())
    gmax = max(float(p.grad.abs().max()) for p in P.values())
    for k, p in P.items():
        if k.endswith("f_key.bias"):  # softmax-invariant: analytically zero
            assert float(named[k].grad.abs().max()) <= 1e-5 * gmax
            continue
        e = rel_err(named[k].grad, p.grad)
        assert e < 1e-4, (k, e)


@pytest.mark.gpu
@pytest.mark.parametrize("B,P,S,ch", [(1, 1, 1, 8), (2, 391, 110, 40), (3, 2048, 110, 40),
                                      (2, 5001, 17, 64), (1, 4097, 33, 20), (4, 64, 110, 12)])
def test_nlm_attn_dkv_kernel(cuda, B, P, S, ch):
    """dK = dS . q, dV = P . dctx (nlm_attn.hip dkv kernels) vs fp64 bmm: chunk
    boundaries (P over 2048), ragged P, S not a multiple of 16, ch tiles."""
    import ctypes
    from jabd_amd._lib import call, lib
    g = torch.Generator().manual_seed(P + S + ch)
    dsm, pm = torch.randn(B, S, P, generator=g), torch.rand(B, S, P, generator=g)
    q, dctx = torch.randn(B, P, ch, generator=g), torch.randn(B, P, ch, generator=g)
    ref_k, ref_v = (torch.bmm(a.double(), x.double()) for a, x in ((dsm, q), (pm, dctx)))
    nws = int(lib().jabd_nlm_attn_dkv_ws_floats(B, P, S, ch))
    t = [v.to(cuda).contiguous() for v in (dsm, pm, q, dctx)]
    ws = torch.empty(nws, device=cuda)
    dk = torch.full((B, S, ch), float("nan"), device=cuda)
    dv = torch.full((B, S, ch), float("nan"), device=cuda)
    call("jabd_nlm_attn_dkv_f32", *(v.data_ptr() for v in t), B, P, S, ch, ws.data_ptr(), nws,
         dk.data_ptr(), dv.data_ptr(), None)
    torch.cuda.synchronize()
    # fp32 accumulation over P terms: |err| <= ~P * eps * sum|a x|, bar 1e-5 of max
    assert rel_err(dk, ref_k) < 1e-5, rel_err(dk, ref_k)
    assert rel_err(dv, ref_v) < 1e-5, rel_err(dv, ref_v)
    with pytest.raises(RuntimeError):
        call("jabd_nlm_attn_dkv_f32", *(v.data_ptr() for v in t), B, P, S, ch, ws.data_ptr(),
             nws - 1, dk.data_ptr(), dv.data_ptr(), None)


@pytest.mark.gpu
def test_bicubic_fpn_module_parity(cuda):
    """FPN (bicubic + NLM(40)) as a standalone module, eval and training forward."""
    from nets.retinaface_beca import FPN
    g = torch.Generator().manual_seed(9)
    m = init_for_parity(FPN([40, 80, 160], 40), seed=5).eval()
    feats = [torch.randn(2, c, s, s, generator=g) for c, s in ((40, 24), (80, 12), (160, 6))]
    sd = {"fpn." + k: v.clone() for k, v in m.state_dict().items()}
    with torch.no_grad():
        ref = model_ref.fpn(model_ref.Ctx(sd), feats, 0.1, "fpn.nlm.", sizes=(1, 3, 6, 8),
                            up="bicubic")
    mg = m.to(cuda)
    with torch.no_grad():
        got = mg([f.to(cuda) for f in feats])
    for a, b in zip(got, ref):
        assert rel_err(a, b) < 1e-5, rel_err(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,mode", [((2, 128, 128), "eval"), ((1, 96, 160), "train"),
                                        ((1, 104, 136), "eval")])
def test_beca_detector_forward_parity(cuda, shape, mode):
    m = _model()
    B, H, W = shape
    x = torch.randn(B, 3, H, W, generator=torch.Generator().manual_seed(H + W)) * 50
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    with torch.no_grad():
        ref = model_ref.retinaface_mnv3_beca(sd, x, mode)
    m.mode = mode
    mg = m.to(cuda)
    with torch.no_grad():
        got = mg(x.to(cuda))
    for g_, r, name in zip(got, ref, ("loc", "conf", "landm")):
        assert g_.shape == r.shape, name
        e = rel_err(g_, r)
        print(f"{name}: max-norm rel {e:.2e}, elementwise {elem_rel_err(g_, r):.2e}")
        assert e < TOL, f"{name}: rel err {e:.2e}"


@pytest.mark.gpu
def test_beca_detector_training_parity(cuda):
    """Training-mode forward + backward of the whole BECA detector (batch-stat
    BN, BECA gates through BecaFn, bicubic + NLM(40) through UpsampleFn /
    NlmAttnFn) against fp64 autograd through the oracle."""
    from test_train import _train_compare
    m = _model(mode="train", seed=22)
    x = torch.randn(2, 3, 96, 96, generator=torch.Generator().manual_seed(4)) * 50
    _train_compare(m, model_ref.retinaface_mnv3_beca, x, cuda)


# ----------------------------------------------------------------------------- MobileNetV3_Small
def _small(mode="eval", seed=31):
    from nets.retinaface_r import RetinaFace_Small
    from utils.config import cfg_mnv3_small
    m = init_for_parity(RetinaFace_Small(cfg=cfg_mnv3_small, mode=mode), seed=seed)
    return m.eval() if mode == "eval" else m


def test_small_detector_layout():
    """BASELINE config 1's MobileNetV3-small + ECA head: the classifier's keys
    under body., taps at strides 8/16/32, the cfg_mnet anchor count."""
    from utils.anchors import Anchors
    from utils.config import cfg_mnv3_small
    m = _small()
    sd = m.state_dict()
    for k in ("body.conv1.weight", "body.bneck.0.se.se.1.weight", "body.bneck.10.bn3.running_var",
              "fpn.output1.0.weight", "eca_24.conv.weight", "eca_96.conv.weight"):
        assert k in sd, k
    assert sd["fpn.output1.0.weight"].shape[1] == 24 and sd["fpn.output3.0.weight"].shape[1] == 96
    with torch.no_grad():
        loc, conf, landm = model_ref.retinaface_mnv3_small(sd, torch.randn(1, 3, 640, 640))
    assert loc.shape[1] == Anchors(cfg_mnv3_small, image_size=(640, 640)).get_anchors().shape[0]


@pytest.mark.gpu
@pytest.mark.parametrize("shape,mode", [((1, 640, 640), "eval"), ((2, 96, 160), "train")])
def test_small_detector_forward_parity(cuda, shape, mode):
    m = _small()
    B, H, W = shape
    x = torch.randn(B, 3, H, W, generator=torch.Generator().manual_seed(H)) * 50
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    with torch.no_grad():
        ref = model_ref.retinaface_mnv3_small(sd, x, mode)
    m.mode = mode
    mg = m.to(cuda)
    with torch.no_grad():
        got = mg(x.to(cuda))
    for g_, r, name in zip(got, ref, ("loc", "conf", "landm")):
        e = rel_err(g_, r)
        print(f"{name}: max-norm rel {e:.2e}, elementwise {elem_rel_err(g_, r):.2e}")
        assert e < TOL, f"{name}: rel err {e:.2e}"


@pytest.mark.gpu
def test_small_detector_training_parity(cuda):
    from test_train import _train_compare
    m = _small(mode="train", seed=32)
    x = torch.randn(2, 3, 96, 96, generator=torch.Generator().manual_seed(6)) * 50
    _train_compare(m, model_ref.retinaface_mnv3_small, x, cuda)
