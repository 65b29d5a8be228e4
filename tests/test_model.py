"""A1-A5 detector forward: product modules vs the oracle restatement.

CPU: the product modules carry the reference's state_dict layout (the
oracle, written from the reference text, finds every weight it needs).
GPU: eval-mode forward of the fused HIP plan against the oracle in fp32
(tolerance: max-abs error <= 1e-3 of the output's max magnitude, per
north-star "logits within 1e-3 relative fp32").
"""
import pytest
import torch

from _util import elem_rel_err, init_for_parity, rel_err
from oracle import model_ref

TOL = 1e-3


def _mnv3():
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    return init_for_parity(RetinaFace(cfg=cfg_mnet, mode="eval"), seed=1).eval()


def _r50():
    from nets.retinaface_eca_nonlocal import RetinaFace
    from utils.config import cfg_re50
    return init_for_parity(RetinaFace(cfg=cfg_re50, mode="eval"), seed=2).eval()


def test_mnv3_state_dict_layout():
    m = _mnv3()
    sd = m.state_dict()
    for k in ("body.conv1.weight", "body.layer1.0.conv1.weight", "body.layer1.3.se.se.1.weight",
              "body.layer1.3.skip.2.bias", "body.layer3.4.eca.conv.weight",
              "fpn.nlm.f_query.weight", "fpn.nlm.W.bias", "ssh3.conv7x7_3.1.running_var",
              "ClassHead.2.conv1x1.bias", "eca_fpn.conv.weight", "eca_160.conv.weight"):
        assert k in sd, k
    assert not any(k.startswith("body.conv2") or k.startswith("body.linear") for k in sd)
    with torch.no_grad():  # the oracle consumes exactly these keys
        loc, conf, landm = model_ref.retinaface_mnv3(sd, torch.randn(1, 3, 64, 64))
    assert loc.shape == (1, 2 * (8 * 8 + 4 * 4 + 2 * 2), 4)
    assert conf.shape[-1] == 2 and landm.shape[-1] == 10


def test_r50_state_dict_layout():
    m = _r50()
    sd = m.state_dict()
    for k in ("body.layer2.0.downsample.0.weight", "body.layer4.2.bn3.running_mean",
              "fpn.Nlm.f_key.bias", "Nlm.W.weight", "IouHead.2.conv1x1.weight",
              "eca_256.conv.weight"):
        assert k in sd, k
    assert sd["eca_256.conv.weight"].shape[-1] == 7
    with torch.no_grad():
        loc, _, _ = model_ref.retinaface_r50(sd, torch.randn(1, 3, 64, 64))
    assert loc.shape == (1, 2 * (8 * 8 + 4 * 4 + 2 * 2), 4)


def _compare(model, fn, x, cuda, mode, elem_tol=None):
    """Max-norm bar (north-star 1e-3) on every output; with elem_tol also an
    elementwise bar |got - ref| / max(|ref|, 1e-2 * max|ref|) <= elem_tol, so
    small logits are bounded individually and not only relative to the largest."""
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = fn(sd, x, mode)
    model.mode = mode
    mg = model.to(cuda)
    with torch.no_grad():
        got = mg(x.to(cuda))
    for g, r, name in zip(got, ref, ("loc", "conf", "landm")):
        assert g.shape == r.shape, name
        e = rel_err(g, r)
        ee = elem_rel_err(g, r)
        print(f"{name}: max-norm rel {e:.2e}, elementwise rel (1e-2 floor) {ee:.2e}")
        assert e < TOL, f"{name}: rel err {e:.2e}"
        if elem_tol is not None:
            assert ee < elem_tol, f"{name}: elementwise rel err {ee:.2e}"


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 128, 128), (1, 96, 160), (1, 104, 136)])
@pytest.mark.parametrize("mode", ["eval", "train"])
def test_mnv3_forward_parity(cuda, shape, mode):
    B, H, W = shape
    x = torch.randn(B, 3, H, W, generator=torch.Generator().manual_seed(H)) * 50
    _compare(_mnv3(), model_ref.retinaface_mnv3, x, cuda, mode)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1, 128, 128), (2, 96, 160)])
def test_r50_forward_parity(cuda, shape):
    B, H, W = shape
    x = torch.randn(B, 3, H, W, generator=torch.Generator().manual_seed(W)) * 50
    _compare(_r50(), model_ref.retinaface_r50, x, cuda, "eval")


@pytest.mark.gpu
def test_mnv3_forward_parity_c2_full_size(cuda):
    """C2's shape at bs1: 1024x1024 (BASELINE configs[1]).  Exercises what the
    small cases do not: 512x512 expand+depthwise tiles, the two-level ECA
    partial reduce over > 64 tile partials and the large-M conv32 paths."""
    from jabd_amd import synth
    x = synth.images(1, 1024, seed=1234)
    _compare(_mnv3(), model_ref.retinaface_mnv3, x, cuda, "eval", elem_tol=1e-2)


@pytest.mark.gpu
def test_r50_forward_parity_full_size(cuda):
    """C3's model (R50 RetinaFace + ECA/NLM head) at 1024x1024, bs1."""
    from jabd_amd import synth
    x = synth.images(1, 1024, seed=4321)
    _compare(_r50(), model_ref.retinaface_r50, x, cuda, "eval", elem_tol=1e-2)


@pytest.mark.gpu
def test_mnv3_eval_stream_split(cuda):
    """Engine.run with EVAL_STREAMS = 2 splits a batch of >= EVAL_SPLIT_MIN
    images over two HIP streams: the outputs equal the one-stream forward's,
    image by image (every op is per image), and the oracle's."""
    from jabd_amd import engine as E
    m = _mnv3().to(cuda)
    x = torch.randn(9, 3, 96, 128, generator=torch.Generator().manual_seed(3)) * 60
    xg = x.to(cuda)
    assert x.shape[0] >= E.EVAL_SPLIT_MIN
    saved = E.EVAL_STREAMS
    with torch.no_grad():
        try:
            E.EVAL_STREAMS = 2
            split = [t.clone() for t in m(xg)]
            E.EVAL_STREAMS = 1
            one = m(xg)
        finally:
            E.EVAL_STREAMS = saved
    eng = m._jabd_cached(xg.device, None, tag="engine")
    assert eng.split_ok
    for a, b in zip(split, one):
        assert a.shape == b.shape
        assert torch.equal(a, b)
    ref = model_ref.retinaface_mnv3({k: v.cpu() for k, v in m.state_dict().items()}, x)
    for a, r in zip(split, ref):
        assert rel_err(a.cpu(), r) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("kind,B", [("mnv3", 32), ("r50", 64)])
def test_benchmarked_batch_last_image(cuda, kind, B):
    """The benchmarked batches at 1024x1024 (C2: JABD-MobileNetV3 bs32; C3's
    model: R50 RetinaFace bs64, whose layer1 activations are [64,256,256,256]
    = 1.07e9 elements): images 0 and B-1 of the full batch equal bs1 runs of
    the same images bit for bit (per-image batch strides, no cross-image
    mixing) with split-K off (functional.split_k, off by default); with it on
    (the bs1 predict path: the R50's bs1 3x3 convs split their K sum over
    workgroups, conv32.hip m32_ksplit)
    the bs1 outputs differ only in fp32 rounding: each within the oracle bar,
    and apart by no more than their two oracle errors.  Image B-1 matches the
    oracle (nets/retinaface_r.py:304-343,
    nets/retinaface_eca_nonlocal.py:314-359)."""
    model, fn = (_mnv3(), model_ref.retinaface_mnv3) if kind == "mnv3" else \
        (_r50(), model_ref.retinaface_r50)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    mg = model.to(cuda)
    gen = torch.Generator(device=cuda).manual_seed(77)
    x = torch.rand((B, 3, 1024, 1024), generator=gen, device=cuda) * 255.0 - 117.0
    from jabd_amd import functional as JF
    assert not JF.ksplit_enabled()  # batched eval is batch-invariant by default
    with torch.no_grad():
        full = [t.clone() for t in mg(x)]
        with JF.split_k():
            split = [t.clone() for t in mg(x[B - 1:B].contiguous())]
        for i in (0, B - 1):
            one = mg(x[i:i + 1].contiguous())
            for f, o, name in zip(full, one, ("loc", "conf", "landm")):
                assert torch.equal(f[i:i + 1], o), (i, name, rel_err(f[i:i + 1], o))
        ref = fn(sd, x[B - 1:B].cpu(), "eval")
    for f, s, r, name in zip(full, split, ref, ("loc", "conf", "landm")):
        e, es, d = rel_err(f[B - 1:B], r), rel_err(s, r), rel_err(s, f[B - 1:B])
        print(f"{kind} image {B - 1} vs oracle: {name} rel {e:.2e}; bs1 split-K {es:.2e},"
              f" split-K vs batch {d:.2e}")
        assert e < TOL and es < TOL, (name, e, es)
        assert d <= e + es + 1e-6, (name, d, e, es)


@pytest.mark.gpu
def test_eval_batch_chunks(cuda, monkeypatch):
    """Batches whose activations would pass 2^31 elements run in image chunks
    (engine.CHUNK_ELEMS; 32-bit kernel offsets): forced here at 5 x 64x96
    with 2-image chunks, the outputs equal the one-pass forward bit for bit."""
    from jabd_amd import engine as E
    for model in (_mnv3(), _r50()):
        m = model.to(cuda)
        x = (torch.randn(5, 3, 64, 96, generator=torch.Generator().manual_seed(9)) * 50).to(cuda)
        with torch.no_grad():
            one = [t.clone() for t in m(x)]
            monkeypatch.setattr(E, "CHUNK_ELEMS", 2 * 16 * 64 * 96)
            chunked = m(x)
            monkeypatch.setattr(E, "CHUNK_ELEMS", (1 << 31) - 1)
        for a, b in zip(one, chunked):
            assert torch.equal(a, b)
