"""A4: the fused SSH tail + heads kernel (csrc/ssh.hip) against the unfused
launches (the 10-channel SSH GEMMs + heads_kernel) and against the oracle, on
the MobileNetV3 detector's levels — ragged tiles (level widths not a multiple
of the 8 x 32 tile), several images, eval softmax on and off."""
import pytest
import torch

from _util import init_for_parity, rel_err


def _run(m, x, fused):
    from jabd_amd import engine, hipmodule
    prev = engine.SSH_TAIL
    engine.SSH_TAIL = fused
    hipmodule.invalidate()
    try:
        with torch.no_grad():
            return [t.clone() for t in m(x)]
    finally:
        engine.SSH_TAIL = prev
        hipmodule.invalidate()


@pytest.mark.gpu
@pytest.mark.parametrize("bhw", [(2, 96, 160), (3, 200, 136), (1, 640, 640)])
def test_ssh_tail_matches_unfused(cuda, bhw):
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    B, H, W = bhw
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="eval"), seed=3).eval().to(cuda)
    g = torch.Generator().manual_seed(H + W)
    x = torch.randn(B, 3, H, W, generator=g).to(cuda)
    a = _run(m, x, True)
    b = _run(m, x, False)
    for got, ref in zip(a, b):
        assert got.shape == ref.shape
        assert rel_err(got, ref) < 2e-5, rel_err(got, ref)


@pytest.mark.gpu
def test_ssh_tail_vs_oracle_train_mode_logits(cuda):
    """mode='train' (no softmax) through the fused tail vs the oracle."""
    from oracle import model_ref
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=4).eval()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 3, 128, 96, generator=g)
    with torch.no_grad():
        ref = model_ref.retinaface_mnv3(sd, x, "train")
        got = _run(m.to(cuda), x.to(cuda), True)
    for gg, r in zip(got, ref):
        assert rel_err(gg, r) < 1e-3
