"""Golden vectors (tests/golden/box_ops_golden.npz, made by
tests/golden/make_golden.py): the CPU tests re-derive them from the oracle
(pinning it against drift; the anchor count is the reference's own KAT), the
GPU tests check the HIP path against the committed expected outputs with the
same bars as the parity tests (bit-exact indices/assignments)."""
import os

import numpy as np
import pytest
import torch

from oracle import box_ref

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "box_ops_golden.npz"))
CFG = {"min_sizes": [[16, 32], [64, 128], [256, 512]], "steps": [8, 16, 32], "clip": False}


def _targets():
    return [torch.from_numpy(G["match_targets0"]), torch.from_numpy(G["match_targets1"])]


# ---------------------------------------------------------------- CPU: oracle vs fixture
def test_golden_anchors():
    np.testing.assert_array_equal(box_ref.anchors(CFG, (256, 256)).numpy(), G["anchors_256"])
    assert int(G["anchor_count_840_ref_kat"]) == 29518  # utils/anchors.py:104-105


@pytest.mark.parametrize("i", [0, 1, 2])
def test_golden_nms_oracle(i):
    keep = box_ref.nms(G[f"nms{i}_boxes"], G[f"nms{i}_scores"], float(G[f"nms{i}_thr"]))
    np.testing.assert_array_equal(keep, G[f"nms{i}_keep"])


def test_golden_match_and_loss_oracle():
    pri = box_ref.anchors(CFG, (128, 128))
    lt, ct, lmt = box_ref.match_batch(_targets(), pri)
    np.testing.assert_array_equal(ct.numpy(), G["match_conf_t"])
    np.testing.assert_array_equal(lt.numpy(), G["match_loc_t"])
    np.testing.assert_array_equal(lmt.numpy(), G["match_landm_t"])
    rl, rc, rlm, info = box_ref.multibox_loss(torch.from_numpy(G["loss_loc"]),
                                              torch.from_numpy(G["loss_conf"]),
                                              torch.from_numpy(G["loss_landm"]), lt, ct, lmt)
    np.testing.assert_allclose([float(rl), float(rc), float(rlm)], G["loss_values"], rtol=1e-6)
    assert tuple(info["counts"]) == tuple(G["loss_counts"])


# ---------------------------------------------------------------- GPU: HIP vs fixture
@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 1, 2])
def test_golden_nms_hip(cuda, i):
    from jabd_amd import ops
    keep = ops.nms(torch.from_numpy(G[f"nms{i}_boxes"]).to(cuda),
                   torch.from_numpy(G[f"nms{i}_scores"]).to(cuda), float(G[f"nms{i}_thr"]))
    np.testing.assert_array_equal(keep.cpu().numpy(), G[f"nms{i}_keep"])


@pytest.mark.gpu
def test_golden_match_and_loss_hip(cuda):
    from nets.retinaface_training import MultiBoxLoss
    from jabd_amd import ops
    pri = box_ref.anchors(CFG, (128, 128)).to(cuda)
    tg = [t.to(cuda) for t in _targets()]
    gl, gc, glm = ops.match_encode(tg, pri, 0.35, [0.1, 0.2])
    np.testing.assert_array_equal(gc.cpu().numpy(), G["match_conf_t"])
    np.testing.assert_allclose(gl.cpu().numpy(), G["match_loc_t"], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(glm.cpu().numpy(), G["match_landm_t"])
    crit = MultiBoxLoss(2, 0.35, 7, [0.1, 0.2], True)
    preds = tuple(torch.from_numpy(G[k]).to(cuda) for k in ("loss_loc", "loss_conf", "loss_landm"))
    l, c, lm = crit(preds, pri, tg)
    np.testing.assert_allclose([float(l), float(c), float(lm)], G["loss_values"], rtol=1e-5)


@pytest.mark.gpu
def test_golden_decode_hip(cuda):
    from jabd_amd import ops
    pri = box_ref.anchors(CFG, (128, 128)).to(cuda)
    loc = torch.from_numpy(G["loss_loc"][0]).to(cuda)
    landm = torch.from_numpy(G["loss_landm"][0]).to(cuda)
    # exp() may differ by an ulp between HIP and the CPU library (as in test_decode_parity)
    np.testing.assert_allclose(ops.decode(loc, pri, [0.1, 0.2]).cpu().numpy(), G["decode_boxes"],
                               rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(ops.decode_landm(landm, pri, [0.1, 0.2]).cpu().numpy(),
                                  G["decode_landms"])
