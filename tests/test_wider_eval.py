"""§8f rank 3: WIDER FACE evaluation core (utils/evaluation.py:255-305 summed
over images) on the device vs the numpy oracle (oracle/wider_ref.py).  The
reference ships no WIDER files; the oracle is pinned by the hand cases below.
GPU parity is exact: the pr curve holds integer counts."""
import numpy as np
import pytest

from oracle import wider_ref


def test_wider_oracle_kat():
    gt = np.array([[0, 0, 10, 10], [100, 100, 10, 10]], np.float64)
    pred = np.array([[0, 0, 10, 10, 0.95],      # IoU 1 with gt 0 (kept) -> recalled
                     [50, 50, 10, 10, 0.55],    # no overlap -> a false proposal
                     [100, 100, 10, 10, 0.15]]) # IoU 1 with gt 1 (ignored) -> not a proposal
    rec, prop = wider_ref.image_eval(pred, gt, np.array([1, 0]), 0.5)
    assert rec.tolist() == [1, 1, 1] and prop.tolist() == [1, 1, -1]
    pr = wider_ref.img_pr_info(10, pred, prop, rec)
    assert pr[0].tolist() == [1, 1]      # thresh 0.9: first pred only
    assert pr[4].tolist() == [2, 1]      # thresh 0.5: two proposals, one face
    assert pr[9].tolist() == [2, 1]      # thresh 0.0: the ignored hit is no proposal


def test_voc_ap_kat():
    from utils.evaluation import voc_ap
    assert voc_ap(np.array([0.5, 1.0]), np.array([1.0, 0.5])) == pytest.approx(0.75)


def _synth(n_img, seed):
    g = np.random.default_rng(seed)
    preds, gts, igs = [], [], []
    for i in range(n_img):
        m = int(g.integers(0, 20))
        gt = np.c_[g.uniform(0, 200, (m, 2)), g.uniform(4, 40, (m, 2))]
        n = int(g.integers(0, 40))
        src = gt[g.integers(0, max(m, 1), n)] if m else np.zeros((n, 4))
        pr = src + g.normal(0, 3, (n, 4))
        pr[: n // 4, :2] = g.uniform(0, 200, (n // 4, 2))
        scores = np.sort(g.uniform(0, 1, n))[::-1]
        preds.append(np.c_[pr, scores])
        gts.append(gt)
        igs.append((g.uniform(0, 1, m) < 0.7).astype(np.uint8))
    return preds, gts, igs


@pytest.mark.gpu
@pytest.mark.parametrize("iou", [0.5, 0.3])
def test_wider_pr_curve_parity(cuda, iou):
    from jabd_amd import ops
    preds, gts, igs = _synth(60, 7)
    got = ops.wider_pr_curve(preds, gts, igs, iou, 1000, device=cuda).cpu().numpy()
    ref = wider_ref.pr_curve(preds, gts, igs, iou, 1000)
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_setting_ap(cuda):
    from utils.evaluation import dataset_pr_info, setting_ap, voc_ap
    preds, gts, igs = _synth(40, 8)
    keeps = [np.nonzero(ig)[0] + 1 for ig in igs]
    ap = setting_ap(preds, gts, keeps)
    ref = wider_ref.pr_curve(preds, gts, igs, 0.5, 1000)
    curve = dataset_pr_info(1000, ref, sum(len(k) for k in keeps))
    assert ap == voc_ap(curve[:, 1], curve[:, 0])
    assert 0.0 < ap <= 1.0
