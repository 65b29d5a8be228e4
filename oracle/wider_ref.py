"""ORACLE (test infrastructure only) — utils/evaluation.py:45-63 (bbox_overlaps),
:255-287 (image_eval), :290-305 (img_pr_info) restated in numpy float64, summed
over images as evaluation() does (:347-375).  The reference ships no WIDER
ground truth or prediction files, so this is pinned by the hand-derived cases
in tests/test_wider_eval.py."""
import numpy as np


def overlaps(a, b):
    mx = np.minimum(a[:, None, 2:], b[None, :, 2:])
    mn = np.maximum(a[:, None, :2], b[None, :, :2])
    wh = np.maximum(mx - mn, 0)
    inter = wh[..., 0] * wh[..., 1]
    aa = ((a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1]))[:, None]
    bb = ((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]))[None, :]
    with np.errstate(divide="ignore", invalid="ignore"):
        return inter / (aa + bb - inter)


def image_eval(pred, gt, ignore, iou_thresh):
    p = pred.copy()
    g = gt.copy()
    p[:, 2] += p[:, 0]
    p[:, 3] += p[:, 1]
    g[:, 2] += g[:, 0]
    g[:, 3] += g[:, 1]
    ov = overlaps(p[:, :4], g)
    recall = np.zeros(len(g))
    prop = np.ones(len(p))
    pred_recall = np.zeros(len(p))
    for h in range(len(p)):
        mo, mi = ov[h].max(), ov[h].argmax()
        if mo >= iou_thresh:
            if ignore[mi] == 0:
                recall[mi] = -1
                prop[h] = -1
            elif recall[mi] == 0:
                recall[mi] = 1
        pred_recall[h] = np.count_nonzero(recall == 1)
    return pred_recall, prop


def img_pr_info(thresh_num, pred, prop, pred_recall):
    pr = np.zeros((thresh_num, 2))
    for t in range(thresh_num):
        thresh = 1 - (t + 1) / thresh_num
        idx = np.where(pred[:, 4] >= thresh)[0]
        if len(idx):
            r = idx[-1]
            pr[t, 0] = np.count_nonzero(prop[:r + 1] == 1)
            pr[t, 1] = pred_recall[r]
    return pr


def pr_curve(preds, gts, ignores, iou_thresh=0.5, thresh_num=1000):
    out = np.zeros((thresh_num, 2))
    for p, g, ig in zip(preds, gts, ignores):
        if len(p) == 0 or len(g) == 0:
            continue
        rec, prop = image_eval(np.asarray(p, np.float64), np.asarray(g, np.float64), ig,
                               iou_thresh)
        out += img_pr_info(thresh_num, np.asarray(p, np.float64), prop, rec)
    return out
