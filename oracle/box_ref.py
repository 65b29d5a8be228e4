"""ORACLE (test infrastructure only) — anchors, matching, encoding, decoding,
MultiBoxLoss and NMS restated on the CPU.

Each function cites the reference text it restates (paths relative to
/root/reference/JABD2080ti).  Tensor ops are PyTorch-CPU fp32, issued one
reference op at a time so every intermediate rounds as the reference's does.
"""
import ctypes
import itertools
import math
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


# ----------------------------------------------------------------------------- anchors
def anchors(cfg, image_size):
    """utils/anchors.py:8-42 (Anchors.get_anchors).

    Feature map k is ceil(H/step_k) x ceil(W/step_k); priors are emitted level
    -> row i -> column j -> min_size, each (cx, cy, w, h) normalised, computed
    in Python double and converted to fp32 at the end (torch.Tensor(list)).
    """
    H, W = image_size[0], image_size[1]
    out = []
    for k, step in enumerate(cfg["steps"]):
        fh, fw = math.ceil(H / step), math.ceil(W / step)
        for i, j in itertools.product(range(fh), range(fw)):
            for m in cfg["min_sizes"][k]:
                out.extend([(j + 0.5) * step / W, (i + 0.5) * step / H, m / W, m / H])
    t = torch.tensor(out, dtype=torch.float64).to(torch.float32).view(-1, 4)
    if cfg.get("clip", False):
        t.clamp_(min=0, max=1)
    return t


def num_anchors(cfg, image_size):
    H, W = image_size
    return sum(math.ceil(H / s) * math.ceil(W / s) * len(m)
               for s, m in zip(cfg["steps"], cfg["min_sizes"]))


# ----------------------------------------------------------------------------- IoU
def point_form(p):
    """nets/retinaface_training.py:8-10 — (cx,cy,w,h) -> (x1,y1,x2,y2)."""
    half = p[:, 2:] / 2
    return torch.cat((p[:, :2] - half, p[:, :2] + half), 1)


def jaccard(a, b):
    """nets/retinaface_training.py:22-59 — pairwise IoU [len(a), len(b)]."""
    hi = torch.min(a[:, None, 2:].expand(-1, b.shape[0], 2), b[None, :, 2:].expand(a.shape[0], -1, 2))
    lo = torch.max(a[:, None, :2].expand(-1, b.shape[0], 2), b[None, :, :2].expand(a.shape[0], -1, 2))
    wh = torch.clamp(hi - lo, min=0)
    inter = wh[:, :, 0] * wh[:, :, 1]
    area_a = ((a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1]))[:, None]
    area_b = ((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]))[None, :]
    return inter / (area_a + area_b - inter)


# ----------------------------------------------------------------------------- encode
def encode(matched, priors, var):
    """nets/retinaface_training.py:62-73."""
    c = (matched[:, :2] + matched[:, 2:]) / 2 - priors[:, :2]
    c = c / (var[0] * priors[:, 2:])
    wh = (matched[:, 2:] - matched[:, :2]) / priors[:, 2:]
    wh = torch.log(wh) / var[1]
    return torch.cat([c, wh], 1)


def encode_landm(matched, priors, var):
    """nets/retinaface_training.py:75-86."""
    m = matched.reshape(-1, 5, 2)
    d = (m - priors[:, None, :2]) / (var[0] * priors[:, None, 2:])
    return d.reshape(-1, 10)


def match(threshold, truths, priors, var, labels, landms):
    """nets/retinaface_training.py:93-162 for one image.

    Returns (loc [A,4], conf [A] int64, landm [A,10], best_truth_idx [A],
    best_truth_overlap [A]).
    """
    ov = jaccard(truths, point_form(priors))
    _, best_prior = ov.max(1)                 # per truth, first index on ties
    bto, bti = ov.max(0)                      # per prior
    bto = bto.clone()
    bti = bti.clone()
    bto.index_fill_(0, best_prior, 2)
    for j in range(best_prior.shape[0]):      # sequential: the last j wins
        bti[best_prior[j]] = j
    conf = labels[bti].clone()
    conf[bto < threshold] = 0
    loc = encode(truths[bti], priors, var)
    landm = encode_landm(landms[bti], priors, var)
    return loc, conf.to(torch.int64), landm, bti, bto


def match_batch(targets, priors, threshold=0.35, var=(0.1, 0.2)):
    """MultiBoxLoss.forward's per-image loop (nets/retinaface_training.py:201-214)."""
    locs, confs, landms = [], [], []
    for t in targets:
        loc, conf, landm, _, _ = match(threshold, t[:, :4], priors, var, t[:, -1], t[:, 4:14])
        locs.append(loc)
        confs.append(conf)
        landms.append(landm)
    return torch.stack(locs), torch.stack(confs), torch.stack(landms)


def match_iou_batch(targets, priors, threshold=0.35, var=(0.1, 0.2)):
    """nets/retinaface_training_DIOU.py:176-246 (match_iou) over the per-image loop
    (:566-580): match()'s assignment, but loc_t = the matched truth corners
    (:230 `loc = matches`)."""
    locs, confs, landms = [], [], []
    for t in targets:
        _, conf, landm, bti, _ = match(threshold, t[:, :4], priors, var, t[:, -1], t[:, 4:14])
        locs.append(t[:, :4][bti])
        confs.append(conf)
        landms.append(landm)
    return torch.stack(locs), torch.stack(confs), torch.stack(landms)


def bbox_overlaps_diou(b1, b2):
    """nets/retinaface_training_DIOU.py:402-442 for paired rows (rows == cols, so
    the exchange branch never runs)."""
    w1 = b1[:, 2] - b1[:, 0]
    h1 = b1[:, 3] - b1[:, 1]
    w2 = b2[:, 2] - b2[:, 0]
    h2 = b2[:, 3] - b2[:, 1]
    area1 = w1 * h1
    area2 = w2 * h2
    cx1 = (b1[:, 2] + b1[:, 0]) / 2
    cy1 = (b1[:, 3] + b1[:, 1]) / 2
    cx2 = (b2[:, 2] + b2[:, 0]) / 2
    cy2 = (b2[:, 3] + b2[:, 1]) / 2
    inter_max = torch.min(b1[:, 2:], b2[:, 2:])
    inter_min = torch.max(b1[:, :2], b2[:, :2])
    out_max = torch.max(b1[:, 2:], b2[:, 2:])
    out_min = torch.min(b1[:, :2], b2[:, :2])
    inter = torch.clamp(inter_max - inter_min, min=0)
    inter_area = inter[:, 0] * inter[:, 1]
    inter_diag = (cx2 - cx1) ** 2 + (cy2 - cy1) ** 2
    outer = torch.clamp(out_max - out_min, min=0)
    outer_diag = outer[:, 0] ** 2 + outer[:, 1] ** 2
    union = area1 + area2 - inter_area
    d = inter_area / union - inter_diag / outer_diag
    return torch.clamp(d, min=-1.0, max=1.0)


def diou_loss_sum(loc_p, loc_t, priors_p, var):
    """IouLoss(pred_mode='Center', size_sum=True, losstype='Diou').forward
    (nets/retinaface_training_DIOU.py:500-522) with its decode (:319-337)."""
    b = torch.cat((priors_p[:, :2] + loc_p[:, :2] * var[0] * priors_p[:, 2:],
                   priors_p[:, 2:] * torch.exp(loc_p[:, 2:] * var[1])), 1)
    b = torch.cat((b[:, :2] - b[:, 2:] / 2, b[:, 2:]), 1)     # boxes[:, :2] -= boxes[:, 2:]/2
    b = torch.cat((b[:, :2], b[:, 2:] + b[:, :2]), 1)         # boxes[:, 2:] += boxes[:, :2]
    return torch.sum(1.0 - bbox_overlaps_diou(b, loc_t))


# ----------------------------------------------------------------------------- loss
def smooth_l1_sum(x, y):
    return torch.nn.functional.smooth_l1_loss(x, y, reduction="sum")


def multibox_loss(loc, conf, landm, loc_t, conf_t, landm_t, neg_pos=7, num_classes=2,
                  diou=None):
    """nets/retinaface_training.py:219-303 given matched targets.

    diou=(priors, var): the DIoU variant's box term instead
    (nets/retinaface_training_DIOU.py:596-602), loc_t from match_iou_batch.

    Returns (loss_l, loss_c, loss_landm, info) with info carrying the raw sums,
    counts and the hard-negative selection so tests can check each stage.
    """
    conf_t = conf_t.clone()
    pos1 = conf_t > 0
    s_landm = smooth_l1_sum(landm[pos1].view(-1, 10), landm_t[pos1].view(-1, 10))
    pos = conf_t != 0
    if diou is None:
        s_loc = smooth_l1_sum(loc[pos].view(-1, 4), loc_t[pos].view(-1, 4))
    else:
        pri_b = diou[0].to(loc.dtype).unsqueeze(0).expand_as(loc)
        s_loc = diou_loss_sum(loc[pos].view(-1, 4), loc_t[pos].view(-1, 4).to(loc.dtype),
                              pri_b[pos].view(-1, 4), diou[1])
    conf_t[pos] = 1
    bc = conf.reshape(-1, num_classes)
    gmax = bc.max()
    lse = torch.log(torch.sum(torch.exp(bc - gmax), 1, keepdim=True)) + gmax
    mine = lse - bc.gather(1, conf_t.view(-1, 1))
    mine[pos.view(-1, 1)] = 0
    mine = mine.view(loc.shape[0], -1)
    _, order = torch.sort(mine, dim=1, descending=True, stable=True)
    _, rank = order.sort(1)
    num_pos = pos.long().sum(1, keepdim=True)
    num_neg = torch.clamp(neg_pos * num_pos, max=pos.shape[1] - 1)
    neg = rank < num_neg.expand_as(rank)
    sel = (pos | neg)
    s_c = torch.nn.functional.cross_entropy(conf[sel].view(-1, num_classes), conf_t[sel],
                                            reduction="sum")
    n = max(float(num_pos.sum()), 1.0)
    n1 = max(float(pos1.long().sum()), 1.0)
    info = dict(sums=(s_loc, s_c, s_landm), counts=(int(num_pos.sum()), int(pos1.sum())),
                pos=pos, pos1=pos1, sel=sel, mining=mine)
    return s_loc / n, s_c / n, s_landm / n1, info


# ----------------------------------------------------------------------------- decode
def decode(loc, priors, var):
    """utils/utils_bbox.py:29-34."""
    b = torch.cat((priors[:, :2] + loc[:, :2] * var[0] * priors[:, 2:],
                   priors[:, 2:] * torch.exp(loc[:, 2:] * var[1])), 1)
    b[:, :2] -= b[:, 2:] / 2
    b[:, 2:] += b[:, :2]
    return b


def decode_landm(pre, priors, var):
    """utils/utils_bbox.py:39-46."""
    parts = [priors[:, :2] + pre[:, 2 * k:2 * k + 2] * var[0] * priors[:, 2:] for k in range(5)]
    return torch.cat(parts, 1)


# ----------------------------------------------------------------------------- NMS
def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _LIB = ctypes.CDLL(path)
        _LIB.oracle_nms.restype = ctypes.c_int64
        _LIB.oracle_nms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_double, ctypes.c_void_p]
    return _LIB


def nms(boxes, scores, thr):
    """torchvision.ops.nms CPU semantics (oracle/nms_ref.c) -> int64 indices."""
    b = np.ascontiguousarray(np.asarray(boxes, dtype=np.float32).reshape(-1, 4))
    s = np.ascontiguousarray(np.asarray(scores, dtype=np.float32).reshape(-1))
    keep = np.empty(len(s), dtype=np.int64)
    k = _lib().oracle_nms(b.ctypes.data, s.ctypes.data, len(s), float(thr), keep.ctypes.data)
    return keep[:k].copy()


def nms_py(boxes, scores, thr):
    """Pure-Python loop twin of nms() for tiny cases (cross-checks the C)."""
    b = np.asarray(boxes, dtype=np.float32).reshape(-1, 4)
    s = np.asarray(scores, dtype=np.float32).reshape(-1)
    n = len(s)
    order = sorted(range(n), key=lambda i: (0 if math.isnan(s[i]) else 1,
                                            -float(s[i]) if not math.isnan(s[i]) else 0.0, i))
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    sup = [False] * n
    keep = []
    for a, i in enumerate(order):
        if sup[i]:
            continue
        keep.append(i)
        for j in order[a + 1:]:
            if sup[j]:
                continue
            xx1 = b[j, 0] if b[i, 0] < b[j, 0] else b[i, 0]
            yy1 = b[j, 1] if b[i, 1] < b[j, 1] else b[i, 1]
            xx2 = b[j, 2] if b[j, 2] < b[i, 2] else b[i, 2]
            yy2 = b[j, 3] if b[j, 3] < b[i, 3] else b[i, 3]
            dw = np.float32(xx2 - xx1)
            dh = np.float32(yy2 - yy1)
            w = dw if np.float32(0) < dw else np.float32(0)
            h = dh if np.float32(0) < dh else np.float32(0)
            inter = np.float32(w * h)
            with np.errstate(invalid="ignore", divide="ignore"):
                ovr = np.float32(inter / np.float32(np.float32(area[i] + area[j]) - inter))
            if float(ovr) > thr:
                sup[j] = True
    return np.asarray(keep, dtype=np.int64)


def non_max_suppression(det, conf_thres=0.5, nms_thres=0.3):
    """utils/utils_bbox.py:260-296 -> numpy [K,15] (or [] when nothing passes)."""
    det = torch.as_tensor(det)
    det = det[det[:, 4] >= conf_thres]
    if len(det) <= 0:
        return []
    keep = nms(det[:, :4].numpy(), det[:, 4].numpy(), nms_thres)
    return det[torch.from_numpy(keep)].numpy()
