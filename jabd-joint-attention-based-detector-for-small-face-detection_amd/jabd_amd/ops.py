"""Tensor-level wrappers over the libjabd C-ABI (box ops, NMS, match, loss).

Each wrapper validates device/dtype/shape, allocates outputs and workspace
through torch's caching allocator, and launches on torch's current HIP
stream.  CPU tensors are rejected: there is no CPU fallback on the product
path (the CPU restatement lives in oracle/ and is test-only).
"""
import math

import numpy as np
import torch

from ._lib import call, c_size, lib
import ctypes


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _dev(name, t, dtype=torch.float32):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor")
    if not t.is_cuda:
        raise RuntimeError(f"{name}: the JABD HIP path needs a GPU tensor (got {t.device}); "
                           "there is no CPU fallback")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    return t.contiguous()


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def _size_query(fn, *args):
    out = c_size(0)
    call(fn, *args, ctypes.byref(out))
    return out.value


# --------------------------------------------------------------------------- decode
def decode(loc, priors, variances):
    """utils/utils_bbox.py:29-34 — loc [A,4] or [B,A,4] -> corner boxes."""
    loc = _dev("decode.loc", loc)
    priors = _dev("decode.priors", priors)
    A = priors.shape[0]
    if loc.shape[-2:] != (A, 4):
        raise ValueError(f"decode: loc {tuple(loc.shape)} vs priors {tuple(priors.shape)}")
    B = loc.numel() // (A * 4) if A else 0
    out = torch.empty_like(loc)
    call("jabd_decode_f32", _p(loc), _p(priors), B, A, float(variances[0]), float(variances[1]),
         _p(out), _stream())
    return out


def decode_landm(pre, priors, variances):
    """utils/utils_bbox.py:39-46 — pre [A,10] or [B,A,10]."""
    pre = _dev("decode_landm.pre", pre)
    priors = _dev("decode_landm.priors", priors)
    A = priors.shape[0]
    if pre.shape[-2:] != (A, 10):
        raise ValueError(f"decode_landm: pre {tuple(pre.shape)} vs priors {tuple(priors.shape)}")
    B = pre.numel() // (A * 10) if A else 0
    out = torch.empty_like(pre)
    call("jabd_decode_landm_f32", _p(pre), _p(priors), B, A, float(variances[0]), _p(out),
         _stream())
    return out


# --------------------------------------------------------------------------- NMS
def batched_nms(boxes, scores, iou_threshold, score_threshold=-math.inf, n_valid=None):
    """Independent greedy NMS per image.

    boxes [B,N,4] (or a [B,N,>=5] row tensor whose first 4 columns are boxes),
    scores [B,N].  Returns (keep [B,N] int64, n_keep [B] int64), both on the
    device; keep[b,:n_keep[b]] are row indices in decreasing-score order.
    """
    if boxes.dim() != 3 or boxes.shape[-1] < 4:
        raise ValueError(f"batched_nms: boxes must be [B,N,>=4], got {tuple(boxes.shape)}")
    boxes = _dev("nms.boxes", boxes)
    scores = _dev("nms.scores", scores)
    B, N = boxes.shape[0], boxes.shape[1]
    if scores.shape != (B, N):
        raise ValueError(f"batched_nms: scores {tuple(scores.shape)} != {(B, N)}")
    dev = boxes.device
    keep = torch.empty((B, N), dtype=torch.int64, device=dev)
    n_keep = torch.zeros((B,), dtype=torch.int64, device=dev)
    if n_valid is not None:
        n_valid = _dev("nms.n_valid", n_valid, torch.int64)
    ws = _ws(_size_query("jabd_nms_workspace_size", B, N), dev)
    C = boxes.shape[-1]
    call("jabd_batched_nms_f32", _p(boxes), C, N * C, _p(scores), 1, N, _p(n_valid), B, N,
         float(iou_threshold), float(score_threshold), _p(keep), _p(n_keep), _p(ws),
         ws.numel(), _stream())
    return keep, n_keep


def batched_nms_stats(boxes, scores, iou_threshold):
    """batched_nms plus per-image measurement counters: (keep, n_keep,
    tested int64[B], dense bool[B]) where `tested` is the number of exact
    fp32 IoU evaluations the mask producer made (grid: its candidate pairs;
    dense: every pair).  Synchronises (measurement only)."""
    B, N = boxes.shape[0], boxes.shape[1]
    dev = boxes.device
    boxes = _dev("nms.boxes", boxes)
    scores = _dev("nms.scores", scores)
    keep = torch.empty((B, N), dtype=torch.int64, device=dev)
    n_keep = torch.zeros((B,), dtype=torch.int64, device=dev)
    ws = _ws(_size_query("jabd_nms_workspace_size", B, N), dev)
    C = boxes.shape[-1]
    call("jabd_batched_nms_f32", _p(boxes), C, N * C, _p(scores), 1, N, None, B, N,
         float(iou_threshold), float(-math.inf), _p(keep), _p(n_keep), _p(ws), ws.numel(),
         _stream())
    tested = np.zeros(B, np.int64)
    hits = np.zeros(B, np.int32)
    dense = np.zeros(B, np.int32)
    call("jabd_nms_pair_stats", _p(ws), ws.numel(), B, N, tested.ctypes.data, hits.ctypes.data,
         dense.ctypes.data, _stream())
    tested = np.where(dense != 0, N * (N - 1) // 2, tested)
    return keep, n_keep, tested, dense != 0


def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms(boxes[N,4], scores[N], iou_threshold) -> int64[K].

    Returns a device tensor; reading K synchronises the stream once.
    """
    if boxes.dim() != 2 or boxes.shape[-1] != 4:
        raise ValueError(f"nms: boxes must be [N,4], got {tuple(boxes.shape)}")
    keep, n_keep = batched_nms(boxes.unsqueeze(0), scores.unsqueeze(0), iou_threshold)
    return keep[0, : int(n_keep[0].item())]


def detect(loc, conf, landm, priors, variances, conf_threshold=0.5, nms_threshold=0.3):
    """predict.py:162-181 on device for a batch: decode + filter + NMS.

    loc [B,A,4], conf [B,A,2] (eval softmax), landm [B,A,10].
    Returns (rows [B,A,15], n_keep [B]); rows[b,:n_keep[b]] are the kept
    detections (x1,y1,x2,y2,score,landmarks) in NMS order.
    """
    loc = _dev("detect.loc", loc)
    conf = _dev("detect.conf", conf)
    landm = _dev("detect.landm", landm)
    priors = _dev("detect.priors", priors)
    B, A = loc.shape[0], loc.shape[1]
    if priors.shape != (A, 4) or conf.shape != (B, A, 2) or landm.shape != (B, A, 10):
        raise ValueError("detect: shape mismatch")
    dev = loc.device
    out = torch.empty((B, A, 15), dtype=torch.float32, device=dev)
    n_keep = torch.empty((B,), dtype=torch.int64, device=dev)   # written by every call
    ws = _ws(_size_query("jabd_detect_workspace_size", B, A), dev)
    call("jabd_detect_f32", _p(loc), _p(conf), _p(landm), _p(priors), B, A,
         float(variances[0]), float(variances[1]), float(conf_threshold), float(nms_threshold),
         _p(out), _p(n_keep), _p(ws), ws.numel(), _stream())
    return out, n_keep


# --------------------------------------------------------------------------- match
def match_encode(targets, priors, threshold, variances, raw_loc=False):
    """Batched match()+encode() — nets/retinaface_training.py:93-162.

    targets: list of B device tensors [n_i,15]; priors [A,4].
    Returns loc_t [B,A,4], conf_t [B,A] int64, landm_t [B,A,10].
    raw_loc=True is match_iou() (nets/retinaface_training_DIOU.py:176-246):
    loc_t holds the matched truth corners instead of the encoded offsets.
    """
    priors = _dev("match.priors", priors)
    dev = priors.device
    B, A = len(targets), priors.shape[0]
    counts = [int(t.shape[0]) for t in targets]
    if any(c == 0 for c in counts):
        raise ValueError("match: an image has no targets (the reference's match() fails too)")
    for t in targets:
        _dev("match.targets", t)
    if len(targets) == 1:
        flat = targets[0].reshape(-1, 15).contiguous()
    else:  # the images' rows back to back, one launch
        flat = torch.empty((sum(counts), 15), dtype=torch.float32, device=dev)
        items, o = [], 0
        for t, c in zip(targets, counts):
            items.append((t.reshape(-1, 15).contiguous(), flat[o:o + c], 0.0))
            o += c
        from .functional import window_copies
        window_copies(items)
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    offsets = torch.tensor(offs, dtype=torch.int64).to(dev, non_blocking=True)
    loc_t = torch.empty((B, A, 4), dtype=torch.float32, device=dev)
    conf_t = torch.empty((B, A), dtype=torch.int64, device=dev)
    landm_t = torch.empty((B, A, 10), dtype=torch.float32, device=dev)
    ws = _ws(_size_query("jabd_match_workspace_size", B, A), dev)
    call("jabd_match_iou_f32" if raw_loc else "jabd_match_encode_f32", _p(flat), _p(offsets), B, max(counts) if counts else 0,
         _p(priors), A, float(threshold), float(variances[0]), float(variances[1]), _p(loc_t),
         _p(conf_t), _p(landm_t), _p(ws), ws.numel(), _stream())
    return loc_t, conf_t, landm_t


# --------------------------------------------------------------------------- loss
def multibox_sums(loc, conf, landm, loc_t, conf_t, landm_t, neg_pos, diou=None):
    """Un-normalised MultiBoxLoss sums [3], counts [2] and the selection mask.

    diou=(priors [A,4], variances): the box term is the DIoU loss of
    nets/retinaface_training_DIOU.py:491-522 (loc_t from match_encode(raw_loc=True)).
    """
    loc, conf, landm = (_dev("loss.loc", loc), _dev("loss.conf", conf),
                        _dev("loss.landm", landm))
    loc_t, landm_t = _dev("loss.loc_t", loc_t), _dev("loss.landm_t", landm_t)
    conf_t = _dev("loss.conf_t", conf_t, torch.int64)
    B, A = loc.shape[0], loc.shape[1]
    dev = loc.device
    sums = torch.empty(3, dtype=torch.float32, device=dev)
    counts = torch.empty(2, dtype=torch.int64, device=dev)
    sel = torch.empty((B, A), dtype=torch.uint8, device=dev)
    ws = _ws(_size_query("jabd_multibox_workspace_size", B, A), dev)
    if diou is None:
        call("jabd_multibox_loss_fwd_f32", _p(loc), _p(conf), _p(landm), _p(loc_t), _p(conf_t),
             _p(landm_t), B, A, int(neg_pos), _p(sums), _p(counts), _p(sel), _p(ws),
             ws.numel(), _stream())
    else:
        pri, var = _diou_priors(diou, A)
        call("jabd_multibox_diou_loss_fwd_f32", _p(loc), _p(conf), _p(landm), _p(loc_t),
             _p(conf_t), _p(landm_t), _p(pri), float(var[0]), float(var[1]), B, A,
             int(neg_pos), _p(sums), _p(counts), _p(sel), _p(ws), ws.numel(), _stream())
    return sums, counts, sel


def _diou_priors(diou, A):
    pri, var = diou
    pri = _dev("loss.priors", pri)
    if tuple(pri.shape) != (A, 4):
        raise ValueError(f"DIoU loss: priors {tuple(pri.shape)} != ({A}, 4)")
    return pri, var


def multibox_normalize(sums, counts):
    loss = torch.empty(3, dtype=torch.float32, device=sums.device)
    call("jabd_multibox_loss_finalize_f32", _p(sums), _p(counts), _p(loss), _stream())
    return loss


def multibox_backward(loc, conf, landm, loc_t, conf_t, landm_t, sel, gout, counts, diou=None):
    B, A = loc.shape[0], loc.shape[1]
    gl = torch.empty_like(loc)
    gc = torch.empty_like(conf)
    glm = torch.empty_like(landm)
    gout = _dev("loss.gout", gout)
    if diou is None:
        call("jabd_multibox_loss_bwd_f32", _p(loc), _p(conf), _p(landm), _p(loc_t), _p(conf_t),
             _p(landm_t), _p(sel), B, A, _p(gout), _p(counts), _p(gl), _p(gc), _p(glm),
             _stream())
    else:
        pri, var = _diou_priors(diou, A)
        call("jabd_multibox_diou_loss_bwd_f32", _p(loc), _p(conf), _p(landm), _p(loc_t),
             _p(conf_t), _p(landm_t), _p(pri), float(var[0]), float(var[1]), _p(sel), B, A,
             _p(gout), _p(counts), _p(gl), _p(gc), _p(glm), _stream())
    return gl, gc, glm


# --------------------------------------------------------------------------- letterbox
def letterbox(image, size, fill=84.0, mean=None):
    """utils/utils.py:8-19 letterbox_image (+ :27-29 preprocess_input when `mean`
    is given) on the device — see jabd_letterbox_f32.

    image: device float32 [ih, iw, 3] or [B, ih, iw, 3]; size = (w, h) as the
    reference passes it.  mean=None -> [.., h, w, 3] canvas; mean=(m0, m1, m2)
    -> [B, 3, h, w] network input (canvas - mean, NCHW).
    """
    image = _dev("letterbox.image", image)
    squeeze = image.dim() == 3
    if squeeze:
        image = image.unsqueeze(0)
    if image.dim() != 4 or image.shape[-1] != 3:
        raise ValueError(f"letterbox: expected [B, H, W, 3], got {tuple(image.shape)}")
    B, ih, iw = image.shape[0], image.shape[1], image.shape[2]
    w, h = int(size[0]), int(size[1])
    if mean is None:
        out = torch.empty((B, h, w, 3), dtype=torch.float32, device=image.device)
        m = None
    else:
        out = torch.empty((B, 3, h, w), dtype=torch.float32, device=image.device)
        m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    call("jabd_letterbox_f32", _p(image), B, ih, iw, _p(out), h, w, float(fill),
         ctypes.cast(m, ctypes.c_void_p) if m is not None else ctypes.c_void_p(0),
         0 if mean is None else 1, _stream())
    return out[0] if (squeeze and mean is None) else out


def correct_boxes(rows, input_shape, image_shape, letterbox=True, to_pixels=True):
    """In place on device rows [n, 15]: retinaface_correct_boxes
    (utils/utils_bbox.py:9-24, if letterbox) then predict.py:195-196's scale to
    image pixels.  input_shape = (H, W) of the network input, image_shape =
    (im_height, im_width)."""
    rows = _dev("correct_boxes.rows", rows)
    if rows.dim() != 2 or rows.shape[1] != 15:
        raise ValueError(f"correct_boxes: expected [n, 15], got {tuple(rows.shape)}")
    call("jabd_correct_boxes_f32", _p(rows), rows.shape[0], int(input_shape[0]),
         int(input_shape[1]), int(image_shape[0]), int(image_shape[1]), 1 if letterbox else 0,
         1 if to_pixels else 0, _stream())
    return rows


# --------------------------------------------------------------------------- augment
def augment(image_u8, input_shape, nw, nh, dx, dy, flip, hue, sat, val):
    """utils/dataloader.py:71-115 + :62-64 image part on the device, given the
    random draws (see utils.dataloader.draw_params).  image_u8: device uint8
    RGB [ih, iw, 3]; input_shape = (h, w).  Returns float32 [3, h, w]."""
    img = _dev("augment.image", image_u8, torch.uint8)
    if img.dim() != 3 or img.shape[2] != 3:
        raise ValueError(f"augment: expected [H, W, 3] uint8, got {tuple(img.shape)}")
    ih, iw = int(img.shape[0]), int(img.shape[1])
    h, w = int(input_shape[0]), int(input_shape[1])
    out = torch.empty((3, h, w), dtype=torch.float32, device=img.device)
    ws = _ws(_size_query("jabd_augment_workspace_size", ih, int(nw)), img.device)
    call("jabd_augment_u8", _p(img), ih, iw, int(nw), int(nh), h, w, int(dx), int(dy),
         1 if flip else 0, float(hue), float(sat), float(val), _p(out), _p(ws), ws.numel(),
         _stream())
    return out


# --------------------------------------------------------------------------- WIDER eval
def wider_pr_curve(preds, gts, ignores, iou_thresh=0.5, thresh_num=1000, device="cuda"):
    """Σ over images of img_pr_info(image_eval(...)) — utils/evaluation.py:255-305,
    347-375 — on the device.  preds: list of [n_i, 5] (x, y, w, h, score) arrays,
    gts: list of [m_i, 4] (x, y, w, h), ignores: list of [m_i] (1 = kept).
    Returns the float64 pr_curve [thresh_num, 2] (device tensor)."""
    def cat(xs, k, dt):
        a = [np.asarray(x, dt).reshape(-1, k) if k else np.asarray(x, dt).reshape(-1) for x in xs]
        offs = np.zeros(len(a) + 1, np.int64)
        offs[1:] = np.cumsum([len(x) for x in a])
        flat = np.concatenate(a) if a else np.zeros((0,) + ((k,) if k else ()), dt)
        return (torch.from_numpy(np.ascontiguousarray(flat)).to(device),
                torch.from_numpy(offs).to(device), int(offs[-1]))
    if not (len(preds) == len(gts) == len(ignores)):
        raise ValueError("wider_pr_curve: preds, gts and ignores differ in length")
    p, poff, npred = cat(preds, 5, np.float64)
    g, goff, ngt = cat(gts, 4, np.float64)
    ig, _, _ = cat(ignores, 0, np.uint8)
    pr = torch.zeros((thresh_num, 2), dtype=torch.float64, device=device)
    ws = _ws(_size_query("jabd_wider_eval_workspace_size", npred, ngt), device)
    call("jabd_wider_eval_f64", _p(p), _p(poff), _p(g), _p(ig), _p(goff), len(preds), npred, ngt,
         float(iou_thresh), int(thresh_num), _p(pr), _p(ws), ws.numel(), _stream())
    return pr


# --------------------------------------------------------------------------- bicubic
def _bicubic_call(fn, src, size_in, size_out):
    B, H, W, C = size_in
    OH, OW = size_out
    dst = torch.empty((B, OH, OW, C) if fn.endswith("ac_f32") else (B, H, W, C),
                      dtype=torch.float32, device=src.device)
    call(fn, _p(src), B, H, W, C, _p(dst), OH, OW, _stream())
    return dst


class UpsampleBicubicFn(torch.autograd.Function):
    """F.interpolate(x, size, mode="bicubic", align_corners=True) on NHWC
    (train_mobilenetV3_ecagai.py:270,279), HIP forward and backward."""

    @staticmethod
    def forward(ctx, x, oh, ow):
        x = _dev("bicubic.x", x)
        if x.dim() != 4:
            raise ValueError(f"bicubic: expected NHWC, got {tuple(x.shape)}")
        ctx.shape = tuple(x.shape)
        return _bicubic_call("jabd_upsample_bicubic_ac_f32", x, ctx.shape, (oh, ow))

    @staticmethod
    def backward(ctx, gy):
        B, H, W, C = ctx.shape
        gy = gy.contiguous()
        gx = _bicubic_call("jabd_upsample_bicubic_ac_bwd_f32", gy, ctx.shape,
                           (gy.shape[1], gy.shape[2]))
        return gx, None, None


def upsample_bicubic(x_nhwc, size):
    """NHWC bicubic align_corners resize to size = (OH, OW)."""
    return UpsampleBicubicFn.apply(x_nhwc, int(size[0]), int(size[1]))


# --------------------------------------------------------------------------- BECA
def beca_part(B, pixels, C, device):
    """Reduction workspace of jabd_beca_fwd_f32 / _bwd_f32."""
    n = int(lib().jabd_beca_ws_floats(B, pixels, C))
    return torch.empty(max(n, 1), dtype=torch.float32, device=device)


class BecaFn(torch.autograd.Function):
    """eca_block of the bicubic variant (train_mobilenetV3_ecagai.py:286-316) on
    NHWC x [B, H, W, C] with the conv1d weight w [k]: x * Hardsigmoid(conv1d(std))."""

    @staticmethod
    def forward(ctx, x, w):
        x = _dev("beca.x", x)
        w = _dev("beca.w", w.reshape(-1))
        B, H, W, C = x.shape
        y = torch.empty_like(x)
        stats = torch.empty((4, B * C), dtype=torch.float32, device=x.device)
        part = beca_part(B, H * W, C, x.device)
        call("jabd_beca_fwd_f32", _p(x), B, H * W, C, _p(w), w.numel(), _p(y), _p(stats),
             _p(part), part.numel(), _stream())
        from .functional import tap
        tap("beca", stats[2].view(B, C))
        ctx.save_for_backward(x, w, stats)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, stats = ctx.saved_tensors
        B, H, W, C = x.shape
        gy = gy.contiguous()
        gx = torch.empty_like(x)
        gw = torch.empty_like(w)
        ws = torch.empty((2, B * C), dtype=torch.float32, device=x.device)
        part = beca_part(B, H * W, C, x.device)
        call("jabd_beca_bwd_f32", _p(x), _p(gy), B, H * W, C, _p(w), w.numel(), _p(stats),
             _p(gx), _p(gw), _p(ws), _p(part), part.numel(), _stream())
        return gx, gw


def beca(x_nhwc, weight):
    """weight: the block's Conv1d(1, 1, k) weight (any shape with k elements)."""
    return BecaFn.apply(x_nhwc, weight.reshape(-1))


def version():
    return lib().jabd_version().decode()
