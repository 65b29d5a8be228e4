"""predict.py's detect_image (predict.py:115-196) as one device pipeline:
letterbox + preprocess_input (jabd_letterbox_f32) -> RetinaFace eval forward ->
decode + score filter + NMS (jabd_detect_f32) -> retinaface_correct_boxes +
pixel rescale (jabd_correct_boxes_f32).  Only the kept rows leave the device.
"""
import collections
import os

import numpy as np
import torch

from jabd_amd import functional as F
from jabd_amd import hipmodule, ops

# JABD_PREDICT_GRAPH=0: launch the forward + detect kernels one by one (A/B).
# The library initialises its workspaces with its own fill kernel (fill.hip),
# not hipMemsetAsync: with captured memset nodes, a replay that followed an
# eager detect launched after the capture read a wrong fill pattern and
# faulted the device (ROCm 7, tools/graph_check.py --between det); with kernel
# nodes only, interleaved eager calls and replays agree bit for bit.
PREDICT_GRAPH = os.environ.get("JABD_PREDICT_GRAPH", "1") != "0"
# graphs kept per module (least recently used dropped first): each holds a
# private memory pool with the whole activation set of its shape
GRAPH_CACHE = int(os.environ.get("JABD_PREDICT_GRAPHS", "4"))


class GraphedDetect:
    """The eval forward + decode / filter / NMS of one input shape, captured
    once as a HIP graph (torch.cuda.CUDAGraph) and replayed per image: a bs1
    predict step is ~170 launches (R50) whose host-side dispatch (ctypes +
    Python per launch) exceeded their GPU time (predict.py get_FPS,
    predict.py:253-333).  The input is copied into the graph's static input;
    the outputs are the graph's static (rows, n_keep) buffers, valid until
    the next replay.  The forward runs with split-K on (functional.split_k),
    as the eager bs1 predict path.  Invalid once the model's packs may have
    changed (hipmodule generation)."""

    def __init__(self, net, shape, priors, variances, conf_thres, nms_thres, device):
        self.net, self.gen = net, hipmodule.generation()
        self.x = torch.zeros(shape, dtype=torch.float32, device=device)
        self.pri = priors
        self.args = (variances, conf_thres, nms_thres)
        cur = torch.cuda.current_stream(device)
        side = torch.cuda.Stream(device=device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):   # packs, workspaces and lazy state first
            for _ in range(2):
                self._body()
        cur.wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self._body()

    def _body(self):
        with torch.no_grad(), F.split_k():
            loc, conf, landm = self.net(self.x)
            v, ct, nt = self.args
            return ops.detect(loc, conf, landm, self.pri, v, ct, nt)

    def __call__(self, x):
        self.x.copy_(x)
        self.graph.replay()
        return self.out


def graphed_detect(net, x, priors, variances, conf_thres=0.5, nms_thres=0.3):
    """ops.detect(*net(x), ...) for a batch of the shape of x, through a HIP
    graph cached on the module per (shape, device, thresholds, priors);
    rebuilt when the module's eval packs may have changed."""
    key = (tuple(x.shape), str(x.device), float(variances[0]), float(variances[1]),
           float(conf_thres), float(nms_thres), priors.data_ptr())
    cache = net.__dict__.setdefault("_jabd_graphs", collections.OrderedDict())
    g = cache.get(key)
    if g is None or g.gen != hipmodule.generation() or g.pri is not priors:
        cache.pop(key, None)
        while len(cache) >= max(1, GRAPH_CACHE):
            cache.popitem(last=False)
        g = cache[key] = GraphedDetect(net, tuple(x.shape), priors, variances, conf_thres,
                                       nms_thres, x.device)
    cache.move_to_end(key)
    return g(x)


def _use_graph(net, shape, fixed_shape):
    """Graph only a shape that will recur: letterboxed inputs (one fixed
    shape), or an image size this module has already run once.  A folder of
    mixed-size images (letterbox_image=False) stays on the eager path instead
    of paying two warm-up forwards, a capture and a private pool per size."""
    if not PREDICT_GRAPH or net.training:
        return False
    if fixed_shape:
        return True
    seen = net.__dict__.setdefault("_jabd_seen_shapes", collections.OrderedDict())
    hit = shape in seen
    seen[shape] = True
    seen.move_to_end(shape)
    while len(seen) > 64:
        seen.popitem(last=False)
    return hit


def detect_image(net, image, input_shape, cfg, confidence=0.5, nms_iou=0.3,
                 letterbox_image=True, device="cuda"):
    """image: RGB HWC array (uint8 or float32), as predict.py's np.array(image,
    np.float32).  input_shape = (H, W) of the network input (used only when
    letterbox_image; otherwise the image's own size, as the reference).
    Returns numpy float32 [K, 15] (x1, y1, x2, y2, score, 5 landmark xy) in image
    pixels, NMS order; [] when nothing survives (the reference returns early)."""
    from utils.anchors import Anchors
    img = torch.from_numpy(np.ascontiguousarray(np.asarray(image, np.float32))).to(device)
    ih, iw = int(img.shape[0]), int(img.shape[1])
    H, W = (int(input_shape[0]), int(input_shape[1])) if letterbox_image else (ih, iw)
    x = ops.letterbox(img, (W, H), mean=(104.0, 117.0, 123.0))   # [1, 3, H, W]
    priors = Anchors(cfg, image_size=(H, W)).get_anchors().to(device).float().contiguous()
    with torch.no_grad():
        if _use_graph(net, (H, W, str(device)), letterbox_image):
            priors = _cached_priors(net, cfg, H, W, device, priors)
            rows, n_keep = graphed_detect(net, x, priors, cfg["variance"], confidence, nms_iou)
        else:
            with F.split_k():
                loc, conf, landm = net(x)
            rows, n_keep = ops.detect(loc, conf, landm, priors, cfg["variance"], confidence,
                                      nms_iou)
        k = int(n_keep[0].item())
        if k == 0:
            return []
        det = rows[0, :k].contiguous()
        ops.correct_boxes(det, (H, W), (ih, iw), letterbox=letterbox_image, to_pixels=True)
    return det.cpu().numpy()


def _cached_priors(net, cfg, H, W, device, priors):
    """One priors tensor per (input size, device, anchor cfg) on the module
    (the graph keys on its storage).  The priors are a function of exactly
    these keys (utils/anchors.py:8-42), so another cfg on the same net gets
    its own tensor (and graph) instead of stale priors."""
    cache = net.__dict__.setdefault("_jabd_priors", {})
    key = (H, W, str(device), repr(cfg.get("min_sizes")), repr(cfg.get("steps")),
           bool(cfg.get("clip", False)))
    p = cache.get(key)
    if p is None or p.shape != priors.shape:
        p = cache[key] = priors
    return p
