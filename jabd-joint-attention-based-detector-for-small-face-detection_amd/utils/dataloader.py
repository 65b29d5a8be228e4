"""GPU data augmentation — drop-in for the image/target part of the reference
utils/dataloader.py:71-149 (DataGenerator.get_random_data) and the
__getitem__ tail (:62-64).

The host draws the random values in the reference's np.random order
(draw_params), the device does the pixel work in two launches
(jabd_augment_u8: PIL BICUBIC resize, paste on grey 128, flip, HSV jitter,
preprocess_input, CHW), and the few target rows are remapped on the host in
numpy exactly as the reference does (including its no-op upper clamps).
"""
import numpy as np
import torch

from jabd_amd import ops


def _rand(a=0.0, b=1.0):
    return np.random.rand() * (b - a) + a


def draw_params(iw, ih, input_shape, jitter=.3, hue=.1, sat=1.5, val=1.5, rand=_rand):
    """The reference's random draws (:75-110), in its call order."""
    h, w = input_shape
    new_ar = w / h * rand(1 - jitter, 1 + jitter) / rand(1 - jitter, 1 + jitter)
    scale = rand(0.25, 3.25)
    if new_ar < 1:
        nh = int(scale * h)
        nw = int(nh * new_ar)
    else:
        nw = int(scale * w)
        nh = int(nw / new_ar)
    dx = int(rand(0, w - nw))
    dy = int(rand(0, h - nh))
    flip = rand() < .5
    hue = rand(-hue, hue)
    sat = rand(1, sat) if rand() < .5 else 1 / rand(1, sat)
    val = rand(1, val) if rand() < .5 else 1 / rand(1, val)
    return dict(nw=nw, nh=nh, dx=dx, dy=dy, flip=flip, hue=hue, sat=sat, val=val)


def remap_targets(box, iw, ih, input_shape, p):
    """Target part of get_random_data (:120-147) for the drawn parameters p."""
    h, w = input_shape
    nw, nh, dx, dy = p["nw"], p["nh"], p["dx"], p["dy"]
    box = np.array(box, copy=True)
    xs, ys = [0, 2, 4, 6, 8, 10, 12], [1, 3, 5, 7, 9, 11, 13]
    if len(box) > 0:
        np.random.shuffle(box)
        box[:, xs] = box[:, xs] * nw / iw + dx
        box[:, ys] = box[:, ys] * nh / ih + dy
        if p["flip"]:
            box[:, xs] = w - box[:, [2, 0, 6, 4, 8, 12, 10]]
            box[:, [5, 7, 9, 11, 13]] = box[:, [7, 5, 9, 13, 11]]
        cx = (box[:, 0] + box[:, 2]) / 2
        cy = (box[:, 1] + box[:, 3]) / 2
        box = box[(cx > 0) & (cy > 0) & (cx < w) & (cy < h)]
        v = box[:, 0:14]
        v[v < 0] = 0
        # the reference's upper clamps (:140-141) assign into fancy-index copies: no-ops
        bw = box[:, 2] - box[:, 0]
        bh = box[:, 3] - box[:, 1]
        box = box[(bw > 1) & (bh > 1)]
    lm = box[:, 4:-1]
    lm[box[:, -1] == -1] = 0
    box[:, xs] /= w
    box[:, ys] /= h
    return box


def get_random_data(image, targets, input_shape, jitter=.3, hue=.1, sat=1.5, val=1.5,
                    device="cuda"):
    """image: PIL image or uint8 RGB [ih, iw, 3] (array or tensor).  Returns
    (float32 [3, h, w] device tensor — already preprocessed and CHW, i.e. the
    reference's __getitem__ image, :62-64 — and the float target rows)."""
    if not torch.cuda.is_available():
        raise RuntimeError("get_random_data runs on the HIP device; no GPU is visible")
    if isinstance(image, torch.Tensor):
        img = image.to(device)
    else:
        img = torch.from_numpy(np.ascontiguousarray(np.asarray(image, np.uint8))).to(device)
    ih, iw = int(img.shape[0]), int(img.shape[1])
    p = draw_params(iw, ih, input_shape, jitter, hue, sat, val)
    out = ops.augment(img, input_shape, p["nw"], p["nh"], p["dx"], p["dy"], p["flip"],
                      p["hue"], p["sat"], p["val"])
    return out, remap_targets(targets, iw, ih, input_shape, p)
