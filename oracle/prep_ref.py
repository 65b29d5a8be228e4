"""ORACLE (test infrastructure only) — predict.py's pre-processing restated on
the CPU in numpy float32: letterbox_image (utils/utils.py:8-19) over the
cv2.resize INTER_LINEAR float path, and preprocess_input (:27-29).

cv2 is not installed here and the reference ships no resized fixture, so the
resize restatement is parity-unpinned against cv2 itself; it is pinned by the
hand-derived known answers in tests/test_prep.py (identity at scale 1, the
half-pixel-centre taps of a 2x upscale, the exact-2x INTER_AREA switch).
Restated cv2 behaviour (resize.cpp, float32 images): per axis
f = (float)((d + 0.5) * scale - 0.5), s = floor(f), f -= s; s < 0 -> (0, 0);
s >= n - 1 -> (n - 1, 0); horizontal taps S0*(1-f) + S1*f first, then the
vertical pair; an exact 2x downscale is INTER_AREA: (a + b + c + d) * 0.25.
"""
import numpy as np


def _taps(n_out, n_in):
    scale = 1.0 / (float(n_out) / n_in)
    d = np.arange(n_out, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    s[lo] = 0
    f[lo] = 0
    hi = s >= n_in - 1
    s[hi] = n_in - 1
    f[hi] = 0
    s1 = np.minimum(s + 1, n_in - 1)
    return s, s1, f


def resize_linear(img, nw, nh):
    """cv2.resize(img, (nw, nh)) for a float32 [ih, iw, 3] image (INTER_LINEAR)."""
    img = np.asarray(img, np.float32)
    ih, iw = img.shape[:2]
    if iw == 2 * nw and ih == 2 * nh:   # cv2 switches exact 2x linear to INTER_AREA
        a, b = img[0::2, 0::2], img[0::2, 1::2]
        c, d = img[1::2, 0::2], img[1::2, 1::2]
        return (((a + b) + c) + d) * np.float32(0.25)
    x0, x1, fx = _taps(nw, iw)
    y0, y1, fy = _taps(nh, ih)
    ax0 = (np.float32(1) - fx)[None, :, None]
    ay0 = (np.float32(1) - fy)[:, None, None]
    fx = fx[None, :, None]
    fy = fy[:, None, None]
    h0 = img[y0][:, x0] * ax0 + img[y0][:, x1] * fx
    h1 = img[y1][:, x0] * ax0 + img[y1][:, x1] * fx
    return (h0 * ay0 + h1 * fy).astype(np.float32)


def letterbox_image(image, size, fill=84.0):
    """utils/utils.py:8-19 (float32 canvas here; the reference's is float64 holding
    the same float32 values)."""
    ih, iw, _ = np.shape(image)
    w, h = size
    scale = min(w / iw, h / ih)
    nw, nh = int(iw * scale), int(ih * scale)
    out = np.full((h, w, 3), fill, np.float32)
    top, left = (h - nh) // 2, (w - nw) // 2
    out[top:top + nh, left:left + nw] = resize_linear(image, nw, nh)
    return out


def preprocess(image, size, mean=(104, 117, 123)):
    """letterbox_image -> preprocess_input (:27-29) -> transpose(2, 0, 1), as
    predict.py:143-152 chains them; returns float32 [3, h, w]."""
    lb = letterbox_image(image, size)
    return (lb - np.array(mean, np.float32)).transpose(2, 0, 1).copy()


def correct_rows(rows, input_shape, image_shape, letterbox=True, to_pixels=True):
    """utils/utils_bbox.py:9-24 (retinaface_correct_boxes, numpy float64 assigned back
    into float32 rows) then predict.py:195-196 (`* scale`, image width/height as
    int64 -> float64 math, assigned back)."""
    r = np.array(rows, np.float32, copy=True)
    input_shape = np.array(input_shape)
    image_shape = np.array(image_shape)
    if letterbox:
        new_shape = image_shape * np.min(input_shape / image_shape)
        offset = (input_shape - new_shape) / 2. / input_shape
        scale = input_shape / new_shape
        r[:, :4] = (r[:, :4] - np.array([offset[1], offset[0]] * 2)) * np.array([scale[1], scale[0]] * 2)
        r[:, 5:] = (r[:, 5:] - np.array([offset[1], offset[0]] * 5)) * np.array([scale[1], scale[0]] * 5)
    if to_pixels:
        ih, iw = int(image_shape[0]), int(image_shape[1])
        r[:, :4] = r[:, :4] * np.array([iw, ih] * 2, np.int64)
        r[:, 5:] = r[:, 5:] * np.array([iw, ih] * 5, np.int64)
    return r
