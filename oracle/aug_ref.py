"""ORACLE (test infrastructure only) — the image part of utils/dataloader.py:71-115
(get_random_data) + :62-64, restated in numpy for given random draws.

The reference holds no augmented fixture.  Pillow (12.2.0) is importable in
the build container: tests/test_augment.py pins resize_bicubic and
compose_canvas bit-exactly against Image.resize(BICUBIC) / Image.paste /
transpose on random images.  cv2 is absent: the HSV round trip stays pinned
only by hand-derived known answers (parity unpinned against cv2).
  * Image.resize(BICUBIC): Pillow Resample.c — precompute_coeffs (bicubic
    a = -0.5, support 2*max(scale, 1), taps [int(c - sup + .5), int(c + sup + .5)),
    double weights normalised by their sum), normalize_coeffs_8bpc (22-bit fixed
    point, round half away from zero), horizontal pass first into uint8 with clip8,
    then the vertical pass; accumulators start at 1 << 21.
  * cv2.cvtColor RGB2HSV / HSV2RGB, float32 path (color_hsv.simd.hpp, scalar code).
"""
import numpy as np

PREC = 22
FLT_EPS = np.float32(1.1920928955078125e-07)


def _bicubic(x):
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def _coeffs(n_in, n_out):
    scale = n_in / n_out
    fs = max(scale, 1.0)
    support = 2.0 * fs
    rows = []
    for o in range(n_out):
        c = (o + 0.5) * scale
        ss = 1.0 / fs
        xmin = max(int(c - support + 0.5), 0)
        xmax = min(int(c + support + 0.5), n_in) - xmin
        w = [_bicubic((x + xmin - c + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        k = [(v / ww if ww != 0.0 else v) for v in w]
        k = [int(-0.5 + v * (1 << PREC)) if v < 0 else int(0.5 + v * (1 << PREC)) for v in k]
        rows.append((xmin, np.array(k, np.int64)))
    return rows


def _clip8(ss):
    return np.clip(ss >> PREC, 0, 255).astype(np.uint8)


def resize_bicubic(img, nw, nh):
    """Image.fromarray(img).resize((nw, nh), Image.BICUBIC) for uint8 RGB."""
    img = np.asarray(img, np.uint8).astype(np.int64)
    ih, iw = img.shape[:2]
    tmp = np.empty((ih, nw, 3), np.uint8)
    for o, (xmin, k) in enumerate(_coeffs(iw, nw)):
        acc = (1 << (PREC - 1)) + (img[:, xmin:xmin + len(k)] * k[None, :, None]).sum(1)
        tmp[:, o] = _clip8(acc)
    t = tmp.astype(np.int64)
    out = np.empty((nh, nw, 3), np.uint8)
    for o, (ymin, k) in enumerate(_coeffs(ih, nh)):
        acc = (1 << (PREC - 1)) + (t[ymin:ymin + len(k)] * k[:, None, None]).sum(0)
        out[o] = _clip8(acc)
    return out


def rgb2hsv(x):
    """cv2 RGB2HSV for float32 [.., 3] in [0, 1]: h in degrees."""
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    v = np.maximum(np.maximum(r, g), b)
    vmin = np.minimum(np.minimum(r, g), b)
    diff = (v - vmin).astype(np.float32)
    s = (diff / (np.abs(v) + FLT_EPS)).astype(np.float32)
    d = (60.0 / (diff + FLT_EPS).astype(np.float64)).astype(np.float32)
    h = np.where(v == r, (g - b) * d,
                 np.where(v == g, (b - r) * d + np.float32(120), (r - g) * d + np.float32(240)))
    h = h.astype(np.float32)
    h = np.where(h < 0, h + np.float32(360), h).astype(np.float32)
    return np.stack([h, s, v], -1).astype(np.float32)


def hsv2rgb(x):
    """cv2 HSV2RGB for float32 (h in degrees); returns [.., 3] RGB in [0, 1]."""
    h, s, v = x[..., 0].copy(), x[..., 1], x[..., 2]
    h = (h * np.float32(6.0 / 360.0)).astype(np.float32)
    h = np.where(h < 0, h + np.float32(6) * np.ceil(-h / 6), h).astype(np.float32)
    while np.any(h >= 6):
        h = np.where(h >= 6, h - np.float32(6), h).astype(np.float32)
    sector = np.floor(h).astype(np.int64)
    h = (h - sector.astype(np.float32)).astype(np.float32)
    bad = (sector < 0) | (sector >= 6)
    sector[bad] = 0
    h[bad] = 0
    one = np.float32(1)
    tab = np.stack([v, v * (one - s), v * (one - s * h), v * (one - s * (one - h))], -1)
    sd = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    idx = sd[sector]                                    # [.., 3] -> (b, g, r) tab slots
    bgr = np.take_along_axis(tab, idx, -1)
    rgb = bgr[..., ::-1]
    gray = (s == 0)[..., None]
    return np.where(gray, np.stack([v, v, v], -1), rgb).astype(np.float32)


def compose_canvas(rs, input_shape, dx, dy, flip):
    """:90-98: Image.new('RGB', (w, h), (128, 128, 128)).paste(rs, (dx, dy)),
    then transpose(FLIP_LEFT_RIGHT) if flip; uint8 [h, w, 3]."""
    h, w = input_shape
    nh, nw = rs.shape[:2]
    canvas = np.full((h, w, 3), 128, np.uint8)
    y0, x0 = max(dy, 0), max(dx, 0)
    y1, x1 = min(dy + nh, h), min(dx + nw, w)
    if y1 > y0 and x1 > x0:
        canvas[y0:y1, x0:x1] = rs[y0 - dy:y1 - dy, x0 - dx:x1 - dx]
    if flip:
        canvas = canvas[:, ::-1]
    return canvas


def augment_image(img_u8, input_shape, nw, nh, dx, dy, flip, hue, sat, val):
    """:84-115 + :62-64 for the given draws: float32 [3, h, w]."""
    canvas = compose_canvas(resize_bicubic(img_u8, nw, nh), input_shape, dx, dy, flip)
    x = rgb2hsv(np.array(canvas, np.float32) / np.float32(255))
    x[..., 0] += np.float32(hue * 360)
    x[..., 0][x[..., 0] > 1] -= 1
    x[..., 0][x[..., 0] < 0] += 1
    x[..., 1] *= np.float32(sat)
    x[..., 2] *= np.float32(val)
    x[x[:, :, 0] > 360, 0] = 360
    x[:, :, 1:][x[:, :, 1:] > 1] = 1
    x[x < 0] = 0
    rgb = hsv2rgb(x) * np.float32(255)
    rgb -= np.array((104, 117, 123), np.float32)
    return np.transpose(rgb, (2, 0, 1)).astype(np.float32)
