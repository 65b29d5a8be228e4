"""§8f rank 2: get_random_data's image path on the device (jabd_augment_u8)
against the numpy restatement in oracle/aug_ref.py (PIL BICUBIC + cv2 float
HSV).  The resize and the paste/flip canvas are pinned byte-exactly against
Pillow itself (importable in the build container; skipped where it is not);
cv2 is absent, so the HSV path is pinned by the hand-derived known answers
below (parity unpinned against cv2); GPU vs oracle is bit-exact for the resize
(integer arithmetic) and within 2e-4 absolute (on a 0..255 scale) for the HSV
round trip, whose fp32 ops the kernel issues in the same order."""
import numpy as np
import pytest
import torch

from oracle import aug_ref


def test_bicubic_kat_identity_and_constant():
    img = np.random.default_rng(0).integers(0, 256, (9, 7, 3)).astype(np.uint8)
    assert np.array_equal(aug_ref.resize_bicubic(img, 7, 9), img)
    const = np.full((13, 11, 3), 77, np.uint8)            # weights sum to 1 -> constant
    assert np.all(aug_ref.resize_bicubic(const, 5, 29) == 77)


@pytest.mark.parametrize("ih,iw,nh,nw", [(37, 53, 61, 29), (120, 90, 47, 63), (16, 16, 16, 16),
                                         (9, 200, 31, 12), (64, 48, 256, 192), (5, 3, 2, 1)])
def test_bicubic_oracle_pinned_to_pillow(ih, iw, nh, nw):
    """oracle.resize_bicubic == PIL Image.resize(BICUBIC) byte for byte (the
    reference's own resampler, utils/dataloader.py:88)."""
    Image = pytest.importorskip("PIL.Image")
    img = np.random.default_rng(ih * 7 + nw).integers(0, 256, (ih, iw, 3)).astype(np.uint8)
    ref = np.asarray(Image.fromarray(img).resize((nw, nh), Image.BICUBIC))
    assert np.array_equal(aug_ref.resize_bicubic(img, nw, nh), ref)


@pytest.mark.parametrize("dx,dy,flip", [(5, -7, False), (-20, 3, True), (0, 0, True),
                                        (40, 40, False), (-100, 0, False)])
def test_canvas_oracle_pinned_to_pillow(dx, dy, flip):
    """oracle.compose_canvas == Image.new grey + paste + FLIP_LEFT_RIGHT
    (utils/dataloader.py:90-98)."""
    Image = pytest.importorskip("PIL.Image")
    rs = np.random.default_rng(abs(dx) + 50).integers(0, 256, (37, 45, 3)).astype(np.uint8)
    h, w = 48, 64
    new = Image.new("RGB", (w, h), (128, 128, 128))
    new.paste(Image.fromarray(rs), (dx, dy))
    if flip:
        new = new.transpose(Image.FLIP_LEFT_RIGHT)
    assert np.array_equal(aug_ref.compose_canvas(rs, (h, w), dx, dy, flip), np.asarray(new))


def test_hsv_kat():
    px = np.array([[1, 0, 0], [0, 1, 0], [0.5, 0.5, 0.5]], np.float32)
    hsv = aug_ref.rgb2hsv(px)
    np.testing.assert_allclose(hsv[:, 0], [0, 120, 0], atol=1e-4)
    np.testing.assert_allclose(hsv[:, 1], [1, 1, 0], atol=1e-6)
    back = aug_ref.hsv2rgb(hsv)
    np.testing.assert_allclose(back, px, atol=1e-6)


def test_augment_kat_reference_hue_wrap():
    """The reference wraps hue at 1 (not 360): with no jitter pure red stays red,
    pure green loses one degree (R = 255/60), grey stays grey."""
    img = np.zeros((1, 3, 3), np.uint8)
    img[0, 0] = [255, 0, 0]
    img[0, 1] = [0, 255, 0]
    img[0, 2] = [128, 128, 128]
    out = aug_ref.augment_image(img, (1, 3), 3, 1, 0, 0, False, 0.0, 1.0, 1.0)
    mean = np.array([104, 117, 123], np.float32)[:, None]
    rgb = out[:, 0, :] + mean
    np.testing.assert_allclose(rgb[:, 0], [255, 0, 0], atol=1e-3)
    np.testing.assert_allclose(rgb[:, 1], [255 / 60, 255, 0], atol=1e-2)
    np.testing.assert_allclose(rgb[:, 2], [128, 128, 128], atol=1e-3)


def test_draw_params_and_targets_host():
    from utils import dataloader
    np.random.seed(3)
    p = dataloader.draw_params(640, 480, (256, 256))
    assert p["nw"] > 0 and p["nh"] > 0 and isinstance(p["flip"], bool)
    p = dict(nw=320, nh=240, dx=0, dy=8, flip=True, hue=0, sat=1, val=1)
    box = np.array([[100, 100, 300, 200] + [150, 150] * 5 + [1.0],
                    [0, 0, 4, 4] + [1, 1] * 5 + [-1.0]])
    np.random.seed(0)
    out = dataloader.remap_targets(box, 640, 480, (256, 256), p)
    # box 0: x*0.5 -> 50..150, y*0.5+8 -> 58..108; flip: x -> 256-150..256-50
    row = out[np.argmax(out[:, 2] - out[:, 0])]
    np.testing.assert_allclose(row[:4], [106 / 256, 58 / 256, 206 / 256, 108 / 256])
    assert len(out) == 2 and np.all(out[out[:, -1] == -1][:, 4:-1] == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("ih,iw,h,w,nw,nh,dx,dy,flip,hue,sat,val", [
    (48, 64, 64, 64, 40, 30, 5, 9, False, 0.05, 1.3, 0.8),
    (64, 48, 64, 64, 150, 180, -40, -60, True, -0.08, 0.7, 1.4),
    (33, 71, 96, 80, 80, 17, 0, 70, True, 0.0, 1.0, 1.0),
    (120, 160, 128, 128, 20, 15, 100, 100, False, 0.1, 1.5, 0.667),
])
def test_augment_parity(cuda, ih, iw, h, w, nw, nh, dx, dy, flip, hue, sat, val):
    from jabd_amd import ops
    img = np.random.default_rng(ih + iw).integers(0, 256, (ih, iw, 3)).astype(np.uint8)
    got = ops.augment(torch.from_numpy(img).to(cuda), (h, w), nw, nh, dx, dy, flip, hue, sat,
                      val).cpu().numpy()
    ref = aug_ref.augment_image(img, (h, w), nw, nh, dx, dy, flip, hue, sat, val)
    assert np.abs(got - ref).max() <= 2e-4, np.abs(got - ref).max()


@pytest.mark.gpu
def test_get_random_data_contract(cuda):
    from utils import dataloader
    img = np.random.default_rng(2).integers(0, 256, (60, 80, 3)).astype(np.uint8)
    box = np.array([[10, 10, 40, 40] + [20, 20] * 5 + [1.0]])
    np.random.seed(5)
    x, t = dataloader.get_random_data(img, box, [64, 64])
    np.random.seed(5)
    p = dataloader.draw_params(80, 60, (64, 64))
    ref = aug_ref.augment_image(img, (64, 64), p["nw"], p["nh"], p["dx"], p["dy"], p["flip"],
                                p["hue"], p["sat"], p["val"])
    assert x.shape == (3, 64, 64) and x.dtype == torch.float32
    assert np.abs(x.cpu().numpy() - ref).max() <= 2e-4
