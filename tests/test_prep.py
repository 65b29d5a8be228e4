"""§8f rank 3: predict.py's letterbox + preprocess_input on the device
(jabd_letterbox_f32) against the numpy restatement in oracle/prep_ref.py.
The oracle is pinned by hand-derived known answers (cv2 is absent here and the
reference holds no resized fixture: parity unpinned against cv2 itself).
GPU parity is bit-exact: the kernel issues the same fp32 ops in the same order."""
import numpy as np
import pytest
import torch

from oracle import prep_ref


def test_resize_kat_identity():
    img = np.random.default_rng(0).uniform(0, 255, (7, 5, 3)).astype(np.float32)
    assert np.array_equal(prep_ref.resize_linear(img, 5, 7), img)


def test_resize_kat_upscale_half_pixel_taps():
    img = np.zeros((1, 2, 3), np.float32)
    img[0, 1] = 10
    out = prep_ref.resize_linear(img, 4, 1)
    assert np.array_equal(out[0, :, 0], np.array([0, 2.5, 7.5, 10], np.float32))


def test_resize_kat_area_2x():
    img = np.arange(4 * 4 * 3, dtype=np.float32).reshape(4, 4, 3)
    out = prep_ref.resize_linear(img, 2, 2)
    assert out[0, 0, 0] == (img[0, 0, 0] + img[0, 1, 0] + img[1, 0, 0] + img[1, 1, 0]) / 4


def test_letterbox_kat_padding():
    img = np.full((10, 20, 3), 7, np.float32)     # 20 wide -> 8x4 inside 8x8
    lb = prep_ref.letterbox_image(img, (8, 8))
    assert np.all(lb[:2] == 84) and np.all(lb[6:] == 84) and np.all(lb[2:6] == 7)
    x = prep_ref.preprocess(img, (8, 8))
    assert x.shape == (3, 8, 8) and x[0, 0, 0] == 84 - 104 and x[2, 4, 4] == 7 - 123


@pytest.mark.gpu
@pytest.mark.parametrize("ih,iw,w,h", [(480, 640, 320, 320), (300, 200, 640, 640),
                                       (128, 256, 64, 64), (97, 131, 160, 96),
                                       (1, 1, 8, 8), (1024, 768, 1024, 1024)])
def test_letterbox_parity(cuda, ih, iw, w, h):
    from jabd_amd import ops
    g = np.random.default_rng(ih * 7 + iw)
    imgs = g.integers(0, 256, (2, ih, iw, 3)).astype(np.float32)
    dev = torch.from_numpy(imgs).to(cuda)
    got = ops.letterbox(dev, (w, h)).cpu().numpy()
    gotn = ops.letterbox(dev, (w, h), mean=(104, 117, 123)).cpu().numpy()
    for b in range(2):
        assert np.array_equal(got[b], prep_ref.letterbox_image(imgs[b], (w, h)))
        assert np.array_equal(gotn[b], prep_ref.preprocess(imgs[b], (w, h)))


@pytest.mark.gpu
def test_letterbox_image_reference_contract(cuda):
    from utils.utils import letterbox_image
    img = np.random.default_rng(1).integers(0, 256, (50, 80, 3)).astype(np.float32)
    out = letterbox_image(img, [64, 64])
    assert out.dtype == np.float64 and out.shape == (64, 64, 3)
    assert np.array_equal(out.astype(np.float32), prep_ref.letterbox_image(img, (64, 64)))


def test_correct_rows_kat():
    """A 200x100 (w x h) image letterboxed into 100x100: scale 0.5, 25-px bars
    top and bottom.  Normalised (0.5, 0.25..0.75) maps back to the full height."""
    rows = np.zeros((1, 15), np.float32)
    rows[0, :4] = [0.0, 0.25, 1.0, 0.75]
    rows[0, 4] = 0.9
    out = prep_ref.correct_rows(rows, (100, 100), (100, 200))
    np.testing.assert_allclose(out[0, :4], [0, 0, 200, 100], atol=1e-4)
    assert out[0, 4] == np.float32(0.9)


@pytest.mark.gpu
@pytest.mark.parametrize("lb,px", [(1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("inp,img", [((640, 640), (480, 640)), ((1024, 1024), (1080, 1920)),
                                     ((320, 480), (333, 211))])
def test_correct_boxes_parity(cuda, lb, px, inp, img):
    from jabd_amd import ops
    rows = np.random.default_rng(sum(img)).uniform(-0.1, 1.1, (257, 15)).astype(np.float32)
    dev = torch.from_numpy(rows).to(cuda)
    ops.correct_boxes(dev, inp, img, letterbox=bool(lb), to_pixels=bool(px))
    ref = prep_ref.correct_rows(rows, inp, img, letterbox=bool(lb), to_pixels=bool(px))
    assert np.array_equal(dev.cpu().numpy(), ref)


@pytest.mark.gpu
def test_correct_boxes_empty(cuda):
    from jabd_amd import ops
    ops.correct_boxes(torch.empty((0, 15), device=cuda), (640, 640), (480, 640))


@pytest.mark.gpu
@pytest.mark.parametrize("lb", [True, False])
def test_detect_image_pipeline(cuda, lb):
    """The device detect_image equals its stages composed by hand with the host
    oracle for the pre/post steps."""
    from jabd_amd import ops
    from jabd_amd.predict import detect_image
    from nets.retinaface_r import RetinaFace
    from utils.anchors import Anchors
    from utils.config import cfg_mnet
    torch.manual_seed(0)
    net = RetinaFace(cfg=cfg_mnet, mode="eval").eval().to(cuda)
    img = np.random.default_rng(5).integers(0, 256, (96, 160, 3)).astype(np.float32)
    got = detect_image(net, img, (128, 128), cfg_mnet, confidence=0.3, letterbox_image=lb)
    H, W = (128, 128) if lb else (96, 160)
    x = torch.from_numpy(prep_ref.preprocess(img, (W, H))).unsqueeze(0).to(cuda)
    pri = Anchors(cfg_mnet, image_size=(H, W)).get_anchors().to(cuda).float()
    from jabd_amd import functional as F
    with torch.no_grad():
        with F.split_k():   # the bs1 predict path's conv setting (detect_image)
            out = net(x)
        rows, nk = ops.detect(*out, pri, cfg_mnet["variance"], 0.3, 0.3)
    k = int(nk[0])
    if k == 0:
        assert len(got) == 0
        return
    ref = prep_ref.correct_rows(rows[0, :k].cpu().numpy(), (H, W), (96, 160), letterbox=lb)
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_detect_image_c1_640(cuda):
    """C1 (BASELINE configs[0]): one 480x640 image through detect_image at
    640x640, every stage against the host oracle on its own terms:
    letterbox + preprocess (bit-exact), the forward (<= 1e-3), decode + the
    >= 0.5 score filter + torchvision-CPU NMS at nms_thres 0.3 (oracle/box_ref +
    nms_ref.c on the device forward's output) and retinaface_correct_boxes with
    the pixel rescale (oracle/prep_ref)."""
    from _util import init_for_parity, rel_err
    from jabd_amd import ops
    from jabd_amd.predict import detect_image
    from nets.retinaface_r import RetinaFace
    from oracle import box_ref, model_ref
    from utils.config import cfg_mnet
    net = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="eval"), seed=3).eval()
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    net = net.to(cuda)
    img = np.random.default_rng(640).integers(0, 256, (480, 640, 3)).astype(np.float32)
    got = detect_image(net, img, (640, 640), cfg_mnet, confidence=0.5, nms_iou=0.3)
    # stage 1: letterbox + preprocess_input
    x_ref = prep_ref.preprocess(img, (640, 640))
    x_dev = ops.letterbox(torch.from_numpy(img).to(cuda), (640, 640), mean=(104, 117, 123))
    assert np.array_equal(x_dev[0].cpu().numpy(), x_ref)
    # stage 2: forward (split-K on, as detect_image runs it)
    from jabd_amd import functional as F
    with torch.no_grad(), F.split_k():
        out = net(x_dev)
        ref = model_ref.retinaface_mnv3(sd, torch.from_numpy(x_ref)[None], "eval")
    for g, r in zip(out, ref):
        assert rel_err(g, r) < 1e-3
    # stage 3: decode + filter + NMS (host oracle on the device forward's output)
    pri = box_ref.anchors(cfg_mnet, (640, 640))
    loc, conf, landm = (t[0].cpu() for t in out)
    var = cfg_mnet["variance"]
    det = torch.cat([box_ref.decode(loc, pri, var), conf[:, 1:2],
                     box_ref.decode_landm(landm, pri, var)], -1)
    rows = box_ref.non_max_suppression(det, 0.5, 0.3)
    assert len(rows) > 10, "the test image must produce detections"
    # stage 4: retinaface_correct_boxes + pixel rescale
    ref_final = prep_ref.correct_rows(np.asarray(rows, np.float32), (640, 640), (480, 640))
    assert got.shape == ref_final.shape
    # decode's exp() may differ by an ulp between HIP and the CPU library
    np.testing.assert_allclose(got, ref_final, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
def test_detect_c5_2048(cuda):
    """C5 end to end (BASELINE configs[4]: 2048x2048, 172,032 anchors per
    image): the eval forward at 2048^2 feeds jabd_detect_f32 (decode, the
    >= 0.5 score filter, NMS 0.3 — utils/utils_bbox.py:29-46,260-296), whose
    kept rows equal the host oracle's decode + non_max_suppression
    (torchvision-CPU NMS, oracle/nms_ref.c) on the same forward output: same
    count, same NMS order; decode's exp may differ by an ulp."""
    from _util import init_for_parity
    from jabd_amd import ops, synth
    from nets.retinaface_r import RetinaFace
    from oracle import box_ref
    from utils.anchors import Anchors
    from utils.config import cfg_mnet
    net = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="eval"), seed=5).eval().to(cuda)
    x = synth.images(1, 2048, seed=99, device=cuda)
    pri_dev = Anchors(cfg_mnet, image_size=(2048, 2048)).get_anchors().to(cuda).float()
    assert pri_dev.shape[0] == 172032
    with torch.no_grad():
        loc, conf, landm = net(x)
        rows, nk = ops.detect(loc, conf, landm, pri_dev, cfg_mnet["variance"], 0.5, 0.3)
    k = int(nk[0])
    pri = box_ref.anchors(cfg_mnet, (2048, 2048))
    var = cfg_mnet["variance"]
    lo, cf, lm = (t[0].cpu() for t in (loc, conf, landm))
    cand = int((cf[:, 1] >= 0.5).sum())
    det = torch.cat([box_ref.decode(lo, pri, var), cf[:, 1:2], box_ref.decode_landm(lm, pri, var)],
                    -1)
    ref = np.asarray(box_ref.non_max_suppression(det, 0.5, 0.3), np.float32)
    print(f"C5 2048^2: {cand} candidates >= 0.5, {k} kept")
    assert cand > 10000, "the input must exercise NMS at scale"
    assert k == ref.shape[0]
    got = rows[0, :k].cpu().numpy()
    np.testing.assert_array_equal(got[:, 4], ref[:, 4])        # scores: the same rows, in order
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,size", [("mnv3", 640), ("r50", 320)])
def test_graphed_detect_equals_eager(cuda, kind, size):
    """predict.py's per-image forward + decode + NMS replayed as one HIP graph
    (jabd_amd.predict.graphed_detect) gives the eager launches' kept rows bit
    for bit, on two different inputs through the same graph, and is rebuilt
    after the packs change: load_state_dict with perturbed class-head biases
    bumps the generation, and the replay must then equal a fresh eager run and
    differ from the old rows."""
    import bench
    from jabd_amd import functional as F
    from jabd_amd import ops
    from jabd_amd.predict import graphed_detect
    from utils.anchors import Anchors
    net, cfg = bench._weights_init_model(kind)
    net = net.eval().to(cuda)
    pri = Anchors(cfg, image_size=(size, size)).get_anchors().to(cuda).float()
    var = cfg["variance"]
    g = torch.Generator().manual_seed(size)
    for _ in range(2):
        x = (torch.rand(1, 3, size, size, generator=g) * 255 - 117).to(cuda)
        with torch.no_grad():
            with F.split_k():   # the predict path's setting (graphed_detect's too)
                out = net(x)
            r0, n0 = ops.detect(*out, pri, var, 0.5, 0.3)
            r1, n1 = graphed_detect(net, x, pri, var, 0.5, 0.3)
        k = int(n0[0])
        assert int(n1[0]) == k and k > 0
        assert torch.equal(r0[0, :k], r1[0, :k])
    # perturbed weights (every class head's face logit +0.7): a stale graph
    # replaying the old packs would return the old rows
    sd = {k_: v.clone() for k_, v in net.state_dict().items()}
    heads = [k_ for k_ in sd if "ClassHead" in k_ and k_.endswith("bias")]
    assert heads
    for k_ in heads:
        sd[k_].view(-1, 2)[:, 1] += 0.7
    net.load_state_dict(sd)
    with torch.no_grad():
        with F.split_k():
            r3, n3 = ops.detect(*net(x), pri, var, 0.5, 0.3)
        r2, n2 = graphed_detect(net, x, pri, var, 0.5, 0.3)
    k3 = int(n3[0])
    assert int(n2[0]) == k3 and torch.equal(r2[0, :k3], r3[0, :k3])
    assert k3 != k or not torch.equal(r3[0, :k], r0[0, :k])
