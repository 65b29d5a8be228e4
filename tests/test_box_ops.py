"""A6-A10 box work: anchors, decode, NMS, matching — oracle KATs on CPU and
HIP-vs-oracle parity on the GPU (bit-exact for indices and assignments)."""
import math

import numpy as np
import pytest
import torch

from oracle import box_ref

CFG_MNET = {"min_sizes": [[16, 32], [64, 128], [256, 512]], "steps": [8, 16, 32],
            "variance": [0.1, 0.2], "clip": False}


# ---------------------------------------------------------------- oracle KATs (CPU)
def test_anchor_count_reference_kat():
    # utils/anchors.py:82-105 prints 29518 for steps 8/16/32/64 at 840².
    cfg = {"min_sizes": [[8, 16], [32, 64], [64, 128], [256, 512]], "steps": [8, 16, 32, 64],
           "clip": False}
    assert box_ref.anchors(cfg, (840, 840)).shape[0] == 29518
    assert box_ref.num_anchors(cfg, (840, 840)) == 29518


@pytest.mark.parametrize("size,count", [(640, 16800), (840, 29126), (1024, 43008),
                                        (2048, 172032)])
def test_anchor_counts_hand_derived(size, count):
    assert box_ref.num_anchors(CFG_MNET, (size, size)) == count


def test_anchor_values_first_rows():
    a = box_ref.anchors(CFG_MNET, (640, 640))
    # level 0, i=0, j=0: cx=cy=0.5*8/640, w=h=16/640 then 32/640
    np.testing.assert_array_equal(a[0].numpy(), np.float32([4 / 640, 4 / 640, 16 / 640, 16 / 640]))
    np.testing.assert_array_equal(a[1].numpy(), np.float32([4 / 640, 4 / 640, 32 / 640, 32 / 640]))
    np.testing.assert_array_equal(a[2].numpy(), np.float32([12 / 640, 4 / 640, 16 / 640, 16 / 640]))


def test_nms_kat_hand_made():
    boxes = np.float32([[0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30], [0, 0, 10, 10]])
    scores = np.float32([0.9, 0.8, 0.7, 0.9])
    # box1 vs box0: inter 81, union 119 -> 0.68 > 0.3 suppressed; box3 ties box0
    # at 0.9 and sorts after it (stable), IoU 1 -> suppressed.
    assert box_ref.nms(boxes, scores, 0.3).tolist() == [0, 2]
    assert box_ref.nms_py(boxes, scores, 0.3).tolist() == [0, 2]
    # IoU exactly 0.5 is NOT suppressed at thr 0.5 (strict >)
    b2 = np.float32([[0, 0, 2, 1], [1, 0, 3, 1]])  # inter 1, union 3 -> 1/3
    assert box_ref.nms(b2, np.float32([1, 0.5]), 1 / 3.0).tolist() in ([0], [0, 1])
    b3 = np.float32([[0, 0, 4, 1], [0, 0, 2, 1]])  # inter 2 union 4 -> 0.5 exactly
    assert box_ref.nms(b3, np.float32([1, 0.9]), 0.5).tolist() == [0, 1]
    assert box_ref.nms(b3, np.float32([1, 0.9]), 0.49).tolist() == [0]


def test_nms_oracle_c_matches_python_twin():
    rng = np.random.default_rng(5)
    for n in (0, 1, 7, 200):
        xy = rng.uniform(0, 1, (n, 2)).astype(np.float32)
        wh = rng.uniform(0.01, 0.3, (n, 2)).astype(np.float32)
        b = np.concatenate([xy, xy + wh], 1)
        s = rng.choice(np.float32([0.5, 0.6, 0.7, 0.8]), n)
        assert box_ref.nms(b, s, 0.3).tolist() == box_ref.nms_py(b, s, 0.3).tolist()


def test_match_kat_shared_best_prior():
    # two truths whose best prior is the same prior 0: the later truth wins it
    # (sequential loop at nets/retinaface_training.py:129-130).
    priors = torch.tensor([[0.5, 0.5, 0.2, 0.2], [0.1, 0.1, 0.05, 0.05]])
    t = torch.tensor([[0.4, 0.4, 0.6, 0.6], [0.41, 0.41, 0.61, 0.61]])
    labels = torch.tensor([1.0, -1.0])
    landms = torch.zeros(2, 10)
    loc, conf, landm, bti, bto = box_ref.match(0.35, t, priors, [0.1, 0.2], labels, landms)
    assert bti.tolist()[0] == 1 and conf.tolist()[0] == -1 and float(bto[0]) == 2.0
    assert conf.tolist()[1] == 0  # prior 1 overlaps nothing


# ---------------------------------------------------------------- HIP parity (GPU)
def _clustered(n, seed, ties=True):
    from jabd_amd import synth
    b, s = synth.nms_boxes(1, n, seed=seed, tie_frac=0.05 if ties else 0.0)
    return b[0], s[0]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 1000, 4096])
def test_nms_parity_sizes(cuda, n):
    from jabd_amd import ops
    b, s = _clustered(max(n, 1), seed=n + 11)
    b, s = b[:n], s[:n]
    ref = box_ref.nms(b, s, 0.3)
    got = ops.nms(torch.from_numpy(b).to(cuda), torch.from_numpy(s).to(cuda), 0.3)
    assert got.cpu().numpy().tolist() == ref.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [0.0, 0.3, 0.45, 0.7, 1.0])
def test_nms_parity_thresholds(cuda, thr):
    from jabd_amd import ops
    b, s = _clustered(3000, seed=7)
    ref = box_ref.nms(b, s, thr)
    got = ops.nms(torch.from_numpy(b).to(cuda), torch.from_numpy(s).to(cuda), thr)
    assert got.cpu().numpy().tolist() == ref.tolist()


@pytest.mark.gpu
def test_nms_parity_degenerate(cuda):
    from jabd_amd import ops
    # identical boxes, zero-area boxes, all-equal scores, -0.0 vs 0.0 scores
    b = np.float32([[0, 0, 1, 1]] * 5 + [[0.5, 0.5, 0.5, 0.5]] * 3 + [[0, 0, 2, 2], [2, 2, 1, 1]])
    s = np.float32([0.5] * 5 + [0.0, -0.0, 0.0] + [0.5, 0.7])
    for thr in (0.0, 0.3, 0.99):
        ref = box_ref.nms(b, s, thr)
        got = ops.nms(torch.from_numpy(b).to(cuda), torch.from_numpy(s).to(cuda), thr)
        assert got.cpu().numpy().tolist() == ref.tolist(), thr


@pytest.mark.gpu
def test_batched_nms_with_filter(cuda):
    from jabd_amd import ops, synth
    B, n = 3, 5000
    bx, sc = synth.nms_boxes(B, n, seed=3)
    sc = sc - 0.25  # half the rows fall under the 0.5 filter
    keep, nk = ops.batched_nms(torch.from_numpy(bx).to(cuda), torch.from_numpy(sc).to(cuda),
                               0.3, score_threshold=0.5)
    keep, nk = keep.cpu().numpy(), nk.cpu().numpy()
    for b in range(B):
        m = np.nonzero(sc[b] >= 0.5)[0]
        ref = m[box_ref.nms(bx[b][m], sc[b][m], 0.3)]
        assert keep[b, : nk[b]].tolist() == ref.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("n,nv", [(16800, 16800), (16800, 9001), (32768, 30000), (3000, 0)])
def test_single_image_compacted_keys(cuda, n, nv):
    """One image (the bs1 predict path: csrc/nms.hip nms_keys_compact + the
    one-workgroup sort over the candidates alone) with the 0.5 score filter,
    ~5% exact score ties and a valid-row limit n_valid, against the oracle on
    the filtered rows; nv = 0: no candidate at all."""
    from jabd_amd import ops, synth
    bx, sc = synth.nms_boxes(1, n, seed=n + nv, tie_frac=0.05)
    sc = sc - 0.25
    keep, nk = ops.batched_nms(torch.from_numpy(bx).to(cuda), torch.from_numpy(sc).to(cuda),
                               0.3, score_threshold=0.5,
                               n_valid=torch.tensor([nv], dtype=torch.int64, device=cuda))
    keep, nk = keep.cpu().numpy(), nk.cpu().numpy()
    m = np.nonzero(sc[0][:nv] >= 0.5)[0]
    ref = m[box_ref.nms(bx[0][m], sc[0][m], 0.3)] if len(m) else np.zeros(0, np.int64)
    assert keep[0, : nk[0]].tolist() == ref.tolist()


@pytest.mark.gpu
def test_decode_parity(cuda):
    from jabd_amd import ops
    pri = box_ref.anchors(CFG_MNET, (256, 256))
    g = torch.Generator().manual_seed(0)
    loc = torch.randn(2, pri.shape[0], 4, generator=g) * 0.5
    lm = torch.randn(2, pri.shape[0], 10, generator=g)
    got = ops.decode(loc.to(cuda), pri.to(cuda), [0.1, 0.2]).cpu()
    gotl = ops.decode_landm(lm.to(cuda), pri.to(cuda), [0.1, 0.2]).cpu()
    for b in range(2):
        ref = box_ref.decode(loc[b], pri, [0.1, 0.2])
        torch.testing.assert_close(got[b], ref, rtol=1e-6, atol=1e-7)  # exp ulp only
        refl = box_ref.decode_landm(lm[b], pri, [0.1, 0.2])
        assert torch.equal(gotl[b], refl)  # no transcendental: bit-exact


@pytest.mark.gpu
@pytest.mark.parametrize("size,batch", [(256, 4), (640, 2)])
def test_match_parity(cuda, size, batch):
    from jabd_amd import ops, synth
    pri = box_ref.anchors(CFG_MNET, (size, size))
    tg = [torch.from_numpy(t) for t in synth.targets(batch, size, seed=size)]
    rl, rc, rlm = box_ref.match_batch(tg, pri)
    gl, gc, glm = ops.match_encode([t.to(cuda) for t in tg], pri.to(cuda), 0.35, [0.1, 0.2])
    assert torch.equal(gc.cpu(), rc)  # bit-exact assignment incl. forced matches
    torch.testing.assert_close(gl.cpu(), rl, rtol=1e-5, atol=1e-5)  # log() ulp
    assert torch.equal(glm.cpu(), rlm)


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [0.3, 0.5, 0.45])
def test_nms_parity_near_threshold(cuda, thr):
    """Pairs whose IoU sits within a few ulp of the threshold exercise the
    exact-division path of the branch-free mask kernel."""
    from jabd_amd import ops
    rng = np.random.default_rng(11)
    rows, scores = [], []
    for k in range(400):
        x0, y0 = rng.uniform(0, 50, 2).astype(np.float32)
        s = np.float32(thr) * np.float32(1 + rng.integers(-8, 9) * 2e-7)
        # IoU([x0,y0,x0+1,y0+1], [x0,y0,x0+s,y0+1]) = s (nested boxes)
        rows += [[x0, y0, x0 + 1, y0 + 1], [x0, y0, x0 + s, y0 + 1]]
        scores += [1.0 - k * 1e-3, 0.5 - k * 1e-4]
    b = np.asarray(rows, np.float32)
    sc = np.asarray(scores, np.float32)
    ref = box_ref.nms(b, sc, thr)
    got = ops.nms(torch.from_numpy(b).to(cuda), torch.from_numpy(sc).to(cuda), thr)
    assert got.cpu().numpy().tolist() == ref.tolist()
    assert 0 < len(ref) < len(sc)  # the set really straddles the threshold


@pytest.mark.gpu
def test_nms_parity_nan_boxes(cuda):
    from jabd_amd import ops
    b, s = _clustered(500, seed=3)
    b = b.copy()
    b[7, 0] = np.nan
    b[100, 3] = np.nan
    ref = box_ref.nms(b, s, 0.3)
    got = ops.nms(torch.from_numpy(b).to(cuda), torch.from_numpy(s).to(cuda), 0.3)
    assert got.cpu().numpy().tolist() == ref.tolist()


def test_diou_oracle_kat():
    """Hand-derived DIoU values for the oracle restatement of
    nets/retinaface_training_DIOU.py:402-442 and IouLoss (:500-522)."""
    pri = torch.tensor([[0.5, 0.5, 1.0, 1.0]] * 3)
    loc = torch.zeros(3, 4)  # decodes to [0, 0, 1, 1]
    tr = torch.tensor([[0.0, 0.0, 1.0, 1.0],    # identical: DIoU 1, loss 0
                       [2.0, 0.0, 3.0, 1.0],    # disjoint: 0 - 4/10 -> loss 1.4
                       [0.5, 0.0, 1.5, 1.0]])   # I/U = .5/1.5, diag .25/(2.25+1)
    d = box_ref.bbox_overlaps_diou(box_ref.decode(loc, pri, [0.1, 0.2]), tr)
    ref = torch.tensor([1.0, -0.4, 0.5 / 1.5 - 0.25 / 3.25])
    torch.testing.assert_close(d, ref, rtol=0, atol=1e-6)
    s = box_ref.diou_loss_sum(loc, tr, pri, [0.1, 0.2])
    assert abs(float(s) - float((1 - ref).sum())) < 1e-6


def test_match_iou_oracle_keeps_truth_corners():
    pri = box_ref.anchors(CFG_MNET, (128, 128))
    from jabd_amd import synth
    tg = [torch.from_numpy(t) for t in synth.targets(2, 128, seed=4)]
    rl, rc, rlm = box_ref.match_batch(tg, pri)
    il, ic, ilm = box_ref.match_iou_batch(tg, pri)
    assert torch.equal(rc, ic) and torch.equal(rlm, ilm)
    for b, t in enumerate(tg):   # every loc_t row is one of the image's truth boxes
        hits = (il[b][:, None, :] == t[None, :, :4]).all(-1).any(-1)
        assert bool(hits.all())


@pytest.mark.gpu
@pytest.mark.parametrize("size,batch", [(256, 4), (640, 2)])
def test_match_iou_parity(cuda, size, batch):
    from jabd_amd import ops, synth
    pri = box_ref.anchors(CFG_MNET, (size, size))
    tg = [torch.from_numpy(t) for t in synth.targets(batch, size, seed=size + 1)]
    rl, rc, rlm = box_ref.match_iou_batch(tg, pri)
    gl, gc, glm = ops.match_encode([t.to(cuda) for t in tg], pri.to(cuda), 0.35, [0.1, 0.2],
                                   raw_loc=True)
    assert torch.equal(gc.cpu(), rc)
    assert torch.equal(gl.cpu(), rl)   # a copy of the truth corners: bit-exact
    assert torch.equal(glm.cpu(), rlm)


def _oracle_nms_many(bx, sc, thr):
    """oracle/nms_ref.c over several images in parallel threads (ctypes drops
    the GIL), so the full C5 check stays within seconds."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=len(bx)) as ex:
        return list(ex.map(lambda b: box_ref.nms(bx[b], sc[b], thr), range(len(bx))))


@pytest.mark.gpu
def test_nms_c5_full_config(cuda):
    """C5 (BASELINE configs[4]) at full size: 8 images x 100k clustered boxes
    (seed 99, the bench's input), every image bit-exact vs oracle/nms_ref.c."""
    from jabd_amd import ops, synth
    bx, sc = synth.nms_boxes(8, 100_000, seed=99)
    keep, nk = ops.batched_nms(torch.from_numpy(bx).to(cuda), torch.from_numpy(sc).to(cuda), 0.3)
    keep, nk = keep.cpu().numpy(), nk.cpu().numpy()
    refs = _oracle_nms_many(bx, sc, 0.3)
    for b in range(8):
        assert nk[b] == len(refs[b]), b
        assert np.array_equal(keep[b, : nk[b]], refs[b]), b


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [0.3, 0.9])
def test_nms_pair_capacity_dense_fallback(cuda, thr):
    """Image 0 is one tight cluster of 24k near-identical boxes: every pair is a
    grid candidate (n^2/2 = 2.9e8 pairs vs the image's pair capacity: each
    64-key wave's 8192 records plus the image's overflow region of 16 per row,
    csrc/nms.hip kPairsPerBox / kOvfPerBox: 3.5e6 in all), so its mask must
    come from the dense fallback producer; image 1 (ordinary clustered boxes)
    stays on the grid producer in the same call.  Both bit-exact vs the
    oracle, and the producers are the ones named (jabd_nms_pair_stats).
    (24k rows: the grid producer runs for images above csrc/nms.hip's
    20480-row dense limit.)"""
    from jabd_amd import ops, synth
    n = 24_000
    rng = np.random.default_rng(17)
    ctr = 0.5 + rng.normal(0, 0.002, (n, 2))
    wh = 0.1 * (1 + rng.uniform(0, 0.05, (n, 2)))
    b0 = np.concatenate([ctr - wh / 2, ctr + wh / 2], 1).astype(np.float32)
    s0 = rng.uniform(0.5, 1.0, n).astype(np.float32)
    b1, s1 = synth.nms_boxes(1, n, seed=23)
    bx = np.stack([b0, b1[0]])
    sc = np.stack([s0, s1[0]])
    keep, nk = ops.batched_nms(torch.from_numpy(bx).to(cuda), torch.from_numpy(sc).to(cuda), thr)
    keep, nk = keep.cpu().numpy(), nk.cpu().numpy()
    refs = _oracle_nms_many(bx, sc, thr)
    for b in range(2):
        assert np.array_equal(keep[b, : nk[b]], refs[b]), b
    _, _, _, dense = ops.batched_nms_stats(torch.from_numpy(bx).to(cuda),
                                           torch.from_numpy(sc).to(cuda), thr)
    assert dense.tolist() == [True, False]


@pytest.mark.gpu
@pytest.mark.parametrize("ncl", [300, 700])
def test_nms_cluster_stays_on_grid(cuda, ncl):
    """A mid-size cluster: ncl near-identical boxes of one face in
    a 24k-row image of ordinary clustered boxes.  They share one cell run of
    the grid key order, so the first key-order wave of the run holds 64 boxes
    that each pair with nearly every later cluster box: about 64 * (ncl - 32)
    off-block records (17k at 300, 43k at 700) against the wave's 8192.  The
    excess spills into the image's overflow region (csrc/nms.hip kOvfPerBox)
    and the image stays on the grid producer (before the spill it went dense:
    an O(n^2) mask for the whole image); bit-exact vs the oracle."""
    from jabd_amd import ops, synth
    n = 24_000
    b1, s1 = synth.nms_boxes(2, n, seed=29)
    bx, sc = b1.copy(), s1.copy()
    rng = np.random.default_rng(ncl)
    rows = rng.choice(n, ncl, replace=False)
    ctr = np.array([0.3, 0.6]) + rng.normal(0, 0.001, (ncl, 2))
    wh = 0.08 * (1 + rng.uniform(0, 0.02, (ncl, 2)))
    bx[0, rows] = np.concatenate([ctr - wh / 2, ctr + wh / 2], 1).astype(np.float32)
    refs = _oracle_nms_many(bx, sc, 0.5)
    # without the overflow region (JABD_NMS_OVF_PER_BOX=0) the cluster's wave
    # overflows and image 0 goes dense: the case exercises the spill
    for ovf, want in (("0", [True, False]), (None, [False, False])):
        with pytest.MonkeyPatch.context() as mp:
            if ovf is not None:
                mp.setenv("JABD_NMS_OVF_PER_BOX", ovf)
            keep, nk, tested, dense = ops.batched_nms_stats(torch.from_numpy(bx).to(cuda),
                                                            torch.from_numpy(sc).to(cuda), 0.5)
        assert dense.tolist() == want, (ovf, dense)
        keep, nk = keep.cpu().numpy(), nk.cpu().numpy()
        for b in range(2):
            assert np.array_equal(keep[b, : nk[b]], refs[b]), (ovf, b)
