"""JABD hot-path benchmark on MI355X (contract: see README / DESIGN.md §Measurement).

Step = one eval-mode forward of JABD-MobileNetV3 (nets/retinaface_r.py) on a
synthetic bs32 1024x1024 batch already resident in HBM (BASELINE.json
configs[1], "C2").  N GPUs run N independent replicas (inference does not
shard further; no collective on the data path) -> weak scaling; value =
images/sec over all ranks, timed as max over ranks between barriers.

Extra fields on the one JSON line:
  roofline     conv-GEMM stack (the dominant kernel family) vs the fp32 MFMA
               peak: algorithmic FLOPs of every jabd conv launch in one step /
               their summed HIP-event durations on the launch stream.
  nms          C5 (configs[4]): batched NMS over 8 x 100k clustered boxes,
               boxes/sec, bit-exact NMS kernel pipeline (sort+mask+scan).
  train        C4 (configs[3]): JABD-MobileNetV3 training step, 32 images/GPU
               at 1024x1024 (forward, MultiBoxLoss with on-device matching,
               backward, SUM gradient all-reduce over RCCL when N>1, fused Adam
               (csrc/adam.hip) wd 5e-4 as train_mobilenetV3_ecagai.py:564) on every rank ->
               whole-job images/sec, data-parallel weak scaling; at N=1 also
               C3 (configs[2]): R50 RetinaFace training step at bs64 1024x1024.
  predict_fps_bs1  the reference's own perf path: predict.py get_FPS (bs1,
               100 iterations of forward + decode + filter + NMS + host copy)
               at 640^2 and 1024^2 for the R50 and MNv3 detectors.
  c5_e2e       C5 end to end: bs8 2048^2 forward + decode + NMS.
  cpu_baseline the oracle's PyTorch-CPU restatement of the same forward at
               1024x1024, bs1, on this host (rank 0, N=1 only), plus legs
               (C1, C2/C3 forwards, C3/C4 training steps at bs1/bs4, C5 NMS).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

import torch  # noqa: E402

METRIC = "images/sec at 1024x1024 bs32 (1/2/4/8 GPU); boxes/sec NMS"
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak (spec)
# process-group backend of the N>1 path: RCCL ("nccl") on the GPU node; "gloo"
# rehearses the same control flow (tests/test_bench_dist.py)
DIST_BACKEND = os.environ.get("JABD_DIST_BACKEND", "nccl")
# 1: the training legs shard one global synthetic batch over the ranks and
# report the job's loss per step and every rank's parameter checksum
GLOBAL_DATA = os.environ.get("JABD_BENCH_GLOBAL_DATA", "0") == "1"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-nms", action="store_true")
    ap.add_argument("--no-predict", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--train-steps", type=int, default=10)
    ap.add_argument("--r50-batch", type=int, default=64)
    ap.add_argument("--pmc-forward-only", action="store_true",
                    help="run exactly --steps eval forwards and nothing else (PMC passes)")
    return ap.parse_args()


def build_model(device):
    from nets.retinaface_r import RetinaFace
    from nets.retinaface_training import weights_init
    from utils.config import cfg_mnet
    torch.manual_seed(0)
    m = RetinaFace(cfg=cfg_mnet, mode="eval")
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        weights_init(m)   # the training scripts' init (nets/retinaface_training.py:305-323)
    return m.eval().to(device)


def _expdw_work(xx, pk, k, stride, y, skip=False, pre=None):
    """(FLOPs, algorithmic bytes) of one fused expand+depthwise launch: the
    expand GEMM over every input pixel plus the k x k depthwise MACs; bytes =
    input read once + output written once + weights (+ the fused stride-2
    skip branch's dw3x3 MACs and output; + the previous block's fused project,
    pre: its 1x1 GEMM over every input pixel and its residual read)."""
    B, H, W, C = xx.shape
    E = pk.Cout
    flops = 2.0 * B * H * W * C * E + 2.0 * y.numel() * k * k
    nbytes = 4.0 * (xx.numel() + y.numel() + C * E + k * k * E)
    if skip:
        npx = y.shape[0] * y.shape[1] * y.shape[2]
        flops += 2.0 * npx * C * 9
        nbytes += 4.0 * npx * C
    if pre is not None:
        ppk = pre[0]
        flops += 2.0 * B * H * W * ppk.Cin * ppk.Cout
        nbytes += 4.0 * (pre[2].numel() + ppk.Cin * ppk.Cout)
    return flops, nbytes


def conv_roofline(model, x, steps):
    """Time every conv-stack launch of `steps` forwards with HIP events: the
    implicit-GEMM convs (F.conv) and the fused expand-GEMM + depthwise kernel
    (F.expand_dw).  Events are recorded on torch's current stream, which is the
    stream every libjabd launch uses."""
    from jabd_amd import functional as F
    from jabd_amd import engine as E
    recs = []
    orig, orig_xd = F.conv, F.expand_dw
    # per-kernel durations in isolation: one stream (the timed C2 loop splits
    # the batch over EVAL_STREAMS streams, where launches overlap)
    streams, E.EVAL_STREAMS = E.EVAL_STREAMS, 1

    def timed_conv(xx, pk, stride=1, pad=0, **kw):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig(xx, pk, stride=stride, pad=pad, **kw)
        e.record()
        o = out
        M = o.shape[0] * o.shape[1] * o.shape[2]
        K = pk.KH * pk.KW * pk.Cin + pk.Cin2
        # algorithmic bytes: input read once, weights once, output written once
        nbytes = 4.0 * (xx.numel() + (kw["x2"].numel() if kw.get("x2") is not None else 0)
                        + (kw["res"].numel() if kw.get("res") is not None else 0)
                        + K * pk.Cout + M * pk.Cout)
        recs.append((s, e, 2.0 * M * K * pk.Cout, nbytes))
        return out

    def timed_xd(xx, pk, w, b, k, stride, **kw):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig_xd(xx, pk, w, b, k, stride, **kw)
        e.record()
        recs.append((s, e) + _expdw_work(xx, pk, k, stride, out[0], kw.get("skip") is not None,
                                         kw.get("pre")))
        return out

    F.conv, F.expand_dw = timed_conv, timed_xd
    try:
        with torch.no_grad():
            for _ in range(steps):
                model(x)
        torch.cuda.synchronize()
    finally:
        F.conv, F.expand_dw = orig, orig_xd
        E.EVAL_STREAMS = streams
    t_ms = sum(r[0].elapsed_time(r[1]) for r in recs)
    flops = sum(r[2] for r in recs)
    nbytes = sum(r[3] for r in recs)
    n = len(recs) // steps
    return flops / steps, t_ms / steps, n, nbytes / steps


def r50_roofline(device, size, batch=16, steps=3):
    """Conv-stack roofline of the R50 RetinaFace (configs[2] model) eval forward:
    the compute-bound backbone of BASELINE.json's north-star conv target."""
    from nets.retinaface_eca_nonlocal import RetinaFace
    from nets.retinaface_training import weights_init
    from utils.config import cfg_re50
    from jabd_amd import synth
    import contextlib
    import io
    torch.manual_seed(0)
    m = RetinaFace(cfg=cfg_re50, mode="eval")
    with contextlib.redirect_stdout(io.StringIO()):
        weights_init(m)
    m = m.eval().to(device)
    x = synth.images(batch, size, seed=99, device=device)
    with torch.no_grad():
        for _ in range(2):
            m(x)
    torch.cuda.synchronize()
    flops, t_ms, n, nbytes = conv_roofline(m, x, steps)
    ach = flops / (t_ms * 1e-3) / 1e12
    del m, x
    torch.cuda.empty_cache()
    return {"bound": "mfma", "kernel": f"R50 RetinaFace eval forward conv stack ({n} launches)",
            "workload": f"bs{batch} {size}x{size}", "achieved": ach,
            "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_FP32_MFMA_TFLOPS,
            "conv_ms_per_step": t_ms, "conv_gflop_per_step": flops / 1e9}


def o1_activation_c2(device, x, steps, warmup):
    """C2 images/s with weights that keep activations O(1) through the network."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _util import init_for_parity
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="eval"), seed=1).eval().to(device)
    with torch.no_grad():
        for _ in range(warmup):
            m(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            m(x)
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    del m
    torch.cuda.empty_cache()
    return {"images_per_sec": x.shape[0] * steps / el, "ms_per_step": el / steps * 1e3,
            "init": "tests/_util.py init_for_parity (conv weights N(0, 1/fan_in), BN running "
                    "stats non-trivial)"}


def forward_flops(size, batch, device):
    """Algorithmic FLOPs (2*MAC) of the JABD-MobileNetV3 eval forward: the
    same census as the training floor (activation_census: every conv-like
    launch -- stem, convs, fused expand+depthwise incl. its skip branch,
    depthwise convs, heads and the fused SSH tail's three 3x3 convs and three
    heads), so the bench line carries one forward GFLOP/image (VERDICT r05
    item 8).  Not counted: the NLM attention (S = 225 bins x C = 4 channels per
    pixel, < 0.1% of the forward) and elementwise work."""
    return batch * activation_census("mnv3", device, size)["flops"]


NMS_OPS_PER_PAIR = 13  # fp32 ops of one exact IoU test: 4 min/max, 2 sub, 2 clamp, mul, 2 add/sub, div, cmp


def nms_bench(device, reps=5):
    """C5: batched NMS over 8 x 100k clustered boxes (seed 99), boxes/s; the IoU
    tests the pair search made (kernel counters, jabd_nms_pair_stats) as
    pairs/s against the non-FMA VALU op rate (the scan after it is
    latency-bound)."""
    from jabd_amd import ops, synth
    from oracle import box_ref
    B, n = 8, 100_000
    bx, sc = synth.nms_boxes(B, n, seed=99)
    b = torch.from_numpy(bx).to(device)
    s = torch.from_numpy(sc).to(device)
    keep, nk = ops.batched_nms(b, s, 0.3)   # warm-up + parity spot check (image 0)
    torch.cuda.synchronize()
    ref0 = box_ref.nms(bx[0], sc[0], 0.3)
    exact = keep[0, : int(nk[0])].cpu().numpy().tolist() == ref0.tolist()
    _, _, tested, dense = ops.batched_nms_stats(b, s, 0.3)
    t0 = time.perf_counter()
    for _ in range(reps):
        ops.batched_nms(b, s, 0.3)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    pairs = int(tested.sum())
    pps = pairs / dt
    return {"config": "C5: 8 images x 100k clustered boxes, iou 0.3", "boxes_per_sec":
            B * n / dt, "ms_per_call": dt * 1e3, "kept_img0": int(nk[0]),
            "bit_exact_img0_vs_oracle": bool(exact),
            "iou_pairs_tested_per_image": [int(v) for v in tested],
            "dense_fallback_images": int(dense.sum()),
            "all_pairs_per_image": n * (n - 1) // 2,
            "iou_pairs_per_sec": pps, "ops_per_pair": NMS_OPS_PER_PAIR,
            # the IoU test's 13 ops are not FMAs: 64 lanes x 1 op per SIMD
            # clock, half the FMA-counted 157.3 TFLOP/s vector peak
            "valu_peak_tops_non_fma": PEAK_FP32_MFMA_TFLOPS / 2,
            "valu_frac": pps * NMS_OPS_PER_PAIR / (PEAK_FP32_MFMA_TFLOPS / 2 * 1e12),
            "algorithmic_bytes": B * (20 * n + 8 * int(nk.sum()) // B),
            "note": "bytes = 20 B read per box + 8 B per kept index; sort/scan passes extra"}


def augment_bench(device, reps=20):
    """§8f rank 2: get_random_data's image path (jabd_augment_u8) for one
    768x1024 RGB source onto a 1024x1024 canvas, timed with HIP events on the
    current stream.  Algorithmic bytes: source u8 read + the u8 horizontal
    intermediate written and read + fp32 CHW output written."""
    from jabd_amd import ops
    ih, iw, h, w = 768, 1024, 1024, 1024
    nw, nh = 900, 700
    img = torch.randint(0, 256, (ih, iw, 3), dtype=torch.uint8, device=device)
    args = ((h, w), nw, nh, 50, 100, True, 0.05, 1.2, 0.9)
    ops.augment(img, *args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.augment(img, *args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = ih * iw * 3 + 2 * ih * nw * 3 + 3 * h * w * 4
    return {"config": "768x1024 u8 RGB -> 1024x1024 (resize 900x700, flip, HSV jitter)",
            "images_per_sec": 1e3 / ms, "ms_per_call": ms,
            "algorithmic_bytes": nbytes, "achieved_gbs": nbytes / (ms * 1e-3) / 1e9}


def _weights_init_model(kind, mode="eval"):
    import contextlib
    import io
    from nets.retinaface_training import weights_init
    RetinaFace, cfg = detector(kind)
    torch.manual_seed(0)
    m = RetinaFace(cfg=cfg, mode=mode)
    with contextlib.redirect_stdout(io.StringIO()):
        weights_init(m)
    return m, cfg


def predict_fps(device, iters=100, warmup=10):
    """The reference's own performance path, predict.py mode 'fps'
    (get_FPS, predict.py:253-333, test_interval=100 at :522-526): bs1, the
    letterboxed network input prepared once, then per iteration the forward,
    decode, conf[:, 1:2], decode_landm, cat and non_max_suppression (score
    >= 0.5, NMS 0.3) with the kept rows handed back to the host — here the
    eval forward + jabd_detect_f32 + one device-to-host copy of the kept
    rows.  `detect_image_fps` is the whole detect_image per call (host image
    upload, letterbox + preprocess, forward, detect, correct_boxes, host
    copy).  R50 is the detector predict.py loads (nets/retinaface_eca_nonlocal,
    predict.py:15,101); JABD-MobileNetV3 beside it.  Weights: weights_init."""
    import numpy as np
    from jabd_amd import functional as F
    from jabd_amd import ops
    from jabd_amd.predict import PREDICT_GRAPH as graphs
    from jabd_amd.predict import detect_image, graphed_detect
    from utils.anchors import Anchors
    out = {}
    for kind in ("r50", "mnv3"):
        net, cfg = _weights_init_model(kind)
        net = net.eval().to(device)
        for size in (640, 1024):
            img = np.random.default_rng(size).integers(0, 256, (size * 3 // 4, size, 3)) \
                .astype(np.float32)
            x = ops.letterbox(torch.from_numpy(img).to(device), (size, size),
                              mean=(104.0, 117.0, 123.0))
            pri = Anchors(cfg, image_size=(size, size)).get_anchors().to(device).float()
            var = cfg["variance"]

            def step_eager():
                with torch.no_grad():
                    with F.split_k():
                        loc, conf, landm = net(x)
                    rows, nk = ops.detect(loc, conf, landm, pri, var, 0.5, 0.3)
                    k = int(nk[0].item())
                    return rows[0, :k].cpu().numpy()

            def step():   # the same work, replayed as one HIP graph (opt-in, jabd_amd.predict)
                with torch.no_grad():
                    rows, nk = graphed_detect(net, x, pri, var, 0.5, 0.3)
                    k = int(nk[0].item())
                    return rows[0, :k].cpu().numpy()
            for _ in range(warmup):
                step_eager()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                kept_e = step_eager()
            el_e = time.perf_counter() - t0
            kept, el = kept_e, el_e
            if graphs:
                for _ in range(warmup):
                    step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(iters):
                    kept = step()
                el = time.perf_counter() - t0
                assert np.array_equal(kept, kept_e), "graph replay differs from the eager launches"
            for _ in range(3):
                detect_image(net, img, (size, size), cfg, 0.5, 0.3)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(iters // 2):
                detect_image(net, img, (size, size), cfg, 0.5, 0.3)
            el2 = time.perf_counter() - t1
            with torch.no_grad():
                cand = int((net(x)[1][0, :, 1] >= 0.5).sum())
            out[f"{kind}_{size}"] = {
                "fps": iters / el, "ms_per_image": el / iters * 1e3,
                "fps_eager_launches": iters / el_e, "graph": bool(graphs),
                "detect_image_fps": (iters // 2) / el2, "iters": iters,
                "anchors": int(pri.shape[0]), "candidates_ge_0.5": cand,
                "kept": int(kept.shape[0])}
        del net
        torch.cuda.empty_cache()
    out["note"] = ("bs1 wall clock per iteration (host-side launch/ctypes/n_keep sync costs "
                   "included), as get_FPS; fps: forward + detect replayed as one HIP graph "
                   "(jabd_amd.predict.graphed_detect; kept rows checked equal to the eager "
                   "launches, which fps_eager_launches times; JABD_PREDICT_GRAPH=0: eager only); "
                   "split-K "
                   "on for the bs1 forward (functional.split_k; off in batched eval); "
                   "weights_init weights put ~half the anchors at a conf of ~0.5, so NMS runs "
                   "over thousands of candidates")
    return out


def c5_e2e(device, batch=8, size=2048, steps=5, warmup=2):
    """C5 end to end (BASELINE configs[4]): JABD-MobileNetV3 eval forward on a
    bs8 2048x2048 batch + jabd_detect_f32 (decode, >= 0.5 filter, NMS 0.3)
    over its 172,032 anchors per image, timed between synchronisations."""
    from jabd_amd import ops, synth
    from utils.anchors import Anchors
    net, cfg = _weights_init_model("mnv3")
    net = net.eval().to(device)
    x = synth.images(batch, size, seed=99, device=device)
    pri = Anchors(cfg, image_size=(size, size)).get_anchors().to(device).float()
    var = cfg["variance"]
    with torch.no_grad():
        for _ in range(warmup):
            rows, nk = ops.detect(*net(x), pri, var, 0.5, 0.3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            rows, nk = ops.detect(*net(x), pri, var, 0.5, 0.3)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps
        loc, conf, landm = net(x)
        cand = (conf[:, :, 1] >= 0.5).sum(1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(steps):
            ops.detect(loc, conf, landm, pri, var, 0.5, 0.3)
        torch.cuda.synchronize()
        el_det = (time.perf_counter() - t1) / steps
    del net
    torch.cuda.empty_cache()
    A = int(pri.shape[0])
    return {"config": f"C5: JABD-MobileNetV3 eval forward bs{batch} {size}x{size} + decode + "
                      f">=0.5 filter + NMS 0.3 (jabd_detect_f32), weights_init weights",
            "images_per_sec": batch / el, "ms_per_batch": el * 1e3,
            "detect_ms_per_batch": el_det * 1e3, "anchors_per_image": A,
            "boxes_per_sec": batch * A / el,
            "nms_candidates_per_image": [int(v) for v in cand],
            "kept_per_image": [int(v) for v in nk]}


def detector(kind):
    """(RetinaFace class, cfg) of a detector kind: mnv3 (JABD-MobileNetV3),
    beca (JABD-MobileNetV3-BECA), small (MobileNetV3_Small + ECA head), r50."""
    from utils import config
    if kind == "mnv3":
        from nets.retinaface_r import RetinaFace
        return RetinaFace, config.cfg_mnet
    if kind == "beca":
        from nets.retinaface_beca import RetinaFace
        return RetinaFace, config.cfg_mnet
    if kind == "small":
        from nets.retinaface_r import RetinaFace_Small
        return RetinaFace_Small, config.cfg_mnv3_small
    from nets.retinaface_eca_nonlocal import RetinaFace
    return RetinaFace, config.cfg_re50


def variant_forward(kind, device, size, batch, steps, warmup=2):
    """Eval-forward images/s of a detector variant at the C2 shape (synthetic
    input, weights_init weights): the f4 rows (BECA, MobileNetV3_Small)."""
    from jabd_amd import synth
    from nets.retinaface_training import weights_init
    import contextlib
    import io
    RetinaFace, cfg = detector(kind)
    torch.manual_seed(0)
    m = RetinaFace(cfg=cfg, mode="eval")
    with contextlib.redirect_stdout(io.StringIO()):
        weights_init(m)
    m = m.eval().to(device)
    x = synth.images(batch, size, seed=99, device=device)
    with torch.no_grad():
        for _ in range(warmup):
            m(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            m(x)
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"workload": f"{kind} eval forward bs{batch} {size}x{size}",
            "images_per_sec": batch * steps / el, "ms_per_step": el / steps * 1e3}


def train_bench(kind, batch, size, steps, warmup, device, dist, rank, conv_roofline_steps=0):
    """steps timed training iterations (parallel.train_step) on this rank."""
    from jabd_amd import optim, parallel, synth
    from nets.retinaface_training import MultiBoxLoss, weights_init
    from utils.anchors import Anchors
    import contextlib
    import io
    RetinaFace, cfg = detector(kind)
    torch.manual_seed(0)
    model = RetinaFace(cfg=cfg, mode="train")
    with contextlib.redirect_stdout(io.StringIO()):
        weights_init(model)
    model = model.to(device).train()
    if dist:
        parallel.broadcast_buffers(model)
        for p in model.parameters():
            dist.broadcast(p.data, src=0)
    opt = optim.Adam(model.parameters(), 1e-3, weight_decay=5e-4)  # fused HIP step
    crit = MultiBoxLoss(2, 0.35, 7, cfg["variance"], True)
    pri = Anchors(cfg, image_size=(size, size)).get_anchors().to(device)
    world = dist.get_world_size() if dist else 1
    if GLOBAL_DATA:
        # every rank synthesises the same global batch and takes its shard
        # (parallel.shard, DataParallel's scatter): the job then sees one
        # global batch, comparable with a one-process run of it
        gx = synth.images(batch * world, size, seed=1234, device=device)
        gt = [torch.from_numpy(t).to(device) for t in synth.targets(batch * world, size, seed=4321)]
        x, tg = parallel.shard(gx, gt, rank, world)
        x = x.contiguous()
        del gx, gt
    else:
        x = synth.images(batch, size, seed=1234 + rank, device=device)
        tg = [torch.from_numpy(t).to(device) for t in synth.targets(batch, size, seed=4321 + rank)]
    reducer = parallel.GradAllReduce(model) if dist else None
    trace = []

    def step():
        loss, _ = parallel.train_step(model, crit, opt, x, tg, pri, reducer=reducer)
        if GLOBAL_DATA:
            trace.append(loss)
        return loss

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    conv = None
    if conv_roofline_steps:
        with TrainConvTimer() as tm:
            for _ in range(conv_roofline_steps):
                step()
        c_ms, c_gf, c_n = tm.summary(conv_roofline_steps)
        ach = c_gf / c_ms  # GFLOP/ms = TFLOP/s
        conv = {"bound": "mfma", "kernel": f"training-step conv stack: forward, data-gradient "
                f"and weight-gradient convolutions ({c_n} launches/step)",
                "workload": f"{kind} training bs{batch} {size}x{size}", "achieved": ach,
                "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / PEAK_FP32_MFMA_TFLOPS, "conv_ms_per_step": c_ms,
                "conv_gflop_per_step": c_gf}
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        # the job's loss of the last step: each rank's loss is its shard's part
        # of the global-batch loss (global positive counts), so the sum over
        # ranks is DataParallel's loss (outside the timed region)
        loss = loss.detach().clone()
        dist.all_reduce(loss)
    mem = torch.cuda.max_memory_allocated(device) / 2**30
    extra = {}
    if GLOBAL_DATA:
        tr = torch.stack(trace).double()
        ck = torch.stack([p.detach().double().sum() for p in model.parameters()]).sum().reshape(1)
        if dist:
            dist.all_reduce(tr)
            cks = [torch.zeros_like(ck) for _ in range(world)]
            dist.all_gather(cks, ck)
            ck = torch.cat(cks)
        extra = {"loss_trace": tr.cpu().tolist(), "param_checksums": ck.cpu().tolist()}
    del model, opt, x, tg
    torch.cuda.empty_cache()
    out = {"images_per_sec": batch * steps * world / el, "ms_per_step": el / steps * 1e3,
           "per_gpu_batch": batch, "global_batch": batch * world, "image_size": size,
           "steps": steps, "warmup": warmup, "loss_last": float(loss), "max_mem_gib": mem}
    out.update(extra)
    if conv is not None:
        out["conv_roofline"] = conv
    return out


class TrainConvTimer:
    """HIP events around every libjabd convolution call of a training step
    (forward conv, data-gradient conv, weight-gradient kernel), on torch's
    current stream (the launch stream); algorithmic FLOPs from the call's
    jabd_conv_args: 2 * pixels * (KH*KW*Cin + Cin2) * Cout of the forward
    convolution each call computes or differentiates."""
    NAMES = ("jabd_conv2d_nhwc_f32", "jabd_conv_wgrad_f32")

    def __init__(self):
        self.recs = []

    def __enter__(self):
        from jabd_amd import functional, train, _lib
        self.mods = (functional, train)
        self.orig = _lib.call

        def timed(name, *args):
            if name not in self.NAMES:
                return self.orig(name, *args)
            a = args[0]._obj
            if name == "jabd_conv_wgrad_f32" or not a.tconv:
                px = a.B * a.OH * a.OW
                flops = 2.0 * px * (a.KH * a.KW * a.Cin + a.Cin2) * a.Cout
            else:  # data gradient of a stride-s conv: x = dY (H x W), out = dX
                flops = 2.0 * a.B * a.H * a.W * a.KH * a.KW * a.Cin * a.Cout
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            r = self.orig(name, *args)
            e1.record()
            self.recs.append((e0, e1, flops))
            return r
        for m in self.mods:
            m.call = timed
        return self

    def __exit__(self, *exc):
        for m in self.mods:
            m.call = self.orig

    def summary(self, steps):
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b, _ in self.recs) / steps
        gf = sum(f for _, _, f in self.recs) / steps / 1e9
        return ms, gf, len(self.recs) // steps


def pmc_traffic():
    """Conv-GEMM HBM bytes per step from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py -> profiles/<round>/pmc_traffic.json), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        return json.load(f)


def activation_census(kind, device, size):
    """Pass-independent work of one training image: the
    forward conv FLOPs and the bytes of every conv output the reference's
    module graph holds, counted from ONE bs1 eval forward of the same
    architecture through wrappers of the conv entry points (F.conv, F.stem,
    F.expand_dw, F.dwconv, F.heads) — whatever the kernels fuse, each reference
    conv is counted once:
      * F.conv: B*OH*OW*Cout output; a K-concatenated second source (the
        stride-2 block's 1x1 skip conv, nets/mobilenetV3.py:126-137) is a
        second reference conv with an output of the same size;
      * F.expand_dw: the expand 1x1 output (B*H*W*E), the depthwise output and,
        fused, the skip branch's dw3x3/s2 output;
      * F.heads: the loc/conf/landm rows.
    FLOPs: 2 MACs per conv tap, depthwise included (_expdw_work's count for
    the fused kernel)."""
    from jabd_amd import functional as F
    if kind == "mnv3":
        m = build_model(device)
    else:
        from nets.retinaface_eca_nonlocal import RetinaFace
        from utils.config import cfg_re50
        torch.manual_seed(0)
        m = RetinaFace(cfg=cfg_re50, mode="eval").eval().to(device)
    tot = {"act_bytes": 0.0, "convs": 0, "flops": 0.0, "stem_flops": 0.0}
    names = ("conv", "stem", "expand_dw", "dwconv", "heads", "ssh_tail_heads")
    orig = {n: getattr(F, n) for n in names}

    def add(nel):
        tot["act_bytes"] += 4.0 * nel
        tot["convs"] += 1

    def w_conv(xx, pk, stride=1, pad=0, **kw):
        out = orig["conv"](xx, pk, stride=stride, pad=pad, **kw)
        B = xx.shape[0]
        H, W = (xx.shape[2], xx.shape[3]) if kw.get("nchw_in") else (xx.shape[1], xx.shape[2])
        OH = (H + 2 * pad - pk.KH) // stride + 1
        OW = (W + 2 * pad - pk.KW) // stride + 1
        M = B * OH * OW
        add(M * pk.Cout)
        fl = 2.0 * M * pk.KH * pk.KW * pk.Cin * pk.Cout
        if kw.get("x2") is not None:
            add(M * pk.Cout)
            fl += 2.0 * M * pk.Cin2 * pk.Cout
        tot["flops"] += fl
        if kw.get("nchw_in"):
            tot["stem_flops"] += fl
        return out

    def w_stem(xx, w, bias, act):
        y = orig["stem"](xx, w, bias, act)
        add(y.numel())
        fl = 2.0 * y.numel() * 27
        tot["flops"] += fl
        tot["stem_flops"] += fl
        return y

    def w_xd(xx, pk, w, b, k, stride, **kw):
        out = orig["expand_dw"](xx, pk, w, b, k, stride, **kw)
        if kw.get("pre") is not None:   # the previous block's project output (kept on chip)
            add(xx.numel())
        add(xx.shape[0] * xx.shape[1] * xx.shape[2] * pk.Cout)
        add(out[0].numel())
        if kw.get("skip") is not None:
            add(out[2].numel())
        tot["flops"] += _expdw_work(xx, pk, k, stride, out[0], kw.get("skip") is not None,
                                    kw.get("pre"))[0]
        return out

    def w_dw(xx, w, bias, k, stride, **kw):
        out = orig["dwconv"](xx, w, bias, k, stride, **kw)
        y = out[0] if isinstance(out, tuple) else out
        add(y.numel())
        tot["flops"] += 2.0 * y.numel() * k * k
        return out

    def w_heads(xx, wt, bias, loc, conf, landm, a_off, softmax):
        r = orig["heads"](xx, wt, bias, loc, conf, landm, a_off, softmax)
        npx = xx.shape[0] * xx.shape[1] * xx.shape[2]
        n_out = wt.numel() // xx.shape[3] if wt.numel() % xx.shape[3] == 0 else 32
        add(npx * n_out)
        tot["flops"] += 2.0 * npx * xx.shape[3] * n_out
        return r

    def w_ssh(c33, t, wb, leaky, loc, conf, landm, a_off, softmax):
        # the fused SSH tail + heads of one level (csrc/ssh.hip): the reference's
        # conv5X5_2, conv7X7_2, conv7x7_3 (C/4 -> C/4, 3x3) and the three 1x1 heads
        r = orig["ssh_tail_heads"](c33, t, wb, leaky, loc, conf, landm, a_off, softmax)
        npx = c33.shape[0] * c33.shape[1] * c33.shape[2]
        C = 2 * c33.shape[3]
        q = C // 4
        n_out = loc.shape[2] + conf.shape[2] + landm.shape[2]   # per anchor
        A = 2                                                  # anchors per position (cfg min_sizes)
        add(npx * (3 * q + n_out * A))
        tot["flops"] += npx * (3 * 2.0 * 9 * q * q + 2.0 * C * n_out * A)
        tot["convs"] += 5   # (add() counted one)
        return r

    for n, f in zip(names, (w_conv, w_stem, w_xd, w_dw, w_heads, w_ssh)):
        setattr(F, n, f)
    try:
        x = torch.randn(1, 3, size, size, device=device)
        tot["act_bytes"] += 4.0 * x.numel()   # the network input
        with torch.no_grad():
            m(x)
        torch.cuda.synchronize()
    finally:
        for n in names:
            setattr(F, n, orig[n])
    del m
    return tot


def step_floor(kind, device, size, batch, step_ms):
    """Pass-independent floor of one training step:
         floor_ms = conv_flops / 157.3 TFLOP/s + 4 * act_bytes / 8 TB/s
    with conv_flops = 3 x the forward conv FLOPs (forward, data gradient,
    weight gradient) minus the first conv's data gradient (the image needs
    none), and act_bytes = every reference conv output of the step's batch:
    one write and one read in the forward, one write and one read of its
    gradient in the backward.  Independent of how many passes the
    implementation makes; frac_floor = floor_ms / step_ms."""
    c = activation_census(kind, device, size)
    conv_flops = batch * (3.0 * c["flops"] - c["stem_flops"])
    act_bytes = batch * c["act_bytes"]
    f_ms = conv_flops / (PEAK_FP32_MFMA_TFLOPS * 1e12) * 1e3
    b_ms = 4.0 * act_bytes / (PEAK_HBM_GBS * 1e9) * 1e3
    return {"formula": "conv_flops / %.1f TFLOP/s + 4 * act_bytes / %.0f TB/s"
                       % (PEAK_FP32_MFMA_TFLOPS, PEAK_HBM_GBS / 1000),
            "conv_flops": conv_flops, "act_bytes": act_bytes, "reference_convs": c["convs"],
            "flop_ms": f_ms, "byte_ms": b_ms, "floor_ms": f_ms + b_ms,
            "frac_floor": (f_ms + b_ms) / step_ms}


def step_roofline(name, step_ms, workload):
    """Training-step roofline: the sum over the step's libjabd launches of
    max(algorithmic FLOPs / fp32 MFMA peak, algorithmic bytes / HBM peak),
    measured per launch by tools/train_roofline.py (committed as
    profiles/<round>/<name>.json), divided by this run's step time."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name + ".json")))
    if not files:
        return None
    with open(files[-1]) as f:
        r = json.load(f)
    if r.get("workload") != workload:
        return None
    return {"bound": "per launch max(FLOP / %.1f TFLOP/s, bytes / %.0f TB/s), summed" %
                     (r["peak_tflops"], r["peak_tbs"]),
            "roof_ms": r["roof_ms"], "step_ms": step_ms, "frac": r["roof_ms"] / step_ms,
            "launches": r["calls"], "workload": r["workload"],
            "source": os.path.relpath(files[-1], ROOT)}


def host_cores():
    """CPU budget of the CPU baseline: BASELINE.md asks for
    torch.set_num_threads(<physical cores>); the threads used are
    min(physical cores, CPUs in this process's affinity mask, the cgroup CPU
    quota) — on the GPU box the job's share of the host is a quota, not the
    affinity mask.  Returns (threads, info dict)."""
    import math
    import subprocess
    phys = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = dict(l.split(":", 1) for l in out.splitlines() if ":" in l)
        phys = int(kv["Core(s) per socket"].strip()) * int(kv["Socket(s)"].strip())
    except Exception:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except Exception:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except Exception:
            pass
    cands = [v for v in (phys, aff, math.floor(quota) if quota else None) if v]
    threads = max(1, min(cands)) if cands else torch.get_num_threads()
    return threads, {"host_physical_cores": phys, "affinity_cpus": aff,
                     "cgroup_cpu_quota": quota,
                     "threads_rule": "min(physical cores, affinity CPUs, cgroup CPU quota)"}


def _time_bounded(fn, seconds, min_iters=1, warm=True):
    if warm:
        fn()  # warm-up
    n, t0 = 0, time.perf_counter()
    while n < min_iters or time.perf_counter() - t0 < seconds:
        fn()
        n += 1
    return n, time.perf_counter() - t0


def _cpu_train_step(fn, sd, cfg, size, batch, seed):
    """One training step of the oracle on the CPU (train_mobilenetV3_ecagai.py:
    518-533): batch-stat forward, match + MultiBoxLoss (oracle/box_ref.py),
    loss = 2 * loss_l + loss_c + loss_landm, autograd backward, Adam (lr 1e-3,
    weight_decay 5e-4, as :564) over the parameters."""
    from jabd_amd import synth
    from oracle import box_ref
    P = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
             else v.clone()) for k, v in sd.items()}
    params = [v for v in P.values() if isinstance(v, torch.Tensor) and v.requires_grad]
    opt = torch.optim.Adam(params, 1e-3, weight_decay=5e-4)
    pri = box_ref.anchors(cfg, (size, size))
    x = synth.images(batch, size, seed=seed)
    tg = [torch.from_numpy(t) for t in synth.targets(batch, size, seed=seed)]

    def step():
        opt.zero_grad()
        loc, conf, landm = fn(P, x, "train", train_bn=True)
        lt, ct, lmt = box_ref.match_batch(tg, pri)
        rl, rc, rlm, _ = box_ref.multibox_loss(loc, conf, landm, lt, ct, lmt)
        (2.0 * rl + rc + rlm).backward()
        opt.step()
    return step


def cpu_baseline(size, seconds):
    """The oracle's PyTorch-CPU restatement timed on this host (rank 0, N=1):
    headline leg C2 (MNv3 eval forward, bs1 1024^2) plus the legs BASELINE.md
    plans — C1 end to end (640^2 bs1: preprocess, forward, decode, score
    filter, torchvision-CPU NMS), C2/C3 forwards at bs4, C3 (R50) at bs1, the
    C3 (R50) and C4 (MNv3) training steps at bs1 and bs4, and C5's NMS over
    one 100k-box image (oracle/nms_ref.c) — each a bounded sample."""
    from oracle import box_ref, model_ref, prep_ref
    from nets.retinaface_r import RetinaFace
    from nets.retinaface_eca_nonlocal import RetinaFace as R50
    from nets.retinaface_training import weights_init
    from utils.config import cfg_mnet, cfg_re50
    from jabd_amd import synth
    import contextlib
    import io
    import numpy as np
    threads, info = host_cores()
    saved_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        m = RetinaFace(cfg=cfg_mnet, mode="eval")
        weights_init(m)
        r = R50(cfg=cfg_re50, mode="eval")
        weights_init(r)
    sd = {k: v.float() for k, v in m.eval().state_dict().items()}
    sdr = {k: v.float() for k, v in r.eval().state_dict().items()}
    legs = {}
    try:
        with torch.no_grad():
            x1 = synth.images(1, size, seed=1234)
            n, dt = _time_bounded(lambda: model_ref.retinaface_mnv3(sd, x1), seconds)
            head = {"value": n / dt, "unit": "images/sec", "cores": threads, **info,
                    "kind": "port",
                    "sample": f"{n} images, bs1 {size}x{size}, oracle model_ref.retinaface_mnv3 "
                              "(PyTorch-CPU fp32 restatement)"}
            x4 = synth.images(4, size, seed=1234)
            n, dt = _time_bounded(lambda: model_ref.retinaface_mnv3(sd, x4), 3.0)
            legs["C2_mnv3_bs4"] = {"images_per_sec": 4 * n / dt, "batches": n}
            n, dt = _time_bounded(lambda: model_ref.retinaface_r50(sdr, x1), 3.0)
            legs["C3_r50_bs1"] = {"images_per_sec": n / dt, "batches": n}
            n, dt = _time_bounded(lambda: model_ref.retinaface_r50(sdr, x4), 3.0)
            legs["C3_r50_bs4"] = {"images_per_sec": 4 * n / dt, "batches": n}
            img = np.random.default_rng(640).integers(0, 256, (480, 640, 3)).astype(np.float32)
            pri = box_ref.anchors(cfg_mnet, (640, 640))

            def c1():
                xx = torch.from_numpy(prep_ref.preprocess(img, (640, 640)))[None]
                loc, conf, landm = model_ref.retinaface_mnv3(sd, xx, "eval")
                det = torch.cat([box_ref.decode(loc[0], pri, cfg_mnet["variance"]),
                                 conf[0][:, 1:2],
                                 box_ref.decode_landm(landm[0], pri, cfg_mnet["variance"])], -1)
                rows = box_ref.non_max_suppression(det, 0.5, 0.3)
                if len(rows):
                    prep_ref.correct_rows(np.asarray(rows, np.float32), (640, 640), (480, 640))
            n, dt = _time_bounded(c1, 3.0)
            legs["C1_detect_image_640"] = {"images_per_sec": n / dt, "images": n,
                                           "stages": "letterbox+preprocess, forward, decode, "
                                                     ">=0.5 filter, NMS 0.3, correct_boxes"}
        # training steps ("the training step for C3", bs 1 and 4)
        for name, fn, sdd, cfg in (("C4_mnv3_train", model_ref.retinaface_mnv3, sd, cfg_mnet),
                                   ("C3_r50_train", model_ref.retinaface_r50, sdr, cfg_re50)):
            for bs in (1, 4):
                step = _cpu_train_step(fn, sdd, cfg, size, bs, 4321)
                # seconds per step already: no separate warm-up step
                n, dt = _time_bounded(step, 3.0, warm=False)
                legs[f"{name}_bs{bs}"] = {
                    "images_per_sec": bs * n / dt, "steps": n,
                    "step": "batch-stat forward, match + MultiBoxLoss (OHEM 7:1), backward, "
                            "Adam wd 5e-4 (train_mobilenetV3_ecagai.py:518-533)"}
        bx, sc = synth.nms_boxes(1, 100_000, seed=99)
        n, dt = _time_bounded(lambda: box_ref.nms(bx[0], sc[0], 0.3), 1.0)
        legs["C5_nms_100k"] = {"boxes_per_sec": 100_000 * n / dt, "images": n,
                               "kind": "oracle/nms_ref.c (torchvision-CPU NMS restated in C), "
                                       "1 thread"}
    finally:
        torch.set_num_threads(saved_threads)
    head["legs"] = legs
    return head


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # ranks beyond the visible devices share them (a gloo rehearsal of the
        # N>1 path on a one-GPU box); on the 8-GPU node this is rank -> GPU
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(DIST_BACKEND)
    device = torch.device("cuda", local)
    from jabd_amd import synth
    model = build_model(device)
    x = synth.images(args.batch, args.size, seed=1234 + rank, device=device)
    if args.pmc_forward_only:
        # one stream, as conv_roofline times the kernels (rocprof durations of
        # overlapping launches would include each other's contention)
        from jabd_amd import engine as E
        E.EVAL_STREAMS = 1
        with torch.no_grad():
            for _ in range(args.steps):
                model(x)
        torch.cuda.synchronize()
        return

    with torch.no_grad():
        for _ in range(args.warmup):
            model(x)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(args.steps):
            model(x)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    n_gpus = world
    imgs = args.batch * args.steps * n_gpus
    value = imgs / el

    extra = {}
    if rank == 0:
        # conv-stack roofline on the C2 model right after its timed loop (before
        # the training legs reshuffle the allocator)
        flops_step, t_ms, n_launch, alg_bytes = conv_roofline(model, x, max(3, min(args.steps, 10)))
        ach = flops_step / (t_ms * 1e-3) / 1e12
        pmc = pmc_traffic()
        extra["roofline"] = {
            "bound": "mfma",
            "kernel": f"conv stack: conv_gemm/conv1x1 + fused expand_dw ({n_launch} launches/step)",
            "achieved": ach, "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / PEAK_FP32_MFMA_TFLOPS,
            "traffic": pmc["conv_hbm_bytes_per_step"] if pmc else None,
            "traffic_unit": "HBM bytes per step over the conv-stack launches (PMC, "
                            "2*FETCH_SIZE + WRITE_SIZE, see DESIGN.md)",
            "traffic_source": pmc["source"] if pmc else None,
            "algorithmic_bytes_per_step": alg_bytes,
            "achieved_hbm_gbs": alg_bytes / (t_ms * 1e-3) / 1e9,
            "hbm_frac": alg_bytes / (t_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
            "conv_ms_per_step": t_ms, "conv_gflop_per_step": flops_step / 1e9}
        # the same C2 step with O(1)-activation weights (tests/_util.py init):
        # weights_init's N(0, 0.02) convs make deep activations vanish, and
        # MFMA loops over near-zero data hold higher clocks (DVFS)
        extra["c2_o1_activations"] = o1_activation_c2(device, x, args.steps, args.warmup)
        if world == 1 and args.r50_batch > 0:
            extra["roofline_r50_eval"] = r50_roofline(device, args.size)
        if world == 1:
            extra["variants"] = {k: variant_forward(k, device, args.size, args.batch, 5)
                                 for k in ("beca", "small")}
    if not args.no_train:
        # every rank runs the conv-timer step: it is a full training step whose
        # backward all-reduces the gradients, so all ranks must take it (a
        # rank-0-only extra step would leave its RCCL all-reduces unmatched);
        # only rank 0 reports it
        tr = {"C4_mnv3": train_bench("mnv3", args.batch, args.size, args.train_steps, 3, device,
                                     dist, rank, conv_roofline_steps=1)}
        if world == 1 and args.r50_batch > 0:
            tr["C3_r50"] = train_bench("r50", args.r50_batch, args.size, max(2, args.train_steps // 2),
                                       2, device, None, rank, conv_roofline_steps=1)
            extra["roofline_r50"] = tr["C3_r50"].get("conv_roofline")
        for k, fn, kind, b in (("C4_mnv3", "c4_step_roofline", "mnv3", args.batch),
                               ("C3_r50", "c3_step_roofline", "r50", args.r50_batch)):
            if k in tr:
                tr[k]["roofline"] = step_roofline(
                    fn, tr[k]["ms_per_step"], f"{kind} training bs{b} {args.size}x{args.size}")
                if rank == 0:
                    fl = step_floor(kind, device, args.size, b, tr[k]["ms_per_step"])
                    if tr[k]["roofline"] is None:
                        tr[k]["roofline"] = {}
                    tr[k]["roofline"].update(fl)
        extra["train"] = tr
    if rank == 0:
        extra["forward_gflop_per_image"] = forward_flops(args.size, 1, device) / 1e9
        if not args.no_nms:
            extra["nms"] = nms_bench(device)
            extra["augment"] = augment_bench(device)
        if world == 1 and not args.no_predict:
            extra["predict_fps_bs1"] = predict_fps(device)
            extra["c5_e2e"] = c5_e2e(device)
        if world == 1 and not args.no_cpu_baseline:
            extra["cpu_baseline"] = cpu_baseline(args.size, args.cpu_seconds)
        line = {
            "metric": METRIC, "value": value, "unit": "images/sec", "n_gpus": n_gpus,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "C2: JABD-MobileNetV3 RetinaFace (nets/retinaface_r.py) "
                       "eval forward, weights_init weights", "global_batch": args.batch * n_gpus,
                       "image_size": args.size, "parallelism": f"replicas x{n_gpus}"},
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
