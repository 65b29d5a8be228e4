"""Per-launch roofline of one training step.

Every libjabd C-ABI call of one step (forward, MultiBoxLoss, backward, the
fused Adam step) is bracketed by HIP events on torch's current stream (the
launch stream) and annotated with
  * algorithmic FLOPs from the call's shapes (convolutions: 2 * pixels *
    (KH*KW*Cin + Cin2) * Cout of the forward conv the call computes or
    differentiates; depthwise: 2 * output pixels * C * k^2; expand+dw: both
    parts; everything else: 0 — they are memory-bound);
  * algorithmic bytes: every distinct device tensor the call's pointer
    arguments (and argument-struct pointer fields) refer to, counted once at
    its requested size (the caching allocator's snapshot taken at the call),
    workspaces excluded; the fused Adam step reads p, g, m, v and writes p, m,
    v: 28 bytes per parameter;
  * roof = max(FLOPs / 157.3 TFLOP/s, bytes / 8 TB/s).
The step's roofline fraction = sum of the roofs / the measured step time.

  python3 tools/train_roofline.py --kind mnv3 --batch 32 --out profiles/r04/c4_step_roofline.json
"""
import argparse
import bisect
import collections
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch  # noqa: E402

PEAK_TF = 157.3
PEAK_TBS = 8.0


class BlockMap:
    """pointer -> (block start, requested bytes) of live caching-allocator blocks."""

    def __init__(self):
        snap = torch.cuda.memory._snapshot()
        rows = []
        for seg in snap["segments"]:
            a = seg["address"]
            for b in seg["blocks"]:
                if b["state"] == "active_allocated":
                    rows.append((a, b.get("requested_size", b["size"]), b["size"]))
                a += b["size"]
        rows.sort()
        self.starts = [r[0] for r in rows]
        self.rows = rows

    def find(self, p):
        i = bisect.bisect_right(self.starts, p) - 1
        if i < 0:
            return None
        a, req, size = self.rows[i]
        if p >= a + size:
            return None
        return a, req


def _ptr_args(name, args, sigs):
    """Device-pointer arguments of a call (workspace pointers excluded)."""
    out = []
    types = sigs.get(name, [])
    for i, a in enumerate(args):
        t = types[i] if i < len(types) else None
        if hasattr(a, "_obj") and isinstance(a._obj, ctypes.Structure):
            st = a._obj
            for f, ft in st._fields_:
                if ft is ctypes.c_void_p and f not in ("ws",):
                    v = getattr(st, f)
                    if v:
                        out.append(v)
            continue
        if (name, i) in (("jabd_conv_bn_stats_f32", 1), ("jabd_conv_bn_bwd_sums_f32", 9),
                         ("jabd_conv_bn_bwd_sums_res_f32", 7), ("jabd_bn_act_bwd_rows_f32", 0)):   # the epilogue rows: workspace
            continue
        if t is ctypes.c_void_p:
            nxt = types[i + 1] if i + 1 < len(types) else None
            if nxt is ctypes.c_size_t:      # (ws, ws_bytes)
                continue
            v = a.value if isinstance(a, ctypes.c_void_p) else a
            if isinstance(v, int) and v:
                out.append(v)
    return out


_INT_TYPES = (ctypes.c_int32, ctypes.c_int, ctypes.c_int64)


def _flops(name, args, sigs=None):
    if name in ("jabd_conv2d_nhwc_f32", "jabd_conv_wgrad_f32", "jabd_conv1x1_bn_stats_f32",
                "jabd_conv_wgrad_eca_f32", "jabd_conv_bn_stats_f32", "jabd_conv_bn_bwd_sums_f32",
                "jabd_conv_bn_bwd_sums_res_f32"):
        a = args[0]._obj if hasattr(args[0], "_obj") else None
        if a is None:
            return 0.0
        if name not in ("jabd_conv2d_nhwc_f32", "jabd_conv_bn_bwd_sums_f32") or not a.tconv:
            return 2.0 * a.B * a.OH * a.OW * (a.KH * a.KW * a.Cin + a.Cin2) * a.Cout
        return 2.0 * a.B * a.H * a.W * a.KH * a.KW * a.Cin * a.Cout
    if name == "jabd_expand_dw_nhwc_f32":
        a = args[0]._obj
        return 2.0 * a.B * a.H * a.W * a.Cin * a.E + 2.0 * a.B * a.OH * a.OW * a.E * a.k * a.k
    if name in ("jabd_dwconv_nhwc_f32", "jabd_dwconv_stats_f32", "jabd_dwconv_bnin_stats_f32"):
        a = args[0]._obj
        return 2.0 * a.B * a.OH * a.OW * a.C * a.k * a.k
    if name in ("jabd_dw_dgrad_f32", "jabd_dw_wgrad_f32", "jabd_dw_dgrad_bn_bwd_f32",
                "jabd_dw_wgrad_bnin_f32"):
        # (dy|x, w, B, H, W, C, OH, OW, k, ...): the integer-typed arguments in order
        types = (sigs or {}).get(name, [])
        ints = [int(v) for v, t in zip(args, types) if t in _INT_TYPES]
        if len(ints) >= 7:
            B, H, W, C, OH, OW, k = ints[:7]
            return 2.0 * B * OH * OW * C * k * k
    return 0.0


def _shape(args):
    """Conv calls: 'B HxW Cin->Cout kKH sS [t]' of the argument struct, else ''."""
    a = args[0]._obj if args and hasattr(args[0], "_obj") else None
    if a is None or not hasattr(a, "KH"):
        return ""
    return (f"{a.B} {a.H}x{a.W} {a.Cin}->{a.Cout} k{a.KH} s{a.stride}" +
            (" t" if a.tconv else ""))


class Tracer:
    def __init__(self, nparams):
        from jabd_amd import _lib
        self.sigs = {k: v for k, v in _lib.SIGNATURES.items()}
        self.recs = []
        self.nparams = nparams

    def __enter__(self):
        import importlib
        from jabd_amd import _lib
        self.orig = _lib.call
        for mn in ("jabd_amd.functional", "jabd_amd.train", "jabd_amd.ops", "jabd_amd.optim",
                   "jabd_amd.parallel", "jabd_amd.modules"):
            importlib.import_module(mn)
        # every loaded module that bound _lib.call by name (nets.*, utils.* included)
        mods = [m for m in list(sys.modules.values())
                if m is not None and getattr(m, "call", None) is self.orig]
        self.mods = mods

        def traced(name, *args):
            bm = BlockMap()
            seen, nbytes = set(), 0
            for p in _ptr_args(name, args, self.sigs):
                f = bm.find(p)
                if f and f[0] not in seen:
                    seen.add(f[0])
                    nbytes += f[1]
            if name == "jabd_adam_step_f32":
                nbytes = 28 * self.nparams
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            r = self.orig(name, *args)
            e1.record()
            self.recs.append((name, e0, e1, _flops(name, args, self.sigs), nbytes, _shape(args)))
            return r
        for m in mods:
            m.call = traced
        return self

    def __exit__(self, *exc):
        for m in self.mods:
            m.call = self.orig


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mnv3")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import contextlib
    import io
    import bench
    from jabd_amd import optim, parallel, synth
    from nets.retinaface_training import MultiBoxLoss, weights_init
    from utils.anchors import Anchors
    dev = torch.device("cuda")
    RetinaFace, cfg = bench.detector(a.kind)
    torch.manual_seed(0)
    model = RetinaFace(cfg=cfg, mode="train")
    with contextlib.redirect_stdout(io.StringIO()):
        weights_init(model)
    model = model.to(dev).train()
    opt = optim.Adam(model.parameters(), 1e-3, weight_decay=5e-4)
    crit = MultiBoxLoss(2, 0.35, 7, cfg["variance"], True)
    pri = Anchors(cfg, image_size=(a.size, a.size)).get_anchors().to(dev)
    x = synth.images(a.batch, a.size, seed=1234, device=dev)
    tg = [torch.from_numpy(t).to(dev) for t in synth.targets(a.batch, a.size, seed=4321)]
    for _ in range(3):
        parallel.train_step(model, crit, opt, x, tg, pri)
    torch.cuda.synchronize()
    steps = 5
    t0 = time.perf_counter()
    for _ in range(steps):
        parallel.train_step(model, crit, opt, x, tg, pri)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / steps * 1e3
    nparams = sum(p.numel() for p in model.parameters() if p.requires_grad)
    with Tracer(nparams) as tr:
        parallel.train_step(model, crit, opt, x, tg, pri)
    torch.cuda.synchronize()
    rows = []
    for name, e0, e1, fl, nb, shp in tr.recs:
        us = e0.elapsed_time(e1) * 1e3
        roof = max(fl / (PEAK_TF * 1e12), nb / (PEAK_TBS * 1e12)) * 1e6
        rows.append({"call": name, "us": us, "gflop": fl / 1e9, "mbytes": nb / 1e6, "roof_us": roof})
        if shp:
            rows[-1]["shape"] = shp
    tot_us = sum(r["us"] for r in rows)
    tot_roof = sum(r["roof_us"] for r in rows)
    g = collections.OrderedDict()
    for r in rows:
        d = g.setdefault(r["call"], {"calls": 0, "us": 0.0, "gflop": 0.0, "mbytes": 0.0, "roof_us": 0.0})
        d["calls"] += 1
        for k in ("us", "gflop", "mbytes", "roof_us"):
            d[k] += r[k]
    print(f"{a.kind} bs{a.batch} {a.size}^2 training step: {step_ms:.2f} ms ({a.batch / step_ms * 1e3:.1f} img/s); "
          f"{len(rows)} C-ABI calls, {tot_us / 1e3:.2f} ms in them, per-launch roof {tot_roof / 1e3:.2f} ms")
    print(f"step roofline fraction (sum of roofs / step time) {tot_roof / 1e3 / step_ms:.3f}; "
          f"inside the calls {tot_roof / tot_us:.3f}")
    print(f"{'call':38s} {'n':>5s} {'ms':>8s} {'GFLOP':>9s} {'GB':>8s} {'TF/s':>7s} {'GB/s':>7s} "
          f"{'roof ms':>8s} {'frac':>5s}")
    for name, d in sorted(g.items(), key=lambda kv: -kv[1]["us"]):
        print(f"{name:38s} {d['calls']:5d} {d['us'] / 1e3:8.3f} {d['gflop']:9.2f} {d['mbytes'] / 1e3:8.3f} "
              f"{d['gflop'] / max(d['us'], 1e-9) * 1e3:7.1f} {d['mbytes'] / max(d['us'], 1e-9) * 1e3:7.0f} "
              f"{d['roof_us'] / 1e3:8.3f} {d['roof_us'] / max(d['us'], 1e-9):5.2f}")
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"workload": f"{a.kind} training bs{a.batch} {a.size}x{a.size}",
                       "step_ms": step_ms, "calls": len(rows), "calls_ms": tot_us / 1e3,
                       "roof_ms": tot_roof / 1e3, "frac_step": tot_roof / 1e3 / step_ms,
                       "frac_in_calls": tot_roof / tot_us, "peak_tflops": PEAK_TF,
                       "peak_tbs": PEAK_TBS, "by_call": g, "launches": rows}, f, indent=1)


if __name__ == "__main__":
    main()
