"""Kink-matched gradient parity (test infrastructure).

A piecewise activation's derivative jumps at its kink (ReLU / LeakyReLU at 0,
Hardswish at -3 and 3, Hardsigmoid at -3 and 3; a max-pool's argmax between
near-equal window values).  When a pre-activation lies within fp32 rounding
of a kink, the HIP run and a float64 oracle run can put it on different
sides; through a training-mode BatchNorm that one flipped element moves its
whole channel's gradient, so a gradient comparison could fail without any
kernel being wrong — or a real kernel error could be excused as a flip.

`Kinks` removes that ambiguity:

  * `with kk.record():` installs itself as jabd_amd.functional.KINK_TAP.  The
    HIP training forward hands it the operands each backward kernel derives
    its activation region from; the recorder recomputes the pre-activation z
    with that kernel's own fp32 operation order (train.hip: bn_bwd_part /
    bn_bwd_apply `fma((x - mean) * invstd, gamma, beta) + res`, the ECA gate
    backward's fma chain over the Conv1d taps; BECA's and the elementwise
    activation's z are the kernels' own saved tensors), so its sign pattern
    is the mask the HIP backward used.
  * `with kk.replay():` installs it as oracle.model_ref.REPLAY.  Each oracle
    kink()/maxpool() call is paired with the recorded tensor of the same
    family and shape that is closest to it (max-abs difference relative to
    the oracle tensor's max, which must be < 1e-2: distinct tensors differ by
    O(1), and a batch-statistics BN over two 1x1 samples — the SE gate —
    amplifies fp32 error to ~1e-3), and the oracle's backward
    takes its region from it.

Both oracle runs (float64 and float32) are replayed, so the float32 run's
error against the float64 run is again pure rounding, and the per-tensor bar
max(tol, 4x that error) no longer hides mask flips.

The replay is bounded, so that it cannot adopt a wrong mask (one a backward
kernel derived from a stale mean/invstd or the wrong residual):
  * pairing tolerance 1e-3 (relative max difference); the one named
    exception is a BatchNorm over 1x1 maps (the SE gate's, B samples per
    channel), which amplifies fp32 rounding to ~1e-3 and pairs at 1e-2;
  * rounding-level: when the float64 replay is followed by the float32 one
    (as every caller does), each HIP pre-activation's distance from the
    float64 oracle's must be within ROUND_FACTOR x the plain float32 oracle's
    own distance from it (floor ROUND_FLOOR) — the HIP tensor may carry fp32
    rounding, not an error of its own;
  * every paired call counts its flips — elements whose region (side of a
    kink, or max-pool argmax) differs between the HIP tensor and the oracle's
    own; a call may flip at most max(FLIP_MIN, FLIP_FRAC * numel) elements,
    each within the rounding distance above of its kink (for a max-pool: the
    two window values within that of each other).
A violation is reported through `unmatched`, which every caller asserts
empty.
`stats()` / JABD_KINK_LOG=<file> expose the pairing distances and flips.
"""
import os
import torch

from jabd_amd import functional as JF
from oracle import model_ref

_FAMILY = {"relu": "pos", "leaky": "pos", "hswish": "hswish", "hsigmoid": "hsig",
           "maxpool": "maxpool"}

PAIR_TOL = 1e-3
PAIR_TOL_SE = 1e-2
FLIP_MIN = 8
FLIP_FRAC = 2e-4
ROUND_FACTOR = 8.0
ROUND_FLOOR = 2e-6
_ULP = 2.0 ** -23
_DEV = "cpu"


def _f32(t):
    return t.detach().float().to(_DEV)


def _region(fam, z):
    """Which side of each kink (PyTorch's *_backward conventions, as
    oracle.model_ref._KinkFn)."""
    if fam == "pos":
        return (z > 0).to(torch.int8)
    if fam == "hswish":
        return torch.where(z < -3, 0, torch.where(z <= 3, 1, 2)).to(torch.int8)
    return ((z > -3) & (z < 3)).to(torch.int8)


def _kink_dist(fam, z):
    if fam == "pos":
        return z.abs()
    return torch.minimum((z + 3).abs(), (z - 3).abs())


def _fma32(a, b, c):
    """fmaf(a, b, c) of fp32 tensors: the product of two fp32 values is exact
    in fp64, so one fp64 add and one rounding to fp32 reproduce it."""
    return (a.double() * b.double() + c.double()).float()


def _bn_z(x, mean, invstd, g, b, res):
    """z of train.hip bn_bwd_*: xh = (x - mu) * is; z = fma(xh, g, b) + r."""
    x, mean, invstd, g, b = (_f32(t) for t in (x, mean, invstd, g, b))
    xh = (x - mean) * invstd
    z = _fma32(xh, g.expand_as(xh), b.expand_as(xh))
    if res is not None:
        z = z + _f32(res)
    return z


def _nchw(z):
    return z.permute(0, 3, 1, 2) if z.dim() == 4 else z


class Kinks:
    def __init__(self, tol=PAIR_TOL, device="cpu"):
        """device: where the recorded pre-activations are kept and compared
        (the oracle run's device; "cuda" for the at-size tests, whose fp64
        oracle runs on the GPU through PyTorch's own kernels)."""
        self.rec = []            # (family, [candidate float64 tensors])
        self.tol = tol
        self.device = device
        self.used = set()
        self.matched = 0
        self.unmatched = []      # (kind, shape, why) of oracle calls not cleanly paired
        self.log = []            # (kind, shape, pairing distance, flips, worst flip in ulps)
        self.nreplay = 0
        self.calls = []          # this replay: (oracle z, scale, HIP pairing distance, worst flip)
        self.prev = []           # the previous replay's calls
        self.dtypes = []         # oracle dtype of each replay

    # ------------------------------------------------------------------ recording
    def _add(self, kind, z, nhwc=True):
        z = z.double()
        cands = [_nchw(z) if nhwc else z]
        if z.dim() == 4:
            cands.append(z if nhwc else z.permute(0, 3, 1, 2))
        self.rec.append((_FAMILY[kind], cands))

    def __call__(self, kind, *a):
        # the recording device only for this call (a module default left at
        # "cuda" would move later tests' _bn_z results off the CPU)
        global _DEV
        prev, _DEV = _DEV, self.device
        try:
            return self._call(kind, *a)
        finally:
            _DEV = prev

    def _call(self, kind, *a):
        if kind == "stats":
            return
        if kind == "bn":
            act, slope, x, mean, invstd, g, b, res = a
            self._add(act, _bn_z(x, mean, invstd, g, b, res))
        elif kind == "eca":
            gate, mean, w1 = a
            mean, w = _f32(mean), _f32(w1)
            k = w.numel()
            h = (k - 1) // 2
            B, C = mean.shape
            z = torch.zeros((B, C), dtype=torch.float32, device=mean.device)
            for t in range(k):   # z = fma(w[t], mean[c + t - h], z), taps in order
                sh = torch.zeros_like(mean)   # out-of-range taps: fma(w, 0, z) == z
                lo, hi = max(0, h - t), min(C, C + h - t)
                sh[:, lo:hi] = mean[:, lo + t - h:hi + t - h]
                z = _fma32(w[t].expand_as(sh), sh, z)
            self._add(gate, z, nhwc=False)
        elif kind == "beca":
            (v,) = a
            self._add("hsigmoid", _f32(v), nhwc=False)
        elif kind == "act":
            act, slope, x = a
            self._add(act, _f32(x), nhwc=True)
        elif kind == "ssh":
            (pieces,) = a
            zs = [_bn_z(x, mean, invstd, g, b, None) for x, g, b, mean, invstd in pieces]
            self.rec.append(("ssh", [torch.cat(zs, 3).double()] + [z.double() for z in zs]))
        elif kind == "maxpool":
            (x,) = a
            self._add("maxpool", _f32(x))
        else:
            raise ValueError(kind)

    def record(self):
        return _Install(self, "tap")

    # ------------------------------------------------------------------ replay
    def _views(self, fam, cands, shape):
        """Candidate tensors reshaped to `shape` (channel dim 1 may carry zero
        padding at its end: 10 -> 12 channel branches)."""
        if fam == "ssh":   # [a | b padded | c padded] pieces, oracle cat(a, b, c)
            _, a, b, c = cands
            if len(shape) != 4:
                return []
            a, b, c = (_nchw(t) for t in (a, b, c))
            q = (shape[1] - a.shape[1]) // 2
            if q <= 0 or q > b.shape[1] or a.shape[0] != shape[0] or \
                    tuple(a.shape[2:]) != tuple(shape[2:]):
                return []
            return [torch.cat([a, b[:, :q], c[:, :q]], 1)]
        out = []
        for z in cands:
            if tuple(z.shape) == tuple(shape):
                out.append(z)
            elif z.dim() == 4 and len(shape) == 4 and z.shape[0] == shape[0] and \
                    tuple(z.shape[2:]) == tuple(shape[2:]) and 0 < z.shape[1] - shape[1] < 4:
                out.append(z[:, :shape[1]])
            elif z.numel() == int(torch.Size(shape).numel()) and z.dim() <= 2:
                out.append(z.reshape(shape))
        return out

    def _tol(self, shape):
        if len(shape) == 4 and shape[2] * shape[3] == 1:
            return max(self.tol, PAIR_TOL_SE)     # SE gate: BN over B 1x1 samples
        return self.tol

    def _flips(self, fam, v, zo, scale):
        """(count, worst distance from the kink in ulps of scale) of the
        elements whose region differs between HIP tensor v and oracle zo."""
        if fam == "maxpool":
            _, io = torch.nn.functional.max_pool2d(zo, 3, 2, 1, return_indices=True)
            _, iv = torch.nn.functional.max_pool2d(v, 3, 2, 1, return_indices=True)
            diff = io != iv
            n = int(diff.sum())
            if not n:
                return 0, 0.0
            flat = zo.flatten(2)
            gap = (flat.gather(2, io.flatten(2)) - flat.gather(2, iv.flatten(2))).abs()
            return n, float(gap.flatten()[diff.flatten()].max()) / (scale * _ULP)
        fo = "pos" if fam == "ssh" else fam
        diff = _region(fo, v) != _region(fo, zo)
        n = int(diff.sum())
        if not n:
            return 0, 0.0
        return n, float(_kink_dist(fo, zo)[diff].max()) / (scale * _ULP)

    def match(self, kind, z):
        if len(self.dtypes) < self.nreplay:
            self.dtypes.append(self._pending_dtype or z.dtype)
        fam = _FAMILY[kind]
        zo = z.detach().double()
        scale = float(zo.abs().max()) or 1.0
        best = (None, None, float("inf"))
        for i, (f, cands) in enumerate(self.rec):
            if i in self.used or not (f == fam or (f == "ssh" and fam == "pos")):
                continue
            for v in self._views(f, cands, zo.shape):
                v = v.to(zo.device)
                d = float((v - zo).abs().max()) / scale
                if d < best[2]:
                    best = (i, v, d)
        shape = tuple(zo.shape)
        if best[0] is None or best[2] >= self._tol(shape):
            self.unmatched.append((kind, shape, f"pairing {best[2]:.2e}"))
            self._note(kind, shape, best[2], None, None)
            return None
        n, worst = self._flips(fam, best[1], zo, scale)
        d32 = self._rounding(kind, shape, zo)
        self._note(kind, shape, best[2], n, worst, d32)
        if n > max(FLIP_MIN, FLIP_FRAC * zo.numel()):
            self.unmatched.append((kind, shape, f"{n} flips, worst {worst:.0f} ulp"))
        self.calls.append((zo if z.dtype == torch.float64 else None, scale, best[2], worst))
        self.used.add(best[0])
        self.matched += 1
        return best[1]

    def _rounding(self, kind, shape, zo):
        """In a float32 replay that follows a float64 one: this call's fp32
        oracle distance from the fp64 oracle, and the check of the fp64
        replay's HIP pairing distance (and flips) against it."""
        i = len(self.calls)
        if self.dtypes[-2:] != [torch.float64, torch.float32] or i >= len(self.prev):
            return None
        z64, scale, dh, worst = self.prev[i]
        if z64 is None or tuple(z64.shape) != shape:
            return None
        d32 = float((zo - z64.to(zo.device)).abs().max()) / scale
        lim = max(ROUND_FACTOR * d32, ROUND_FLOOR)
        if dh > lim or worst * _ULP > lim:
            self.unmatched.append((kind, shape, f"HIP {dh:.2e} / flip {worst * _ULP:.2e} from "
                                   f"fp64 vs fp32 oracle {d32:.2e}"))
        return d32

    def _note(self, kind, shape, d, n, worst, d32=None):
        self.log.append((kind, shape, d, n, worst))
        path = os.environ.get("JABD_KINK_LOG")
        if path:
            with open(path, "a") as f:
                f.write(f"{kind} {list(shape)} pair={d:.3e} flips={n} worst_ulp={worst} "
                        f"o32={d32}\n")

    def stats(self):
        """(max pairing distance, total flips, worst flip in ulps) over the
        paired calls so far."""
        ok = [r for r in self.log if r[3] is not None]
        return (max((r[2] for r in ok), default=0.0), sum(r[3] for r in ok),
                max((r[4] for r in ok), default=0.0))

    def replay(self, dtype=None):
        """dtype: the oracle run's dtype (taken from the first call when
        None)."""
        self.used = set()
        if self.calls or self.nreplay:
            self.prev = self.calls
        self.calls = []
        self.nreplay += 1
        self._pending_dtype = dtype
        return _Install(self, "replay")


class _Install:
    def __init__(self, kk, what):
        self.kk, self.what = kk, what

    def __enter__(self):
        if self.what == "tap":
            JF.KINK_TAP = self.kk
        else:
            model_ref.REPLAY = self.kk
        return self.kk

    def __exit__(self, *exc):
        if self.what == "tap":
            JF.KINK_TAP = None
        else:
            model_ref.REPLAY = None
