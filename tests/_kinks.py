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
"""
import torch

from jabd_amd import functional as JF
from oracle import model_ref

_FAMILY = {"relu": "pos", "leaky": "pos", "hswish": "hswish", "hsigmoid": "hsig",
           "maxpool": "maxpool"}


def _f32(t):
    return t.detach().float().cpu()


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
    def __init__(self, tol=1e-2):
        self.rec = []            # (family, [candidate float64 tensors])
        self.tol = tol
        self.used = set()
        self.matched = 0
        self.unmatched = []      # (kind, shape) of oracle calls left on their own masks

    # ------------------------------------------------------------------ recording
    def _add(self, kind, z, nhwc=True):
        z = z.double()
        cands = [_nchw(z) if nhwc else z]
        if z.dim() == 4:
            cands.append(z if nhwc else z.permute(0, 3, 1, 2))
        self.rec.append((_FAMILY[kind], cands))

    def __call__(self, kind, *a):
        if kind == "bn":
            act, slope, x, mean, invstd, g, b, res = a
            self._add(act, _bn_z(x, mean, invstd, g, b, res))
        elif kind == "eca":
            gate, mean, w1 = a
            mean, w = _f32(mean), _f32(w1)
            k = w.numel()
            h = (k - 1) // 2
            B, C = mean.shape
            z = torch.zeros((B, C), dtype=torch.float32)
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

    def match(self, kind, z):
        fam = _FAMILY[kind]
        zo = z.detach().double()
        scale = float(zo.abs().max()) or 1.0
        best = (None, None, float("inf"))
        for i, (f, cands) in enumerate(self.rec):
            if i in self.used or not (f == fam or (f == "ssh" and fam == "pos")):
                continue
            for v in self._views(f, cands, zo.shape):
                d = float((v - zo).abs().max()) / scale
                if d < best[2]:
                    best = (i, v, d)
        if best[0] is None or best[2] >= self.tol:
            self.unmatched.append((kind, tuple(zo.shape), best[2]))
            return None
        self.used.add(best[0])
        self.matched += 1
        return best[1]

    def replay(self):
        self.used = set()
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
