"""A11 at the benchmarked resolution: the HIP training
path at 1024² against the kink-matched fp64 oracle, and every BatchNorm's
fused batch statistics at the C4 / C3 batch sizes against an fp64 two-pass
reduction of the same saved pre-BN tensor.

The oracle here is oracle/model_ref.py run by PyTorch's own GPU kernels
(MIOpen off, so convolutions are ATen's im2col + rocBLAS GEMMs in the
oracle's dtype) — the same restatement the CPU tests run, moved to the
device so a 1024² fp64 training graph takes seconds.  Reference:
train_mobilenetV3_ecagai.py:518-533 (the training step), nets/mobilenetV3.py:
140-150 (Block_eca), nets/retinaface_eca_nonlocal.py:252-359 (R50 head).

Bars (written in the tests):
  * outputs: relative max error <= 1e-3 vs the fp64 oracle;
  * gradients: per tensor relative Frobenius error <= max(2e-3, 4x the
    mask-matched fp32 oracle's own error) (tests/test_train.py's bar);
  * BN running statistics: relative max error <= 1e-4;
  * batch statistics: |mean - mean64| <= 1e-6 * sqrt(mean64^2 + var64) and
    |var - var64| <= 1e-5 * (var64 + eps), var = invstd^-2 - eps.
"""
import pytest
import torch

from _kinks import Kinks
from _util import init_for_parity, rel_err
from oracle import model_ref


def _fro(a, b):
    a, b = a.double(), b.double().to(a.device)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _oracle_grads(sd, fn, x, dtype, kk, dev):
    P = {k: (v.detach().to(dev, dtype).requires_grad_(True)
             if v.is_floating_point() and "running" not in k
             else (v.detach().to(dev, dtype) if v.is_floating_point() else v.to(dev)))
         for k, v in sd.items()}
    with torch.backends.cudnn.flags(enabled=False), kk.replay():
        ref = fn(P, x.to(dev, dtype), "train", train_bn=True)
    assert not kk.unmatched, f"kink replay: {kk.unmatched[:5]}"
    g = torch.Generator().manual_seed(5)
    wts = [torch.randn(r.shape, generator=g) for r in ref]
    with torch.backends.cudnn.flags(enabled=False):
        sum(((r * w.to(dev, dtype)).sum() for r, w in zip(ref, wts))).backward()
    grads = {k: p.grad for k, p in P.items()
             if isinstance(p, torch.Tensor) and p.requires_grad and p.grad is not None}
    return [r.detach() for r in ref], grads, P, wts


def _train_compare_at_size(model, fn, x, dev, tol=2e-3):
    import re
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    kk = Kinks(device=dev)
    m = model.to(dev).train()
    with kk.record():
        out = m(x.to(dev))
    ref64, g64, P64, wts = _oracle_grads(sd, fn, x, torch.float64, kk, dev)
    ref32, g32, _, _ = _oracle_grads(sd, fn, x, torch.float32, kk, dev)
    pair, flips, worst = kk.stats()
    print(f"kink replay: {kk.matched} pairs, max pairing {pair:.2e}, {flips} flips, "
          f"worst {worst:.0f} ulp")
    assert kk.matched > 20
    sum(((o * w.to(dev)).sum() for o, w in zip(out, wts))).backward()
    for o, r, name in zip(out, ref64, ("loc", "conf", "landm")):
        e = rel_err(o.detach(), r)
        assert e < 1e-3, f"{name} forward rel err {e:.2e}"
    named = dict(m.named_parameters())
    gmax = max(float(g.abs().max()) for g in g64.values())
    zero = re.compile(r"(f_key\.bias|skip\.2\.bias)$")
    rows = []
    for k, rg in g64.items():
        q = named[k]
        assert q.grad is not None, f"no HIP gradient for {k}"
        if zero.search(k) or (k.endswith("skip.1.bias")
                              and k.replace("skip.1.bias", "skip.3.weight") in g64):
            assert float(q.grad.abs().max()) <= 1e-4 * gmax, k
            continue
        rows.append((_fro(q.grad, rg), _fro(g32[k], rg), k))
    assert len(rows) > 50
    rows.sort(reverse=True)
    print("worst gradients (hip, oracle-fp32, name):", rows[:3])
    bad = [r for r in rows if r[0] > max(tol, 4 * r[1])]
    assert not bad, f"gradients off vs fp64 (hip, oracle-fp32, name): {bad[:5]}"
    for k, v in m.state_dict().items():
        if "running" in k:
            e = rel_err(v, P64[k])
            assert e < 1e-4, f"{k} running stat rel err {e:.2e}"


@pytest.mark.gpu
def test_train_step_mnv3_1024(cuda):
    """C4's model (JABD-MNv3) at 1024², bs2: one training forward/backward,
    every parameter gradient and BN running stat vs the fp64 oracle."""
    from jabd_amd import synth
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=14)
    x = synth.images(2, 1024, seed=41)
    _train_compare_at_size(m, model_ref.retinaface_mnv3, x, cuda)


@pytest.mark.gpu
def test_train_step_r50_1024(cuda):
    """C3's model (R50 + ECA/NLM head) at 1024², bs2."""
    from jabd_amd import synth
    from nets.retinaface_eca_nonlocal import RetinaFace
    from utils.config import cfg_re50
    m = init_for_parity(RetinaFace(cfg=cfg_re50, mode="train"), seed=16)
    x = synth.images(2, 1024, seed=43)
    _train_compare_at_size(m, model_ref.retinaface_r50, x, cuda)


class _StatsTap:
    """KINK_TAP stand-in: for every BatchNorm's batch statistics the training
    forward takes, an fp64 two-pass mean / variance of the same tensor on the
    device, in row chunks (no fp64 copy of a multi-GB activation)."""

    def __init__(self):
        self.rows = []   # (src, C, M, mean err, var err)

    def __call__(self, kind, *a):
        if kind != "stats":
            return
        src, x, mean, invstd, eps = a
        C = x.shape[-1]
        xv = x.reshape(-1, C)
        M = xv.shape[0]
        step = max(1, (1 << 26) // C)
        s = torch.zeros(C, dtype=torch.float64, device=x.device)
        for i in range(0, M, step):
            s += xv[i:i + step].sum(0, dtype=torch.float64)
        m64 = s / M
        q = torch.zeros_like(s)
        for i in range(0, M, step):
            q += ((xv[i:i + step].double() - m64) ** 2).sum(0)
        v64 = q / M
        var = invstd.double() ** -2 - eps
        em = float(((mean.double() - m64).abs() / (m64 ** 2 + v64).sqrt().clamp_min(1e-30)).max())
        ev = float(((var - v64).abs() / (v64 + eps)).max())
        self.rows.append((src, C, M, em, ev))


def _stats_at_size(model, x, dev):
    from jabd_amd import functional as JF
    tap = _StatsTap()
    m = model.to(dev).train()
    JF.KINK_TAP = tap
    try:
        with torch.no_grad():
            m(x)
    finally:
        JF.KINK_TAP = None
    torch.cuda.synchronize()
    worst = {}
    for src, C, M, em, ev in tap.rows:
        w = worst.setdefault(src, [0, 0.0, 0.0, 0])
        w[0] += 1
        w[1], w[2], w[3] = max(w[1], em), max(w[2], ev), max(w[3], M)
    print("BN statistics vs fp64 two-pass (calls, mean err, var err, max M):", worst)
    bad = [r for r in tap.rows if r[3] > 1e-6 or r[4] > 1e-5]
    assert not bad, f"(src, C, M, mean err, var err): {bad[:6]}"
    return worst


@pytest.mark.gpu
def test_bn_stats_mnv3_bs32_1024(cuda):
    """C4's per-GPU shape (MNv3, bs32, 1024²: up to 8.4 M pixels per
    channel): every BN's statistics, including the fused ones — the
    depthwise forward's (dw), the streaming expand conv's (conv1x1_stream)
    and the BN-input depthwise path's (dw_bnin)."""
    from jabd_amd import synth
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=17)
    x = synth.images(32, 1024, seed=44, device=cuda)
    worst = _stats_at_size(m, x, cuda)
    assert {"dw", "conv1x1_stream", "dw_bnin", "bn_stats"} <= set(worst), sorted(worst)
    assert worst["conv1x1_stream"][3] == 32 * 512 * 512


@pytest.mark.gpu
def test_bn_stats_r50_bs64_1024(cuda):
    """C3's shape (R50, bs64, 1024²: layer1's BNs over 4.2 M pixels, taken
    in the bottleneck convs' GEMM epilogue)."""
    from jabd_amd import synth
    from nets.retinaface_eca_nonlocal import RetinaFace
    from utils.config import cfg_re50
    m = init_for_parity(RetinaFace(cfg=cfg_re50, mode="train"), seed=18)
    x = synth.images(64, 1024, seed=45, device=cuda)
    worst = _stats_at_size(m, x, cuda)
    assert worst["conv32"][3] >= 64 * 256 * 256   # the bottleneck convs' epilogue statistics
