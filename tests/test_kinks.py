"""CPU checks of the kink-matched oracle replay (tests/_kinks.py,
oracle/model_ref.py kink()/maxpool()): pairing recorded pre-activations with
the oracle's calls, the derivative taken from the recorded region, and the
fp32 emulation of the HIP backward's mask arithmetic."""
import torch

from _kinks import Kinks, _bn_z
from _util import init_for_parity
from oracle import model_ref


class _Grab:
    """REPLAY stand-in that records every oracle kink input (no replay)."""

    def __init__(self):
        self.seen = []

    def match(self, kind, z):
        self.seen.append((kind, z.detach().clone()))
        return None


def _block_run(sd, x, dtype, spec):
    P = {k: (v.to(dtype).requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.to(dtype) if v.is_floating_point() else v)) for k, v in sd.items()}
    ctx = model_ref.Ctx(P, True)
    xr = x.detach().to(dtype).clone().requires_grad_(True)
    y = model_ref.block(ctx, xr, "", spec, "eca")
    w = torch.randn(y.shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    (y * w.to(dtype)).sum().backward()
    return y.detach(), xr.grad


def _setup():
    import nets.mobilenetV3 as mv3
    spec = (3, 16, 64, 24, "relu", False, 1)
    m = init_for_parity(mv3.Block_eca(3, 16, 64, 24, torch.nn.ReLU, False, 1), seed=4)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(2, 16, 12, 10, generator=torch.Generator().manual_seed(5))
    return spec, sd, x


def _recorded(sd, x, spec, dtype):
    """Kinks filled with one oracle run's own pre-activations."""
    grab = _Grab()
    model_ref.REPLAY = grab
    try:
        _block_run(sd, x, dtype, spec)
    finally:
        model_ref.REPLAY = None
    kk = Kinks()
    for kind, z in grab.seen:
        kk._add(kind, z, nhwc=False)
    return kk, grab.seen


def test_replay_pairs_every_call_and_keeps_values():
    spec, sd, x = _setup()
    kk, seen = _recorded(sd, x, spec, torch.float64)
    assert [k for k, _ in seen] == ["relu", "relu", "hsigmoid", "relu"]
    y0, g0 = _block_run(sd, x, torch.float64, spec)
    with kk.replay():
        y1, g1 = _block_run(sd, x, torch.float64, spec)
    assert kk.matched == 4 and not kk.unmatched
    assert torch.equal(y0, y1)                    # forward values are the oracle's own
    assert float((g0 - g1).abs().max()) <= 1e-8 * float(g0.abs().max())  # own masks


def test_one_flipped_mask_is_what_replay_removes():
    """At 2x16x12x10 this block has one BN1 output 2.2e-8 from the ReLU kink
    whose sign differs between the fp32 and the fp64 run: the fp32 input
    gradient is then ~8% off the fp64 one although no arithmetic is wrong.
    With the fp32 run's masks replayed, the fp64 gradient agrees with it to
    fp32 rounding — the comparison now measures arithmetic only."""
    spec, sd, x = _setup()
    kk, seen = _recorded(sd, x, spec, torch.float32)
    _, g32 = _block_run(sd, x, torch.float32, spec)
    _, g64 = _block_run(sd, x, torch.float64, spec)
    with kk.replay():
        _, g64r = _block_run(sd, x, torch.float64, spec)
    rel = lambda a, b: float((a.double() - b).abs().max() / b.abs().max())  # noqa: E731
    assert rel(g32, g64) > 1e-2
    assert rel(g32, g64r) < 1e-5


def test_unmatched_when_far():
    spec, sd, x = _setup()
    kk, _ = _recorded(sd, x, spec, torch.float64)
    for _, cands in kk.rec:
        cands[0].mul_(1.1)                          # 10% off: no pairing
    with kk.replay():
        _block_run(sd, x, torch.float64, spec)
    assert kk.matched == 0 and len(kk.unmatched) == 4


def test_maxpool_replay_uses_recorded_argmax():
    """A near-tie in window (0, 0): the oracle's own maximum is at (1, 1), the
    recorded tensor's at (0, 1); the gradient follows the recorded argmax."""
    x = torch.randn(1, 2, 7, 7, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    x[0, 0, 1, 1] = 5.0
    x[0, 0, 0, 1] = 5.0 - 1e-6
    xr = x.clone()
    xr[0, 0, 0, 1] = 5.0 + 1e-6
    kk = Kinks()
    kk._add("maxpool", xr, nhwc=False)
    xx = x.clone().requires_grad_(True)
    with kk.replay():
        y = model_ref.maxpool(xx)
    assert kk.matched == 1
    y[0, 0, 0, 0].backward()
    assert xx.grad[0, 0, 0, 1] == 1.0 and xx.grad[0, 0, 1, 1] == 0.0
    assert y.shape == torch.nn.functional.max_pool2d(x, 3, 2, 1).shape


def test_bn_z_is_the_kernels_fma_order():
    """fma((x - mu) * is, g, b) emulated in fp64 rounds like the fused op."""
    g = torch.Generator().manual_seed(2)
    x = torch.randn(3, 4, 5, 8, generator=g)
    mu, inv = torch.randn(8, generator=g), torch.rand(8, generator=g) + 0.5
    gm, bt = torch.randn(8, generator=g), torch.randn(8, generator=g)
    z = _bn_z(x, mu, inv, gm, bt, None)
    xh = (x - mu) * inv
    exact = xh.double() * gm.double() + bt.double()
    assert z.dtype == torch.float32
    assert torch.equal(z, exact.float())


def test_pairing_rejects_a_stale_operand():
    """A recorded pre-activation 0.5% off (e.g. a backward mask taken from a
    stale mean/invstd) no longer pairs: the tolerance is 1e-3, not 1e-2."""
    spec, sd, x = _setup()
    kk, _ = _recorded(sd, x, spec, torch.float64)
    for _, cands in kk.rec:
        cands[0].add_(5e-3 * float(cands[0].abs().max()))
    with kk.replay():
        _block_run(sd, x, torch.float64, spec)
    assert kk.matched == 0 and len(kk.unmatched) == 4


def test_flips_beyond_rounding_are_reported():
    """Elements moved across the ReLU kink by more than fp32 rounding (here:
    every |z| < 2e-4 max|z| negated, a pairing distance well inside 1e-3)
    are flips the replay refuses to adopt silently; the fp32 run's own
    rounding-level flips are accepted and counted."""
    spec, sd, x = _setup()
    kk, _ = _recorded(sd, x, spec, torch.float64)
    fam0, cands = kk.rec[0]
    z = cands[0]
    near = z.abs() < 2e-4 * float(z.abs().max())
    assert int(near.sum()) >= 1
    z[near] = -z[near] - 1e-5 * float(z.abs().max())
    with kk.replay():
        _block_run(sd, x, torch.float64, spec)
    assert any("flips" in u[2] for u in kk.unmatched), kk.unmatched
    kk32, _ = _recorded(sd, x, spec, torch.float32)
    with kk32.replay():
        _block_run(sd, x, torch.float64, spec)
    assert not kk32.unmatched
    pair, flips, worst = kk32.stats()
    assert flips >= 1 and worst <= 16 and pair < 1e-5   # the 2.2e-8 flip of the test above


def test_rounding_check_against_the_fp32_oracle():
    """The fp64-then-fp32 replay pair bounds each HIP tensor's distance from
    the fp64 oracle by ROUND_FACTOR x the fp32 oracle's own: recorded fp32
    tensors pass; one shifted by 3e-5 of its max (inside the 1e-3 pairing
    tolerance, far outside fp32 rounding at this size) is reported."""
    spec, sd, x = _setup()
    for shift, expect in ((0.0, False), (3e-5, True)):
        kk, _ = _recorded(sd, x, spec, torch.float32)
        if shift:
            z = kk.rec[1][1][0]
            z.add_(shift * float(z.abs().max()))
        with kk.replay():
            _block_run(sd, x, torch.float64, spec)
        assert not kk.unmatched
        with kk.replay():
            _block_run(sd, x, torch.float32, spec)
        assert any("fp32 oracle" in u[2] for u in kk.unmatched) == expect, kk.unmatched
