"""Shared test helpers (seeded parity init, tolerance metric)."""
import math

import torch


def init_for_parity(model, seed=0):
    """Seeded init that keeps activations O(1) through the whole detector so
    a parity check is sensitive to every layer (weights_init's N(0, 0.02)
    makes deep activations vanish and hides backbone errors).  BatchNorm gets
    non-trivial running stats so eval-mode folding is exercised."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, m in model.named_modules():
            cls = m.__class__.__name__
            if cls in ("Conv2d", "Conv1d"):
                fan_in = m.weight[0].numel()
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * math.sqrt(1.0 / fan_in))
                if m.bias is not None:
                    m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
            elif cls == "BatchNorm2d":
                m.weight.copy_(1.0 + 0.2 * torch.randn(m.weight.shape, generator=g))
                m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))
                m.running_mean.copy_(0.1 * torch.randn(m.running_mean.shape, generator=g))
                m.running_var.copy_(0.5 + torch.rand(m.running_var.shape, generator=g))
    return model


def rel_err(got, ref):
    """max |got - ref| / max |ref|  (scale-aware fp32 error)."""
    got, ref = got.double().cpu(), ref.double().cpu()
    return float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))


def elem_rel_err(got, ref, floor=1e-2):
    """max_i |got_i - ref_i| / max(|ref_i|, floor * max|ref|): an elementwise
    relative error whose denominator is floored so exact zeros do not blow it up."""
    got, ref = got.double().cpu(), ref.double().cpu()
    den = ref.abs().clamp_min(floor * float(ref.abs().max().clamp_min(1e-30)))
    return float(((got - ref).abs() / den).max())
