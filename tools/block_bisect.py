"""Bisect a Block_eca training-gradient mismatch: the per-op training graph
(jabd_amd.train, JABD_FUSED_BLOCKS=0 style) with retain_grad on every
intermediate vs the same ops in float64 PyTorch-CPU.

  python3 tools/block_bisect.py k cin exp cout act stride B H W
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd"),
                os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as tF  # noqa: E402

import nets.mobilenetV3 as mv3  # noqa: E402
from _util import init_for_parity  # noqa: E402
from jabd_amd import train as T  # noqa: E402

k, cin, exp, cout = (int(v) for v in sys.argv[1:5])
act = sys.argv[5]
stride = int(sys.argv[6])
B, H, W = (int(v) for v in sys.argv[7:10])
dev = torch.device("cuda")
m = init_for_parity(mv3.Block_eca(k, cin, exp, cout, nn.ReLU if act == "relu" else nn.Hardswish,
                                  True, stride), seed=cin)
g = torch.Generator().manual_seed(cin)
x = torch.randn(B, cin, H, W, generator=g)
ACTF = tF.relu if act == "relu" else tF.hardswish


def ref_forward(P, x, keep):
    def bn(t, n):
        return tF.batch_norm(t, None, None, P[n + ".weight"], P[n + ".bias"], True, 0.1, 1e-5)

    e_pre = tF.conv2d(x, P["conv1.weight"]); keep["e_pre"] = e_pre
    e = ACTF(bn(e_pre, "bn1")); keep["e"] = e
    d_pre = tF.conv2d(e, P["conv2.weight"], None, stride, k // 2, 1, exp); keep["d_pre"] = d_pre
    d = ACTF(bn(d_pre, "bn2")); keep["d"] = d
    w1 = P["eca.conv.weight"]
    y = d.mean(dim=(2, 3))
    y = tF.conv1d(y.unsqueeze(1), w1, padding=(w1.shape[-1] - 1) // 2).squeeze(1)
    a = d * tF.hardsigmoid(y)[:, :, None, None]; keep["a"] = a
    p = tF.conv2d(a, P["conv3.weight"]); keep["p"] = p
    sk = m.skip
    if sk is None:
        res = x
    else:
        res = bn(tF.conv2d(x, P["skip.0.weight"], P.get("skip.0.bias")), "skip.1")
    out = ACTF(bn(p, "bn3") + res)
    for t in keep.values():
        t.retain_grad()
    return out


P64 = {n: v.detach().double().clone().requires_grad_() for n, v in m.named_parameters()}
xr = x.double().requires_grad_()
keep_r = {}
out_r = ref_forward(P64, xr, keep_r)
wt = torch.randn(out_r.shape, generator=torch.Generator().manual_seed(12), dtype=torch.float64)
(out_r * wt).sum().backward()

# ours, per-op graph
T.FUSED_BLOCKS = False
m = m.to(dev).train()
keep = {}
s = x.to(dev).permute(0, 2, 3, 1).contiguous().requires_grad_()
e_pre = T.conv(s, m.conv1); e_pre.retain_grad()
e = T.bn_act(e_pre, m.bn1, act); e.retain_grad()
d_pre = T.DwConvFn.apply(e, m.conv2.weight, stride); d_pre.retain_grad()
d = T.bn_act(d_pre, m.bn2, act); d.retain_grad()
p = T.EcaConvFn.apply(d, m.eca.conv.weight, m.conv3.weight, 1, 0, "hsigmoid"); p.retain_grad()
sk = m.skip
res = s if sk is None else T.bn_act(T.conv(s, sk[0]), sk[1])
out = T.bn_act(p, m.bn3, act, res=res)
(out * wt.permute(0, 2, 3, 1).float().to(dev)).sum().backward()
ours = dict(e_pre=e_pre, e=e, d_pre=d_pre, d=d, p=p)


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


print("fwd out", rel(out.detach().permute(0, 3, 1, 2).cpu().double(), out_r.detach()))
for n in ("p", "d", "d_pre", "e", "e_pre"):
    print("%-6s val %.2e  grad %.2e" % (n, rel(ours[n].detach().permute(0, 3, 1, 2).cpu().double(), keep_r[n].detach()),
                                         rel(ours[n].grad.permute(0, 3, 1, 2).cpu().double(), keep_r[n].grad)))
print("input grad %.2e" % rel(s.grad.permute(0, 3, 1, 2).cpu().double(), xr.grad))
for n, v in m.named_parameters():
    if v.grad is not None:
        print("%-20s %.2e" % (n, rel(v.grad.cpu().double(), P64[n].grad)))
gd = (ours["d_pre"].grad.permute(0, 3, 1, 2).cpu().double() - keep_r["d_pre"].grad).abs()
per_c = gd.amax(dim=(0, 2, 3))
c = int(per_c.argmax())
xc = keep_r["d_pre"].detach()[:, c]
print("worst channel", c, "err", float(per_c[c]), "ref grad max", float(keep_r["d_pre"].grad[:, c].abs().max()))
print("  d_pre mean %.4e var %.4e min %.4e max %.4e  zeros %d/%d" % (float(xc.mean()), float(xc.var(unbiased=False)),
      float(xc.min()), float(xc.max()), int((xc == 0).sum()), xc.numel()))
print("  bn2 gamma %.4e beta %.4e" % (float(P64["bn2.weight"][c]), float(P64["bn2.bias"][c])))
z = tF.batch_norm(keep_r["d_pre"].detach(), None, None, P64["bn2.weight"].detach(), P64["bn2.bias"].detach(), True, 0.1, 1e-5)[:, c]
print("  bn out near 0: min|z| %.3e  n(|z|<1e-5) %d" % (float(z.abs().min()), int((z.abs() < 1e-5).sum())))
print("  top channels err:", [(int(i), round(float(per_c[i]), 5)) for i in per_c.argsort(descending=True)[:6]])
