"""Per-launch conv-GEMM timing of one C2 forward (HIP events): achieved TF/s,
algorithmic GB/s and the per-layer roofline time max(FLOP/peak, bytes/8TB/s)."""
import sys, torch
import os
os.chdir(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = ['.', 'jabd-joint-attention-based-detector-for-small-face-detection_amd']
import bench
from jabd_amd import functional as F, synth
dev = torch.device('cuda')
m = bench.build_model(dev)
x = synth.images(32, 1024, device=dev)
with torch.no_grad():
    for _ in range(3): m(x)
recs = []
orig = F.conv
def tc(xx, pk, stride=1, pad=0, **kw):
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record(); o = orig(xx, pk, stride=stride, pad=pad, **kw); e.record()
    M = o.shape[0] * o.shape[1] * o.shape[2]; K = pk.KH * pk.KW * pk.Cin + pk.Cin2
    nb = 4.0 * (xx.numel() + (kw['x2'].numel() if kw.get('x2') is not None else 0) + K * pk.Cout + M * pk.Cout)
    recs.append((s, e, M, K, pk.Cout, pk.KH, stride, 2.0 * M * K * pk.Cout, nb, xx.shape[1], kw.get('x2') is not None, kw.get('ascale') is not None, kw.get('res') is not None))
    return o
F.conv = tc
with torch.no_grad(): m(x)
torch.cuda.synchronize()
tot = 0
for r in recs:
    t = r[0].elapsed_time(r[1]) * 1e3; tot += t
    print('M %8d K %4d N %4d k%d s%d H%4d x2 %d as %d res %d  %7.1f us  %6.1f TF  %6.0f GB/s  roof %6.1f us' % (r[2], r[3], r[4], r[5], r[6], r[9], r[10], r[11], r[12], t, r[7] / t / 1e6, r[8] / t / 1e3, max(r[7] / 157.3e6, r[8] / 8e6)))
print('total', tot, 'roof', sum(max(r[7] / 157.3e6, r[8] / 8e6) for r in recs))
