import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]
import torch
import bench
from jabd_amd import synth
dev = torch.device("cuda", 0)
m = bench.build_model(dev)
x = synth.images(32, 1024, seed=1234, device=dev)
with torch.no_grad():
    for _ in range(3):
        ref = m(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        m(x)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / 20
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            m(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = m(x)
    g.replay()
    torch.cuda.synchronize()
    err = max(float((a - b).abs().max()) for a, b in zip(out, ref))
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    gr = (time.perf_counter() - t0) / 20
print(f"eager {eager*1e3:.3f} ms  graph {gr*1e3:.3f} ms  maxdiff {err}")
