"""The N>1 path of bench.py, executed.

bench.py is launched exactly as the driver launches it for N GPUs
(`python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
... bench.py --gpus 2`), with the process-group backend taken from the
environment (JABD_DIST_BACKEND=gloo: the same control flow as RCCL, on the
one GPU both ranks share) and JABD_BENCH_GLOBAL_DATA=1 (the ranks shard one
global synthetic batch, so the job is comparable with one process).

Checked:
  * both ranks exit 0 and rank 0 prints exactly one JSON line with
    n_gpus == 2 and the C4 training leg;
  * every rank ends with the same parameters (bitwise-equal checksums): the
    SUM all-reduce of the gradient buckets hands each rank the same sum, and
    the fused Adam step is deterministic;
  * the job's loss at every training step (warmup, conv-timer and timed
    steps; the sum of the ranks' parts) against one process emulating
    nn.DataParallel on the global batch (train_mobilenetV3_ecagai.py:462-466,
    nets/retinaface_training.py:295-302): a replica per shard (BN statistics
    per shard), the loss on the gathered batch, gradients summed, replica 0's
    BN buffers kept, then the same fused Adam (wd 5e-4).  Step 0 depends only
    on the initial weights and the data: 1e-4.  Later steps compound fp32
    reassociation through Adam (whose first steps move each weight by about
    lr * sign(g)): 1e-3.
"""
import copy
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZE, B = 96, 2
WARMUP, TIMER_STEPS, STEPS = 3, 1, 2     # bench.main: C4 warmup 3, one conv-timer step


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_bench(world, tmp_path):
    env = dict(os.environ, JABD_DIST_BACKEND="gloo", JABD_BENCH_GLOBAL_DATA="1",
               MASTER_ADDR="127.0.0.1")
    args = ["bench.py", "--gpus", str(world), "--steps", "2", "--warmup", "1",
            "--size", str(SIZE), "--batch", str(B), "--train-steps", str(STEPS),
            "--r50-batch", "0", "--no-nms", "--no-predict", "--no-cpu-baseline"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port())] + args
    log = tmp_path / f"bench_w{world}.log"
    with open(log, "w") as f:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=f,
                           text=True, timeout=400)
    assert r.returncode == 0, f"bench world={world} rc={r.returncode}\n{log.read_text()[-4000:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _dataparallel_losses(world, nsteps):
    """One process, nn.DataParallel semantics over `world` replicas."""
    sys.path.insert(0, ROOT)
    import contextlib
    import io
    import bench
    from jabd_amd import optim, synth
    from nets.retinaface_training import MultiBoxLoss, weights_init
    from utils.anchors import Anchors
    RetinaFace, cfg = bench.detector("mnv3")
    torch.manual_seed(0)
    m = RetinaFace(cfg=cfg, mode="train")
    with contextlib.redirect_stdout(io.StringIO()):
        weights_init(m)
    m = m.cuda().train()
    opt = optim.Adam(m.parameters(), 1e-3, weight_decay=5e-4)
    crit = MultiBoxLoss(2, 0.35, 7, cfg["variance"], True)
    pri = Anchors(cfg, image_size=(SIZE, SIZE)).get_anchors().cuda()
    x = synth.images(B * world, SIZE, seed=1234, device="cuda")
    tg = [torch.from_numpy(t).cuda() for t in synth.targets(B * world, SIZE, seed=4321)]
    losses = []
    for _ in range(nsteps):
        opt.zero_grad()
        reps = [m] + [copy.deepcopy(m) for _ in range(world - 1)]
        outs = [r(x[i * B:(i + 1) * B]) for i, r in enumerate(reps)]
        out = tuple(torch.cat(t) for t in zip(*outs))
        lo, c, lm = crit(out, pri, tg)
        loss = 2.0 * lo + c + lm
        loss.backward()
        for r in reps[1:]:
            for p, q in zip(m.parameters(), r.parameters()):
                if q.grad is not None:
                    p.grad = q.grad.clone() if p.grad is None else p.grad + q.grad
        opt.step()
        losses.append(float(loss))
    ck = float(torch.stack([p.detach().double().sum() for p in m.parameters()]).sum())
    return losses, ck


@pytest.mark.gpu
def test_bench_two_ranks_gloo(cuda, tmp_path):
    line = _run_bench(2, tmp_path)
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 2 * B
    c4 = line["train"]["C4_mnv3"]
    assert c4["global_batch"] == 2 * B and c4["images_per_sec"] > 0
    cks = c4["param_checksums"]
    assert len(cks) == 2 and cks[0] == cks[1], cks
    trace = c4["loss_trace"]
    n = WARMUP + TIMER_STEPS + STEPS
    assert len(trace) == n, trace
    ref, _ = _dataparallel_losses(2, n)
    errs = [abs(a - b) / abs(b) for a, b in zip(trace, ref)]
    assert errs[0] < 1e-4, (trace, ref)
    assert max(errs) < 1e-3, (errs, trace, ref)
    assert abs(c4["loss_last"] - trace[-1]) <= 1e-6 * abs(trace[-1])
