"""§8e data-parallel equivalence on the real detector: two ranks (gloo over
the one GPU's CUDA tensors), each running parallel.train_step on half of a
4-image batch — RetinaFace (JABD-MobileNetV3) + MultiBoxLoss with the
positive counts all-reduced and the gradients SUM-all-reduced by
GradAllReduce (step 1 synchronous, step 2 from the backward hooks) — against
one process emulating nn.DataParallel exactly (train_mobilenetV3_ecagai.py:
462-466 + nets/retinaface_training.py:295-302): each half through its own
replica (BN statistics per shard), the loss on the concatenated global batch,
gradients summed, replica 0's BN running buffers kept.  Bar: gradients and
the summed losses within 1e-4 relative (fp32 reduction order differs)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

B, SIZE = 4, 96


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from _util import init_for_parity
    from jabd_amd import synth
    from nets.retinaface_r import RetinaFace
    from utils.anchors import Anchors
    from utils.config import cfg_mnet
    m = init_for_parity(RetinaFace(cfg=cfg_mnet, mode="train"), seed=31).cuda().train()
    x = synth.images(B, SIZE, seed=5).cuda()
    tg = [torch.from_numpy(t).cuda() for t in synth.targets(B, SIZE, seed=6)]
    pri = Anchors(cfg_mnet, image_size=(SIZE, SIZE)).get_anchors().cuda()
    return m, x, tg, pri, cfg_mnet


def _worker(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import conftest  # noqa: F401  (package paths)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jabd_amd import parallel
        from nets.retinaface_training import MultiBoxLoss
        m, x, tg, pri, cfg = _setup()
        xs, ts = parallel.shard(x, tg, rank, world)
        crit = MultiBoxLoss(2, 0.35, 7, cfg["variance"], True)
        opt = torch.optim.SGD(m.parameters(), lr=0.0)   # gradients only; weights fixed
        red = parallel.GradAllReduce(m, bucket_bytes=1 << 18)
        res = {}
        for step in range(2):
            _, parts = parallel.train_step(m, crit, opt, xs, ts, pri, reducer=red)
            res[step] = {"loss": torch.stack(parts).cpu(),
                         "grads": {k: p.grad.detach().cpu().clone()
                                   for k, p in m.named_parameters() if p.grad is not None}}
        res["buffers"] = {k: v.cpu().clone() for k, v in m.named_buffers()
                          if v.is_floating_point()}
        res["hooked"] = len(red.hooks)
        torch.save(res, os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_dataparallel_equivalence_two_ranks(cuda, tmp_path):
    import copy
    from _util import rel_err
    from nets.retinaface_training import MultiBoxLoss
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    ranks = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    # DataParallel emulation in one process: a replica per half, loss on the whole batch
    m, x, tg, pri, cfg = _setup()
    rep = copy.deepcopy(m)
    o0, o1 = m(x[:2]), rep(x[2:])
    out = tuple(torch.cat([a, b]) for a, b in zip(o0, o1))
    crit = MultiBoxLoss(2, 0.35, 7, cfg["variance"], True)
    l, c, lm = crit(out, pri, tg)
    (2.0 * l + c + lm).backward()
    ref_loss = torch.stack([l, c, lm]).detach().cpu()
    named_rep = dict(rep.named_parameters())
    ref_grads = {k: (p.grad + named_rep[k].grad).cpu() for k, p in m.named_parameters()
                 if p.grad is not None}
    assert ranks[0]["hooked"] > 0
    for step in (0, 1):
        got_loss = ranks[0][step]["loss"] + ranks[1][step]["loss"]
        assert rel_err(got_loss, ref_loss) < 1e-4, (step, got_loss, ref_loss)
        g0, g1 = ranks[0][step]["grads"], ranks[1][step]["grads"]
        assert g0.keys() == ref_grads.keys(), set(g0) ^ set(ref_grads)
        worst = max((rel_err(g0[k], ref_grads[k]), k) for k in ref_grads
                    if not k.endswith("f_key.bias") and not k.endswith("skip.2.bias"))
        assert worst[0] < 1e-4, worst
        for k in g0:
            assert torch.equal(g0[k], g1[k]), k   # every rank holds the same sum
    # rank 0's running statistics (after two identical steps) reach every rank
    for k, v in ranks[0]["buffers"].items():
        assert torch.equal(v, ranks[1]["buffers"][k]), k
