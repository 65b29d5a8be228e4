"""Data-parallel plumbing (§8e) on CPU with gloo, world_size 2: gradient
SUM all-reduce in buckets (unused parameters skipped), rank-0 BN buffer
broadcast, DataParallel-style batch sharding."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jabd_amd.parallel import GradAllReduce, broadcast_buffers, shard
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(8, 300), torch.nn.BatchNorm1d(300),
                                torch.nn.Linear(300, 4), torch.nn.Linear(4, 4))
        for i, p in enumerate(m.parameters()):
            if i == 6:  # last Linear's weight unused (like the SE weights): no grad
                continue
            p.grad = torch.full_like(p, float(rank + 1) * (i + 1))
        m[1].running_mean.fill_(rank + 10.0)
        GradAllReduce(m, bucket_bytes=2048)()   # tiny buckets: many collectives
        broadcast_buffers(m)
        ok = True
        for i, p in enumerate(m.parameters()):
            if i == 6:
                ok &= p.grad is None
            else:
                ok &= bool(torch.all(p.grad == 3.0 * (i + 1)))
        ok &= bool(torch.all(m[1].running_mean == 10.0))
        imgs = torch.arange(5 * 2).view(5, 2)
        tg = [torch.tensor([k]) for k in range(5)]
        a, t = shard(imgs, tg, rank, world)
        ok &= (a[:, 0].tolist() == ([0, 2, 4] if rank == 0 else [6, 8]))
        ok &= len(t) == len(a)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_and_buffers_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
