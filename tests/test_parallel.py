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


def _overlap_worker(rank, world, port, q):
    """Two real backward passes through GradAllReduce(overlap=True): step 1 is
    synchronous and installs the hooks, step 2 all-reduces from the hooks
    during backward.  Both must equal the sum of the per-rank gradients."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jabd_amd.parallel import GradAllReduce
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(8, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64),
                                torch.nn.ReLU(), torch.nn.Linear(64, 3))
        unused = torch.nn.Linear(3, 3)  # parameters that never get a gradient
        m.add_module("unused", unused)
        red = GradAllReduce(m, bucket_bytes=4096)  # several buckets
        ok = red.buckets is None              # no plan before the first step
        for step in range(3):
            x = torch.randn(5, 8, generator=torch.Generator().manual_seed(10 * step + rank))
            m.zero_grad()
            m[4](m[3](m[2](m[1](m[0](x))))).square().sum().backward()
            mine = [p.grad.clone() for p in m.parameters() if p.grad is not None]
            allg = [torch.zeros_like(t) for t in mine]
            for t, a in zip(mine, allg):  # reference: explicit sum of both ranks' grads
                lst = [torch.zeros_like(t) for _ in range(world)]
                dist.all_gather(lst, t)
                a.copy_(sum(lst))
            red()
            got = [p.grad for p in m.parameters() if p.grad is not None]
            ok &= len(got) == 6 and all(torch.allclose(g, a, rtol=1e-6, atol=1e-6)
                                         for g, a in zip(got, allg))
            ok &= unused.weight.grad is None
            ok &= red.hooks != [] and len(red.buckets) > 1   # planned after step 1
            ok &= red.works == {} and red.pending == {}
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_overlap_hooks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _freeze_worker(rank, world, port, q):
    """The reference's Freeze_Train schedule (train_mobilenetV3_ecagai.py:
    576-610) on one model: the first part frozen for two steps, then
    unfrozen.  After unfreezing, its gradients must be SUM-reduced too (the
    reducer plans again), and every step equals the explicit sum of both
    ranks' gradients; a parameter that stops receiving a gradient also
    triggers a re-plan instead of an error."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jabd_amd.parallel import GradAllReduce
        torch.manual_seed(0)
        body = torch.nn.Sequential(torch.nn.Linear(8, 32), torch.nn.ReLU())
        head = torch.nn.Sequential(torch.nn.Linear(32, 32), torch.nn.ReLU(),
                                   torch.nn.Linear(32, 2))
        m = torch.nn.Sequential(body, head)
        red = GradAllReduce(m, bucket_bytes=1024)
        ok = True
        plan = {}
        for step in range(7):
            frozen = step < 2
            for p in body.parameters():
                p.requires_grad_(not frozen)
            skip_last = step == 5          # the last layer unused for one step
            x = torch.randn(4, 8, generator=torch.Generator().manual_seed(100 * step + rank))
            m.zero_grad()
            h = head[1](head[0](body(x)))
            out = h.sum() if skip_last else head[2](h).square().sum()
            out.backward()
            mine = [(n, p.grad.clone()) for n, p in m.named_parameters() if p.grad is not None]
            want = {}
            for n, t in mine:
                lst = [torch.zeros_like(t) for _ in range(world)]
                dist.all_gather(lst, t)
                want[n] = sum(lst)
            red()
            got = {n: p.grad for n, p in m.named_parameters() if p.grad is not None}
            ok &= set(got) == set(want)
            ok &= all(torch.allclose(got[n], want[n], rtol=1e-6, atol=1e-6) for n in want)
            ok &= any(n.startswith("0.") for n in got) == (not frozen)
            plan[step] = sum(len(b) for b in red.buckets)
        # planned sizes: head only (4 tensors), then head + body (6), then the
        # step without the last layer (4), then all 6 again
        ok &= plan[0] == 4 and plan[1] == 4 and plan[2] == 6 and plan[4] == 6
        ok &= plan[5] == 4 and plan[6] == 6
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_freeze_unfreeze_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_freeze_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _stale_worker(rank, world, port, q):
    """zero_grad(set_to_none=False) leaves a zero .grad on a
    parameter that no longer receives a gradient.  The plan is made from the
    parameters whose gradient hook fired, so that stale tensor is not
    planned, the buckets complete from the hooks and no step re-plans."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from jabd_amd.parallel import GradAllReduce
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 2))
        extra = torch.nn.Linear(2, 2)
        m.add_module("extra", extra)
        extra.weight.grad = torch.zeros_like(extra.weight)     # stale, from an earlier use
        red = GradAllReduce(m, bucket_bytes=256)
        ok = True
        for step in range(4):
            x = torch.randn(4, 8, generator=torch.Generator().manual_seed(step + 7 * rank))
            m.zero_grad(set_to_none=False)
            m[2](m[1](m[0](x))).sum().backward()
            red()
            planned = {id(p) for b in red.buckets for p in b}
            ok &= id(extra.weight) not in planned
            if step >= 1:
                ok &= red.replans == 0
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_ignores_stale_zero_grads_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stale_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
