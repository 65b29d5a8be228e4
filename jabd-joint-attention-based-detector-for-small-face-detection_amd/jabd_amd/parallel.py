"""Data-parallel training over RCCL (one process per GPU) with the
reference's DataParallel semantics.

The reference wraps the model in nn.DataParallel (train_mobilenetV3_ecagai.py:
462-466): the batch is scattered over GPUs, BatchNorm statistics are per
shard, the loss is computed on the gathered global batch (so its
normalisers are global positive counts) and gradients are summed onto GPU 0;
only GPU 0's BN running buffers survive.  Here each rank holds a full
replica, MultiBoxLoss all-reduces the positive counts (nets/
retinaface_training.py), and this module:

  * all-reduces gradients with SUM (not DDP's mean) in flat buckets sized for
    xGMI ring all-reduce — parameters without a gradient (the built-but-unused
    SeModule weights) are skipped;
  * broadcasts BN running buffers from rank 0 after each step.

Collectives run on torch.distributed ("nccl" = RCCL on ROCm, or "gloo" in
the CPU tests).
"""
import torch
import torch.distributed as dist

BUCKET_BYTES = 32 << 20  # per all-reduce: large enough to amortise the ring's latency


class GradAllReduce:
    def __init__(self, model, group=None, bucket_bytes=BUCKET_BYTES):
        self.model = model
        self.group = group
        self.bucket_bytes = bucket_bytes

    def _buckets(self, params):
        bucket, size = [], 0
        for p in params:
            nbytes = p.grad.numel() * p.grad.element_size()
            if bucket and size + nbytes > self.bucket_bytes:
                yield bucket
                bucket, size = [], 0
            bucket.append(p)
            size += nbytes
        if bucket:
            yield bucket

    def __call__(self):
        """SUM-all-reduce every existing gradient (call after backward)."""
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        params = [p for p in self.model.parameters() if p.grad is not None]
        # identical order on every rank: parameters() order is deterministic
        for bucket in self._buckets(params):
            flat = torch.cat([p.grad.reshape(-1) for p in bucket])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            off = 0
            for p in bucket:
                n = p.grad.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n


def broadcast_buffers(model, src=0, group=None):
    """Rank 0's BN running buffers win (DataParallel keeps only replica 0's)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    bufs = [b for b in model.buffers() if b.is_floating_point()]
    if not bufs:
        return
    flat = torch.cat([b.reshape(-1) for b in bufs])
    dist.broadcast(flat, src=src, group=group)
    off = 0
    for b in bufs:
        n = b.numel()
        b.copy_(flat[off:off + n].view_as(b))
        off += n


def shard(batch_images, batch_targets, rank, world):
    """Split a global batch on dim 0 like DataParallel's scatter (rank-major)."""
    B = batch_images.shape[0]
    per = (B + world - 1) // world
    lo, hi = rank * per, min(B, (rank + 1) * per)
    return batch_images[lo:hi], batch_targets[lo:hi]


def train_step(model, criterion, optimizer, images, targets, priors, loc_weight=2.0,
               reducer=None):
    """One fit_one_epoch iteration (train_mobilenetV3_ecagai.py:518-533) on
    this rank's shard: zero_grad -> forward -> MultiBoxLoss -> backward ->
    gradient SUM all-reduce -> optimizer step -> rank-0 BN buffers."""
    optimizer.zero_grad()
    out = model(images)
    r_loss, c_loss, landm_loss = criterion(out, priors, targets)
    loss = loc_weight * r_loss + c_loss + landm_loss
    loss.backward()
    if reducer is not None:
        reducer()
    optimizer.step()
    broadcast_buffers(model)
    return loss.detach(), (r_loss.detach(), c_loss.detach(), landm_loss.detach())
