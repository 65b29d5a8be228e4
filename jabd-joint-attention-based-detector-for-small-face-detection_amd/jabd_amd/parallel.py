"""Data-parallel training over RCCL (one process per GPU) with the
reference's DataParallel semantics.

The reference wraps the model in nn.DataParallel (train_mobilenetV3_ecagai.py:
462-466): the batch is scattered over GPUs, BatchNorm statistics are per
shard, the loss is computed on the gathered global batch (so its
normalisers are global positive counts) and gradients are summed onto GPU 0;
only GPU 0's BN running buffers survive.  Here each rank holds a full
replica and:

  * MultiBoxLoss all-reduces the positive counts `(sum pos, sum pos1)` over
    the group (`MultiBoxLoss.global_counts(True, group)`, entered by
    train_step) before normalising — 16 bytes, latency-bound.  Outside it the
    loss normalises by its own batch's counts, as the reference's;
  * GradAllReduce SUM-all-reduces gradients (not DDP's mean) in flat buckets
    sized for xGMI ring all-reduce.  Buckets are launched from gradient hooks
    while backward is still running (overlap), in one fixed order on every
    rank; parameters that never get a gradient (the reference's built-but-
    unused SeModule weights) are found on the first step and left out, and
    the buckets are planned again whenever the set of parameters with
    gradients changes (freezing / unfreezing the backbone);
  * broadcast_buffers copies rank 0's BN running buffers to every rank.

Collectives run on torch.distributed ("nccl" = RCCL on ROCm, or "gloo").
"""
import torch
import torch.distributed as dist

BUCKET_BYTES = 32 << 20  # per all-reduce: large enough to amortise the ring's latency


def _world(group):
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


class GradAllReduce:
    """SUM all-reduce of every gradient after backward.

    overlap=True: buckets are filled by post-accumulate-grad hooks and their
    all-reduces launched asynchronously during backward — bucket i only after
    buckets 0..i-1, so every rank issues the same collective sequence.  Call
    the object after loss.backward() to wait for the collectives and write
    the sums back into .grad.

    The plan (which parameters, in which buckets) is made from the
    parameters that actually received a gradient in a synchronous step, and
    is made again whenever that set changes: when the requires_grad flags
    change (the reference's Freeze_Train schedule, train_mobilenetV3_ecagai.py:
    576-610, freezes the backbone and later unfreezes it on the same model),
    when a parameter outside the plan gets a gradient, or when a planned
    bucket stays incomplete.  Such a step waits for (and discards) the
    collectives already launched and all-reduces synchronously instead; every
    rank runs the same graph, so every rank takes the same branch."""

    def __init__(self, model, group=None, bucket_bytes=BUCKET_BYTES, overlap=True):
        self.model = model
        self.group = group
        self.bucket_bytes = bucket_bytes
        self.overlap = overlap
        self.buckets = None      # [[param, ...], ...] in launch order
        self.plan_key = None     # requires_grad flags the plan was made under
        self.hooks = []
        self.hooked = set()      # parameters whose post-accumulate hook is installed
        self.replans = 0         # consecutive steps that had to plan again
        self._reset()
        if overlap:
            self._observe()

    # ---------------------------------------------------------------- buckets
    def _plan(self, params):
        """Buckets over `params` in reverse registration order (backward
        produces the last layers' gradients first)."""
        buckets, cur, size = [], [], 0
        for p in reversed(params):
            nbytes = p.numel() * p.element_size()
            if cur and size + nbytes > self.bucket_bytes:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            buckets.append(cur)
        return buckets

    def _reset(self):
        self.pending = {}
        self.flat = {}
        self.works = {}
        self.next_launch = 0
        self.unplanned = False
        self.fired = set()       # parameters whose gradient was accumulated this step

    def _observe(self):
        """Hooks that only record which parameters receive a gradient (the
        first step's plan is made from them)."""
        self.remove()
        self.where = {}
        for p in self.model.parameters():
            if p.requires_grad:
                self.hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
                self.hooked.add(p)

    def _key(self):
        return tuple(p.requires_grad for p in self.model.parameters())

    def _install(self, params):
        """Hooks on every parameter that can receive a gradient: the planned
        ones fill buckets, any other one marks the step as unplanned."""
        self.remove()
        self.buckets = self._plan(params)
        self.plan_key = self._key()
        self.where = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.where[p] = bi
        for p in self.model.parameters():
            if p.requires_grad:
                self.hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
                self.hooked.add(p)

    def _on_grad(self, p):
        self.fired.add(p)
        if self.buckets is None:
            return
        bi = self.where.get(p)
        if bi is None:
            self.unplanned = True
            return
        left = self.pending.get(bi, len(self.buckets[bi])) - 1
        self.pending[bi] = left
        if left == 0 and not self.unplanned:
            b = self.buckets[bi]
            self.flat[bi] = torch.cat([q.grad.reshape(-1) for q in b])
            while self.next_launch in self.flat and self.next_launch not in self.works:
                i = self.next_launch
                self.works[i] = dist.all_reduce(self.flat[i], op=dist.ReduceOp.SUM,
                                                group=self.group, async_op=True)
                self.next_launch += 1

    def _with_grad(self):
        """The parameters that received a gradient this step: those whose hook
        fired (a stale .grad kept by zero_grad(set_to_none=False) does not
        count), plus any un-hooked one (requires_grad switched on since the
        hooks were installed) holding a gradient; with no hook fired at all
        (gradients written by hand, no backward) every .grad counts."""
        return [p for p in self.model.parameters() if p.requires_grad and p.grad is not None and
                (not self.fired or p in self.fired or p not in self.hooked)]

    def _sync_all(self, params):
        for b in self._plan(params):
            flat = torch.cat([p.grad.reshape(-1) for p in b])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            self._scatter(b, flat)

    @staticmethod
    def _scatter(bucket, flat):
        off = 0
        for p in bucket:
            n = p.grad.numel()
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
            off += n

    def __call__(self):
        """Finish the step's gradient SUM all-reduce (call after backward)."""
        if not _world(self.group):
            self._reset()
            return
        if not self.overlap:
            self._sync_all(self._with_grad())
            return
        ok = (self.buckets is not None and not self.unplanned and self.plan_key == self._key()
              and len(self.works) == len(self.buckets))
        if ok:
            for i, b in enumerate(self.buckets):
                self.works[i].wait()
                self._scatter(b, self.flat[i])
            self._reset()
            self.replans = 0
            return
        self.replans += 1
        if self.replans == 3:
            import warnings
            warnings.warn("GradAllReduce: the gradient set changed on 3 consecutive steps; "
                          "the all-reduce runs synchronously (no overlap with backward)")
        # first step, or the set of parameters with gradients changed: drain
        # what was launched (those sums went to flat copies, .grad is intact),
        # all-reduce this step synchronously and plan again from it
        for w in self.works.values():
            w.wait()
        params = self._with_grad()
        self._sync_all(params)
        self._install(params)
        self._reset()

    def remove(self):
        for h in self.hooks:
            h.remove()
        self.hooks = []
        self.hooked = set()


def broadcast_buffers(model, src=0, group=None):
    """Rank 0's BN running buffers win (DataParallel keeps only replica 0's)."""
    if not _world(group):
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


class _WeightedLossFn(torch.autograd.Function):
    """loss = w * loss_l + loss_c + loss_landm (train_mobilenetV3_ecagai.py:529)
    in one launch; the backward hands (w * g, g, g) to MultiBoxLoss."""

    @staticmethod
    def forward(ctx, r, c, lm, w):
        out = torch.empty((), dtype=torch.float32, device=r.device)
        from ._lib import call
        from .functional import _stream
        call("jabd_weighted_sum3_f32", r.data_ptr(), c.data_ptr(), lm.data_ptr(), w,
             out.data_ptr(), _stream())
        ctx.w = w
        return out

    @staticmethod
    def backward(ctx, g):
        from .functional import window_copies
        g = g.contiguous()
        gr = torch.empty((), dtype=torch.float32, device=g.device)
        window_copies([(g, gr, 0.0, 0, ctx.w)])
        return gr, g, g, None


_ONE = {}


def _one(dev):
    """The backward seed d(loss)/d(loss) = 1, allocated once per device."""
    t = _ONE.get(str(dev))
    if t is None:
        t = _ONE[str(dev)] = torch.ones((), dtype=torch.float32, device=dev)
    return t


def train_step(model, criterion, optimizer, images, targets, priors, loc_weight=2.0,
               reducer=None):
    """One fit_one_epoch iteration (train_mobilenetV3_ecagai.py:518-533) on
    this rank's shard: zero_grad -> forward -> MultiBoxLoss with global
    positive counts -> backward (bucketed gradient SUM all-reduce overlapped)
    -> optimizer step -> rank-0 BN buffers."""
    group = reducer.group if reducer is not None else None
    optimizer.zero_grad()
    out = model(images)
    with criterion.global_counts(reducer is not None and _world(group), group):
        r_loss, c_loss, landm_loss = criterion(out, priors, targets)
    loss = _WeightedLossFn.apply(r_loss, c_loss, landm_loss, float(loc_weight))
    torch.autograd.backward(loss, _one(loss.device))
    if reducer is not None:
        reducer()
    optimizer.step()
    broadcast_buffers(model, group=group)
    return loss.detach(), (r_loss.detach(), c_loss.detach(), landm_loss.detach())
