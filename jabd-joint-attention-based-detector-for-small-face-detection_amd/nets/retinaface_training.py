"""MultiBoxLoss, matching and weight init — drop-in for the reference
nets/retinaface_training.py:1-323.

`MultiBoxLoss.forward(predictions, priors, targets)` runs the whole loss on
the device: one batched match/encode kernel for all images (replacing the
reference's per-image Python loop and host round trips, :201-227), then the
loss kernel with on-device hard-negative mining, and a backward kernel wired
through autograd.  In jabd_amd.parallel's data-parallel step the positive
counts that normalise the loss are all-reduced (MultiBoxLoss.global_counts)
so the summed gradient equals the reference's DataParallel gradient of the
global-batch loss.
"""
import contextlib

import torch
import torch.nn as nn

from jabd_amd import ops
from jabd_amd.functional import window_copies


class _MultiBoxLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, loc, conf, landm, loc_t, conf_t, landm_t, neg_pos, group, diou=None):
        sums, counts, sel = ops.multibox_sums(loc, conf, landm, loc_t, conf_t, landm_t, neg_pos,
                                              diou)
        if group is not None:  # (process group,) — see MultiBoxLoss.global_counts
            import torch.distributed as dist
            dist.all_reduce(counts, group=group[0])
        loss = ops.multibox_normalize(sums, counts)
        ctx.save_for_backward(loc, conf, landm, loc_t, conf_t, landm_t, sel, counts)
        ctx.diou = diou
        return loss[0], loss[1], loss[2]

    @staticmethod
    def backward(ctx, g_l, g_c, g_lm):
        loc, conf, landm, loc_t, conf_t, landm_t, sel, counts = ctx.saved_tensors
        dev = loc.device
        # the three scalar gradients as one [3] vector, one launch
        gout = torch.empty(3, dtype=torch.float32, device=dev)
        window_copies([(g.detach().float().contiguous() if g is not None else None,
                        gout[i:i + 1], 0.0) for i, g in enumerate((g_l, g_c, g_lm))])
        gl, gc, glm = ops.multibox_backward(loc, conf, landm, loc_t, conf_t, landm_t, sel,
                                            gout, counts, ctx.diou)
        return gl, gc, glm, None, None, None, None, None, None


def match(threshold, truths, priors, variances, labels, landms, loc_t, conf_t, landm_t, idx):
    """Single-image match() with the reference's in-place output contract (:93-162)."""
    t = torch.cat([truths, landms, labels.reshape(-1, 1)], 1)
    lt, ct, lmt = ops.match_encode([t.to(priors.device).float()], priors, threshold, variances)
    loc_t[idx] = lt[0].to(loc_t.device)
    conf_t[idx] = ct[0].to(conf_t.device)
    landm_t[idx] = lmt[0].to(landm_t.device)


def log_sum_exp(x):
    """Reference :86-88 (kept for API compatibility; the loss kernel fuses it)."""
    x_max = x.data.max()
    return torch.log(torch.sum(torch.exp(x - x_max), 1, keepdim=True)) + x_max


class MultiBoxLoss(nn.Module):
    """nets/retinaface_training.py:165-303.  Normalisers are this call's own
    positive counts, as the reference's.  Under one-process-per-GPU data
    parallelism with SUM-reduced gradients (jabd_amd.parallel.train_step), the
    counts must be the global batch's: that step enters
    `with criterion.global_counts(True, group):` and the counts are
    all-reduced before normalising.  (Never enable it under DDP, which
    averages gradients: the global normaliser would then shrink the gradient
    by the world size.)"""

    def __init__(self, num_classes, overlap_thresh, neg_pos, variance, cuda=True):
        super().__init__()
        if num_classes != 2:
            raise ValueError("the JABD loss kernel is built for 2 classes (face/background)")
        self.num_classes = num_classes
        self.threshold = overlap_thresh
        self.negpos_ratio = neg_pos
        self.variance = variance
        self.cuda = cuda
        self._count_group = None   # (group,) while global_counts is active

    @contextlib.contextmanager
    def global_counts(self, enabled=True, group=None):
        prev = self._count_group
        self._count_group = (group,) if enabled else None
        try:
            yield self
        finally:
            self._count_group = prev

    def forward(self, predictions, priors, targets):
        loc_data, conf_data, landm_data = predictions
        priors = priors.to(loc_data.device).float().contiguous()
        tg = [t.to(loc_data.device).float() for t in targets]
        with torch.no_grad():
            loc_t, conf_t, landm_t = ops.match_encode(tg, priors, self.threshold, self.variance)
        return _MultiBoxLossFn.apply(loc_data.contiguous(), conf_data.contiguous(),
                                     landm_data.contiguous(), loc_t, conf_t, landm_t,
                                     int(self.negpos_ratio), self._count_group)


def weights_init(net, init_type="normal", init_gain=0.02):
    """Reference :305-323: conv weights N(0, gain) (or xavier/kaiming/orthogonal),
    BatchNorm2d weight N(1, 0.02), bias 0."""
    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, "weight") and classname.find("Conv") != -1:
            if init_type == "normal":
                torch.nn.init.normal_(m.weight.data, 0.0, init_gain)
            elif init_type == "xavier":
                torch.nn.init.xavier_normal_(m.weight.data, gain=init_gain)
            elif init_type == "kaiming":
                torch.nn.init.kaiming_normal_(m.weight.data, a=0, mode="fan_in")
            elif init_type == "orthogonal":
                torch.nn.init.orthogonal_(m.weight.data, gain=init_gain)
            else:
                raise NotImplementedError(f"initialization method [{init_type}] is not implemented")
        elif classname.find("BatchNorm2d") != -1:
            torch.nn.init.normal_(m.weight.data, 1.0, 0.02)
            torch.nn.init.constant_(m.bias.data, 0.0)
    print(f"initialize network with {init_type} type")
    net.apply(init_func)
