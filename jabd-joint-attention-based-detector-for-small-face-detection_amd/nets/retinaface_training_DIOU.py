"""The DIoU MultiBoxLoss variant — drop-in for the reference
nets/retinaface_training_DIOU.py:176-246 (match_iou) and :491-665
(IouLoss 'Diou' inside MultiBoxLoss).

Differences from nets/retinaface_training.py, all on the device:
  * match_iou() assigns priors exactly like match() but keeps the matched
    truth corners as loc_t (:230 `loc = matches`), one batched kernel
    (`jabd_match_iou_f32`);
  * the box term is Σ_pos 1 - clamp(DIoU(decode(loc, prior), truth), -1, 1)
    (:600-602, bbox_overlaps_diou :402-442), fused into the loss kernel
    (`jabd_multibox_diou_loss_fwd_f32`) with an analytic backward
    (`jabd_multibox_diou_loss_bwd_f32`).
The CE hard-negative mining, landmark term and normalisation are the base
loss's (:604-665 == nets/retinaface_training.py:238-303).
"""
import torch

from jabd_amd import ops
from nets.retinaface_training import (  # noqa: F401  (reference module surface)
    MultiBoxLoss as _BaseMultiBoxLoss, _MultiBoxLossFn, log_sum_exp, match, weights_init)


def match_iou(threshold, truths, priors, variances, labels, landms, loc_t, conf_t, landm_t, idx):
    """Single-image match_iou() with the reference's in-place output contract (:176-246)."""
    t = torch.cat([truths, landms, labels.reshape(-1, 1)], 1)
    lt, ct, lmt = ops.match_encode([t.to(priors.device).float()], priors, threshold, variances,
                                   raw_loc=True)
    loc_t[idx] = lt[0].to(loc_t.device)
    conf_t[idx] = ct[0].to(conf_t.device)
    landm_t[idx] = lmt[0].to(landm_t.device)


class MultiBoxLoss(_BaseMultiBoxLoss):
    """MultiBoxLoss(num_classes, overlap_thresh, neg_pos, variance, cuda) with the
    DIoU box loss (:524-665).  forward((loc, conf, landm), priors, targets) ->
    (loss_l, loss_c, loss_landm)."""

    def forward(self, predictions, priors, targets):
        loc_data, conf_data, landm_data = predictions
        priors = priors.to(loc_data.device).float().contiguous()
        tg = [t.to(loc_data.device).float() for t in targets]
        with torch.no_grad():
            loc_t, conf_t, landm_t = ops.match_encode(tg, priors, self.threshold, self.variance,
                                                      raw_loc=True)
        return _MultiBoxLossFn.apply(loc_data.contiguous(), conf_data.contiguous(),
                                     landm_data.contiguous(), loc_t, conf_t, landm_t,
                                     int(self.negpos_ratio), self._count_group,
                                     (priors, tuple(float(v) for v in self.variance)))
