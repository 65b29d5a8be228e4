"""Box decoding and NMS — drop-in for the reference utils/utils_bbox.py
(decode :29-34, decode_landm :39-46, non_max_suppression :260-296,
retinaface_correct_boxes :9-24) with the device work on the HIP path.

`nms` replaces `torchvision.ops.nms` (same signature and result); the
reference imports it at utils/utils_bbox.py:3.
"""
import math

import numpy as np
import torch

from jabd_amd import ops


def retinaface_correct_boxes(result, input_shape, image_shape):
    """Undo the letterbox (reference :9-24).  A device tensor [n, 15] is corrected
    in place by jabd_correct_boxes_f32; host numpy rows (the reference's own
    contract) keep the numpy bookkeeping."""
    if isinstance(result, torch.Tensor):
        return ops.correct_boxes(result, [int(v) for v in input_shape],
                                 [int(v) for v in image_shape], letterbox=True,
                                 to_pixels=False)
    new_shape = image_shape * np.min(input_shape / image_shape)
    offset = (input_shape - new_shape) / 2. / input_shape
    scale = input_shape / new_shape
    sb = np.array([scale[1], scale[0]] * 2)
    sl = np.array([scale[1], scale[0]] * 5)
    ob = np.array([offset[1], offset[0]] * 2)
    ol = np.array([offset[1], offset[0]] * 5)
    result[:, :4] = (result[:, :4] - ob) * sb
    result[:, 5:] = (result[:, 5:] - ol) * sl
    return result


def decode(loc, priors, variances):
    return ops.decode(loc, priors, variances)


def decode_landm(pre, priors, variances):
    return ops.decode_landm(pre, priors, variances)


def nms(boxes, scores, iou_threshold):
    return ops.nms(boxes, scores, iou_threshold)


def non_max_suppression(detection, conf_thres=0.5, nms_thres=0.3):
    """Score filter + greedy NMS on the device; returns numpy [K,15] or []."""
    if detection.dim() != 2 or detection.shape[1] < 5:
        raise ValueError("non_max_suppression expects [N, >=5] rows")
    det = detection.contiguous()
    keep, n_keep = ops.batched_nms(det.unsqueeze(0), det[:, 4].contiguous().unsqueeze(0),
                                   nms_thres, score_threshold=conf_thres)
    k = int(n_keep[0].item())
    if k == 0:
        return []
    return det[keep[0, :k]].cpu().numpy()
