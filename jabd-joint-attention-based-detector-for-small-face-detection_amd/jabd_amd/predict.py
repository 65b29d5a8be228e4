"""predict.py's detect_image (predict.py:115-196) as one device pipeline:
letterbox + preprocess_input (jabd_letterbox_f32) -> RetinaFace eval forward ->
decode + score filter + NMS (jabd_detect_f32) -> retinaface_correct_boxes +
pixel rescale (jabd_correct_boxes_f32).  Only the kept rows leave the device.
"""
import numpy as np
import torch

from jabd_amd import ops


def detect_image(net, image, input_shape, cfg, confidence=0.5, nms_iou=0.3,
                 letterbox_image=True, device="cuda"):
    """image: RGB HWC array (uint8 or float32), as predict.py's np.array(image,
    np.float32).  input_shape = (H, W) of the network input (used only when
    letterbox_image; otherwise the image's own size, as the reference).
    Returns numpy float32 [K, 15] (x1, y1, x2, y2, score, 5 landmark xy) in image
    pixels, NMS order; [] when nothing survives (the reference returns early)."""
    from utils.anchors import Anchors
    img = torch.from_numpy(np.ascontiguousarray(np.asarray(image, np.float32))).to(device)
    ih, iw = int(img.shape[0]), int(img.shape[1])
    H, W = (int(input_shape[0]), int(input_shape[1])) if letterbox_image else (ih, iw)
    x = ops.letterbox(img, (W, H), mean=(104.0, 117.0, 123.0))   # [1, 3, H, W]
    priors = Anchors(cfg, image_size=(H, W)).get_anchors().to(device).float().contiguous()
    with torch.no_grad():
        loc, conf, landm = net(x)
        rows, n_keep = ops.detect(loc, conf, landm, priors, cfg["variance"], confidence, nms_iou)
        k = int(n_keep[0].item())
        if k == 0:
            return []
        det = rows[0, :k].contiguous()
        ops.correct_boxes(det, (H, W), (ih, iw), letterbox=letterbox_image, to_pixels=True)
    return det.cpu().numpy()
