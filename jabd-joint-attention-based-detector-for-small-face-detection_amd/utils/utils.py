"""Pre-processing helpers — reference utils/utils.py:8-30.

letterbox_image runs on the device (jabd_letterbox_f32, a restatement of the
cv2.resize INTER_LINEAR float path the reference uses; cv2 is not needed).
Use jabd_amd.ops.letterbox(image, size, mean=(104, 117, 123)) to get the
network's NCHW input in one launch (letterbox + preprocess_input + transpose).
"""
import numpy as np
import torch


def letterbox_image(image, size):
    """Aspect-preserving resize + centred pad with 84 (:8-19).  image: HWC array
    or tensor; returns a float64 HWC numpy array like the reference."""
    from jabd_amd import ops
    if not torch.cuda.is_available():
        raise RuntimeError("letterbox_image runs on the HIP device; no GPU is visible")
    t = torch.as_tensor(np.asarray(image, np.float32)).to("cuda")
    out = ops.letterbox(t, size, fill=84.0)
    return out.cpu().numpy().astype(np.float64)


def get_lr(optimizer):
    for param_group in optimizer.param_groups:
        return param_group["lr"]


def preprocess_input(image):
    image -= np.array((104, 117, 123), np.float32)
    return image
