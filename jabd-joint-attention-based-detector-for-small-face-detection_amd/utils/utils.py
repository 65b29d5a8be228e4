"""Pre-processing helpers — reference utils/utils.py:8-30."""
import numpy as np


def letterbox_image(image, size):
    """Aspect-preserving resize + pad with 84 (needs OpenCV, as the reference)."""
    try:
        import cv2
    except ImportError as e:  # OpenCV is not part of this image
        raise RuntimeError("letterbox_image needs OpenCV (cv2), which is not installed") from e
    ih, iw, _ = np.shape(image)
    w, h = size
    scale = min(w / iw, h / ih)
    nw, nh = int(iw * scale), int(ih * scale)
    image = cv2.resize(image, (nw, nh))
    new_image = np.ones([size[1], size[0], 3]) * 84
    new_image[(h - nh) // 2:nh + (h - nh) // 2, (w - nw) // 2:nw + (w - nw) // 2] = image
    return new_image


def get_lr(optimizer):
    for param_group in optimizer.param_groups:
        return param_group["lr"]


def preprocess_input(image):
    image -= np.array((104, 117, 123), np.float32)
    return image
