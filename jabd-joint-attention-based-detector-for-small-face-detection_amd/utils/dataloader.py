"""GPU data augmentation — drop-in for the image/target part of the reference
utils/dataloader.py:71-149 (DataGenerator.get_random_data) and the
__getitem__ tail (:62-64).

The host draws the random values in the reference's np.random order
(draw_params), the device does the pixel work in two launches
(jabd_augment_u8: PIL BICUBIC resize, paste on grey 128, flip, HSV jitter,
preprocess_input, CHW), and the few target rows are remapped on the host in
numpy exactly as the reference does (including its no-op upper clamps).
"""
import numpy as np
import torch

from jabd_amd import ops


def _rand(a=0.0, b=1.0):
    return np.random.rand() * (b - a) + a


def draw_params(iw, ih, input_shape, jitter=.3, hue=.1, sat=1.5, val=1.5, rand=_rand):
    """The reference's random draws (:75-110), in its call order."""
    h, w = input_shape
    new_ar = w / h * rand(1 - jitter, 1 + jitter) / rand(1 - jitter, 1 + jitter)
    scale = rand(0.25, 3.25)
    if new_ar < 1:
        nh = int(scale * h)
        nw = int(nh * new_ar)
    else:
        nw = int(scale * w)
        nh = int(nw / new_ar)
    dx = int(rand(0, w - nw))
    dy = int(rand(0, h - nh))
    flip = rand() < .5
    hue = rand(-hue, hue)
    sat = rand(1, sat) if rand() < .5 else 1 / rand(1, sat)
    val = rand(1, val) if rand() < .5 else 1 / rand(1, val)
    return dict(nw=nw, nh=nh, dx=dx, dy=dy, flip=flip, hue=hue, sat=sat, val=val)


def remap_targets(box, iw, ih, input_shape, p):
    """Target part of get_random_data (:120-147) for the drawn parameters p."""
    h, w = input_shape
    nw, nh, dx, dy = p["nw"], p["nh"], p["dx"], p["dy"]
    box = np.array(box, copy=True)
    xs, ys = [0, 2, 4, 6, 8, 10, 12], [1, 3, 5, 7, 9, 11, 13]
    if len(box) > 0:
        np.random.shuffle(box)
        box[:, xs] = box[:, xs] * nw / iw + dx
        box[:, ys] = box[:, ys] * nh / ih + dy
        if p["flip"]:
            box[:, xs] = w - box[:, [2, 0, 6, 4, 8, 12, 10]]
            box[:, [5, 7, 9, 11, 13]] = box[:, [7, 5, 9, 13, 11]]
        cx = (box[:, 0] + box[:, 2]) / 2
        cy = (box[:, 1] + box[:, 3]) / 2
        box = box[(cx > 0) & (cy > 0) & (cx < w) & (cy < h)]
        v = box[:, 0:14]
        v[v < 0] = 0
        # the reference's upper clamps (:140-141) assign into fancy-index copies: no-ops
        bw = box[:, 2] - box[:, 0]
        bh = box[:, 3] - box[:, 1]
        box = box[(bw > 1) & (bh > 1)]
    lm = box[:, 4:-1]
    lm[box[:, -1] == -1] = 0
    box[:, xs] /= w
    box[:, ys] /= h
    return box


def get_random_data(image, targets, input_shape, jitter=.3, hue=.1, sat=1.5, val=1.5,
                    device="cuda"):
    """image: PIL image or uint8 RGB [ih, iw, 3] (array or tensor).  Returns
    (float32 [3, h, w] device tensor — already preprocessed and CHW, i.e. the
    reference's __getitem__ image, :62-64 — and the float target rows)."""
    if not torch.cuda.is_available():
        raise RuntimeError("get_random_data runs on the HIP device; no GPU is visible")
    if isinstance(image, torch.Tensor):
        img = image.to(device)
    else:
        img = torch.from_numpy(np.ascontiguousarray(np.asarray(image, np.uint8))).to(device)
    ih, iw = int(img.shape[0]), int(img.shape[1])
    p = draw_params(iw, ih, input_shape, jitter, hue, sat, val)
    out = ops.augment(img, input_shape, p["nw"], p["nh"], p["dx"], p["dy"], p["flip"],
                      p["hue"], p["sat"], p["val"])
    return out, remap_targets(targets, iw, ih, input_shape, p)


def _annotations(labels):
    """WIDER label rows -> [n, 15] targets (utils/dataloader.py:27-58): corners,
    the five landmark points (columns 4,5,7,8,10,11,13,14,16,17), label -1
    when the first landmark is missing (< 0), else 1."""
    ann = np.zeros((0, 15))
    for label in labels:
        a = np.zeros((1, 15))
        a[0, 0], a[0, 1] = label[0], label[1]
        a[0, 2], a[0, 3] = label[0] + label[2], label[1] + label[3]
        for k, col in enumerate((4, 5, 7, 8, 10, 11, 13, 14, 16, 17)):
            a[0, 4 + k] = label[col]
        a[0, 14] = -1 if a[0, 4] < 0 else 1
        ann = np.append(ann, a, axis=0)
    return ann


def process_labels(txt_path):
    """WIDER `label.txt` -> (image paths, per-image label rows) (:151-174)."""
    imgs_path, words, labels = [], [], []
    first = True
    with open(txt_path, "r") as f:
        for line in f.readlines():
            line = line.rstrip()
            if line.startswith("#"):
                if first:
                    first = False
                else:
                    words.append(labels.copy())
                    labels.clear()
                imgs_path.append(txt_path.replace("label.txt", "images/") + line[2:])
            else:
                labels.append([float(x) for x in line.split(" ")])
    words.append(labels)
    return imgs_path, words


class DataGenerator(torch.utils.data.Dataset):
    """Drop-in for the reference DataGenerator (utils/dataloader.py:8-69): WIDER
    label parsing on the host, the augmentation's pixel work on the device
    (get_random_data above).

    output="numpy" (default) returns the image as the reference does (a
    float32 CHW numpy array, what fit_one_epoch's torch.from_numpy expects);
    output="device" keeps it on the GPU (no round trip; detection_collate then
    stacks device tensors).  The device work cannot run in forked DataLoader
    workers (HIP is not fork-safe): use num_workers=0 — one image costs
    ~30 us on the device, so workers buy nothing."""

    def __init__(self, txt_path, img_size, output="numpy", device="cuda"):
        if output not in ("numpy", "device"):
            raise ValueError("output must be 'numpy' or 'device'")
        self.img_size = img_size
        self.txt_path = txt_path
        self.output = output
        self.device = device
        self.imgs_path, self.words = process_labels(txt_path)

    def __len__(self):
        return len(self.imgs_path)

    def get_len(self):
        return len(self.imgs_path)

    def __getitem__(self, index):
        if torch.utils.data.get_worker_info() is not None:
            raise RuntimeError("DataGenerator runs its augmentation on the HIP device, which "
                               "forked DataLoader workers cannot use: pass num_workers=0")
        from PIL import Image
        img = Image.open(self.imgs_path[index]).convert("RGB")
        labels = self.words[index]
        if len(labels) == 0:
            return img, np.zeros((0, 15))
        out, target = get_random_data(img, _annotations(labels), [self.img_size, self.img_size],
                                      device=self.device)
        if self.output == "numpy":
            out = out.cpu().numpy()
        return out, target

    def rand(self, a=0, b=1):
        return _rand(a, b)

    def get_random_data(self, image, targets, input_shape, jitter=.3, hue=.1, sat=1.5, val=1.5):
        return get_random_data(image, targets, input_shape, jitter, hue, sat, val, self.device)

    def process_labels(self):
        return process_labels(self.txt_path)


def detection_collate(batch):
    """Drop images without targets and stack (:177-186): numpy images as the
    reference does, device tensors with torch.stack."""
    images, targets = [], []
    for img, box in batch:
        if len(box) == 0:
            continue
        images.append(img)
        targets.append(box)
    if images and isinstance(images[0], torch.Tensor):
        return torch.stack(images), targets
    return np.array(images), targets
