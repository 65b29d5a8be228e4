"""One training epoch — drop-in for the reference utils/utils_fit_change.py:11-64
(the loop train_50_4self.py imports; the other train_*.py inline the same
loop): zero_grad -> forward -> MultiBoxLoss -> backward -> optimizer step,
per-epoch checkpoint and LossHistory.  Batches may hold numpy images (the
reference's DataGenerator output) or device tensors (DataGenerator(output=
"device")); both reach the model as float32 GPU tensors."""
import os

import numpy as np
import torch

from utils.utils import get_lr


def _to_device(images, targets, cuda):
    dev = "cuda" if cuda else "cpu"
    if isinstance(images, np.ndarray):
        images = torch.from_numpy(images)
    images = images.to(dev, torch.float32)
    targets = [(torch.from_numpy(a) if isinstance(a, np.ndarray) else a).to(dev, torch.float32)
               for a in targets]
    return images, targets


def fit_one_epoch(model_train, model, loss_history, optimizer, criterion, epoch, epoch_step, gen,
                  Epoch, anchors, cfg, cuda, save_dir="logs_50_4", save_period=2):
    total_r, total_c, total_l = 0.0, 0.0, 0.0
    print("Start Train")
    try:
        from tqdm import tqdm
        pbar = tqdm(total=epoch_step, desc=f"Epoch {epoch + 1}/{Epoch}", postfix=dict,
                    mininterval=0.3)
    except ImportError:
        pbar = None
    for iteration, batch in enumerate(gen):
        if iteration >= epoch_step:
            break
        images, targets = batch[0], batch[1]
        if len(images) == 0:
            continue
        with torch.no_grad():
            images, targets = _to_device(images, targets, cuda)
        optimizer.zero_grad()
        out = model_train(images)
        r_loss, c_loss, landm_loss = criterion(out, anchors, targets)
        loss = cfg["loc_weight"] * r_loss + c_loss + landm_loss
        loss.backward()
        optimizer.step()
        total_c += c_loss.item()
        total_r += cfg["loc_weight"] * r_loss.item()
        total_l += landm_loss.item()
        if pbar is not None:
            pbar.set_postfix(**{"Conf Loss": total_c / (iteration + 1),
                                "Regression Loss": total_r / (iteration + 1),
                                "LandMark Loss": total_l / (iteration + 1),
                                "lr": get_lr(optimizer)})
            pbar.update(1)
    if pbar is not None:
        pbar.close()
    print("Saving state, iter:", str(epoch + 1))
    mean_loss = (total_c + total_r + total_l) / (epoch_step + 1)
    if (epoch + 1) % save_period == 0:
        os.makedirs(save_dir, exist_ok=True)
        torch.save(model.state_dict(), os.path.join(
            save_dir, "Epoch%d-Total_Loss%.4f.pth" % (epoch + 1, mean_loss)),
            _use_new_zipfile_serialization=False)
    loss_history.append_loss(mean_loss)
    return mean_loss
