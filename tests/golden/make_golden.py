"""Generate the committed golden vectors of tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

The reference (JABD2080ti) may not be imported or executed in this pipeline
(SURVEY.md §8c), so these vectors come from the oracle restatement
(oracle/box_ref.py, oracle/nms_ref.c) on small seeded inputs, plus the
reference's own known answer for the anchor count.  They pin the oracle
against silent drift (tests/test_golden.py re-derives them on the CPU) and
give the GPU tests fixed expected outputs that do not need the oracle at run
time.  Inputs and expected outputs only; no reference source.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")]

from oracle import box_ref  # noqa: E402

CFG = {"min_sizes": [[16, 32], [64, 128], [256, 512]], "steps": [8, 16, 32], "clip": False}


def nms_case(seed, n, tie_frac=0.1):
    rng = np.random.default_rng(seed)
    c = rng.uniform(0, 1, (n // 8 + 1, 2))[rng.integers(0, n // 8 + 1, n)]
    c = c + rng.normal(0, 0.01, c.shape)
    wh = np.exp(rng.uniform(np.log(0.01), np.log(0.2), (n, 2)))
    boxes = np.concatenate([c - wh / 2, c + wh / 2], 1).astype(np.float32)
    scores = rng.uniform(0.5, 1.0, n).astype(np.float32)
    ties = rng.uniform(size=n) < tie_frac
    scores[ties] = scores[0]
    return boxes, scores


def main():
    out = {}
    # A6 anchors (cfg_mnet steps/min_sizes) at 256x256 and the reference's own KAT
    out["anchors_256"] = box_ref.anchors(CFG, (256, 256)).numpy()
    out["anchor_count_840_ref_kat"] = np.array(
        box_ref.num_anchors({"steps": [8, 16, 32, 64], "min_sizes": [[16, 32]] * 4}, (840, 840)))
    # A10 NMS (torchvision-CPU semantics) at three thresholds, ties included
    for i, (n, thr) in enumerate([(300, 0.3), (1000, 0.5), (2000, 0.7)]):
        b, s = nms_case(100 + i, n)
        out[f"nms{i}_boxes"], out[f"nms{i}_scores"] = b, s
        out[f"nms{i}_thr"] = np.array(thr)
        out[f"nms{i}_keep"] = box_ref.nms(b, s, thr)
    # A7/A8 match + encode on two WIDER-shaped 128x128 images
    from jabd_amd import synth
    tg = synth.targets(2, 128, seed=77)
    pri = box_ref.anchors(CFG, (128, 128))
    lt, ct, lmt = box_ref.match_batch([torch.from_numpy(t) for t in tg], pri)
    for k, t in enumerate(tg):
        out[f"match_targets{k}"] = t
    out["match_loc_t"], out["match_conf_t"], out["match_landm_t"] = lt.numpy(), ct.numpy(), lmt.numpy()
    # A9 MultiBoxLoss on seeded predictions for the matched targets
    g = torch.Generator().manual_seed(5)
    A = pri.shape[0]
    loc = torch.randn(2, A, 4, generator=g)
    conf = torch.randn(2, A, 2, generator=g) * 2
    landm = torch.randn(2, A, 10, generator=g)
    rl, rc, rlm, info = box_ref.multibox_loss(loc, conf, landm, lt, ct, lmt)
    out["loss_loc"], out["loss_conf"], out["loss_landm"] = loc.numpy(), conf.numpy(), landm.numpy()
    out["loss_values"] = np.array([float(rl), float(rc), float(rlm)], dtype=np.float64)
    out["loss_counts"] = np.array(info["counts"], dtype=np.int64)
    # A10 decode
    out["decode_boxes"] = box_ref.decode(loc[0], pri, (0.1, 0.2)).numpy()
    out["decode_landms"] = box_ref.decode_landm(landm[0], pri, (0.1, 0.2)).numpy()
    np.savez_compressed(os.path.join(HERE, "box_ops_golden.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
