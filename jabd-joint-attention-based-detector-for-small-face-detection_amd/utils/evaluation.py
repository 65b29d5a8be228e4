"""WIDER FACE evaluation — drop-in for the reference utils/evaluation.py.

The per-image work (bbox_overlaps + image_eval + img_pr_info, :45-63 and
:255-305) runs for every image of a setting in one device launch
(jabd_wider_eval_f64); the 1000-point curve normalisation and the VOC AP
(:308-330) are host numpy over thresh_num rows, as in the reference.
"""
import os

import numpy as np

from jabd_amd import ops


def dataset_pr_info(thresh_num, pr_curve, count_face):
    """:308-313: (precision, recall) per threshold."""
    pr = np.asarray(pr_curve, np.float64)
    out = np.zeros((thresh_num, 2))
    out[:, 0] = pr[:, 1] / pr[:, 0]
    out[:, 1] = pr[:, 1] / count_face
    return out


def voc_ap(rec, prec):
    """:316-330: all-point interpolated AP."""
    mrec = np.concatenate(([0.], rec, [1.]))
    mpre = np.concatenate(([0.], prec, [0.]))
    for i in range(mpre.size - 1, 0, -1):
        mpre[i - 1] = max(mpre[i - 1], mpre[i])
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1])


def norm_score(pred):
    """:226-252: min-max normalise every score over the whole prediction dict."""
    max_score, min_score = 0, 1
    for k in pred.values():
        for v in k.values():
            if len(v) == 0:
                continue
            max_score = max(np.max(v[:, -1]), max_score)
            min_score = min(np.min(v[:, -1]), min_score)
    diff = max_score - min_score
    for k in pred.values():
        for v in k.values():
            if len(v) == 0:
                continue
            v[:, -1] = (v[:, -1] - min_score) / diff


def setting_ap(preds, gts, keep_lists, iou_thresh=0.5, thresh_num=1000):
    """AP of one setting (easy/medium/hard) — the body of :347-382 for flat lists
    of per-image preds [n,5] (x,y,w,h,score normalised), gts [m,4] (x,y,w,h) and
    1-based keep indices."""
    count_face = 0
    P, G, IG = [], [], []
    for pred, gt, keep in zip(preds, gts, keep_lists):
        keep = np.asarray(keep, np.int64).reshape(-1)
        count_face += len(keep)
        gt = np.asarray(gt, np.float64).reshape(-1, 4)
        pred = np.asarray(pred, np.float64).reshape(-1, 5)
        if len(gt) == 0 or len(pred) == 0:
            continue
        ig = np.zeros(len(gt), np.uint8)
        if len(keep):
            ig[keep - 1] = 1
        P.append(pred)
        G.append(gt)
        IG.append(ig)
    pr = ops.wider_pr_curve(P, G, IG, iou_thresh, thresh_num).cpu().numpy()
    curve = dataset_pr_info(thresh_num, pr, count_face)
    return voc_ap(curve[:, 1], curve[:, 0])


def get_gt_boxes(gt_dir):
    """:22-43: the WIDER ground-truth .mat files."""
    from scipy.io import loadmat
    gt = loadmat(os.path.join(gt_dir, "wider_face_val.mat"))
    hard = loadmat(os.path.join(gt_dir, "wider_hard_val.mat"))["gt_list"]
    medium = loadmat(os.path.join(gt_dir, "wider_medium_val.mat"))["gt_list"]
    easy = loadmat(os.path.join(gt_dir, "wider_easy_val.mat"))["gt_list"]
    return gt["face_bbx_list"], gt["event_list"], gt["file_list"], hard, medium, easy


def read_pred_file(filepath):
    """:184-203: '<name>\\n<count>\\n<x y w h s>...'."""
    with open(filepath) as f:
        lines = f.readlines()
    img_file = lines[0].rstrip("\n\r")
    boxes = np.array([[float(x) for x in ln.rstrip("\r\n").split(" ")[:5]] for ln in lines[2:]
                      if ln.strip()]).reshape(-1, 5)
    return img_file.split("/")[-1], boxes


def get_preds(pred_dir):
    """:206-223: {event: {image: boxes}}."""
    boxes = {}
    for event in sorted(os.listdir(pred_dir)):
        current = {}
        for imgtxt in os.listdir(os.path.join(pred_dir, event)):
            name, b = read_pred_file(os.path.join(pred_dir, event, imgtxt))
            current[imgtxt.rstrip(".txt")] = b
        boxes[event] = current
    return boxes


def evaluation(pred, gt_path, iou_thresh=0.5):
    """:333-392: Easy / Medium / Hard AP of a prediction directory."""
    pred = get_preds(pred)
    norm_score(pred)
    facebox_list, event_list, file_list, hard, medium, easy = get_gt_boxes(gt_path)
    aps = []
    for gt_list in (easy, medium, hard):
        P, G, K = [], [], []
        for i in range(len(event_list)):
            pred_list = pred[str(event_list[i][0][0])]
            img_list = file_list[i][0]
            for j in range(len(img_list)):
                P.append(pred_list[str(img_list[j][0][0])])
                G.append(facebox_list[i][0][j][0].astype("float"))
                K.append(gt_list[i][0][j][0])
        aps.append(setting_ap(P, G, K, iou_thresh))
    print("==================== Results ====================")
    print("Easy   Val AP: {}".format(aps[0]))
    print("Medium Val AP: {}".format(aps[1]))
    print("Hard   Val AP: {}".format(aps[2]))
    print("=================================================")
    return aps
