"""Detector configs — the reference's utils/config.py:1-152 (every dict the
reference's scripts import).  cfg_mnet drives JABD-MobileNetV3, cfg_re50 the
R50 detector; the others are the ablation configs (ResNet-101/152, the
5-stage "self" ResNets, the 4-level MobileNetV3) kept for import parity."""
cfg_mnet = {
    "name": "mobilenet0.25",
    "min_sizes": [[16, 32], [64, 128], [256, 512]],
    "steps": [8, 16, 32],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer1": 1, "layer2": 2, "layer3": 3},
    "in_channel": 20,
    "out_channel": 40,
}

# MobileNetV3_Small + the JABD ECA head (BASELINE config 1; no reference
# counterpart — see nets.retinaface_r.RetinaFace_Small).  Same anchors as cfg_mnet.
cfg_mnv3_small = dict(cfg_mnet, name="mobilenetv3_small", return_layers={}, in_channel=None)

cfg_mnet_4 = {
    "name": "mobilenetV3",
    "min_sizes": [[4, 12], [16, 32], [64, 128], [256, 512]],
    "steps": [8, 16, 16, 32],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer1": 1, "layer2": 2, "layer3": 3, "layer4": 4},
    "in_channel": 20,
    "out_channel": 40,
}

cfg_re50 = {
    "name": "Resnet50",
    "min_sizes": [[16, 32], [64, 128], [256, 512]],
    "steps": [8, 16, 32],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer2": 1, "layer3": 2, "layer4": 3},
    "in_channel": 256,
    "out_channel": 256,
}

cfg_re50_self = {
    "name": "Resnet50_self",
    "min_sizes": [[8, 16], [32, 64], [64, 128], [256, 512]],
    "steps": [8, 16, 32, 64],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer2": 1, "layer3": 2, "layer4": 3, "layer5": 4},
    "in_channel": 256,
    "out_channel": 256,
}

cfg_re152_ = {
    "name": "Resnet152",
    "min_sizes": [[16, 32], [64, 128], [256, 512]],
    "steps": [8, 16, 32],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer2": 1, "layer3": 2, "layer4": 3},
    "in_channel": 256,
    "out_channel": 256,
}

cfg_re152 = {
    "name": "Resnet152",
    "min_sizes": [[8, 16], [32, 64], [64, 128], [256, 512]],
    "steps": [4, 8, 16, 32],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer1": 1, "layer2": 2, "layer3": 3, "layer4": 4},
    "in_channel": 256,
    "out_channel": 256,
}

cfg_re101 = {
    "name": "Resnet101",
    "min_sizes": [[32, 64], [64, 128], [256, 512], [240, 480]],
    "steps": [8, 16, 32, 60],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer2": 2, "layer3": 3, "layer4": 4, "layer5": 5},
    "in_channel": 256,
    "out_channel": 256,
}

cfg_re152_new = {
    "name": "Resnet152",
    "min_sizes": [[8, 16], [32, 64], [64, 128], [256, 512]],
    "steps": [4, 8, 16, 32],
    "variance": [0.1, 0.2],
    "clip": False,
    "loc_weight": 2.0,
    "train_image_size": 840,
    "return_layers": {"layer2": 1, "layer3": 2, "layer4": 3, "layer5": 4},
    "in_channel": 256,
    "out_channel": 256,
}
