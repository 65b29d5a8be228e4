"""Detector configs — the reference's utils/config.py:1-57 entries used by
the JABD hot path (cfg_mnet for JABD-MobileNetV3, cfg_re50 for R50)."""
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
