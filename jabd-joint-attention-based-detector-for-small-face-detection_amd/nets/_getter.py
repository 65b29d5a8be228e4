"""IntermediateLayerGetter with torchvision's key layout (children kept in
order until every return layer has been seen), used as `RetinaFace.body`
so checkpoints keep keys like `body.layer1.0.conv1.weight`."""
from collections import OrderedDict

import torch.nn as nn


class IntermediateLayerGetter(nn.ModuleDict):
    def __init__(self, model, return_layers):
        names = [n for n, _ in model.named_children()]
        if not set(return_layers).issubset(names):
            raise ValueError("return_layers are not present in model")
        want = dict(return_layers)
        layers = OrderedDict()
        for name, module in model.named_children():
            layers[name] = module
            want.pop(name, None)
            if not want:
                break
        super().__init__(layers)
        self.return_layers = dict(return_layers)

    def forward(self, x):
        raise NotImplementedError(
            "RetinaFace.body runs inside the fused HIP forward (RetinaFace.forward)")
