"""IntermediateLayerGetter with torchvision's semantics and key layout
(children kept in order until every return layer has been seen; forward
returns an OrderedDict of the requested outputs), used as `RetinaFace.body`
so checkpoints keep keys like `body.layer1.0.conv1.weight`.

Its forward walks the children like torchvision's, with the backbone stem's
conv -> BN -> act run as one fused launch (jabd_amd.modules.run_sequential's
peephole); every child runs libjabd kernels."""
from collections import OrderedDict

import torch.nn as nn

from jabd_amd import modules as M
from jabd_amd.hipmodule import HipModule


class IntermediateLayerGetter(HipModule, nn.ModuleDict):
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
        out = OrderedDict()
        items = list(self.items())
        i = 0
        while i < len(items):
            name, m = items[i]
            if isinstance(m, nn.Conv2d) and i + 1 < len(items) and \
                    isinstance(items[i + 1][1], nn.BatchNorm2d) and \
                    name not in self.return_layers and items[i + 1][0] not in self.return_layers:
                a = M.act_of(items[i + 2][1]) if i + 2 < len(items) else None
                n = 3 if a is not None else 2
                with M._Mode(m):
                    x = M.nchw(M.conv_bn_act(m, m, items[i + 1][1], x, *(a or ("none", 0.0))))
                last = items[i + n - 1][0]
                i += n
                if last in self.return_layers:
                    out[self.return_layers[last]] = x
                continue
            x = m(x)
            if name in self.return_layers:
                out[self.return_layers[name]] = x
            i += 1
        return out
