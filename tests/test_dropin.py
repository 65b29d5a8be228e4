"""The drop-in surface on CPU (no kernel calls): every `from nets... / from
utils...` name the reference's callers import exists here (the list is parsed
from the reference text by tests/golden/make_ref_imports.py), every exported
nn.Module runs on the HIP path (HipModule), and the host-side pieces
(configs, label parsing, collate, loss history, pack-cache invalidation)
behave like the reference's."""
import importlib
import json
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REF_IMPORTS = json.load(open(os.path.join(HERE, "golden", "ref_imports.json")))


@pytest.mark.parametrize("key", sorted(REF_IMPORTS))
def test_reference_import_resolves(key):
    mod, name = key.split(":")
    m = importlib.import_module(mod)
    assert hasattr(m, name), f"{key} (imported at {REF_IMPORTS[key]})"


def test_every_exported_module_runs_on_the_hip_path():
    """No exported nn.Module falls back to torch's own forward: each is a
    HipModule (a subclass of the torch class where the reference used one)."""
    from jabd_amd.hipmodule import HipModule
    allowed = {nn.Sequential, nn.ModuleList, nn.Identity, nn.Dropout, nn.Conv1d, nn.MaxPool2d}
    for modname in ("nets.retinaface_r", "nets.retinaface_eca_nonlocal", "nets.mobilenetV3",
                    "nets.mobilenet025", "nets.layers", "nets.resnet_pytorch_r",
                    "nets.retinaface_beca"):
        mod = importlib.import_module(modname)
        for name, cls in vars(mod).items():
            if isinstance(cls, type) and issubclass(cls, nn.Module) and \
                    cls.__module__ == modname:
                assert issubclass(cls, HipModule), f"{modname}.{name}"
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    for name, m in RetinaFace(cfg_mnet).named_modules():
        if type(m) in allowed:
            continue  # containers / parameter holders the fused modules read
        assert isinstance(m, HipModule), f"{name}: {type(m)}"


def test_state_dict_keys_unchanged_by_hip_subclasses():
    from nets.retinaface_r import RetinaFace
    from utils.config import cfg_mnet
    sd = RetinaFace(cfg_mnet).state_dict()
    for k in ("body.conv1.weight", "body.layer1.3.skip.2.bias", "body.layer3.4.se.se.2.running_var",
              "fpn.merge1.1.num_batches_tracked", "fpn.output1.0.weight", "ssh1.conv7x7_3.1.bias",
              "LandmarkHead.2.conv1x1.weight", "eca_fpn.conv.weight"):
        assert k in sd, k
    assert len(sd) == 555


def test_backbone_names_and_classifier_shapes():
    from nets import mobilenetV3 as mv3
    from nets.resnet_pytorch_r import resnet18, resnet50, resnet101
    assert sum(p.numel() for p in mv3.MobileNetV3_Small().parameters()) == 2950524
    assert sum(p.numel() for p in resnet18().parameters()) == 11689512
    assert sum(p.numel() for p in resnet50().parameters()) == 25557032
    assert len(resnet101().layer3) == 23


@pytest.mark.parametrize("ctor", [
    lambda: importlib.import_module("nets.retinaface50_self").RetinaFace({}),
    lambda: importlib.import_module("nets.resnet_pytorch_r").resnext50_32x4d(),
])
def test_out_of_scope_models_fail_at_construction(ctor):
    with pytest.raises(NotImplementedError):
        ctor()


def test_configs_match_reference_values():
    from utils import config as C
    assert C.cfg_re152["steps"] == [4, 8, 16, 32] and C.cfg_re101["steps"] == [8, 16, 32, 60]
    assert C.cfg_re50_self["return_layers"]["layer5"] == 4
    assert C.cfg_mnet_4["min_sizes"][0] == [4, 12] and C.cfg_re152_["name"] == "Resnet152"


def test_label_parsing_and_collate(tmp_path):
    """utils/dataloader.py:27-58,151-186 on a two-image label.txt."""
    from utils.dataloader import DataGenerator, _annotations, detection_collate, process_labels
    d = tmp_path / "train"
    d.mkdir()
    (d / "label.txt").write_text(
        "# 0--Parade/a.jpg\n"
        "10 20 30 40 15.0 25.0 0.0 20.0 26.0 0.0 18.0 30.0 0.0 14.0 35.0 0.0 22.0 35.0 0.0 0.9\n"
        "5 5 8 9 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1.0 -1\n"
        "# 0--Parade/b.jpg\n")
    paths, words = process_labels(str(d / "label.txt"))
    assert paths == [str(d / "images/0--Parade/a.jpg"), str(d / "images/0--Parade/b.jpg")]
    assert len(words) == 2 and len(words[0]) == 2 and words[1] == []
    ann = _annotations(words[0])
    np.testing.assert_array_equal(ann[0, :4], [10, 20, 40, 60])
    np.testing.assert_array_equal(ann[0, 4:14], [15, 25, 20, 26, 18, 30, 14, 35, 22, 35])
    assert ann[0, 14] == 1 and ann[1, 14] == -1
    gen = DataGenerator(str(d / "label.txt"), 64)
    assert len(gen) == 2 and gen.get_len() == 2
    imgs, tg = detection_collate([(np.zeros((3, 4, 4), np.float32), ann), ("pil", np.zeros((0, 15)))])
    assert imgs.shape == (1, 3, 4, 4) and len(tg) == 1
    timgs, _ = detection_collate([(torch.zeros(3, 4, 4), ann)] * 2)
    assert isinstance(timgs, torch.Tensor) and timgs.shape == (2, 3, 4, 4)


def test_loss_history(tmp_path, monkeypatch):
    import time
    from utils.callbacks import LossHistory
    monkeypatch.setattr(time, "strftime", lambda fmt, *a: "2026_01_02_03_04_05")
    h = LossHistory(str(tmp_path))
    for v in (3.0, 2.5, 2.0):
        h.append_loss(v)
    txt = [f for f in os.listdir(h.save_path) if f.endswith(".txt")]
    # the reference's names: loss_<stamp>/epoch_loss_<stamp>.txt (utils/callbacks.py:14,21)
    assert txt == ["epoch_loss_" + h.time_str + ".txt"]
    assert os.path.basename(h.save_path) == "loss_" + h.time_str
    assert open(os.path.join(h.save_path, txt[0])).read().split() == ["3.0", "2.5", "2.0"]
    with pytest.raises(FileExistsError):   # a second run in the same second fails, as the reference's
        LossHistory(str(tmp_path))


def test_pack_cache_invalidation_events():
    """Eval packs are rebuilt after train()/eval(), .to(), load_state_dict at any
    depth and jabd_amd.hipmodule.invalidate(); a plain forward does not walk
    the parameters (hipmodule.py)."""
    from jabd_amd import hipmodule as H
    from nets.layers import SSH
    m = SSH(40, 40)
    builds = []
    dev = torch.device("cpu")

    def get():
        return m._jabd_cached(dev, lambda: builds.append(1) or len(builds))

    assert get() == 1 and get() == 1
    m.eval()
    assert get() == 2
    m.conv3X3.load_state_dict(m.conv3X3.state_dict())
    assert get() == 3
    m.float()
    assert get() == 4
    H.invalidate()
    assert get() == 5
    with torch.no_grad():
        m.conv3X3[0].weight = nn.Parameter(m.conv3X3[0].weight * 2)  # a new tensor
    assert get() == 6 and get() == 6
