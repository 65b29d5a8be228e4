"""The reference's 5-stage "self" ResNet-50 ablation (nets/retinaface50_self.py,
used by train_50_4self.py) is outside the JABD hot path:
the name exists so the script imports, and constructing it says so."""


class RetinaFace:
    def __init__(self, cfg=None, pretrained=False, mode="train"):
        raise NotImplementedError(
            "nets.retinaface50_self.RetinaFace (the 5-stage ResNet ablation) is not part of the "
            "MI355X JABD path; use nets.retinaface_eca_nonlocal.RetinaFace (cfg_re50) or "
            "nets.retinaface_r.RetinaFace (cfg_mnet)")
