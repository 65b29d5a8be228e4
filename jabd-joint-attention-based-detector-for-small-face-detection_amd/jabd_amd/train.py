"""Training-mode (batch-statistics BatchNorm) forward/backward — see DESIGN.md."""


def train_forward(model, kind, x):
    raise NotImplementedError(
        "training-mode RetinaFace.forward on the HIP path is not built yet; call model.eval()")
