"""A6: the product `utils.anchors.Anchors` (what MultiBoxLoss, predict and the
bench consume) against the committed golden priors, the hand-derived counts
and the reference's own printed KAT (utils/anchors.py:82-105 prints 29518)."""
import os

import numpy as np
import pytest

from oracle import box_ref

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "box_ops_golden.npz"))


def _cfg():
    from utils.config import cfg_mnet
    return cfg_mnet


def test_product_anchors_match_golden_256():
    from utils.anchors import Anchors
    got = Anchors(_cfg(), image_size=(256, 256)).get_anchors()
    assert got.dtype.is_floating_point and str(got.dtype) == "torch.float32"
    np.testing.assert_array_equal(got.numpy(), G["anchors_256"])


@pytest.mark.parametrize("size,count", [(640, 16800), (840, 29126), (1024, 43008),
                                        (2048, 172032)])
def test_product_anchor_counts(size, count):
    from utils.anchors import Anchors
    a = Anchors(_cfg(), image_size=(size, size)).get_anchors()
    assert tuple(a.shape) == (count, 4)


def test_product_anchors_reference_kat_29518():
    """utils/anchors.py:82-105: four levels (steps 8/16/32/64) at 840x840."""
    from utils.anchors import Anchors
    cfg = {"min_sizes": [[8, 16], [32, 64], [64, 128], [256, 512]], "steps": [8, 16, 32, 64],
           "clip": False}
    a = Anchors(cfg, image_size=(840, 840)).get_anchors()
    assert a.shape[0] == 29518 == 2 * (105 ** 2 + 53 ** 2 + 27 ** 2 + 14 ** 2)


@pytest.mark.parametrize("size", [(640, 640), (96, 160), (1024, 1024)])
def test_product_anchors_equal_oracle(size):
    from utils.anchors import Anchors
    got = Anchors(_cfg(), image_size=size).get_anchors()
    np.testing.assert_array_equal(got.numpy(), box_ref.anchors(_cfg(), size).numpy())


def test_product_anchors_cache_returns_copies():
    from utils.anchors import Anchors
    a = Anchors(_cfg(), image_size=(128, 128)).get_anchors()
    a.zero_()
    b = Anchors(_cfg(), image_size=(128, 128)).get_anchors()
    np.testing.assert_array_equal(b.numpy(), box_ref.anchors(_cfg(), (128, 128)).numpy())
