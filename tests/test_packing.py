"""Weight packing into the MFMA fragment order (conv.hip header) — CPU."""
import pytest
import torch

from jabd_amd import functional as F


def _unpack(pk):
    # Wp[kc][nt][lane=16g+j][e] holds W[16kc+4g+e][16nt+j]
    Kc, Nt = pk.Kc, pk.Ntiles
    w = pk.w.view(Kc, Nt, 4, 16, 4).permute(0, 2, 4, 1, 3).reshape(Kc * 16, Nt * 16)
    return w


def test_pack_roundtrip_and_bn_fold():
    conv = torch.nn.Conv2d(24, 40, 3, padding=1, bias=False)
    bn = torch.nn.BatchNorm2d(40).eval()
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-1, 1)
    pk = F.pack_conv(conv, bn)
    assert pk.Kc == (9 * 24 + 15) // 16 and pk.Ntiles % pk.tn == 0
    w = _unpack(pk)
    s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    ref = conv.weight.permute(2, 3, 1, 0).reshape(9 * 24, 40) * s
    assert torch.allclose(w[: 9 * 24, :40], ref)
    assert torch.count_nonzero(w[9 * 24:]) == 0 and torch.count_nonzero(w[:, 40:]) == 0
    # the folded conv equals conv -> bn on an input
    x = torch.randn(2, 24, 5, 7)
    y_ref = bn(conv(x))
    cols = torch.nn.functional.unfold(x, 3, padding=1)  # [B, Cin*9, L] (ci-major)
    cols = cols.view(2, 24, 9, -1).permute(0, 2, 1, 3).reshape(2, 9 * 24, -1)  # tap-major
    y = torch.einsum("bkl,kn->bnl", cols, w[: 9 * 24, :40]) + pk.bias[None, :, None]
    assert torch.allclose(y.view(2, 40, 5, 7), y_ref, atol=1e-5)


def test_pack_tn_choices():
    from jabd_amd._lib import lib
    assert [lib().jabd_conv_pack_tn(c) for c in (16, 24, 40, 80)] == [1, 2, 3, 5]
    for c in (112, 160, 480, 672, 960, 2048):
        tn = lib().jabd_conv_pack_tn(c)
        assert tn in (4, 5, 8)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,transposed", [((64, 16, 1, 1), False), ((64, 16, 1, 1), True),
                                               ((40, 40, 3, 3), False), ((40, 40, 3, 3), True),
                                               ((12, 10, 3, 3), True), ((160, 960, 1, 1), False),
                                               ((256, 64, 3, 3), True), ((16, 3, 3, 3), False),
                                               ((10, 12, 3, 3), False)])
def test_device_pack_matches_host_pack(cuda, shape, transposed):
    """jabd_conv_pack_f32 (the training convs' per-step repack) writes exactly
    the host PackedConv layouts, both the 16x16x4 and the 32x32x2 one."""
    w = torch.randn(shape, generator=torch.Generator().manual_seed(sum(shape))).to(cuda)
    wt = w.transpose(0, 1) if transposed else w
    ref = F.PackedConv(F.conv_weight_2d(wt).contiguous(), None, shape[2], shape[3], wt.shape[1])
    got = F.pack_weight_device(w, transposed)
    for a in ("KH", "KW", "Cin", "Cout", "tn", "Ntiles", "Kc"):
        assert getattr(got, a) == getattr(ref, a), a
    assert torch.equal(got.w, ref.w)
    assert (got.w32 is None) == (ref.w32 is None)
    if ref.w32 is not None:
        assert got.ntiles32 == ref.ntiles32 and got.tn32 == ref.tn32
        assert torch.equal(got.w32, ref.w32)
