"""The NMS pipeline's hand-written wavefront radix sort and scan (csrc/radix.hip,
jabd_sort_u64 / jabd_scan_excl_i32) against numpy: a stable sort by the key
bits [lo, lo + 8 npass) (numpy's stable argsort of the masked keys) must give
bit-identical keys and values; the exclusive scan must equal the int64
cumulative sum.  The NMS ordering these serve is torchvision's stable
descending score sort (utils/utils_bbox.py:275)."""
import ctypes

import numpy as np
import pytest
import torch


def _sort(keys, vals, lo, npass, skip_ones=False):
    from jabd_amd._lib import call, lib
    dev = torch.device("cuda")
    n = keys.size
    kin = torch.from_numpy(keys.view(np.int64)).to(dev)
    kout = torch.empty_like(kin)
    vin = torch.from_numpy(vals).to(dev) if vals is not None else None
    vout = torch.empty_like(vin) if vals is not None else None
    sz = ctypes.c_size_t()
    call("jabd_sort_workspace_size", n, int(vals is not None), ctypes.byref(sz))
    ws = torch.empty(max(sz.value, 1), dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    call("jabd_sort_u64", kin.data_ptr(), kout.data_ptr(), vin.data_ptr() if vin is not None else None,
         vout.data_ptr() if vout is not None else None, n, lo, npass, int(skip_ones), ws.data_ptr(),
         sz.value, st)
    torch.cuda.synchronize()
    assert torch.equal(kin.cpu(), torch.from_numpy(keys.view(np.int64)))   # input untouched
    ko = kout.cpu().numpy().view(np.uint64)
    return ko, (vout.cpu().numpy() if vout is not None else None)


def _ref(keys, vals, lo, npass):
    mask = np.uint64(((1 << (8 * npass)) - 1) if 8 * npass < 64 else (1 << 64) - 1)
    sel = (keys >> np.uint64(lo)) & mask
    order = np.argsort(sel, kind="stable")
    return keys[order], (vals[order] if vals is not None else None)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 4095, 4096, 4097, 8193, 16800, 32768, 32769, 70001,
                               800000])
@pytest.mark.parametrize("lo,npass,vals", [(24, 5, False), (0, 8, True), (8, 3, True)])
def test_sort_u64_vs_numpy_stable(cuda, n, lo, npass, vals):
    r = np.random.default_rng(n + lo)
    keys = r.integers(0, 2 ** 63, n, dtype=np.uint64) | (r.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
    # ties in the sorted bits (so stability shows): few distinct digit values
    keys = keys & ~np.uint64(0xFF00FF << lo) if n > 100 else keys
    keys[: n // 3] = keys[n // 3: 2 * (n // 3)] if n > 3 else keys[: n // 3]
    v = r.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32) if vals else None
    ko, vo = _sort(keys, v, lo, npass)
    kr, vr = _ref(keys, v, lo, npass)
    assert np.array_equal(ko, kr)
    if vals:
        assert np.array_equal(vo, vr)


@pytest.mark.gpu
def test_sort_nms_keys_and_skipped_passes(cuda):
    """NMS-shaped keys [image 8 | ~score 32 | row 24] over 8 images x 100k
    with 2% exact score ties and filtered rows (image 255), sorted by bits
    24-63; and grid-shaped keys whose high bits are constant (skipped passes)
    with ~0 'not binned' keys mixed in (skip_ones)."""
    r = np.random.default_rng(7)
    B, n = 8, 100000
    img = np.repeat(np.arange(B, dtype=np.uint64), n)
    img[r.random(B * n) < 0.1] = 255
    sc = r.random(B * n).astype(np.float32)
    sc[r.random(B * n) < 0.02] = np.float32(0.75)
    u = sc.view(np.uint32).astype(np.uint64)
    desc = (~(u | np.uint64(0x80000000))) & np.uint64(0xFFFFFFFF)
    row = np.tile(np.arange(n, dtype=np.uint64), B)
    keys = (img << np.uint64(56)) | (desc << np.uint64(24)) | row
    ko, _ = _sort(keys, None, 24, 5)
    kr, _ = _ref(keys, None, 24, 5)
    assert np.array_equal(ko, kr)
    # grid keys: image | classes near 512 | small cells; 5% not binned (~0)
    N = B * n
    gk = (np.repeat(np.arange(B, dtype=np.uint64), n) << np.uint64(56)) | \
        (r.integers(500, 520, N, dtype=np.uint64) << np.uint64(46)) | \
        (r.integers(505, 515, N, dtype=np.uint64) << np.uint64(36)) | \
        ((r.integers(0, 40, N, dtype=np.uint64) + np.uint64(1 << 17)) << np.uint64(18)) | \
        (r.integers(0, 40, N, dtype=np.uint64) + np.uint64(1 << 17))
    gk[r.random(N) < 0.05] = np.uint64(2 ** 64 - 1)
    gv = np.arange(N, dtype=np.int32)
    ko, vo = _sort(gk, gv, 0, 8, skip_ones=True)
    assert np.array_equal(ko, np.sort(gk, kind="stable"))
    valid = ko != np.uint64(2 ** 64 - 1)
    kr, vr = _ref(gk, gv, 0, 8)
    nv = int(valid.sum())
    assert np.array_equal(vo[:nv], vr[:nv])      # binned keys: stable, values follow
    assert np.array_equal(np.sort(vo[nv:]), np.sort(vr[nv:]))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [700, 16800, 32768])
def test_sort_small_skip_ones_and_copy(cuda, n):
    """The one-workgroup form (n <= 32768, csrc/radix.hip radix_small):
    grid-shaped keys with constant high bits (skipped passes) and ~0 keys
    (skip_ones), and keys identical in every sorted bit (no pass runs: the
    output is a copy)."""
    r = np.random.default_rng(n)
    gk = (np.uint64(3) << np.uint64(56)) | \
        (r.integers(500, 503, n, dtype=np.uint64) << np.uint64(46)) | \
        ((r.integers(0, 9, n, dtype=np.uint64) + np.uint64(1 << 17)) << np.uint64(18)) | \
        (r.integers(0, 300, n, dtype=np.uint64) + np.uint64(1 << 17))
    gk[r.random(n) < 0.05] = np.uint64(2 ** 64 - 1)
    gv = np.arange(n, dtype=np.int32)
    ko, vo = _sort(gk, gv, 0, 8, skip_ones=True)
    assert np.array_equal(ko, np.sort(gk, kind="stable"))
    kr, vr = _ref(gk, gv, 0, 8)
    nv = int((ko != np.uint64(2 ** 64 - 1)).sum())
    assert np.array_equal(vo[:nv], vr[:nv])
    same = np.full(n, 0x1234_5678_9ABC_DEF0, dtype=np.uint64)
    same[::7] ^= np.uint64(0xFF)         # differ only below the sorted bits
    ko, vo = _sort(same, gv, 8, 7)
    assert np.array_equal(ko, same) and np.array_equal(vo, gv)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 4096, 4097, 1000003])
def test_scan_excl_i32(cuda, n):
    from jabd_amd._lib import call
    r = np.random.default_rng(n)
    x = r.integers(0, 200, n, dtype=np.int32)
    dev = torch.device("cuda")
    xi = torch.from_numpy(x).to(dev)
    out = torch.empty_like(xi)
    sz = ctypes.c_size_t()
    call("jabd_scan_workspace_size", n, ctypes.byref(sz))
    ws = torch.empty(max(sz.value, 1), dtype=torch.uint8, device=dev)
    call("jabd_scan_excl_i32", xi.data_ptr(), out.data_ptr(), n, ws.data_ptr(), sz.value,
         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    ref = np.concatenate([[0], np.cumsum(x.astype(np.int64))[:-1]])
    assert np.array_equal(out.cpu().numpy().astype(np.int64), ref)
