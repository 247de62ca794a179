"""The layout built on the GPU (layout_gpu.hip: what every additive handle's setup now uses) is the host
builder's (layout.cpp) array for array, bit for bit: tile offsets, meta words, the local-index bytes and the
coordinate words, for ragged last blocks, a partial last window group, small blocks, clustered points (long
runs in one cell), duplicated coordinates and an empty input."""
import ctypes as C

import numpy as np
import pytest

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

pytestmark = pytest.mark.gpu


def build(fn, qc, n, nw, B, CG, rec=5):
    L = amd.lib()
    cnt = (C.c_longlong * 3)()
    assert getattr(L, fn)(qc.ctypes.data, n, nw, B, CG, rec, cnt, None, None, None, None) == 0
    ntiles, ngroups, nblocks = cnt[0], cnt[1], cnt[2]
    meta = np.zeros(max(ntiles, 1) * 64, np.uint16)
    lo = np.zeros(max(ntiles, 1) * 4 * 64, np.uint32)
    q = np.zeros(max(ntiles, 1) * 16 * 64, np.uint32)
    toff = np.zeros(nblocks * ngroups + 1, np.int32)
    assert getattr(L, fn)(qc.ctypes.data, n, nw, B, CG, rec, cnt, meta.ctypes.data, lo.ctypes.data, q.ctypes.data,
                          toff.ctypes.data) == 0
    return ntiles, toff, meta[:ntiles * 64], lo[:ntiles * 256] if rec == 5 else lo[:0], q[:ntiles * 1024]


def quantised(X):
    L = amd.lib()
    n, nw = X.shape
    qc = np.zeros((nw, n), np.uint32)
    for c in range(nw):
        col = np.ascontiguousarray(X[:, c])
        assert L.Nfft4GPAmdHostPrepare(col.ctypes.data, n, qc[c].ctypes.data) > 0
    return np.ascontiguousarray(qc)


@pytest.mark.parametrize("n,nw,B,CG,kind,rec", [(20000, 7, 4064, 3, "uniform", 5), (9000, 4, 512, 3, "clustered", 5),
                                                (5000, 3, 4064, 3, "duplicates", 5), (4064 * 3, 6, 4064, 3, "uniform", 5),
                                                (777, 2, 100, 1, "uniform", 5), (4064 * 10 + 17, 8, 4064, 4, "uniform", 5),
                                                (9000, 5, 512, 4, "clustered", 5), (4064 * 10 + 17, 8, 4064, 4, "uniform", 4),
                                                (9000, 5, 512, 3, "duplicates", 4)])
def test_device_layout_equals_host(torch_cuda, n, nw, B, CG, kind, rec):
    rng = np.random.default_rng(n + nw)
    if kind == "uniform":
        X = rng.random((n, nw))
    elif kind == "clustered":
        X = np.where(rng.random((n, nw)) < 0.7, 0.5 + 0.001 * rng.random((n, nw)), rng.random((n, nw)))
    else:
        X = rng.integers(0, 9, (n, nw)) / 8.0
    qc = quantised(X)
    h = build("Nfft4GPAmdHostLayoutRec", qc, n, nw, B, CG, rec)
    d = build("Nfft4GPAmdDeviceLayoutRec", qc, n, nw, B, CG, rec)
    assert h[0] == d[0]
    for a, b, name in zip(h[1:], d[1:], ("tile_off", "meta", "lo", "q")):
        np.testing.assert_array_equal(a, b, err_msg=name)
