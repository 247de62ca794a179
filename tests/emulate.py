"""TEST INFRASTRUCTURE: numpy emulation of the three HIP kernels (k_spread, k_grid, k_interp).

It drives the PRODUCT's host-side setup (Nfft4GPAmdHostPrepare / HostLayout / HostTapPoly /
HostCirculant, exported by libnfft4gp_amd.so and runnable without a GPU) and replays, in numpy, the
arithmetic each kernel performs on that layout.  Comparing it with the oracle checks the design
(polynomial taps, circulant, chunk layout, epilogue) on the CPU; the GPU tests then check that the
kernels execute it.  Also provides a CPU backend for the row-sharded (gloo) distributed tests.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import preconditioned_additive_gaussian_processes_with_fourier_acceleration_amd as amd

R = 16
NOS = 64
M = 4
NTAP = 10
NC = amd.lib().Nfft4GPAmdHostTapPoly(None)  # coefficients per tap polynomial (degree + 1)


def tap_poly():
    Cm = np.zeros(NTAP * NC)
    assert amd.lib().Nfft4GPAmdHostTapPoly(Cm.ctypes.data) == NC
    return Cm.reshape(NTAP, NC)


def circulant(kind, c, weight):
    bh = np.zeros(32)
    w = np.zeros(NOS)
    amd.lib().Nfft4GPAmdHostCirculant(kind, c, weight, bh.ctypes.data, w.ctypes.data)
    return bh, w


def prepare(col):
    col = np.ascontiguousarray(col, dtype=np.float64)
    q = np.zeros(col.size, dtype=np.uint32)
    sc = amd.lib().Nfft4GPAmdHostPrepare(col.ctypes.data, col.size, q.ctypes.data)
    return sc, q


def layout(qc, n, nw, B=4064, CG=8, rec=5):
    """The product's host layout (rec 5: the fp64 default's 5-byte records; rec 4: the 32-bit mode's one word)."""
    qc = np.ascontiguousarray(qc, dtype=np.uint32)
    cnt = (C.c_longlong * 3)()
    L = amd.lib()
    assert L.Nfft4GPAmdHostLayoutRec(qc.ctypes.data, n, nw, B, CG, rec, cnt, None, None, None, None) == 0
    ntiles, ngroups, nblocks = cnt[0], cnt[1], cnt[2]
    meta = np.zeros(ntiles * 64, np.uint16)
    lo = np.zeros(ntiles * (R // 4) * 64, np.uint32)
    q = np.zeros(ntiles * R * 64, np.uint32)
    toff = np.zeros(nblocks * ngroups + 1, np.int32)
    assert L.Nfft4GPAmdHostLayoutRec(qc.ctypes.data, n, nw, B, CG, rec, cnt, meta.ctypes.data, lo.ctypes.data,
                                     q.ctypes.data, toff.ctypes.data) == 0

    def quads(a, words):  # the 16-byte-quad layout [tile][w/4][lane][w%4] (layout.cpp) -> [tile][lane][w]
        return a.reshape(ntiles, words // 4, 64, 4).transpose(0, 2, 1, 3).reshape(ntiles, 64, words)

    # 12-bit local index split over lo (bits 4-11, a byte per point) and q (bits 0-3); q read as int32 is the
    # centred offset in the cell scaled by 2^32 (slot_word, internal.h)
    lw = quads(lo, R // 4).astype(np.int64)
    qw = quads(q, R)
    lob = np.empty((ntiles, 64, R), np.int64)
    for k in range(4):
        lob[:, :, k::4] = (lw >> (8 * k)) & 255
    loc = (lob << 4) | (qw.astype(np.int64) & 15)      # local index (B + lane % 32 for dummies)
    if rec == 4:                                       # slot_word4: the whole index in the low 12 bits
        loc = qw.astype(np.int64) & 4095
    u = qw.view(np.int32).astype(np.float64) * 2.0 ** -32   # offset in the cell - 1/2
    frac = (((qw ^ np.uint32(0x80000000)).astype(np.int64) + 32) >> 6)  # the nearest 26-bit offset, 2^-26 units
    return dict(ntiles=ntiles, ngroups=ngroups, nblocks=nblocks, meta=meta.reshape(ntiles, 64).astype(np.int64),
                loc=loc, q=frac, u=u, tile_off=toff, B=B, CG=CG)


class EmulatedPlan:
    """Host setup + numpy replay of the device plan for 1-D windows (rows [rb, re) of n_global)."""

    def __init__(self, X, windows, B=4064, CG=8, shard=None, rec=5):
        X = np.asarray(X, dtype=np.float64)
        self.n_global = X.shape[0]
        self.windows = list(windows)
        self.nw = len(self.windows)
        self.rb, self.re = shard if shard else (0, self.n_global)
        self.n = self.re - self.rb
        self.scales = []
        qc = np.zeros((self.nw, self.n), np.uint32)
        for c, feat in enumerate(self.windows):
            sc, q = prepare(X[:, feat])
            assert sc > 0
            self.scales.append(sc)
            qc[c] = q[self.rb:self.re]
        self.L = layout(qc.ravel(), self.n, self.nw, B, CG, rec)
        self.C = tap_poly()

    def setup(self, kernel, f, l, mu):
        self.f, self.mu = f, mu
        self.W = np.zeros((self.nw, NOS))
        self.Wd = np.zeros((self.nw, NOS))
        for c in range(self.nw):
            sc = self.scales[c]
            sig = l * sc * np.sqrt(2.0) if kernel == 0 else l * sc
            dscale = 2.0 * sc * np.sqrt(2.0) / sig if kernel == 0 else sc / sig
            _, self.W[c] = circulant(0 if kernel == 0 else 2, sig, 1.0 / self.nw)
            _, self.Wd[c] = circulant(1 if kernel == 0 else 3, sig, dscale / self.nw)

    # ---- k_spread: per-block partial grids -> summed grid ----
    def spread(self, x_local):
        L = self.L
        B = L["B"]
        grid = np.zeros((self.nw, NOS))
        u = L["u"]                                           # [tile][lane][r]
        comp = L["meta"] >> 6
        cell = L["meta"] & 63
        ng = L["ngroups"]
        for b in range(L["nblocks"]):
            base = b * B
            nloc = min(B, self.n - base)
            alpha = np.zeros(B + 32)  # 32 zero pad entries for the dummy slots
            alpha[:nloc] = x_local[base:base + nloc]
            t0, t1 = L["tile_off"][b * ng], L["tile_off"][(b + 1) * ng]
            a = alpha[L["loc"][t0:t1]]                       # [t][lane][r]
            pw = u[t0:t1, :, :, None] ** np.arange(NC)        # [t][lane][r][d]
            mom = np.einsum("tlr,tlrd->tld", a, pw)
            taps = mom @ self.C.T                             # [t][lane][10]
            cc = comp[t0:t1]
            ce = cell[t0:t1]
            for tp in range(NTAP):
                np.add.at(grid, (cc, (ce - M + tp) % NOS), taps[:, :, tp])
        return grid

    # ---- k_grid + k_interp ----
    def finish(self, grid, x_local, alpha=1.0, beta=0.0, y=None, grad=False):
        L = self.L
        B = L["B"]
        idx = (np.arange(NOS)[:, None] - np.arange(NOS)[None, :]) % NOS
        h = np.einsum("cls,cs->cl", self.W[:, idx], grid)
        hd = np.einsum("cls,cs->cl", self.Wd[:, idx], grid)
        cells = np.arange(NOS)
        Hm = np.zeros((self.nw, NOS, NC))
        Hdm = np.zeros((self.nw, NOS, NC))
        for tp in range(NTAP):
            Hm += h[:, (cells - M + tp) % NOS, None] * self.C[tp][None, None, :]
            Hdm += hd[:, (cells - M + tp) % NOS, None] * self.C[tp][None, None, :]
        u = L["u"]
        comp = L["meta"] >> 6
        cell = L["meta"] & 63
        acc = np.zeros(self.n)
        accd = np.zeros(self.n)
        ng = L["ngroups"]
        for b in range(L["nblocks"]):
            base = b * B
            t0, t1 = L["tile_off"][b * ng], L["tile_off"][(b + 1) * ng]
            loc = L["loc"][t0:t1]
            pw = u[t0:t1, :, :, None] ** np.arange(NC)
            coef = Hm[comp[t0:t1], cell[t0:t1]]               # [t][lane][d]
            fv = np.einsum("tlrd,tld->tlr", pw, coef)
            fdv = np.einsum("tlrd,tld->tlr", pw, Hdm[comp[t0:t1], cell[t0:t1]])
            ok = loc < B
            np.add.at(acc, base + loc[ok], fv[ok])
            np.add.at(accd, base + loc[ok], fdv[ok])
        f, mu = self.f, self.mu
        ff = f * f
        x_local = np.asarray(x_local)
        if not grad:
            v = ff * (acc + mu * x_local)
            return alpha * v if beta == 0.0 else beta * y + alpha * v
        v = np.concatenate([2.0 * f * (acc + mu * x_local), ff * accd, ff * x_local])
        return alpha * v if beta == 0.0 else beta * y + alpha * v

    def matsymv(self, x, alpha=1.0, beta=0.0, y=None, grad=False):
        return self.finish(self.spread(x), x, alpha, beta, y, grad)
