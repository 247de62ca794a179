"""TEST INFRASTRUCTURE ONLY (never imported by the product): a numpy restatement of the reference's MATLAB
RAN (randomized Nystrom) preconditioner with gradients -- the branch afn_setup.m builds when the estimated
rank is below max_k or the AFN's factors break down (afn_setup.m:80-83, 93-98).  The reference's C afn.c
calls AfnPrecondNysSetupWithKernelandPerm2 there, which is not in its sources; this MATLAB code is the
executable specification of that branch.  Followed line by line, dense, small n:

  ran_setup.m   K1 = K(perm(1:k), perm) with mu = 0, K11 = K1(:, 1:k), dK_mu = 0;
                nu = sqrt(n) eps(||K1||_2); M = K1' / chol(K11 + nu I); [U, S] = svds(M, k);
                S = max(S.^2 - nu, 0); eta = f^2 mu; M = (S + eta).^-1
  ran_solve.m   y(perm) = U (M .* (U' b(perm))) + (b(perm) - U U' b(perm)) / eta
  ran_logdet.m  sum(log(S + eta)) + (n - k) log(eta)
  ran_dvp.m     dM/dtheta_g x for the noise-free Nystrom K1' K11^{-1} K1 (g = f, l), f^2 x (g = mu)
  ran_trace.m   tr(M^{-1} dM/dtheta_g) through ran_dvp on the columns of L = K1' / chol(K11 + k eps I)
with the additive kernel of additiveKernelMat.m (the average of the windows' Gaussian kernels,
gaussianKernelMat.m:80-97: K = f^2 exp(-D2 / 2 l^2), dK = {2 K / f, f^2 D2 exp(-D2 / 2 l^2) / l^3}).
"""
from __future__ import annotations

import numpy as np


def additive_noise_free(X, windows, f, l, rows, cols):
    """K and [dK/df, dK/dl, dK/dmu = 0] of the additive Gaussian kernel block (additiveKernelMat.m)."""
    K = np.zeros((len(rows), len(cols)))
    dKl = np.zeros_like(K)
    for w in windows:
        D2 = np.zeros_like(K)
        for c in w:
            D2 += (X[rows, c][:, None] - X[cols, c][None, :]) ** 2
        E = np.exp(-D2 / (2.0 * l * l))
        K += f * f * E
        dKl += f * f * D2 * E / l ** 3
    K /= len(windows)
    dKl /= len(windows)
    return K, [2.0 * K / f, dKl, np.zeros_like(K)]


def ran_setup(X, windows, f, l, mu, perm, k):
    n = X.shape[0]
    perm = np.asarray(perm)
    k = min(n, k)
    K1, dK1 = additive_noise_free(X, windows, f, l, perm[:k], perm)
    K11 = K1[:, :k]
    dK11 = [d[:, :k] for d in dK1]
    nu = np.sqrt(n) * np.spacing(np.linalg.norm(K1, 2))
    R = np.linalg.cholesky(K11 + nu * np.eye(k)).T  # chol(.) is upper in MATLAB
    M = np.linalg.solve(R.T, K1).T                   # K1' / R
    U, sig, _ = np.linalg.svd(M, full_matrices=False)
    S = np.maximum(sig ** 2 - nu, 0.0)
    f2 = f * f
    eta = f2 * mu
    return {"K1": K1, "K11": K11, "dK1": dK1, "dK11": dK11, "U": U, "S": S, "M": 1.0 / (S + eta), "perm": perm,
            "eta": eta, "f2": f2, "n": n, "k": k}


def ran_solve(P, x):
    perm = P["perm"]
    b = x[perm]
    U = P["U"]
    Ub = U.T @ b
    py = U @ (P["M"] * Ub) + (b - U @ Ub) / P["eta"]
    y = np.zeros_like(x)
    y[perm] = py
    return y


def ran_logdet(P):
    n, k = P["n"], P["k"]
    return float(np.sum(np.log(P["S"] + P["eta"])) + (n - k) * np.log(P["eta"]))


def ran_dvp(P, x, nonperm=False):
    perm = P["perm"]
    px = x if nonperm else x[perm]
    K1, K11 = P["K1"], P["K11"]
    K11K1x = np.linalg.solve(K11, K1 @ px)
    out = []
    for i in range(2):
        pyi = P["dK1"][i].T @ K11K1x
        pyi = pyi - K1.T @ np.linalg.solve(K11, P["dK11"][i] @ K11K1x)
        pyi = pyi + K1.T @ np.linalg.solve(K11, P["dK1"][i] @ px)
        if nonperm:
            yi = pyi
        else:
            yi = np.zeros_like(x)
            yi[perm] = pyi
        out.append(yi)
    out.append(P["f2"] * x)
    return out


def ran_trace(P):
    n, k = P["n"], P["k"]
    K11 = P["K11"]
    L11 = np.linalg.cholesky(K11 + k * np.spacing(np.linalg.norm(K11, 2)) * np.eye(k)).T  # upper
    L = np.linalg.solve(L11.T, P["K1"]).T  # K1' / L11
    val = np.zeros(3)
    for i in range(2):
        dL = np.linalg.solve(L11.T, P["dK1"][i]).T
        dKL = L @ np.linalg.solve(L11.T, np.linalg.solve(L11.T, P["dK11"][i].T).T)
        val[i] = 2.0 * np.sum(dL * L) - np.sum(dKL * L)
    val[2] = n * P["f2"]
    LP = np.linalg.solve((P["eta"] * np.eye(k) + L.T @ L).T, L.T).T  # L / (eta I + L'L)
    dLP = [np.zeros((n, k)) for _ in range(3)]
    for j in range(k):
        d = ran_dvp(P, L[:, j], nonperm=True)
        for i in range(3):
            dLP[i][:, j] = d[i]
    for i in range(3):
        val[i] = (val[i] - np.sum(dLP[i] * LP)) / P["eta"]
    return val
