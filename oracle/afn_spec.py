"""TEST INFRASTRUCTURE ONLY (never imported by the product): a numpy restatement of the reference's MATLAB AFN
preconditioner with gradients, the only executable specification of it -- the reference's C afn.c is not
built and has no gradient.

Followed line by line, dense, for small n (natural order, predefined rank k: the first k points are the
landmarks, as Nfft4GPAmdPrecondAFNCreate(-k, ...) builds it):

  kernel blocks      MATLAB/+nfftgp/+kernels/+kernels/gaussianKernelMat.m:80-97
                     K = f^2 (exp(-D2 / 2 l^2) + mu I), dK = {K * 2 / f, f^2 D2 exp(-D2 / 2 l^2) / l^3, f^2 I}
                     (the noise only on a diagonal block; an off-diagonal block has dK_mu = 0)
  L11, dL11          +preconds/chol_setup.m:36-63, 116: L = chol(K11), dL_g = L PHI(L^{-1} dK11_g L^{-T}),
                     PHI(A) = tril(A, -1) + diag(diag(A) / 2)
  GK12, GdK12, ...   +kernels/schurCombinedKernel.m:87-104: GK12 = L \\ K12, GdK12_g = L \\ dK12_g,
                     GdK11GK12_g = (L^{-1} dK11_g L^{-T}) GK12
  Schur kernel       +kernels/schurCombinedKernelMat.m:45, 59-66: S = K22 - GK12' GK12,
                     dS_g = dK22_g - GK12' GdK12_g - (GK12' GdK12_g)' + GK12' GdK11GK12_g
  FSAI of S          +preconds/fsai_setup.m (require_grad branch): row i over its pattern P_i (neighbours,
                     then i): iKe = A_i \\ e / sqrt(e' (A_i \\ e)); dG_g = -A_i \\ (dA_i iKe) - (e' idKe) / 2 / dd * iKe
  dvp / trace / logdet   +preconds/afn_dvp.m:24-85, afn_trace.m:24-45, afn_logdet.m:23-25
  M = U' U with U = [L', L^{-1} K12; 0, G^{-T}] (afn_dvp.m:41-43), so M^{-1} = G'G on the Schur block as
  fsai_solve.m:34-37 applies it.

afn_dvp.m returns (dM/dtheta_g) x; the reference's C interface (nys.c, fsai.c, and this library's AFN) returns
M^{-1} (dM/dtheta_g) x -- the test applies M^{-1} to the restatement's result.
"""
from __future__ import annotations

import numpy as np


def _sqdist(A, B):
    return np.maximum(np.sum(A * A, 1)[:, None] + np.sum(B * B, 1)[None, :] - 2.0 * A @ B.T, 0.0)


def gaussian_block(X, f, l, mu, rows, cols, diagonal):
    """K and [dK/df, dK/dl, dK/dmu] of the Gaussian kernel block X[rows] x X[cols] (gaussianKernelMat.m:80-97)."""
    D2 = np.array([[np.sum((X[i] - X[j]) ** 2) for j in cols] for i in rows])  # exact differences
    E = np.exp(-D2 / (2.0 * l * l))
    K = f * f * E
    dKmu = np.zeros_like(K)
    if diagonal:
        K = K + f * f * mu * np.eye(len(rows))
        dKmu = f * f * np.eye(len(rows))
    return K, [K * 2.0 / f, f * f * D2 * E / l ** 3, dKmu]


def phi(A):
    """chol_setup.m:116."""
    return np.tril(A, -1) + np.diag(np.diag(A) / 2.0)


def afn_setup(X, k, f, l, mu, pattern):
    """The AFN with gradients of the first k points (afn_setup.m with a given order, k = maxrank).  pattern[i]:
    the column indices (Schur-point numbering, all < i) of row i of the Schur FSAI without the diagonal."""
    n = X.shape[0]
    r1, r2 = np.arange(k), np.arange(k, n)
    K11, dK11 = gaussian_block(X, f, l, mu, r1, r1, True)
    K12, dK12 = gaussian_block(X, f, l, mu, r1, r2, False)
    K22, dK22 = gaussian_block(X, f, l, mu, r2, r2, True)
    L = np.linalg.cholesky(K11)
    Gi = np.linalg.inv(L)
    GdKG = [Gi @ d @ Gi.T for d in dK11]
    dL = [L @ phi(g) for g in GdKG]
    GK12 = Gi @ K12
    GdK12 = [Gi @ d for d in dK12]
    GdK11GK12 = [g @ GK12 for g in GdKG]
    S = K22 - GK12.T @ GK12
    dS = []
    for g in range(3):
        t = GK12.T @ GdK12[g]
        dS.append(dK22[g] - t - t.T + GK12.T @ GdK11GK12[g])
    n2 = n - k
    G = np.zeros((n2, n2))
    dG = [np.zeros((n2, n2)) for _ in range(3)]
    for i in range(n2):
        Pi = np.concatenate([np.sort(np.asarray(pattern[i], dtype=np.int64)), [i]])
        A = S[np.ix_(Pi, Pi)]
        e = np.zeros(len(Pi))
        e[-1] = 1.0
        iKe = np.linalg.solve(A, e)
        dd = np.sqrt(e @ iKe)
        iKe = iKe / dd
        G[i, Pi] = iKe
        for g in range(3):
            idKe = -np.linalg.solve(A, dS[g][np.ix_(Pi, Pi)] @ iKe)
            dG[g][i, Pi] = idKe - (e @ idKe) / 2.0 / dd * iKe
    return {"L": L, "dL": dL, "K12": K12, "dK12": dK12, "G": G, "dG": dG, "k": k, "n": n}


def afn_solve(P, x):
    """M^{-1} x with M = U'U, U = [L', L^{-1} K12; 0, G^{-T}] (afn_solve.m; fsai_solve.m:34-37 on the Schur block)."""
    k, n = P["k"], P["n"]
    L, K12, G = P["L"], P["K12"], P["G"]
    U = np.zeros((n, n))
    U[:k, :k] = L.T
    U[:k, k:] = np.linalg.solve(L, K12)
    U[k:, k:] = np.linalg.inv(G).T
    return np.linalg.solve(U, np.linalg.solve(U.T, x))


def afn_dvp(P, x):
    """[dM/dtheta_g x for g = f, l, mu] (afn_dvp.m:24-85), natural order."""
    k = P["k"]
    L, dL, K12, dK12, G, dG = P["L"], P["dL"], P["K12"], P["dK12"], P["G"], P["dG"]
    xu, xl = x[:k], x[k:]
    Lt = L.T
    z1u = Lt @ xu + np.linalg.solve(L, K12 @ xl)
    z1l = np.linalg.solve(G.T, xl)
    out = []
    for i in range(3):
        y1u = dL[i] @ z1u
        y1l_i = np.linalg.solve(Lt, z1u)
        y1l = dK12[i].T @ y1l_i - K12.T @ np.linalg.solve(Lt, dL[i].T @ y1l_i) - \
            np.linalg.solve(G, dG[i] @ np.linalg.solve(G, z1l))
        z2l = -np.linalg.solve(G.T, dG[i].T @ np.linalg.solve(G.T, xl))
        y2u_i = dK12[i] @ xl - dL[i] @ np.linalg.solve(L, K12 @ xl)
        z2u = dL[i].T @ xu + np.linalg.solve(L, y2u_i)
        y2u = L @ z2u
        y2l = K12.T @ np.linalg.solve(Lt, z2u) + np.linalg.solve(G, z2l)
        out.append(np.concatenate([y1u + y2u, y1l + y2l]))
    return out


def afn_trace(P):
    """tr(M^{-1} dM/dtheta_g) (afn_trace.m:24-45)."""
    diagU = np.concatenate([np.diag(P["L"]), 1.0 / np.diag(P["G"])])
    val = []
    for i in range(3):
        diagdU = np.concatenate([np.diag(P["dL"][i]), -1.0 / np.diag(P["G"]) ** 2 * np.diag(P["dG"][i])])
        val.append(2.0 * np.sum(diagdU / diagU))
    return np.array(val)


def afn_logdet(P):
    """log det M (afn_logdet.m:23-25)."""
    return 2.0 * (np.sum(np.log(np.diag(P["L"]))) + np.sum(np.log(1.0 / np.diag(P["G"]))))


def knn_pattern(Xs, lfil):
    """fsai_setup.m knnpattern: rows i <= lfil dense (all earlier points), row i > lfil its lfil nearest earlier
    points (ties by index, as this library ranks them)."""
    n = Xs.shape[0]
    pat = []
    for i in range(n):
        if i <= lfil:
            pat.append(list(range(i)))
            continue
        d2 = np.sum((Xs[:i] - Xs[i]) ** 2, 1)
        order = np.lexsort((np.arange(i), d2))
        pat.append(sorted(order[:lfil].tolist()))
    return pat
