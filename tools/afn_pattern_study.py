"""Why the AFN (BASELINE configs[1-2]'s preconditioner) loses to no preconditioner on the additive kernel at
l = 0.1: a dense CPU study at small n that isolates the two suspected causes.

A = K + mu I, K the additive Gaussian kernel of nw 1-D windows (weights 1/nw), X ~ U[0,1)^d, f = 1.
AFN (afn.c:161-489 structure): landmarks X1 (k random points), A11 = K11 + mu I (the reference's Cholesky
includes the noise), Schur complement S = A22 - A21 A11^-1 A12, and M^-1 = the exact block-LDL^T inverse with
S^-1 replaced by (a) I / mu, (b) an FSAI of S on the reference's pattern -- each row's lfil nearest earlier
points in ALL d features (fsai.c / kernels.c KNN), (c) an FSAI of S with the same number of entries per row but
the pattern chosen from S's largest earlier entries (what an additive kernel couples: points close in ANY one
feature), (d) exact S^-1 (the block structure alone: 1-2 iterations).  PCG iterations to 1e-6 for each,
against no preconditioner and the rank-k Nystrom.

    python tools/afn_pattern_study.py [--n 3000 --d 32 --k 100 --lfil 20 --l 0.1]
"""
import argparse
import json

import numpy as np


def additive_kernel(X, Y, l):
    d = X.shape[1]
    K = np.zeros((X.shape[0], Y.shape[0]))
    for c in range(d):
        diff = X[:, c:c + 1] - Y[:, c][None, :]
        K += np.exp(-diff * diff / (2.0 * l * l))
    return K / d


def pcg(A, b, apply_m, tol=1e-6, maxits=5000):
    x = np.zeros_like(b)
    r = b.copy()
    z = apply_m(r)
    p = z.copy()
    rz = r @ z
    nb = np.linalg.norm(b)
    for it in range(1, maxits + 1):
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        if np.linalg.norm(r) <= tol * nb:
            return it
        z = apply_m(r)
        rz_new = r @ z
        p = z + (rz_new / rz) * p
        rz = rz_new
    return maxits


def fsai(S, pattern):
    """Lower-triangular FSAI G with G S G^T ~ I: row i solves S[P,P] g = e_last on P = pattern[i] + [i]
    (fsai.c's construction), scaled so that (G S G^T)_ii = 1."""
    n = S.shape[0]
    G = np.zeros((n, n))
    for i in range(n):
        P = list(pattern[i]) + [i]
        Sp = S[np.ix_(P, P)]
        e = np.zeros(len(P))
        e[-1] = 1.0
        g = np.linalg.solve(Sp, e)
        g /= np.sqrt(g[-1])
        G[i, P] = g
    return G


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--lfil", type=int, default=20)
    ap.add_argument("--l", type=float, default=0.1)
    ap.add_argument("--mu", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=906)
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    n, d, k, lfil, l, mu = args.n, args.d, args.k, args.lfil, args.l, args.mu
    X = rng.random((n, d))
    b = rng.random(n) - 0.5
    A = additive_kernel(X, X, l) + mu * np.eye(n)
    perm = rng.permutation(n)
    Xp = X[perm]
    Ap = A[np.ix_(perm, perm)]
    bp = b[perm]
    A11, A12, A22 = Ap[:k, :k], Ap[:k, k:], Ap[k:, k:]
    L11 = np.linalg.cholesky(A11)
    W = np.linalg.solve(L11, A12)            # L11^-1 A12
    S = A22 - W.T @ W
    m = n - k
    X2 = Xp[k:]
    # (b) the reference's pattern: the lfil nearest EARLIER points in all d features
    D2 = ((X2[:, None, :] - X2[None, :, :]) ** 2).sum(-1)
    knn = [np.argsort(D2[i, :i])[:lfil] if i > 0 else np.array([], int) for i in range(m)]
    # (c) the same entries per row chosen from |S| (largest earlier entries)
    big = [np.argsort(-np.abs(S[i, :i]))[:lfil] if i > 0 else np.array([], int) for i in range(m)]
    # overlap of the two patterns, and the share of |S|'s off-diagonal mass each captures
    ov = np.mean([len(set(knn[i]) & set(big[i])) / max(1, len(big[i])) for i in range(1, m)])
    off = np.abs(np.tril(S, -1))
    mass = off.sum()
    mk = sum(off[i, knn[i]].sum() for i in range(1, m)) / mass
    mb = sum(off[i, big[i]].sum() for i in range(1, m)) / mass
    G_knn, G_big = fsai(S, knn), fsai(S, big)

    def afn(apply_sinv):
        def f(r):
            rp = r[perm]
            r1, r2 = rp[:k], rp[k:]
            y1 = np.linalg.solve(L11, r1)                 # L11^-1 r1
            s = r2 - W.T @ y1                             # r2 - A21 A11^-1 r1
            z2 = apply_sinv(s)
            z1 = np.linalg.solve(L11.T, y1 - W @ z2)      # A11^-1 (r1 - A12 z2)
            out = np.empty(n)
            out[perm] = np.concatenate([z1, z2])
            return out
        return f

    Sinv = np.linalg.inv(S)
    res = {"n": n, "d": d, "k": k, "lfil": lfil, "l": l, "mu": mu,
           "pattern_overlap_knn_vs_largest": ov, "offdiag_mass_captured_knn": mk, "offdiag_mass_captured_largest": mb}
    res["pcg_none"] = pcg(A, b, lambda r: r)
    # rank-k Nystrom with the same landmarks: K1 K11^-1 K1^T + mu I, applied exactly (Woodbury)
    K1 = additive_kernel(X, Xp[:k], l)
    K11 = additive_kernel(Xp[:k], Xp[:k], l) + 1e-10 * np.eye(k)
    C = np.linalg.cholesky(K11)
    U = np.linalg.solve(C, K1.T).T                        # K1 C^-T: Nystrom = U U^T
    Sm = mu * np.eye(k) + U.T @ U
    res["pcg_nystrom"] = pcg(A, b, lambda r: (r - U @ np.linalg.solve(Sm, U.T @ r)) / mu)
    res["pcg_afn_schur_noise"] = pcg(A, b, afn(lambda s: s / mu))
    res["pcg_afn_fsai_knn_all_features"] = pcg(A, b, afn(lambda s: G_knn.T @ (G_knn @ s)))
    res["pcg_afn_fsai_largest_entries"] = pcg(A, b, afn(lambda s: G_big.T @ (G_big @ s)))
    res["pcg_afn_exact_schur"] = pcg(A, b, afn(lambda s: Sinv @ s))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
