"""Numerical check of the adjoint (vector-Jacobian) form of the world-frame
RNEA derivatives used by the backward kernel: w^T dtau/dq and w^T dtau/dqdot
at fixed qddot from subtree sums of seven per-body 6-vectors, against
central finite differences.  Revolute joints on a branching tree."""
import numpy as np

rng = np.random.default_rng(0)


def skew(a):
    return np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])


def crm(v):  # motion cross product [v x]
    w, u = v[:3], v[3:]
    M = np.zeros((6, 6))
    M[:3, :3] = skew(w); M[3:, :3] = skew(u); M[3:, 3:] = skew(w)
    return M


def crf(v):  # force cross product [v x*] = -crm(v)^T
    return -crm(v).T


def rot(axis, th):
    a = axis / np.linalg.norm(axis)
    K = skew(a)
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


nb = 7
parent = [-1, 0, 1, 1, 3, 0, 5]
axes = [rng.standard_normal(3) for _ in range(nb)]
offs = [rng.standard_normal(3) * 0.3 for _ in range(nb)]
mass = rng.uniform(0.5, 2.0, nb)
coms = [rng.standard_normal(3) * 0.1 for _ in range(nb)]
Ib = []
for i in range(nb):
    A = rng.standard_normal((3, 3)); Ib.append(A @ A.T * 0.1 + np.eye(3) * 0.05)
g = np.array([0, 0, -9.81])


def kin(q):
    """world rotation/translation of each body frame; joint i rotates about its
    (body-frame) axis at the body origin, placed at offs[i] in the parent."""
    R, p = [None] * nb, [None] * nb
    for i in range(nb):
        Rl, pl = (np.eye(3), np.zeros(3)) if parent[i] < 0 else (R[parent[i]], p[parent[i]])
        p[i] = pl + Rl @ offs[i]
        R[i] = Rl @ rot(axes[i], q[i])
    return R, p


def spatial(q):
    R, p = kin(q)
    S, I = [], []
    for i in range(nb):
        w = R[i] @ (axes[i] / np.linalg.norm(axes[i]))
        S.append(np.concatenate([w, np.cross(p[i], w)]))
        c = p[i] + R[i] @ coms[i]
        Ic = R[i] @ Ib[i] @ R[i].T
        C = skew(c)
        M = np.zeros((6, 6))
        M[:3, :3] = Ic + mass[i] * C @ C.T
        M[:3, 3:] = mass[i] * C
        M[3:, :3] = mass[i] * C.T
        M[3:, 3:] = mass[i] * np.eye(3)
        I.append(M)
    return S, I


ag = np.concatenate([np.zeros(3), g])


def rnea(q, qd, qdd):
    S, I = spatial(q)
    V, A, f = [None] * nb, [None] * nb, [None] * nb
    for i in range(nb):
        Vl = np.zeros(6) if parent[i] < 0 else V[parent[i]]
        Al = np.zeros(6) if parent[i] < 0 else A[parent[i]]
        V[i] = Vl + S[i] * qd[i]
        A[i] = Al + S[i] * qdd[i] + crm(V[i]) @ S[i] * qd[i]
        f[i] = I[i] @ (A[i] - ag) + crf(V[i]) @ I[i] @ V[i]
    F = [x.copy() for x in f]
    for i in reversed(range(nb)):
        if parent[i] >= 0:
            F[parent[i]] += F[i]
    tau = np.array([S[i] @ F[i] for i in range(nb)])
    return tau, S, I, V, A, F


def adjoint(q, qd, qdd, w):
    tau, S, I, V, A, F = rnea(q, qd, qdd)
    W = [None] * nb
    for i in range(nb):
        Wl = np.zeros(6) if parent[i] < 0 else W[parent[i]]
        W[i] = Wl + S[i] * w[i]
    vec = np.zeros((nb, 7, 6))
    for c in range(nb):
        Wl = np.zeros(6) if parent[c] < 0 else W[parent[c]]
        u = A[c] - ag
        p_ = I[c] @ u
        h = I[c] @ V[c]
        beta = I[c] @ W[c]
        alpha = crf(W[c]) @ p_
        gamma = -crf(V[c]) @ beta
        eps = crf(W[c]) @ h
        delta = crf(crm(V[c]) @ W[c]) @ h - crf(V[c]) @ eps
        zeta = -I[c] @ (crm(V[c]) @ W[c])
        kappa = crf(W[c] - Wl) @ F[c]
        vec[c] = [alpha, beta, gamma, delta, eps, zeta, kappa]
    for c in reversed(range(nb)):
        if parent[c] >= 0:
            vec[parent[c]] += vec[c]
    gq, gv = np.zeros(nb), np.zeros(nb)
    for k in range(nb):
        b, l = k, parent[k]
        Vl = np.zeros(6) if l < 0 else V[l]
        ul = (np.zeros(6) if l < 0 else A[l]) - ag
        Al_, B_, G_, D_, E_, Zt_, K_ = vec[b]
        Z = S[k]
        gq[k] = Z @ (-Al_ - crf(ul) @ B_ + crf(Vl) @ G_ + crf(Vl) @ (crf(Vl) @ B_) + D_ + crf(Vl) @ E_
                     - crf(Vl) @ Zt_ + K_)
        gv[k] = S[k] @ (-crf(Vl + V[b]) @ B_ - G_ - E_ + Zt_)
    return gq, gv


q, qd, qdd, w = (rng.standard_normal(nb) for _ in range(4))
gq, gv = adjoint(q, qd, qdd, w)
eps = 1e-6
fq = np.array([(w @ rnea(q + eps * e, qd, qdd)[0] - w @ rnea(q - eps * e, qd, qdd)[0]) / (2 * eps) for e in np.eye(nb)])
fv = np.array([(w @ rnea(q, qd + eps * e, qdd)[0] - w @ rnea(q, qd - eps * e, qdd)[0]) / (2 * eps) for e in np.eye(nb)])
print("gq adjoint", np.round(gq, 6))
print("gq fd     ", np.round(fq, 6))
print("gv adjoint", np.round(gv, 6))
print("gv fd     ", np.round(fv, 6))
print("max err q", np.abs(gq - fq).max(), "v", np.abs(gv - fv).max())
