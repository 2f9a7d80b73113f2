# listed-row fractions under Hamerly bounds: cumulative max drift (current) vs
# displacement since the row's last exact refresh (stamped)
import numpy as np
from sklearn.cluster import kmeans_plusplus
rng = np.random.default_rng(0)
n, F, k = 200000, 50, 8
means = rng.normal(0, 1.0, (40, F)) * 0.35
comp = rng.integers(0, 12, n)
X = (means[comp] + rng.normal(0, 1, (n, F))).astype(np.float64)
C, _ = kmeans_plusplus(X, k, random_state=18)
def dists(X, C):
    return np.sqrt(np.maximum(((X[:, None, :] - C[None]) ** 2).sum(-1), 0))
D = dists(X, C); lab = D.argmin(1); srt = np.sort(D, 1)
ub = srt[:, 0].copy(); lb = srt[:, 1].copy()
ub2, lb2 = ub.copy(), lb.copy(); stamp = np.zeros(n, int)
hist = [C.copy()]
for it in range(1, 300):
    newC = np.stack([X[lab == j].mean(0) if (lab == j).any() else C[j] for j in range(k)])
    drift = np.linalg.norm(newC - C, axis=1); C = newC; hist.append(C.copy())
    cc = dists(C, C); np.fill_diagonal(cc, np.inf); half = cc.min(1) / 2
    # scheme A (current): per-iteration drift update of every row
    ubA = ub + drift[lab]; lbA = lb - drift.max()
    needA = ~(ubA < np.maximum(lbA, half[lab]))
    # scheme B: displacement since the stamp
    disp = np.stack([np.linalg.norm(C - hist[t], axis=1) for t in range(it + 1)])  # [t0, j]
    dB = disp[stamp]  # [n, k]
    ubB = ub2 + dB[np.arange(n), lab]
    dB2 = dB.copy(); dB2[np.arange(n), lab] = -1
    lbB = lb2 - dB2.max(1)
    needB = ~(ubB < np.maximum(lbB, half[lab]))
    D = dists(X, C); newlab = D.argmin(1); srt = np.sort(D, 1)
    # A: listed rows get exact bounds (tighten/recompute: exact ub, and lb if recomputed;
    # simplify: exact both), others keep drifted
    ub = np.where(needA, srt[:, 0], ubA); lb = np.where(needA, srt[:, 1], lbA)
    ub2 = np.where(needB, srt[:, 0], ub2); lb2 = np.where(needB, srt[:, 1], lb2); stamp = np.where(needB, it, stamp)
    ch = (newlab != lab).sum(); lab = newlab
    if it % 10 == 0 or ch == 0:
        print(it, "changed", ch, "listed A %.4f B %.4f" % (needA.mean(), needB.mean()))
    if ch == 0: break
