"""Test infrastructure (never imported by the product path): a loop restatement of
src/vbhem/my_weighted_kmeans.m, one point and one cluster at a time in the
reference's order, as the checker of h3m.weighted_kmeans.  Points are rows here
(columns in the reference); clusters are 0-based."""
import math


def _centroids(point, cluster, weight, K):
    """my_weighted_kmeans.m gcentroids (:72-88)."""
    dim = len(point[0])
    cen = [[0.0] * dim for _ in range(K)]
    cw = [0.0] * K
    for j in range(K):
        for n, p in enumerate(point):
            if cluster[n] == j:
                cw[j] += weight[n]
                for a in range(dim):
                    cen[j][a] += p[a] * weight[n]
        if cw[j] > 0:
            cen[j] = [c / cw[j] for c in cen[j]]
    return cen, cw


def _div(x, y):
    """MATLAB division: x/0 = +-Inf, 0/0 = NaN."""
    if y == 0:
        return math.nan if x == 0 else math.copysign(math.inf, x)
    return x / y


def _energy(point, weight, cen, cw, cluster):
    """my_weighted_kmeans.m genergy (:94-108)."""
    f = [0.0] * len(point)
    energy = [0.0] * len(cen)
    for j in range(len(cen)):
        for n, p in enumerate(point):
            if cluster[n] == j:
                f[n] = sum((p[a] - cen[j][a]) ** 2 for a in range(len(p)))
                energy[j] += weight[n] * f[n]
        for n in range(len(point)):
            if cluster[n] == j:
                f[n] = _div(f[n] * cw[j], cw[j] - weight[n])
    return f, energy


def _argmin(col):
    """MATLAB min: NaN skipped, first of equal minima, all NaN -> first."""
    best, bi = math.inf, 0
    for i, v in enumerate(col):
        if not math.isnan(v) and v < best:
            best, bi = v, i
    return bi


def weighted_kmeans(K, it_max, point, weight, centres):
    """my_weighted_kmeans.m:1-66."""
    point = [list(map(float, p)) for p in point]
    weight = [float(w) for w in weight]
    cen = [list(map(float, c)) for c in centres]
    cluster = [_argmin([sum((p[a] - cen[j][a]) ** 2 for a in range(len(p))) for j in range(K)])
               for p in point]
    cen, cw = _centroids(point, cluster, weight, K)
    f, energy = _energy(point, weight, cen, cw, cluster)
    old = sum(energy)
    it = 0
    while it < it_max:
        fmat = [[0.0] * len(point) for _ in range(K)]
        for j in range(K):
            for n, p in enumerate(point):
                if cluster[n] == j:
                    fmat[j][n] = f[n]
                else:
                    adj = _div(cw[j], cw[j] + weight[n])
                    fmat[j][n] = sum((p[a] - cen[j][a]) ** 2 for a in range(len(p))) * adj
        cluster = [_argmin([fmat[j][n] for j in range(K)]) for n in range(len(point))]
        cen, cw = _centroids(point, cluster, weight, K)
        f, energy = _energy(point, weight, cen, cw, cluster)
        new = sum(energy)
        if abs(new - old) < 1e-6:
            break
        old = new
        it += 1
    return cluster, cen


def hier_em_full(X, C, T, virtual_samples, iterations, cent):
    """GMM_MixHierEM.m:90-206 (full covariance) from given initial centres, one
    component and one point at a time (numpy only for the d x d inverse and
    determinant); returns (priors, centres, covars)."""
    import numpy as np
    X = [np.asarray(x, dtype=float) for x in X]
    C = [np.asarray(c, dtype=float) for c in C]
    n, dim = len(X), X[0].size
    prior = 1.0 / n
    cent = [np.asarray(c, dtype=float) for c in cent]
    mean_cov = sum(C) / n
    vr = [mean_cov.copy() for _ in range(T)]
    mxwt = [1.0 / T] * T
    coef = -(dim / 2.0) * math.log(2 * math.pi)
    dpp = prior * virtual_samples
    last = -1.7976931348623157e308
    for _ in range(iterations):
        xpt = [[0.0] * n for _ in range(T)]
        for t in range(T):
            ivr = np.linalg.inv(vr[t])
            ld = math.log(np.linalg.det(vr[t]))
            for k in range(n):
                tr = float((ivr * C[k]).sum())
                df = cent[t] - X[k]
                xpt[t][k] = math.log(mxwt[t]) + dpp * (coef - 0.5 * (tr + float(df @ ivr @ df) + ld))
        lx = []
        post = [[0.0] * n for _ in range(T)]
        for k in range(n):
            mv = max(xpt[t][k] for t in range(T))
            s = mv + math.log(sum(math.exp(xpt[t][k] - mv) for t in range(T)))
            lx.append(s)
            for t in range(T):
                post[t][k] = math.exp(xpt[t][k] - s)
        logp = sum(lx) / n
        if not math.isfinite(logp) or logp - last < 1e-6:
            break
        last = logp
        mxwt = [sum(post[t]) / n for t in range(T)]
        for t in range(T):
            w = [post[t][k] * prior for k in range(n)]
            sw = sum(w)
            w = [x / sw for x in w]
            cent[t] = sum(w[k] * X[k] for k in range(n))
            acc = np.zeros((dim, dim))
            for k in range(n):
                df = X[k] - cent[t]
                acc = acc + w[k] * (np.outer(df, df) + C[k])
            vr[t] = acc
    return mxwt, cent, vr
