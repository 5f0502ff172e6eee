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
