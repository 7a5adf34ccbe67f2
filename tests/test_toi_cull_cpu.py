"""The exact TOI cull's lower bound (csrc/nascar_device.h toi_far / toi_far_rot2), checked on the host.

Box2D's b2TimeOfImpact (src/car_physics.py:363 -> b2World::Step -> SolveTOI) can only return TOUCHING -- the one
outcome that changes a contact's alpha -- if the swept car comes within target + tolerance of the wall.  The device
skips the call when a lower bound of the car-wall distance over the whole sweep exceeds that by a margin.  This test
restates both bounds in float64 and checks, on random sweeps near random walls (including cars sliding along and
turning next to a wall), that each is below the true box-box distance at every sampled sweep parameter, i.e. that
a culled call can never have been TOUCHING.  (The GPU check build -DNASCAR_TOI_CULL_CHECK re-runs every culled call
at the steady state: 0 of ~30 k per step TOUCHING)
"""
import numpy as np

CAR_HX, CAR_HY = 5.042 / 2.0, 1.996 / 2.0
R_CAR = 2.80389


def rot(a):
    return np.stack([np.cos(a), np.sin(a)], -1)


def box_vertices(c, a, hx, hy):
    """[n, 4, 2] world vertices of boxes centred at c [n, 2] with angle a [n] and half extents hx, hy ([n] or scalar)."""
    hx = np.broadcast_to(hx, a.shape)
    hy = np.broadcast_to(hy, a.shape)
    loc = np.stack([np.stack([-hx, -hy], -1), np.stack([hx, -hy], -1), np.stack([hx, hy], -1), np.stack([-hx, hy], -1)], 1)
    cs, sn = np.cos(a)[:, None], np.sin(a)[:, None]
    x = cs * loc[..., 0] - sn * loc[..., 1]
    y = sn * loc[..., 0] + cs * loc[..., 1]
    return np.stack([x, y], -1) + c[:, None, :]


def seg_point_dist(p, a, b):
    ab = b - a
    t = np.clip(((p - a) * ab).sum(-1) / np.maximum((ab * ab).sum(-1), 1e-300), 0.0, 1.0)
    d = p - (a + t[..., None] * ab)
    return np.sqrt((d * d).sum(-1))


def box_distance(P, Q):
    """Exact distance between convex quads P, Q [n, 4, 2] (0 when they overlap: separating-axis test)."""
    n = P.shape[0]
    best = np.full(n, np.inf)
    for A, B in ((P, Q), (Q, P)):
        for i in range(4):
            a, b = B[:, i], B[:, (i + 1) % 4]
            for k in range(4):
                best = np.minimum(best, seg_point_dist(A[:, k], a, b))
    sep = np.zeros(n, bool)
    for S in (P, Q):
        for i in range(4):
            e = S[:, (i + 1) % 4] - S[:, i]
            u = np.stack([-e[:, 1], e[:, 0]], -1)
            pp = (P * u[:, None]).sum(-1)
            qq = (Q * u[:, None]).sum(-1)
            sep |= (pp.max(1) < qq.min(1)) | (qq.max(1) < pp.min(1))
    return np.where(sep, best, 0.0)


def ext(u, ax, ay, hx, hy):
    return hx * np.abs((u * ax).sum(-1)) + hy * np.abs((u * ay).sum(-1))


def bounds(c0, a0, c1, a1, w, wa, whx, why):
    """(first-order bound, second-order bound) as toi_far / toi_far_rot2 compute them (float64 here)."""
    q1 = rot(a1)
    cx1, cy1 = q1, np.stack([-q1[:, 1], q1[:, 0]], -1)
    q0 = rot(a0)
    cx0, cy0 = q0, np.stack([-q0[:, 1], q0[:, 0]], -1)
    wx = rot(wa)
    wy = np.stack([-wx[:, 1], wx[:, 0]], -1)
    d1, d0, dc = c1 - w, c0 - w, c1 - c0
    b1 = np.full(len(a0), -np.inf)
    b2 = np.full(len(a0), -np.inf)
    for u in (wx, wy, cx1, cy1):
        s1, s0 = (u * d1).sum(-1), (u * d0).sum(-1)
        we = ext(u, wx, wy, whx, why)
        g1 = np.abs(s1) - ext(u, cx1, cy1, CAR_HX, CAR_HY) - we
        away = np.where(s1 >= 0, (u * dc).sum(-1), -(u * dc).sum(-1))
        b1 = np.maximum(b1, g1 - np.maximum(0.0, away))
        g0 = np.where(s1 >= 0, s0, -s0) - ext(u, cx0, cy0, CAR_HX, CAR_HY) - we
        b2 = np.maximum(b2, np.minimum(g0, g1))
    da = np.abs(a1 - a0)
    return b1 - da * R_CAR, b2 - da * da * (R_CAR / 8.0)


def test_toi_cull_bounds_below_swept_distance():
    rng = np.random.default_rng(7)
    n = 20000
    wa = rng.uniform(-np.pi, np.pi, n)
    whx, why = rng.uniform(0.5, 6.0, n), rng.uniform(0.05, 0.6, n)
    w = rng.uniform(-500, 500, (n, 2))
    # car end pose near the wall: along its long side at a gap of -0.05 .. 1 m, nearly parallel or at any angle
    wx = rot(wa)
    wy = np.stack([-wx[:, 1], wx[:, 0]], -1)
    side = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    par = rng.random(n) < 0.7
    a1 = np.where(par, wa + rng.normal(0, 0.05, n) + np.where(rng.random(n) < 0.5, 0, np.pi), rng.uniform(-np.pi, np.pi, n))
    gap = rng.uniform(-0.05, 1.0, n)
    along = rng.uniform(-1, 1, n) * (whx + CAR_HX)
    q1 = rot(a1)
    e_car = ext(wy, q1, np.stack([-q1[:, 1], q1[:, 0]], -1), CAR_HX, CAR_HY)
    c1 = w + along[:, None] * wx + (side * (why + e_car + gap))[:, None] * wy
    # sweep start: up to 1 m back along a random direction, up to 0.1 rad of rotation (the culled range)
    c0 = c1 - rng.uniform(0, 1.0, (n, 1)) * rot(rng.uniform(-np.pi, np.pi, n))
    a0 = a1 - rng.uniform(-0.1, 0.1, n)
    b1, b2 = bounds(c0, a0, c1, a1, w, wa, whx, why)
    W = box_vertices(w, wa, whx, why)
    dmin = np.full(n, np.inf)
    for beta in np.linspace(0.0, 1.0, 65):
        cb = (1 - beta) * c0 + beta * c1
        ab = (1 - beta) * a0 + beta * a1
        dmin = np.minimum(dmin, box_distance(box_vertices(cb, ab, CAR_HX, CAR_HY), W))
    assert np.all(b1 <= dmin + 1e-9), np.max(b1 - dmin)
    assert np.all(b2 <= dmin + 1e-9), np.max(b2 - dmin)
    # the second-order bound is what culls a car scraping along a wall while turning (the round-3 change)
    scrape = par & (gap > 0.012) & (gap < 0.03) & (np.abs(a1 - a0) > 0.003)
    assert scrape.sum() > 20
    assert np.mean(b2[scrape] > 0.00925) > np.mean(b1[scrape] > 0.00925)
