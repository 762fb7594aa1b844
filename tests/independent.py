"""Independent float64 Monte-Carlo estimator of the reference's image —
TEST INFRASTRUCTURE (the statistical leg of SURVEY §8c).

It follows the reference's semantics (main.cpp:354-446: thin-lens camera
pinhole.h:20-56 with lens radius 0, closest hit in [1e-3, inf) with
un-normalised directions ray.h:15-26, miss -> film += throughput x sky
main.cpp:407, interpolated un-normalised shading normal optix_backend.h:412-420,
Frame3 coordframe.h:17-30, cosine hemisphere mapping.h:5-11, albedo and
emission per material) but shares no code and no arithmetic choice with
oracle/oracle.c or the HIP kernels:

  - float64 throughout, numpy's sin / cos / sqrt (no Cephes sincos, no
    reciprocal-square-root normalise, no fixed fp32 operation order);
  - Moller-Trumbore against every triangle (no BVH, no watertight test, no
    tie rule);
  - numpy Philox streams instead of PCG32 (so no 4 + 2D draw layout, no
    y-first argument order), and its own Russian-roulette draws.

Its images therefore agree with the fp32 restatement only in distribution;
tests/test_statistical.py (oracle, CPU) and tests/test_gpu_parity.py (GPU)
check that with per-pixel and whole-image z scores.
"""
from __future__ import annotations

import math

import numpy as np


def _normalize(v):
    return v / np.linalg.norm(v)


def _camera(cam, W, H):
    """pinhole.h:9-25 (+ :40-41): basis, distance lens->film, aspect ratio."""
    frm = np.asarray(cam["look_from"], np.float64)
    at = np.asarray(cam["look_at"], np.float64)
    up = np.asarray(cam["up"], np.float64)
    z = _normalize(at - frm)
    x = _normalize(np.cross(up, z))
    y = _normalize(np.cross(z, x))
    assert cam["lens_radius"] == 0.0, "the estimator covers the reference's pinhole (lens radius 0)"
    dist = cam["film_size_y"] * 0.5 / math.tan(cam["fov_y"] * 0.5)
    return frm, x, y, z, dist, W / H


def _intersect(tris, ox, oy, oz, dx, dy, dz, tmin=1e-3):
    """Closest Moller-Trumbore hit over all triangles (float64).
    Returns (tri, t, u, v); tri = -1 on a miss."""
    n = ox.size
    best = np.full(n, np.inf)
    tri = np.full(n, -1, np.int64)
    bu = np.zeros(n)
    bv = np.zeros(n)
    for k in range(tris.shape[0]):
        v0, v1, v2 = tris[k]
        e1 = v1 - v0
        e2 = v2 - v0
        px = dy * e2[2] - dz * e2[1]
        py = dz * e2[0] - dx * e2[2]
        pz = dx * e2[1] - dy * e2[0]
        det = e1[0] * px + e1[1] * py + e1[2] * pz
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1.0 / det
            tx, ty, tz = ox - v0[0], oy - v0[1], oz - v0[2]
            u = (tx * px + ty * py + tz * pz) * inv
            qx = ty * e1[2] - tz * e1[1]
            qy = tz * e1[0] - tx * e1[2]
            qz = tx * e1[1] - ty * e1[0]
            v = (dx * qx + dy * qy + dz * qz) * inv
            t = (e2[0] * qx + e2[1] * qy + e2[2] * qz) * inv
            ok = (det != 0) & (u >= 0) & (v >= 0) & (u + v <= 1) & (t >= tmin) & (t < best)
        best = np.where(ok, t, best)
        tri = np.where(ok, k, tri)
        bu = np.where(ok, u, bu)
        bv = np.where(ok, v, bv)
    return tri, best, bu, bv


def _spheres(sph, ox, oy, oz, dx, dy, dz, tri, best, tmin=1e-3):
    """smallpt's analytic spheres after the triangles (float64, the textbook
    quadratic in the ray's own t units): ids -2 - k."""
    for k in range(sph.shape[0]):
        cx, cy, cz, r = sph[k]
        px, py, pz = cx - ox, cy - oy, cz - oz
        a = dx * dx + dy * dy + dz * dz
        b = px * dx + py * dy + pz * dz
        c = px * px + py * py + pz * pz - r * r
        disc = b * b - a * c
        with np.errstate(invalid="ignore"):
            sq = np.sqrt(np.maximum(disc, 0.0))
        t0, t1 = (b - sq) / a, (b + sq) / a
        t = np.where(t0 >= tmin, t0, np.where(t1 >= tmin, t1, np.inf))
        ok = (disc >= 0) & (t < best)
        best = np.where(ok, t, best)
        tri = np.where(ok, -2 - k, tri)
    return tri, best


def _reflect(dx, dy, dz, nx, ny, nz):
    k = 2.0 * (dx * nx + dy * ny + dz * nz)
    return dx - k * nx, dy - k * ny, dz - k * nz


def render(mesh: dict, W: int, H: int, spp: int, depth: int, camera: dict, env=(1.0, 1.0, 1.0), albedo=None,
           emission=None, rr_start_depth: int = 1 << 30, seed: int = 0, samples: bool = False):
    """Mean radiance per pixel, (3, H, W) float64; with samples=True also the
    per-sample radiance (3, H, W, spp) for variance estimates.  mesh may carry
    smallpt's "spheres" / "sphere_mat" and per-material "kinds" (0 diffuse,
    1 mirror, 2 glass: smallpt's radiance(), with the Fresnel choice made with
    probability Re and weight 1 — a different unbiased choice from the
    product's P = 1/4 + Re/2 with weights Re/P, Tr/(1-P))."""
    pos = np.asarray(mesh["pos"], np.float64).reshape(-1, 3)
    pt = np.asarray(mesh["pos_tri"], np.int64).reshape(-1, 3)
    tris = pos[pt]                                                    # (T, 3, 3)
    T = tris.shape[0]
    g = np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0])
    g = g / np.linalg.norm(g, axis=1, keepdims=True)                  # add_math.h:9-16 (missing normals)
    if mesh.get("nrm_tri") is not None:
        nt = np.asarray(mesh["nrm_tri"], np.int64).reshape(-1, 3)
        nrm = np.asarray(mesh["nrm"], np.float64).reshape(-1, 3)
        vn = np.where((nt >= 0)[..., None], nrm[np.maximum(nt, 0)], g[:, None, :])
    else:
        vn = np.repeat(g[:, None, :], 3, 1)
    mat = np.zeros(T, np.int64) if mesh.get("mat_id") is None else np.asarray(mesh["mat_id"], np.int64)
    alb = np.ones((1, 3)) if albedo is None else np.asarray(albedo, np.float64).reshape(-1, 3)
    emi = None if emission is None else np.asarray(emission, np.float64).reshape(-1, 3)
    env = np.asarray(env, np.float64)
    sph = None if mesh.get("spheres") is None else np.asarray(mesh["spheres"], np.float64).reshape(-1, 4)
    sph_mat = None if sph is None else np.asarray(mesh["sphere_mat"], np.int64).reshape(-1)
    kinds = None if mesh.get("kinds") is None else np.asarray(mesh["kinds"], np.int64).reshape(-1)

    frm, cx, cy, cz, dist, ratio = _camera(camera, W, H)
    rng = np.random.Generator(np.random.Philox(seed))
    P = W * H
    N = P * spp
    pix = np.repeat(np.arange(P), spp)
    px = (pix % W).astype(np.float64)
    py = (pix // W).astype(np.float64)
    xi = rng.random((2, N))
    fx = (0.5 - (px + xi[0]) / W) * (ratio * camera["film_size_y"])  # pinhole.h:43-50
    fy = (0.5 - (py + xi[1]) / H) * camera["film_size_y"]
    fd = camera["focal_dist"]
    lx, ly, lz = fd * fx / dist, fd * fy / dist, np.full(N, fd)
    ln = np.sqrt(lx * lx + ly * ly + lz * lz)
    lx, ly, lz = lx / ln, ly / ln, lz / ln
    dx = cx[0] * lx + cy[0] * ly + cz[0] * lz
    dy = cx[1] * lx + cy[1] * ly + cz[1] * lz
    dz = cx[2] * lx + cy[2] * ly + cz[2] * lz
    ox, oy, oz = (np.full(N, frm[i]) for i in range(3))
    thr = np.ones((N, 3))
    L = np.zeros((N, 3))
    idx = np.arange(N)                                                # live paths
    for j in range(depth):
        tri, t, u, v = _intersect(tris, ox, oy, oz, dx, dy, dz)
        if sph is not None:
            tri, t = _spheres(sph, ox, oy, oz, dx, dy, dz, tri, t)
        miss = tri == -1
        L[idx[miss]] += thr[miss] * env                               # main.cpp:407
        hit = ~miss
        # material per hit (triangles: mat_id; spheres: sphere_mat)
        mhit = np.where(tri >= 0, mat[np.maximum(tri, 0)],
                        sph_mat[np.maximum(-2 - tri, 0)] if sph is not None else 0)
        if emi is not None:
            m = mhit[hit]
            ok = (m >= 0) & (m < emi.shape[0])
            e = np.zeros((int(hit.sum()), 3))
            e[ok] = emi[m[ok]]
            L[idx[hit]] += thr[hit] * e
        if j + 1 >= depth:
            break                                                     # a hit on the last cast ends the path
        keep = hit
        tri, t, u, v = tri[keep], t[keep], u[keep], v[keep]
        ox, oy, oz, dx, dy, dz = ox[keep], oy[keep], oz[keep], dx[keep], dy[keep], dz[keep]
        thr, idx, mh = thr[keep], idx[keep], mhit[keep]
        is_s = tri < -1
        tt = np.maximum(tri, 0)
        w = 1.0 - u - v
        n = w[:, None] * vn[tt, 0] + u[:, None] * vn[tt, 1] + v[:, None] * vn[tt, 2]  # un-normalised
        kind = np.zeros(idx.size, np.int64) if kinds is None else np.where(
            (mh >= 0) & (mh < kinds.size), kinds[np.clip(mh, 0, max(kinds.size - 1, 0))], 0)
        if sph is not None and is_s.any():
            hp = np.stack([ox + t * dx, oy + t * dy, oz + t * dz], 1)
            c = sph[-2 - tri[is_s]]
            sn = (hp[is_s] - c[:, :3]) / c[:, 3:4]
            n[is_s] = sn
        special = is_s | (kind != 0)
        if special.any():      # smallpt: unit normal, flipped toward the ray for diffuse
            n[special] = n[special] / np.linalg.norm(n[special], axis=1, keepdims=True)
            flip = special & (kind == 0) & ((n * np.stack([dx, dy, dz], 1)).sum(1) >= 0)
            n[flip] = -n[flip]
        nx, ny, nz = n[:, 0], n[:, 1], n[:, 2]
        sign = np.where(ny >= 0, 1.0, -1.0)                           # coordframe.h:17-30
        a = -1.0 / (sign + ny)
        b = nz * nx * a
        bxx, bxy, bxz = sign + nx * nx * a, -nx, b
        bzx, bzy, bzz = sign * b, -sign * nz, 1.0 + sign * nz * nz * a
        r = rng.random((2, idx.size))
        sp = np.sqrt(1.0 - r[0])                                      # mapping.h:5-11
        phi = 2.0 * math.pi * r[1]
        ux, uy, uz = np.cos(phi) * sp, np.sqrt(r[0]), np.sin(phi) * sp
        hx, hy, hz = ox + t * dx, oy + t * dy, oz + t * dz
        ndx = bxx * ux + nx * uy + bzx * uz
        ndy = bxy * ux + ny * uy + bzy * uz
        ndz = bxz * ux + nz * uy + bzz * uz
        if (kind != 0).any():
            ln = np.sqrt(dx * dx + dy * dy + dz * dz)
            ux_, uy_, uz_ = dx / ln, dy / ln, dz / ln
            rx, ry, rz = _reflect(ux_, uy_, uz_, nx, ny, nz)
            mir = kind == 1
            ndx, ndy, ndz = np.where(mir, rx, ndx), np.where(mir, ry, ndy), np.where(mir, rz, ndz)
            gl = kind == 2
            if gl.any():
                cosi = ux_ * nx + uy_ * ny + uz_ * nz
                into = cosi < 0
                eta = np.where(into, 1.0 / 1.5, 1.5)
                cn = np.abs(cosi)
                k = 1.0 - eta * eta * (1.0 - cn * cn)
                sk = np.sqrt(np.maximum(k, 0.0))
                nlx, nly, nlz = (np.where(into, nx, -nx), np.where(into, ny, -ny), np.where(into, nz, -nz))
                tx_ = eta * ux_ + (eta * cn - sk) * nlx
                ty_ = eta * uy_ + (eta * cn - sk) * nly
                tz_ = eta * uz_ + (eta * cn - sk) * nlz
                r0 = (0.5 / 2.5) ** 2
                cc = 1.0 - np.where(into, cn, sk)                       # cos of the air-side angle
                re = r0 + (1.0 - r0) * cc ** 5
                pick = rng.random(idx.size)
                refl = (k < 0) | (pick < re)
                ndx = np.where(gl, np.where(refl, rx, tx_), ndx)
                ndy = np.where(gl, np.where(refl, ry, ty_), ndy)
                ndz = np.where(gl, np.where(refl, rz, tz_), ndz)
        dx, dy, dz = ndx, ndy, ndz
        ox, oy, oz = hx, hy, hz
        thr = thr * alb[np.where((mh >= 0) & (mh < alb.shape[0]), mh, 0)]   # main.cpp:422
        if j + 1 >= rr_start_depth:
            q = thr.max(axis=1)
            roll = rng.random(idx.size)
            live = (q >= 1.0) | (roll < q)
            thr = np.where((q < 1.0)[:, None], thr / np.maximum(q, 1e-300)[:, None], thr)
            ox, oy, oz, dx, dy, dz = ox[live], oy[live], oz[live], dx[live], dy[live], dz[live]
            thr, idx = thr[live], idx[live]
        if idx.size == 0:
            break
    per = L.reshape(H, W, spp, 3).transpose(3, 0, 1, 2)
    mean = per.mean(axis=3)
    return (mean, per) if samples else mean


def bernoulli_z(a, b, n_a: int, n_b: int):
    """Per-pixel two-sample z of escape fractions a, b (counts / n): pooled
    p(1-p)(1/n_a + 1/n_b); pixels where both are 0 or both 1 score 0."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    p = (a * n_a + b * n_b) / (n_a + n_b)
    var = p * (1.0 - p) * (1.0 / n_a + 1.0 / n_b)
    with np.errstate(divide="ignore", invalid="ignore"):
        z = np.where(var > 0, np.abs(a - b) / np.sqrt(var), 0.0)
    mean_z = abs(a.mean() - b.mean()) / math.sqrt(max(var.sum(), 1e-300)) * var.size if var.sum() > 0 else 0.0
    return z, mean_z


def stat_scene() -> dict:
    """A small scene for the statistical checks (every triangle is tested for
    every ray): a ground quad, back and left walls, a smooth low-poly sphere
    (interpolated, un-normalised shading normals) and a flat-shaded box,
    around the reference camera's view (main.cpp:383).  Materials 1-4."""
    pos, nrm, pt, nt, mat = [], [], [], [], []

    def add(p, n, tri, ntri, m):
        bp, bn = len(pos), len(nrm)
        pos.extend(p)
        nrm.extend(n)
        pt.extend([[a + bp for a in t] for t in tri])
        nt.extend([[a + bn for a in t] for t in ntri])
        mat.extend([m] * len(tri))

    s = 2.5
    add([[-s, 0, -s], [s, 0, -s], [s, 0, s], [-s, 0, s]], [[0, 1, 0]], [[0, 2, 1], [0, 3, 2]], [[0, 0, 0]] * 2, 1)
    # a back wall and a left wall (occluders: escape fractions well inside (0, 1))
    add([[-s, 0, -1.2], [s, 0, -1.2], [s, 2.0, -1.2], [-s, 2.0, -1.2]], [[0, 0, 1]], [[0, 1, 2], [0, 2, 3]],
        [[0, 0, 0]] * 2, 1)
    add([[-1.6, 0, -s], [-1.6, 0, s], [-1.6, 1.6, s], [-1.6, 1.6, -s]], [[1, 0, 0]], [[0, 1, 2], [0, 2, 3]],
        [[0, 0, 0]] * 2, 4)
    c, r, nlon, nlat = np.array([-0.3, 0.7, 0.0]), 0.7, 10, 6
    sp, sn = [], []
    for i in range(nlat + 1):
        th = math.pi * i / nlat
        for k in range(nlon):
            ph = 2 * math.pi * k / nlon
            d = np.array([math.sin(th) * math.cos(ph), math.cos(th), math.sin(th) * math.sin(ph)])
            sp.append(list(c + r * d))
            sn.append(list(d))
    st = []
    for i in range(nlat):
        for k in range(nlon):
            a, b = i * nlon + k, i * nlon + (k + 1) % nlon
            a2, b2 = a + nlon, b + nlon
            if i > 0:
                st.append([a, b, a2])
            if i < nlat - 1:
                st.append([b, b2, a2])
    add(sp, sn, st, st, 2)
    lo, hi = np.array([0.6, 0.0, -0.2]), np.array([1.3, 0.8, 0.6])
    corners = [[lo[0] if i & 1 == 0 else hi[0], lo[1] if i & 2 == 0 else hi[1], lo[2] if i & 4 == 0 else hi[2]]
               for i in range(8)]
    faces = [((0, 2, 6, 4), (-1, 0, 0)), ((1, 5, 7, 3), (1, 0, 0)), ((0, 4, 5, 1), (0, -1, 0)),
             ((2, 3, 7, 6), (0, 1, 0)), ((0, 1, 3, 2), (0, 0, -1)), ((4, 6, 7, 5), (0, 0, 1))]
    for (a, b, cc, d), n in faces:
        add([corners[a], corners[b], corners[cc], corners[d]], [list(n)], [[0, 1, 2], [0, 2, 3]], [[0, 0, 0]] * 2, 3)
    return {"pos": np.array(pos, np.float32), "nrm": np.array(nrm, np.float32),
            "pos_tri": np.array(pt, np.int32), "nrm_tri": np.array(nt, np.int32), "mat_id": np.array(mat, np.int32)}
