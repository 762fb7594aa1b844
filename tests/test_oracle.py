"""CPU oracle pins (no GPU): published PCG32 known answers, formula-derived
camera known answers, analytic scenes, BVH vs brute force, and
the committed golden vectors (tests/golden/make_golden.py)."""
import math
import os

import numpy as np
import pytest

import oracle as O
from sptamd import scenes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_small.npz")
MULT = 0x5851F42D4C957F2D
M64 = (1 << 64) - 1


def test_pcg32_canonical_kat():
    # pcg32 reference implementation, pcg32_srandom_r(42, 54): the published demo output
    got = O.pcg32_seq(42, 54, 6)
    assert [f"{x:08x}" for x in got] == ["a15c02b7", "7b47f409", "ba1d3330", "83d2f293", "bfa4784b", "cbed606e"]


@pytest.mark.parametrize("seq,expect", [
    (0, ["69c87837", "6694bd1c", "a37b7ac6", "572d246c"]),
    (1, ["73c29fdb", "fbaa1ff7", "db022af6", "12d7398c"]),
    (1023, ["0a82b6cb", "7666067b", "68efb589", "a03cf93b"]),
])
def test_pcg32_reference_seeding(seq, expect):
    # main.cpp:376 — initstate PCG32_DEFAULT_STATE, initseq = pixel index
    assert [f"{x:08x}" for x in O.pcg32_seq(O.PCG32_DEFAULT_STATE, seq, 4)] == expect


def test_next_float32_mapping():
    u = O.pcg32_seq(O.PCG32_DEFAULT_STATE, 7, 64)
    f = O.pcg32_floats(O.PCG32_DEFAULT_STATE, 7, 64)
    expect = ((u >> 9) | 0x3F800000).astype(np.uint32).view(np.float32) - np.float32(1.0)
    np.testing.assert_array_equal(f, expect)
    assert f.min() >= 0.0 and f.max() < 1.0


def _jump(n):
    """Restatement of spt_math.h pcg_jump_coeffs (used by the GPU refill)."""
    am, aa, cm, ca = 1, 0, MULT, 1
    while n:
        if n & 1:
            am, aa = (am * cm) & M64, (aa * cm + ca) & M64
        ca = ((cm + 1) * ca) & M64
        cm = (cm * cm) & M64
        n >>= 1
    return am, aa


@pytest.mark.parametrize("n", [0, 1, 2, 3, 20, 68, 4 * 68 + 2, 1000])
def test_pcg32_jump_ahead(n):
    # seeding state, then n LCG steps == one affine jump
    inc = (12345 << 1) | 1
    st = 0
    st = (st * MULT + inc) & M64
    st = (st + O.PCG32_DEFAULT_STATE) & M64
    st = (st * MULT + inc) & M64
    s = st
    for _ in range(n):
        s = (s * MULT + inc) & M64
    am, aa = _jump(n)
    assert (am * st + aa * inc) & M64 == s


@pytest.mark.parametrize("seq", [0, 1, 1023, 2 ** 24 - 1])
@pytest.mark.parametrize("n", [0, 4, 68, 63 * 68])
def test_pcg32_seeded_jump_fold(seq, n):
    """spt_math.h pcg_seeded_jump / pcg_start: seeding with initstate S0 and then
    jumping n draws is one affine map of inc, A inc + B with A = mul (M + 1) +
    add and B = mul S0 M: the draws that follow equal the oracle's sequential
    PCG32 from draw n on."""
    am, aa = _jump(n)
    A = (am * (MULT + 1) + aa) & M64
    B = (am * O.PCG32_DEFAULT_STATE * MULT) & M64
    inc = ((seq << 1) | 1) & M64
    st = (A * inc + B) & M64
    out = []
    for _ in range(6):  # pcg32 next_u32 (A1)
        old = st
        st = (old * MULT + inc) & M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        out.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF)
    np.testing.assert_array_equal(np.array(out, np.uint32),
                                  O.pcg32_seq(O.PCG32_DEFAULT_STATE, seq, n + 6)[n:])


def test_camera_known_answers():
    p = O.reference_params(1024, 1024, 1, 1)
    o, d, basis = O.camera_ray(p, 0, 0, [0, 0, 0, 0])
    np.testing.assert_allclose(basis[0], [-1, 0, 0], atol=1e-6)
    np.testing.assert_allclose(basis[1], [0, 0.857493, -0.514496], atol=1e-6)
    np.testing.assert_allclose(basis[2], [0, -0.514496, -0.857493], atol=1e-6)
    np.testing.assert_array_equal(o, np.array([0.0, 3.03, 5.0], np.float32))  # lens radius 0
    np.testing.assert_allclose(d, [-0.323616, -0.179954, -0.928919], atol=2e-6)
    _, d2, _ = O.camera_ray(p, 512, 512, [0, 0, 0, 0])
    np.testing.assert_allclose(d2, [0, -0.514496, -0.857493], atol=2e-6)


def test_sincos_accuracy():
    xs = np.linspace(-4 * math.pi, 4 * math.pi, 20001).astype(np.float32)
    err = 0.0
    for x in xs[::7]:
        s, c = O.sincos(float(x))
        err = max(err, abs(s - math.sin(float(x))), abs(c - math.cos(float(x))))
    assert err < 3e-7


def test_cosine_hemisphere():
    g = (np.arange(64) + 0.5) / 64
    ys, norms = [], []
    for a in g:
        for b in g[::4]:
            v = O.cosine_hemisphere(float(a), float(b))
            ys.append(v[1])
            norms.append(np.linalg.norm(v))
            assert v[1] == np.float32(math.sqrt(np.float32(a)))  # mapping.h:10
    np.testing.assert_allclose(norms, 1.0, atol=1e-6)
    assert abs(np.mean(ys) - 2.0 / 3.0) < 2e-3                 # E[cos] under cos/pi


def test_disk_from_square():
    for a in np.linspace(0.0, 0.999, 37):
        for b in np.linspace(0.001, 0.999, 41):
            p = O.disk_from_square(float(a), float(b))
            assert np.hypot(*p) <= 1.0 + 1e-6
    np.testing.assert_allclose(np.hypot(*O.disk_from_square(0.0, 0.5)), 1.0, atol=1e-6)


def test_frame_unit_normal_orthonormal():
    rng = np.random.default_rng(0)
    for _ in range(200):
        n = rng.normal(size=3).astype(np.float32)
        n /= np.linalg.norm(n)
        y = O.frame_to_world(n, [0, 1, 0])
        np.testing.assert_allclose(y, n, atol=1e-7)
        bx = O.frame_to_world(n, [1, 0, 0])
        bz = O.frame_to_world(n, [0, 0, 1])
        m = np.stack([bx, y, bz])
        np.testing.assert_allclose(m @ m.T, np.eye(3), atol=2e-6)


def _mt64(o, d, v0, v1, v2):
    """float64 Moller-Trumbore reference."""
    e1, e2 = v1 - v0, v2 - v0
    p = np.cross(d, e2)
    det = e1 @ p
    if abs(det) < 1e-300:
        return None
    tv = o - v0
    u = (tv @ p) / det
    q = np.cross(tv, e1)
    v = (d @ q) / det
    t = (e2 @ q) / det
    return t, u, v


def test_watertight_triangle_vs_float64():
    rng = np.random.default_rng(3)
    n = 3000
    tri = rng.normal(size=(n, 3, 3)).astype(np.float32)
    mesh = {"pos": tri.reshape(-1, 3), "pos_tri": np.arange(3 * n, dtype=np.int32).reshape(-1, 3)}
    sc = O.OracleScene(mesh, use_bvh=False)
    agree = 0
    for k in range(n):
        o = rng.normal(size=3).astype(np.float32) * 3
        target = tri[k].mean(0) + rng.normal(size=3).astype(np.float32) * 0.3
        d = (target - o).astype(np.float32)
        single = O.OracleScene({"pos": tri[k], "pos_tri": np.array([[0, 1, 2]], np.int32)}, use_bvh=False)
        hid, t, u, v = single.intersect(o.reshape(3, 1), d.reshape(3, 1), tmin=np.zeros(1, np.float32))
        ref = _mt64(o.astype(np.float64), d.astype(np.float64), *tri[k].astype(np.float64))
        inside = ref is not None and ref[1] >= 0 and ref[2] >= 0 and ref[1] + ref[2] <= 1 and ref[0] >= 0
        margin = ref is not None and min(abs(ref[1]), abs(ref[2]), abs(1 - ref[1] - ref[2])) < 1e-4
        if margin:
            continue
        assert (hid[0] == 0) == inside
        if inside:
            np.testing.assert_allclose(t[0], ref[0], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose([u[0], v[0]], [ref[1], ref[2]], atol=1e-5)
        agree += 1
    assert agree > 2500
    del sc


def test_bvh_equals_bruteforce():
    mesh = scenes.mitsuba_synth(detail=0.1)
    g = np.load(GOLDEN)
    o, d = g["isect_o"], g["isect_d"]
    a = O.OracleScene(mesh, use_bvh=True).intersect(o, d)
    b = O.OracleScene(mesh, use_bvh=False).intersect(o, d)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert (a[0] >= 0).sum() > 1000


def test_bvh_equals_bruteforce_on_surface_leaving_rays():
    """Tree independence where it is at stake: rays leaving the surfaces they
    hit (origins on or next to triangle planes, both hemispheres), BVH2 =
    brute force bit for bit, with the box-exit rule."""
    from conftest import surface_rays
    mesh = scenes.mitsuba_synth(detail=0.25)
    bvh = O.OracleScene(mesh, use_bvh=True)
    brute = O.OracleScene(mesh, use_bvh=False)
    pos = np.asarray(mesh["pos"], np.float32)
    o, d = surface_rays(lambda o, d: bvh.intersect(o, d), pos.min(0), pos.max(0), 24000, seed=11)
    a = bvh.intersect(o, d)
    b = brute.intersect(o, d)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert o.shape[1] > 8000 and (a[0] >= 0).sum() > 500


def test_golden_regenerations_recorded():
    """every file a regeneration replaced is kept beside the
    current one; the current vectors differ from each by exactly the counts
    tests/golden/regen_log.json records, all within SURVEY §8(c)'s tolerance
    (make_golden.compare), so a silent regeneration fails here."""
    import json
    import sys
    sys.path.insert(0, os.path.dirname(GOLDEN))
    import make_golden as MG
    log = json.load(open(os.path.join(os.path.dirname(GOLDEN), "regen_log.json")))
    kept = MG.kept_files()
    assert kept, "no replaced golden file kept"
    cur = np.load(GOLDEN)
    for f in kept:
        res = MG.compare(np.load(os.path.join(os.path.dirname(GOLDEN), f)), cur)
        assert all(v["ok"] for v in res.values()), (f, res)
        changed = {k: v["changed"] for k, v in res.items() if v["changed"]}
        assert f in log and log[f]["changed"] == changed, (f, changed)


def test_golden_vectors():
    g = np.load(GOLDEN)
    for s, row in zip(g["pcg_seeds"], g["pcg_u32"]):
        np.testing.assert_array_equal(O.pcg32_seq(O.PCG32_DEFAULT_STATE, int(s), 32), row)
    mesh = scenes.mitsuba_synth(detail=0.1)
    sc = O.OracleScene(mesh)
    tri, t, u, v = sc.intersect(g["isect_o"], g["isect_d"])
    np.testing.assert_array_equal(tri, g["isect_tri"])
    h = tri >= 0
    for a, b in ((t, g["isect_t"]), (u, g["isect_u"]), (v, g["isect_v"])):
        np.testing.assert_array_equal(a[h], b[h])
    np.testing.assert_array_equal(sc.render(O.reference_params(32, 24, 4, 4))[0], g["film_32x24_4spp_d4"])
    np.testing.assert_array_equal(sc.render(O.reference_params(32, 24, 4, 4, rng_order=1))[0],
                                  g["film_32x24_4spp_d4_xfirst"])
    np.testing.assert_array_equal(sc.render(O.reference_params(16, 16, 100, 2))[0], g["film_16x16_100spp_d2"])
    alb = O.OracleScene(mesh, albedo=g["albedo"])
    np.testing.assert_array_equal(alb.render(O.reference_params(20, 16, 6, 6, rr_start_depth=2))[0],
                                  g["film_albedo_rr2"])


def _big_plane(y=-1.0, half=100.0):
    pos = np.array([[-half, y, -half], [half, y, -half], [half, y, half], [-half, y, half]], np.float32)
    return {"pos": pos, "pos_tri": np.array([[0, 1, 2], [0, 2, 3]], np.int32),
            "nrm": np.array([[0, 1, 0]], np.float32), "nrm_tri": np.zeros((2, 3), np.int32)}


def test_analytic_plane():
    """Camera above a plane wide enough to fill the view (half-size 100: at
    1e4 the fp32 hit points drift ~1e-3 off the plane and re-hit it), looking
    down: every camera
    ray hits it; a bounce leaves upward and always escapes.  So with one cast
    no path escapes (image 0) and with >= 2 casts every path does (image 1)."""
    sc = O.OracleScene(_big_plane())
    f1, casts1 = sc.render(O.reference_params(24, 24, 3, 1))
    assert np.all(f1 == 0.0) and casts1 == 24 * 24 * 3
    f3, casts3 = sc.render(O.reference_params(24, 24, 3, 3))
    assert np.all(f3 == 1.0) and casts3 == 2 * 24 * 24 * 3


def test_analytic_closed_box():
    """A closed box around the camera: nothing escapes, at any depth."""
    c = np.array([[x, y, z] for x in (-20, 20) for y in (-20, 20) for z in (-20, 20)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    tris = np.array([t for a, b, cc, d in quads for t in ((a, b, cc), (a, cc, d))], np.int32)
    # inward normals: the bounce hemisphere follows the shading normal, unflipped (coordframe.h:17-30)
    nrm = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    nt = np.repeat(np.arange(6, dtype=np.int32), 2)[:, None].repeat(3, 1)
    sc = O.OracleScene({"pos": c, "pos_tri": tris, "nrm": nrm, "nrm_tri": nt})
    f, casts = sc.render(O.reference_params(16, 16, 2, 5))
    assert np.all(f == 0.0) and casts == 16 * 16 * 2 * 5


def test_emissive_closed_box_geometric_series():
    """Every wall emits Le = 1 with albedo 1/2 and nothing escapes: with D casts
    and no roulette each sample gathers 1 + 1/2 + ... + 2^(1-D), exact in fp32."""
    c = np.array([[x, y, z] for x in (-20, 20) for y in (-20, 20) for z in (-20, 20)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    tris = np.array([t for a, b, cc, d in quads for t in ((a, b, cc), (a, cc, d))], np.int32)
    nrm = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    nt = np.repeat(np.arange(6, dtype=np.int32), 2)[:, None].repeat(3, 1)
    mesh = {"pos": c, "pos_tri": tris, "nrm": nrm, "nrm_tri": nt, "mat_id": np.ones(12, np.int32)}
    sc = O.OracleScene(mesh, albedo=[[1, 1, 1], [0.5, 0.5, 0.5]], emission=[[0, 0, 0], [1, 1, 1]])
    for depth in (1, 4, 7):
        f, casts = sc.render(O.reference_params(12, 10, 3, depth, rr_start_depth=depth))
        assert casts == 12 * 10 * 3 * depth
        assert np.all(f == np.float32(2.0 - 2.0 ** (1 - depth))), depth


def test_emission_off_material_and_sky_sum():
    """Emitters on one material, sky on: each sample is its emitted hits plus
    the sky term; with emission all zero the image equals the reference's."""
    m = scenes.mitsuba_synth(detail=0.1)
    p = O.reference_params(24, 20, 4, 4)
    base, _ = O.OracleScene(m).render(p)
    zero, _ = O.OracleScene(m, emission=np.zeros((len(m["kd"]), 3), np.float32)).render(p)
    np.testing.assert_array_equal(base, zero)
    emi = np.zeros((len(m["kd"]), 3), np.float32)
    emi[1] = (0.5, 0.25, 0.0)
    lit, _ = O.OracleScene(m, emission=emi).render(p)
    assert np.all(lit >= base) and np.any(lit[0] > base[0]) and np.all(lit[2] == base[2])


def test_film_is_escape_fraction():
    """Albedo 1, sky 1: every pixel is an exact count / spp, R=G=B."""
    sc = O.OracleScene(scenes.mitsuba_synth(detail=0.1))
    f, _ = sc.render(O.reference_params(32, 32, 7, 4))
    np.testing.assert_array_equal(f[0], f[1])
    np.testing.assert_array_equal(f[0], f[2])
    counts = f[0] * np.float32(7)
    np.testing.assert_allclose(counts, np.round(counts), atol=1e-5)
    assert 0.0 < f.mean() < 1.0


def test_bvh_ties_and_parallel_rays_equal_bruteforce():
    """The oracle's BVH gives brute force's answer on rays aimed at shared
    edges and vertices (t ties: the smaller triangle id must win whatever
    box is entered first) and on rays parallel to slab planes with the
    origin on a plane (d = +-0: 0 * inf would be NaN)."""
    n = 16
    xs = np.linspace(-1.0, 1.0, n + 1, dtype=np.float32)
    gx, gz = np.meshgrid(xs, xs, indexing="ij")
    pos = np.stack([gx.ravel(), np.zeros(gx.size, np.float32), gz.ravel()], 1)
    i = np.arange(n)[:, None] * (n + 1) + np.arange(n)[None, :]
    a, b, c, d = i, i + n + 1, i + n + 2, i + 1
    tris = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    m = {"pos_tri": tris.astype(np.int32), "pos": pos}
    rng = np.random.default_rng(5)
    targets = pos[rng.integers(0, len(pos), 3000)]
    o = (targets + rng.normal(size=targets.shape).astype(np.float32) * np.float32([0.3, 0.0, 0.3]))
    o[:, 1] = rng.uniform(0.5, 3.0, size=len(o))
    o = o.astype(np.float32)
    dd = (targets - o).astype(np.float32)
    dd[::4, 0] = 0.0                        # parallel to the x slabs, origin on a grid plane
    o[::4, 0] = targets[::4, 0]
    o, dd = o.T.copy(), dd.T.copy()
    bvh = O.OracleScene(m, use_bvh=True).intersect(o, dd)
    brute = O.OracleScene(m, use_bvh=False).intersect(o, dd)
    for x, y in zip(bvh, brute):
        np.testing.assert_array_equal(x, y)
    assert (brute[0] >= 0).mean() > 0.95


def test_texture_eval_known_answers():
    """ImageTexture::eval (main.cpp:62-76): texel centres return the texel, the
    edges clamp, the index is y * height + x (main.cpp:52), and a 1 x 1 image
    is its colour up to the rounding of the bilinear weights."""
    img = np.arange(2 * 2 * 3, dtype=np.float32).reshape(2, 2, 3)
    for (x, y) in ((0, 0), (1, 0), (0, 1), (1, 1)):
        np.testing.assert_array_equal(O.texture_eval(img, (x + 0.5) / 2, (y + 0.5) / 2), img[y, x])
    np.testing.assert_array_equal(O.texture_eval(img, -3.0, -3.0), img[0, 0])      # clamped
    np.testing.assert_array_equal(O.texture_eval(img, 7.0, 7.0), img[1, 1])
    mid = O.texture_eval(img, 0.5, 0.5)                                                 # bilinear centre
    np.testing.assert_allclose(mid, img.reshape(4, 3).mean(0), rtol=1e-6)
    # non-square: 4 wide, 2 high -> texel (x, y) read from flat index y * 2 + x
    wide = np.arange(2 * 4 * 3, dtype=np.float32).reshape(2, 4, 3)
    flat = wide.reshape(-1, 3)
    np.testing.assert_array_equal(O.texture_eval(wide, 3.5 / 4, 1.5 / 2), flat[1 * 2 + 3])
    # 2 wide, 4 high: y * 4 + x past the end is kept inside the image (last texel)
    tall = np.arange(4 * 2 * 3, dtype=np.float32).reshape(4, 2, 3)
    np.testing.assert_array_equal(O.texture_eval(tall, 1.5 / 2, 3.5 / 4), tall.reshape(-1, 3)[-1])
    one = np.full((1, 1, 3), 0.7, np.float32)
    rng = np.random.default_rng(0)
    vals = np.array([O.texture_eval(one, *rng.uniform(-2, 2, 2)) for _ in range(500)])
    assert np.all(np.abs(vals - np.float32(0.7)) <= 2 * np.spacing(np.float32(0.7)))
    assert np.any(vals != np.float32(0.7))     # the reference's weights do not always sum to exactly 1


def test_tex1x1_variant_within_tolerance():
    """The albedo table stands in for the reference's 1 x 1 ImageTexture of each
    material's colour (main.cpp:40-44); evaluated as the reference does, the
    bilinear weights differ from 1 by rounding only — inside §8c's tolerance."""
    from test_parity_tolerance import assert_within_tolerance
    m = scenes.with_planar_uv(scenes.mitsuba_synth(detail=0.25))
    p = O.reference_params(128, 128, 32, 6)
    base, _ = O.OracleScene(m).render(p)
    alt, _ = O.OracleScene(m, lib=O.variant("tex1x1")).render(p)
    assert_within_tolerance(alt, base, 32, "tex1x1")
    # at 32 spp the 1-ulp weight sums vanish in the film sum; one sample per
    # pixel shows them (the variant is live: texcoords vary)
    p1 = O.reference_params(128, 128, 1, 3)
    one, _ = O.OracleScene(m).render(p1)
    one_alt, _ = O.OracleScene(m, lib=O.variant("tex1x1")).render(p1)
    assert not np.array_equal(one_alt, one)
    np.testing.assert_allclose(one_alt, one, rtol=1e-6, atol=0)


def _tiny_far_mesh():
    """One small triangle far from everything (the spheres do the work)."""
    return {"pos": np.array([[100, 100, 100], [101, 100, 100], [100, 101, 100]], np.float32),
            "pos_tri": np.array([[0, 1, 2]], np.int32), "mat_id": np.zeros(1, np.int32)}


def test_sphere_intersection_known_answers():
    """smallpt Sphere::intersect in the ray's t units: from outside the nearer
    root, from inside the far one, tmin / tmax windows, misses; ids -2 - k."""
    m = _tiny_far_mesh()
    sph = np.array([[0, 0, 0, 1], [0, 0, 10, 2]], np.float32)
    sc = O.OracleScene(m, spheres=sph, sphere_mat=[3, 4])
    o = np.array([[0, 0, 0, 0, 0, 5], [0, 0, 0, 0, 0, 0], [-5, 0, -5, -5, 10, 0]], np.float32)
    d = np.array([[0, 1, 0, 0, 0, 0], [0, 0, 0, 0, 0, 1], [2, 0, 2, 2, -1, 0]], np.float32)
    tmax = np.array([1e20, 1e20, 1.5, 1e20, 1e20, 1e20], np.float32)
    tmin = np.array([1e-3, 1e-3, 1e-3, 2.5, 1e-3, 1e-3], np.float32)
    tri, t, _, _ = sc.intersect(o, d, tmin=tmin, tmax=tmax)
    # 0: outside -> t = (5 - 1) / 2; 1: inside -> t = 1; 2: tmax 1.5 < 2 -> miss;
    # 3: tmin 2.5 -> far root (5 + 1) / 2; 4: inside sphere 1 (r 2) toward -z -> 2;
    # 5: from (5, 0, 0) along +y misses both
    np.testing.assert_array_equal(tri, [-2, -2, -1, -2, -3, -1])
    np.testing.assert_array_equal(t[[0, 1, 3, 4]], np.float32([2.0, 1.0, 3.0, 2.0]))
    # any-hit: the same hit / miss answer
    tri_a, *_ = sc.intersect(o, d, tmin=tmin, tmax=tmax, closest=False)
    np.testing.assert_array_equal(tri_a != -1, tri != -1)


@pytest.mark.parametrize("kind", [0, 1])
def test_emissive_sphere_geometric_series(kind):
    """The camera inside a sphere that emits Le = 1 with albedo 1/2: a diffuse
    (nl flipped inward) or mirror wall is hit on every cast, so each sample
    gathers 1 + 1/2 + ... + 2^(1-D), exact in fp32."""
    m = _tiny_far_mesh()
    cam = (0.0, 3.03, 5.0)
    sph = np.array([[cam[0], cam[1], cam[2], 3.0]], np.float32)
    sc = O.OracleScene(m, albedo=[[1, 1, 1], [0.5, 0.5, 0.5]], emission=[[0, 0, 0], [1, 1, 1]],
                       spheres=sph, sphere_mat=[1], kinds=np.array([0, kind], np.uint32))
    for depth in (1, 5):
        f, casts = sc.render(O.reference_params(10, 8, 3, depth, rr_start_depth=depth, env=(0, 0, 0)))
        assert casts == 10 * 8 * 3 * depth
        assert np.all(f == np.float32(2.0 - 2.0 ** (1 - depth))), (kind, depth)


def test_glass_sphere_conserves_energy():
    """The camera inside a clear glass ball under a unit sky: Fresnel splits
    only redistribute weight (Re/P, Tr/(1-P)), so the image's expectation is
    the probability of escaping within the cast budget, ~1 at depth 24."""
    m = _tiny_far_mesh()
    sph = np.array([[0.0, 3.03, 5.0, 0.5]], np.float32)
    sc = O.OracleScene(m, spheres=sph, sphere_mat=[1], kinds=np.array([0, 2], np.uint32))
    f, _ = sc.render(O.reference_params(16, 16, 64, 24, rr_start_depth=99, env=(1, 1, 1)))
    assert abs(f.mean() - 1.0) < 0.03, f.mean()
    assert f.std() > 0.05      # the weights differ per sample



def test_hit_past_tmin_outside_triangle_box_known_case():
    """Pinned known case (config 4's city_synth, found by tools/diag_parity.py in
    round 3): a ray leaving a column surface, its origin on the triangle's
    plane, gets a Woop hit at t = 0.0015 (past tmin = 0.001) outside the
    triangle's own box, which the ray leaves at t = 0.0003 (in x and z).
    Without the box-exit rule brute force kept the hit and a tree that culls
    boxes left before tmin dropped it, so the answer depended on the tree.
    With the rule (spt_math.h left_box_before_tmin, oracle.c woop_test) the
    hit is dropped by every tracer: brute force and BVH agree on a miss."""
    pos = np.array([[-0.249440879, -1, 8.8333292], [-0.212132037, 5, 8.78786755], [-0.249440879, 5, 8.8333292]],
                   np.float32)
    m = {"pos_tri": np.array([[0, 1, 2]], np.int32), "pos": pos}
    o = np.array([[-0.24933969974517822], [1.7225027084350586], [8.833206176757812]], np.float32)
    d = np.array([[-0.3425644636154175], [0.8412052392959595], [0.4182586371898651]], np.float32)
    brute = O.OracleScene(m, use_bvh=False).intersect(o, d)
    bvh = O.OracleScene(m).intersect(o, d)
    assert brute[0][0] == -1
    assert bvh[0][0] == -1
    # the same ray from just behind the plane's neighbourhood (tmin 0) hits:
    # the rule only drops hits whose box the ray has left before tmin
    t0 = np.zeros(1, np.float32)
    hit0 = O.OracleScene(m, use_bvh=False).intersect(o, d, tmin=t0)
    assert hit0[0][0] == 0


def test_box_exit_rule_keeps_hits_on_axis_aligned_triangles():
    """The rule must not drop genuine hits where the Woop t and the slab t
    round differently: axis-aligned walls hit head-on, at grazing angles and
    close to tmin, BVH = brute force, every ray that crosses the wall inside
    its extent beyond tmin hits it."""
    rng = np.random.default_rng(7)
    # a wall x = 1 (two triangles over y, z in [-1, 1]) and a floor y = 0
    pos = np.array([[1, -1, -1], [1, 1, -1], [1, 1, 1], [1, -1, 1],
                    [-3, 0, -3], [3, 0, -3], [3, 0, 3], [-3, 0, 3]], np.float32)
    tri = np.array([[0, 1, 2], [0, 2, 3], [4, 5, 6], [4, 6, 7]], np.int32)
    m = {"pos_tri": tri, "pos": pos}
    n = 20000
    o = np.stack([rng.uniform(-0.5, 0.999, n), rng.uniform(0.0005, 0.9, n), rng.uniform(-0.9, 0.9, n)]).astype(np.float32)
    d = np.stack([rng.uniform(0.01, 1, n), rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)]).astype(np.float32)
    brute = O.OracleScene(m, use_bvh=False).intersect(o, d)
    bvh = O.OracleScene(m).intersect(o, d)
    for a, b in zip(brute, bvh):
        np.testing.assert_array_equal(a, b)
    # float64 ground truth for the wall: t = (1 - ox) / dx, point inside the square
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    tw = (1.0 - o64[0]) / d64[0]
    yw, zw = o64[1] + tw * d64[1], o64[2] + tw * d64[2]
    tf = np.where(d64[1] < 0, -o64[1] / np.where(d64[1] < 0, d64[1], -1), np.inf)  # floor first?
    clear = (np.abs(yw) < 0.999) & (np.abs(zw) < 0.999) & (tw > 0.0011) & (tw < tf * 0.999)
    assert clear.sum() > 1000
    assert np.all(np.isin(brute[0][clear], [0, 1])), "a clear wall hit was dropped"


def test_box_exit_rule_keeps_hits_at_negative_tmin():
    """with a negative per-ray tmin a box exit can be negative too;
    the rule pads it toward +inf (spt_math.h pad_up), so a genuine hit whose
    exact exit equals tmin is kept.  A wall z = -1 behind the origin, rays
    along +z with tmin = -1: the hit at t = -1 is exact (its box exit is
    exactly -1), and so is one at tmin = -0.5 - ... (the wall at t = -0.5)."""
    pos = np.array([[-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1]], np.float32)
    m = {"pos_tri": np.array([[0, 1, 2], [0, 2, 3]], np.int32), "pos": pos}
    n = 64
    rng = np.random.default_rng(2)
    o = np.stack([rng.uniform(-0.5, 0.5, n), rng.uniform(-0.5, 0.5, n), np.zeros(n)]).astype(np.float32)
    d = np.stack([np.zeros(n), np.zeros(n), np.ones(n)]).astype(np.float32)
    for scale in (1.0, 2.0):  # d = (0, 0, 1) hits at t = -1; d = (0, 0, 2) at t = -0.5
        dd = d * np.float32(scale)
        tmin = np.full(n, -1.0 / scale, np.float32)
        for use_bvh in (False, True):
            tri, t, _, _ = O.OracleScene(m, use_bvh=use_bvh).intersect(o, dd, tmin=tmin)
            assert np.all(tri >= 0), (scale, use_bvh)
            np.testing.assert_array_equal(t, tmin)
        # just past the exit (tmin above it) the wall is not hit
        tmin2 = np.full(n, np.nextafter(np.float32(-1.0 / scale), np.float32(1.0)), np.float32)
        assert np.all(O.OracleScene(m, use_bvh=False).intersect(o, dd, tmin=tmin2)[0] == -1)


def box_exit_audit(mesh_pos, pos_tri, sc, o, d, tmin=0.001):
    """Every Woop hit in [tmin, tmax] that the box-exit rule drops
    (oracle_box_rule_audit, enumerating triangles along the whole ray line)
    against a float64 box exit: the exact exit of a dropped hit's triangle box
    must lie before tmin — so no genuine hit (whose point lies in the box at
    t >= tmin) is dropped.  Returns (dropped pairs, accepted pairs, the
    largest exit / tmin ratio among the dropped)."""
    import ctypes
    n = o.shape[1]
    lib = sc.lib
    lib.oracle_box_rule_audit.restype = ctypes.c_int64
    vp = ctypes.c_void_p
    lib.oracle_box_rule_audit.argtypes = [vp] + [vp] * 8 + [ctypes.c_int64, vp, vp, vp, ctypes.c_int64, vp, ctypes.c_int32]
    o = np.ascontiguousarray(o, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    tmn = np.full(n, tmin, np.float32)
    tmx = np.full(n, 1e20, np.float32)
    cap = 1 << 20
    ray = np.zeros(cap, np.int64)
    tri = np.zeros(cap, np.int32)
    tt = np.zeros(cap, np.float32)
    acc = ctypes.c_int64(0)
    p = lambda a: a.ctypes.data  # noqa: E731
    found = lib.oracle_box_rule_audit(sc.h, p(o[0]), p(o[1]), p(o[2]), p(d[0]), p(d[1]), p(d[2]), p(tmn), p(tmx), n,
                                      p(ray), p(tri), p(tt), cap, ctypes.byref(acc), 8)
    assert found <= cap
    ray, tri = ray[:found], tri[:found]
    v = np.asarray(mesh_pos, np.float64)[np.asarray(pos_tri, np.int64)[tri]]  # (k, 3 vertices, 3)
    lo, hi = v.min(axis=1), v.max(axis=1)
    oo, dd = o[:, ray].T.astype(np.float64), d[:, ray].T.astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        far = np.where(dd > 0, hi, lo)
        ex = np.where(dd != 0, (far - oo) / dd, np.inf)
        # a zero direction component: inside the slab for every t, or never
        inside = (oo >= lo) & (oo <= hi)
        ex = np.where((dd == 0) & ~inside, -np.inf, ex)
    exit64 = ex.min(axis=1)
    worst = float((exit64 / tmin).max()) if found else 0.0
    assert np.all(exit64 < tmin), f"{int((exit64 >= tmin).sum())} dropped hits with a float64 box exit >= tmin"
    return found, int(acc.value), worst


def test_box_exit_rule_against_float64_on_surface_rays():
    """the one leg of the parity argument that is not
    lockstep.  On ~2M rays leaving mitsuba_synth's surfaces (conftest
    surface_rays: origins on or next to triangle planes, both hemispheres)
    every Woop hit the rule drops has a float64 box exit before tmin, so no
    genuine hit in [tmin, tmax] is dropped (test_gpu_configs runs the same
    audit on config 4's city).  The rule acts on none of those rays here, so
    1M adversarial rays (conftest.edge_leaving_rays: leaving a triangle across
    an edge, nearly in its plane) make the audit non-vacuous."""
    from conftest import edge_leaving_rays, surface_rays
    mesh = scenes.mitsuba_synth(detail=0.25)
    sc = O.OracleScene(mesh, use_bvh=True)
    pos = np.asarray(mesh["pos"], np.float32)
    o, d = surface_rays(lambda o, d: sc.intersect(o, d), pos.min(0), pos.max(0), 2_000_000, seed=23)
    found, accepted, worst = box_exit_audit(mesh["pos"], mesh["pos_tri"], sc, o, d)
    print(f"surface rays {o.shape[1]}: Woop hits {accepted}, dropped by the rule {found} "
          f"(largest float64 exit / tmin among them {worst:.4f})")
    assert o.shape[1] > 500_000 and accepted > 100_000
    o, d = edge_leaving_rays(mesh["pos"], mesh["pos_tri"], 1_000_000, seed=5)
    found2, accepted2, worst2 = box_exit_audit(mesh["pos"], mesh["pos_tri"], sc, o, d)
    print(f"edge-leaving rays {o.shape[1]}: Woop hits {accepted2}, dropped by the rule {found2} "
          f"(largest float64 exit / tmin among them {worst2:.4f})")
    assert found2 > 0  # the rule acts on these, and every drop was before tmin
