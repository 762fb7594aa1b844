"""The pbrt-v3 scene reader (spt_pbrt_load, csrc/pbrt_io.cpp; the reference's
pbrt-parser dependency), on the host: round trips of the
generated scenes through pbrt + PLY, transforms, attribute scopes, object
instances, materials and lights, camera and film, Include, errors.  The
renders of a round-tripped scene are compared with the OBJ-loaded scene's on
the CPU oracle."""
import math
import os

import numpy as np
import pytest

import oracle as O
import sptamd
from sptamd import _lib, scenes


def soup(m):
    """Per-triangle vertex positions and normals (the data the renderer sees)."""
    p = np.asarray(m["pos"], np.float32)[np.asarray(m["pos_tri"]).reshape(-1, 3)]
    nt = np.asarray(m["nrm_tri"]).reshape(-1, 3)
    n = np.asarray(m["nrm"], np.float32)[nt] if len(m["nrm"]) else None
    return p, n


def write(tmp_path, text, name="s.pbrt"):
    path = tmp_path / name
    path.write_text(text)
    return str(path)


@pytest.mark.parametrize("binary", [True, False])
def test_round_trip_mitsuba(tmp_path, binary):
    m = scenes.mitsuba_synth(detail=0.1)
    path = str(tmp_path / "mitsuba.pbrt")
    scenes.write_pbrt(path, m, binary=binary)
    got, info = scenes.load_pbrt(path)
    p0, n0 = soup(m)
    p1, n1 = soup(got)
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(n1, n0)
    np.testing.assert_array_equal(got["mat_id"], m["mat_id"])
    np.testing.assert_array_equal(got["kd"][1:], np.asarray(m["kd"], np.float32)[1:])
    cam = sptamd.reference_camera()
    assert info["camera"] is not None
    np.testing.assert_allclose(info["camera"]["look_from"], cam["look_from"], atol=1e-6)
    fwd = np.subtract(info["camera"]["look_at"], info["camera"]["look_from"])
    ref_fwd = np.subtract(cam["look_at"], cam["look_from"])
    np.testing.assert_allclose(fwd / np.linalg.norm(fwd), ref_fwd / np.linalg.norm(ref_fwd), atol=1e-6)
    assert abs(info["camera"]["fov_y"] - cam["fov_y"]) < 1e-6
    assert (info["xres"], info["yres"]) == (1024, 1024)
    assert info["shapes"] == 1 + int((np.diff(m["mat_id"]) != 0).sum()) and info["shapes_skipped"] == 0


def test_round_trip_renders_equal_on_the_oracle(tmp_path):
    """Same triangles, normals and order: the oracle's image is bit-equal."""
    m = scenes.mitsuba_synth(detail=0.1)
    path = str(tmp_path / "mitsuba.pbrt")
    scenes.write_pbrt(path, m)
    got, _ = scenes.load_pbrt(path)
    p = O.reference_params(32, 24, 4, 4)
    a, _ = O.OracleScene(m).render(p)
    b, _ = O.OracleScene(got).render(p)
    np.testing.assert_array_equal(a, b)


def test_cornell_round_trip_lights(tmp_path):
    m = scenes.cornell_spheres(detail=0.25)
    path = str(tmp_path / "cornell.pbrt")
    scenes.write_pbrt(path, m, camera=scenes.cornell_camera(), width=64, height=48)
    got, info = scenes.load_pbrt(path)
    # emitters survive as emission of their material slots
    ke_in = np.asarray(m["ke"], np.float32)[np.asarray(m["mat_id"])]
    ke_out = got["ke"][got["mat_id"]]
    np.testing.assert_array_equal(ke_out, ke_in)
    kd_in = np.asarray(m["kd"], np.float32)[np.asarray(m["mat_id"])]
    kd_out = got["kd"][got["mat_id"]]
    np.testing.assert_array_equal(kd_out[np.asarray(m["mat_id"]) > 0], kd_in[np.asarray(m["mat_id"]) > 0])
    # landscape film: pbrt's fov is the vertical one
    assert abs(info["camera"]["fov_y"] - scenes.cornell_camera()["fov_y"]) < 1e-6


TRI = '"point P" [0 0 0  1 0 0  0 1 0] "normal N" [0 0 1 0 0 1 0 0 1] "integer indices" [0 1 2]'


def test_transforms_and_scopes(tmp_path):
    path = write(tmp_path, f"""
WorldBegin
AttributeBegin
  Translate 1 2 3
  Scale 2 2 2
  Shape "trianglemesh" {TRI}
AttributeEnd
AttributeBegin
  Rotate 90 0 0 1
  Shape "trianglemesh" {TRI}
AttributeEnd
TransformBegin
  ConcatTransform [1 0 0 0  0 1 0 0  0 0 1 0  5 6 7 1]
  Shape "trianglemesh" {TRI}
TransformEnd
Shape "trianglemesh" {TRI}
WorldEnd
""")
    m, info = scenes.load_pbrt(path)
    p, n = soup(m)
    base = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    np.testing.assert_allclose(p[0], base * 2 + [1, 2, 3], atol=1e-6)
    np.testing.assert_allclose(p[1], [[0, 0, 0], [0, 1, 0], [-1, 0, 0]], atol=1e-6)
    np.testing.assert_allclose(p[2], base + [5, 6, 7], atol=1e-6)
    np.testing.assert_allclose(p[3], base, atol=0)      # scopes restored the identity
    # normals by the inverse transpose (not renormalised): scale 2 -> 0.5
    np.testing.assert_allclose(n[0], [[0, 0, 0.5]] * 3, atol=1e-7)
    assert info["shapes"] == 4 and info["camera"] is None


def test_instances_materials_textures(tmp_path):
    path = write(tmp_path, f"""
Texture "grey" "spectrum" "constant" "rgb value" [0.25 0.5 0.75]
WorldBegin
LightSource "infinite" "rgb L" [0.5 0.5 0.5] "float scale" 2
MakeNamedMaterial "red" "string type" "matte" "rgb Kd" [0.8 0.1 0.1]
MakeNamedMaterial "tex" "string type" "matte" "texture Kd" "grey"
ObjectBegin "tri"
  NamedMaterial "red"
  Shape "trianglemesh" {TRI}
ObjectEnd
AttributeBegin
  Translate 10 0 0
  ObjectInstance "tri"
AttributeEnd
ObjectInstance "tri"
AttributeBegin
  NamedMaterial "tex"
  AreaLightSource "diffuse" "rgb L" [4 4 4]
  Shape "trianglemesh" {TRI}
AttributeEnd
Material "plastic"
Shape "trianglemesh" {TRI}
Shape "sphere" "float radius" 1
""")
    m, info = scenes.load_pbrt(path)
    p, _ = soup(m)
    assert len(p) == 4 and info["instances"] == 2 and info["shapes_skipped"] == 1
    np.testing.assert_allclose(p[0][:, 0], [10, 11, 10])
    np.testing.assert_allclose(p[1][:, 0], [0, 1, 0])
    kd = m["kd"][m["mat_id"]]
    ke = m["ke"][m["mat_id"]]
    np.testing.assert_allclose(kd[0], [0.8, 0.1, 0.1], rtol=1e-6)
    np.testing.assert_allclose(kd[2], [0.25, 0.5, 0.75], rtol=1e-6)
    np.testing.assert_allclose(ke[2], [4, 4, 4])
    np.testing.assert_allclose(kd[3], [0.5, 0.5, 0.5])       # pbrt's default Kd
    assert m["mat_id"][0] == m["mat_id"][1] > 0               # instances share the material
    np.testing.assert_allclose(info["env"], [1, 1, 1])
    assert np.all(m["ke"][0] == 0) and np.all(m["kd"][0] == 1)  # slot 0: the reference default


def test_ply_quads_uv_big_endian_and_include(tmp_path):
    # a quad in a big-endian PLY with uv, fanned into 2 triangles
    hdr = ("ply\nformat binary_big_endian 1.0\ncomment quad\nelement vertex 4\nproperty float x\n"
           "property float y\nproperty float z\nproperty float u\nproperty float v\n"
           "element face 1\nproperty list uchar uint vertex_indices\nend_header\n")
    v = np.array([[0, 0, 0, 0, 0], [1, 0, 0, 1, 0], [1, 1, 0, 1, 1], [0, 1, 0, 0, 1]], ">f4")
    f = np.array([4], ">u1").tobytes() + np.array([0, 1, 2, 3], ">u4").tobytes()
    (tmp_path / "quad.ply").write_bytes(hdr.encode() + v.tobytes() + f)
    write(tmp_path, 'Shape "plymesh" "string filename" "quad.ply"\n', "inc.pbrt")
    path = write(tmp_path, 'LookAt 0 0 5  0 0 0  0 1 0\nCamera "perspective" "float fov" 30\n'
                           'Film "image" "integer xresolution" 200 "integer yresolution" 400\n'
                           'WorldBegin\nInclude "inc.pbrt"\nWorldEnd\n')
    m, info = scenes.load_pbrt(path)
    p, _ = soup(m)
    np.testing.assert_array_equal(p[0], [[0, 0, 0], [1, 0, 0], [1, 1, 0]])
    np.testing.assert_array_equal(p[1], [[0, 0, 0], [1, 1, 0], [0, 1, 0]])
    tc = m["tc"][m["tc_tri"]]
    np.testing.assert_array_equal(tc[1], [[0, 0], [1, 1], [0, 1]])
    assert np.all(m["nrm_tri"] == -1)                          # no normals: geometric fallback
    np.testing.assert_allclose(info["camera"]["look_from"], [0, 0, 5], atol=1e-6)
    np.testing.assert_allclose(info["camera"]["look_at"], [0, 0, 4], atol=1e-6)
    np.testing.assert_allclose(info["camera"]["up"], [0, 1, 0], atol=1e-6)
    # portrait film: the 30-degree fov spans x; vertical = 2 atan(tan 15deg * 2)
    assert abs(info["camera"]["fov_y"] - 2 * math.atan(math.tan(math.radians(15)) * 2)) < 1e-6


@pytest.mark.parametrize("text,code,needle", [
    ("WorldBegin\nFoo 1 2\n", 1, b"s.pbrt:2"),
    ('Shape "trianglemesh" "point P" [0 0 0 1 0 0 0 1 0] "integer indices" [0 1 7]\n', 1, b"out of range"),
    ('Shape "plymesh" "string filename" "missing.ply"\n', 5, b"missing.ply"),
    ('Shape "trianglemesh" "point P" [0 0 0 1 0 0\n', 1, b"unterminated"),
    ('AttributeBegin\nShape "trianglemesh" ' + TRI + '\n', 1, b"AttributeBegin"),
    ('NamedMaterial "nope"\n', 1, b"nope"),
])
def test_errors(tmp_path, text, code, needle):
    path = write(tmp_path, text)
    with pytest.raises(sptamd.SptError) as e:
        scenes.load_pbrt(path)
    assert e.value.code == code
    assert needle.decode() in str(e.value)


def test_missing_file():
    with pytest.raises(sptamd.SptError) as e:
        scenes.load_pbrt("/nonexistent/scene.pbrt")
    assert e.value.code == 5
