"""The binary scene cache format (include/spt.h spt_scene_save / _load /
_cache_info) checked on the CPU: files written here by an independent
restatement of the documented layout (header, section order, the four-lane
section checksum) are accepted by spt_scene_cache_info and pass
spt_scene_load's checks up to the device; every kind of damage — a flipped
byte in any section, another version or layout, inconsistent sizes, a
truncated or over-long file — is refused with SPT_ERR_INVALID, a missing file
with SPT_ERR_IO.  The GPU round trips are tests/test_gpu_scene_cache.py."""
import ctypes
from ctypes import c_char, c_uint32, c_uint64

import numpy as np
import pytest

import sptamd
from sptamd import _lib

SECTIONS = ["nodes", "triangles", "normals", "texcoords", "orig2slot", "albedo", "emission", "spheres",
            "sphere materials", "material kinds", "texture sizes", "texels", "extra"]
TRI_QUADS, NODE6_QUADS = 4, 4   # spt_internal.h kTriQuads / kNode6Quads
CACHE_VERSION = 2               # capi.cpp kCacheVersion (2: 64-B rotated triangle records)


def tri_records(v9, ids):
    """spt_internal.h tri_record_fill: per triangle 16 floats, each vertex as
    x y z x y, the original id's bits in float 15."""
    v = np.asarray(v9, np.float32).reshape(-1, 3, 3)
    rec = np.zeros((v.shape[0], 16), np.float32)
    for k in range(3):
        rec[:, 5 * k:5 * k + 3] = v[:, k]
        rec[:, 5 * k + 3:5 * k + 5] = v[:, k, :2]
    rec[:, 15] = np.asarray(ids, np.uint32).view(np.float32)
    return rec


class Header(ctypes.Structure):
    _fields_ = ([("magic", c_char * 8)] +
                [(n, c_uint32) for n in ("version", "header_bytes", "tri_quads", "node_quads", "node6",
                                         "group_shift", "config_bytes", "stats_bytes", "stack_depth", "nmat",
                                         "nemit", "nsph", "nkind", "ntexmat")] +
                [("ntri", c_uint64), ("bytes", c_uint64 * 13), ("sum", c_uint64 * 13),
                 ("cfg", _lib.Config), ("stats", _lib.SceneStats)])


M, MASK = 0x9FB21C651E98DF25, (1 << 64) - 1


def cache_sum(data: bytes) -> int:
    h = [0x243F6A8885A308D3, 0x13198A2E03707344, 0xA4093822299F31D0, 0x082EFA98EC4E6C89]
    padded = data + b"\0" * (32 - len(data) % 32)     # the tail block (all zero when len % 32 == 0)
    words = np.frombuffer(padded, "<u8").tolist()
    for i in range(0, len(words), 4):
        for k in range(4):
            x = ((h[k] ^ words[i + k]) * M) & MASK
            h[k] = x ^ (x >> 31)
    r = len(data)
    for k in range(4):
        r = ((r ^ h[k]) * M) & MASK
        r ^= r >> 29
    return r


def sections():
    """A two-triangle six-wide scene with one 2 x 2 texture and extra bytes."""
    rng = np.random.default_rng(0)
    node = np.zeros(NODE6_QUADS * 4, np.uint32)
    tris = tri_records(rng.normal(size=(2, 9)), [1, 0])
    snrm = rng.normal(size=(2 * 3, 4)).astype(np.float32)
    return [node.tobytes(), tris.tobytes(), snrm.tobytes(), b"", np.array([1, 0], np.int32).tobytes(),
            np.full(3, 0.5, np.float32).tobytes(), b"", b"", b"", b"",
            np.array([2, 2], np.uint32).tobytes(), np.ones((4, 4), np.float32).tobytes(), b"camera"]


def header(secs, **over):
    h = Header()
    h.magic = b"SPTSCENE"
    h.version, h.header_bytes = CACHE_VERSION, ctypes.sizeof(Header)
    h.tri_quads, h.node_quads, h.node6, h.group_shift = TRI_QUADS, NODE6_QUADS, 1, 0
    h.config_bytes, h.stats_bytes = ctypes.sizeof(_lib.Config), ctypes.sizeof(_lib.SceneStats)
    h.stack_depth, h.nmat, h.nemit, h.nsph, h.nkind, h.ntexmat = 1, 1, 0, 0, 0, 1
    h.ntri = 2
    h.cfg = sptamd.default_config()
    h.stats.ntri, h.stats.nodes, h.stats.leaves, h.stats.bvh_width = 2, 1, 1, 6
    h.stats.max_depth, h.stats.max_leaf, h.stats.builder = 1, 3, _lib.SPT_BUILD_HOST_SAH
    for i, s in enumerate(secs):
        h.bytes[i] = len(s)
        h.sum[i] = cache_sum(s)
    for k, v in over.items():
        setattr(h, k, v)
    return h


def write(path, h, secs, tail=b""):
    with open(path, "wb") as f:
        f.write(bytes(h))
        for s in secs:
            f.write(s)
        f.write(tail)
    return str(path)


def info_status(path):
    st, cfg, n = _lib.SceneStats(), _lib.Config(), ctypes.c_uint64()
    code = _lib.lib.spt_scene_cache_info(str(path).encode(), ctypes.byref(st), ctypes.byref(cfg), ctypes.byref(n))
    return code, st, cfg, n.value


def test_checksum_restatement():
    """Properties of the restatement; test_well_formed_file_accepted pins it to the library's."""
    assert cache_sum(b"") == cache_sum(b"")
    assert cache_sum(b"\0" * 32) != cache_sum(b"")           # the length is folded in
    assert cache_sum(b"a" * 31) != cache_sum(b"a" * 31 + b"\0")


def test_well_formed_file_accepted(tmp_path):
    secs = sections()
    p = write(tmp_path / "ok.sptc", header(secs), secs)
    code, st, cfg, n = info_status(p)
    assert code == _lib.SPT_OK, _lib.lib.spt_last_error()
    assert st.ntri == 2 and st.bvh_width == 6 and n == len(b"camera")
    assert bytes(cfg) == bytes(sptamd.default_config())
    # spt_scene_load checks the same file and stops at the device (none here)
    out, m = ctypes.c_void_p(), ctypes.c_uint64()
    buf = ctypes.create_string_buffer(16)
    code = _lib.lib.spt_scene_load(p.encode(), ctypes.byref(out), buf, 16, ctypes.byref(m))
    if code == _lib.SPT_OK:       # a GPU is visible: the scene loaded
        assert buf.raw[:6] == b"camera" and m.value == 6
        _lib.lib.spt_scene_destroy(out)
    else:
        assert code == _lib.SPT_ERR_NO_DEVICE, _lib.lib.spt_last_error()


@pytest.mark.parametrize("sec", range(13))
def test_flipped_byte_refused(tmp_path, sec):
    secs = sections()
    if not secs[sec]:
        pytest.skip(f"section {SECTIONS[sec]} is empty in this file")
    h = header(secs)
    bad = list(secs)
    b = bytearray(bad[sec])
    b[len(b) // 2] ^= 0x10
    bad[sec] = bytes(b)
    code, *_ = info_status(write(tmp_path / "bad.sptc", h, bad))
    assert code == _lib.SPT_ERR_INVALID
    msg = _lib.lib.spt_last_error().decode()
    assert "checksum" in msg and SECTIONS[sec] in msg


@pytest.mark.parametrize("over", [dict(version=1), dict(tri_quads=3), dict(node_quads=8), dict(node6=0),
                                  dict(group_shift=1), dict(nmat=2), dict(ntri=3), dict(nsph=300),
                                  dict(stack_depth=0), dict(config_bytes=4)])
def test_header_mismatch_refused(tmp_path, over):
    secs = sections()
    code, *_ = info_status(write(tmp_path / "h.sptc", header(secs, **over), secs))
    assert code == _lib.SPT_ERR_INVALID


def test_sizes_and_length_refused(tmp_path):
    secs = sections()
    h = header(secs)
    assert info_status(write(tmp_path / "long.sptc", h, secs, tail=b"x"))[0] == _lib.SPT_ERR_INVALID
    p = write(tmp_path / "short.sptc", h, secs)
    data = open(p, "rb").read()
    for cut in (1, len(data) - ctypes.sizeof(Header), len(data) - 5):
        with open(p, "wb") as f:
            f.write(data[:cut])
        assert info_status(p)[0] == _lib.SPT_ERR_INVALID, cut
    # texture sizes that disagree with the texel section (checksums consistent)
    bad = list(secs)
    bad[10] = np.array([3, 2], np.uint32).tobytes()
    assert info_status(write(tmp_path / "tex.sptc", header(bad), bad))[0] == _lib.SPT_ERR_INVALID
    # a node section that is not whole nodes
    bad = list(secs)
    bad[0] = secs[0] + b"\0" * 16
    assert info_status(write(tmp_path / "node.sptc", header(bad), bad))[0] == _lib.SPT_ERR_INVALID
    # an unknown config value (load re-checks the saved spt_config)
    h = header(secs)
    h.cfg.streams = 99
    out = ctypes.c_void_p()
    p = write(tmp_path / "cfg.sptc", h, secs)
    assert _lib.lib.spt_scene_load(p.encode(), ctypes.byref(out), None, 0, None) == _lib.SPT_ERR_INVALID


def test_missing_and_null(tmp_path):
    assert info_status(tmp_path / "none.sptc")[0] == _lib.SPT_ERR_IO
    assert _lib.lib.spt_scene_cache_info(None, None, None, None) == _lib.SPT_ERR_INVALID
    out = ctypes.c_void_p()
    assert _lib.lib.spt_scene_load(None, ctypes.byref(out), None, 0, None) == _lib.SPT_ERR_INVALID
    assert _lib.lib.spt_scene_save(None, b"x", None, 0) == _lib.SPT_ERR_INVALID
    p = write(tmp_path / "junk.sptc", header(sections()), [])
    assert info_status(p)[0] == _lib.SPT_ERR_INVALID
