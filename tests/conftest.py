import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "smallpt-enoki-optix_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libspt.so on cuda:0)")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def assert_work_complete(st, rows, width, spp):
    """spt_render_stats' device-counted work (include/spt.h): every (sample,
    pixel) of the tile started, ended and wrote its film slot exactly once —
    the reference renders every pixel x sample (main.cpp:385-429)."""
    want = rows * width * spp
    assert st["paths_started"] == want, (st["paths_started"], want)
    assert st["paths_terminated"] == want, (st["paths_terminated"], want)
    assert st["film_slots_unwritten"] == 0, st["film_slots_unwritten"]
    assert st["paths"] == want
    assert want == 0 or st["work_order"] in (1, 2)


def spaced_rows(height, n):
    """n evenly spaced rows of [0, height) (first and last included)."""
    import numpy as np
    return np.unique(np.linspace(0, height - 1, n).round().astype(np.int32))
