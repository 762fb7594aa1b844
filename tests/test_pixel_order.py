"""CPU check of the camera-path pixel order (spt_internal.h work_pixel, used by
refill_kernel and render_fused_kernel): the function is compiled on its own
with g++, and for every tile shape and block size the q -> (x, y) map must
visit every pixel of the tile exactly once (the image cannot depend on the
order), stay scanline for B <= 1, and keep each aligned run of B*B work items
of a full block inside one B x B footprint."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "smallpt-enoki-optix_amd", "csrc", "spt_internal.h")
MATH_SRC = os.path.join(ROOT, "smallpt-enoki-optix_amd", "csrc", "spt_math.h")

MAIN = r"""
#include <cstdio>
int main(int argc, char** argv) {
    const uint32_t W = atoi(argv[1]), H = atoi(argv[2]), B = atoi(argv[3]);
    const uint32_t P = W * H;
    std::vector<uint8_t> seen(P, 0);
    std::vector<uint32_t> xs(P), ys(P);
    for (uint32_t q = 0; q < P; q++) {
        uint32_t x, y;
        work_pixel(q, W, P, B, x, y);
        if (x >= W || y >= H) { printf("out of range q=%u (%u, %u)\n", q, x, y); return 1; }
        if (seen[y * W + x]++) { printf("twice q=%u (%u, %u)\n", q, x, y); return 1; }
        if (B <= 1 && (x != q % W || y != q / W)) { printf("not scanline q=%u\n", q); return 1; }
        xs[q] = x; ys[q] = y;
    }
    // full blocks: B*B consecutive items starting at a band's block boundary
    // share one B x B footprint
    unsigned full = 0;
    if (B > 1)
        for (uint32_t band = 0; (band + 1) * B <= H; band++)
            for (uint32_t cb = 0; (cb + 1) * B <= W; cb++) {
                const uint32_t q0 = band * B * W + cb * B * B;
                for (uint32_t i = 0; i < B * B; i++) {
                    const uint32_t x = xs[q0 + i], y = ys[q0 + i];
                    if (x / B != cb || y / B != band) { printf("block %u,%u item %u at (%u, %u)\n", cb, band, i, x, y); return 1; }
                }
                full++;
            }
    printf("%u %u\n", P, full);
    return 0;
}
"""


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    src = open(SRC).read()
    m = re.search(r"^SPT_HD void work_pixel\(.*?^}\n", src, re.S | re.M)
    assert m, "work_pixel not found in spt_internal.h"
    # its division helper (a shift for power-of-two widths), from spt_math.h
    u = re.search(r"^SPT_HD uint32_t udiv\(.*?^}\n", open(MATH_SRC).read(), re.S | re.M)
    assert u, "udiv not found in spt_math.h"
    d = tmp_path_factory.mktemp("pixorder")
    cpp = d / "pixorder.cpp"
    cpp.write_text("#include <cstdint>\n#include <cstdlib>\n#include <vector>\n#define SPT_HD static inline\n"
                   + u.group(0) + m.group(0) + MAIN)
    exe = d / "pixorder"
    subprocess.run([gxx, "-O2", "-std=c++17", "-o", str(exe), str(cpp)], check=True)
    return exe


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (64, 48), (1024, 128), (1920, 135), (37, 1), (1, 29), (13, 17)])
@pytest.mark.parametrize("b", [0, 1, 2, 3, 8, 16, 64])
def test_work_pixel_bijection(checker, w, h, b):
    out = subprocess.run([str(checker), str(w), str(h), str(b)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout
    p, full = map(int, out.stdout.split())
    assert p == w * h
    if b > 1:
        assert full == (w // b) * (h // b)
