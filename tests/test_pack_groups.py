"""CPU check of the packed child-group layout (gpu_build.hip pack_groups, the
host part of gpu_bvh8_holes): the function is compiled on its own with g++
against random octant-slot masks (and edge cases), and every group's slots
must be distinct, slot 0 must stay the root's, the slot count must be one past
the highest slot used, and the density must stay high (the search window)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "smallpt-enoki-optix_amd", "csrc", "gpu_build.hip")

MAIN = r"""
#include <cstdio>
#include <random>
int main(int argc, char** argv) {
    const size_t n = (size_t)atoll(argv[1]);
    const int kind = atoi(argv[2]);
    std::mt19937 rng(7);
    std::vector<uint8_t> m(n);
    size_t occ = 0;
    for (size_t g = 0; g < n; g++) {
        uint8_t x = 0;
        if (kind == 0) { do { x = 0; for (int t = 0; t < 8; t++) if (rng() % 8 < 3) x |= 1u << t; } while (!x); }
        else if (kind == 1) x = 0xff;                 // full groups
        else x = (uint8_t)(1u << (rng() % 8));        // one inner child each
        m[g] = x;
        occ += __builtin_popcount(x);
    }
    std::vector<uint32_t> w;
    const size_t slots = pack_groups(m, w);
    std::vector<uint8_t> used(slots + 16, 0);
    used[0] = 1;
    size_t top = 0;
    for (size_t g = 0; g < n; g++)
        for (int t = 0; t < 8; t++)
            if ((m[g] >> t) & 1) {
                const size_t x = (size_t)w[g] + t;
                if (x == 0 || x >= slots || used[x]) { printf("collision %zu %d\n", g, t); return 1; }
                used[x] = 1;
                if (x > top) top = x;
            }
    if (n && top + 1 != slots) { printf("slots %zu top %zu\n", slots, top); return 1; }
    printf("%zu %zu %zu\n", n, occ, slots);
    return 0;
}
"""


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    src = open(SRC).read()
    m = re.search(r"^constexpr size_t kPackWindow.*?^}\n", src, re.S | re.M)
    assert m, "pack_groups not found in gpu_build.hip"
    d = tmp_path_factory.mktemp("pack")
    cpp = d / "pack.cpp"
    cpp.write_text("#include <algorithm>\n#include <cstdint>\n#include <cstdlib>\n#include <vector>\n"
                   + m.group(0) + MAIN)
    exe = d / "pack"
    subprocess.run([gxx, "-O2", "-std=c++17", "-o", str(exe), str(cpp)], check=True)
    return exe


@pytest.mark.parametrize("n,kind,min_density", [(0, 0, 0.0), (1, 0, 0.0), (1000, 0, 0.9), (200000, 0, 0.93),
                                                (5000, 1, 0.99), (50000, 2, 0.95)])
def test_pack_groups(checker, n, kind, min_density):
    out = subprocess.run([str(checker), str(n), str(kind)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout
    groups, occ, slots = map(int, out.stdout.split())
    assert groups == n
    if n:
        assert occ / slots >= min_density
