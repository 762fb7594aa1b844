"""CPU check of the packed child-group layout (gpu_build.hip pack_groups, the
host part of gpu_bvh8_holes): the function is compiled on its own with g++
against random octant-slot masks (and edge cases), and every group's slots
must be distinct, slot 0 must stay the root's, the slot count must be one past
the highest slot used, and the density must stay high (the search window).
depth_first_groups (spt_config.pack_groups 2) is compiled the same way over
random compact trees: its order must be a permutation of the groups with every
group after its parent's and a subtree's groups contiguous."""
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


DFS_MAIN = r"""
#include <cstdio>
#include <random>
// random compact tree, level by level like the GPU builder: node i's inner
// children are nodes first .. first + popcount(imask) - 1
int main(int argc, char** argv) {
    const uint32_t want = (uint32_t)atoi(argv[1]);
    std::mt19937 rng(atoi(argv[2]));
    std::vector<uint32_t> w34{0u, 0u};
    std::vector<uint32_t> level{0u};
    uint32_t n = 1;
    while (!level.empty() && n < want) {
        std::vector<uint32_t> next;
        for (uint32_t i : level) {
            uint32_t m = 0;
            for (int t = 0; t < 8 && n + __builtin_popcount(m) < want; t++) if (rng() % 3 == 0) m |= 1u << t;
            if (!m) continue;
            w34[2 * i] = m << 24;
            w34[2 * i + 1] = n;
            for (int c = 0; c < __builtin_popcount(m); c++) { next.push_back(n); w34.push_back(0u); w34.push_back(0u); n++; }
        }
        level.swap(next);
    }
    uint32_t groups = 0;
    std::vector<uint32_t> gid(n, UINT32_MAX), parent_group(n, UINT32_MAX);
    for (uint32_t i = 0; i < n; i++) if (w34[2 * i] >> 24) gid[i] = groups++;
    for (uint32_t i = 0; i < n; i++)
        if (gid[i] != UINT32_MAX)
            for (int c = 0; c < __builtin_popcount(w34[2 * i] >> 24); c++) parent_group[w34[2 * i + 1] + c] = gid[i];
    const std::vector<uint32_t> order = depth_first_groups(w34, n, groups);
    if (order.size() != groups) { printf("size %zu %u\n", order.size(), groups); return 1; }
    std::vector<int64_t> pos(groups, -1);
    for (size_t k = 0; k < order.size(); k++) {
        if (order[k] >= groups || pos[order[k]] >= 0) { printf("not a permutation\n"); return 1; }
        pos[order[k]] = (int64_t)k;
    }
    // every group after the group holding its node (the group of the node's parent)
    std::vector<uint32_t> owner(n, UINT32_MAX), span(groups, 1);
    for (uint32_t i = 0; i < n; i++)
        if (gid[i] != UINT32_MAX && parent_group[i] != UINT32_MAX && pos[gid[i]] <= pos[parent_group[i]]) {
            printf("group %u before its parent's\n", gid[i]); return 1;
        }
    // subtree contiguity: the groups below a node occupy one run of the order
    for (uint32_t i = n; i-- > 0;)
        if (gid[i] != UINT32_MAX)
            for (int c = 0; c < __builtin_popcount(w34[2 * i] >> 24); c++) {
                const uint32_t ch = w34[2 * i + 1] + c;
                if (gid[ch] != UINT32_MAX) span[gid[i]] += span[gid[ch]];
            }
    for (uint32_t i = 0; i < n; i++)
        if (gid[i] != UINT32_MAX) {
            const int64_t p = pos[gid[i]];
            for (int c = 0; c < __builtin_popcount(w34[2 * i] >> 24); c++) {
                const uint32_t ch = w34[2 * i + 1] + c;
                if (gid[ch] != UINT32_MAX && (pos[gid[ch]] <= p || pos[gid[ch]] + span[gid[ch]] > p + span[gid[i]])) {
                    printf("subtree of group %u not contiguous\n", gid[i]); return 1;
                }
            }
        }
    printf("%u %u\n", n, groups);
    return 0;
}
"""


@pytest.fixture(scope="module")
def dfs_checker(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    src = open(SRC).read()
    m = re.search(r"^static std::vector<uint32_t> depth_first_groups.*?^}\n", src, re.S | re.M)
    assert m, "depth_first_groups not found in gpu_build.hip"
    d = tmp_path_factory.mktemp("dfs")
    cpp = d / "dfs.cpp"
    cpp.write_text("#include <cstdint>\n#include <cstdlib>\n#include <vector>\n" + m.group(0) + DFS_MAIN)
    exe = d / "dfs"
    subprocess.run([gxx, "-O2", "-std=c++17", "-o", str(exe), str(cpp)], check=True)
    return exe


@pytest.mark.parametrize("nodes,seed", [(1, 1), (9, 2), (1000, 3), (200000, 4)])
def test_depth_first_groups(dfs_checker, nodes, seed):
    out = subprocess.run([str(dfs_checker), str(nodes), str(seed)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout
    n, groups = map(int, out.stdout.split())
    assert n >= 1 and (groups >= 1 or n == 1)


@pytest.mark.parametrize("n,kind,min_density", [(0, 0, 0.0), (1, 0, 0.0), (1000, 0, 0.9), (200000, 0, 0.93),
                                                (5000, 1, 0.99), (50000, 2, 0.95)])
def test_pack_groups(checker, n, kind, min_density):
    out = subprocess.run([str(checker), str(n), str(kind)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout
    groups, occ, slots = map(int, out.stdout.split())
    assert groups == n
    if n:
        assert occ / slots >= min_density
