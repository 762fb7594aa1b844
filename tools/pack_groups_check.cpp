// CPU check of gpu_build.hip's pack_groups (copied in by sed, see below):
// random octant masks, no slot used twice, slot 0 left to the root, density
// and time.   sed -n '/^constexpr size_t kPackWindow/,/^}/p' smallpt-enoki-optix_amd/csrc/gpu_build.hip
#include <vector>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <chrono>
#include <random>
constexpr size_t kPackWindow = 64;
static size_t pack_groups(const std::vector<uint8_t>& gmask, std::vector<uint32_t>& gword) {
    std::vector<uint64_t> used(2, 0u);
    used[0] = 1u;  // slot 0: the root
    const auto window = [&](size_t x) -> uint32_t {  // used bits of slots x .. x + 7
        const size_t w = x / 64, o = x % 64;
        uint64_t v = used[w] >> o;
        if (o) v |= used[w + 1] << (64 - o);
        return (uint32_t)(v & 0xffu);
    };
    size_t lo = 1, end = 1;
    gword.resize(gmask.size());
    for (size_t g = 0; g < gmask.size(); g++) {
        const uint32_t m = gmask[g];
        if (end > lo + kPackWindow) lo = end - kPackWindow;  // give up the old holes
        while (window(lo) & 1u) lo++;
        const size_t c = (size_t)__builtin_ctz(m | 0x100u);
        size_t b = lo > c ? lo - c : 1;
        while (window(b) & m) b++;
        if (b + 8 >= (1u << 24)) return 0;
        gword[g] = (uint32_t)b;
        if ((b + 8) / 64 + 2 > used.size()) used.resize((b + 8) / 64 + 2, 0u);
        const size_t w = b / 64, o = b % 64;
        used[w] |= (uint64_t)m << o;
        if (o > 56) used[w + 1] |= (uint64_t)m >> (64 - o);
        end = std::max(end, b + 8 - (size_t)__builtin_clz(m) + 24);  // one past the highest occupied slot
    }
    return end;
}
int main() {
    std::mt19937 rng(1);
    for (size_t n : {1ul, 30000ul, 500000ul, 2000000ul}) {
        std::vector<uint8_t> m(n);
        size_t occ = 0;
        for (auto& x : m) { do { x = 0; for (int t = 0; t < 8; t++) if (rng() % 8 < 3) x |= 1u << t; } while (!x); occ += __builtin_popcount(x); }
        std::vector<uint32_t> w;
        auto t0 = std::chrono::steady_clock::now();
        size_t slots = pack_groups(m, w);
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::vector<uint8_t> u(slots + 16, 0); bool ok = true; size_t mx = 0;
        u[0] = 1;
        for (size_t g = 0; g < n; g++) for (int t = 0; t < 8; t++) if ((m[g] >> t) & 1) { if (w[g] + t == 0 || u[w[g] + t]) ok = false; u[w[g] + t] = 1; mx = std::max<size_t>(mx, w[g] + t); }
        printf("groups %zu occupied %zu slots %zu maxslot+1 %zu (density %.3f) %.1f ms ok=%d\n", n, occ, slots, mx + 1, (double)occ / slots, ms, ok && mx + 1 == slots);
    }
}
