// FETCH_SIZE calibration for the traversal's access pattern:
// random 64-B half-line gathers (a node visit: 4 x 16 B of one 64-B node; a
// triangle record: 64 B) over a table far larger than the Infinity Cache, so
// every gather misses to HBM, with a known byte count.  rocprofv3's FETCH_SIZE
// per dispatch divided by the true bytes is the factor DESIGN.md §5 and
// bench.py apply to the drain's config-4 traffic; MI355X_MICROARCH.md measured
// x2 only for wide coalesced streaming reads.
//
// Variants (one dispatch each, named by the kernel):
//   stream16  coalesced 16 B per lane, consecutive (the guide's calibrated case)
//   half64    one random 64-B half line per lane (4 x dwordx4)
//   full128   one random 128-B line per lane (8 x dwordx4)
//   tri60     one random 64-B record read as the triangle test does (3 x dwordx3 at 20-B strides)
//   quad16    one random 16 B per lane (a single dwordx4)
//
//   hipcc --offload-arch=gfx950 -O3 -o build/micro_fetch tools/micro_fetch.hip
//   rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- ./build/micro_fetch
// prints one JSON line per variant with its true bytes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

constexpr int kIters = 64;

__global__ __launch_bounds__(256) void stream16(const float4* __restrict__ t, size_t n, float4* __restrict__ out) {
    float4 acc = make_float4(0, 0, 0, 0);
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const float4 v = t[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (acc.x == 1234.5f) out[0] = acc;
}

template <int kQuads, int kOff>
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ t, uint32_t lines_mask, float4* __restrict__ out) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    float4 acc = make_float4(0, 0, 0, 0);
    uint32_t seed = hash(gid * 2654435761u + 1u);
    for (int it = 0; it < kIters; it++) {
        seed = hash(seed + (uint32_t)it);
        const uint32_t line = seed & lines_mask;
        const uint32_t half = kOff ? (seed >> 31) * 4u : 0u;  // which 64-B half
        const float4* p = t + (size_t)line * 8u + half;
        float4 v[kQuads];
#pragma unroll
        for (int j = 0; j < kQuads; j++) v[j] = p[j];
#pragma unroll
        for (int j = 0; j < kQuads; j++) { acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w; }
    }
    if (acc.x == 1234.5f) out[0] = acc;
}

// the triangle test's loads: floats 0-2, 5-7, 10-12 of a random 64-B record (as dwordx3)
__global__ __launch_bounds__(256) void tri60(const float* __restrict__ t, uint32_t recs_mask, float4* __restrict__ out) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    float acc = 0.0f;
    uint32_t seed = hash(gid * 2654435761u + 7u);
    for (int it = 0; it < kIters; it++) {
        seed = hash(seed + (uint32_t)it);
        const float* f = t + (size_t)(seed & recs_mask) * 16u;
        const float3 a = *(const float3*)(f), b = *(const float3*)(f + 5), c = *(const float3*)(f + 10);
        acc += a.x + a.y + a.z + b.x + b.y + b.z + c.x + c.y + c.z;
    }
    if (acc == 1234.5f) out[0] = make_float4(acc, 0, 0, 0);
}

int main() {
    const size_t kLines = (size_t)1 << 25;  // 2^25 128-B lines = 4 GiB: 16x the Infinity Cache
    float4 *d_t, *d_o;
    CHECK(hipMalloc(&d_t, kLines * 128));
    CHECK(hipMalloc(&d_o, sizeof(float4)));
    CHECK(hipMemset(d_t, 0, kLines * 128));
    const uint32_t blocks = 256 * 32, lanes = blocks * 256;
    const uint32_t mask = (uint32_t)(kLines - 1);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto report = [&](const char* name, double bytes) -> int {
        float ms = 0;
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"%s\", \"true_bytes\": %.0f, \"ms\": %.3f, \"GB_s\": %.1f}\n", name, bytes, ms,
                    bytes / (ms * 1e-3) / 1e9);
        return 0;
    };
    // streaming: 1 GiB, once
    const size_t n16 = (size_t)1 << 26;  // float4s = 1 GiB
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(stream16, dim3(blocks), dim3(256), 0, 0, d_t, n16, d_o);
    CHECK(hipEventRecord(e1));
    if (report("stream16", (double)n16 * 16)) return 1;
    const double g = (double)lanes * kIters;  // gathers
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((gather<4, 1>), dim3(blocks), dim3(256), 0, 0, d_t, mask, d_o);
    CHECK(hipEventRecord(e1));
    if (report("gather<4, 1> half64", g * 64)) return 1;
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((gather<8, 0>), dim3(blocks), dim3(256), 0, 0, d_t, mask, d_o);
    CHECK(hipEventRecord(e1));
    if (report("gather<8, 0> full128", g * 128)) return 1;
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((gather<1, 1>), dim3(blocks), dim3(256), 0, 0, d_t, mask, d_o);
    CHECK(hipEventRecord(e1));
    if (report("gather<1, 1> quad16", g * 16)) return 1;
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(tri60, dim3(blocks), dim3(256), 0, 0, (const float*)d_t, (uint32_t)(kLines * 2 - 1), d_o);
    CHECK(hipEventRecord(e1));
    if (report("tri60 (64-B records, 3 x 12 B used)", g * 64)) return 1;
    return 0;
}
