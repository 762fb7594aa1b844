// Microbenchmark: cost of a 16-B-per-lane gather (global_load_dwordx4) by the
// number of distinct cache lines one wave-instruction touches, from an
// L2-resident table, next to the same gather from LDS (ds_read_b128).  Answers
// whether traversal's coherent top-level node fetches cost the vector-memory
// data path as much as its divergent deep ones ("what bounds
// isect").
//
//   hipcc --offload-arch=gfx950 -O3 -o build/micro_gather tools/micro_gather.hip
//   ./build/micro_gather
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// distinct = addresses per wave-instruction: lane l reads entry key(l % distinct);
// entries are 128-B lines (8 float4), a lane takes float4 (l / distinct) % 8 of it.
template <bool kLds>
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ table, uint32_t lines_mask,
                                              uint32_t distinct, int iters, float4* __restrict__ out) {
    extern __shared__ float4 lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (kLds) {
        for (uint32_t k = threadIdx.x; k <= lines_mask * 8u + 7u; k += blockDim.x) lds[k] = table[k];
        __syncthreads();
    }
    const uint32_t sub = (lane / distinct) & 7u;
    float4 acc = make_float4(0, 0, 0, 0);
    uint32_t seed = hash(wave * 9781u + 17u);
    for (int it = 0; it < iters; it++) {
        float4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t line = hash(seed + (lane % distinct) * 131u + j * 7919u) & lines_mask;
            const uint32_t k = line * 8u + sub;
            v[j] = kLds ? lds[k] : table[k];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w;
        }
        seed = hash(seed + (uint32_t)it + __float_as_uint(acc.x) * 0u);
    }
    if (acc.x == 1234.5f) out[0] = acc;  // keep the loads
}

// kq quads per lane from the lane's own random 128-B line (a node fetch):
// is the cost per wave-instruction or per line?
template <int kq>
__global__ __launch_bounds__(256) void node_fetch(const float4* __restrict__ table, uint32_t lines_mask, int iters,
                                                  float4* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    float4 acc = make_float4(0, 0, 0, 0);
    uint32_t seed = hash(wave * 9781u + 17u);
    for (int it = 0; it < iters; it++) {
        const uint32_t line = hash(seed + lane * 131u) & lines_mask;
        const float4* p = table + line * 8u;
        float4 v[kq];
#pragma unroll
        for (int j = 0; j < kq; j++) v[j] = p[j];
#pragma unroll
        for (int j = 0; j < kq; j++) { acc.x += v[j].x; acc.y += v[j].y; acc.z += v[j].z; acc.w += v[j].w; }
        seed = hash(seed + (uint32_t)it);
    }
    if (acc.x == 1234.5f) out[0] = acc;
}

template <int kq>
static int time_node(const float4* d_t, uint32_t mask, float4* d_o, hipEvent_t e0, hipEvent_t e1) {
    const int iters = 256, blocks = 256 * 8;
    for (int rep = 0; rep < 2; rep++) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(node_fetch<kq>, dim3(blocks), dim3(256), 0, 0, d_t, mask, iters, d_o);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double fetches = (double)blocks * 4 * iters;  // wave-level node fetches
        if (rep)
            std::printf("{\"node_quads\": %d, \"table_lines\": %u, \"ms\": %.3f, \"ns_per_fetch_per_cu\": %.2f, "
                        "\"ns_per_inst_per_cu\": %.2f}\n", kq, mask + 1, ms, ms * 1e6 / (fetches / 256.0),
                        ms * 1e6 / (fetches * kq / 256.0));
    }
    return 0;
}

int main() {
    const uint32_t kLines = 16384;  // 2 MiB table, L2-resident
    std::vector<float4> h(kLines * 8);
    for (size_t i = 0; i < h.size(); i++) h[i] = make_float4(1e-9f * i, 0, 0, 0);
    float4 *d_t, *d_o;
    CHECK(hipMalloc(&d_t, h.size() * sizeof(float4)));
    CHECK(hipMalloc(&d_o, sizeof(float4)));
    CHECK(hipMemcpy(d_t, h.data(), h.size() * sizeof(float4), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int iters = 256, blocks = 256 * 8;
    for (int lds = 0; lds < 2; lds++) {
        // the LDS variant gathers from a 6-KiB image (48 lines): the top of a BVH8
        const uint32_t mask = lds ? 31u : kLines - 1u;
        const size_t shm = lds ? (mask + 1) * 8 * sizeof(float4) : 0;
        for (uint32_t distinct : {1u, 2u, 8u, 16u, 32u, 64u}) {
            for (int rep = 0; rep < 2; rep++) {
                CHECK(hipEventRecord(e0));
                if (lds)
                    hipLaunchKernelGGL(gather<true>, dim3(blocks), dim3(256), shm, 0, d_t, mask, distinct, iters, d_o);
                else
                    hipLaunchKernelGGL(gather<false>, dim3(blocks), dim3(256), 0, 0, d_t, mask, distinct, iters, d_o);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double insts = (double)blocks * 4 * iters * 4;  // wave-instructions
                if (rep)
                    std::printf("{\"src\": \"%s\", \"distinct\": %u, \"ms\": %.3f, \"lane_TB_s\": %.2f, "
                                "\"ns_per_inst_per_cu\": %.2f}\n",
                                lds ? "lds" : "l2", distinct, ms, insts * 1024.0 / (ms * 1e-3) / 1e12,
                                ms * 1e6 / (insts / 256.0));
            }
        }
    }
    // node fetches: L2-resident (2 MiB) and beyond L2 (256 MiB, like the 26-MB scene x lines)
    const uint32_t big = 1u << 21;  // 2M lines = 256 MiB
    float4* d_big;
    CHECK(hipMalloc(&d_big, (size_t)big * 8 * sizeof(float4)));
    CHECK(hipMemset(d_big, 0, (size_t)big * 8 * sizeof(float4)));
    for (uint32_t mask : {kLines - 1u, big - 1u}) {
        const float4* t = mask == kLines - 1u ? d_t : d_big;
        if (time_node<1>(t, mask, d_o, e0, e1) || time_node<2>(t, mask, d_o, e0, e1) ||
            time_node<3>(t, mask, d_o, e0, e1) || time_node<4>(t, mask, d_o, e0, e1) ||
            time_node<5>(t, mask, d_o, e0, e1) || time_node<8>(t, mask, d_o, e0, e1))
            return 1;
    }
    return 0;
}
