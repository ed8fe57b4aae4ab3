// Does prefetching the next round's inputs overlap stage 0's HBM reads with
// its search?  A stage-0-shaped kernel (diagnostic for compact.hip):
// 16384 workgroups of one wavefront with 10 KB of LDS (4 per SIMD), each
// staging its group's 17 KB (16-B loads, XOR-folded into LDS), then a
// dependent VALU chain standing in for the search (`spin` iterations), then
// one store per lane.  With `dist` > 0, before the chain a wavefront touches
// group g + dist's bytes with one 4-B LDS-DMA load per 128-B line
// (global_load_lds_dword into a 256-B row no one reads), so that group's
// staging finds them in L2 / the Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 prefetch_overlap.hip -o prefetch_overlap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr uint32_t LDS_WORDS = 2560;   // 10 KB

__global__ void k_flush(const uint4* __restrict__ p, size_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) acc ^= p[i].x;
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(64) void k_sim(const uint4* __restrict__ src, uint32_t* __restrict__ out,
                                            uint32_t words, uint32_t spin, uint32_t dist, int stage) {
    __shared__ uint32_t s[LDS_WORDS];
    const uint32_t lane = threadIdx.x, g = blockIdx.x;
    const uint64_t base = (uint64_t)g * words;
    uint32_t acc = 0;
    for (uint32_t k = 0; k < (stage ? words : 0u); k += 256u) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = k + u * 64u + lane;
            v[u] = i < words ? src[base + i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        s[(k / 64u) % 32u * 64u + lane] = acc;
    }
    if (dist && g + dist < gridDim.x) {
        // one dword per 128-B line: 64 lanes cover 8 KB per instruction
        const char* p = (const char*)(src + (uint64_t)(g + dist) * words);
        const uint32_t bytes = words * 16u;
        for (uint32_t off = 0; off < bytes; off += 8192u) {
            const uint32_t o = off + lane * 128u;
            const char* q = p + (o < bytes ? o : 0u);
            __builtin_amdgcn_global_load_lds((const void*)q, (void __attribute__((address_space(3)))*)&s[LDS_WORDS - 64], 4, 0, 0);
        }
    }
    // the search stand-in: a dependent chain
    uint32_t x = acc | 1u;
    for (uint32_t i = 0; i < spin; ++i) x = x * 0x9E3779B1u + (x >> 7);
    __builtin_amdgcn_s_waitcnt(0);
    out[g * 64u + lane] = x ^ s[lane];
}

int main(int argc, char** argv) {
    const int groups = 16384;
    const uint32_t words = 272u * 64u / 16u;
    const size_t n = (size_t)groups * words;
    uint4* src;
    uint32_t* out;
    CK(hipMalloc(&src, n * 16));
    CK(hipMalloc(&out, (size_t)groups * 64 * 4));
    CK(hipMemset(src, 1, n * 16));
    // a buffer larger than the Infinity Cache, read between runs, so every
    // run starts with the inputs out of it
    char* flush;
    const size_t fl = 512ull << 20;
    CK(hipMalloc(&flush, fl));
    CK(hipMemset(flush, 3, fl));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t spins[] = {0, 1000, 2000, 4000};
    const uint32_t dists[] = {0, 1024, 2048, 4096, 8192, 99};
    for (uint32_t sp : spins) {
        for (uint32_t d : dists) {
            const int stage = d != 99;
            float tot = 0;
            int cnt = 0;
            for (int r = 0; r < 6; ++r) {
                hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, (const uint4*)flush, fl / 16, out);
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_sim, dim3(groups), dim3(64), 0, 0, src, out, words, sp, stage ? d : 0u, stage);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r > 0) { tot += ms; ++cnt; }
            }
            printf("spin %5u dist %5u%s  %.4f ms\n", sp, stage ? d : 0u, stage ? "" : " (no staging)", tot / cnt);
        }
    }
    return 0;
}
