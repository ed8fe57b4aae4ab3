// What a stage-0-shaped read costs on gfx950 with nothing else in the kernel
// (diagnostic for compact.hip's staging): 16384 workgroups of one wavefront,
// each reading its group's bytes (64 histories x BYTES_PER_HIST) with
// 16-byte loads, STEPS loads per lane in flight, the words XOR-folded into
// LDS (so the loads are live) and one store per lane.  Variants:
//   lds_kb     LDS per workgroup (10 = stage 0's 4 wavefronts per SIMD)
//   hdr        a dependent 16-B header load first (the group's offset comes
//              from it, like stage 0's ev_off)
//   l2         every group reads group (g & 63)'s bytes (L2-resident)
// Prints the kernel time (hipEvent) and the rate over the bytes read.
//   hipcc --offload-arch=gfx950 -O3 stream_read.hip -o stream_read
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int STEPS>
__global__ __launch_bounds__(64) void k_read(const uint4* __restrict__ src, const uint4* __restrict__ hdr,
                                             uint32_t* __restrict__ out, uint32_t words_per_group, int use_hdr,
                                             int l2) {
    extern __shared__ uint32_t s[];
    const uint32_t lane = threadIdx.x;
    uint32_t g = blockIdx.x;
    if (l2) g &= 63u;
    uint64_t base = (uint64_t)g * words_per_group;      // in uint4 units
    if (use_hdr) base = hdr[g * 64u + lane].x;            // 16-B header per history, lane 0's offset used
    base = __builtin_amdgcn_readfirstlane((uint32_t)base);
    uint32_t acc = 0;
    for (uint32_t k = 0; k < words_per_group; k += 64u * STEPS) {
        uint4 v[STEPS];
#pragma unroll
        for (int u = 0; u < STEPS; ++u) {
            const uint32_t i = k + u * 64u + lane;
            v[u] = i < words_per_group ? src[base + i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < STEPS; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        s[(k / 64u) % 32u * 64u + lane] = acc;
    }
    out[blockIdx.x * 64u + lane] = acc ^ s[lane];
}

int main(int argc, char** argv) {
    const int groups = 16384;
    const int bytes_per_hist = argc > 1 ? atoi(argv[1]) : 272;   // 256 B of events + 16 B header
    const uint32_t words = (uint32_t)(bytes_per_hist * 64 / 16);
    const size_t n = (size_t)groups * words;
    uint4 *src, *hdr;
    uint32_t* out;
    CK(hipMalloc(&src, n * 16));
    CK(hipMalloc(&hdr, (size_t)groups * 64 * 16));
    CK(hipMalloc(&out, (size_t)groups * 64 * 4));
    CK(hipMemset(src, 1, n * 16));
    std::vector<uint4> h((size_t)groups * 64);
    for (int g = 0; g < groups; ++g)
        for (int l = 0; l < 64; ++l) h[(size_t)g * 64 + l] = make_uint4((uint32_t)((size_t)g * words), 0, 0, 0);
    CK(hipMemcpy(hdr, h.data(), h.size() * 16, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V { const char* name; int steps, lds_kb, use_hdr, l2; };
    const V vs[] = {{"steps4 lds10", 4, 10, 0, 0},  {"steps4 lds10 hdr", 4, 10, 1, 0}, {"steps4 lds10 l2", 4, 10, 0, 1},
                    {"steps8 lds10", 8, 10, 0, 0},  {"steps4 lds5", 4, 5, 0, 0},      {"steps4 lds20", 4, 20, 0, 0},
                    {"steps4 lds5 hdr", 4, 5, 1, 0}};
    for (const V& v : vs) {
        float best = 1e9f;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(e0));
            const size_t lds = (size_t)v.lds_kb * 1024;
            if (v.steps == 4)
                hipLaunchKernelGGL(k_read<4>, dim3(groups), dim3(64), lds, 0, src, hdr, out, words, v.use_hdr, v.l2);
            else
                hipLaunchKernelGGL(k_read<8>, dim3(groups), dim3(64), lds, 0, src, hdr, out, words, v.use_hdr, v.l2);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0 && ms < best) best = ms;
        }
        printf("%-20s %.4f ms  %.2f TB/s\n", v.name, best, (double)n * 16 / (best * 1e-3) / 1e12);
    }
    return 0;
}
