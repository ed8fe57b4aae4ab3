// Latency of one wavefront's dependent chains on gfx950 (diagnostic for the
// wave-mode heavy stage, csrc/wave.hip): cycles (s_memtime) per iteration of
//   salu     a dependent scalar chain (s_xor / s_add / s_lshl)
//   rl       v_readlane at an index computed by the previous step (VALU -> SGPR -> VALU)
//   rl_salu  readlane + 4 dependent scalar ops per step
//   branch   a data-dependent uniform branch per step
//   ballot   v_cmp (lane compare with a scalar) -> SGPR mask -> s_ff1 per step
// One wavefront, one workgroup; the chain length N is a kernel argument so
// nothing is folded.   hipcc --offload-arch=gfx950 -O3 chain_latency.hip -o chain_latency
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }

__global__ void k_salu(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    uint32_t x = __builtin_amdgcn_readfirstlane(seed);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) x = ((x ^ (x << 3)) + 0x9E3779B1u) ^ (x >> 7);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = x; }
}

__global__ void k_rl(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    const uint32_t v = threadIdx.x * 0x9E3779B1u + seed;
    uint32_t x = __builtin_amdgcn_readfirstlane(seed);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) x = rl(v, x & 63u);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = x; }
}

__global__ void k_rl_salu(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    const uint32_t v = threadIdx.x * 0x9E3779B1u + seed;
    uint32_t x = __builtin_amdgcn_readfirstlane(seed);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) {
        x = rl(v, x & 63u);
        x = ((x ^ (x << 3)) + 0x9E3779B1u) ^ (x >> 7);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = x; }
}

__global__ void k_branch(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    uint32_t x = __builtin_amdgcn_readfirstlane(seed), y = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) {
        if (x & 1u) { x = x * 3u + 1u; y += x; }
        else { x >>= 1; y ^= x; }
        x ^= i;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = x + y; }
}

__global__ void k_ballot(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    const uint32_t v = (threadIdx.x * 7u) & 15u;
    uint32_t x = __builtin_amdgcn_readfirstlane(seed);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t m = __ballot(v == (x & 15u));
        x = (uint32_t)__builtin_ctzll(m | (1ull << 63)) + i;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = x; }
}

__global__ void k_lds(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    __shared__ uint32_t t[64];
    t[threadIdx.x] = threadIdx.x * 0x9E3779B1u + seed;
    __syncthreads();
    uint32_t x = __builtin_amdgcn_readfirstlane(seed);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) x = t[(x + threadIdx.x) & 63u] >> 3;
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = x; }
}

__global__ void k_valu(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    uint32_t x = seed + threadIdx.x;               // per-lane: VALU
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) x = ((x ^ (x << 3)) + 0x9E3779B1u) ^ (x >> 7);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; }
    sink[threadIdx.x & 0] = x;
}

__global__ void k_valu64(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    uint64_t x = seed + threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) x = ((x ^ (x << 3)) + 0x9E3779B97F4A7C15ull) & (x | 0x55ull);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; }
    sink[0] = (uint32_t)x;
}

__global__ void k_perm(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    const uint32_t v = threadIdx.x * 0x9E3779B1u + seed;
    uint32_t x = seed + threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) x = __shfl(v, (int)(x & 63u), 64);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; }
    sink[0] = x;
}

// four independent scalar chains interleaved (issue rate, not latency)
__global__ void k_salu4(uint32_t n, uint32_t seed, unsigned long long* out, uint32_t* sink) {
    uint32_t a = __builtin_amdgcn_readfirstlane(seed), b = a + 1, c = a + 2, d = a + 3;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; ++i) {
        a = ((a ^ (a << 3)) + 0x9E3779B1u) ^ (a >> 7);
        b = ((b ^ (b << 3)) + 0x9E3779B1u) ^ (b >> 7);
        c = ((c ^ (c << 3)) + 0x9E3779B1u) ^ (c >> 7);
        d = ((d ^ (d << 3)) + 0x9E3779B1u) ^ (d >> 7);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = a + b + c + d; }
}

int main() {
    unsigned long long* d_out;
    uint32_t* d_sink;
    (void)hipMalloc(&d_out, 8);
    (void)hipMalloc(&d_sink, 4);
    const uint32_t n = 100000;
    struct K { const char* name; void (*f)(uint32_t, uint32_t, unsigned long long*, uint32_t*); };
    K ks[] = {{"salu (3 dependent ops)", k_salu}, {"readlane chain", k_rl}, {"readlane + 3 salu", k_rl_salu},
              {"uniform branch", k_branch}, {"ballot + ctz", k_ballot}, {"lds read chain", k_lds},
              {"valu (3 dependent ops)", k_valu}, {"valu u64 (3 dep. ops)", k_valu64}, {"ds_bpermute chain", k_perm},
              {"salu 4 chains x 3 ops", k_salu4}};
    for (auto& k : ks) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, n, 12345u, d_out, d_sink);
            (void)hipDeviceSynchronize();
        }
        unsigned long long c = 0;
        (void)hipMemcpy(&c, d_out, 8, hipMemcpyDeviceToHost);
        printf("%-24s %8.2f cycles/step\n", k.name, (double)c / n);
    }
    // the clock of s_memtime: cycles per microsecond over a timed launch
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k_salu, dim3(1), dim3(64), 0, 0, 20000000u, 1u, d_out, d_sink);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long c = 0;
    (void)hipMemcpy(&c, d_out, 8, hipMemcpyDeviceToHost);
    printf("s_memtime: %.0f ticks in %.3f ms = %.3f GHz\n", (double)c, ms, c / (ms * 1e6));
    return 0;
}
