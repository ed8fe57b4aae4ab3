// split.hip -- the giant stage's kernels and launchers (the device code is
// split.h: frontier, tasks, combine, fixup, finish; see its header).
#include <hip/hip_runtime.h>

#include "split.h"

namespace qsmd {

template <uint32_t MODEL>
__global__ __launch_bounds__(64) void giant_search(SplitArgs p) {
    __shared__ GiantLds<MODEL> u;
    const int lane = threadIdx.x;
    const uint32_t n_g = ld_cnt(p.cnt + C_GIANT);
    if (n_g == 0 && !p.early) {                 // nothing to do but the totals
        if (blockIdx.x == 0) finish_call(p, lane);
        return;
    }
    // the arguments where the launch put them (the kernel's one argument, at
    // offset 0 of the kernarg segment): no private copy of them
    // (a constant-address-space pointer: the same 64-bit global address)
    const SplitArgs* kp = reinterpret_cast<const SplitArgs*>((uintptr_t)__builtin_amdgcn_kernarg_segment_ptr());
    giant_work<MODEL>(*kp, n_g, u);
}

// qsmd_split_frontier: one giant (giant_list[0]), one lane.
template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
__global__ __launch_bounds__(LANES) void frontier_kernel(SplitArgs p, uint32_t variant) {
    __shared__ GLds<MODEL, MaskT, MAXEV, MAXPID, LANES> s;
    const int lane = threadIdx.x;
    const uint64_t t0 = p.s.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    if (lane == 0) {
        const uint32_t h = p.giant_list[0];
        const qsmd_hdr H = p.s.hdr[h];
        frontier_one<MODEL, MaskT, MAXEV, MAXPID, LANES>(p, 0u, h, H, variant, s, lane, t0);
    }
}

// qsmd_check_tasks: the task phase alone over the caller's tasks.
template <uint32_t MODEL, typename MaskT, int MAXEV, int MAXPID, int LANES>
__global__ __launch_bounds__(LANES) void task_kernel(SplitArgs p, uint32_t variant) {
    __shared__ GLds<MODEL, MaskT, MAXEV, MAXPID, LANES> s;
    const uint64_t t0 = p.s.time_limit ? __builtin_amdgcn_s_memrealtime() : 0;
    task_loop<MODEL, MaskT, MAXEV, MAXPID, LANES>(p, variant, s, threadIdx.x, t0, p.cnt + C_TQ0 + variant);
}

// ------------------------------------------------------------------ launch

namespace {
template <uint32_t MODEL>
hipError_t launch_parts(bool frontier, int variant, const SplitArgs& p, uint32_t grid, hipStream_t s) {
    if (variant == 0) {
        if (frontier)
            hipLaunchKernelGGL((frontier_kernel<MODEL, uint64_t, 64, 8, 64>), dim3(1), dim3(64), 0, s, p, 0u);
        else
            hipLaunchKernelGGL((task_kernel<MODEL, uint64_t, 64, 8, 64>), dim3(grid), dim3(64), 0, s, p, 0u);
    } else {
        if (frontier)
            hipLaunchKernelGGL((frontier_kernel<MODEL, M128, 128, 128, 16>), dim3(1), dim3(16), 0, s, p, 1u);
        else
            hipLaunchKernelGGL((task_kernel<MODEL, M128, 128, 128, 16>), dim3(grid), dim3(16), 0, s, p, 1u);
    }
    return hipGetLastError();
}
}  // namespace

hipError_t launch_giants(const SplitArgs& p, uint32_t grid, hipStream_t s) {
    if (p.s.model_id == QSMD_MODEL_BANK)
        hipLaunchKernelGGL(giant_search<QSMD_MODEL_BANK>, dim3(grid), dim3(64), 0, s, p);
    else
        hipLaunchKernelGGL(giant_search<QSMD_MODEL_TICKET>, dim3(grid), dim3(64), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_frontier_only(int variant, const SplitArgs& p, hipStream_t s) {
    if (p.s.model_id == QSMD_MODEL_BANK) return launch_parts<QSMD_MODEL_BANK>(true, variant, p, 1, s);
    return launch_parts<QSMD_MODEL_TICKET>(true, variant, p, 1, s);
}

hipError_t launch_tasks_only(int variant, const SplitArgs& p, uint32_t grid, hipStream_t s) {
    if (p.s.model_id == QSMD_MODEL_BANK) return launch_parts<QSMD_MODEL_BANK>(false, variant, p, grid, s);
    return launch_parts<QSMD_MODEL_TICKET>(false, variant, p, grid, s);
}

}  // namespace qsmd
