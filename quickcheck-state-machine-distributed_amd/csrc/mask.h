// mask.h -- fixed-width event bitsets (one bit per event of a history) used as
// the search state "remaining events" of SURVEY.md §8a Lemma L1.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qsmd {

template <typename T> struct MaskOps;

template <> struct MaskOps<uint32_t> {
    static constexpr int BITS = 32;
    __device__ __host__ static __forceinline__ uint32_t bit(int i) { return 1u << i; }
    __device__ static __forceinline__ int ctz(uint32_t x) { return __builtin_ctz(x); }
    __device__ static __forceinline__ int msb(uint32_t x) { return 31 - __builtin_clz(x); }
    __device__ static __forceinline__ bool any(uint32_t x) { return x != 0u; }
    __device__ static __forceinline__ uint32_t below(int r) { return r >= 32 ? ~0u : (1u << r) - 1u; }
    __device__ static __forceinline__ uint32_t lowest(uint32_t x) { return x & (0u - x); }
    __device__ static __forceinline__ uint32_t clear_lowest(uint32_t x) { return x & (x - 1u); }
};

template <> struct MaskOps<uint64_t> {
    static constexpr int BITS = 64;
    __device__ __host__ static __forceinline__ uint64_t bit(int i) { return 1ull << i; }
    __device__ static __forceinline__ int ctz(uint64_t x) { return __builtin_ctzll(x); }
    __device__ static __forceinline__ int msb(uint64_t x) { return 63 - __builtin_clzll(x); }
    __device__ static __forceinline__ bool any(uint64_t x) { return x != 0ull; }
    __device__ static __forceinline__ uint64_t below(int r) { return r >= 64 ? ~0ull : (1ull << r) - 1ull; }
    __device__ static __forceinline__ uint64_t lowest(uint64_t x) { return x & (0ull - x); }
    __device__ static __forceinline__ uint64_t clear_lowest(uint64_t x) { return x & (x - 1ull); }
};

// 128-bit mask (histories of up to 64 operations).
struct M128;
__device__ __host__ __forceinline__ M128 mk128(uint64_t l, uint64_t h);
struct M128 {
    uint64_t lo, hi;   // trivial aggregate: usable in __shared__ arrays
    __device__ __forceinline__ M128 operator&(const M128& o) const { return {lo & o.lo, hi & o.hi}; }
    __device__ __forceinline__ M128 operator|(const M128& o) const { return {lo | o.lo, hi | o.hi}; }
    __device__ __forceinline__ M128 operator^(const M128& o) const { return {lo ^ o.lo, hi ^ o.hi}; }
    __device__ __forceinline__ M128 operator~() const { return {~lo, ~hi}; }
    __device__ __forceinline__ M128& operator&=(const M128& o) { lo &= o.lo; hi &= o.hi; return *this; }
    __device__ __forceinline__ M128& operator|=(const M128& o) { lo |= o.lo; hi |= o.hi; return *this; }
};

__device__ __host__ __forceinline__ M128 mk128(uint64_t l, uint64_t h) {
    M128 m;
    m.lo = l;
    m.hi = h;
    return m;
}

template <> struct MaskOps<M128> {
    static constexpr int BITS = 128;
    __device__ __host__ static __forceinline__ M128 bit(int i) {
        return i < 64 ? mk128(1ull << i, 0ull) : mk128(0ull, 1ull << (i - 64));
    }
    __device__ static __forceinline__ int ctz(const M128& x) {
        return x.lo ? __builtin_ctzll(x.lo) : 64 + __builtin_ctzll(x.hi);
    }
    __device__ static __forceinline__ int msb(const M128& x) {
        return x.hi ? 127 - __builtin_clzll(x.hi) : 63 - __builtin_clzll(x.lo);
    }
    __device__ static __forceinline__ bool any(const M128& x) { return (x.lo | x.hi) != 0ull; }
    __device__ static __forceinline__ M128 below(int r) {
        if (r >= 128) return mk128(~0ull, ~0ull);
        if (r >= 64) return mk128(~0ull, r == 64 ? 0ull : (1ull << (r - 64)) - 1ull);
        return mk128((1ull << r) - 1ull, 0ull);
    }
    __device__ static __forceinline__ M128 lowest(const M128& x) {
        return x.lo ? mk128(x.lo & (0ull - x.lo), 0ull) : mk128(0ull, x.hi & (0ull - x.hi));
    }
    __device__ static __forceinline__ M128 clear_lowest(const M128& x) {
        return x.lo ? mk128(x.lo & (x.lo - 1ull), x.hi) : mk128(0ull, x.hi & (x.hi - 1ull));
    }
};

}  // namespace qsmd
