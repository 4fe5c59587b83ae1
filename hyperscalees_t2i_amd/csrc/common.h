// Shared helpers for libeggroll (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>
#include <type_traits>

#include "../../include/eggroll.h"

namespace eggroll {

void set_error(const char* fmt, ...);

#define EGG_CHECK_ARG(cond, ...)                 \
    do {                                         \
        if (!(cond)) {                           \
            ::eggroll::set_error(__VA_ARGS__);   \
            return EGGROLL_ERR_ARG;              \
        }                                        \
    } while (0)

#define EGG_CHECK_LAUNCH(what)                                                        \
    do {                                                                              \
        hipError_t e_ = hipGetLastError();                                            \
        if (e_ != hipSuccess) {                                                       \
            ::eggroll::set_error("%s: launch failed: %s", what, hipGetErrorString(e_)); \
            return EGGROLL_ERR_LAUNCH;                                                \
        }                                                                             \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- wave (64-lane) reductions -------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---- XCD-contiguous block order ------------------------------------------------------
// The dispatcher deals workgroups round-robin over the 8 XCDs (bid % 8 labels the blocks that share
// an XCD's private L2).  Bijective remap so the blocks sharing an L2 are CONSECUTIVE logical indices:
// neighbours in the logical order (the two 64-byte halves of a 128-byte line read by adjacent
// channel slices, adjacent heads of one token row) then share that L2 instead of each half-line
// being fetched once per XCD (cdna_hip_programming.md "XCD swizzle must be bijective", T1).
// Placement only changes speed, never results.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int xcd = bid & 7, q = nblk >> 3, rem = nblk & 7;
    return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
}

// ---- Philox4x32-10 (Salmon et al., SC'11; Random123 constants) ----------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
        u32x4 n;
        n.x = hi1 ^ c.y ^ k0;
        n.y = lo1;
        n.z = hi0 ^ c.w ^ k1;
        n.w = lo0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// Device Philox: each round's 32x32 -> 64-bit products as ONE v_mad_u64_u32 (hi and lo halves
// together) instead of the v_mul_lo_u32 + v_mul_hi_u32 pair the compiler emits for mulhi32 —
// half the quarter-rate integer multiplies.  Bit-identical to philox4x32_10.
__device__ __forceinline__ uint64_t mul_wide_u32(uint32_t a, uint32_t b) {
    uint64_t p, carry;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(carry) : "s"(a), "v"(b));
    (void)carry;
    return p;
}

__device__ __forceinline__ u32x4 philox4x32_10_dev(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = mul_wide_u32(M0, c.x);
        const uint64_t p1 = mul_wide_u32(M1, c.z);
        u32x4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

constexpr uint32_t kNoiseTag = 0xE6606011u;

// ---- factor layout + work tiles of perturb / update (include/eggroll.h) ------------------
// Per matrix, one base sample's factors are a [rows][r] at factor_off, then b [cols][r] at
// factor_off + pad4(rows * r): every segment starts 16-byte aligned when factor_off % 4 == 0.
__host__ __device__ inline int64_t egg_pad4(int64_t x) { return (x + 3) & ~(int64_t)3; }
__host__ __device__ inline int64_t egg_b_off(const eggroll_mat_t& mt, int r) {
    return mt.factor_off + egg_pad4(mt.rows * (int64_t)r);
}

enum EggTileKind { T_VEC4 = 0, T_WIDE = 1, T_TALL = 2, T_VEC = 3, T_GEN = 4 };

__host__ __device__ inline int egg_tile_kind(const eggroll_mat_t& mt, int r) {
    const bool al = (mt.theta_off & 3) == 0 && (mt.factor_off & 3) == 0;
    if (mt.cols == 0) return (al && (mt.rows & 3) == 0) ? T_VEC4 : T_VEC;
    const bool rok = r == 1 || r == 2 || r == 4;
    if (rok && al && mt.rows <= mt.cols && (mt.rows == 1 || mt.rows == 2 || mt.rows == 4) && (mt.cols & 3) == 0)
        return T_WIDE;
    if (rok && al && mt.cols < mt.rows && (mt.cols == 1 || mt.cols == 2 || mt.cols == 4) && (mt.rows & 3) == 0)
        return T_TALL;
    return T_GEN;
}

// workgroups of one matrix: fast kinds 1024 long-dimension positions each, generic 1024 elements
__host__ __device__ inline int64_t egg_tile_count(const eggroll_mat_t& mt, int r) {
    const int k = egg_tile_kind(mt, r);
    const int64_t n = k == T_WIDE ? mt.cols : (k == T_TALL || k == T_VEC4 || k == T_VEC) ? mt.rows
                                                                                        : mt.rows * mt.cols;
    return (n + 1023) / 1024;
}

}  // namespace eggroll
