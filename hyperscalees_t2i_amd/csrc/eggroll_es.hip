// libeggroll — ES arithmetic kernels for gfx950 (MI355X):
//   (1) counter-based low-rank noise factors, perturb / eps materialisation,
//   (3) fused promptnorm + z-score fitness + stable rank sort,
//   (4) rank-(N*r) ES update with step / theta norm caps.
// Reference semantics: utills.py:14-178, 310-349 and unifed_es.py:120-281
// (amit154154/HyperscaleES_T2I).  Floating-point contraction is disabled in every kernel
// whose result is compared bit-for-bit with the CPU oracle (oracle/eggroll_oracle.py).
#include <math.h>
#include <stdarg.h>

#include "common.h"

namespace eggroll {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// ------------------------------------------------------------------------------------
// (1) noise factors
// ------------------------------------------------------------------------------------
// Box-Muller on the CDNA4 transcendental unit: v_log_f32 (log2), v_sqrt_f32 and v_sin_f32 /
// v_cos_f32 (which take their argument in revolutions: sin(2 pi x)), ~10 VALU ops per pair instead
// of the ~60 of the correctly-rounded libm expansions — the noise kernel becomes HBM-bound instead
// of VALU-bound.  Accuracy vs the oracle's correctly-rounded fp32 restatement is pinned by
// tests/test_gpu_kernels.py (|dz| <= 2e-5).
__device__ __forceinline__ void box_muller(uint32_t w0, uint32_t w1, float& z0, float& z1) {
#pragma clang fp contract(off)
    // 23-bit uniforms: exact in fp32.  u1 in (0,1), u2 in [0,1).
    const float u1 = ((float)(w0 >> 9) + 0.5f) * 1.1920928955078125e-07f;  // 2^-23
    const float u2 = (float)(w1 >> 9) * 1.1920928955078125e-07f;
    const float rr = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // -2 ln2 log2(u1)
    z0 = rr * __builtin_amdgcn_cosf(u2);
    z1 = rr * __builtin_amdgcn_sinf(u2);
}

// One thread = NOISE_QPT quads (16-byte stores) of one base sample, 256 quads apart so every store
// instruction of a wave is one contiguous KiB.  The kernel is VALU-bound (Philox4x32-10: 20 quarter-rate
// 32x32->64 multiplies per quad, plus Box-Muller on the transcendental unit) about as much as store-
// bound: 4 quads per thread measured 20.9 vs 20.3 us at pop 64 (interleaved chains, a quarter of the
// workgroups), so one quad per thread stays.
#ifndef EGG_NOISE_QPT  // A/B knob
#define EGG_NOISE_QPT 1
#endif
constexpr int NOISE_QPT = EGG_NOISE_QPT;

// The factor rows are a write-once stream (read back by perturb for the local members and by the update
// at the end of the epoch): non-temporal 16-B stores, 29.7 -> 27.2 us at one GPU's share of configs[2]
// and 500 -> 448 us at configs[3] (same process, tools/es_nt_probe.py).  (The same stores made perturb's
// theta_pop rows 8-26 % slower: those stay default-policy.)
__device__ __forceinline__ void st4_nt(float* __restrict__ p, float4 v) {
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    const f32x4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4v*>(p));
}

__global__ __launch_bounds__(256) void k_noise(uint32_t k0, uint32_t k1, int64_t base_lo,
                                               int64_t factor_len, int64_t ld, float* __restrict__ out) {
    const int64_t quads = (factor_len + 3) / 4;
    const int64_t qb = (int64_t)blockIdx.x * (256 * NOISE_QPT) + threadIdx.x;
    const int64_t j = base_lo + blockIdx.y;
    float* row = out + (int64_t)blockIdx.y * ld;
    float4 v[NOISE_QPT];
#pragma unroll
    for (int u = 0; u < NOISE_QPT; ++u) {
        const int64_t q = qb + u * 256;
        u32x4 c{(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)j, kNoiseTag};
        const u32x4 w = philox4x32_10_dev(c, k0, k1);
        box_muller(w.x, w.y, v[u].x, v[u].y);
        box_muller(w.z, w.w, v[u].z, v[u].w);
    }
#pragma unroll
    for (int u = 0; u < NOISE_QPT; ++u) {
        const int64_t q = qb + u * 256;
        if (q >= quads) break;
        const int64_t g0 = q * 4;
        float* dst = row + g0;
        if (g0 + 4 <= factor_len) {
            st4_nt(dst, v[u]);
        } else {
            const float t[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            for (int i = 0; i < 4 && g0 + i < factor_len; ++i) dst[i] = t[i];
        }
    }
}

__global__ void k_philox_words(uint32_t k0, uint32_t k1, int64_t j, int64_t n_quads, uint32_t* out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n_quads) return;
    u32x4 c{(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)j, kNoiseTag};
    const u32x4 w = philox4x32_10_dev(c, k0, k1);
    out[4 * q + 0] = w.x;
    out[4 * q + 1] = w.y;
    out[4 * q + 2] = w.z;
    out[4 * q + 3] = w.w;
}

// member -> (base sample, sign); reference antithetic layout utills.py:88-105
__host__ __device__ __forceinline__ void member_to_base(int64_t k, int32_t pop, int32_t antithetic,
                                                        int64_t& j, float& sgn) {
    if (!antithetic) {
        j = k;
        sgn = 1.0f;
        return;
    }
    const int64_t h = pop / 2;
    if (k < h) {
        j = k;
        sgn = 1.0f;
    } else if (k < 2 * h) {
        j = k - h;
        sgn = -1.0f;
    } else {
        j = h;
        sgn = 1.0f;
    }
}

// ------------------------------------------------------------------------------------
// Factor source.  Stored (GEN = false): base sample j's factor row j * ld of the buffer k_noise wrote.
// Regenerated (GEN = true, the seeded entry points): element g of base sample j is recomputed where it
// is consumed — Philox4x32-10 of counter (g / 4, j, kNoiseTag) under key (k0, k1), then the same
// Box-Muller as k_noise — so the values are bit-identical to the stored path while no factor byte is
// written to or read from HBM (north_star kernel (1): "noise is regenerated rather than stored").
// The fast tiles consume factors in 4-aligned quads (segments are padded to 4 floats), so one Philox
// call yields exactly the 4 values a 16-byte load would have.
// ------------------------------------------------------------------------------------
struct FacSrc {
    const float* f;  // stored rows (GEN = false)
    int64_t ld;
    uint32_t k0, k1; // Philox key = the epoch seed (GEN = true)
};

template <bool GEN>
__device__ __forceinline__ float4 fac4(const FacSrc& s, int64_t j, int64_t off) {  // off % 4 == 0
    if constexpr (GEN) {
        const int64_t q = off >> 2;
        const u32x4 c{(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)j, kNoiseTag};
        const u32x4 w = philox4x32_10_dev(c, s.k0, s.k1);
        float4 v;
        box_muller(w.x, w.y, v.x, v.y);
        box_muller(w.z, w.w, v.z, v.w);
        return v;
    } else {
        return *reinterpret_cast<const float4*>(s.f + j * s.ld + off);
    }
}

template <bool GEN>
__device__ __forceinline__ float fac1(const FacSrc& s, int64_t j, int64_t g) {
    if constexpr (GEN) {
        const float4 v = fac4<true>(s, j, g & ~(int64_t)3);
        const int c = (int)(g & 3);
        return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
    } else {
        return s.f[j * s.ld + g];
    }
}

// ------------------------------------------------------------------------------------
// Work decomposition shared by perturb and update: a host-built tile table (eggroll_tile_table)
// gives every workgroup its (matrix, tile) with ONE scalar load — no search over the matrix list.
// Fast tiles (T_VEC4 / T_WIDE / T_TALL, egg rank 1, 2 or 4) cover 1024 positions of the matrix's
// LONG dimension — 4 consecutive positions per thread, so theta, the long-dimension factor and the
// outputs move as 16-byte vectors — times all NU <= 4 entries of its SHORT dimension:
//   T_WIDE  PEFT lora_A [r_l, in]  (rows in {1,2,4} <= cols): long = columns, uniform = a[row]
//   T_TALL  PEFT lora_B [out, r_l] (cols in {1,2,4} <  rows): long = rows,    uniform = b[col]
//   T_VEC4  1-D parameter (dense noise, the factor is the eps itself)
// The short-dimension ("uniform") factors are the same for the whole workgroup: lane l of every wave
// holds base sample / member l's, broadcast with v_readlane (an SGPR operand).  Anything else
// (other ranks, unaligned 1-D params, matrices with no short dimension <= 4) runs the generic
// per-element path on 1024-element chunks (T_VEC / T_GEN).
// Every eps is computed in the reference's fp32 op order (sum_q a[i,q] b[c,q] sequential) / sqrt(r),
// so the result does not depend on the tile kind.
// ------------------------------------------------------------------------------------
struct Slots {  // generic path: this thread's element slots inside one 1024-element chunk
    int row[4], col[4];
    bool ok[4];
};

template <bool VEC1D>
__device__ __forceinline__ Slots make_slots(const eggroll_mat_t& mt, int64_t cidx, int tid) {
    Slots sl;
    const int cols = (int)mt.cols;
    const int numel = VEC1D ? (int)mt.rows : (int)mt.rows * cols;
    const int e0 = (int)cidx * EGGROLL_CHUNK;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int e = e0 + s * 256 + tid;
        sl.ok[s] = e < numel;
        if (VEC1D) {
            sl.row[s] = e;
            sl.col[s] = 0;
        } else {
            const int r = sl.ok[s] ? e / cols : 0;
            sl.row[s] = r;
            sl.col[s] = e - r * cols;
        }
    }
    return sl;
}

// eps of (row, col) of matrix mt for the base-sample factor row fj (utills.py:59-65 restated)
template <bool VEC1D, bool GEN>
__device__ __forceinline__ float eps_rc(const eggroll_mat_t& mt, const FacSrc& src, int64_t j, int row, int col,
                                        int r, float sqrt_r) {
#pragma clang fp contract(off)
    if constexpr (VEC1D) {
        return fac1<GEN>(src, j, mt.factor_off + row);
    } else {
        const int64_t a = mt.factor_off + (int64_t)row * r;
        const int64_t b = egg_b_off(mt, r) + (int64_t)col * r;
        float acc = fac1<GEN>(src, j, a) * fac1<GEN>(src, j, b);
        for (int q = 1; q < r; ++q) acc = acc + fac1<GEN>(src, j, a + q) * fac1<GEN>(src, j, b + q);
        return r == 1 ? acc : acc / sqrt_r;
    }
}

// 16-byte (V4) or scalar (unaligned caller buffers) access to 4 consecutive floats
template <bool V4>
__device__ __forceinline__ float4 ld4(const float* __restrict__ p) {
    if constexpr (V4) {
        return *reinterpret_cast<const float4*>(p);
    } else {
        return float4{p[0], p[1], p[2], p[3]};
    }
}
template <bool V4>
__device__ __forceinline__ void st4(float* __restrict__ p, float4 v) {
    if constexpr (V4) {
        *reinterpret_cast<float4*>(p) = v;
    } else {
        p[0] = v.x;
        p[1] = v.y;
        p[2] = v.z;
        p[3] = v.w;
    }
}
__device__ __forceinline__ float f4(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
__device__ __forceinline__ void f4set(float4& v, int i, float x) {
    if (i == 0) v.x = x;
    else if (i == 1) v.y = x;
    else if (i == 2) v.z = x;
    else v.w = x;
}

__device__ __forceinline__ float bcast(float v, int lane) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// Fast-tile geometry.  Element (v, u) of a thread: long position p0 + v (v < 4), short index u.
//   theta index: WIDE  toff + u * cols + p0 + v      TALL  toff + (p0 + v) * NU + u     VEC4 toff + p0 + v
//   long factor: WIDE  b[(p0+v)][q]                  TALL  a[(p0+v)][q]                 VEC4 x[p0+v]
// The thread's theta / output entries are NU float4s: TH[i] holds flat entries 4i..4i+3 of its block
// (WIDE: row u = i; TALL: the 4 * NU contiguous floats of rows p0..p0+3).
template <int KIND, int NU>
struct FastGeo {
    __device__ static int64_t th_off(const eggroll_mat_t& mt, int64_t p0, int i) {
        return KIND == T_WIDE ? mt.theta_off + (int64_t)i * mt.cols + p0 : mt.theta_off + p0 * NU + 4 * i;
    }
    // (v, u) -> (float4 index, component)
    __device__ static int vi(int v, int u) { return KIND == T_WIDE ? u : (v * NU + u) >> 2; }
    __device__ static int vc(int v, int u) { return KIND == T_WIDE ? v : (v * NU + u) & 3; }
    __device__ static int64_t x_off(const eggroll_mat_t& mt, int r) {  // long-dimension factor segment
        return KIND == T_WIDE ? egg_b_off(mt, r) : mt.factor_off;
    }
    __device__ static int64_t u_off(const eggroll_mat_t& mt, int r) {  // short-dimension factor segment
        return KIND == T_WIDE ? mt.factor_off : egg_b_off(mt, r);
    }
};

// Uniform factors of the base sample / member held by lane `ln`, broadcast once (NU * R SGPRs).
template <int NW>
__device__ __forceinline__ void bcast_all(float (&wb)[NW], const float (&W)[NW], int ln) {
#pragma unroll
    for (int w = 0; w < NW; ++w) wb[w] = bcast(W[w], ln);
}

// eps(v, u) of one base sample from its long factors X (4 positions x R) and its broadcast uniform
// factors wb[u * R + q]; reference op order.
template <int KIND, int R, int NU>
__device__ __forceinline__ float fast_eps(const float4 (&X)[R], const float (&wb)[NU * R], int v, int u,
                                          float sqrt_r) {
#pragma clang fp contract(off)
    if constexpr (KIND == T_VEC4) {
        return f4(X[0], v);
    } else {
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float x = f4(X[(v * R + q) >> 2], (v * R + q) & 3);
            const float w = wb[u * R + q];
            const float pr = KIND == T_WIDE ? w * x : x * w;  // a * b
            acc = q == 0 ? pr : acc + pr;
        }
        // rank 4: sqrt(4) = 2 exactly, and x / 2 and x * 0.5 are the same correctly rounded value (both
        // round the same real number, subnormals included) — one multiply instead of the ~10-instruction
        // correctly rounded divide (bit-identical; time-neutral on its own, the rank-4 update was
        // latency-bound: see the software pipeline in update_fast)
        if constexpr (R == 4) return acc * 0.5f;
        return R == 1 ? acc : acc / sqrt_r;
    }
}

// k_update at rank >= 2: the next base group's long-factor loads issued before this group's math
// (A/B knob; perturb measured 2-5 % slower with the same pipeline at rank 4, so it has none)
#ifndef EGG_UPD_PREFETCH
#define EGG_UPD_PREFETCH 1
#endif
// members / base samples whose long-factor loads are in flight together: 8 float4 loads per
// thread whatever the rank (rank 4 at 8 samples needed 228 VGPRs and halved the occupancy)
#ifndef EGG_PTB_PGRR  // k_perturb, rank >= 2: float4 loads per group (A/B knob)
#define EGG_PTB_PGRR 8
#endif
#ifndef EGG_UPD_PGRR  // k_update, rank >= 2: float4 loads per group (x2 with the pipeline)
#define EGG_UPD_PGRR 4
#endif
#ifndef EGG_UPD_PGRP1
#define EGG_UPD_PGRP1 8
#endif
template <int KIND, int R, bool UPD = false>
struct PGrp {
    static constexpr int value = (KIND == T_VEC4 || R == 1) ? (UPD ? EGG_UPD_PGRP1 : 8) : (UPD ? EGG_UPD_PGRR : EGG_PTB_PGRR) / R;
};

// Uniform (short-dimension) factors of one base sample: NW floats from the 4-aligned segment start uo
// (NW <= the segment's padded length); 1.0 where !use (1-D params, members / base samples past the end).
template <int KIND, int NW, bool GEN>
__device__ __forceinline__ void load_uniform(float (&W)[NW], const FacSrc& src, int64_t j, int64_t uo, bool use) {
    if constexpr (GEN) {
#pragma unroll
        for (int w0 = 0; w0 < NW; w0 += 4) {
            const float4 v = use ? fac4<true>(src, j, uo + w0) : float4{1.0f, 1.0f, 1.0f, 1.0f};
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (w0 + c < NW) W[w0 + c] = f4(v, c);
        }
    } else {
#pragma unroll
        for (int w = 0; w < NW; ++w) W[w] = use ? src.f[j * src.ld + uo + w] : 1.0f;
    }
}

// ------------------------------------------------------------------------------------
// perturb / materialise: out[k] = theta + sigma * s_k * E_j(k) for the members [lo, lo + n).
// One workgroup per tile; theta is read once and every member's row is written from registers.
// ------------------------------------------------------------------------------------
template <int KIND, int R, int NU, bool V4, bool GEN>
__device__ __forceinline__ void perturb_fast(const float* __restrict__ theta, const FacSrc& src,
                                             const eggroll_mat_t& mt, int64_t tidx, float sqrt_r,
                                             int32_t pop, int32_t antithetic, int64_t member_lo, int n_members,
                                             float sigma, float* __restrict__ out, int64_t ld_out) {
#pragma clang fp contract(off)
    using G = FastGeo<KIND, NU>;
    constexpr int NX = KIND == T_VEC4 ? 1 : R;  // float4s of long factor per base sample
    constexpr int NW = KIND == T_VEC4 ? 1 : NU * R;
    const int lane = threadIdx.x & 63;
    const int64_t lng = KIND == T_WIDE ? mt.cols : mt.rows;
    const int64_t p0 = tidx * 1024 + 4 * (int64_t)threadIdx.x;
    const bool ok = p0 < lng;
    float4 TH[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) TH[i] = (theta && ok) ? ld4<V4>(theta + G::th_off(mt, p0, i)) : float4{0, 0, 0, 0};
    const int64_t xo = G::x_off(mt, R) + p0 * (KIND == T_VEC4 ? 1 : R);
    const int64_t uo = G::u_off(mt, R);
    for (int g = 0; g < n_members; g += 64) {
        // lane l: member g+l's base sample, sign and uniform factors
        float W[NW];
        int jl;
        float sl;
        {
            int64_t jb;
            member_to_base(member_lo + g + lane, pop, antithetic, jb, sl);
            const bool mok = g + lane < n_members;
            jl = mok ? (int)jb : 0;
            load_uniform<KIND, NW, GEN>(W, src, jb, uo, KIND != T_VEC4 && mok);
        }
        const int n = (n_members - g) < 64 ? (n_members - g) : 64;
        constexpr int PG = PGrp<KIND, R>::value;
        for (int i0 = 0; i0 < n; i0 += PG) {
            float4 X[PG][NX];
#pragma unroll
            for (int t = 0; t < PG; ++t) {
                const int64_t j = __builtin_amdgcn_readlane(jl, (i0 + t) & 63);
                const bool lok = ok && (i0 + t < n);
#pragma unroll
                for (int c = 0; c < NX; ++c) X[t][c] = lok ? fac4<GEN>(src, j, xo + 4 * c) : float4{0, 0, 0, 0};
            }
#pragma unroll
            for (int t = 0; t < PG; ++t) {
                if (i0 + t >= n) break;
                const float sgn = bcast(sl, i0 + t);
                float wb[NW];
                bcast_all(wb, W, i0 + t);
                float4 O[NU];
#pragma unroll
                for (int v = 0; v < 4; ++v)
#pragma unroll
                    for (int u = 0; u < NU; ++u) {
                        const float e = sgn * fast_eps<KIND, R, NU>(X[t], wb, v, u, sqrt_r);
                        const float th = f4(TH[G::vi(v, u)], G::vc(v, u));
                        float val;
                        if (theta) {
                            const float tt = sigma * e;
                            val = th + tt;
                        } else {
                            val = sigma * e;
                        }
                        f4set(O[G::vi(v, u)], G::vc(v, u), val);
                    }
                if (ok) {
                    float* dst = out + (int64_t)(g + i0 + t) * ld_out;
#pragma unroll
                    for (int i = 0; i < NU; ++i) st4<V4>(dst + G::th_off(mt, p0, i), O[i]);
                }
            }
        }
    }
}

template <bool VEC1D, bool GEN>
__device__ __forceinline__ void perturb_chunk(const float* __restrict__ theta, const FacSrc& src,
                                              const eggroll_mat_t& mt, int64_t cidx, int r,
                                              float sqrt_r, int32_t pop, int32_t antithetic, int64_t member_lo,
                                              int n_members, float sigma, float* __restrict__ out, int64_t ld_out) {
#pragma clang fp contract(off)
    const Slots sl = make_slots<VEC1D>(mt, cidx, threadIdx.x);
    float th[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int e = VEC1D ? sl.row[s] : sl.row[s] * (int)mt.cols + sl.col[s];
        th[s] = (theta && sl.ok[s]) ? theta[mt.theta_off + e] : 0.0f;
    }
#pragma unroll 4
    for (int i = 0; i < n_members; ++i) {
        int64_t j;
        float sgn;
        member_to_base(member_lo + i, pop, antithetic, j, sgn);
        float* dst = out + (int64_t)i * ld_out + mt.theta_off;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (!sl.ok[s]) continue;
            const float eps = sgn * eps_rc<VEC1D, GEN>(mt, src, j, sl.row[s], sl.col[s], r, sqrt_r);
            float v;
            if (theta) {
                const float t = sigma * eps;
                v = th[s] + t;
            } else {
                v = sigma * eps;
            }
            dst[VEC1D ? sl.row[s] : sl.row[s] * (int)mt.cols + sl.col[s]] = v;
        }
    }
}

// Dispatch of one tile to its kind's instantiation (R = egg rank, a template parameter).
template <int R, bool V4, class FastFn, class GenFn>
__device__ __forceinline__ void dispatch_tile(const eggroll_mat_t& mt, int r, FastFn&& fast, GenFn&& gen) {
    const int kind = egg_tile_kind(mt, r);
    const int nu = kind == T_WIDE ? (int)mt.rows : (kind == T_TALL ? (int)mt.cols : 1);
    if (kind == T_VEC4) fast(std::integral_constant<int, T_VEC4>{}, std::integral_constant<int, 1>{});
    else if (kind == T_WIDE && nu == 1) fast(std::integral_constant<int, T_WIDE>{}, std::integral_constant<int, 1>{});
    else if (kind == T_WIDE && nu == 2) fast(std::integral_constant<int, T_WIDE>{}, std::integral_constant<int, 2>{});
    else if (kind == T_WIDE) fast(std::integral_constant<int, T_WIDE>{}, std::integral_constant<int, 4>{});
    else if (kind == T_TALL && nu == 1) fast(std::integral_constant<int, T_TALL>{}, std::integral_constant<int, 1>{});
    else if (kind == T_TALL && nu == 2) fast(std::integral_constant<int, T_TALL>{}, std::integral_constant<int, 2>{});
    else if (kind == T_TALL) fast(std::integral_constant<int, T_TALL>{}, std::integral_constant<int, 4>{});
    else if (kind == T_VEC) gen(std::true_type{});
    else gen(std::false_type{});
}

template <int R, bool V4, bool GEN>
__global__ __launch_bounds__(256) void k_perturb(const float* __restrict__ theta, FacSrc src,
                                                 const eggroll_mat_t* __restrict__ mats,
                                                 const eggroll_tile_t* __restrict__ tiles, int r, float sqrt_r,
                                                 int32_t pop, int32_t antithetic, int64_t member_lo, int n_all,
                                                 int mpb, float sigma, float* __restrict__ out_all, int64_t ld_out) {
    const eggroll_tile_t tl = tiles[blockIdx.x];
    const eggroll_mat_t mt = mats[tl.mat];
    // grid.y splits the members into groups of mpb (perturb_launch): a member's row is computed the same
    // way whichever group holds it
    const int g0 = (int)blockIdx.y * mpb;
    const int n_members = n_all - g0 < mpb ? n_all - g0 : mpb;
    member_lo += g0;
    float* __restrict__ out = out_all + (int64_t)g0 * ld_out;
    dispatch_tile<R, V4>(
        mt, r,
        [&](auto KD, auto NUv) {
            constexpr int KK = decltype(KD)::value;
            if constexpr (KK == T_VEC4)
                perturb_fast<T_VEC4, 1, 1, V4, GEN>(theta, src, mt, tl.index, sqrt_r, pop, antithetic, member_lo,
                                                    n_members, sigma, out, ld_out);
            else if constexpr (R > 0)
                perturb_fast<KK, R, decltype(NUv)::value, V4, GEN>(theta, src, mt, tl.index, sqrt_r, pop,
                                                                   antithetic, member_lo, n_members, sigma, out, ld_out);
        },
        [&](auto VD) {
            perturb_chunk<decltype(VD)::value, GEN>(theta, src, mt, tl.index, r, sqrt_r, pop, antithetic,
                                                    member_lo, n_members, sigma, out, ld_out);
        });
}

// ------------------------------------------------------------------------------------
// (3) fitness: promptnorm -> finite mask -> z-score -> stable argsort.  One workgroup.
// Summation orders are fixed (sequential) and mirrored by the oracle.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ bool lt_nan_last(float a, float b) {  // a < b with NaN = +max
    const bool an = isnan(a), bn = isnan(b);
    if (an) return false;
    if (bn) return true;
    return a < b;
}
__device__ __forceinline__ bool eq_nan(float a, float b) {
    const bool an = isnan(a), bn = isnan(b);
    if (an || bn) return an && bn;
    return a == b;
}

__global__ __launch_bounds__(1024) void k_fitness(const float* __restrict__ S, int n, int m, int promptnorm,
                                                  float pn_eps, float* __restrict__ scores, float* __restrict__ mu,
                                                  float* __restrict__ stats, float* __restrict__ fit,
                                                  int32_t* __restrict__ finite, int32_t* __restrict__ order) {
#pragma clang fp contract(off)
    __shared__ float s_mu[1024];
    __shared__ float s_row[4096];
    __shared__ float s_sc[4096];
    __shared__ float s_misc[4];
    __shared__ float s_S[4096];
    const int tid = threadIdx.x;
    // S staged in LDS with one coalesced pass when it fits (pop x prompts <= 4096): the sequential
    // fixed-order loops below then read LDS instead of issuing one dependent global load per step
    if (n * m <= 4096) {
        for (int i = tid; i < n * m; i += blockDim.x) s_S[i] = S[i];
        __syncthreads();
        S = s_S;
    }
    // column means (thread j, sequential over k)
    for (int jj = tid; jj < m; jj += blockDim.x) {
        float acc = 0.0f;
#pragma unroll 16
        for (int k = 0; k < n; ++k) acc = acc + S[(int64_t)k * m + jj];
        const float v = acc / (float)n;
        s_mu[jj] = v;
        mu[jj] = v;
    }
    __syncthreads();
    if (promptnorm) {
        for (int k = tid; k < n; k += blockDim.x) {
            float acc = 0.0f;
            for (int jj = 0; jj < m; ++jj) {
                const float c = S[(int64_t)k * m + jj] - s_mu[jj];
                acc = acc + c * c;
            }
            s_row[k] = acc;
        }
        __syncthreads();
        if (tid == 0) {
            float ss = 0.0f;
#pragma unroll 16
            for (int k = 0; k < n; ++k) ss = ss + s_row[k];
            float sb = sqrtf(ss / (float)(n * m));
            if (sb < pn_eps) sb = pn_eps;  // clamp_min(eps) keeps NaN
            s_misc[0] = sb;
        }
        __syncthreads();
        const float sb = s_misc[0];
        for (int k = tid; k < n; k += blockDim.x) {
            float acc = 0.0f;
            for (int jj = 0; jj < m; ++jj) acc = acc + (S[(int64_t)k * m + jj] - s_mu[jj]) / sb;
            s_sc[k] = acc / (float)m;
        }
    } else {
        for (int k = tid; k < n; k += blockDim.x) {
            float acc = 0.0f;
            for (int jj = 0; jj < m; ++jj) acc = acc + S[(int64_t)k * m + jj];
            s_sc[k] = acc / (float)m;
        }
    }
    __syncthreads();
    if (tid == 0) {
        int nf = 0;
        float sum = 0.0f;
#pragma unroll 16
        for (int k = 0; k < n; ++k)
            if (isfinite(s_sc[k])) { sum = sum + s_sc[k]; ++nf; }
        const float mean = sum / (float)nf;
        float sq = 0.0f;
#pragma unroll 16
        for (int k = 0; k < n; ++k)
            if (isfinite(s_sc[k])) { const float d = s_sc[k] - mean; sq = sq + d * d; }
        const float std = sqrtf(sq / (float)(nf - 1));  // torch.std unbiased; nf==1 -> NaN
        s_misc[1] = (float)nf;
        s_misc[2] = mean;
        s_misc[3] = std;
        stats[0] = promptnorm ? s_misc[0] : __builtin_nanf("");
        stats[1] = (float)nf;
        stats[2] = mean;
        stats[3] = std;
    }
    __syncthreads();
    const float mean = s_misc[2], std = s_misc[3];
    const bool degenerate = std < 1e-8f;  // NaN std is not degenerate (reference quirk)
    for (int k = tid; k < n; k += blockDim.x) {
        const float s = s_sc[k];
        const bool fin = isfinite(s);
        scores[k] = s;
        finite[k] = fin ? 1 : 0;
        fit[k] = fin ? (degenerate ? 0.0f : (s - mean) / (std + 1e-8f)) : 0.0f;
        int rank = 0;
#pragma unroll 16
        for (int i = 0; i < n; ++i) {
            const float o = s_sc[i];
            rank += lt_nan_last(o, s) || (i < k && eq_nan(o, s));
        }
        order[rank] = k;
    }
}

// ------------------------------------------------------------------------------------
// (4) update: theta' = theta + lr * (1/N_f) sum_j c_j E_j per tile (c_j = antithetic-collapsed
// fitness), then the norm caps.  With caps enabled every workgroup also writes its fp64 partial
// sums {|d|^2, |theta'|^2, theta.d, |theta|^2}; k_update_caps reduces them in a FIXED order
// (bit-reproducible on every rank) and rescales only if a cap triggers.
// ------------------------------------------------------------------------------------
struct UpdScalars {  // tail of the update workspace
    double step_scale, theta_scale;
    int32_t step_on, theta_on, nf, pad;
};

__device__ __forceinline__ void norm_acc(double (&part)[4], float v, float th) {
    const double d = (double)v - (double)th;
    part[0] += d * d;
    part[1] += (double)v * (double)v;
    part[2] += (double)th * d;
    part[3] += (double)th * (double)th;
}

template <int KIND, int R, int NU, bool V4, bool NORMS, bool GEN>
__device__ __forceinline__ void update_fast(const float* __restrict__ theta, const FacSrc& src,
                                            int64_t n_base, const float* __restrict__ s_c, int nf,
                                            const eggroll_mat_t& mt, int64_t tidx, float sqrt_r, float lr,
                                            float* __restrict__ out, double (&part)[4]) {
#pragma clang fp contract(off)
    using G = FastGeo<KIND, NU>;
    constexpr int NX = KIND == T_VEC4 ? 1 : R;
    constexpr int NW = KIND == T_VEC4 ? 1 : NU * R;
    const int lane = threadIdx.x & 63;
    const int64_t lng = KIND == T_WIDE ? mt.cols : mt.rows;
    const int64_t p0 = tidx * 1024 + 4 * (int64_t)threadIdx.x;
    const bool ok = p0 < lng;
    float4 TH[NU];
#pragma unroll
    for (int i = 0; i < NU; ++i) TH[i] = ok ? ld4<V4>(theta + G::th_off(mt, p0, i)) : float4{0, 0, 0, 0};
    float acc[4][NU];
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int u = 0; u < NU; ++u) acc[v][u] = 0.0f;
    const int64_t xo = G::x_off(mt, R) + p0 * (KIND == T_VEC4 ? 1 : R);
    const int64_t uo = G::u_off(mt, R);
    if (nf > 0) {
        for (int64_t g = 0; g < n_base; g += 64) {
            // lane l: base g+l's uniform factors; rank 1 pre-multiplies c_j into them (w = c_j a_j[u]),
            // the other ranks keep eps_j = (sum_q a b) / sqrt(r) and multiply by c_j afterwards
            float W[NW], C;
            {
                const int64_t jl = g + lane;
                const bool jok = jl < n_base;
                C = jok ? s_c[jl] : 0.0f;
                load_uniform<KIND, NW, GEN>(W, src, jl, uo, KIND != T_VEC4 && jok);
#pragma unroll
                for (int w = 0; w < NW; ++w) W[w] = (R == 1 && KIND != T_VEC4) ? C * W[w] : W[w];
            }
            const int n = (int)((n_base - g) < 64 ? (n_base - g) : 64);
            constexpr int PG = PGrp<KIND, R, true>::value;
            // rank >= 2: software-pipelined — the next group's long factors are in flight while this
            // group's eps math runs (rank 4 at configs[3]: 559 -> 432 us with one base sample per group,
            // 3 % faster than two; a pure read of the same stream runs 367 us); rank 1 keeps one group in
            // registers (the second set costs an occupancy step there: 24.7 -> 27.0 us at pop 64)
            constexpr bool PF = EGG_UPD_PREFETCH && R >= 2 && KIND != T_VEC4 && !GEN;  // nothing to prefetch when regenerated
            float4 XN[PF ? PG : 1][NX];
            auto load_grp = [&](float4 (&D)[PF ? PG : 1][NX], int j0) {
#pragma unroll
                for (int t = 0; t < (PF ? PG : 1); ++t)
#pragma unroll
                    for (int c = 0; c < NX; ++c)
                        D[t][c] = (ok && j0 + t < n) ? fac4<GEN>(src, g + j0 + t, xo + 4 * c) : float4{0, 0, 0, 0};
            };
            if constexpr (PF) load_grp(XN, 0);
            for (int j0 = 0; j0 < n; j0 += PG) {
                float4 X[PG][NX];
                if constexpr (PF) {
#pragma unroll
                    for (int t = 0; t < PG; ++t)
#pragma unroll
                        for (int c = 0; c < NX; ++c) X[t][c] = XN[t % (PF ? PG : 1)][c];
                    if (j0 + PG < n) load_grp(XN, j0 + PG);
                } else {
#pragma unroll
                    for (int t = 0; t < PG; ++t)
#pragma unroll
                        for (int c = 0; c < NX; ++c)
                            X[t][c] = (ok && j0 + t < n) ? fac4<GEN>(src, g + j0 + t, xo + 4 * c) : float4{0, 0, 0, 0};
                }
#pragma unroll
                for (int t = 0; t < PG; ++t) {
                    if (j0 + t >= n) break;
                    const float cj = bcast(C, j0 + t);
                    float wb[NW];
                    bcast_all(wb, W, j0 + t);
#pragma unroll
                    for (int v = 0; v < 4; ++v)
#pragma unroll
                        for (int u = 0; u < NU; ++u) {
                            if constexpr (KIND == T_VEC4) {
                                acc[v][u] = acc[v][u] + cj * f4(X[t][0], v);
                            } else if constexpr (R == 1) {
                                acc[v][u] = acc[v][u] + wb[u] * f4(X[t][0], v);
                            } else {
                                const float e = fast_eps<KIND, R, NU>(X[t], wb, v, u, sqrt_r);
                                acc[v][u] = acc[v][u] + cj * e;
                            }
                        }
                }
            }
        }
    }
    float4 O[NU];
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const float th = f4(TH[G::vi(v, u)], G::vc(v, u));
            float val = th;
            if (nf > 0) {
                const float gq = acc[v][u] / (float)nf;
                const float t = lr * gq;
                val = th + t;
            }
            f4set(O[G::vi(v, u)], G::vc(v, u), val);
            if (NORMS && ok) norm_acc(part, val, th);
        }
    if (ok) {
#pragma unroll
        for (int i = 0; i < NU; ++i) st4<V4>(out + G::th_off(mt, p0, i), O[i]);
    }
}

template <bool VEC1D, bool NORMS, bool GEN>
__device__ __forceinline__ void update_chunk(const float* __restrict__ theta, const FacSrc& src,
                                             int64_t n_base, const float* __restrict__ s_c, int nf,
                                             const eggroll_mat_t& mt, int64_t cidx, int r, float sqrt_r, float lr,
                                             float* __restrict__ out, double (&part)[4]) {
#pragma clang fp contract(off)
    const Slots sl = make_slots<VEC1D>(mt, cidx, threadIdx.x);
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (nf > 0) {
        // sum_j c_j eps_j in base order j = 0, 1, ...
#pragma unroll 2
        for (int64_t j = 0; j < n_base; ++j) {
            const float cj = s_c[j];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float ev = eps_rc<VEC1D, GEN>(mt, src, j, sl.ok[s] ? sl.row[s] : 0, sl.ok[s] ? sl.col[s] : 0, r,
                                                    sqrt_r);
                acc[s] = acc[s] + cj * ev;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if (!sl.ok[s]) continue;
        const int64_t e = mt.theta_off + (VEC1D ? sl.row[s] : sl.row[s] * (int)mt.cols + sl.col[s]);
        const float th = theta[e];
        float v = th;
        if (nf > 0) {
            const float g = acc[s] / (float)nf;
            const float t = lr * g;
            v = th + t;
        }
        out[e] = v;
        if (NORMS) norm_acc(part, v, th);
    }
}

template <int R, bool V4, bool NORMS, bool GEN>
__global__ __launch_bounds__(256) void k_update(const float* __restrict__ theta, FacSrc src,
                                                int64_t n_base, const float* __restrict__ fit,
                                                const float* __restrict__ stats, int32_t pop, int32_t antithetic,
                                                const eggroll_mat_t* __restrict__ mats,
                                                const eggroll_tile_t* __restrict__ tiles, int r, float sqrt_r,
                                                float lr, float* __restrict__ out, double* __restrict__ partials) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float s_c[];  // [n_base]
    __shared__ double s_red[4][4];
    const int tid = threadIdx.x;
    const eggroll_tile_t tl = tiles[blockIdx.x];
    const eggroll_mat_t mt = mats[tl.mat];
    const int nf = (int)stats[1];
    // the unpaired last member (odd pop) is read at an index clamped into [0, pop): its address is
    // uniform, so the compiler issues it as a scalar load, which runs even when no lane takes the
    // branch — at even pop an unclamped fit[2h] read one float past the fitness vector (a fault
    // when that vector ends a mapped segment)
    const int64_t h = pop / 2, lastk = (2 * h < pop) ? 2 * h : pop - 1;
    for (int64_t j = tid; j < n_base; j += blockDim.x) {
        float c;
        if (!antithetic) {
            c = fit[j];
        } else {
            c = (j < h) ? fit[j] - fit[j + h] : fit[lastk];
        }
        s_c[j] = c;
    }
    __syncthreads();
    double part[4] = {0.0, 0.0, 0.0, 0.0};
    dispatch_tile<R, V4>(
        mt, r,
        [&](auto KD, auto NUv) {
            constexpr int KK = decltype(KD)::value;
            if constexpr (KK == T_VEC4)
                update_fast<T_VEC4, 1, 1, V4, NORMS, GEN>(theta, src, n_base, s_c, nf, mt, tl.index, sqrt_r, lr,
                                                          out, part);
            else if constexpr (R > 0)
                update_fast<KK, R, decltype(NUv)::value, V4, NORMS, GEN>(theta, src, n_base, s_c, nf, mt,
                                                                         tl.index, sqrt_r, lr, out, part);
        },
        [&](auto VD) {
            update_chunk<decltype(VD)::value, NORMS, GEN>(theta, src, n_base, s_c, nf, mt, tl.index, r, sqrt_r,
                                                          lr, out, part);
        });
    if constexpr (NORMS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) part[q] = wave_sum_d(part[q]);
        const int w = tid >> 6, lane = tid & 63;
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) s_red[w][q] = part[q];
        }
        __syncthreads();
        if (tid < 4) partials[(int64_t)blockIdx.x * 4 + tid] = (s_red[0][tid] + s_red[1][tid]) + (s_red[2][tid] + s_red[3][tid]);
    }
}

// Caps (utills.py:333-349: cap_step_norm then cap_theta_norm).  EVERY workgroup reduces all the
// per-tile partials in the same fixed order (thread t: tiles t, t+256, ... sequentially, then a
// fixed LDS tree), so every workgroup — and every rank — derives bit-identical scales with no
// cross-workgroup handshake; then, only if a cap triggers, the grid rescales theta' (grid-stride).
__global__ __launch_bounds__(256) void k_update_caps(const float* __restrict__ theta, int64_t D,
                                                     const double* __restrict__ partials, int64_t n_part,
                                                     const float* __restrict__ stats, float max_step, float max_theta,
                                                     UpdScalars* __restrict__ sc, float* __restrict__ out) {
#pragma clang fp contract(off)
    __shared__ double s[4][4];
    __shared__ float s_scale[2];
    __shared__ int s_on[2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double a[4] = {0, 0, 0, 0};
    for (int64_t c0 = 0; c0 < n_part; c0 += 1024) {  // 4 independent 32-byte loads per thread in flight
        double4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t c = c0 + u * 256 + tid;
            v[u] = c < n_part ? reinterpret_cast<const double4*>(partials)[c] : double4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[0] += v[u].x;
            a[1] += v[u].y;
            a[2] += v[u].z;
            a[3] += v[u].w;
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = wave_sum_d(a[q]);  // fixed butterfly order: same bits everywhere
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) s[w][q] = a[q];
    __syncthreads();
    if (tid == 0) {
        const double dd = (s[0][0] + s[1][0]) + (s[2][0] + s[3][0]), oo = (s[0][1] + s[1][1]) + (s[2][1] + s[3][1]);
        const double td = (s[0][2] + s[1][2]) + (s[2][2] + s[3][2]), tt = (s[0][3] + s[1][3]) + (s[2][3] + s[3][3]);
        const int nf = (int)stats[1];
        const double dn = sqrt(dd);
        const int step_on = (nf > 0) && (max_step > 0.0f) && (dn > (double)max_step);
        const double ss = step_on ? (double)max_step / (dn + 1e-8) : 1.0;
        const double n2 = step_on ? (tt + 2.0 * ss * td + ss * ss * dd) : oo;
        const double tn = sqrt(n2 > 0.0 ? n2 : 0.0);
        // no finite member: the reference returns theta unchanged, caps included (unifed_es.py:237-240)
        const int theta_on = (nf > 0) && (max_theta > 0.0f) && (tn > (double)max_theta);
        const double ts = theta_on ? (double)max_theta / (tn + 1e-8) : 1.0;
        s_on[0] = step_on;
        s_on[1] = theta_on;
        s_scale[0] = (float)ss;
        s_scale[1] = (float)ts;
        if (blockIdx.x == 0) {
            sc->step_scale = ss;
            sc->theta_scale = ts;
            sc->step_on = step_on;
            sc->theta_on = theta_on;
            sc->nf = nf;
        }
    }
    __syncthreads();
    const int step_on = s_on[0], theta_on = s_on[1];
    if (!step_on && !theta_on) return;
    const float ss = s_scale[0], ts = s_scale[1];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + tid; i < D; i += (int64_t)gridDim.x * blockDim.x) {
        float v = out[i];
        if (step_on) {
            const float th = theta[i];
            const float d = v - th;
            v = th + d * ss;
        }
        if (theta_on) v = v * ts;
        out[i] = v;
    }
}

}  // namespace eggroll

using namespace eggroll;

// ======================================================================================
// C-ABI
// ======================================================================================
extern "C" {

const char* eggroll_version(void) { return "eggroll-mi355x 0.1.0 (gfx950)"; }
const char* eggroll_last_error(void) { return g_err; }

int eggroll_noise_factors(uint64_t seed, int64_t base_lo, int64_t base_hi, int64_t factor_len, int64_t ld,
                          float* out, void* stream) {
    EGG_CHECK_ARG(base_lo >= 0 && base_hi >= base_lo, "noise_factors: bad base range [%lld,%lld)",
                  (long long)base_lo, (long long)base_hi);
    EGG_CHECK_ARG(factor_len >= 0 && ld >= factor_len && ld % 4 == 0, "noise_factors: need ld >= factor_len, ld %% 4 == 0");
    EGG_CHECK_ARG(base_hi - base_lo <= 65535, "noise_factors: at most 65535 base samples per call");
    if (base_hi == base_lo || factor_len == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(out != nullptr, "noise_factors: out is NULL");
    const int64_t quads = (factor_len + 3) / 4;
    dim3 grid((unsigned)((quads + 256 * NOISE_QPT - 1) / (256 * NOISE_QPT)), (unsigned)(base_hi - base_lo));
    hipLaunchKernelGGL(k_noise, grid, dim3(256), 0, as_stream(stream), (uint32_t)seed, (uint32_t)(seed >> 32),
                       base_lo, factor_len, ld, out);
    EGG_CHECK_LAUNCH("noise_factors");
    return EGGROLL_OK;
}

int eggroll_philox_words(uint64_t seed, int64_t j, int64_t n_quads, uint32_t* out, void* stream) {
    EGG_CHECK_ARG(n_quads >= 0 && (n_quads == 0 || out), "philox_words: bad args");
    if (!n_quads) return EGGROLL_OK;
    hipLaunchKernelGGL(k_philox_words, dim3((unsigned)((n_quads + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (uint32_t)seed, (uint32_t)(seed >> 32), j, n_quads, out);
    EGG_CHECK_LAUNCH("philox_words");
    return EGGROLL_OK;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

#ifndef EGG_PTB_SPLIT  // perturb: target workgroup count for the member split over grid.y (0: no split; A/B knob)
#define EGG_PTB_SPLIT 4096
#endif
#ifndef EGG_PTB_MIN_GROUP
#define EGG_PTB_MIN_GROUP 16
#endif

static int launch_rank(int32_t rank) { return (rank == 1 || rank == 2 || rank == 4) ? rank : 0; }

static int perturb_launch(const float* theta, FacSrc src, bool gen, const eggroll_mat_t* mats,
                          const eggroll_tile_t* tiles, int64_t n_tiles, int64_t D, int32_t rank, int32_t pop,
                          int32_t antithetic, int64_t member_lo, int64_t member_hi, float sigma, float* out,
                          int64_t ld_out, void* stream) {
    EGG_CHECK_ARG(member_hi - member_lo <= 65535, "perturb: at most 65535 members per call");
    EGG_CHECK_ARG(n_tiles >= 1 && n_tiles < (1ll << 31), "perturb: bad n_tiles");
    if (member_hi == member_lo || D == 0) return EGGROLL_OK;
    const float sqrt_r = (float)sqrt((double)rank);
    const bool v4 = (theta == nullptr || al16(theta)) && al16(out) && ld_out % 4 == 0;
#define EGG_PTB_K(RV) (gen ? (v4 ? k_perturb<RV, true, true> : k_perturb<RV, false, true>) \
                           : (v4 ? k_perturb<RV, true, false> : k_perturb<RV, false, false>))
    auto* k = launch_rank(rank) == 1 ? EGG_PTB_K(1) : launch_rank(rank) == 2 ? EGG_PTB_K(2)
            : launch_rank(rank) == 4 ? EGG_PTB_K(4) : EGG_PTB_K(0);
#undef EGG_PTB_K
    // A launch of n_tiles workgroups that walk every member is one wave round at the product sizes (Sana:
    // ~1500 tiles x 4 waves), each thread a serial chain of per-member factor loads / Philox + stores.
    // With many members (>= 2 x EGG_PTB_MIN_GROUP) the members are split over grid.y until ~EGG_PTB_SPLIT
    // workgroups exist (theta re-read once per group, from L2): Sana, all 64 members in one call 95.8 ->
    // 85.7 us.  Splitting 8 members (one GPU's share of pop 64) measured 14.3 -> 24.1 us (per-workgroup
    // setup and the regenerated factors' VALU, not memory, bound it), so groups keep >= 16 members.
    // Same bits either way: each member row is computed the same way (profiles/r13b_es_perturb_split_ab.log).
    const int n = (int)(member_hi - member_lo);
    int ny = 1;
    if (EGG_PTB_SPLIT > 0 && n_tiles < EGG_PTB_SPLIT && n >= 2 * EGG_PTB_MIN_GROUP) {
        const int64_t want = (EGG_PTB_SPLIT + n_tiles - 1) / n_tiles, cap = n / EGG_PTB_MIN_GROUP;
        ny = (int)(want < cap ? want : cap);
    }
    const int mpb = (n + ny - 1) / ny;
    ny = (n + mpb - 1) / mpb;
    hipLaunchKernelGGL(k, dim3((unsigned)n_tiles, (unsigned)ny), dim3(256), 0, as_stream(stream), theta, src, mats,
                       tiles, rank, sqrt_r, pop, antithetic, member_lo, n, mpb, sigma, out, ld_out);
    EGG_CHECK_LAUNCH("perturb");
    return EGGROLL_OK;
}

int eggroll_perturb(const float* theta, const float* factors, int64_t ld_f, int64_t n_base,
                    const eggroll_mat_t* mats, const eggroll_tile_t* tiles, int64_t n_tiles, int64_t D, int32_t rank,
                    int32_t pop, int32_t antithetic, int64_t member_lo, int64_t member_hi, float sigma, float* out,
                    int64_t ld_out, void* stream) {
    EGG_CHECK_ARG(rank >= 1, "perturb: rank must be >= 1");
    EGG_CHECK_ARG(pop >= 1 && member_lo >= 0 && member_hi <= pop && member_lo <= member_hi,
                  "perturb: members [%lld,%lld) outside pop %d", (long long)member_lo, (long long)member_hi, pop);
    EGG_CHECK_ARG(mats && tiles && factors && out && ld_out >= D, "perturb: bad pointers/sizes");
    EGG_CHECK_ARG(al16(factors) && ld_f % 4 == 0, "perturb: factors must be 16-byte aligned with ld_f %% 4 == 0");
    const int64_t need_base = antithetic ? (pop / 2 + (pop % 2)) : pop;
    EGG_CHECK_ARG(n_base >= need_base, "perturb: n_base %lld < %lld needed", (long long)n_base, (long long)need_base);
    return perturb_launch(theta, FacSrc{factors, ld_f, 0u, 0u}, false, mats, tiles, n_tiles, D, rank, pop, antithetic,
                          member_lo, member_hi, sigma, out, ld_out, stream);
}

int eggroll_perturb_seeded(uint64_t seed, const float* theta, const eggroll_mat_t* mats, const eggroll_tile_t* tiles,
                           int64_t n_tiles, int64_t D, int32_t rank, int32_t pop, int32_t antithetic,
                           int64_t member_lo, int64_t member_hi, float sigma, float* out, int64_t ld_out,
                           void* stream) {
    EGG_CHECK_ARG(rank >= 1, "perturb_seeded: rank must be >= 1");
    EGG_CHECK_ARG(pop >= 1 && member_lo >= 0 && member_hi <= pop && member_lo <= member_hi,
                  "perturb_seeded: members [%lld,%lld) outside pop %d", (long long)member_lo, (long long)member_hi, pop);
    EGG_CHECK_ARG(mats && tiles && out && ld_out >= D, "perturb_seeded: bad pointers/sizes");
    return perturb_launch(theta, FacSrc{nullptr, 0, (uint32_t)seed, (uint32_t)(seed >> 32)}, true, mats, tiles,
                          n_tiles, D, rank, pop, antithetic, member_lo, member_hi, sigma, out, ld_out, stream);
}

int eggroll_fitness(const float* S, int32_t n, int32_t m, int32_t use_promptnorm, float promptnorm_eps, float* scores,
                    float* mu, float* stats, float* fitness, int32_t* finite, int32_t* order, void* stream) {
    EGG_CHECK_ARG(n >= 1 && n <= 4096 && m >= 1 && m <= 1024, "fitness: need 1<=n<=4096, 1<=m<=1024 (got %d,%d)", n, m);
    EGG_CHECK_ARG(S && scores && mu && stats && fitness && finite && order, "fitness: NULL pointer");
    EGG_CHECK_ARG(!(promptnorm_eps < 0.0f), "fitness: promptnorm_eps must be >= 0");
    hipLaunchKernelGGL(k_fitness, dim3(1), dim3(1024), 0, as_stream(stream), S, n, m, use_promptnorm, promptnorm_eps,
                       scores, mu,
                       stats, fitness, finite, order);
    EGG_CHECK_LAUNCH("fitness");
    return EGGROLL_OK;
}

int64_t eggroll_update_workspace_bytes(int64_t n_tiles) {
    return n_tiles * 4 * (int64_t)sizeof(double) + 64;
}

static int update_launch(const float* theta, FacSrc src, bool gen, int64_t n_base, const float* fitness,
                         const float* stats, int32_t pop, int32_t antithetic, const eggroll_mat_t* mats,
                         const eggroll_tile_t* tiles, int64_t n_tiles, int64_t D, int32_t rank, float lr,
                         float max_step_norm, float theta_max_norm, void* workspace, float* theta_out, void* stream) {
    EGG_CHECK_ARG(n_base <= 16384, "update: n_base > 16384 unsupported");
    EGG_CHECK_ARG(n_tiles >= 1 && n_tiles < (1ll << 31), "update: bad n_tiles");
    EGG_CHECK_ARG(al16(workspace), "update: workspace must be 16-byte aligned");
    if (D == 0) return EGGROLL_OK;
    const float sqrt_r = (float)sqrt((double)rank);
    double* partials = reinterpret_cast<double*>(workspace);
    UpdScalars* sc = reinterpret_cast<UpdScalars*>(partials + n_tiles * 4);
    hipStream_t st = as_stream(stream);
    const bool v4 = al16(theta) && al16(theta_out);
    const bool caps = max_step_norm > 0.0f || theta_max_norm > 0.0f;
    const int lr_ = launch_rank(rank);
#define EGG_UPD_K(RV, V4V, NV) (gen ? k_update<RV, V4V, NV, true> : k_update<RV, V4V, NV, false>)
#define EGG_UPD_PICK(RV) (v4 ? (caps ? EGG_UPD_K(RV, true, true) : EGG_UPD_K(RV, true, false)) \
                             : (caps ? EGG_UPD_K(RV, false, true) : EGG_UPD_K(RV, false, false)))
    auto* k = lr_ == 1 ? EGG_UPD_PICK(1) : lr_ == 2 ? EGG_UPD_PICK(2) : lr_ == 4 ? EGG_UPD_PICK(4) : EGG_UPD_PICK(0);
#undef EGG_UPD_PICK
#undef EGG_UPD_K
    hipLaunchKernelGGL(k, dim3((unsigned)n_tiles), dim3(256), (size_t)n_base * sizeof(float), st, theta, src,
                       n_base, fitness, stats, pop, antithetic, mats, tiles, rank, sqrt_r, lr, theta_out, partials);
    EGG_CHECK_LAUNCH("update");
    if (caps) {
        // every block re-reduces all per-tile partials (fixed order) before deciding, so the decision
        // costs blocks x n_tiles x 32 B of L2 reads; 64 blocks still rescale D in one sweep if a cap fires
        int64_t blocks = (D + 1023) / 1024;
        if (blocks > 64) blocks = 64;
        hipLaunchKernelGGL(k_update_caps, dim3((unsigned)blocks), dim3(256), 0, st, theta, D, partials, n_tiles, stats,
                           max_step_norm, theta_max_norm, sc, theta_out);
        EGG_CHECK_LAUNCH("update_caps");
    }
    return EGGROLL_OK;
}

int eggroll_update(const float* theta, const float* factors, int64_t ld_f, int64_t n_base, const float* fitness,
                   const float* stats, int32_t pop, int32_t antithetic, const eggroll_mat_t* mats,
                   const eggroll_tile_t* tiles, int64_t n_tiles, int64_t D, int32_t rank, float lr,
                   float max_step_norm, float theta_max_norm, void* workspace, float* theta_out, void* stream) {
    EGG_CHECK_ARG(rank >= 1 && pop >= 1, "update: bad rank/pop");
    EGG_CHECK_ARG(theta && factors && fitness && stats && mats && tiles && workspace && theta_out, "update: NULL pointer");
    EGG_CHECK_ARG(theta != theta_out, "update: theta_out may not alias theta");
    EGG_CHECK_ARG(al16(factors) && ld_f % 4 == 0, "update: factors must be 16-byte aligned with ld_f %% 4 == 0");
    const int64_t need_base = antithetic ? (pop / 2 + (pop % 2)) : pop;
    EGG_CHECK_ARG(n_base == need_base, "update: n_base %lld != %lld", (long long)n_base, (long long)need_base);
    return update_launch(theta, FacSrc{factors, ld_f, 0u, 0u}, false, n_base, fitness, stats, pop, antithetic, mats,
                         tiles, n_tiles, D, rank, lr, max_step_norm, theta_max_norm, workspace, theta_out, stream);
}

int eggroll_update_seeded(uint64_t seed, const float* theta, const float* fitness, const float* stats, int32_t pop,
                          int32_t antithetic, const eggroll_mat_t* mats, const eggroll_tile_t* tiles, int64_t n_tiles,
                          int64_t D, int32_t rank, float lr, float max_step_norm, float theta_max_norm,
                          void* workspace, float* theta_out, void* stream) {
    EGG_CHECK_ARG(rank >= 1 && pop >= 1, "update_seeded: bad rank/pop");
    EGG_CHECK_ARG(theta && fitness && stats && mats && tiles && workspace && theta_out, "update_seeded: NULL pointer");
    EGG_CHECK_ARG(theta != theta_out, "update_seeded: theta_out may not alias theta");
    const int64_t n_base = antithetic ? (pop / 2 + (pop % 2)) : pop;
    return update_launch(theta, FacSrc{nullptr, 0, (uint32_t)seed, (uint32_t)(seed >> 32)}, true, n_base, fitness,
                         stats, pop, antithetic, mats, tiles, n_tiles, D, rank, lr, max_step_norm, theta_max_norm,
                         workspace, theta_out, stream);
}

int64_t eggroll_tile_table(const eggroll_mat_t* mats_host, int32_t n_mats, int32_t rank, eggroll_tile_t* tiles_host,
                           int64_t capacity) {
    if (!mats_host || n_mats < 1 || rank < 1) {
        set_error("tile_table: need mats_host, n_mats >= 1, rank >= 1");
        return EGGROLL_ERR_ARG;
    }
    int64_t n = 0;
    for (int32_t i = 0; i < n_mats; ++i) {
        const eggroll_mat_t& mt = mats_host[i];
        if (mt.rows < 1 || mt.cols < 0) {
            set_error("tile_table: mat %d has rows=%lld cols=%lld", i, (long long)mt.rows, (long long)mt.cols);
            return EGGROLL_ERR_ARG;
        }
        // the generic per-element path (T_VEC / T_GEN) indexes elements in 32-bit ints
        const int kind = egg_tile_kind(mt, rank);
        const int64_t numel = mt.cols ? mt.rows * mt.cols : mt.rows;
        if ((kind == T_VEC || kind == T_GEN) && numel >= (1ll << 31) - EGGROLL_CHUNK) {
            set_error("tile_table: mat %d (%lld elements) is too large for the generic per-element path", i,
                      (long long)numel);
            return EGGROLL_ERR_ARG;
        }
        const int64_t c = egg_tile_count(mt, rank);
        for (int64_t t = 0; t < c; ++t, ++n) {
            if (tiles_host && n < capacity) {
                tiles_host[n].mat = i;
                tiles_host[n].index = (int32_t)t;
            }
        }
    }
    return n;
}

}  // extern "C"
