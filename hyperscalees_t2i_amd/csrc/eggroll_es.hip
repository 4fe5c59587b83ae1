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

__global__ __launch_bounds__(256) void k_noise(uint32_t k0, uint32_t k1, int64_t base_lo,
                                               int64_t factor_len, int64_t ld, float* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t g0 = q * 4;
    if (g0 >= factor_len) return;
    const int64_t j = base_lo + blockIdx.y;
    u32x4 c{(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)j, kNoiseTag};
    const u32x4 w = philox4x32_10_dev(c, k0, k1);
    float4 v;
    box_muller(w.x, w.y, v.x, v.y);
    box_muller(w.z, w.w, v.z, v.w);
    float* dst = out + (int64_t)blockIdx.y * ld + g0;
    if (g0 + 4 <= factor_len) {
        *reinterpret_cast<float4*>(dst) = v;
    } else {
        const float t[4] = {v.x, v.y, v.z, v.w};
        for (int i = 0; i < 4 && g0 + i < factor_len; ++i) dst[i] = t[i];
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

// Matrix owning work chunk `chunk`: the number of matrices whose chunk_off <= chunk, minus one
// (chunk_off is a prefix sum).  Every lane tests one matrix per step and a ballot counts — the
// loads are independent (one memory latency for <= 256 matrices) instead of a binary search's
// log2(n) dependent ones.  Wave-uniform result.
__device__ __forceinline__ int find_mat(const eggroll_mat_t* __restrict__ mats, int n_mats, int64_t chunk) {
    const int lane = threadIdx.x & 63;
    int cnt = 0;
    for (int b = 0; b < n_mats; b += 256) {
        int64_t co[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {  // four independent loads in flight
            const int i = b + 64 * t + lane;
            co[t] = i < n_mats ? mats[i].chunk_off : INT64_MAX;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) cnt += __popcll(__ballot(co[t] <= chunk));
    }
    return __builtin_amdgcn_readfirstlane(cnt - 1);
}

// ------------------------------------------------------------------------------------
// Chunk work decomposition shared by perturb and update.  A chunk is EGGROLL_CHUNK = 1024
// elements of one matrix (host prefix table); each of the 256 threads owns 4 element slots:
//   VEC   1-D parameter (eps = the factor itself): e = e0 + tid + 256 u
//   WIDE  rows in {1,2,4} <= cols (PEFT lora_A [r_l, in]): the chunk is 1024/rows whole columns;
//         slot (u, row) = column c0 + tid + 256 u of every row — b loads coalesced, a[row]
//         block-uniform (scalar loads), no integer division
//   TALL  cols in {1,2,4} < rows (lora_B [out, r_l]): the chunk is 1024/cols whole rows;
//         slot (u, col) = row r0 + tid + 256 u — a loads coalesced, b[col] block-uniform
//   GEN   anything else: e = e0 + tid + 256 u, row/col by one 32-bit division per slot
// Every slot's eps is computed with exactly the same fp32 operation order as the reference
// restatement (a[0] b[0] + a[1] b[1] + ...) / sqrt(r), so the result does not depend on the kind.
// ------------------------------------------------------------------------------------
enum ChunkKind { K_VEC = 0, K_WIDE = 1, K_TALL = 2, K_GEN = 3 };

__device__ __forceinline__ int chunk_kind(const eggroll_mat_t& mt) {
    if (mt.cols == 0) return K_VEC;
    if (mt.rows <= mt.cols && (mt.rows == 1 || mt.rows == 2 || mt.rows == 4)) return K_WIDE;
    if (mt.cols < mt.rows && (mt.cols == 1 || mt.cols == 2 || mt.cols == 4)) return K_TALL;
    return K_GEN;
}

struct Slots {  // this thread's element slots inside one chunk
    int row[4], col[4];
    bool ok[4];
};

template <int KIND>
__device__ __forceinline__ Slots make_slots(const eggroll_mat_t& mt, int64_t cidx, int tid) {
    Slots sl;
    const int rows = (int)mt.rows, cols = (int)mt.cols;
    if constexpr (KIND == K_WIDE) {
        const int cpc = EGGROLL_CHUNK / rows, c0 = (int)cidx * cpc;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int u = s / rows, rr = s % rows;  // rows is 1, 2 or 4: 4 / rows column groups
            const int c = c0 + tid + 256 * u;
            sl.row[s] = rr;
            sl.col[s] = c;
            sl.ok[s] = (s < 4) && (u < 4 / rows) && (c < c0 + cpc) && (c < cols);
        }
    } else if constexpr (KIND == K_TALL) {
        const int rpc = EGGROLL_CHUNK / cols, r0 = (int)cidx * rpc;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int u = s / cols, cc = s % cols;
            const int r = r0 + tid + 256 * u;
            sl.row[s] = r;
            sl.col[s] = cc;
            sl.ok[s] = (u < 4 / cols) && (r < r0 + rpc) && (r < rows);
        }
    } else {
        const int numel = KIND == K_VEC ? rows : rows * cols;
        const int e0 = (int)cidx * EGGROLL_CHUNK;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int e = e0 + s * 256 + tid;
            sl.ok[s] = e < numel;
            if (KIND == K_VEC) {
                sl.row[s] = e;
                sl.col[s] = 0;
            } else {
                const int r = sl.ok[s] ? e / cols : 0;
                sl.row[s] = r;
                sl.col[s] = e - r * cols;
            }
        }
    }
    return sl;
}

__device__ __forceinline__ int slot_elem(const eggroll_mat_t& mt, const Slots& sl, int s, int kind) {
    return kind == K_VEC ? sl.row[s] : sl.row[s] * (int)mt.cols + sl.col[s];
}

// eps of (row, col) of matrix mt for the base-sample factor row fj (utills.py:59-65 restated)
// R1: egg rank 1 known at compile time — eps = a[row] b[col] (x / sqrt(1) == x exactly), so the
// loads of consecutive base samples carry no loop-carried control flow and batch up.
template <int KIND, bool R1>
__device__ __forceinline__ float eps_rc(const eggroll_mat_t& mt, const float* __restrict__ fj, int row, int col,
                                        int r, float sqrt_r) {
#pragma clang fp contract(off)
    if constexpr (KIND == K_VEC) {
        return fj[mt.factor_off + row];
    } else if constexpr (R1) {
        return fj[mt.factor_off + row] * fj[mt.factor_off + mt.rows + col];
    } else {
        const float* a = fj + mt.factor_off + (int64_t)row * r;
        const float* b = fj + mt.factor_off + mt.rows * r + (int64_t)col * r;
        float acc = a[0] * b[0];
        for (int q = 1; q < r; ++q) acc = acc + a[q] * b[q];
        return acc / sqrt_r;
    }
}

// ------------------------------------------------------------------------------------
// Rank-1 fast paths (egg rank 1, the Sana / BASELINE configuration) for VEC / WIDE / TALL chunks.
// Each element is x_v * w_q: x is the factor along the chunk's long ("vector") dimension (b for
// WIDE, a for TALL, the 1-D sample for VEC) — coalesced loads, one per slot column — and w the
// factor along the short ("uniform") dimension (a[row] for WIDE, b[col] for TALL, 1 for VEC),
// which is the same for the whole block: lane l of every wave holds the uniform factors of base
// sample / member l and the inner loops broadcast them with v_readlane (an SGPR operand), so the
// base loop carries no memory dependency except the x loads.
// ------------------------------------------------------------------------------------
template <int KIND, int NU>
struct R1Map {  // slot s = u * NU + q: vector index vi(u), uniform index q
    static constexpr int NV = 4 / NU;
    __device__ static int64_t xoff(const eggroll_mat_t& mt) {  // factor offset of the vector dimension
        return KIND == K_WIDE ? mt.factor_off + mt.rows : mt.factor_off;
    }
    __device__ static int64_t woff(const eggroll_mat_t& mt) {  // factor offset of the uniform dimension
        return KIND == K_WIDE ? mt.factor_off : mt.factor_off + mt.rows;
    }
};

#ifndef EGG_UPD_GROUP
#define EGG_UPD_GROUP 8  // base samples whose factor loads are in flight together
#endif
template <int KIND, int NU>
__device__ __forceinline__ void update_chunk_r1(const float* __restrict__ theta, const float* __restrict__ factors,
                                                int64_t ld_f, int64_t n_base, const float* __restrict__ s_c, int nf,
                                                const eggroll_mat_t& mt, int64_t cidx, float lr,
                                                float* __restrict__ out, double (&part)[4]) {
#pragma clang fp contract(off)
    using MP = R1Map<KIND, NU>;
    constexpr int NV = MP::NV;
    const Slots sl = make_slots<KIND>(mt, cidx, threadIdx.x);
    const int lane = threadIdx.x & 63;
    int vi[NV];
    bool vok[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        vi[u] = KIND == K_TALL ? sl.row[u * NU] : (KIND == K_WIDE ? sl.col[u * NU] : sl.row[u]);
        vok[u] = sl.ok[u * NU];
    }
    const int64_t xo = MP::xoff(mt), wo = MP::woff(mt);
    uint32_t vbyte[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) vbyte[u] = (uint32_t)vi[u] * 4u;
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (nf > 0) {
        for (int64_t g = 0; g < n_base; g += 64) {
            // lane l: w_q = c_{g+l} * (uniform factor q of base g+l)
            float w[NU];
            const int64_t jl = g + lane;
#pragma unroll
            for (int q = 0; q < NU; ++q) {
                float c = jl < n_base ? s_c[jl] : 0.0f;
                if (KIND != K_VEC) c = jl < n_base ? c * factors[jl * ld_f + wo + q] : 0.0f;
                w[q] = c;
            }
            const int n = (int)((n_base - g) < 64 ? (n_base - g) : 64);
            const float* fg = factors + g * ld_f + xo;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)fg, (short)0, 0x7fffffff, 0x00020000);
            const int ldb = (int)(ld_f * 4);  // host: 64 * ld_f * 4 < 2^31
            // groups of 8 base samples with a compile-time trip count (readlane is convergent: a
            // runtime-count loop around it cannot be unrolled), 8 * NV loads in flight per thread
            for (int j0 = 0; j0 < n; j0 += EGG_UPD_GROUP) {
                float x[EGG_UPD_GROUP][NV];
#pragma unroll
                for (int t = 0; t < EGG_UPD_GROUP; ++t) {
                    // buffer load: uniform row offset in soffset (SGPR), lane byte offset in voffset —
                    // one VGPR per slot column instead of a 64-bit address per (base, slot)
                    const int sb = (j0 + t) * ldb;
#pragma unroll
                    for (int u = 0; u < NV; ++u)
                        x[t][u] = (j0 + t < n && vok[u])
                                      ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vbyte[u], sb, 0))
                                      : 0.0f;
                }
#pragma unroll
                for (int t = 0; t < EGG_UPD_GROUP; ++t) {
                    if (j0 + t >= n) break;
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        const float ws = __builtin_bit_cast(
                            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, w[s % NU]), j0 + t));
                        acc[s] = acc[s] + ws * x[t][s / NU];
                    }
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if (!sl.ok[s]) continue;
        const int64_t e = mt.theta_off + slot_elem(mt, sl, s, KIND);
        const float th = theta[e];
        float v = th;
        if (nf > 0) {
            const float gq = acc[s] / (float)nf;
            const float t = lr * gq;
            v = th + t;
        }
        out[e] = v;
        const double d = (double)v - (double)th;
        part[0] += d * d;
        part[1] += (double)v * (double)v;
        part[2] += (double)th * d;
        part[3] += (double)th * (double)th;
    }
}

template <int KIND, int NU>
__device__ __forceinline__ void perturb_chunk_r1(const float* __restrict__ theta, const float* __restrict__ factors,
                                                 int64_t ld_f, const eggroll_mat_t& mt, int64_t cidx, int32_t pop,
                                                 int32_t antithetic, int64_t member_lo, int n_members, float sigma,
                                                 float* __restrict__ out, int64_t ld_out) {
#pragma clang fp contract(off)
    using MP = R1Map<KIND, NU>;
    constexpr int NV = MP::NV;
    const Slots sl = make_slots<KIND>(mt, cidx, threadIdx.x);
    const int lane = threadIdx.x & 63;
    float th[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
        th[s] = (theta && sl.ok[s]) ? theta[mt.theta_off + slot_elem(mt, sl, s, KIND)] : 0.0f;
    int vi[NV];
    bool vok[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        vi[u] = KIND == K_TALL ? sl.row[u * NU] : (KIND == K_WIDE ? sl.col[u * NU] : sl.row[u]);
        vok[u] = sl.ok[u * NU];
    }
    const int64_t xo = MP::xoff(mt), wo = MP::woff(mt);
    for (int g = 0; g < n_members; g += 64) {
        // lane l: member g+l's base row offset, sign and uniform factors
        int64_t jb;
        float sg;
        member_to_base(member_lo + g + lane, pop, antithetic, jb, sg);
        const bool mok = g + lane < n_members;
        float w[NU];
#pragma unroll
        for (int q = 0; q < NU; ++q) w[q] = (KIND == K_VEC || !mok) ? 1.0f : factors[jb * ld_f + wo + q];
        const int n = (n_members - g) < 64 ? (n_members - g) : 64;
        for (int i = 0; i < n; ++i) {
            int64_t j;
            float sgn;
            member_to_base(member_lo + g + i, pop, antithetic, j, sgn);
            const float* fj = factors + j * ld_f + xo;
            float x[NV];
#pragma unroll
            for (int u = 0; u < NV; ++u) x[u] = vok[u] ? fj[vi[u]] : 0.0f;
            float* dst = out + (int64_t)(g + i) * ld_out + mt.theta_off;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (!sl.ok[s]) continue;
                const float wq = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, w[s % NU]), i));
                // eps = a[row] * b[col] (/ sqrt(1)); the product order a*b is the reference's
                const float prod = KIND == K_VEC ? x[s / NU] : (KIND == K_WIDE ? wq * x[s / NU] : x[s / NU] * wq);
                const float eps = sgn * prod;
                float v;
                if (theta) {
                    const float t = sigma * eps;
                    v = th[s] + t;
                } else {
                    v = sigma * eps;
                }
                dst[slot_elem(mt, sl, s, KIND)] = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// perturb / materialise: out[k] = theta + sigma * s_k * E_j(k) for the members [lo, lo + n).
// One block per chunk; theta is read once and every member's row written from registers.
// ------------------------------------------------------------------------------------
template <int KIND, bool R1>
__device__ __forceinline__ void perturb_chunk(const float* __restrict__ theta, const float* __restrict__ factors,
                                              int64_t ld_f, const eggroll_mat_t& mt, int64_t cidx, int r,
                                              float sqrt_r, int32_t pop, int32_t antithetic, int64_t member_lo,
                                              int n_members, float sigma, float* __restrict__ out, int64_t ld_out) {
#pragma clang fp contract(off)
    const Slots sl = make_slots<KIND>(mt, cidx, threadIdx.x);
    float th[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
        th[s] = (theta && sl.ok[s]) ? theta[mt.theta_off + slot_elem(mt, sl, s, KIND)] : 0.0f;
#pragma unroll 4
    for (int i = 0; i < n_members; ++i) {
        int64_t j;
        float sgn;
        member_to_base(member_lo + i, pop, antithetic, j, sgn);
        const float* fj = factors + j * ld_f;
        float* dst = out + (int64_t)i * ld_out + mt.theta_off;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (!sl.ok[s]) continue;
            const float eps = sgn * eps_rc<KIND, R1>(mt, fj, sl.row[s], sl.col[s], r, sqrt_r);
            float v;
            if (theta) {
                const float t = sigma * eps;
                v = th[s] + t;
            } else {
                v = sigma * eps;
            }
            dst[slot_elem(mt, sl, s, KIND)] = v;
        }
    }
}

template <bool RANK1>
__global__ __launch_bounds__(256) void k_perturb(const float* __restrict__ theta, const float* __restrict__ factors,
                                                 int64_t ld_f, const eggroll_mat_t* __restrict__ mats, int n_mats,
                                                 int r, float sqrt_r, int32_t pop, int32_t antithetic,
                                                 int64_t member_lo, int n_members, float sigma,
                                                 float* __restrict__ out, int64_t ld_out) {
    const int64_t chunk = blockIdx.x;
    const int mi = find_mat(mats, n_mats, chunk);
    const eggroll_mat_t mt = mats[mi];
    const int64_t cidx = chunk - mt.chunk_off;
#define EGG_PERTURB(KD, R1_)                                                                                  \
    perturb_chunk<KD, R1_>(theta, factors, ld_f, mt, cidx, r, sqrt_r, pop, antithetic, member_lo, n_members, sigma, \
                           out, ld_out)
    const int kind = chunk_kind(mt);
#define EGG_PERTURB1(KD, NU_) \
    perturb_chunk_r1<KD, NU_>(theta, factors, ld_f, mt, cidx, pop, antithetic, member_lo, n_members, sigma, out, ld_out)
    if constexpr (RANK1) {  // host launches this instantiation only for r == 1
        const int nu = kind == K_WIDE ? (int)mt.rows : (kind == K_TALL ? (int)mt.cols : 1);
        if (kind == K_VEC) EGG_PERTURB1(K_VEC, 1);
        else if (kind == K_WIDE && nu == 1) EGG_PERTURB1(K_WIDE, 1);
        else if (kind == K_WIDE && nu == 2) EGG_PERTURB1(K_WIDE, 2);
        else if (kind == K_WIDE) EGG_PERTURB1(K_WIDE, 4);
        else if (kind == K_TALL && nu == 1) EGG_PERTURB1(K_TALL, 1);
        else if (kind == K_TALL && nu == 2) EGG_PERTURB1(K_TALL, 2);
        else if (kind == K_TALL) EGG_PERTURB1(K_TALL, 4);
        else EGG_PERTURB(K_GEN, true);
    } else {
        switch (kind) {
            case K_VEC: EGG_PERTURB(K_VEC, false); break;
            case K_WIDE: EGG_PERTURB(K_WIDE, false); break;
            case K_TALL: EGG_PERTURB(K_TALL, false); break;
            default: EGG_PERTURB(K_GEN, false); break;
        }
    }
#undef EGG_PERTURB
#undef EGG_PERTURB1
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
    const int tid = threadIdx.x;
    // column means (thread j, sequential over k)
    for (int jj = tid; jj < m; jj += blockDim.x) {
        float acc = 0.0f;
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
        for (int k = 0; k < n; ++k)
            if (isfinite(s_sc[k])) { sum = sum + s_sc[k]; ++nf; }
        const float mean = sum / (float)nf;
        float sq = 0.0f;
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
        for (int i = 0; i < n; ++i) {
            const float o = s_sc[i];
            rank += lt_nan_last(o, s) || (i < k && eq_nan(o, s));
        }
        order[rank] = k;
    }
}

// ------------------------------------------------------------------------------------
// (4) update
// ------------------------------------------------------------------------------------
struct UpdScalars {  // tail of the update workspace
    double step_scale, theta_scale;
    int32_t step_on, theta_on, nf, pad;
};

template <int KIND, bool R1>
__device__ __forceinline__ void update_chunk(const float* __restrict__ theta, const float* __restrict__ factors,
                                             int64_t ld_f, int64_t n_base, const float* __restrict__ s_c, int nf,
                                             const eggroll_mat_t& mt, int64_t cidx, int r, float sqrt_r, float lr,
                                             float* __restrict__ out, double (&part)[4]) {
#pragma clang fp contract(off)
    const Slots sl = make_slots<KIND>(mt, cidx, threadIdx.x);
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (nf > 0) {
        // sum_j c_j eps_j in base order j = 0, 1, ... (the order is the oracle's)
#pragma unroll 2
        for (int64_t j = 0; j < n_base; ++j) {
            const float* fj = factors + j * ld_f;
            const float cj = s_c[j];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float ev = eps_rc<KIND, R1>(mt, fj, sl.ok[s] ? sl.row[s] : 0, sl.ok[s] ? sl.col[s] : 0, r, sqrt_r);
                acc[s] = acc[s] + cj * ev;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if (!sl.ok[s]) continue;
        const int64_t e = mt.theta_off + slot_elem(mt, sl, s, KIND);
        const float th = theta[e];
        float v = th;
        if (nf > 0) {
            const float g = acc[s] / (float)nf;
            const float t = lr * g;
            v = th + t;
        }
        out[e] = v;
        const double d = (double)v - (double)th;
        part[0] += d * d;
        part[1] += (double)v * (double)v;
        part[2] += (double)th * d;
        part[3] += (double)th * (double)th;
    }
}

template <bool RANK1>
__global__ __launch_bounds__(256) void k_update_delta(const float* __restrict__ theta, const float* __restrict__ factors,
                                                      int64_t ld_f, int64_t n_base, const float* __restrict__ fit,
                                                      const float* __restrict__ stats, int32_t pop, int32_t antithetic,
                                                      const eggroll_mat_t* __restrict__ mats, int n_mats, int r,
                                                      float sqrt_r, float lr, float* __restrict__ out,
                                                      double* __restrict__ partials) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float s_c[];  // [n_base]
    __shared__ double s_red[4][4];
    const int tid = threadIdx.x;
    const int nf = (int)stats[1];
    for (int64_t j = tid; j < n_base; j += blockDim.x) {
        float c;
        if (!antithetic) {
            c = fit[j];
        } else {
            const int64_t h = pop / 2;
            c = (j < h) ? fit[j] - fit[j + h] : fit[2 * h];
        }
        s_c[j] = c;
    }
    __syncthreads();
    const int64_t chunk = blockIdx.x;
    const int mi = find_mat(mats, n_mats, chunk);
    const eggroll_mat_t mt = mats[mi];
    const int64_t cidx = chunk - mt.chunk_off;
    double part[4] = {0.0, 0.0, 0.0, 0.0};
#define EGG_UPDATE(KD, R1_) \
    update_chunk<KD, R1_>(theta, factors, ld_f, n_base, s_c, nf, mt, cidx, r, sqrt_r, lr, out, part)
    const int kind = chunk_kind(mt);
#define EGG_UPDATE1(KD, NU_) \
    update_chunk_r1<KD, NU_>(theta, factors, ld_f, n_base, s_c, nf, mt, cidx, lr, out, part)
    if constexpr (RANK1) {  // host launches this instantiation only for r == 1
        const int nu = kind == K_WIDE ? (int)mt.rows : (kind == K_TALL ? (int)mt.cols : 1);
        if (kind == K_VEC) EGG_UPDATE1(K_VEC, 1);
        else if (kind == K_WIDE && nu == 1) EGG_UPDATE1(K_WIDE, 1);
        else if (kind == K_WIDE && nu == 2) EGG_UPDATE1(K_WIDE, 2);
        else if (kind == K_WIDE) EGG_UPDATE1(K_WIDE, 4);
        else if (kind == K_TALL && nu == 1) EGG_UPDATE1(K_TALL, 1);
        else if (kind == K_TALL && nu == 2) EGG_UPDATE1(K_TALL, 2);
        else if (kind == K_TALL) EGG_UPDATE1(K_TALL, 4);
        else EGG_UPDATE(K_GEN, true);
    } else {
        switch (kind) {
            case K_VEC: EGG_UPDATE(K_VEC, false); break;
            case K_WIDE: EGG_UPDATE(K_WIDE, false); break;
            case K_TALL: EGG_UPDATE(K_TALL, false); break;
            default: EGG_UPDATE(K_GEN, false); break;
        }
    }
#undef EGG_UPDATE
#undef EGG_UPDATE1
#pragma unroll
    for (int q = 0; q < 4; ++q) part[q] = wave_sum_d(part[q]);
    const int w = tid >> 6, lane = tid & 63;
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) s_red[w][q] = part[q];
    }
    __syncthreads();
    if (tid < 4) {
        partials[chunk * 4 + tid] = s_red[0][tid] + s_red[1][tid] + s_red[2][tid] + s_red[3][tid];
    }
}

__global__ __launch_bounds__(256) void k_update_finalize(const double* __restrict__ partials, int64_t n_chunks,
                                                         const float* __restrict__ stats, float max_step,
                                                         float max_theta, UpdScalars* __restrict__ sc) {
    __shared__ double s[4][256];
    const int tid = threadIdx.x;
    double a[4] = {0, 0, 0, 0};
    for (int64_t c = tid; c < n_chunks; c += 256)
        for (int q = 0; q < 4; ++q) a[q] += partials[c * 4 + q];
    for (int q = 0; q < 4; ++q) s[q][tid] = a[q];
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (tid < st)
            for (int q = 0; q < 4; ++q) s[q][tid] += s[q][tid + st];
        __syncthreads();
    }
    if (tid == 0) {
        const double dd = s[0][0], oo = s[1][0], td = s[2][0], tt = s[3][0];
        const int nf = (int)stats[1];
        // cap_step_norm (utills.py:342-349) then cap_theta_norm (utills.py:333-339)
        const double dn = sqrt(dd);
        int step_on = (nf > 0) && (max_step > 0.0f) && (dn > (double)max_step);
        double ss = step_on ? (double)max_step / (dn + 1e-8) : 1.0;
        const double n2 = step_on ? (tt + 2.0 * ss * td + ss * ss * dd) : oo;
        const double tn = sqrt(n2 > 0.0 ? n2 : 0.0);
        // no finite member: the reference returns theta unchanged, caps included (unifed_es.py:237-240)
        int theta_on = (nf > 0) && (max_theta > 0.0f) && (tn > (double)max_theta);
        sc->step_scale = ss;
        sc->theta_scale = theta_on ? (double)max_theta / (tn + 1e-8) : 1.0;
        sc->step_on = step_on;
        sc->theta_on = theta_on;
        sc->nf = nf;
    }
}

__global__ __launch_bounds__(256) void k_update_apply(const float* __restrict__ theta, int64_t D,
                                                      const UpdScalars* __restrict__ sc, float* __restrict__ out) {
#pragma clang fp contract(off)
    const int step_on = sc->step_on, theta_on = sc->theta_on;
    if (!step_on && !theta_on) return;
    const float ss = (float)sc->step_scale, ts = (float)sc->theta_scale;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < D; i += (int64_t)gridDim.x * blockDim.x) {
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
    dim3 grid((unsigned)((quads + 255) / 256), (unsigned)(base_hi - base_lo));
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

int eggroll_perturb(const float* theta, const float* factors, int64_t ld_f, int64_t n_base,
                    const eggroll_mat_t* mats, int32_t n_mats, int64_t total_chunks, int64_t D, int32_t rank,
                    int32_t pop, int32_t antithetic, int64_t member_lo, int64_t member_hi, float sigma, float* out,
                    int64_t ld_out, void* stream) {
    EGG_CHECK_ARG(rank >= 1, "perturb: rank must be >= 1");
    EGG_CHECK_ARG(pop >= 1 && member_lo >= 0 && member_hi <= pop && member_lo <= member_hi,
                  "perturb: members [%lld,%lld) outside pop %d", (long long)member_lo, (long long)member_hi, pop);
    EGG_CHECK_ARG(n_mats >= 1 && mats && factors && out && ld_out >= D, "perturb: bad pointers/sizes");
    const int64_t need_base = antithetic ? (pop / 2 + (pop % 2)) : pop;
    EGG_CHECK_ARG(n_base >= need_base, "perturb: n_base %lld < %lld needed", (long long)n_base, (long long)need_base);
    EGG_CHECK_ARG(member_hi - member_lo <= 65535, "perturb: at most 65535 members per call");
    EGG_CHECK_ARG(total_chunks >= 1 && total_chunks <= (1ll << 21), "perturb: bad total_chunks (<= 2^21: 32-bit element indices)");
    if (member_hi == member_lo || D == 0) return EGGROLL_OK;
    const float sqrt_r = (float)sqrt((double)rank);
    hipLaunchKernelGGL(rank == 1 ? k_perturb<true> : k_perturb<false>, dim3((unsigned)total_chunks), dim3(256), 0, as_stream(stream), theta, factors, ld_f,
                       mats, n_mats, rank, sqrt_r, pop, antithetic, member_lo, (int)(member_hi - member_lo), sigma,
                       out, ld_out);
    EGG_CHECK_LAUNCH("perturb");
    return EGGROLL_OK;
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

int64_t eggroll_update_workspace_bytes(int64_t total_chunks) {
    return total_chunks * 4 * (int64_t)sizeof(double) + 64;
}

int eggroll_update(const float* theta, const float* factors, int64_t ld_f, int64_t n_base, const float* fitness,
                   const float* stats, int32_t pop, int32_t antithetic, const eggroll_mat_t* mats, int32_t n_mats,
                   int64_t total_chunks, int64_t D, int32_t rank, float lr, float max_step_norm,
                   float theta_max_norm, void* workspace, float* theta_out, void* stream) {
    EGG_CHECK_ARG(rank >= 1 && pop >= 1 && n_mats >= 1, "update: bad rank/pop/n_mats");
    EGG_CHECK_ARG(theta && factors && fitness && stats && mats && workspace && theta_out, "update: NULL pointer");
    EGG_CHECK_ARG(theta != theta_out, "update: theta_out may not alias theta");
    const int64_t need_base = antithetic ? (pop / 2 + (pop % 2)) : pop;
    EGG_CHECK_ARG(n_base == need_base, "update: n_base %lld != %lld", (long long)n_base, (long long)need_base);
    EGG_CHECK_ARG(n_base <= 16384, "update: n_base > 16384 unsupported");
    EGG_CHECK_ARG(total_chunks >= 1 && total_chunks <= (1ll << 21), "update: bad total_chunks (<= 2^21: 32-bit element indices)");
    EGG_CHECK_ARG(((uintptr_t)workspace & 15) == 0, "update: workspace must be 16-byte aligned");
    if (D == 0) return EGGROLL_OK;
    const float sqrt_r = (float)sqrt((double)rank);
    double* partials = reinterpret_cast<double*>(workspace);
    UpdScalars* sc = reinterpret_cast<UpdScalars*>(partials + total_chunks * 4);
    hipStream_t st = as_stream(stream);
    const bool r1 = rank == 1 && ld_f * 4 * 64 < (1ll << 31);  // rank-1 path's 32-bit buffer offsets
    hipLaunchKernelGGL(r1 ? k_update_delta<true> : k_update_delta<false>, dim3((unsigned)total_chunks), dim3(256), (size_t)n_base * sizeof(float), st,
                       theta, factors, ld_f, n_base, fitness, stats, pop, antithetic, mats, n_mats, rank, sqrt_r, lr,
                       theta_out, partials);
    EGG_CHECK_LAUNCH("update_delta");
    hipLaunchKernelGGL(k_update_finalize, dim3(1), dim3(256), 0, st, partials, total_chunks, stats, max_step_norm,
                       theta_max_norm, sc);
    EGG_CHECK_LAUNCH("update_finalize");
    int64_t blocks = (D + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(k_update_apply, dim3((unsigned)blocks), dim3(256), 0, st, theta, D, sc, theta_out);
    EGG_CHECK_LAUNCH("update_apply");
    return EGGROLL_OK;
}

}  // extern "C"
