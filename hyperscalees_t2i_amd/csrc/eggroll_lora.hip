// libeggroll — (2) population-batched perturbed LoRA linear for gfx950 (MI355X).
//
// Replaces, for all members of one rank at once, the reference's per-member
//   unflatten_to_params(theta + sigma*eps[k])  (unifed_es.py:160-161, utills.py:155-162)
//   PEFT lora.Linear: y = x W^T + bias + (alpha/r) * (x A_k^T) B_k^T   (es_backend.py:193-200)
// Rows of X are stacked member-major, so the frozen base weight W streams through LDS once
// per M-tile for every member instead of once per member-forward.
//
//   k_lora_project : T[row, q] = X[row,:] . A_k[q,:]   (fp32; HBM-bound X read)
//   k_lora_gemm    : Y = X W^T (bf16 MFMA 16x16x32, 128x128x64 tiles, global_load_lds staging,
//                    XOR-swizzled LDS, 2-stage pipeline) with the epilogue
//                    + bias[n] + scale * sum_q T[row,q] * B_k[n,q]
//   k_lora_expand  : Y += scale * T B_k^T  (for hosts that run the base GEMM elsewhere)
#include <algorithm>
#include "common.h"

namespace eggroll {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;

__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
    return __uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {  // RNE, NaN-preserving cast
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<unsigned short*>(&b);
}

// ------------------------------------------------------------------------------------
// T = X A_k^T : one wave per row, 16-byte X loads, fp32 accumulate, wave reduction.
// ------------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void k_lora_project(const unsigned short* __restrict__ X, int64_t ldx,
                                                      const float* __restrict__ theta_pop, int64_t ld_theta,
                                                      int64_t offA, int64_t rows_per_member, int64_t M, int64_t K,
                                                      float* __restrict__ T) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int64_t kl = row / rows_per_member;
    const float* A = theta_pop + kl * ld_theta + offA;
    const unsigned short* x = X + row * ldx;
    float acc[R];
#pragma unroll
    for (int q = 0; q < R; ++q) acc[q] = 0.0f;
    for (int64_t c = lane * 8; c < K; c += 64 * 8) {
        const u16x8 xv = *reinterpret_cast<const u16x8*>(x + c);
        float xf[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) xf[t] = bf16_to_f32(xv[t]);
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float4 a0 = *reinterpret_cast<const float4*>(A + q * K + c);
            const float4 a1 = *reinterpret_cast<const float4*>(A + q * K + c + 4);
            acc[q] += xf[0] * a0.x + xf[1] * a0.y + xf[2] * a0.z + xf[3] * a0.w + xf[4] * a1.x + xf[5] * a1.y +
                      xf[6] * a1.z + xf[7] * a1.w;
        }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const float v = wave_sum(acc[q]);
        if (lane == 0) T[row * R + q] = v;
    }
}

// Register-resident-A variant (R <= 2, K <= 512 NI): each wave keeps its member's A_k slice
// (NI x 8 columns x R per lane) in VGPRs and sweeps PR_ROWS rows, two rows' X loads in flight at a
// time — the per-row A re-reads of k_lora_project (4 float4 A loads per X load) are gone, so the
// kernel issues almost only the X stream.  Same lane->column map and summation order as
// k_lora_project: bit-identical T.
constexpr int PR_ROWS = 8;  // rows per wave

template <int R, int NI>
__global__ __launch_bounds__(256) void k_lora_project_ra(const unsigned short* __restrict__ X, int64_t ldx,
                                                         const float* __restrict__ theta_pop, int64_t ld_theta,
                                                         int64_t offA, int64_t rows_per_member, int64_t M, int64_t K,
                                                         float* __restrict__ T) {
    const int lane = threadIdx.x & 63;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * PR_ROWS;
    if (row0 >= M) return;
    const int64_t row_end = row0 + PR_ROWS < M ? row0 + PR_ROWS : M;
    int64_t cur = -1;
    float a[NI][R][8];
    auto load_a = [&](int64_t kl) {
        const float* A = theta_pop + kl * ld_theta + offA;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int64_t c = lane * 8 + 512 * i;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
                if (c < K) {
                    a0 = *reinterpret_cast<const float4*>(A + q * K + c);
                    a1 = *reinterpret_cast<const float4*>(A + q * K + c + 4);
                }
                a[i][q][0] = a0.x; a[i][q][1] = a0.y; a[i][q][2] = a0.z; a[i][q][3] = a0.w;
                a[i][q][4] = a1.x; a[i][q][5] = a1.y; a[i][q][6] = a1.z; a[i][q][7] = a1.w;
            }
        }
    };
    for (int64_t row = row0; row < row_end; row += 2) {
        const bool two = row + 1 < row_end;
        u16x8 xv[2][NI];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int64_t c = lane * 8 + 512 * i;
                xv[h][i] = (c < K && (h == 0 || two)) ? *reinterpret_cast<const u16x8*>(X + (row + h) * ldx + c)
                                                      : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h == 1 && !two) break;
            const int64_t kl = (row + h) / rows_per_member;
            if (kl != cur) {  // wave-uniform: only at member boundaries
                load_a(kl);
                cur = kl;
            }
            float acc[R];
#pragma unroll
            for (int q = 0; q < R; ++q) acc[q] = 0.0f;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                if (lane * 8 + 512 * i >= K) break;
                float xf[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) xf[t] = bf16_to_f32(xv[h][i][t]);
#pragma unroll
                for (int q = 0; q < R; ++q)
                    acc[q] += xf[0] * a[i][q][0] + xf[1] * a[i][q][1] + xf[2] * a[i][q][2] + xf[3] * a[i][q][3] +
                              xf[4] * a[i][q][4] + xf[5] * a[i][q][5] + xf[6] * a[i][q][6] + xf[7] * a[i][q][7];
            }
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const float v = wave_sum(acc[q]);
                if (lane == 0) T[(row + h) * R + q] = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// Multi-linear projection on MFMA: T_l[row, q] = X[row,:] . A_{k,l}[q,:] for n_lin LoRA linears that
// read the SAME X (Sana attn1 to_q / to_k / to_v, attn2 to_k / to_v): X streams from HBM once instead
// of once per linear.  As a GEMM it is [M x K] x [K x 16]: the B operand holds the NQ = n_lin * r
// rows of A as bf16 hi / lo pairs (columns q and NQ + q: hi = bf16(a), lo = bf16(a - hi), so
// hi + lo carries a to ~2^-16 relative), X is the A operand straight from global memory, fp32
// accumulation.  The reduction over K is order-free, so K is permuted to make every lane's X read
// contiguous: in each 128-column group lane-group h = lane >> 4 owns columns [h*32, h*32 + 32) as
// four 16-byte pieces, piece j feeding MFMA k-step j; the B image in LDS uses the same permutation
// (a K % 128 tail runs in the plain 8-column layout).  The B image of the block's member is built in
// LDS once (K * 32 bytes); each wave runs two 16-row groups (32 rows, 8 KiB of X in flight) per pass.
//   img[s][lane] = 8 bf16: column n = lane & 15, K-columns col(s, lane >> 4, 0..7).
// ------------------------------------------------------------------------------------
constexpr int PM_ROWS_PER_BLOCK = 256;  // 4 waves x 2 groups x 16 rows x 2 passes

__device__ __forceinline__ int64_t pm_col(int s, int h, int64_t ng) {
    // first of the 8 consecutive K-columns of k-step s held by lane-group h
    return s < 4 * ng ? (int64_t)(s >> 2) * 128 + h * 32 + (s & 3) * 8 : ng * 128 + (int64_t)(s - 4 * ng) * 32 + h * 8;
}

template <int NQ>
__global__ __launch_bounds__(256) void k_lora_project_mfma(const unsigned short* __restrict__ X, int64_t ldx,
                                                           const float* __restrict__ theta_pop, int64_t ld_theta,
                                                           int64_t offA0, int64_t offA1, int64_t offA2,
                                                           int64_t offA3, int r, int64_t rows_per_member,
                                                           int64_t M, int64_t K, float* __restrict__ T) {
    extern __shared__ __attribute__((aligned(16))) char pm_smem[];
    bf16x8* img = reinterpret_cast<bf16x8*>(pm_smem);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 4, n = lane & 15;
    const int nsteps = (int)(K / 32);
    const int64_t ng = K / 128;
    const int64_t r0 = (int64_t)blockIdx.x * PM_ROWS_PER_BLOCK;
    const int64_t r1 = r0 + PM_ROWS_PER_BLOCK < M ? r0 + PM_ROWS_PER_BLOCK : M;
    const int64_t kl_first = r0 / rows_per_member, kl_last = (r1 - 1) / rows_per_member;
    for (int64_t kl = kl_first; kl <= kl_last; ++kl) {
        // ---- B image of member kl: entry (s, ln) = 8 bf16 of column ln & 15 ----
        if (kl != kl_first) __syncthreads();  // every wave is done with the previous image
        for (int e = threadIdx.x; e < nsteps * 64; e += 256) {
            const int s = e >> 6, ln = e & 63, cn = ln & 15;
            bf16x8 v;
            if (cn < 2 * NQ) {
                const int q = cn < NQ ? cn : cn - NQ, l = q / r, qq = q - l * r;
                const int64_t off = l == 0 ? offA0 : l == 1 ? offA1 : l == 2 ? offA2 : offA3;
                const float* a = theta_pop + kl * ld_theta + off + (int64_t)qq * K + pm_col(s, ln >> 4, ng);
                const float4 a0 = *reinterpret_cast<const float4*>(a);
                const float4 a1 = *reinterpret_cast<const float4*>(a + 4);
                const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const __bf16 hi = (__bf16)av[t];
                    v[t] = cn < NQ ? hi : (__bf16)(av[t] - (float)hi);
                }
            } else {
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = (__bf16)0.0f;
            }
            img[e] = v;
        }
        __syncthreads();
        const int64_t mlo = kl * rows_per_member > r0 ? kl * rows_per_member : r0;
        const int64_t mhi = (kl + 1) * rows_per_member < r1 ? (kl + 1) * rows_per_member : r1;
        for (int64_t g0 = r0 + wave * 32; g0 < r1; g0 += 4 * 32) {
            if (g0 + 32 <= mlo || g0 >= mhi) continue;  // wave-uniform: no row of this pass in member kl
            const int64_t ra = g0 + n, rb = g0 + 16 + n;
            const bool va = ra >= mlo && ra < mhi, vb = rb >= mlo && rb < mhi;
            const unsigned short* xa = X + (va ? ra : mlo) * ldx + h * 32;
            const unsigned short* xb = X + (vb ? rb : mlo) * ldx + h * 32;
            f32x4 acc_a = {0.f, 0.f, 0.f, 0.f}, acc_b = acc_a;
            const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
            u16x8 ca[4], cb[4];
            if (ng > 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    ca[j] = va ? *reinterpret_cast<const u16x8*>(xa + j * 8) : z;
                    cb[j] = vb ? *reinterpret_cast<const u16x8*>(xb + j * 8) : z;
                }
            }
            for (int64_t G = 0; G < ng; ++G) {
                u16x8 na[4], nb[4];
                const bool more = G + 1 < ng;
#pragma unroll
                for (int j = 0; j < 4; ++j) {  // next group's X in flight under this group's MFMAs
                    na[j] = (more && va) ? *reinterpret_cast<const u16x8*>(xa + (G + 1) * 128 + j * 8) : z;
                    nb[j] = (more && vb) ? *reinterpret_cast<const u16x8*>(xb + (G + 1) * 128 + j * 8) : z;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bf16x8 bfr = img[(G * 4 + j) * 64 + lane];
                    acc_a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ca[j]), bfr, acc_a,
                                                                    0, 0, 0);
                    acc_b = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, cb[j]), bfr, acc_b,
                                                                    0, 0, 0);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    ca[j] = na[j];
                    cb[j] = nb[j];
                }
            }
            for (int s = (int)(4 * ng); s < nsteps; ++s) {  // K % 128 tail, plain layout
                const int64_t c = pm_col(s, h, ng) - h * 32;
                const u16x8 xa8 = va ? *reinterpret_cast<const u16x8*>(xa + c) : z;
                const u16x8 xb8 = vb ? *reinterpret_cast<const u16x8*>(xb + c) : z;
                const bf16x8 bfr = img[s * 64 + lane];
                acc_a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xa8), bfr, acc_a, 0, 0, 0);
                acc_b = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xb8), bfr, acc_b, 0, 0, 0);
            }
            // D[4h + i][n]: T[q] = D[q] (hi) + D[NQ + q] (lo), joined across lanes n and n + NQ
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float ta = acc_a[i] + __shfl(acc_a[i], (lane + NQ) & 63, 64);
                const float tb = acc_b[i] + __shfl(acc_b[i], (lane + NQ) & 63, 64);
                if (n < NQ) {
                    const int l = n / r, qq = n - l * r;
                    float* Tl = T + (int64_t)l * M * r;
                    const int64_t rowa = g0 + 4 * h + i, rowb = g0 + 16 + 4 * h + i;
                    if (rowa >= mlo && rowa < mhi) Tl[rowa * r + qq] = ta;
                    if (rowb >= mlo && rowb < mhi) Tl[rowb * r + qq] = tb;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// Base GEMM + fused LoRA epilogue, templated on the tile:
//   Tile<BM, BN, WM, WN>: BM x BN output tile, BK = 64, WM x WN waves (wave tile (BM/WM) x (BN/WN)),
//   2 LDS stages of (BM + BN) rows x 128 B, one barrier per K-tile: the global_load_lds of K-tile
//   k+1 is issued right after the barrier and lands while the MFMAs of K-tile k run.
//   kT128: 128x128, 4 waves (2 blocks/CU, 64 KiB LDS).  kT256: 256x256, 8 waves (1 block/CU,
//   128 KiB LDS) — half the LDS bytes per FLOP.
// ------------------------------------------------------------------------------------
constexpr int BK = 64;
#ifndef EGG_GROUP_M
#define EGG_GROUP_M 8
#endif
constexpr int GROUP_M = EGG_GROUP_M;  // row-tiles per rasterisation group

// Phase stamps for the tools-only diagnostic build (tools/stamp_probe.py compiles this file with
// -DEGG_STAMPS into a separate library; the shipped libeggroll.so has none): wave 0 of every
// workgroup records s_memtime at fixed points of the 8-phase kernels (vector stores from lane 0).
#ifdef EGG_STAMPS
constexpr int EGG_NSTAMP = 8;
__device__ unsigned long long g_egg_stamps[131072 * EGG_NSTAMP];
#define EGG_STAMP(k)                                                                                         \
    do {                                                                                                     \
        if (threadIdx.x == 0)                                                                                \
            g_egg_stamps[(size_t)blockIdx.x * EGG_NSTAMP + (k)] = __builtin_amdgcn_s_memtime();              \
    } while (0)
#define EGG_STAMP_RT(k)                                                                                      \
    do {                                                                                                     \
        if (threadIdx.x == 0)                                                                                \
            g_egg_stamps[(size_t)blockIdx.x * EGG_NSTAMP + (k)] = __builtin_amdgcn_s_memrealtime();          \
    } while (0)
#define EGG_STAMP_DRAIN() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define EGG_STAMP(k) \
    do {             \
    } while (0)
#define EGG_STAMP_RT(k) \
    do {                \
    } while (0)
#define EGG_STAMP_DRAIN() \
    do {                  \
    } while (0)
#endif

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

template <int BM_, int BN_, int WM_, int WN_>
struct Tile {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
    static constexpr int WAVES = WM * WN, THREADS = 64 * WAVES;
    static constexpr int WTM = BM / WM, WTN = BN / WN;   // wave tile
    static constexpr int FM = WTM / 16, FN = WTN / 16;   // 16x16 fragments per wave
    static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
    static constexpr int STAGE = A_BYTES + B_BYTES;
    static constexpr int LDS = 2 * STAGE;
    static constexpr int GA = BM / 8 / WAVES, GB = BN / 8 / WAVES;   // glds per wave per K-tile
    static constexpr int MIN_BLOCKS = (LDS <= 80 * 1024) ? 2 : 1;
    static_assert(BM % (8 * WAVES) == 0 && BN % (8 * WAVES) == 0, "staging split");
    static_assert(WTM * WTN * 2 <= LDS / WAVES, "epilogue staging must fit");
};
using kT128 = Tile<128, 128, 2, 2>;
using kT256 = Tile<256, 256, 2, 4>;

// Stage `nglds` x 8 rows of a K-contiguous bf16 matrix into an LDS tile.  LDS image: row r at
// byte 128*r; 16-B slot s' of row r holds global chunk s' ^ (r & 7)  (conflict-free b128
// fragment reads).  One global_load_lds_dwordx4 = 1 KiB = 8 rows.
template <int NG>
__device__ __forceinline__ void stage_rows(const unsigned short* __restrict__ G, int64_t ld, int64_t row0,
                                           int64_t row_max, int64_t k0, char* lds_tile, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < NG; ++i) {
        const int R0 = (wave * NG + i) * 8;
        const int r = R0 + (lane >> 3);
        const int chunk = (lane & 7) ^ (r & 7);
        int64_t gr = row0 + r;
        gr = gr < row_max ? gr : row_max;  // clamp: rows past the end are never stored
        const unsigned short* src = G + gr * ld + k0 + chunk * 8;
        __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds_tile + R0 * 128), 16, 0, 0);
    }
}

__device__ __forceinline__ bf16x8 read_frag(const char* lds_tile, int row, int chunk) {
    return *reinterpret_cast<const bf16x8*>(lds_tile + row * 128 + ((chunk ^ (row & 7)) << 4));
}

template <int R, class TL>
__global__ __launch_bounds__(TL::THREADS, TL::MIN_BLOCKS) void k_lora_gemm(
    const unsigned short* __restrict__ X, int64_t ldx, const unsigned short* __restrict__ W, int64_t ldw,
    const unsigned short* __restrict__ bias, const float* __restrict__ T, const float* __restrict__ theta_pop,
    int64_t ld_theta, int64_t offB, float scale, int rows_per_member, int M, int N, int64_t K, int tiles_n,
    unsigned short* __restrict__ Y, int64_t ldy) {
    constexpr int FM = TL::FM, FN = TL::FN;
    __shared__ __attribute__((aligned(16))) char smem[TL::LDS];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / TL::WN, wn = wave % TL::WN;
    // XCD-aware bijective remap: consecutive tile ids (sharing X rows) land on one XCD.
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
    const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
    // grouped rasterisation: consecutive tiles (one XCD's concurrently resident set) walk GROUP_M
    // row-tiles before moving to the next column-tile, so X and W panels are both reused in L2.
    const int tiles_m = (M + TL::BM - 1) / TL::BM;
    const int per_group = GROUP_M * tiles_n;
    const int grp = tile / per_group, first_m = grp * GROUP_M;
    const int gsize = (tiles_m - first_m) < GROUP_M ? (tiles_m - first_m) : GROUP_M;
    const int in_grp = tile - grp * per_group;
    const int tm = first_m + in_grp % gsize, tn = in_grp / gsize;
    const int m0 = tm * TL::BM, n0 = tn * TL::BN;

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (int)(K / BK);
    stage_rows<TL::GA>(X, ldx, m0, M - 1, 0, smem, wave, lane);
    stage_rows<TL::GB>(W, ldw, n0, N - 1, 0, smem + TL::A_BYTES, wave, lane);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const char* cur = smem + (kt & 1) * TL::STAGE;
        if (kt + 1 < nk) {
            char* nxt = smem + ((kt + 1) & 1) * TL::STAGE;
            stage_rows<TL::GA>(X, ldx, m0, M - 1, (int64_t)(kt + 1) * BK, nxt, wave, lane);
            stage_rows<TL::GB>(W, ldw, n0, N - 1, (int64_t)(kt + 1) * BK, nxt + TL::A_BYTES, wave, lane);
        }
#pragma unroll
        for (int kk = 0; kk < (FM <= 4 ? 2 : 0); ++kk) {
            const int ch = kk * 4 + (lane >> 4);
            bf16x8 b[FN];
#pragma unroll
            for (int f = 0; f < FN; ++f) b[f] = read_frag(cur + TL::A_BYTES, wn * TL::WTN + f * 16 + (lane & 15), ch);
            if constexpr (FM <= 4) {
                bf16x8 a[FM];
#pragma unroll
                for (int f = 0; f < FM; ++f) a[f] = read_frag(cur, wm * TL::WTM + f * 16 + (lane & 15), ch);
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
                __builtin_amdgcn_s_setprio(0);
            } else {
                // large wave tile: handled below as one software-pipelined K-tile
            }
        }
        if constexpr (FM > 4) {
            // 8 steps per K-tile (2 k-substeps x 4 A-fragment pairs); the operands of step s+1
            // are read from LDS before the 8 MFMAs of step s are issued, so LDS latency hides
            // under MFMA work (counted lgkmcnt) instead of a full drain per fragment pair.
            const char* bt = cur + TL::A_BYTES;
            const int rA = wm * TL::WTM + (lane & 15), rB = wn * TL::WTN + (lane & 15);
            const int ch0 = lane >> 4, ch1 = 4 + (lane >> 4);
            bf16x8 b[FN], bn[FN], a0, a1, n0, n1;
#pragma unroll
            for (int f = 0; f < FN; ++f) b[f] = read_frag(bt, rB + f * 16, ch0);
            a0 = read_frag(cur, rA, ch0);
            a1 = read_frag(cur, rA + 16, ch0);
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                const int pair = st & 3;
                if (st < 7) {
                    const int np = (st + 1) & 3, nch = ((st + 1) >> 2) ? ch1 : ch0;
                    if (np == 0) {
#pragma unroll
                        for (int f = 0; f < FN; ++f) bn[f] = read_frag(bt, rB + f * 16, nch);
                    }
                    n0 = read_frag(cur, rA + (2 * np) * 16, nch);
                    n1 = read_frag(cur, rA + (2 * np + 1) * 16, nch);
                }
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[2 * pair][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b[j], acc[2 * pair][j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[2 * pair + 1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b[j], acc[2 * pair + 1][j], 0, 0, 0);
                __builtin_amdgcn_s_setprio(0);
                if (st < 7) {
                    a0 = n0;
                    a1 = n1;
                    if (((st + 1) & 3) == 0) {
#pragma unroll
                        for (int f = 0; f < FN; ++f) b[f] = bn[f];
                    }
                }
            }
        }
        __syncthreads();
    }

    // ---- epilogue: + bias[n] + scale * T[row,:] . B_k[n,:]  ->  bf16 via LDS, 16-B stores ----
    const int col_l = lane & 15, rq = (lane >> 4) * 4;
    float bv[FN];
    int colv[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int col = n0 + wn * TL::WTN + j * 16 + col_l;
        colv[j] = col < N ? col : N - 1;
        bv[j] = bias ? bf16_to_f32(bias[colv[j]]) : 0.0f;
    }
    // stage this wave's WTM x WTN bf16 sub-tile in LDS (rows of WTN*2 bytes, 16-B slots XOR-swizzled);
    // the LoRA term is added row by row so accumulators retire as they are written.
    constexpr int ROWB = TL::WTN * 2, SLOTS = ROWB / 16;
    char* ctile = smem + wave * (TL::WTM * ROWB);
    float bk[FN][R > 0 ? R : 1];
    bool one_member = true;
    if constexpr (R > 0) {
        const int first = m0 / rows_per_member;
        const int last_row = (m0 + TL::BM - 1 < M ? m0 + TL::BM - 1 : M - 1);
        one_member = (last_row / rows_per_member) == first;
        const float* Bk = theta_pop + (int64_t)first * ld_theta + offB;
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int qq = 0; qq < R; ++qq) bk[j][qq] = Bk[colv[j] * R + qq];
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int rr = i * 16 + rq + e;
            float add[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) add[j] = bv[j];
            if constexpr (R > 0) {
                int row = m0 + wm * TL::WTM + rr;
                row = row < M ? row : M - 1;
                float t[R];
#pragma unroll
                for (int qq = 0; qq < R; ++qq) t[qq] = T[(int64_t)row * R + qq];
                if (!one_member) {
                    const float* Bk = theta_pop + (int64_t)(row / rows_per_member) * ld_theta + offB;
#pragma unroll
                    for (int j = 0; j < FN; ++j)
#pragma unroll
                        for (int qq = 0; qq < R; ++qq) bk[j][qq] = Bk[colv[j] * R + qq];
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    float d = 0.0f;
#pragma unroll
                    for (int qq = 0; qq < R; ++qq) d += t[qq] * bk[j][qq];
                    add[j] += scale * d;
                }
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int cc = j * 16 + col_l;
                const int slot = (cc >> 3) ^ (rr & (SLOTS - 1));
                *reinterpret_cast<unsigned short*>(ctile + rr * ROWB + slot * 16 + (cc & 7) * 2) =
                    f32_to_bf16(acc[i][j][e] + add[j]);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (wave-private tile)
    constexpr int ROWS_PER_IT = 64 / SLOTS;
#pragma unroll
    for (int it = 0; it < TL::WTM / ROWS_PER_IT; ++it) {
        const int rr = it * ROWS_PER_IT + lane / SLOTS, sl = lane % SLOTS;
        const int row = m0 + wm * TL::WTM + rr;
        const int col = n0 + wn * TL::WTN + sl * 8;
        if (row >= M || col >= N) continue;
        const u16x8 v = *reinterpret_cast<const u16x8*>(ctile + rr * ROWB + ((sl ^ (rr & (SLOTS - 1))) << 4));
        unsigned short* dst = Y + (int64_t)row * ldy + col;
        if (col + 8 <= N && (((uintptr_t)dst) & 15) == 0) {
            *reinterpret_cast<u16x8*>(dst) = v;
        } else {
            for (int u = 0; u < 8 && col + u < N; ++u) dst[u] = v[u];
        }
    }
}

// ------------------------------------------------------------------------------------
// 8-phase 256x256x64 variant (the large-M path).  8 waves = 2 groups of 4 (wm = 0 / 1), each
// wave owns a 128x64 output sub-tile = 4 C-quadrants of 64x32 (16 MFMA 16x16x32 per K-tile each).
// Every K-tile is split into 4 LDS half-tile regions by quadrant: A0 / A1 = rows of quadrant-row
// qa = 0 / 1 of both wave rows, B0 / B1 = columns of quadrant-column qb = 0 / 1 of all four wave
// columns.  One phase = {ds_read the quadrant's fragments, issue one half-tile prefetch (2 glds),
// lgkmcnt(0), s_barrier, 16 MFMA, s_barrier}; group 1 runs one barrier behind group 0, so on every
// SIMD one wave does MFMA while its partner reads LDS / issues DMA.  Quadrant order per K-tile
// (0,0) (0,1) (1,1) (1,0): A0+B0 read in phase 1, B1 in 2, A1 in 3, B0 again in 4, and each
// region is restaged in the phase after its last read (lgkmcnt(0) before the barrier retired those
// reads).  The prefetch of K-tile t+1 therefore spans phases (t,2)..(t,4)+(t+1,1) and the counted
// vmcnt(6) that retires a buffer leaves 3 half-tiles (6 glds) in flight across the barrier; nothing
// drains vmcnt to 0 inside the loop (cdna_hip_programming.md §5 "256² 8-phase template", T3/T4).
// ------------------------------------------------------------------------------------
namespace p8 {
constexpr int HALF = 128 * 128;  // one half-tile region: 128 rows x 64 bf16 (16 KiB)
constexpr int BUF = 4 * HALF;    // A0 | A1 | B0 | B1
constexpr int LDS = 2 * BUF;     // 128 KiB, two K-tile buffers
constexpr int RA0 = 0, RA1 = HALF, RB0 = 2 * HALF, RB1 = 3 * HALF;
}  // namespace p8

// Per-thread staging descriptor of one half-tile region: 2 DMAs (buffer_load_dwordx4 ... lds), each
// 8 rows x 128 B.  `off[i]` is the lane's 32-bit BYTE offset (row * ld + swizzled chunk) at k = 0;
// the K-tile's byte offset goes in the wave-uniform soffset.  The host guarantees rows*ld*2 < 2^31.
struct HalfStage {
    uint32_t off[2];
};

template <bool IS_A>
__device__ __forceinline__ HalfStage make_stage(int base_row, int row_max, int64_t ld, int h, int wave, int lane) {
    HalfStage s;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int j = (i * 8 + wave) * 8 + (lane >> 3);               // region row
        const int chunk = (lane & 7) ^ (j & 7);
        const int tr = IS_A ? ((j >> 6) * 128 + h * 64 + (j & 63))   // A: wave row wm = j/64
                            : ((j >> 5) * 64 + h * 32 + (j & 31));   // B: wave col wn = j/32
        int gr = base_row + tr;
        gr = gr < row_max ? gr : row_max;  // clamp: rows past the end are never stored
        s.off[i] = ((uint32_t)gr * (uint32_t)ld + chunk * 8) * 2;
    }
    return s;
}

__device__ __forceinline__ void issue_half(__amdgpu_buffer_rsrc_t rs, const HalfStage& s, int kbytes, char* region,
                                           int wave) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(region + (i * 8 + wave) * 1024), 16, s.off[i], kbytes,
                                                 0, 0);
}

#define P8_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define P8_VM6() asm volatile("s_waitcnt vmcnt(6)" ::: "memory")
#define P8_VM0() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
// s_barrier as a full compiler fence: the builtin alone is IntrNoMem, so IR passes may move the
// next phase's ds_reads (or this phase's MFMAs) across it.
#define P8_BAR()                              \
    do {                                      \
        asm volatile("" ::: "memory");        \
        __builtin_amdgcn_sched_barrier(0);    \
        __builtin_amdgcn_s_barrier();         \
        __builtin_amdgcn_sched_barrier(0);    \
        asm volatile("" ::: "memory");        \
    } while (0)

// TR: W as the MFMA A-operand, i.e. the fragment is computed transposed: lane l holds Y row (l & 15),
// columns 4 (l >> 4) .. +3 — one 8-byte LDS write in the epilogue instead of four 2-byte ones.
template <int QA, int QB, bool TR>
__device__ __forceinline__ void p8_mma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int g = 0; g < 2; ++g)
                acc[QA * 4 + f][QB * 2 + g] =
                    TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[g][kk], a[f][kk], acc[QA * 4 + f][QB * 2 + g], 0, 0, 0)
                       : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f][kk], b[g][kk], acc[QA * 4 + f][QB * 2 + g], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
}

// Fragment reads with one per-lane base per k-substep: row r = r0 + 16 f keeps (r & 7) fixed, so
// fragment f is base[kk] + 2048 f (an immediate offset) — no per-fragment address registers.
__device__ __forceinline__ void p8_read_a(bf16x8 (&a)[4][2], const char* region, const int (&off)[2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < 4; ++f) a[f][kk] = *reinterpret_cast<const bf16x8*>(region + off[kk] + f * 2048);
}
__device__ __forceinline__ void p8_read_b(bf16x8 (&b)[2][2], const char* region, const int (&off)[2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int g = 0; g < 2; ++g) b[g][kk] = *reinterpret_cast<const bf16x8*>(region + off[kk] + g * 2048);
}
__device__ __forceinline__ void p8_frag_offsets(int (&off)[2], int r0, int lane) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) off[kk] = r0 * 128 + ((((kk * 4) + (lane >> 4)) ^ (r0 & 7)) << 4);
}

#define P8_LGKM0_ asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

// s_waitcnt vmcnt(N) with a compile-time N (the counts of the 8-phase tiles: see G8)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N == 6 || N == 9 || N == 10 || N == 14, "add the literal");
    if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
}

// Early first K-tile.  The prologue issues K-tile 0 as A0, B0, B1, A1 and waits only for A0 + B0
// (what phase 1 reads); phase 1 retires B1 (read in phase 2) and phase 2 retires A1 (read in phase 3),
// each before its first barrier — "wait in phase q, read in phase q+1", which also covers the wave
// group that runs one barrier behind.  Younger than each of these DMAs are exactly 3 A-halves + 2
// B-halves (NA / NB DMAs each), so all three waits are vmcnt(3 NA + 2 NB); in steady state at most
// that many are outstanding at those points, so the two in-loop waits are no-ops after K-tile 0.
// One phase: read the quadrant's fragments (RD: 0 = A+B, 1 = B only, 2 = A only), issue one
// half-tile DMA, [vmcnt(6)], retire the reads, barrier, 16 MFMA, barrier.
template <int QA, int QB, int RD, bool VM, bool TR, int EW = 0>
__device__ __forceinline__ void p8_phase(f32x4 (&acc)[8][4], bf16x8 (&a)[4][2], bf16x8 (&b)[2][2], const char* buf,
                                         const int (&oA)[2], const int (&oB)[2], __amdgpu_buffer_rsrc_t rs,
                                         const HalfStage& st, int kbytes, char* dst, int wave) {
    if (RD != 2) p8_read_b(b, buf + (QB ? p8::RB1 : p8::RB0), oB);
    if (RD != 1) p8_read_a(a, buf + (QA ? p8::RA1 : p8::RA0), oA);
    issue_half(rs, st, kbytes, dst, wave);
    if constexpr (EW > 0) wait_vm<EW>();  // early first K-tile (no-op in steady state)
    if (VM) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    P8_LGKM0_;
    P8_BAR();
    p8_mma<QA, QB, TR>(acc, a, b);
    P8_BAR();
}

// Epilogue shared by the 256x256 kernels: + bias[n] + scale * T[row,:] . B_k[n,:], bf16 via a
// per-wave LDS staging tile (16-B slots XOR-swizzled by row), 16-B stores.
template <int R, int WTM, int WTN>
__device__ __forceinline__ void lora_epilogue(f32x4 (&acc)[WTM / 16][WTN / 16], char* smem, int wave, int lane,
                                              int m0, int n0, int rbase, int cbase, const unsigned short* __restrict__ bias,
                                              const float* __restrict__ T, const float* __restrict__ theta_pop,
                                              int64_t ld_theta, int64_t offB, float scale, int rows_per_member,
                                              int BMtile, int M, int N, unsigned short* __restrict__ Y, int64_t ldy) {
    constexpr int FM = WTM / 16, FN = WTN / 16;
    const int col_l = lane & 15, rq = (lane >> 4) * 4;
    float bv[FN];
    int colv[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int col = n0 + cbase + j * 16 + col_l;
        colv[j] = col < N ? col : N - 1;
        bv[j] = bias ? bf16_to_f32(bias[colv[j]]) : 0.0f;
    }
    constexpr int ROWB = WTN * 2, SLOTS = ROWB / 16;
    char* ctile = smem + wave * (WTM * ROWB);
    float bk[FN][R > 0 ? R : 1];
    bool one_member = true;
    if constexpr (R > 0) {
        const int first = m0 / rows_per_member;
        const int last_row = (m0 + BMtile - 1 < M ? m0 + BMtile - 1 : M - 1);
        one_member = (last_row / rows_per_member) == first;
        const float* Bk = theta_pop + (int64_t)first * ld_theta + offB;
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int qq = 0; qq < R; ++qq) bk[j][qq] = Bk[colv[j] * R + qq];
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int rr = i * 16 + rq + e;
            float add[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) add[j] = bv[j];
            if constexpr (R > 0) {
                int row = m0 + rbase + rr;
                row = row < M ? row : M - 1;
                float t[R];
#pragma unroll
                for (int qq = 0; qq < R; ++qq) t[qq] = T[(int64_t)row * R + qq];
                if (!one_member) {
                    const float* Bk = theta_pop + (int64_t)(row / rows_per_member) * ld_theta + offB;
#pragma unroll
                    for (int j = 0; j < FN; ++j)
#pragma unroll
                        for (int qq = 0; qq < R; ++qq) bk[j][qq] = Bk[colv[j] * R + qq];
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    float d = 0.0f;
#pragma unroll
                    for (int qq = 0; qq < R; ++qq) d += t[qq] * bk[j][qq];
                    add[j] += scale * d;
                }
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int cc = j * 16 + col_l;
                const int slot = (cc >> 3) ^ (rr & (SLOTS - 1));
                *reinterpret_cast<unsigned short*>(ctile + rr * ROWB + slot * 16 + (cc & 7) * 2) =
                    f32_to_bf16(acc[i][j][e] + add[j]);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (wave-private tile)
    constexpr int ROWS_PER_IT = 64 / SLOTS;
#pragma unroll
    for (int it = 0; it < WTM / ROWS_PER_IT; ++it) {
        const int rr = it * ROWS_PER_IT + lane / SLOTS, sl = lane % SLOTS;
        const int row = m0 + rbase + rr;
        const int col = n0 + cbase + sl * 8;
        if (row >= M || col >= N) continue;
        const u16x8 v = *reinterpret_cast<const u16x8*>(ctile + rr * ROWB + ((sl ^ (rr & (SLOTS - 1))) << 4));
        unsigned short* dst = Y + (int64_t)row * ldy + col;
        if (col + 8 <= N && (((uintptr_t)dst) & 15) == 0) {
            *reinterpret_cast<u16x8*>(dst) = v;
        } else {
            for (int u = 0; u < 8 && col + u < N; ++u) dst[u] = v[u];
        }
    }
}

// Store of a transposed (TR) 128x64 wave tile: acc[i][j][e] = Y[rbase + 16 i + (l & 15)]
// [cbase + 16 j + 4 (l >> 4) + e]; 4 columns -> one ds_write_b64 into the wave's swizzled LDS
// staging tile, then 16-B global stores of whole 128-B row segments.
// Epilogue ops applied to the bf16-rounded GEMM output y (one rounding per torch op it replaces):
//   EPI_SILU  : out = bf16(silu(y))                        (GLUMBConv: 1x1 conv -> SiLU)
//   EPI_RES   : out = bf16(res + y)                        (x = x + attn2(...))
//   EPI_GATED : out = bf16(res + gate[row / rpg] * y)      (x += gate * attn1(...), k_gated_residual)
// res may alias Y (each element is read and written by the same lane).
// fp32 residual stream (Sana blocks) — res is an fp32 [M, ldr] stream updated in place,
// Y (optional, may be NULL) receives its bf16 shadow copy (the next GEMM's operand):
//   EPI_RES32   : res = res + float(y)                     (x = x + attn2(...))
//   EPI_GATED32 : res = fma(gate32[row / rpg], float(y), res)  (x += gate * attn1(...); gate fp32)
// The same expressions as eggroll_gated_residual_f32, so fused == unfused bit for bit.
//   EPI_GELU  : out = bf16(gelu_tanh(y))                   (Infinity / VAR ffn: fc1 -> GELU(tanh))
//   EPI_MUL   : out = bf16(res * y)                        (Z-Image SwiGLU: silu(w1 x) * w3 x)
//   EPI_GELU_ERF : out = bf16(gelu(y))                     (PickScore CLIP-H/14 mlp: fc1 -> exact GELU)
enum { EPI_NONE = 0, EPI_SILU = 1, EPI_RES = 2, EPI_GATED = 3, EPI_RES32 = 4, EPI_GATED32 = 5, EPI_GELU = 6, EPI_MUL = 7,
       EPI_GELU_ERF = 8 };
struct EpiArgs {
    const unsigned short* res;
    int64_t ldr;
    const unsigned short* gate;
    int64_t gstride;
    int64_t rpg;
};
__device__ __forceinline__ float epi_silu(float v) { return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v)); }
// GELU, approximate = "tanh": 0.5 x (1 + tanh(k)) = x * sigmoid(2k), k = sqrt(2/pi) (x + 0.044715 x^3),
// with the hardware exp2 / rcp as the SiLU epilogue (ocml's tanhf made the fc1 store phase 15 % of the
// GEMM: tools/gelu_epi_probe.py); within 1 bf16 ulp of torch's tanh form
__device__ __forceinline__ float epi_gelu(float x) {
    constexpr float kBeta2L = (float)(M_SQRT2 * M_2_SQRTPI * 0.5 * 2.0 * 1.4426950408889634);
    constexpr float kKappa = 0.044715f;
    const float u = x + kKappa * (x * x * x);
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-kBeta2L * u));
}
// GELU, approximate = "none": x * 0.5 * (1 + erf(x / sqrt 2)) in fp32, the expression (and the erff) torch's
// GeluCUDAKernelImpl evaluates on a bf16 tensor, so fused == F.gelu(bf16 GEMM output) bit for bit
// (test_lora_linear_pop_gelu_erf_bitexact)
__device__ __forceinline__ float epi_gelu_erf(float x) {
    return x * 0.5f * (1.0f + erff(x * (float)M_SQRT1_2));
}

// x * sigmoid(x) on two values: the multiplies / add as packed fp32 ops (v_pk_mul_f32 / v_pk_add_f32),
// exp2 and rcp per value: the same operations, value by value, as x * rcp(1 + __expf(-x)) (v_mul by
// log2(e), v_exp_f32, v_add, v_rcp_f32, v_mul), so the same bits (test_lora_linear_pop_epilogue_bitexact)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 silu2(f32x2 v) {
    f32x2 t = v * (f32x2){-1.4426950408889634f, -1.4426950408889634f};
    t.x = __builtin_amdgcn_exp2f(t.x);
    t.y = __builtin_amdgcn_exp2f(t.y);
    t = t + (f32x2){1.0f, 1.0f};
    t.x = __builtin_amdgcn_rcpf(t.x);
    t.y = __builtin_amdgcn_rcpf(t.y);
    return v * t;
}


template <int EPI>
__device__ __forceinline__ u16x8 epi_apply(u16x8 v, int row, int col, const EpiArgs& ea) {
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            const f32x2 t = silu2((f32x2){bf16_to_f32(v[u]), bf16_to_f32(v[u + 1])});
            v[u] = f32_to_bf16(t.x);
            v[u + 1] = f32_to_bf16(t.y);
        }
    } else if constexpr (EPI == EPI_GELU) {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = f32_to_bf16(epi_gelu(bf16_to_f32(v[u])));
    } else if constexpr (EPI == EPI_GELU_ERF) {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = f32_to_bf16(epi_gelu_erf(bf16_to_f32(v[u])));
    } else if constexpr (EPI == EPI_RES || EPI == EPI_GATED || EPI == EPI_MUL) {
        const u16x8 r = *reinterpret_cast<const u16x8*>(ea.res + (int64_t)row * ea.ldr + col);
        if constexpr (EPI == EPI_MUL) {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = f32_to_bf16(bf16_to_f32(r[u]) * bf16_to_f32(v[u]));
        } else if constexpr (EPI == EPI_RES) {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = f32_to_bf16(bf16_to_f32(r[u]) + bf16_to_f32(v[u]));
        } else {
            const u16x8 g = *reinterpret_cast<const u16x8*>(ea.gate + (row / ea.rpg) * ea.gstride + col);
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = f32_to_bf16(bf16_to_f32(r[u]) + bf16_to_f32(g[u]) * bf16_to_f32(v[u]));
        }
    }
    return v;
}
// EPI_RES32 / EPI_GATED32 on one 8-column chunk (vector) or one element (tail)
template <int EPI>
__device__ __forceinline__ void epi_store32(u16x8 v, int row, int col, const EpiArgs& ea, unsigned short* Y, int64_t ldy) {
    float* r = const_cast<float*>(reinterpret_cast<const float*>(ea.res)) + (int64_t)row * ea.ldr + col;
    float4 a0 = *reinterpret_cast<const float4*>(r), a1 = *reinterpret_cast<const float4*>(r + 4);
    float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    if constexpr (EPI == EPI_GATED32) {
        const float* g = reinterpret_cast<const float*>(ea.gate) + (row / ea.rpg) * ea.gstride + col;
        const float4 g0 = *reinterpret_cast<const float4*>(g), g1 = *reinterpret_cast<const float4*>(g + 4);
        const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = __builtin_fmaf(gv[u], bf16_to_f32(v[u]), x[u]);
    } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = x[u] + bf16_to_f32(v[u]);
    }
    *reinterpret_cast<float4*>(r) = float4{x[0], x[1], x[2], x[3]};
    *reinterpret_cast<float4*>(r + 4) = float4{x[4], x[5], x[6], x[7]};
    if (Y) {
        u16x8 o;
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = f32_to_bf16(x[u]);
        *reinterpret_cast<u16x8*>(Y + (int64_t)row * ldy + col) = o;
    }
}
template <int EPI>
__device__ __forceinline__ void epi_store32_1(unsigned short v, int row, int col, const EpiArgs& ea, unsigned short* Y,
                                              int64_t ldy) {
    float* r = const_cast<float*>(reinterpret_cast<const float*>(ea.res)) + (int64_t)row * ea.ldr + col;
    float x = *r;
    if constexpr (EPI == EPI_GATED32)
        x = __builtin_fmaf(reinterpret_cast<const float*>(ea.gate)[(row / ea.rpg) * ea.gstride + col], bf16_to_f32(v), x);
    else
        x = x + bf16_to_f32(v);
    *r = x;
    if (Y) Y[(int64_t)row * ldy + col] = f32_to_bf16(x);
}

template <int EPI>
__device__ __forceinline__ unsigned short epi_apply1(unsigned short v, int row, int col, const EpiArgs& ea) {
    if constexpr (EPI == EPI_SILU) return f32_to_bf16(epi_silu(bf16_to_f32(v)));
    if constexpr (EPI == EPI_GELU) return f32_to_bf16(epi_gelu(bf16_to_f32(v)));
    if constexpr (EPI == EPI_GELU_ERF) return f32_to_bf16(epi_gelu_erf(bf16_to_f32(v)));
    if constexpr (EPI == EPI_RES) return f32_to_bf16(bf16_to_f32(ea.res[(int64_t)row * ea.ldr + col]) + bf16_to_f32(v));
    if constexpr (EPI == EPI_MUL) return f32_to_bf16(bf16_to_f32(ea.res[(int64_t)row * ea.ldr + col]) * bf16_to_f32(v));
    if constexpr (EPI == EPI_GATED)
        return f32_to_bf16(bf16_to_f32(ea.res[(int64_t)row * ea.ldr + col]) +
                           bf16_to_f32(ea.gate[(row / ea.rpg) * ea.gstride + col]) * bf16_to_f32(v));
    return v;
}

template <int EPI = EPI_NONE>
__device__ __forceinline__ void store_tile_t(f32x4 (&acc)[8][4], char* smem, int wave, int lane, int m0, int n0,
                                             int rbase, int cbase, int M, int N, unsigned short* __restrict__ Y,
                                             int64_t ldy, const EpiArgs& ea = EpiArgs{}) {
    constexpr int ROWB = 128, SLOTS = 8;
    char* ctile = smem + wave * (128 * ROWB);
    const int r_l = lane & 15, c_l = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rr = i * 16 + r_l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int cc = j * 16 + c_l;
            const int slot = (cc >> 3) ^ (rr & (SLOTS - 1));
            u16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f32_to_bf16(acc[i][j][e]);
            *reinterpret_cast<u16x4*>(ctile + rr * ROWB + slot * 16 + (cc & 7) * 2) = o;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (wave-private tile)
    constexpr bool E32 = EPI == EPI_RES32 || EPI == EPI_GATED32;
    const bool full = m0 + rbase + 128 <= M && n0 + cbase + 64 <= N && (ldy & 7) == 0 && (((uintptr_t)Y) & 15) == 0;
    const bool epi_vec = EPI == EPI_NONE || EPI == EPI_SILU || EPI == EPI_GELU || EPI == EPI_GELU_ERF ||
                         ((ea.ldr & 7) == 0 && (((uintptr_t)ea.res) & 15) == 0 &&
                          ((EPI != EPI_GATED && EPI != EPI_GATED32) ||
                           ((ea.gstride & 7) == 0 && (((uintptr_t)ea.gate) & 15) == 0)));
    if (full && epi_vec) {  // interior wave tile: all 16 row reads in flight, then 16 unconditional 16-B stores
        u16x8 v[16];
#pragma unroll
        for (int it = 0; it < 16; ++it) {
            const int rr = it * 8 + (lane >> 3), sl = lane & 7;
            v[it] = *reinterpret_cast<const u16x8*>(ctile + rr * ROWB + ((sl ^ (rr & (SLOTS - 1))) << 4));
        }
        const int row0 = m0 + rbase + (lane >> 3), col0 = n0 + cbase + (lane & 7) * 8;
        if constexpr (E32) {
            // the fp32 residual rows (and gates) of 8 row-steps are all loaded before any is stored: one
            // epi_store32 per row-step put every res load behind the previous row-step's stores (the
            // compiler cannot prove they do not alias), i.e. 16 serial HBM round trips per wave
            float* rb = const_cast<float*>(reinterpret_cast<const float*>(ea.res));
            const float* gb = reinterpret_cast<const float*>(ea.gate);
#pragma unroll
            for (int h = 0; h < 16; h += 8) {
                float4 rv[8][2], gv[8][2];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int row = row0 + (h + i) * 8;
                    const float* r = rb + (int64_t)row * ea.ldr + col0;
                    rv[i][0] = *reinterpret_cast<const float4*>(r);
                    rv[i][1] = *reinterpret_cast<const float4*>(r + 4);
                    if constexpr (EPI == EPI_GATED32) {
                        const float* g = gb + (int64_t)(row / ea.rpg) * ea.gstride + col0;
                        gv[i][0] = *reinterpret_cast<const float4*>(g);
                        gv[i][1] = *reinterpret_cast<const float4*>(g + 4);
                    }
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int row = row0 + (h + i) * 8;
                    const u16x8 yv = v[h + i];
                    float x[8] = {rv[i][0].x, rv[i][0].y, rv[i][0].z, rv[i][0].w,
                                  rv[i][1].x, rv[i][1].y, rv[i][1].z, rv[i][1].w};
                    if constexpr (EPI == EPI_GATED32) {
                        const float gg[8] = {gv[i][0].x, gv[i][0].y, gv[i][0].z, gv[i][0].w,
                                             gv[i][1].x, gv[i][1].y, gv[i][1].z, gv[i][1].w};
#pragma unroll
                        for (int u = 0; u < 8; ++u) x[u] = __builtin_fmaf(gg[u], bf16_to_f32(yv[u]), x[u]);
                    } else {
#pragma unroll
                        for (int u = 0; u < 8; ++u) x[u] = x[u] + bf16_to_f32(yv[u]);
                    }
                    float* r = rb + (int64_t)row * ea.ldr + col0;
                    *reinterpret_cast<float4*>(r) = float4{x[0], x[1], x[2], x[3]};
                    *reinterpret_cast<float4*>(r + 4) = float4{x[4], x[5], x[6], x[7]};
                    if (Y) {
                        u16x8 o;
#pragma unroll
                        for (int u = 0; u < 8; ++u) o[u] = f32_to_bf16(x[u]);
                        *reinterpret_cast<u16x8*>(Y + (int64_t)row * ldy + col0) = o;
                    }
                }
            }
            return;
        }
        if constexpr (EPI != EPI_NONE && !E32) {
#pragma unroll
            for (int it = 0; it < 16; ++it) v[it] = epi_apply<EPI>(v[it], row0 + it * 8, col0, ea);
        }
        unsigned short* dst = Y + (int64_t)row0 * ldy + col0;
#pragma unroll
        for (int it = 0; it < 16; ++it) *reinterpret_cast<u16x8*>(dst + (int64_t)it * 8 * ldy) = v[it];
        return;
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int rr = it * 8 + (lane >> 3), sl = lane & 7;
        const int row = m0 + rbase + rr;
        const int col = n0 + cbase + sl * 8;
        if (row >= M || col >= N) continue;
        u16x8 v = *reinterpret_cast<const u16x8*>(ctile + rr * ROWB + ((sl ^ (rr & (SLOTS - 1))) << 4));
        if constexpr (E32) {
            if (col + 8 <= N && epi_vec && (ldy & 7) == 0 && (((uintptr_t)Y) & 15) == 0)
                epi_store32<EPI>(v, row, col, ea, Y, ldy);
            else
                for (int u = 0; u < 8 && col + u < N; ++u) epi_store32_1<EPI>(v[u], row, col + u, ea, Y, ldy);
            continue;
        }
        unsigned short* dst = Y + (int64_t)row * ldy + col;
        if (col + 8 <= N && (((uintptr_t)dst) & 15) == 0 && epi_vec) {
            if constexpr (EPI != EPI_NONE) v = epi_apply<EPI>(v, row, col, ea);
            *reinterpret_cast<u16x8*>(dst) = v;
        } else {
            for (int u = 0; u < 8 && col + u < N; ++u) dst[u] = epi_apply1<EPI>(v[u], row, col + u, ea);
        }
    }
}

__device__ __forceinline__ short bf16_bits(float f) { return (short)f32_to_bf16(f); }

// acc[i][j] += L_i . R_j over one 32-deep k-step, which adds bias[n] + scale * T[m,:] . B_k[n,:] to
// every element of the wave's 128x64 tile.  k-slots 0..7 (lanes 0-15 of a fragment) carry the
// tile's first member a = m0 / rows_per_member, slots 8..15 (lanes 16-31) the next member b (a tile
// spans at most two members when rows_per_member >= 256); each row puts its data in its own
// member's block and zeros in the other:
//   L[m] = [Th_q (R) | Tl_q (R) | Th_q (R) | 1 | 0..]      R[n] = [sBh_q | sBh_q | sBl_q | bias | 0..]
// with T = Th + Tl and s*B = sBh + sBl split into bf16 pairs, so the product is
// Th.sBh + Tl.sBh + Th.sBl + bias: fp32-accurate to ~2^-16 relative (the Tl.sBl term is dropped).
// TL: T comes from the fused projection's LDS rows [256][member a q0 q1 | member b q0 q1] instead of
// the global [M][R] array of k_lora_project.
template <int R, bool TL = false>
__device__ __forceinline__ void lora_mfma_addend(f32x4 (&acc)[8][4], int lane, int m0, int n0, int rbase, int cbase,
                                                 const unsigned short* __restrict__ bias, const float* __restrict__ T,
                                                 const float* __restrict__ theta_pop, int64_t ld_theta, int64_t offB,
                                                 float scale, int rows_per_member, int M, int N) {
    static_assert(3 * R + 1 <= 8, "MFMA epilogue needs 3R+1 <= 8 k-slots per member");
    const int h = lane >> 4, l16 = lane & 15;
    const int ma = m0 / rows_per_member;
    const int last = (m0 + 255 < M ? m0 + 255 : M - 1);
    const bool straddle = last / rows_per_member != ma;
    bf16x8 rf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int col = n0 + cbase + j * 16 + l16;
        col = col < N ? col : N - 1;
        short v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (h == 0 || (h == 1 && straddle)) {
            if constexpr (R > 0) {
                const float* Bk = theta_pop + (int64_t)(ma + h) * ld_theta + offB;
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    const float sb = scale * Bk[col * R + q];
                    const short hi = bf16_bits(sb);
                    v[q] = hi;
                    v[R + q] = hi;
                    v[2 * R + q] = bf16_bits(sb - bf16_to_f32((unsigned short)hi));
                }
            }
            v[3 * R] = bias ? (short)bias[col] : (short)0;
        }
        rf[j] = *reinterpret_cast<bf16x8*>(v);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int row = m0 + rbase + i * 16 + l16;
        row = row < M ? row : M - 1;
        short v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (h == row / rows_per_member - ma) {
            if constexpr (R > 0) {
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    const float t = TL ? T[(row - m0) * 4 + h * 2 + q] : T[(int64_t)row * R + q];
                    const short th = bf16_bits(t);
                    v[q] = th;
                    v[R + q] = bf16_bits(t - bf16_to_f32((unsigned short)th));
                    v[2 * R + q] = th;
                }
            }
            v[3 * R] = (short)0x3F80;  // 1.0
        }
        const bf16x8 lf = *reinterpret_cast<bf16x8*>(v);
#pragma unroll
        for (int j = 0; j < 4; ++j)  // transposed fragments (TR main loop): D[n][m]
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rf[j], lf, acc[i][j], 0, 0, 0);
    }
}

// Epilogue operands of the MFMA LoRA addend, prefetched into LDS (after the 128 KiB ring) by
// 4-byte LDS-DMAs issued before the GEMM prologue — the prologue's counted vmcnt retires them, so
// the epilogue reads LDS instead of waiting on dependent global loads after the last MFMA:
// T rows [m0, m0 + 256) x R, B_k columns [n0, n0 + 256) x R of the tile's first member (and of the
// next one when the tile straddles two), bias[n0, n0 + 256).  Out-of-range bytes read as 0.
namespace epi {
constexpr int T = 0, B0 = 2048, B1 = 4096, BIAS = 6144, BYTES = 6656;
}

template <int R>
__device__ __forceinline__ void epi_prefetch(char* ep, int wave, int lane, int m0, int n0, int M, int N,
                                             const float* __restrict__ T, const float* __restrict__ theta_pop,
                                             int64_t ld_theta, int64_t offB, const unsigned short* __restrict__ bias,
                                             int rows_per_member) {
    static_assert(R >= 0 && R <= 2, "MFMA addend: r <= 2");
    constexpr int TB = 256 * R * 4;  // bytes of the tile's T rows / B_k columns
    const uint32_t vo = lane * 4;
    if (R > 0 && wave * 256 < TB) {
        const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(T + (int64_t)m0 * R), (short)0, (int)((int64_t)(M - m0) * R * 4), 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void*)(ep + epi::T + wave * 256), 4, vo, wave * 256, 0, 0);
        const int ma = m0 / rows_per_member;
        const int nrec = (N - n0) * R * 4;
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(theta_pop + (int64_t)ma * ld_theta + offB + (int64_t)n0 * R), (short)0, nrec, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(ep + epi::B0 + wave * 256), 4, vo, wave * 256, 0, 0);
        const int last = m0 + 255 < M ? m0 + 255 : M - 1;
        if (last / rows_per_member != ma) {
            const __amdgpu_buffer_rsrc_t rb1 = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(theta_pop + (int64_t)(ma + 1) * ld_theta + offB + (int64_t)n0 * R), (short)0, nrec, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rb1, (lds_void*)(ep + epi::B1 + wave * 256), 4, vo, wave * 256, 0,
                                                     0);
        }
    }
    if (bias && wave < 2) {
        const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)(bias + n0), (short)0,
                                                                            (N - n0) * 2, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rz, (lds_void*)(ep + epi::BIAS + wave * 256), 4, vo, wave * 256, 0, 0);
    }
}

// lora_mfma_addend with every operand read from the prefetched LDS block (same k-slot layout).
// Branch-free: every lane reads its candidate operands (all inside the LDS block) back to back under
// one lgkmcnt wait, and a lane whose k-slot block is not its row's / column's member keeps zeros by
// select — divergent ifs around the reads serialised eight LDS round trips.  A row's member offset is
// one compare against the tile-local start of the next member (the tile spans at most two).
template <int R>
__device__ __forceinline__ void lora_mfma_addend_lds(f32x4 (&acc)[8][4], int lane, int m0, int rbase, int cbase,
                                                     const char* ep, bool has_bias, float scale, int rows_per_member,
                                                     int M) {
    const int h = lane >> 4, l16 = lane & 15;
    const int ma = m0 / rows_per_member;
    const int last = (m0 + 255 < M ? m0 + 255 : M - 1);
    const bool straddle = last / rows_per_member != ma;
    const int bnd = (ma + 1) * rows_per_member - m0;  // tile-local first row of member a + 1
    const float* Tl = reinterpret_cast<const float*>(ep + epi::T);
    const unsigned short* bl = reinterpret_cast<const unsigned short*>(ep + epi::BIAS);
    const float* Bk = reinterpret_cast<const float*>(ep + (h == 1 ? epi::B1 : epi::B0));
    const bool con = h == 0 || (h == 1 && straddle);
    float bv[4][R > 0 ? R : 1], tv[8][R > 0 ? R : 1];
    unsigned short bb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = cbase + j * 16 + l16;  // tile-local column
#pragma unroll
        for (int q = 0; q < R; ++q) bv[j][q] = Bk[c * R + q];
        bb[j] = bl[c];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < R; ++q) tv[i][q] = Tl[(rbase + i * 16 + l16) * R + q];
    bf16x8 rf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        short v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float sb = scale * bv[j][q];
            const short hi = bf16_bits(sb);
            v[q] = hi;
            v[R + q] = hi;
            v[2 * R + q] = bf16_bits(sb - bf16_to_f32((unsigned short)hi));
        }
        v[3 * R] = has_bias ? (short)bb[j] : (short)0;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = con ? v[e] : (short)0;
        rf[j] = *reinterpret_cast<bf16x8*>(v);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rl = rbase + i * 16 + l16;  // tile-local row
        const bool ron = h == (rl >= bnd ? 1 : 0);
        short v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float t = tv[i][q];
            const short th = bf16_bits(t);
            v[q] = th;
            v[R + q] = bf16_bits(t - bf16_to_f32((unsigned short)th));
            v[2 * R + q] = th;
        }
        v[3 * R] = (short)0x3F80;  // 1.0
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ron ? v[e] : (short)0;
        const bf16x8 lf = *reinterpret_cast<bf16x8*>(v);
#pragma unroll
        for (int j = 0; j < 4; ++j)  // transposed fragments (TR main loop): D[n][m]
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rf[j], lf, acc[i][j], 0, 0, 0);
    }
}

template <int R, bool MF, int EPI = EPI_NONE>
__global__ __launch_bounds__(512, 1) void k_lora_gemm8(
    const unsigned short* __restrict__ X, int64_t ldx, const unsigned short* __restrict__ W, int64_t ldw,
    const unsigned short* __restrict__ bias, const float* __restrict__ T, const float* __restrict__ theta_pop,
    int64_t ld_theta, int64_t offB, float scale, int rows_per_member, int M, int N, int64_t K, int tiles_n,
    unsigned short* __restrict__ Y, int64_t ldy, EpiArgs ea = EpiArgs{}) {
    static_assert(EPI == EPI_NONE || MF, "epilogue ops ride the MFMA-addend path");
    __shared__ __attribute__((aligned(16))) char smem[p8::LDS + (MF ? epi::BYTES : 0)];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    // XCD-aware bijective remap + grouped rasterisation (as k_lora_gemm).
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
    const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
    const int tiles_m = (M + 255) / 256;
    const int per_group = GROUP_M * tiles_n;
    const int grp = tile / per_group, first_m = grp * GROUP_M;
    const int gsize = (tiles_m - first_m) < GROUP_M ? (tiles_m - first_m) : GROUP_M;
    const int in_grp = tile - grp * per_group;
    const int tm = first_m + in_grp % gsize, tn = in_grp / gsize;
    const int m0 = tm * 256, n0 = tn * 256;
    EGG_STAMP_RT(6);
    EGG_STAMP(0);

    const HalfStage sA0 = make_stage<true>(m0, M - 1, ldx, 0, wave, lane);
    const HalfStage sA1 = make_stage<true>(m0, M - 1, ldx, 1, wave, lane);
    const HalfStage sB0 = make_stage<false>(n0, N - 1, ldw, 0, wave, lane);
    const HalfStage sB1 = make_stage<false>(n0, N - 1, ldw, 1, wave, lane);
    char* const e_buf = smem;
    char* const o_buf = smem + p8::BUF;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, 0x7fffffff, 0x00020000);

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[4][2], b[2][2];
    int oA[2], oB[2];
    p8_frag_offsets(oA, wm * 64 + (lane & 15), lane);
    p8_frag_offsets(oB, wn * 32 + (lane & 15), lane);

    const int nk = (int)(K / BK);
    // K-tile byte offset; tiles past the end re-load the last K-tile (into regions nothing reads
    // again), so every phase issues exactly 2 DMAs and the vmcnt counts stay static.
    auto kb = [nk](int t) -> int { return (t < nk ? t : nk - 1) * (BK * 2); };
    if constexpr (MF)  // older than every ring DMA: the prologue's vmcnt(6) retires it
        epi_prefetch<(MF ? R : 0)>(smem + p8::LDS, wave, lane, m0, n0, M, N, T, theta_pop, ld_theta, offB, bias,
                                   rows_per_member);
    // prologue: K-tile 0 complete, K-tile 1 minus its B0 half (issued in phase 1)
    issue_half(rX, sA0, 0, e_buf + p8::RA0, wave);
    issue_half(rW, sB0, 0, e_buf + p8::RB0, wave);
    issue_half(rW, sB1, 0, e_buf + p8::RB1, wave);
    issue_half(rX, sA1, 0, e_buf + p8::RA1, wave);
    issue_half(rX, sA0, kb(1), o_buf + p8::RA0, wave);
    issue_half(rW, sB1, kb(1), o_buf + p8::RB1, wave);
    issue_half(rX, sA1, kb(1), o_buf + p8::RA1, wave);
    wait_vm<10>();  // K-tile 0's A0 + B0 only (early first K-tile, above)
    P8_BAR();
    EGG_STAMP(1);
    if (wm == 1) P8_BAR();  // stagger: group 1 runs one barrier behind

    // Phase p restages the region last read in phase p-1 (quadrant order (0,0) (0,1) (1,1) (1,0)):
    //   1: B0 of t+1 (odd)  2: A0 of t+2  3: B1 of t+2  4: A1 of t+2 + vmcnt(6) retires t+1
    //   5: B0 of t+2 (even) 6: A0 of t+3  7: B1 of t+3  8: A1 of t+3 + vmcnt(6) retires t+2
    int t0 = 0;
    for (; t0 + 1 < nk; t0 += 2) {
        const int k1 = kb(t0 + 1), k2 = kb(t0 + 2), k3 = kb(t0 + 3);
        p8_phase<0, 0, 0, false, MF, 10>(acc, a, b, e_buf, oA, oB, rW, sB0, k1, o_buf + p8::RB0, wave);
        p8_phase<0, 1, 1, false, MF, 10>(acc, a, b, e_buf, oA, oB, rX, sA0, k2, e_buf + p8::RA0, wave);
        p8_phase<1, 1, 2, false, MF>(acc, a, b, e_buf, oA, oB, rW, sB1, k2, e_buf + p8::RB1, wave);
        p8_phase<1, 0, 1, true, MF>(acc, a, b, e_buf, oA, oB, rX, sA1, k2, e_buf + p8::RA1, wave);
        p8_phase<0, 0, 0, false, MF>(acc, a, b, o_buf, oA, oB, rW, sB0, k2, e_buf + p8::RB0, wave);
        p8_phase<0, 1, 1, false, MF>(acc, a, b, o_buf, oA, oB, rX, sA0, k3, o_buf + p8::RA0, wave);
        p8_phase<1, 1, 2, false, MF>(acc, a, b, o_buf, oA, oB, rW, sB1, k3, o_buf + p8::RB1, wave);
        p8_phase<1, 0, 1, true, MF>(acc, a, b, o_buf, oA, oB, rX, sA1, k3, o_buf + p8::RA1, wave);
    }
    if (t0 < nk) {  // odd K-tile count: the last tile is in the even buffer (retired by phase 8)
        const int k1 = kb(t0 + 1), k2 = kb(t0 + 2);
        p8_phase<0, 0, 0, false, MF, 10>(acc, a, b, e_buf, oA, oB, rW, sB0, k1, o_buf + p8::RB0, wave);
        p8_phase<0, 1, 1, false, MF, 10>(acc, a, b, e_buf, oA, oB, rX, sA0, k2, e_buf + p8::RA0, wave);
        p8_phase<1, 1, 2, false, MF>(acc, a, b, e_buf, oA, oB, rW, sB1, k2, e_buf + p8::RB1, wave);
        p8_phase<1, 0, 1, false, MF>(acc, a, b, e_buf, oA, oB, rX, sA1, k2, e_buf + p8::RA1, wave);
    }
    if (wm == 0) P8_BAR();  // balance the stagger
    EGG_STAMP(2);
    P8_VM0();
    __syncthreads();  // every wave is past its last LDS read: the epilogue reuses the ring
    EGG_STAMP(3);

    if constexpr (MF) {  // bias + LoRA term as one extra MFMA k-step, then a plain bf16 store
        lora_mfma_addend_lds<(MF ? R : 0)>(acc, lane, m0, wm * 128, wn * 64, smem + p8::LDS, bias != nullptr, scale,
                                           rows_per_member, M);
        EGG_STAMP(4);
        store_tile_t<EPI>(acc, smem, wave, lane, m0, n0, wm * 128, wn * 64, M, N, Y, ldy, ea);
        EGG_STAMP_DRAIN();
        EGG_STAMP(5);
        EGG_STAMP_RT(7);
    } else {
        lora_epilogue<R, 128, 64>(acc, smem, wave, lane, m0, n0, wm * 128, wn * 64, bias, T, theta_pop, ld_theta,
                                  offB, scale, rows_per_member, 256, M, N, Y, ldy);
    }
}

// ------------------------------------------------------------------------------------
// 256 x 320 variant of the 8-phase kernel (kernel 10): the same schedule, 8 waves (2 M x 4 N), each
// wave a 128 x 80 sub-tile = 8 x 5 fragments of 16 x 16.  The N side of a K-tile is split into two
// LDS regions by fragment column: B0 = n-fragments 0-2 of every wave column (192 rows, 3 DMAs per
// wave), B1 = n-fragments 3-4 (128 rows, 2 DMAs); A0 / A1 as in k_lora_gemm8.  Quadrant order
// (0,0) (0,1) (1,1) (1,0) = 24, 16, 16, 24 MFMAs.  Why: per 64-deep K-tile the ring moves
// (256 + 320) x 128 B = 72 KiB for 2,560 MFMA cycles per SIMD (28.1 B/cycle/CU) instead of 64 KiB for
// 2,048 (32 B/cycle/CU) — the 256 x 256 main loop is bound by the per-CU LDS-DMA fill rate (28-30
// B/cycle/CU measured), so 10 % fewer fill bytes per MFMA; 2240 and 11200 (the Sana
// widths) are multiples of 320, so the 256-wide tiling's 2.8 % of padded columns at N = 2240 go away;
// and the per-tile prologue / addend / C tile amortise over 25 % more MFMAs.  Ring: 2 x 72 KiB.
// vmcnt: the waits retire everything older than the last three half-tiles issued (A0, B1, A1 of
// the next-but-one K-tile = 6 DMAs) exactly as in k_lora_gemm8; the early-first-K-tile waits in
// phases 1 and 2 count 11 (B0 carries 3 DMAs).  Every output element accumulates the same MFMAs in
// the same k order as k_lora_gemm8, so the two kernels are bit-identical.
// ------------------------------------------------------------------------------------
namespace p8n {
constexpr int HA = 128 * 128;            // A half: 128 rows x 128 B
constexpr int HB0 = 192 * 128;           // B0: 4 wave columns x 48 rows
constexpr int HB1 = 128 * 128;           // B1: 4 wave columns x 32 rows
constexpr int RA0 = 0, RA1 = HA, RB0 = 2 * HA, RB1 = 2 * HA + HB0;
constexpr int BUF = 2 * HA + HB0 + HB1;  // 72 KiB
constexpr int LDS = 2 * BUF;             // 144 KiB
constexpr int BN = 320, NF = 5;
// epilogue operand block after the ring: T rows, B_k columns (tile's members a / a+1), bias
constexpr int ET = 0, EB0 = 2048, EB1 = 4608, EBIAS = 7168, EBYTES = 7936;
}  // namespace p8n

template <int NP>
struct StageN {
    uint32_t off[NP];
};

// B-side staging: region row j -> tile column (j / PER) * 80 + FIRST + (j % PER)
template <int NP, int PER, int FIRST>
__device__ __forceinline__ StageN<NP> make_stage_bn(int n0, int row_max, int64_t ld, int wave, int lane) {
    StageN<NP> s;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int j = (i * 8 + wave) * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ (j & 7);
        int gr = n0 + (j / PER) * 80 + FIRST + (j % PER);
        gr = gr < row_max ? gr : row_max;
        s.off[i] = ((uint32_t)gr * (uint32_t)ld + chunk * 8) * 2;
    }
    return s;
}
__device__ __forceinline__ StageN<2> as_stage(const HalfStage& h) { return StageN<2>{{h.off[0], h.off[1]}}; }

// Non-template overloads: the host compilation pass rejects __amdgpu_buffer_rsrc_t in a deduced template.
__device__ __forceinline__ void issue_n(__amdgpu_buffer_rsrc_t rs, const StageN<2>& s, int kbytes, char* region,
                                        int wave) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(region + (i * 8 + wave) * 1024), 16, s.off[i], kbytes,
                                                 0, 0);
}
__device__ __forceinline__ void issue_n(__amdgpu_buffer_rsrc_t rs, const StageN<3>& s, int kbytes, char* region,
                                        int wave) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(region + (i * 8 + wave) * 1024), 16, s.off[i], kbytes,
                                                 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm_n() {
    static_assert(N == 6 || N == 11, "add the literal");
    if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
}

// QB = 0: n-fragments 0..2 (region B0), QB = 1: 3..4 (region B1); W is the MFMA A operand (TR)
template <int QA, int QB>
__device__ __forceinline__ void p8n_mma(f32x4 (&acc)[8][5], const bf16x8 (&a)[4][2], const bf16x8 (&b)[3][2]) {
    constexpr int NB = QB ? 2 : 3, G0 = QB ? 3 : 0;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int g = 0; g < NB; ++g)
                acc[QA * 4 + f][G0 + g] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[g][kk], a[f][kk], acc[QA * 4 + f][G0 + g], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
}

template <int NB>
__device__ __forceinline__ void p8n_read_b(bf16x8 (&b)[3][2], const char* region, const int (&off)[2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int g = 0; g < NB; ++g) b[g][kk] = *reinterpret_cast<const bf16x8*>(region + off[kk] + g * 2048);
}

// one phase: read the quadrant's fragments (RD: 0 = A+B, 1 = B only, 2 = A only), issue one half-tile
// DMA, [early vmcnt], [vmcnt(6)], retire the reads, barrier, 24 or 16 MFMA, barrier
template <int QA, int QB, int RD, bool VM, int EW, int NP>
__device__ __forceinline__ void p8n_phase(f32x4 (&acc)[8][5], bf16x8 (&a)[4][2], bf16x8 (&b)[3][2], const char* buf,
                                          const int (&oA)[2], const int (&oB0)[2], const int (&oB1)[2],
                                          __amdgpu_buffer_rsrc_t rs, const StageN<NP>& st, int kbytes, char* dst,
                                          int wave) {
    if (RD != 2) {
        if (QB) p8n_read_b<2>(b, buf + p8n::RB1, oB1);
        else p8n_read_b<3>(b, buf + p8n::RB0, oB0);
    }
    if (RD != 1) p8_read_a(a, buf + (QA ? p8n::RA1 : p8n::RA0), oA);
    issue_n(rs, st, kbytes, dst, wave);
    if constexpr (EW > 0) wait_vm_n<EW>();
    if (VM) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    P8_LGKM0_;
    P8_BAR();
    p8n_mma<QA, QB>(acc, a, b);
    P8_BAR();
}

template <int R>
__device__ __forceinline__ void epi_prefetch_n(char* ep, int wave, int lane, int m0, int n0, int M, int N,
                                               const float* __restrict__ T, const float* __restrict__ theta_pop,
                                               int64_t ld_theta, int64_t offB, const unsigned short* __restrict__ bias,
                                               int rows_per_member) {
    static_assert(R >= 0 && R <= 2, "MFMA addend: r <= 2");
    const uint32_t vo = lane * 4;
    if constexpr (R > 0) {
        constexpr int TB = 256 * R * 4, BB = p8n::BN * R * 4;
        if (wave * 256 < TB) {
            const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(T + (int64_t)m0 * R), (short)0, (int)((int64_t)(M - m0) * R * 4), 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (lds_void*)(ep + p8n::ET + wave * 256), 4, vo, wave * 256, 0, 0);
        }
        const int ma = m0 / rows_per_member;
        const int nrec = (N - n0) * R * 4;
        const int last = m0 + 255 < M ? m0 + 255 : M - 1;
        const bool straddle = last / rows_per_member != ma;
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(theta_pop + (int64_t)ma * ld_theta + offB + (int64_t)n0 * R), (short)0, nrec, 0x00020000);
        const __amdgpu_buffer_rsrc_t rb1 = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(theta_pop + (int64_t)(ma + 1) * ld_theta + offB + (int64_t)n0 * R), (short)0, straddle ? nrec : 0,
            0x00020000);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int pc = wave + 8 * p;
            if (pc * 256 < BB) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(ep + p8n::EB0 + pc * 256), 4, vo, pc * 256, 0, 0);
                if (straddle)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb1, (lds_void*)(ep + p8n::EB1 + pc * 256), 4, vo, pc * 256,
                                                             0, 0);
            }
        }
    }
    if (bias && wave < 3) {
        const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)(bias + n0), (short)0,
                                                                            (N - n0) * 2, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rz, (lds_void*)(ep + p8n::EBIAS + wave * 256), 4, vo, wave * 256, 0, 0);
    }
}

// lora_mfma_addend_lds over the 128 x 80 wave tile (5 n-fragments), operands from the p8n epilogue block
template <int R>
__device__ __forceinline__ void lora_mfma_addend_n(f32x4 (&acc)[8][5], int lane, int m0, int rbase, int cbase,
                                                   const char* ep, bool has_bias, float scale, int rows_per_member,
                                                   int M) {
    const int h = lane >> 4, l16 = lane & 15;
    const int ma = m0 / rows_per_member;
    const int last = (m0 + 255 < M ? m0 + 255 : M - 1);
    const bool straddle = last / rows_per_member != ma;
    const int bnd = (ma + 1) * rows_per_member - m0;
    const float* Tl = reinterpret_cast<const float*>(ep + p8n::ET);
    const unsigned short* bl = reinterpret_cast<const unsigned short*>(ep + p8n::EBIAS);
    const float* Bk = reinterpret_cast<const float*>(ep + (h == 1 ? p8n::EB1 : p8n::EB0));
    const bool con = h == 0 || (h == 1 && straddle);
    float bv[5][R > 0 ? R : 1], tv[8][R > 0 ? R : 1];
    unsigned short bb[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int c = cbase + j * 16 + l16;
#pragma unroll
        for (int q = 0; q < R; ++q) bv[j][q] = Bk[c * R + q];
        bb[j] = bl[c];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < R; ++q) tv[i][q] = Tl[(rbase + i * 16 + l16) * R + q];
    bf16x8 rf[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        short v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float sb = scale * bv[j][q];
            const short hi = bf16_bits(sb);
            v[q] = hi;
            v[R + q] = hi;
            v[2 * R + q] = bf16_bits(sb - bf16_to_f32((unsigned short)hi));
        }
        v[3 * R] = has_bias ? (short)bb[j] : (short)0;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = con ? v[e] : (short)0;
        rf[j] = *reinterpret_cast<bf16x8*>(v);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rl = rbase + i * 16 + l16;
        const bool ron = h == (rl >= bnd ? 1 : 0);
        short v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float t = tv[i][q];
            const short th = bf16_bits(t);
            v[q] = th;
            v[R + q] = bf16_bits(t - bf16_to_f32((unsigned short)th));
            v[2 * R + q] = th;
        }
        v[3 * R] = (short)0x3F80;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ron ? v[e] : (short)0;
        const bf16x8 lf = *reinterpret_cast<bf16x8*>(v);
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rf[j], lf, acc[i][j], 0, 0, 0);
    }
}

// C tile of the 256 x 320 workgroup tile, staged through ONE shared LDS tile (256 rows x 640 B = all
// 160 KiB; the caller has passed a barrier after the epilogue block's last read) so that the global
// stores write whole 128-B lines: with per-wave staging each wave's 80-column row segment (160 B)
// straddles lines shared with the neighbouring wave and the store phase took 2x the 256 x 256
// kernel's per byte (stamped).  16-B slots are rotated by row ((slot + row) mod 40): the
// 8-B fragment writes are at most 2-way bank-conflicted.  After a barrier, wave w stores rows
// [32w, 32w + 32): 40 lanes per 640-B row, 20 16-B stores per lane.  EPI ops as store_tile_t.
template <int EPI = EPI_NONE>
__device__ __forceinline__ void store_tile_wg(f32x4 (&acc)[8][5], char* smem, int wave, int lane, int m0, int n0,
                                              int wm, int wn, int M, int N, unsigned short* __restrict__ Y,
                                              int64_t ldy, const EpiArgs& ea = EpiArgs{}) {
    constexpr int RB = 640, SL = 40;
    const int r_l = lane & 15, c_l = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rr = wm * 128 + i * 16 + r_l;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            u16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f32_to_bf16(acc[i][j][e]);
            const int c = wn * 80 + j * 16 + c_l;  // tile column: 16-B slot c >> 3, 8-B half (c >> 2) & 1
            *reinterpret_cast<u16x4*>(smem + rr * RB + ((c >> 3) + rr) % SL * 16 + ((c >> 2) & 1) * 8) = o;
        }
    }
    __syncthreads();
    constexpr bool E32 = EPI == EPI_RES32 || EPI == EPI_GATED32;
    const bool vec = (ldy & 7) == 0 && (((uintptr_t)Y) & 15) == 0 &&
                     (EPI == EPI_NONE || EPI == EPI_SILU || EPI == EPI_GELU || EPI == EPI_GELU_ERF ||
                      ((ea.ldr & 7) == 0 && (((uintptr_t)ea.res) & 15) == 0 &&
                       ((EPI != EPI_GATED && EPI != EPI_GATED32) ||
                        ((ea.gstride & 7) == 0 && (((uintptr_t)ea.gate) & 15) == 0))));
    if constexpr (E32) {
        // fp32 residual stream: per group of 5 chunks, every residual (and gate) load issued before any
        // store (one load -> fma -> store per chunk serialises the loads behind the earlier stores)
        float* rb = const_cast<float*>(reinterpret_cast<const float*>(ea.res));
        const float* gb = reinterpret_cast<const float*>(ea.gate);
#pragma unroll
        for (int h = 0; h < 20; h += 5) {
            u16x8 v[5];
            float4 rv[5][2], gv[5][2];
            int rows[5], cols[5];
            bool ok[5];
#pragma unroll
            for (int it = 0; it < 5; ++it) {
                const int idx = (h + it) * 64 + lane, rr = wave * 32 + idx / SL, ch = idx % SL;
                v[it] = *reinterpret_cast<const u16x8*>(smem + rr * RB + (ch + rr) % SL * 16);
                rows[it] = m0 + rr;
                cols[it] = n0 + ch * 8;
                ok[it] = rows[it] < M && cols[it] + 8 <= N && vec;
                if (ok[it]) {
                    const float* r = rb + (int64_t)rows[it] * ea.ldr + cols[it];
                    rv[it][0] = *reinterpret_cast<const float4*>(r);
                    rv[it][1] = *reinterpret_cast<const float4*>(r + 4);
                    if constexpr (EPI == EPI_GATED32) {
                        const float* g = gb + (int64_t)(rows[it] / ea.rpg) * ea.gstride + cols[it];
                        gv[it][0] = *reinterpret_cast<const float4*>(g);
                        gv[it][1] = *reinterpret_cast<const float4*>(g + 4);
                    }
                }
            }
#pragma unroll
            for (int it = 0; it < 5; ++it) {
                const int row = rows[it], col = cols[it];
                if (row >= M || col >= N) continue;
                if (!ok[it]) {   // ragged tail / unaligned: the element form
                    for (int u = 0; u < 8 && col + u < N; ++u) epi_store32_1<EPI>(v[it][u], row, col + u, ea, Y, ldy);
                    continue;
                }
                float x[8] = {rv[it][0].x, rv[it][0].y, rv[it][0].z, rv[it][0].w,
                              rv[it][1].x, rv[it][1].y, rv[it][1].z, rv[it][1].w};
                if constexpr (EPI == EPI_GATED32) {
                    const float gg[8] = {gv[it][0].x, gv[it][0].y, gv[it][0].z, gv[it][0].w,
                                         gv[it][1].x, gv[it][1].y, gv[it][1].z, gv[it][1].w};
#pragma unroll
                    for (int u = 0; u < 8; ++u) x[u] = __builtin_fmaf(gg[u], bf16_to_f32(v[it][u]), x[u]);
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) x[u] = x[u] + bf16_to_f32(v[it][u]);
                }
                float* r = rb + (int64_t)row * ea.ldr + col;
                *reinterpret_cast<float4*>(r) = float4{x[0], x[1], x[2], x[3]};
                *reinterpret_cast<float4*>(r + 4) = float4{x[4], x[5], x[6], x[7]};
                if (Y) {
                    u16x8 o;
#pragma unroll
                    for (int u = 0; u < 8; ++u) o[u] = f32_to_bf16(x[u]);
                    *reinterpret_cast<u16x8*>(Y + (int64_t)row * ldy + col) = o;
                }
            }
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < 20; h += 10) {
        u16x8 v[10];
#pragma unroll
        for (int it = 0; it < 10; ++it) {
            const int idx = (h + it) * 64 + lane, rr = wave * 32 + idx / SL, ch = idx % SL;
            v[it] = *reinterpret_cast<const u16x8*>(smem + rr * RB + (ch + rr) % SL * 16);
        }
#pragma unroll
        for (int it = 0; it < 10; ++it) {
            const int idx = (h + it) * 64 + lane, rr = wave * 32 + idx / SL, ch = idx % SL;
            const int row = m0 + rr, col = n0 + ch * 8;
            if (row >= M || col >= N) continue;
            unsigned short* dst = Y + (int64_t)row * ldy + col;
            if (vec && col + 8 <= N) {
                u16x8 w = v[it];
                if constexpr (EPI != EPI_NONE) w = epi_apply<EPI>(w, row, col, ea);
                *reinterpret_cast<u16x8*>(dst) = w;
            } else {
                for (int u = 0; u < 8 && col + u < N; ++u) dst[u] = epi_apply1<EPI>(v[it][u], row, col + u, ea);
            }
        }
    }
}

// MF path only (r <= 2, rows_per_member >= 256, or r = 0): bias + LoRA term as the MFMA addend
template <int R, int EPI = EPI_NONE>
__global__ __launch_bounds__(512, 1) void k_lora_gemm8n(
    const unsigned short* __restrict__ X, int64_t ldx, const unsigned short* __restrict__ W, int64_t ldw,
    const unsigned short* __restrict__ bias, const float* __restrict__ T, const float* __restrict__ theta_pop,
    int64_t ld_theta, int64_t offB, float scale, int rows_per_member, int M, int N, int64_t K, int tiles_n,
    unsigned short* __restrict__ Y, int64_t ldy, EpiArgs ea = EpiArgs{}) {
    __shared__ __attribute__((aligned(16))) char smem[256 * 640];  // ring + epilogue block; the C tile: all of it
    static_assert(p8n::LDS + p8n::EBYTES <= 256 * 640, "LDS layout");
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
    const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
    const int tiles_m = (M + 255) / 256;
    const int per_group = GROUP_M * tiles_n;
    const int grp = tile / per_group, first_m = grp * GROUP_M;
    const int gsize = (tiles_m - first_m) < GROUP_M ? (tiles_m - first_m) : GROUP_M;
    const int in_grp = tile - grp * per_group;
    const int tm = first_m + in_grp % gsize, tn = in_grp / gsize;
    const int m0 = tm * 256, n0 = tn * p8n::BN;
    EGG_STAMP_RT(6);
    EGG_STAMP(0);

    const StageN<2> sA0 = as_stage(make_stage<true>(m0, M - 1, ldx, 0, wave, lane));
    const StageN<2> sA1 = as_stage(make_stage<true>(m0, M - 1, ldx, 1, wave, lane));
    const StageN<3> sB0 = make_stage_bn<3, 48, 0>(n0, N - 1, ldw, wave, lane);
    const StageN<2> sB1 = make_stage_bn<2, 32, 48>(n0, N - 1, ldw, wave, lane);
    char* const e_buf = smem;
    char* const o_buf = smem + p8n::BUF;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, 0x7fffffff, 0x00020000);

    f32x4 acc[8][5];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[4][2], b[3][2];
    int oA[2], oB0[2], oB1[2];
    p8_frag_offsets(oA, wm * 64 + (lane & 15), lane);
    p8_frag_offsets(oB0, wn * 48 + (lane & 15), lane);
    p8_frag_offsets(oB1, wn * 32 + (lane & 15), lane);

    const int nk = (int)(K / BK);
    auto kb = [nk](int t) -> int { return (t < nk ? t : nk - 1) * (BK * 2); };
    epi_prefetch_n<R>(smem + p8n::LDS, wave, lane, m0, n0, M, N, T, theta_pop, ld_theta, offB, bias, rows_per_member);
    issue_n(rX, sA0, 0, e_buf + p8n::RA0, wave);
    issue_n(rW, sB0, 0, e_buf + p8n::RB0, wave);
    issue_n(rW, sB1, 0, e_buf + p8n::RB1, wave);
    issue_n(rX, sA1, 0, e_buf + p8n::RA1, wave);
    issue_n(rX, sA0, kb(1), o_buf + p8n::RA0, wave);
    issue_n(rW, sB1, kb(1), o_buf + p8n::RB1, wave);
    issue_n(rX, sA1, kb(1), o_buf + p8n::RA1, wave);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // K-tile 0's A0 + B0 (5 younger halves x 2 DMAs)
    P8_BAR();
    EGG_STAMP(1);
    if (wm == 1) P8_BAR();

    int t0 = 0;
    for (; t0 + 1 < nk; t0 += 2) {
        const int k1 = kb(t0 + 1), k2 = kb(t0 + 2), k3 = kb(t0 + 3);
        p8n_phase<0, 0, 0, false, 11>(acc, a, b, e_buf, oA, oB0, oB1, rW, sB0, k1, o_buf + p8n::RB0, wave);
        p8n_phase<0, 1, 1, false, 11>(acc, a, b, e_buf, oA, oB0, oB1, rX, sA0, k2, e_buf + p8n::RA0, wave);
        p8n_phase<1, 1, 2, false, 0>(acc, a, b, e_buf, oA, oB0, oB1, rW, sB1, k2, e_buf + p8n::RB1, wave);
        p8n_phase<1, 0, 1, true, 0>(acc, a, b, e_buf, oA, oB0, oB1, rX, sA1, k2, e_buf + p8n::RA1, wave);
        p8n_phase<0, 0, 0, false, 0>(acc, a, b, o_buf, oA, oB0, oB1, rW, sB0, k2, e_buf + p8n::RB0, wave);
        p8n_phase<0, 1, 1, false, 0>(acc, a, b, o_buf, oA, oB0, oB1, rX, sA0, k3, o_buf + p8n::RA0, wave);
        p8n_phase<1, 1, 2, false, 0>(acc, a, b, o_buf, oA, oB0, oB1, rW, sB1, k3, o_buf + p8n::RB1, wave);
        p8n_phase<1, 0, 1, true, 0>(acc, a, b, o_buf, oA, oB0, oB1, rX, sA1, k3, o_buf + p8n::RA1, wave);
    }
    if (t0 < nk) {
        const int k1 = kb(t0 + 1), k2 = kb(t0 + 2);
        p8n_phase<0, 0, 0, false, 11>(acc, a, b, e_buf, oA, oB0, oB1, rW, sB0, k1, o_buf + p8n::RB0, wave);
        p8n_phase<0, 1, 1, false, 11>(acc, a, b, e_buf, oA, oB0, oB1, rX, sA0, k2, e_buf + p8n::RA0, wave);
        p8n_phase<1, 1, 2, false, 0>(acc, a, b, e_buf, oA, oB0, oB1, rW, sB1, k2, e_buf + p8n::RB1, wave);
        p8n_phase<1, 0, 1, false, 0>(acc, a, b, e_buf, oA, oB0, oB1, rX, sA1, k2, e_buf + p8n::RA1, wave);
    }
    if (wm == 0) P8_BAR();
    EGG_STAMP(2);
    P8_VM0();
    __syncthreads();  // every wave is past its last ring read: the epilogue reuses the ring
    EGG_STAMP(3);

    lora_mfma_addend_n<R>(acc, lane, m0, wm * 128, wn * 80, smem + p8n::LDS, bias != nullptr, scale, rows_per_member,
                          M);
    EGG_STAMP(4);
    __syncthreads();  // the C tile overwrites the epilogue block every wave's addend has just read
    store_tile_wg<EPI>(acc, smem, wave, lane, m0, n0, wm, wn, M, N, Y, ldy, ea);
    EGG_STAMP_DRAIN();
    EGG_STAMP(5);
    EGG_STAMP_RT(7);
}

// ------------------------------------------------------------------------------------
// Y += scale * T B_k^T   (8 bf16 per thread)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_lora_expand(const float* __restrict__ T, const float* __restrict__ theta_pop,
                                                     int64_t ld_theta, int64_t offB, int r, float scale,
                                                     int64_t rows_per_member, int64_t M, int64_t N,
                                                     unsigned short* __restrict__ Y, int64_t ldy) {
    const int64_t nch = (N + 7) / 8;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= M * nch) return;
    const int64_t row = idx / nch, c0 = (idx - row * nch) * 8;
    const int64_t kl = row / rows_per_member;
    const float* Bk = theta_pop + kl * ld_theta + offB;
    const float* t = T + row * r;
    unsigned short* y = Y + row * ldy + c0;
    for (int u = 0; u < 8 && c0 + u < N; ++u) {
        float d = 0.0f;
        for (int qq = 0; qq < r; ++qq) d += t[qq] * Bk[(c0 + u) * r + qq];
        y[u] = f32_to_bf16(bf16_to_f32(y[u]) + scale * d);
    }
}

// fp32 population LoRA term of LoRALinear.forward_fp32 (the time / guidance embedders, AdaLN modulation and
// proj_out — the few small linears whose bf16 rounding moved whole members):
//   y[m, :] += scale * (x[m, :] A_k^T) B_k^T,   k = m / rows_per_member,
// A_k = A + k * lda_member as [R][K], B_k = B + k * ldb_member as [N][R] (the PEFT lora_A / lora_B layouts of
// es_backend.py:193-200; member stride 0 = one adapter for every row).  One wave per row, grid-stride: the
// skinny product T = x A_k^T as per-lane fp32 partial sums over k = lane + 64 i, reduced by a fixed xor
// butterfly (a row's bits do not depend on the member count or the grid), then the rank-R expansion
// y[m, n] + (T B_k^T)[n] * scale in PEFT's order (result + lora_B(lora_A(x)) * scaling).
template <int R>
__global__ __launch_bounds__(256) void k_lora_delta_f32(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ A, int64_t lda_m,
                                                        const float* __restrict__ B, int64_t ldb_m, float scale,
                                                        int64_t rows_per_member, int64_t M, int N, int K,
                                                        float* __restrict__ y, int64_t ldy) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t m = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); m < M; m += nwaves) {
        const int64_t kl = m / rows_per_member;
        const float* xr = x + m * ldx;
        const float* Ak = A + kl * lda_m;
        float t[R];
#pragma unroll
        for (int q = 0; q < R; ++q) t[q] = 0.0f;
#pragma unroll 4
        for (int k = lane; k < K; k += 64) {
            const float xv = xr[k];
#pragma unroll
            for (int q = 0; q < R; ++q) t[q] = fmaf(xv, Ak[(int64_t)q * K + k], t[q]);
        }
#pragma unroll
        for (int q = 0; q < R; ++q)
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) t[q] += __shfl_xor(t[q], o, 64);
        const float* Bk = B + kl * ldb_m;
        float* yr = y + m * ldy;
        for (int n = lane; n < N; n += 64) {
            float d = 0.0f;
#pragma unroll
            for (int q = 0; q < R; ++q) d = fmaf(t[q], Bk[(int64_t)n * R + q], d);
            yr[n] = yr[n] + d * scale;
        }
    }
}

template <int R, int NI>
static void launch_project_ra(const void* X, int64_t ldx, const float* tp, int64_t ldt, int64_t offA, int64_t rpm,
                              int64_t M, int64_t K, float* T, hipStream_t st) {
    const int64_t rows_per_block = 4 * PR_ROWS;
    hipLaunchKernelGGL((k_lora_project_ra<R, NI>), dim3((unsigned)((M + rows_per_block - 1) / rows_per_block)),
                       dim3(256), 0, st, (const unsigned short*)X, ldx, tp, ldt, offA, rpm, M, K, T);
}

template <int R>
static void launch_project(const void* X, int64_t ldx, const float* tp, int64_t ldt, int64_t offA, int64_t rpm,
                           int64_t M, int64_t K, float* T, hipStream_t st) {
    if constexpr (R <= 2) {  // register-resident A for K <= 4096
        const int64_t ni = (K + 511) / 512;
        switch (ni) {
            case 1: return launch_project_ra<R, 1>(X, ldx, tp, ldt, offA, rpm, M, K, T, st);
            case 2: return launch_project_ra<R, 2>(X, ldx, tp, ldt, offA, rpm, M, K, T, st);
            case 3: return launch_project_ra<R, 3>(X, ldx, tp, ldt, offA, rpm, M, K, T, st);
            case 4: return launch_project_ra<R, 4>(X, ldx, tp, ldt, offA, rpm, M, K, T, st);
            case 5: return launch_project_ra<R, 5>(X, ldx, tp, ldt, offA, rpm, M, K, T, st);
            case 6: return launch_project_ra<R, 6>(X, ldx, tp, ldt, offA, rpm, M, K, T, st);
            case 8: return launch_project_ra<R, 8>(X, ldx, tp, ldt, offA, rpm, M, K, T, st);
            default: break;
        }
    }
    hipLaunchKernelGGL(k_lora_project<R>, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st,
                       (const unsigned short*)X, ldx, tp, ldt, offA, rpm, M, K, T);
}

static int project(const void* X, int64_t ldx, const float* tp, int64_t ldt, int64_t offA, int32_t r, int64_t rpm,
                   int64_t M, int64_t K, float* T, hipStream_t st) {
    switch (r) {
        case 1: launch_project<1>(X, ldx, tp, ldt, offA, rpm, M, K, T, st); break;
        case 2: launch_project<2>(X, ldx, tp, ldt, offA, rpm, M, K, T, st); break;
        case 3: launch_project<3>(X, ldx, tp, ldt, offA, rpm, M, K, T, st); break;
        case 4: launch_project<4>(X, ldx, tp, ldt, offA, rpm, M, K, T, st); break;
        case 8: launch_project<8>(X, ldx, tp, ldt, offA, rpm, M, K, T, st); break;
        case 16: launch_project<16>(X, ldx, tp, ldt, offA, rpm, M, K, T, st); break;
        default: set_error("lora: r=%d unsupported (1,2,3,4,8,16)", r); return EGGROLL_ERR_UNSUPPORTED;
    }
    EGG_CHECK_LAUNCH("lora_project");
    return EGGROLL_OK;
}

// ------------------------------------------------------------------------------------
// Fused-projection variant of the 8-phase kernel (r <= 2, rows_per_member >= 256): T = X A_k^T is
// computed inside the GEMM from the X fragments already in registers, so X is read from HBM once
// per LoRA linear instead of twice (k_lora_project's pre-pass is gone).
//   AK[k][16][K] bf16 (k_lora_ak): rows q < R hold hi(A_k[q]), rows R+q lo(A_k[q] - hi), rest 0.
//   Per K-tile a 2 KiB AK block is DMA'd next to the half-tiles: LDS rows 0..7 = member a (the
//   tile's first member), rows 8..15 = member b (the next one; a tile spans at most two).
//   In phases 2 and 4 (resp. 6, 8) wave (wm, wn) runs one extra transposed MFMA per k-substep on
//   its X fragment f = wn:  D[q][m] += AK[q, k] X[m, k]  -> 4 MFMA per K-tile per wave (+6.25 %).
//   At the end T[m][q] = D[q] + D[R + q] (hi + lo) per member goes to LDS for the MFMA epilogue.
// ------------------------------------------------------------------------------------
namespace p8f {
constexpr int AKB = 2048;                  // AK block per K-tile: 16 rows x 64 bf16
constexpr int BUF = p8::BUF + AKB;         // 66 KiB per K-tile buffer
constexpr int RK = p8::BUF;                // AK region inside a buffer
constexpr int TOFF = 2 * BUF;              // T rows after the ring: [256][4] fp32
constexpr int LDS = TOFF + 256 * 4 * 4;    // 136 KiB
}  // namespace p8f

__global__ __launch_bounds__(256) void k_lora_ak(const float* __restrict__ theta_pop, int64_t ld_theta, int64_t offA,
                                                 int R, int64_t K, int n_members, unsigned short* __restrict__ AK) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one thread per 8 elements
    const int64_t per_row = K / 8, total = (int64_t)n_members * 16 * per_row;
    if (idx >= total) return;
    const int64_t c = (idx % per_row) * 8;
    const int row = (int)((idx / per_row) % 16);
    const int k = (int)(idx / (per_row * 16));
    u16x8 o;
    if (row < 2 * R) {
        const int q = row % R;
        const float* A = theta_pop + (int64_t)k * ld_theta + offA + (int64_t)q * K + c;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const unsigned short hi = f32_to_bf16(A[u]);
            o[u] = row < R ? hi : f32_to_bf16(A[u] - bf16_to_f32(hi));
        }
    } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = 0;
    }
    *reinterpret_cast<u16x8*>(AK + ((int64_t)k * 16 + row) * K + c) = o;
}

template <int R>
__global__ __launch_bounds__(512, 1) void k_lora_gemm8f(
    const unsigned short* __restrict__ X, int64_t ldx, const unsigned short* __restrict__ W, int64_t ldw,
    const unsigned short* __restrict__ bias, const unsigned short* __restrict__ AK, const float* __restrict__ theta_pop,
    int64_t ld_theta, int64_t offB, float scale, int rows_per_member, int n_members, int M, int N, int64_t K,
    int tiles_n, unsigned short* __restrict__ Y, int64_t ldy) {
    __shared__ __attribute__((aligned(16))) char smem[p8f::LDS];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
    const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
    const int tiles_m = (M + 255) / 256;
    const int per_group = GROUP_M * tiles_n;
    const int grp = tile / per_group, first_m = grp * GROUP_M;
    const int gsize = (tiles_m - first_m) < GROUP_M ? (tiles_m - first_m) : GROUP_M;
    const int in_grp = tile - grp * per_group;
    const int tm = first_m + in_grp % gsize, tn = in_grp / gsize;
    const int m0 = tm * 256, n0 = tn * 256;

    const HalfStage sA0 = make_stage<true>(m0, M - 1, ldx, 0, wave, lane);
    const HalfStage sA1 = make_stage<true>(m0, M - 1, ldx, 1, wave, lane);
    const HalfStage sB0 = make_stage<false>(n0, N - 1, ldw, 0, wave, lane);
    const HalfStage sB1 = make_stage<false>(n0, N - 1, ldw, 1, wave, lane);
    // AK DMA: one dword per lane per K-tile; wave w fills LDS AK rows 2w, 2w+1 (swizzled like the tiles)
    const int ma = m0 / rows_per_member;
    const int mb = (ma + 1 < n_members) ? ma + 1 : ma;
    uint32_t akoff;
    {
        const int row = 2 * wave + (lane >> 5), d = lane & 31, slot = d >> 2;
        const int src_row = (row < 8 ? ma : mb) * 16 + (row & 7);
        const int chunk = slot ^ (row & 7);
        akoff = ((uint32_t)src_row * (uint32_t)K + chunk * 8 + (d & 3) * 2) * 2;
    }
    char* const e_buf = smem;
    char* const o_buf = smem + p8f::BUF;
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rK = __builtin_amdgcn_make_buffer_rsrc((void*)AK, (short)0, 0x7fffffff, 0x00020000);
    auto issue_ak = [&](int kbytes, char* buf) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rK, (lds_void*)(buf + p8f::RK + wave * 256), 4, akoff, kbytes, 0, 0);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 tacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    bf16x8 a[4][2], b[2][2], ak[2];
    int oA[2], oB[2], oK[2];
    p8_frag_offsets(oA, wm * 64 + (lane & 15), lane);
    p8_frag_offsets(oB, wn * 32 + (lane & 15), lane);
    p8_frag_offsets(oK, lane & 15, lane);

    auto tmma = [&](int h) {  // T-MFMA on this wave's X fragment f = wn (wave-uniform branches, no selects)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            if (wn == 0) tacc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak[kk], a[0][kk], tacc[h], 0, 0, 0);
            else if (wn == 1) tacc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak[kk], a[1][kk], tacc[h], 0, 0, 0);
            else if (wn == 2) tacc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak[kk], a[2][kk], tacc[h], 0, 0, 0);
            else tacc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak[kk], a[3][kk], tacc[h], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
    };
    auto read_ak = [&](const char* buf) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) ak[kk] = *reinterpret_cast<const bf16x8*>(buf + p8f::RK + oK[kk]);
    };

    const int nk = (int)(K / BK);
    auto kb = [nk](int t) -> int { return (t < nk ? t : nk - 1) * (BK * 2); };
    issue_half(rX, sA0, 0, e_buf + p8::RA0, wave);
    issue_half(rW, sB1, 0, e_buf + p8::RB1, wave);
    issue_ak(0, e_buf);
    issue_half(rX, sA1, 0, e_buf + p8::RA1, wave);
    issue_half(rW, sB0, 0, e_buf + p8::RB0, wave);
    issue_half(rX, sA0, kb(1), o_buf + p8::RA0, wave);
    issue_half(rW, sB1, kb(1), o_buf + p8::RB1, wave);
    issue_ak(kb(1), o_buf);
    issue_half(rX, sA1, kb(1), o_buf + p8::RA1, wave);
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    P8_BAR();
    if (wm == 1) P8_BAR();

    // As k_lora_gemm8, plus: AK read in phase 2/6 (last read -> restaged with B1 in phase 3/7),
    // T-MFMA on A0 in phase 2/6 and on A1 in phase 4/8; 7 DMAs issued after a buffer's last one.
#define P8F_K(buf_, dst_, kA, kB, DO_TAIL)                                                          \
    /* phase 1 */                                                                                   \
    p8_read_b(b, buf_ + p8::RB0, oB);                                                               \
    p8_read_a(a, buf_ + p8::RA0, oA);                                                               \
    issue_half(rW, sB0, kA, (buf_ == e_buf ? o_buf : e_buf) + p8::RB0, wave);                       \
    P8_LGKM0_;                                                                                      \
    P8_BAR();                                                                                       \
    p8_mma<0, 0, true>(acc, a, b);                                                                  \
    P8_BAR();                                                                                       \
    /* phase 2 */                                                                                   \
    p8_read_b(b, buf_ + p8::RB1, oB);                                                               \
    read_ak(buf_);                                                                                  \
    issue_half(rX, sA0, kB, dst_ + p8::RA0, wave);                                                  \
    P8_LGKM0_;                                                                                      \
    P8_BAR();                                                                                       \
    p8_mma<0, 1, true>(acc, a, b);                                                                  \
    tmma(0);                                                                                        \
    P8_BAR();                                                                                       \
    /* phase 3 */                                                                                   \
    p8_read_a(a, buf_ + p8::RA1, oA);                                                               \
    issue_half(rW, sB1, kB, dst_ + p8::RB1, wave);                                                  \
    issue_ak(kB, dst_);                                                                             \
    P8_LGKM0_;                                                                                      \
    P8_BAR();                                                                                       \
    p8_mma<1, 1, true>(acc, a, b);                                                                  \
    P8_BAR();                                                                                       \
    /* phase 4 */                                                                                   \
    p8_read_b(b, buf_ + p8::RB0, oB);                                                               \
    issue_half(rX, sA1, kB, dst_ + p8::RA1, wave);                                                  \
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");                                                \
    P8_LGKM0_;                                                                                      \
    P8_BAR();                                                                                       \
    p8_mma<1, 0, true>(acc, a, b);                                                                  \
    tmma(1);                                                                                        \
    P8_BAR();

    int t0 = 0;
    for (; t0 + 1 < nk; t0 += 2) {
        const int k1 = kb(t0 + 1), k2 = kb(t0 + 2), k3 = kb(t0 + 3);
        // even buffer: tile t0; phase 1 restages B0 of t0+1 (odd), phases 2-4 tile t0+2 (even)
        P8F_K(e_buf, e_buf, k1, k2, 0)
        // odd buffer: tile t0+1; phase 5 restages B0 of t0+2 (even), phases 6-8 tile t0+3 (odd)
        P8F_K(o_buf, o_buf, k2, k3, 0)
    }
    if (t0 < nk) {
        const int k1 = kb(t0 + 1), k2 = kb(t0 + 2);
        P8F_K(e_buf, e_buf, k1, k2, 1)
    }
#undef P8F_K
    if (wm == 0) P8_BAR();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // T rows -> LDS: lanes 0-15 hold member a's D rows 0..3, lanes 32-47 member b's D rows 8..11
    {
        float* Tl = reinterpret_cast<float*>(smem + p8f::TOFF);
        const int hq = lane >> 4;
        if (hq == 0 || hq == 2) {
            const int mem = hq >> 1;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int rl = wm * 128 + h * 64 + wn * 16 + (lane & 15);
#pragma unroll
                for (int qq = 0; qq < R; ++qq) Tl[rl * 4 + mem * 2 + qq] = tacc[h][qq] + tacc[h][R + qq];
            }
        }
    }
    __syncthreads();
    lora_mfma_addend<R, true>(acc, lane, m0, n0, wm * 128, wn * 64, bias,
                              reinterpret_cast<const float*>(smem + p8f::TOFF), theta_pop, ld_theta, offB, scale,
                              rows_per_member, M, N);
    store_tile_t(acc, smem, wave, lane, m0, n0, wm * 128, wn * 64, M, N, Y, ldy);
}

// The fused-projection kernel is opt-in (tile 12): measured at the Sana shapes it is 1-10 % SLOWER
// than k_lora_project + k_lora_gemm8 (1.205 vs 1.189 ms at 131072x2240x2240, 5.82 vs 5.25 ms at
// N = 11200) — the extra AK DMA and T-MFMA per K-tile cost more than the 10 % X re-read they save.
static bool fused_ok(int tsel, int32_t r, int64_t K, int64_t rows_per_member) {
    return tsel == 12 && (r == 1 || r == 2) && rows_per_member >= 256 && K % 64 == 0;
}

static int launch_gemm8f(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                         const float* theta_pop, int64_t ld_theta, int64_t offA, int64_t offB, int32_t r, float scale,
                         int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy, void* ws,
                         hipStream_t st) {
    const int64_t n_members = (M + rows_per_member - 1) / rows_per_member;
    EGG_CHECK_ARG(M * ldx * 2 < (1ll << 31) && N * ldw * 2 < (1ll << 31) && n_members * 16 * K * 2 < (1ll << 31),
                  "lora_linear_pop: operand > 2 GiB");
    unsigned short* AK = reinterpret_cast<unsigned short*>(ws);
    const int64_t work = n_members * 16 * (K / 8);
    hipLaunchKernelGGL(k_lora_ak, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, theta_pop, ld_theta, offA,
                       (int)r, K, (int)n_members, AK);
    EGG_CHECK_LAUNCH("lora_ak");
    const int64_t tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256;
    const dim3 grid((unsigned)(tiles_m * tiles_n));
    if (r == 1)
        hipLaunchKernelGGL((k_lora_gemm8f<1>), grid, dim3(512), 0, st, (const unsigned short*)X, ldx,
                           (const unsigned short*)W, ldw, (const unsigned short*)bias, AK, theta_pop, ld_theta, offB,
                           scale, (int)rows_per_member, (int)n_members, (int)M, (int)N, K, (int)tiles_n,
                           (unsigned short*)Y, ldy);
    else
        hipLaunchKernelGGL((k_lora_gemm8f<2>), grid, dim3(512), 0, st, (const unsigned short*)X, ldx,
                           (const unsigned short*)W, ldw, (const unsigned short*)bias, AK, theta_pop, ld_theta, offB,
                           scale, (int)rows_per_member, (int)n_members, (int)M, (int)N, K, (int)tiles_n,
                           (unsigned short*)Y, ldy);
    EGG_CHECK_LAUNCH("lora_gemm8f");
    return EGGROLL_OK;
}

template <bool MF>
static int launch_gemm8(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                        const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                        int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy, hipStream_t st) {
    const int64_t tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256;
    EGG_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "lora_gemm: grid too large");
    const dim3 grid((unsigned)(tiles_m * tiles_n));
#define EGG_GEMM8(RV)                                                                                            \
    hipLaunchKernelGGL((k_lora_gemm8<RV, MF && (RV <= 2)>), grid, dim3(512), 0, st, (const unsigned short*)X, ldx,                \
                       (const unsigned short*)W, ldw, (const unsigned short*)bias, T, theta_pop, ld_theta,      \
                       offB, scale, (int)rows_per_member, (int)M, (int)N, K, (int)tiles_n, (unsigned short*)Y, ldy)
    switch (r) {
        case 0: EGG_GEMM8(0); break;
        case 1: EGG_GEMM8(1); break;
        case 2: EGG_GEMM8(2); break;
        case 3: EGG_GEMM8(3); break;
        case 4: EGG_GEMM8(4); break;
        case 8: EGG_GEMM8(8); break;
        case 16: EGG_GEMM8(16); break;
        default: set_error("lora_gemm: r=%d unsupported (0,1,2,3,4,8,16)", r); return EGGROLL_ERR_UNSUPPORTED;
    }
#undef EGG_GEMM8
    EGG_CHECK_LAUNCH("lora_gemm8");
    return EGGROLL_OK;
}

// The MFMA-addend 8-phase kernel with an epilogue op (r <= 2; any grid size).
static int launch_gemm8_epi(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                            const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                            int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy, int32_t epi,
                            const EpiArgs& ea, hipStream_t st) {
    const int64_t tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256;
    EGG_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "lora_gemm: grid too large");
    const dim3 grid((unsigned)(tiles_m * tiles_n));
#define EGG_GEMM8E(RV, EV)                                                                                         \
    hipLaunchKernelGGL((k_lora_gemm8<RV, true, EV>), grid, dim3(512), 0, st, (const unsigned short*)X, ldx,         \
                       (const unsigned short*)W, ldw, (const unsigned short*)bias, T, theta_pop, ld_theta, offB,  \
                       scale, (int)rows_per_member, (int)M, (int)N, K, (int)tiles_n, (unsigned short*)Y, ldy, ea)
#define EGG_GEMM8E_R(EV)                       \
    switch (r) {                               \
        case 0: EGG_GEMM8E(0, EV); break;      \
        case 1: EGG_GEMM8E(1, EV); break;      \
        default: EGG_GEMM8E(2, EV); break;     \
    }
    switch (epi) {
        case EPI_SILU: EGG_GEMM8E_R(EPI_SILU); break;
        case EPI_GELU: EGG_GEMM8E_R(EPI_GELU); break;
        case EPI_GELU_ERF: EGG_GEMM8E_R(EPI_GELU_ERF); break;
        case EPI_MUL: EGG_GEMM8E_R(EPI_MUL); break;
        case EPI_RES: EGG_GEMM8E_R(EPI_RES); break;
        case EPI_GATED: EGG_GEMM8E_R(EPI_GATED); break;
        case EPI_RES32: EGG_GEMM8E_R(EPI_RES32); break;
        default: EGG_GEMM8E_R(EPI_GATED32); break;
    }
#undef EGG_GEMM8E_R
#undef EGG_GEMM8E
    EGG_CHECK_LAUNCH("lora_gemm8_epi");
    return EGGROLL_OK;
}

// The 256 x 320 kernel (kernel 10): MFMA-addend path only (r <= 2 with rows_per_member >= 256, or r = 0).
static bool gemm8n_ok(int32_t r, int64_t rows_per_member) { return r == 0 || (r <= 2 && rows_per_member >= 256); }

// Automatic choice between the 8-phase tiles (256 x 256 = 8, 256 x 320 = 10): rounds of one tile per
// CU (256 CUs) times the tile's cost, a 256 x 320 tile measured at 1.22x a 256 x 256 one (25 % more
// MFMAs, ~2.5 % fewer cycles per output element and a slightly higher clock; tools/gemm10_probe.py,
// DESIGN §5).  131072 x 2240: 18 vs 14 x 1.22 rounds -> 10 (+3-6 % measured); 9600 x 2240: 2 vs 2 x 1.22
// -> 8.  The residual / gated-residual epilogues stay on 8 (their loads slow kernel 10's store phase).
static int gemm8_auto(int64_t M, int64_t N, int32_t r, int64_t rows_per_member, int32_t epi) {
    // the bf16 residual epilogues stay on 8 (their per-chunk loads slow kernel 10's store phase); the fp32
    // ones load in batches and run equal (to_out) or 3 % faster (FFN point conv, K 5632) on 10
    // (profiles/r05h_epi32_kernel8_vs_10_ab.log)
    if (!gemm8n_ok(r, rows_per_member) || epi == EPI_RES || epi == EPI_GATED || epi == EPI_MUL) return 8;
    const int64_t tm = (M + 255) / 256;
    const int64_t rounds8 = (tm * ((N + 255) / 256) + 255) / 256, rounds10 = (tm * ((N + 319) / 320) + 255) / 256;
    return 122 * rounds10 < 100 * rounds8 ? 10 : 8;
}

static int launch_gemm8n(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                         const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                         int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy, int32_t epi,
                         const EpiArgs& ea, hipStream_t st) {
    const int64_t tiles_m = (M + 255) / 256, tiles_n = (N + p8n::BN - 1) / p8n::BN;
    EGG_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "lora_gemm: grid too large");
    EGG_CHECK_ARG(gemm8n_ok(r, rows_per_member), "lora_gemm: kernel 10 needs r <= 2 and rows_per_member >= 256");
    const dim3 grid((unsigned)(tiles_m * tiles_n));
#define EGG_GEMM8N(RV, EV)                                                                                        \
    hipLaunchKernelGGL((k_lora_gemm8n<RV, EV>), grid, dim3(512), 0, st, (const unsigned short*)X, ldx,             \
                       (const unsigned short*)W, ldw, (const unsigned short*)bias, T, theta_pop, ld_theta, offB,  \
                       scale, (int)rows_per_member, (int)M, (int)N, K, (int)tiles_n, (unsigned short*)Y, ldy, ea)
#define EGG_GEMM8N_R(EV)                       \
    switch (r) {                               \
        case 0: EGG_GEMM8N(0, EV); break;      \
        case 1: EGG_GEMM8N(1, EV); break;      \
        default: EGG_GEMM8N(2, EV); break;     \
    }
    switch (epi) {
        case EPI_NONE: EGG_GEMM8N_R(EPI_NONE); break;
        case EPI_SILU: EGG_GEMM8N_R(EPI_SILU); break;
        case EPI_GELU: EGG_GEMM8N_R(EPI_GELU); break;
        case EPI_GELU_ERF: EGG_GEMM8N_R(EPI_GELU_ERF); break;
        case EPI_MUL: EGG_GEMM8N_R(EPI_MUL); break;
        case EPI_RES: EGG_GEMM8N_R(EPI_RES); break;
        case EPI_GATED: EGG_GEMM8N_R(EPI_GATED); break;
        case EPI_RES32: EGG_GEMM8N_R(EPI_RES32); break;
        default: EGG_GEMM8N_R(EPI_GATED32); break;
    }
#undef EGG_GEMM8N_R
#undef EGG_GEMM8N
    EGG_CHECK_LAUNCH("lora_gemm8n");
    return EGGROLL_OK;
}

template <class TL>
static int launch_gemm(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                       const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                       int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy, hipStream_t st) {
    const int64_t tiles_m = (M + TL::BM - 1) / TL::BM, tiles_n = (N + TL::BN - 1) / TL::BN;
    EGG_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "lora_gemm: grid too large");
    const dim3 grid((unsigned)(tiles_m * tiles_n));
#define EGG_GEMM(RV)                                                                                              \
    hipLaunchKernelGGL((k_lora_gemm<RV, TL>), grid, dim3(TL::THREADS), 0, st, (const unsigned short*)X, ldx,      \
                       (const unsigned short*)W, ldw, (const unsigned short*)bias, T, theta_pop, ld_theta,      \
                       offB, scale, (int)rows_per_member, (int)M, (int)N, K, (int)tiles_n, (unsigned short*)Y, ldy)
    switch (r) {
        case 0: EGG_GEMM(0); break;
        case 1: EGG_GEMM(1); break;
        case 2: EGG_GEMM(2); break;
        case 3: EGG_GEMM(3); break;
        case 4: EGG_GEMM(4); break;
        case 8: EGG_GEMM(8); break;
        case 16: EGG_GEMM(16); break;
        default: set_error("lora_gemm: r=%d unsupported (0,1,2,3,4,8,16)", r); return EGGROLL_ERR_UNSUPPORTED;
    }
#undef EGG_GEMM
    EGG_CHECK_LAUNCH("lora_gemm");
    return EGGROLL_OK;
}

// ------------------------------------------------------------------------------------
// Implicit-GEMM 3x3 convolution (stride 1, zero pad 1), NHWC bf16, on the 8-phase template.
// The DC-AE decoder's ResBlock convs (models/SanaSprint.py:157-160 -> diffusers AutoencoderDC):
//   GEMM rows    = "super-pixels" of PX horizontally adjacent output pixels (M' = B*H*W/PX)
//   GEMM columns = PX * Cout (the PX pixels' output channels, contiguous in NHWC)
//   GEMM K       = 3 * (PX+2) taps * Cin: tap (ty, tx) reads input pixel (y+ty-1, x0+tx-1) of the
//                  super-pixel whose first pixel is x0; K-tile kt = (tap, 64-channel slice)
// Two tile shapes, the same 8-phase schedule and wave tile (128 x 64, 8 waves, BK = 64):
//   WMW = 2: 256 x 256 (2 x 4 waves) for PX * Cout >= 256.  PX = 2 serves Cout = 128 with a full
//            256-column tile, but the packed weight is zero where a tap does not touch a pixel
//            (25 % of the MACs).
//   WMW = 4: 512 x 128 (4 x 2 waves) for Cout = 128 at PX = 1 — no zero MACs.  The A half-tile is
//            32 KiB (4 DMAs per wave), the B half-tile 8 KiB (1 DMA); the ring is the whole 160 KiB.
// A operand: each lane's DMA rows keep ONE byte offset (its pixel, relative to a per-block buffer
// base) and a tap-validity bit mask; the tap's shift and channel slice go in the wave-uniform
// soffset, and a tap outside the image turns the lane's offset out of range (0x80000000 >
// num_records), which the buffer unit returns as zeros: the zero padding costs one v_cndmask
// per DMA.  B operand: the packed weight [PX*Cout][3][PX+2][Cin] streams like the GEMM's W.
// Epilogue: bias through the MFMA addend (one k-step), optional SiLU in fp32, one bf16 rounding.
// ------------------------------------------------------------------------------------
template <int WMW>
struct G8 {
    static constexpr int WNW = 8 / WMW, BM = WMW * 128, BN = WNW * 64;
    static constexpr int HA = BM * 64, HB = BN * 64;  // half-tile region bytes ((BM or BN)/2 rows x 128 B)
    static constexpr int RA0 = 0, RA1 = HA, RB0 = 2 * HA, RB1 = 2 * HA + HB;
    static constexpr int BUF = 2 * HA + 2 * HB, LDS = 2 * BUF;
    static constexpr int NA = HA / 8192, NB = HB / 8192;  // DMAs per wave per half-tile (8 waves x 1 KiB)
    // glds left in flight when a K-tile retires (the next K-tile's A0, B1, A1 halves; T3/T4 formula)
    static constexpr int VMC = 2 * NA + NB;
    static constexpr int VMC0 = 3 * NA + 2 * NB;  // early first K-tile waits (see wait_vm)
    static constexpr int CSTAGE = 8 * 128 * 64 * 2;  // epilogue C staging: one 128x64 bf16 tile per wave
    static_assert(LDS <= 160 * 1024, "ring exceeds the 160 KiB LDS");
};

template <int ND>
struct ConvStage {
    uint32_t off[ND];   // lane byte offset of its pixel's channel chunk, tap (0,0) = pixel - (W+1)
    uint32_t mask[ND];  // bit t set: tap t reads inside the image
};
template <int ND>
struct WStage {
    uint32_t off[ND];
};

template <int PX, int KS, int ND>
__device__ __forceinline__ ConvStage<ND> make_conv_stage(int m0, int Mp, int H, int W, int Cin, int h, int wave,
                                                         int lane) {
    constexpr int TW = PX + KS - 1;
    const int Ho = H + 3 - KS, Ws = (W + 3 - KS) / PX;  // output grid (pad 1)
    // input pixel of a super-pixel row's first output pixel (monotone in the row index)
    auto pin = [&](int gr) -> int64_t {
        const int xs = gr % Ws, yrow = gr / Ws;
        return ((int64_t)(yrow / Ho) * H + yrow % Ho) * W + xs * PX;
    };
    const int64_t pin0 = pin(m0);
    ConvStage<ND> s;
#pragma unroll
    for (int i = 0; i < ND; ++i) {
        const int j = (i * 8 + wave) * 8 + (lane >> 3);  // region row (as make_stage<true>)
        const int chunk = (lane & 7) ^ (j & 7);
        const int tr = (j >> 6) * 128 + h * 64 + (j & 63);  // wave row wm = j / 64
        const int gr = m0 + tr;
        uint32_t mk = 0;
        int64_t pg = pin0;
        if (gr < Mp) {
            const int xs = gr % Ws, yrow = gr / Ws, y = yrow % Ho;
            pg = pin(gr);
#pragma unroll
            for (int ty = 0; ty < KS; ++ty)
#pragma unroll
                for (int tx = 0; tx < TW; ++tx) {
                    const int yy = y + ty - 1, xx = xs * PX + tx - 1;
                    if (yy >= 0 && yy < H && xx >= 0 && xx < W) mk |= 1u << (ty * TW + tx);
                }
        }
        s.mask[i] = mk;
        s.off[i] = ((uint32_t)(pg - pin0) * (uint32_t)Cin + chunk * 8) * 2;  // from the block base pixel + (W+1)
    }
    return s;
}

// B (weight) half-tile staging with ND DMAs per wave: region row j -> tile column
// (j / 32) * 64 + h * 32 + j % 32 (wave column wn = j / 32), as make_stage<false>.
template <int ND>
__device__ __forceinline__ WStage<ND> make_stage_b(int base_row, int row_max, int64_t ld, int h, int wave, int lane) {
    WStage<ND> s;
#pragma unroll
    for (int i = 0; i < ND; ++i) {
        const int j = (i * 8 + wave) * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ (j & 7);
        int gr = base_row + (j >> 5) * 64 + h * 32 + (j & 31);
        gr = gr < row_max ? gr : row_max;
        s.off[i] = ((uint32_t)gr * (uint32_t)ld + chunk * 8) * 2;
    }
    return s;
}

template <int ND>
__device__ __forceinline__ void issue_conv_half(__amdgpu_buffer_rsrc_t rs, const ConvStage<ND>& s, int tap, int kbytes,
                                                char* region, int wave) {
#pragma unroll
    for (int i = 0; i < ND; ++i) {
        const uint32_t v = ((s.mask[i] >> tap) & 1u) ? s.off[i] : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(region + (i * 8 + wave) * 1024), 16, v, kbytes, 0, 0);
    }
}
template <int ND>
__device__ __forceinline__ void issue_half_n(__amdgpu_buffer_rsrc_t rs, const WStage<ND>& s, int kbytes, char* region,
                                             int wave) {
#pragma unroll
    for (int i = 0; i < ND; ++i) {
        const uint32_t v = s.off[i];  // (a local: hipcc rejects the member access inside the builtin here)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(region + (i * 8 + wave) * 1024), 16, v, kbytes, 0, 0);
    }
}

// p8_phase with the DMA supplied by the caller (A: masked conv staging, B: weight staging)
template <class G, int QA, int QB, int RD, bool VM, bool EW, class Issue>
__device__ __forceinline__ void p8c_phase(f32x4 (&acc)[8][4], bf16x8 (&a)[4][2], bf16x8 (&b)[2][2], const char* buf,
                                          const int (&oA)[2], const int (&oB)[2], Issue&& issue) {
    if (RD != 2) p8_read_b(b, buf + (QB ? G::RB1 : G::RB0), oB);
    if (RD != 1) p8_read_a(a, buf + (QA ? G::RA1 : G::RA0), oA);
    issue();
    if constexpr (EW) wait_vm<G::VMC0>();  // early first K-tile (no-op in steady state)
    if (VM) wait_vm<G::VMC>();
    P8_LGKM0_;
    P8_BAR();
    p8_mma<QA, QB, true>(acc, a, b);
    P8_BAR();
}

// store_tile_t with an optional fp32 SiLU before the bf16 rounding
template <int ACT>
__device__ __forceinline__ void store_tile_t_act(f32x4 (&acc)[8][4], char* smem, int wave, int lane, int m0, int n0,
                                                 int rbase, int cbase, int M, int N, unsigned short* __restrict__ Y,
                                                 int64_t ldy) {
    if constexpr (ACT == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
                    const f32x2 t = silu2((f32x2){acc[i][j][e], acc[i][j][e + 1]});
                    acc[i][j][e] = t.x;
                    acc[i][j][e + 1] = t.y;
                }
    }
    store_tile_t(acc, smem, wave, lane, m0, n0, rbase, cbase, M, N, Y, ldy);
}

// ResBlock tail fused into conv2's epilogue (NORM): RMSNorm over each pixel's COUT = BN / PX
// channels (a tile holds whole pixels: N = BN), * w[c] + b[c] + res[row, col], on the fp32
// accumulators.  Row sums of squares: 16 values per lane, xor-16/32 shuffles across the wave's 4
// column lanes, then a [BM rows][WNW waves] LDS table for the WPP = COUT / 64 waves that share a
// pixel, summed in a fixed order.
// RowOf(tile row) -> the row of res (and of the output) that tile row holds.
template <int PX, int WMW, int WNW = 8 / WMW, class RowOf>
__device__ __forceinline__ void conv_rmsnorm_epilogue(f32x4 (&acc)[8][4], float* red, int wm, int wn, int lane,
                                                      RowOf row_of, float eps, const unsigned short* __restrict__ nw,
                                                      const unsigned short* __restrict__ nb,
                                                      const unsigned short* __restrict__ res) {
    constexpr int BN = WNW * 64, COUT = BN / PX, WPP = COUT / 64;
    static_assert(WPP == 2 || WPP == 4, "a pixel spans 2 or 4 waves");
    const int rl = lane & 15, cg = lane >> 4;
    // norm weight / bias: 4 consecutive channels per load, issued ahead of the row-sum barrier
    u16x4 wq[4], bq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c4 = (wn * 64 + 16 * j + 4 * cg) % COUT;
        wq[j] = *reinterpret_cast<const u16x4*>(nw + c4);
        bq[j] = nb ? *reinterpret_cast<const u16x4*>(nb + c4) : u16x4{0, 0, 0, 0};
    }
    float ss[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float sq = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) sq += acc[i][j][e] * acc[i][j][e];
        // xor-16 then xor-32 butterfly on v_permlane16_swap / v_permlane32_swap (VALU; the ds_bpermute
        // shuffles were LDS round trips): each returns the lane's own value and its partner's, whose sum
        // is the butterfly step — the same additions, the same bits
        {
            const auto r16 = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, sq),
                                                              __builtin_bit_cast(unsigned, sq), false, false);
            sq = __builtin_bit_cast(float, (unsigned)r16[0]) + __builtin_bit_cast(float, (unsigned)r16[1]);
            const auto r32 = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, sq),
                                                              __builtin_bit_cast(unsigned, sq), false, false);
            sq = __builtin_bit_cast(float, (unsigned)r32[0]) + __builtin_bit_cast(float, (unsigned)r32[1]);
        }
        ss[i] = sq;
    }
    if (cg == 0)
#pragma unroll
        for (int i = 0; i < 8; ++i) red[(wm * 128 + 16 * i + rl) * WNW + wn] = ss[i];
    __syncthreads();
    float wv[4][4], bv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            wv[j][e] = bf16_to_f32(wq[j][e]);
            bv[j][e] = bf16_to_f32(bq[j][e]);
        }
    const int w0 = (wn / WPP) * WPP;  // first wave of this pixel
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rr = wm * 128 + 16 * i + rl;
        const float* rp = red + rr * WNW + w0;
        const float tot = WPP == 4 ? (rp[0] + rp[1]) + (rp[2] + rp[3]) : rp[0] + rp[1];
        const float rs = rsqrtf(tot / COUT + eps);
        const int64_t row = row_of(rr);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (res) {
                const u16x4 r4 = *reinterpret_cast<const u16x4*>(res + row * BN + wn * 64 + 16 * j + 4 * cg);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[i][j][e] = acc[i][j][e] * rs * wv[j][e] + bv[j][e] + bf16_to_f32(r4[e]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[i][j][e] = acc[i][j][e] * rs * wv[j][e] + bv[j][e];
            }
        }
    }
}

// DC-AE up-block epilogue (eggroll_conv2x2_subpixel_nhwc): the phase conv's C tile goes straight to the
// up-sampled output instead of a y4 [B, H+1, W+1, 4*Cout] intermediate read back by
// k_subpixel_shortcut4.  Row = phase-conv position (b, h', w') of the (H+1) x (W+1) grid, column =
// (phase k = 2i + j, output channel): out[b, 2h + i, 2w + j, c] = bf16(y) + bias[c] + src[b, h, w,
// (4c + k) / REP] with (h, w) = (h' - i, w' - j) (positions with h or w outside the input are dropped),
// y rounded to bf16 first and the two adds in that order — the arithmetic of k_subpixel_shortcut4, so the
// output is bitwise the two-kernel path's.  SP 1: bf16 src and out; SP 2: fp32 src (the DC-AE fp32
// residual stream) and fp32 out, plus its bf16 shadow when given.
struct SubpixArgs {
    const unsigned short* bias;  // [Cout] or null
    const void* src;             // shortcut source [B, H, W, Cin]
    void* out;                   // [B, 2H, 2W, Cout]
    unsigned short* shadow;      // SP 2: optional bf16 copy of out
    int H, W, Cin, Cout;
};

#ifndef EGG_SPX_REGS  // VGPRs of shortcut words in flight per batch in the sub-pixel epilogue (A/B knob)
#define EGG_SPX_REGS 64
#endif
// KP: the wave's phase (wave-uniform, dispatched by the caller) — a compile-time shortcut channel index
template <int SP, int REP, int KP>
__device__ __forceinline__ void store_tile_subpix(f32x4 (&acc)[8][4], char* smem, int wave, int lane, int rbase,
                                                  int col0, int Mp, const SubpixArgs& sp) {
    constexpr int ROWB = 128, SLOTS = 8;
    constexpr int XW = 32 / REP;                     // shortcut channels spanned by 8 outputs
    constexpr int WD = SP == 2 ? XW : XW / 2;        // their dwords (raw, converted at use)
    // rows whose shortcut loads are in flight together (<= EGG_SPX_REGS VGPRs of raw shortcut words)
    constexpr int RBAT_ = EGG_SPX_REGS / WD > 16 ? 16 : (EGG_SPX_REGS / WD > 0 ? EGG_SPX_REGS / WD : 1);
    constexpr int RBAT = 16 % RBAT_ == 0 ? RBAT_ : 8;
    char* ctile = smem + wave * (128 * ROWB);
    {
        const int r_l = lane & 15, c_l = (lane >> 4) * 4;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int rr = i * 16 + r_l;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int cc = j * 16 + c_l;
                const int slot = (cc >> 3) ^ (rr & (SLOTS - 1));
                u16x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = f32_to_bf16(acc[i][j][e]);
                *reinterpret_cast<u16x4*>(ctile + rr * ROWB + slot * 16 + (cc & 7) * 2) = o;
            }
        }
    }
    // the wave's 64 columns lie in one phase (Cout % 64 == 0, host-checked)
    constexpr int k = KP, pi = KP >> 1, pj = KP & 1;
    const int c0 = col0 - k * sp.Cout + (lane & 7) * 8;
    float bv[8];
    if (sp.bias) {
        const u16x8 q = *reinterpret_cast<const u16x8*>(sp.bias + c0);
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = bf16_to_f32(q[e]);
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = 0.f;
    }
    const int H = sp.H, W = sp.W, Ho = H + 1, Wo = W + 1;
    int p = rbase + (lane >> 3);
    int bb = p / (Ho * Wo), hp = (p - bb * Ho * Wo) / Wo, wp = p - bb * Ho * Wo - hp * Wo;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (wave-private tile)
#pragma unroll
    for (int it0 = 0; it0 < 16; it0 += RBAT) {
        uint32_t raw[RBAT][WD];
        int32_t opix[RBAT];   // B * 4 * H * W * Cout < 2^31 (host check): pixel and element offsets fit 32 bits
        bool ok[RBAT];
#pragma unroll
        for (int u = 0; u < RBAT; ++u) {
            const int h = hp - pi, w = wp - pj;
            ok[u] = p < Mp && h >= 0 && h < H && w >= 0 && w < W;
            const int64_t lp = ok[u] ? ((int64_t)bb * H + h) * W + w : 0;
            opix[u] = (bb * 2 * H + 2 * h + pi) * (2 * W) + 2 * w + pj;
            // window of channels (4c + k) / REP, c = c0 .. c0+7: XW channels from 4 c0 / REP
            const uint32_t* src = reinterpret_cast<const uint32_t*>(
                reinterpret_cast<const char*>(sp.src) + (lp * sp.Cin + 4 * c0 / REP) * (SP == 2 ? 4 : 2));
#pragma unroll
            for (int t = 0; t < WD / 4; ++t) {
                typedef __attribute__((ext_vector_type(4))) unsigned int sp_u32x4;
                const sp_u32x4 q = *reinterpret_cast<const sp_u32x4*>(src + 4 * t);
#pragma unroll
                for (int e = 0; e < 4; ++e) raw[u][4 * t + e] = q[e];
            }
            p += 8;
            wp += 8;
            while (wp >= Wo) {
                wp -= Wo;
                if (++hp == Ho) { hp = 0; ++bb; }
            }
        }
#pragma unroll
        for (int u = 0; u < RBAT; ++u) {
            const int it = it0 + u, rr = it * 8 + (lane >> 3), sl = lane & 7;
            const u16x8 v = *reinterpret_cast<const u16x8*>(ctile + rr * ROWB + ((sl ^ (rr & (SLOTS - 1))) << 4));
            if (!ok[u]) continue;
            float f[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int ch = (4 * q + k) / REP;  // compile-time: q unrolled, k = KP
                const float xsv = SP == 2 ? __uint_as_float(raw[u][ch])
                                          : bf16_to_f32((unsigned short)(raw[u][ch >> 1] >> (16 * (ch & 1))));
                f[q] = bf16_to_f32(v[q]) + bv[q] + xsv;
            }
            const int32_t oo = opix[u] * sp.Cout + c0;
            if constexpr (SP == 2) {
                float* o32 = reinterpret_cast<float*>(sp.out) + oo;
                *reinterpret_cast<f32x4*>(o32) = f32x4{f[0], f[1], f[2], f[3]};
                *reinterpret_cast<f32x4*>(o32 + 4) = f32x4{f[4], f[5], f[6], f[7]};
            }
            if (SP == 1 || sp.shadow) {
                u16x8 o;
#pragma unroll
                for (int q = 0; q < 8; ++q) o[q] = f32_to_bf16(f[q]);
                *reinterpret_cast<u16x8*>((SP == 2 ? sp.shadow : reinterpret_cast<unsigned short*>(sp.out)) + oo) = o;
            }
        }
    }
}

template <int WMW, bool NORM>
constexpr int conv_smem_bytes() {
    using G = G8<WMW>;
    constexpr int need = G::CSTAGE + (NORM ? G::BM * G::WNW * 4 : 0);  // RMSNorm table after the C staging
    return G::LDS > need ? G::LDS : need;
}

template <int PX, int ACT, bool NORM = false, int KS = 3, int WMW = 2, int SP = 0, int REP = 2>
__global__ __launch_bounds__(512, 1) void k_conv3x3_gemm8(const unsigned short* __restrict__ X,
                                                          const unsigned short* __restrict__ Wt,
                                                          const unsigned short* __restrict__ bias, int H, int W,
                                                          int Cin, int lcpt, int Mp, int N, int tiles_n,
                                                          unsigned short* __restrict__ Y, float eps = 0.0f,
                                                          const unsigned short* __restrict__ nw = nullptr,
                                                          const unsigned short* __restrict__ nb = nullptr,
                                                          const unsigned short* __restrict__ res = nullptr,
                                                          SubpixArgs spa = SubpixArgs{}) {
    static_assert(SP == 0 || (KS == 2 && PX == 1 && ACT == 0 && !NORM), "sub-pixel epilogue: the up-block phase conv");
    using G = G8<WMW>;
    constexpr int TW = PX + KS - 1;
    __shared__ __attribute__((aligned(16))) char smem[conv_smem_bytes<WMW, NORM>()];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / G::WNW, wn = wave % G::WNW;
    const int grp8 = wave >> 2;  // the two staggered wave groups (one wave of each per SIMD)
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
    const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
    const int tiles_m = (Mp + G::BM - 1) / G::BM;
    const int per_group = GROUP_M * tiles_n;
    const int grp = tile / per_group, first_m = grp * GROUP_M;
    const int gsize = (tiles_m - first_m) < GROUP_M ? (tiles_m - first_m) : GROUP_M;
    const int in_grp = tile - grp * per_group;
    const int tm = first_m + in_grp % gsize, tn = in_grp / gsize;
    const int m0 = tm * G::BM, n0 = tn * G::BN;
    const int64_t K = (int64_t)KS * TW * Cin;
    const int nk = (int)(K / BK);
    EGG_STAMP_RT(6);
    EGG_STAMP(0);

    const ConvStage<G::NA> sA0 = make_conv_stage<PX, KS, G::NA>(m0, Mp, H, W, Cin, 0, wave, lane);
    const ConvStage<G::NA> sA1 = make_conv_stage<PX, KS, G::NA>(m0, Mp, H, W, Cin, 1, wave, lane);
    const WStage<G::NB> sB0 = make_stage_b<G::NB>(n0, N - 1, K, 0, wave, lane);
    const WStage<G::NB> sB1 = make_stage_b<G::NB>(n0, N - 1, K, 1, wave, lane);
    char* const e_buf = smem;
    char* const o_buf = smem + G::BUF;
    // block base = input pixel of output row m0, minus (W+1); tap (ty, tx) adds (ty*W + tx) pixels in
    // soffset, so every address offset is >= 0
    int64_t pin0;
    {
        const int Ho = H + 3 - KS, Ws = (W + 3 - KS) / PX, xs = m0 % Ws, yrow = m0 / Ws;
        pin0 = ((int64_t)(yrow / Ho) * H + yrow % Ho) * W + xs * PX;
    }
    // (readfirstlane: the divisions above run on the VALU; an SGPR resource keeps every DMA a single
    // instruction instead of a readfirstlane waterfall)
    const uint64_t xbu = (uint64_t)(X + (pin0 - W - 1) * Cin);
    const unsigned short* xb = (const unsigned short*)(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(xbu >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xbu));
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)xb, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, 0x7fffffff, 0x00020000);

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[4][2], b[2][2];
    int oA[2], oB[2];
    p8_frag_offsets(oA, wm * 64 + (lane & 15), lane);
    p8_frag_offsets(oB, wn * 32 + (lane & 15), lane);

    const int cmask = (1 << lcpt) - 1;
    // K-tile t (clamped to the last one, as the GEMM): tap = t >> lcpt, channel slice t & cmask
    auto A = [&](const ConvStage<G::NA>& s, int t, char* dst) {
        t = t < nk ? t : nk - 1;
        const int tap = t >> lcpt, ty = tap / TW, tx = tap - ty * TW;
        const int soff = __builtin_amdgcn_readfirstlane(((ty * W + tx) * Cin + (t & cmask) * BK) * 2);
        issue_conv_half(rX, s, tap, soff, dst, wave);
    };
    auto B = [&](const WStage<G::NB>& s, int t, char* dst) {
        t = t < nk ? t : nk - 1;
        issue_half_n(rW, s, t * (BK * 2), dst, wave);
    };
    A(sA0, 0, e_buf + G::RA0);
    B(sB0, 0, e_buf + G::RB0);
    B(sB1, 0, e_buf + G::RB1);
    A(sA1, 0, e_buf + G::RA1);
    A(sA0, 1, o_buf + G::RA0);
    B(sB1, 1, o_buf + G::RB1);
    A(sA1, 1, o_buf + G::RA1);
    wait_vm<G::VMC0>();  // K-tile 0's A0 + B0 only (early first K-tile, see wait_vm)
    P8_BAR();
    EGG_STAMP(1);
    if (grp8 == 1) P8_BAR();

    int t0 = 0;
    for (; t0 + 1 < nk; t0 += 2) {
        p8c_phase<G, 0, 0, 0, false, true>(acc, a, b, e_buf, oA, oB, [&] { B(sB0, t0 + 1, o_buf + G::RB0); });
        p8c_phase<G, 0, 1, 1, false, true>(acc, a, b, e_buf, oA, oB, [&] { A(sA0, t0 + 2, e_buf + G::RA0); });
        p8c_phase<G, 1, 1, 2, false, false>(acc, a, b, e_buf, oA, oB, [&] { B(sB1, t0 + 2, e_buf + G::RB1); });
        p8c_phase<G, 1, 0, 1, true, false>(acc, a, b, e_buf, oA, oB, [&] { A(sA1, t0 + 2, e_buf + G::RA1); });
        p8c_phase<G, 0, 0, 0, false, false>(acc, a, b, o_buf, oA, oB, [&] { B(sB0, t0 + 2, e_buf + G::RB0); });
        p8c_phase<G, 0, 1, 1, false, false>(acc, a, b, o_buf, oA, oB, [&] { A(sA0, t0 + 3, o_buf + G::RA0); });
        p8c_phase<G, 1, 1, 2, false, false>(acc, a, b, o_buf, oA, oB, [&] { B(sB1, t0 + 3, o_buf + G::RB1); });
        p8c_phase<G, 1, 0, 1, true, false>(acc, a, b, o_buf, oA, oB, [&] { A(sA1, t0 + 3, o_buf + G::RA1); });
    }
    if (t0 < nk) {
        p8c_phase<G, 0, 0, 0, false, true>(acc, a, b, e_buf, oA, oB, [&] { B(sB0, t0 + 1, o_buf + G::RB0); });
        p8c_phase<G, 0, 1, 1, false, true>(acc, a, b, e_buf, oA, oB, [&] { A(sA0, t0 + 2, e_buf + G::RA0); });
        p8c_phase<G, 1, 1, 2, false, false>(acc, a, b, e_buf, oA, oB, [&] { B(sB1, t0 + 2, e_buf + G::RB1); });
        p8c_phase<G, 1, 0, 1, false, false>(acc, a, b, e_buf, oA, oB, [&] { A(sA1, t0 + 2, e_buf + G::RA1); });
    }
    if (grp8 == 0) P8_BAR();
    EGG_STAMP(2);
    P8_VM0();
    __syncthreads();
    EGG_STAMP(3);
    if (bias)
        lora_mfma_addend<0>(acc, lane, m0, n0, wm * 128, wn * 64, bias, nullptr, nullptr, 0, 0, 0.0f, 1 << 30, Mp, N);
    if constexpr (SP != 0) {
        EGG_STAMP(4);
        const int kp = __builtin_amdgcn_readfirstlane((n0 + wn * 64) / spa.Cout);
        if (kp == 0) store_tile_subpix<SP, REP, 0>(acc, smem, wave, lane, m0 + wm * 128, n0 + wn * 64, Mp, spa);
        else if (kp == 1) store_tile_subpix<SP, REP, 1>(acc, smem, wave, lane, m0 + wm * 128, n0 + wn * 64, Mp, spa);
        else if (kp == 2) store_tile_subpix<SP, REP, 2>(acc, smem, wave, lane, m0 + wm * 128, n0 + wn * 64, Mp, spa);
        else store_tile_subpix<SP, REP, 3>(acc, smem, wave, lane, m0 + wm * 128, n0 + wn * 64, Mp, spa);
    } else if constexpr (NORM) {
        conv_rmsnorm_epilogue<PX, WMW>(
            acc, reinterpret_cast<float*>(smem + G::CSTAGE), wm, wn, lane,
            [&](int rr) -> int64_t { return m0 + rr < Mp ? m0 + rr : Mp - 1; }, eps, nw, nb, res);
        EGG_STAMP(4);
        store_tile_t(acc, smem, wave, lane, m0, n0, wm * 128, wn * 64, Mp, N, Y, N);
    } else {
        EGG_STAMP(4);
        store_tile_t_act<ACT>(acc, smem, wave, lane, m0, n0, wm * 128, wn * 64, Mp, N, Y, N);
    }
    EGG_STAMP_DRAIN();
    EGG_STAMP(5);
    EGG_STAMP_RT(7);
}

// ------------------------------------------------------------------------------------
// Halo-staged 3x3 conv (stride 1, pad 1, px 1): the tile-sliced implicit GEMM above re-stages its
// A operand once per tap (9 x the input bytes through the LDS-DMA path, which is what bounds it:
// DESIGN.md §5).  Here a tile is TH x TWD output pixels (16 x 32 for the 512 x 128 tile, 16 x 16
// for 256 x 256) and its (TH+2) x (TWD+2) input halo is staged ONCE per 32-channel slice; the nine
// taps read their A fragments from it at a pixel shift.  K-step = (slice, tap), K = 32:
//   halo    [halo pixel][32 ch] bf16, 64-B rows, double-buffered by slice: slice s+1 streams in as
//           one 1-KiB piece per wave at taps 0..NPW-1 of slice s
//   weights [BN rows][32 ch] per K-step, a ring of D+1 slots, K-step k+D issued during step k
// 64-B rows read as 16x16x32 fragments (lane: row l&15, chunk l>>4) are bank-conflict-free for any
// run of 16 consecutive rows with slot = chunk ^ 2*((row >> 2) & 1), i.e. byte L -> L ^ ((L>>3)&32);
// the tap shift is added to the logical byte before the swizzle.  Per K-step each wave runs two
// phases of 16 MFMAs (A fragments 0-3, then 4-7, against the same 4 B fragments) with the p8 wave-
// group stagger; all DMA waits are counted vmcnt (compile-time per tap, see hc_wait_n).
// ------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void wait_vmn() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PAD: halo rows HS = HW2 rounded up to 8 pixels (the pad columns are zero-filled, never read).  The
// fragment swizzle keys on bit 2 of the halo pixel index; with HS % 8 == 0 a tap's row shift dy (HS
// pixels) leaves that bit alone, so a fragment needs one swizzled address per column shift dx and the
// row shift is the ds_read immediate (3 addresses per fragment instead of 9: 24 VGPRs instead of 72).
template <int WMW, int WNW = 8 / WMW, bool PAD = true>
struct HC {
    static constexpr int WM_ = WMW, WN_ = WNW;
    static constexpr int NW = WMW * WNW, BM = WMW * 128, BN = WNW * 64;  // waves, tile
    static constexpr int TH = 16, TWD = BM / TH;                 // output pixels of a tile
    static constexpr int HW2 = TWD + 2;                          // halo pixels per row
    static constexpr int HS = PAD ? (HW2 + 7) / 8 * 8 : HW2;     // halo row stride in LDS (pixels)
    static constexpr int HP = (TH + 2) * HS;                     // halo pixel slots
    static constexpr int NPW = (HP + 16 * NW - 1) / (16 * NW);  // halo pieces (16 px x 64 B) per wave
    static constexpr int HALO = NPW * NW * 1024;
    static constexpr int NBW = BN / (16 * NW);                    // weight pieces per wave per K-step
    static constexpr int BSLOT = BN * 64;
    static constexpr int D = 3, NBUF = D + 1;                     // weight prefetch distance / ring slots
    static constexpr int RB = 2 * HALO, LDS = 2 * HALO + NBUF * BSLOT;
    // the halo of slice s+1 (taps 0..NPW-1 of slice s) is older than the weights of K-step (s+1, 0)
    // (issued at tap 9-D of slice s), so the weight wait also retires the halo
    static_assert(NPW <= 9 - D, "halo pieces must precede the next slice's first weight DMA");
    static constexpr int CSTAGE = NW * 128 * 64 * 2;               // epilogue C staging (one 128x64 tile per wave)
    static_assert(NBW >= 1 && BN % (16 * NW) == 0, "weight pieces");
};

__device__ __forceinline__ uint32_t hc_swz(uint32_t L) { return L ^ ((L >> 3) & 32u); }

// DMAs younger than K-step k+1's weights when step k (tap T) retires them in its second phase
template <class G, int T, bool NEXT, bool LAST>
constexpr int hc_wait_n() {
    int n = 0;
    for (int i = 2; i <= G::D; ++i)
        if (!LAST || T + i < 9) n += G::NBW;
    if (NEXT)
        for (int t = T + 1 - G::D; t <= T; ++t)
            if (t >= 0 && t < G::NPW) n += 1;
    return n;
}

template <int I, int N, class F>
__device__ __forceinline__ void hc_static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        hc_static_for<I + 1, N>(f);
    }
}

template <class G, bool NORM>
constexpr int halo_smem_bytes() {
    constexpr int need = G::CSTAGE + (NORM ? G::BM * G::WN_ * 4 : 0);
    return G::LDS > need ? G::LDS : need;
}

// store_tile_t (fast path only: every conv tile is full) with tile row -> output row through row_of
// the residual rows of a wave's 128 x 64 tile as coalesced 16-B loads (store_tile_rows' order)
template <int I0 = 0, int I1 = 16, class RowOf, int NR>
__device__ __forceinline__ void load_res_rows(u16x8 (&rv)[NR], const unsigned short* __restrict__ res, int lane,
                                              int rbase, int col0, int64_t ldy, RowOf row_of) {
#pragma unroll
    for (int it = I0; it < I1; ++it)
        rv[it] = *reinterpret_cast<const u16x8*>(res + row_of(rbase + it * 8 + (lane >> 3)) * ldy + col0 + (lane & 7) * 8);
}

template <int ACT, class RowOf, bool RES = false, bool PRE = false>
__device__ __forceinline__ void store_tile_rows(f32x4 (&acc)[8][4], char* smem, int wave, int lane, int rbase,
                                                int col0, unsigned short* __restrict__ Y, int64_t ldy, RowOf row_of,
                                                const unsigned short* __restrict__ res = nullptr,
                                                const u16x8* pre = nullptr) {
    constexpr int ROWB = 128, SLOTS = 8;
    char* ctile = smem + wave * (128 * ROWB);
    const int r_l = lane & 15, c_l = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rr = i * 16 + r_l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int cc = j * 16 + c_l;
            const int slot = (cc >> 3) ^ (rr & (SLOTS - 1));
            u16x4 o;
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
                f32x2 v = {acc[i][j][e], acc[i][j][e + 1]};
                if constexpr (ACT == 1) v = silu2(v);
                o[e] = f32_to_bf16(v.x);
                o[e + 1] = f32_to_bf16(v.y);
            }
            *reinterpret_cast<u16x4*>(ctile + rr * ROWB + slot * 16 + (cc & 7) * 2) = o;
        }
    }
    u16x8 rv[RES ? 16 : 1];
    if constexpr (RES) {  // residual rows as coalesced 16-B loads, in flight while the tile goes through LDS
        if constexpr (PRE) {  // the first 8 rows were loaded by the caller
#pragma unroll
            for (int it = 0; it < 8; ++it) rv[it] = pre[it];
            load_res_rows<8, 16>(rv, res, lane, rbase, col0, ldy, row_of);
        } else {
            load_res_rows(rv, res, lane, rbase, col0, ldy, row_of);
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (wave-private tile)
    u16x8 v[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int rr = it * 8 + (lane >> 3), sl = lane & 7;
        v[it] = *reinterpret_cast<const u16x8*>(ctile + rr * ROWB + ((sl ^ (rr & (SLOTS - 1))) << 4));
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int rr = it * 8 + (lane >> 3);
        if constexpr (RES) {
#pragma unroll
            for (int u = 0; u < 8; ++u) v[it][u] = f32_to_bf16(bf16_to_f32(v[it][u]) + bf16_to_f32(rv[it][u]));
        }
        *reinterpret_cast<u16x8*>(Y + row_of(rbase + rr) * ldy + col0 + (lane & 7) * 8) = v[it];
    }
}

// WMW x WNW waves: (4, 2) 512 x 128 and (2, 4) 256 x 256 tiles run one 8-wave workgroup per CU
// with the two wave groups staggered by a barrier (as the p8 kernels); (2, 2) 256 x 128 runs two
// 4-wave workgroups per CU (80 KiB LDS each), which overlap each other's prologue and epilogue.
template <int ACT, bool NORM, int WMW, int WNW, bool PAD = true>
__global__ __launch_bounds__(64 * WMW * WNW, 8 / (WMW * WNW)) void k_conv3x3_halo(const unsigned short* __restrict__ X,
                                                         const unsigned short* __restrict__ Wt,
                                                         const unsigned short* __restrict__ bias, int H, int W,
                                                         int Cin, int N, int tiles_n, unsigned short* __restrict__ Y,
                                                         float eps = 0.0f, const unsigned short* __restrict__ nw = nullptr,
                                                         const unsigned short* __restrict__ nb = nullptr,
                                                         const unsigned short* __restrict__ res = nullptr) {
    using G = HC<WMW, WNW, PAD>;
    static_assert(halo_smem_bytes<G, NORM>() * (8 / G::NW) <= 160 * 1024, "LDS per CU");
    __shared__ __attribute__((aligned(16))) char smem[halo_smem_bytes<G, NORM>()];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WNW, wn = wave % WNW;
    const int grp8 = wave >> 2;
    // XCD-contiguous tile ranges (neighbouring tiles share halo rows and all share the weights);
    // the N-tiles of one pixel tile are adjacent
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
    const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int n0 = tn * G::BN;
    const int tpr = W / G::TWD, tpi = (H / G::TH) * tpr;
    const int img = tm / tpi, trm = tm - img * tpi;
    const int y0 = (trm / tpr) * G::TH, x0 = (trm - (trm / tpr) * tpr) * G::TWD;
    const int K = 9 * Cin, S = Cin / 32;
    EGG_STAMP_RT(6);
    EGG_STAMP(0);

    // halo DMA: piece i*8 + wave holds halo pixels 16p .. 16p+15; out-of-image pixels (and the pad
    // past HP) read as zeros through an out-of-range offset
    uint32_t hoff[G::NPW];
#pragma unroll
    for (int i = 0; i < G::NPW; ++i) {
        const int hp = (i * G::NW + wave) * 16 + (lane >> 2);
        const int c = (lane & 3) ^ (((hp >> 2) & 1) << 1);
        const int hy = hp / G::HS, hx = hp - hy * G::HS;
        const int y = y0 - 1 + hy, x = x0 - 1 + hx;
        const bool ok = hp < G::HP && hx < G::HW2 && y >= 0 && y < H && x >= 0 && x < W;
        hoff[i] = ok ? (uint32_t)(((hy * W + hx) * Cin + c * 8) * 2) : 0x80000000u;
    }
    uint32_t boff[G::NBW];
#pragma unroll
    for (int i = 0; i < G::NBW; ++i) {
        const int n = (i * G::NW + wave) * 16 + (lane >> 2);
        const int c = (lane & 3) ^ (((n >> 2) & 1) << 1);
        boff[i] = (uint32_t)(((n0 + n) * K + c * 8) * 2);
    }
    // fragment reads: A row f of the wave at tap (0,0) as a logical halo byte (!PAD: swizzled per tap);
    // PAD: the swizzled byte of A row f at column shift dx (row shift dy = immediate dy * HS * 64)
    uint32_t la[8];
    uint32_t ad[PAD ? 8 : 1][PAD ? 3 : 1];
#pragma unroll
    for (int f = 0; f < 8; ++f) {
        const int m = wm * 128 + 16 * f + (lane & 15);
        const int ty = m / G::TWD, tx = m % G::TWD;
        la[f] = (uint32_t)((ty * G::HS + tx) * 64 + (lane >> 4) * 16);
        if constexpr (PAD)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) ad[f][dx] = hc_swz(la[f] + dx * 64);
    }
    auto afrag = [&](const char* hb, int f, auto T_) -> bf16x8 {
        constexpr int T = decltype(T_)::value;
        if constexpr (PAD)
            return *reinterpret_cast<const bf16x8*>(hb + ad[f][T % 3] + (T / 3) * G::HS * 64);
        else
            return *reinterpret_cast<const bf16x8*>(hb + hc_swz(la[f] + (uint32_t)(((T / 3) * G::HS + T % 3) * 64)));
    };
    const uint32_t lb = hc_swz((uint32_t)((wn * 64 + (lane & 15)) * 64 + (lane >> 4) * 16));

    const int64_t pb = ((int64_t)img * H + y0 - 1) * W + (x0 - 1);  // halo pixel (0, 0)
    const uint64_t xbu = (uint64_t)(X + pb * Cin);
    const unsigned short* xb = (const unsigned short*)(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(xbu >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xbu));
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)xb, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, 0x7fffffff, 0x00020000);

    auto issue_b = [&](int sl, int tap, int slot) {
        const int so = __builtin_amdgcn_readfirstlane((tap * Cin + sl * 32) * 2);
        char* dst = smem + G::RB + slot * G::BSLOT;
#pragma unroll
        for (int i = 0; i < G::NBW; ++i) {
            const uint32_t v = boff[i];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(dst + (i * G::NW + wave) * 1024), 16, v, so, 0, 0);
        }
    };
    auto issue_h = [&](auto I, int sl) {
        constexpr int i = decltype(I)::value;
        const uint32_t v = hoff[i];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)(smem + (sl & 1) * G::HALO + (i * G::NW + wave) * 1024),
                                                 16, v, sl * 64, 0, 0);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[4], b[4];

    hc_static_for<0, G::NPW>([&](auto I) { issue_h(I, 0); });
#pragma unroll
    for (int d = 0; d < G::D; ++d) issue_b(0, d, d);
    wait_vmn<(G::D - 1) * G::NBW>();  // halo 0 + weights of K-step 0
    P8_BAR();
    EGG_STAMP(1);
    if (G::NW == 8 && grp8 == 1) P8_BAR();

    auto slice = [&](int s, auto NEXT_, auto LAST_) {
        constexpr bool NEXT = decltype(NEXT_)::value, LAST = decltype(LAST_)::value;
        const char* hb = smem + (s & 1) * G::HALO;
        hc_static_for<0, 9>([&](auto T_) {
            constexpr int T = decltype(T_)::value;
            const int k = s * 9 + T;
            const char* bs = smem + G::RB + (k & (G::NBUF - 1)) * G::BSLOT;
            // phase 1: weights + A fragments 0-3, prefetch K-step k+D's weights
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(bs + lb + j * 1024);
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = afrag(hb, u, T_);
            if constexpr (!LAST || T + G::D < 9) {
                if constexpr (T + G::D < 9) issue_b(s, T + G::D, (k + G::D) & (G::NBUF - 1));
                else issue_b(s + 1, T + G::D - 9, (k + G::D) & (G::NBUF - 1));
            }
            P8_LGKM0_;
            P8_BAR();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[u], acc[u][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            P8_BAR();
            // phase 2: A fragments 4-7, one halo piece of slice s+1, retire K-step k+1's weights
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = afrag(hb, 4 + u, T_);
            if constexpr (NEXT && T < G::NPW) issue_h(std::integral_constant<int, T>{}, s + 1);
            if constexpr (!(LAST && T == 8)) wait_vmn<hc_wait_n<G, T, NEXT, LAST>()>();
            P8_LGKM0_;
            P8_BAR();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[4 + u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[u], acc[4 + u][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            P8_BAR();
        });
    };
    for (int s = 0; s < S - 1; ++s) slice(s, std::true_type{}, std::false_type{});
    slice(S - 1, std::false_type{}, std::true_type{});
    if (G::NW == 8 && grp8 == 0) P8_BAR();
    EGG_STAMP(2);
    P8_VM0();
    __syncthreads();
    EGG_STAMP(3);
    const int64_t prow = ((int64_t)img * H + y0) * W + x0;  // output pixel of tile row 0
    auto row_of = [&](int r) -> int64_t { return prow + (int64_t)(r / G::TWD) * W + (r % G::TWD); };
    if (bias)
        lora_mfma_addend<0>(acc, lane, 0, n0, wm * 128, wn * 64, bias, nullptr, nullptr, 0, 0, 0.0f, 1 << 30, 1 << 30, N);
    if constexpr (NORM) {
        // the residual joins in the store phase (coalesced 16-B rows, one more bf16 rounding of the
        // normalised value: bf16(bf16(norm) + res), as the eager bf16 graph x + norm(conv(h)) rounds)
        // (half its loads are issued first, so their latency hides behind the row-sum barrier; all 16
        // would spill)
        u16x8 rv[16];
        load_res_rows<0, 8>(rv, res, lane, wm * 128, n0 + wn * 64, N, row_of);
        conv_rmsnorm_epilogue<1, WMW, WNW>(acc, reinterpret_cast<float*>(smem + G::CSTAGE), wm, wn, lane, row_of, eps,
                                           nw, nb, (const unsigned short*)nullptr);
        EGG_STAMP(4);
        store_tile_rows<0, decltype(row_of), true, true>(acc, smem, wave, lane, wm * 128, n0 + wn * 64, Y, N, row_of,
                                                         res, rv);
    } else {
        EGG_STAMP(4);
        store_tile_rows<ACT>(acc, smem, wave, lane, wm * 128, n0 + wn * 64, Y, N, row_of);
    }
    EGG_STAMP_DRAIN();
    EGG_STAMP(5);
    EGG_STAMP_RT(7);
}

// ------------------------------------------------------------------------------------
// Multi-tile halo conv (eggroll_conv_nhwc_sel kernel 4): one workgroup runs MT vertically stacked
// tiles of one image column as ONE K-step stream, so the next tile's slice-0 halo and first D weight
// K-steps stream in during the current tile's last slice exactly as a middle slice streams slice s+1
// — the per-tile prologue (the first halo + weights, ~11 % of a 128-channel tile) is paid once per
// MT tiles.  What that needs:
//   * the C tile goes out through a DEDICATED wave-private 4-KiB staging region, 32 rows at a time
//     (after the ring: nothing the in-flight DMAs write), so the epilogue overlaps them;
//   * the next tile's halo offsets / buffer base are recomputed in place right before the last slice
//     (the current tile's are dead by then): no extra state is carried through the MFMA loop;
//   * the first two counted waits of the next tile target weights issued BEFORE the epilogue, so
//     they add the epilogue's 16 C-tile stores (a lower bound of its vector-memory ops: waiting for
//     fewer younger ops than exist only over-waits) instead of draining the stores.
// Same MFMA sequence per tile, same epilogue arithmetic: bit-identical to kernel 2.
// ------------------------------------------------------------------------------------
constexpr int HMT_EPI_STORES = 16;  // store_tile_rows_c32: 4 passes x 4 16-B stores per lane

// RES: + the residual rows (the same 16-B row segments as the stores), streamed one pass ahead: the
// caller loads pass 0's four rows (rv) before its norm math, pass p + 1's are issued while pass p goes
// through LDS — 2 x 16 registers instead of all 64 next to the accumulators.
template <int ACT, class RowOf, bool RES = false>
__device__ __forceinline__ void store_tile_rows_c32(f32x4 (&acc)[8][4], char* ctile, int lane, int rbase, int col0,
                                                    unsigned short* __restrict__ Y, int64_t ldy, RowOf row_of,
                                                    const unsigned short* __restrict__ res, u16x8 (&rv)[4]) {
    constexpr int ROWB = 128, SLOTS = 8;
    const int r_l = lane & 15, c_l = (lane >> 4) * 4;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        u16x8 rn[4];
        if constexpr (RES) {
            if (p < 3) load_res_rows<0, 4>(rn, res, lane, rbase + (p + 1) * 32, col0, ldy, row_of);
        }
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
            const int rr = ii * 16 + r_l;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int cc = j * 16 + c_l;
                const int slot = (cc >> 3) ^ (rr & (SLOTS - 1));
                u16x4 o;
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
                    f32x2 v = {acc[2 * p + ii][j][e], acc[2 * p + ii][j][e + 1]};
                    if constexpr (ACT == 1) v = silu2(v);
                    o[e] = f32_to_bf16(v.x);
                    o[e + 1] = f32_to_bf16(v.y);
                }
                *reinterpret_cast<u16x4*>(ctile + rr * ROWB + slot * 16 + (cc & 7) * 2) = o;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this pass's LDS writes done
        u16x8 v[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int rr = it * 8 + (lane >> 3), sl = lane & 7;
            v[it] = *reinterpret_cast<const u16x8*>(ctile + rr * ROWB + ((sl ^ (rr & (SLOTS - 1))) << 4));
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // reads done before the next pass overwrites the region
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int rr = it * 8 + (lane >> 3);
            if constexpr (RES) {
#pragma unroll
                for (int u = 0; u < 8; ++u) v[it][u] = f32_to_bf16(bf16_to_f32(v[it][u]) + bf16_to_f32(rv[it][u]));
            }
            *reinterpret_cast<u16x8*>(Y + row_of(rbase + p * 32 + rr) * ldy + col0 + (lane & 7) * 8) = v[it];
        }
        if constexpr (RES) {
            if (p < 3)
#pragma unroll
                for (int it = 0; it < 4; ++it) rv[it] = rn[it];
        }
    }
}

template <class G, bool NORM>
constexpr int halo_mt_smem_bytes() {
    static_assert(!NORM || G::BM * G::WN_ * 4 <= G::HALO, "RMSNorm row sums go to halo buffer 1");
    return G::LDS + G::NW * 4096;
}

template <int ACT, bool NORM, int WMW, int WNW>
__global__ __launch_bounds__(64 * WMW * WNW, 1) void k_conv3x3_halo_mt(const unsigned short* __restrict__ X,
                                                                      const unsigned short* __restrict__ Wt,
                                                                      const unsigned short* __restrict__ bias, int H,
                                                                      int W, int Cin, int N, int tiles_n, int mt,
                                                                      unsigned short* __restrict__ Y, float eps = 0.0f,
                                                                      const unsigned short* __restrict__ nw = nullptr,
                                                                      const unsigned short* __restrict__ nb = nullptr,
                                                                      const unsigned short* __restrict__ res = nullptr) {
    using G = HC<WMW, WNW>;
    static_assert(G::NW == 8, "one 8-wave workgroup per CU");
    static_assert(halo_mt_smem_bytes<G, NORM>() <= 160 * 1024, "LDS per CU");
    __shared__ __attribute__((aligned(16))) char smem[halo_mt_smem_bytes<G, NORM>()];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WNW, wn = wave % WNW;
    const int grp8 = wave >> 2;
    char* const ctile = smem + G::LDS + wave * 4096;
    // RMSNorm row sums: halo buffer 1 (slice S-1's, S even), free between a tile's last MFMA and the next
    // tile's first slice-1 halo DMA (the prefetch only writes buffer 0 and ring slots 0..D-1)
    float* const red = reinterpret_cast<float*>(smem + G::HALO);
    // XCD-contiguous group ranges; a group = mt vertically stacked tiles of one column, horizontally
    // neighbouring groups (sharing halo columns) adjacent, the N-tiles of one group adjacent
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
    const int grp = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
    const int gm = grp / tiles_n, tn = grp - gm * tiles_n;
    const int n0 = tn * G::BN;
    const int tpr = W / G::TWD, bgs = (H / G::TH) / mt;  // tiles per row band, band groups per image
    const int xt = gm % tpr, gr = gm / tpr;
    const int img = gr / bgs, bg = gr - img * bgs;
    const int x0 = xt * G::TWD;
    const int K = 9 * Cin, S = Cin / 32;
    EGG_STAMP_RT(6);
    EGG_STAMP(0);

    // halo DMA of tile row band y0: piece i*8 + wave holds halo pixels 16p .. 16p+15; out-of-image
    // pixels (and the pad past HP) read as zeros through an out-of-range offset
    uint32_t hoff[G::NPW];
    __amdgpu_buffer_rsrc_t rX;
    auto halo_setup = [&](int y0, int ln) {
#pragma unroll
        for (int i = 0; i < G::NPW; ++i) {
            const int hp = (i * G::NW + wave) * 16 + (ln >> 2);
            const int c = (ln & 3) ^ (((hp >> 2) & 1) << 1);
            const int hy = hp / G::HS, hx = hp - hy * G::HS;
            const int y = y0 - 1 + hy, x = x0 - 1 + hx;
            const bool ok = hp < G::HP && hx < G::HW2 && y >= 0 && y < H && x >= 0 && x < W;
            hoff[i] = ok ? (uint32_t)(((hy * W + hx) * Cin + c * 8) * 2) : 0x80000000u;
        }
        const int64_t pb = ((int64_t)img * H + y0 - 1) * W + (x0 - 1);  // halo pixel (0, 0)
        const uint64_t xbu = (uint64_t)(X + pb * Cin);
        const unsigned short* xb = (const unsigned short*)(
            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(xbu >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xbu));
        rX = __builtin_amdgcn_make_buffer_rsrc((void*)xb, (short)0, 0x7fffffff, 0x00020000);
    };
    uint32_t boff[G::NBW];
#pragma unroll
    for (int i = 0; i < G::NBW; ++i) {
        const int n = (i * G::NW + wave) * 16 + (lane >> 2);
        const int c = (lane & 3) ^ (((n >> 2) & 1) << 1);
        boff[i] = (uint32_t)(((n0 + n) * K + c * 8) * 2);
    }
    // A-fragment addresses (HC PAD layout: one swizzled byte per fragment and column shift dx, the row
    // shift is the ds_read immediate); set per tile from an opaque copy of the lane id so nothing derived
    // from them is carried through the epilogue
    uint32_t ad[8][3];
    auto make_la = [&](int ln) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const int m = wm * 128 + 16 * f + (ln & 15);
            const int ty = m / G::TWD, tx = m % G::TWD;
            const uint32_t L = (uint32_t)((ty * G::HS + tx) * 64 + (ln >> 4) * 16);
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) ad[f][dx] = hc_swz(L + dx * 64);
        }
    };
    const uint32_t lb = hc_swz((uint32_t)((wn * 64 + (lane & 15)) * 64 + (lane >> 4) * 16));
    const __amdgpu_buffer_rsrc_t rW = __builtin_amdgcn_make_buffer_rsrc((void*)Wt, (short)0, 0x7fffffff, 0x00020000);

    auto issue_b = [&](int sl, int tap, int slot) {
        const int so = __builtin_amdgcn_readfirstlane((tap * Cin + sl * 32) * 2);
        char* dst = smem + G::RB + slot * G::BSLOT;
#pragma unroll
        for (int i = 0; i < G::NBW; ++i) {
            const uint32_t v = boff[i];
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(dst + (i * G::NW + wave) * 1024), 16, v, so, 0, 0);
        }
    };
    auto issue_h = [&](auto I, int sl) {
        constexpr int i = decltype(I)::value;
        const uint32_t v = hoff[i];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)(smem + (sl & 1) * G::HALO + (i * G::NW + wave) * 1024),
                                                 16, v, sl * 64, 0, 0);
    };

    f32x4 acc[8][4];
    bf16x8 a[4], b[4];
    const int yb = bg * mt * G::TH;  // first tile's row band
    // a tile's slice-0 halo + first D weight K-steps: for tile 0 here, for tile t+1 right after tile
    // t's last MFMA (before its epilogue), into LDS the epilogue does not touch
    auto prefetch = [&](int y0, int ln) {
        halo_setup(y0, ln);
        hc_static_for<0, G::NPW>([&](auto I) { issue_h(I, 0); });
#pragma unroll
        for (int d = 0; d < G::D; ++d) issue_b(0, d, d);
    };
    prefetch(yb, lane);

    // Every tile restarts the K-step count at 0 (ring slot = K-step & 3; 9 S K-steps per tile, the ring
    // is drained at the tile boundary).  epi: an epilogue's >= HMT_EPI_STORES vector-memory ops sit
    // between this tile's first D weight K-steps and the rest, so the waits that target K-steps 0..D-1
    // (the tile's first wait and taps 0 .. D-2 of slice 0) count them as younger ops.
    auto slice = [&](int s, bool epi, auto NEXT_, auto LAST_) {
        constexpr bool NEXT = decltype(NEXT_)::value, LAST = decltype(LAST_)::value;
        const char* hb = smem + (s & 1) * G::HALO;
        hc_static_for<0, 9>([&](auto T_) {
            constexpr int T = decltype(T_)::value;
            constexpr int DY = (T / 3) * G::HS * 64;
            const int k = s * 9 + T;
            const char* bs = smem + G::RB + (k & (G::NBUF - 1)) * G::BSLOT;
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(bs + lb + j * 1024);
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const bf16x8*>(hb + ad[u][T % 3] + DY);
            if constexpr (!LAST || T + G::D < 9) {
                if constexpr (T + G::D < 9) issue_b(s, T + G::D, (k + G::D) & (G::NBUF - 1));
                else issue_b(s + 1, T + G::D - 9, (k + G::D) & (G::NBUF - 1));
            }
            P8_LGKM0_;
            P8_BAR();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[u], acc[u][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            P8_BAR();
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const bf16x8*>(hb + ad[4 + u][T % 3] + DY);
            if constexpr (NEXT && T < G::NPW) issue_h(std::integral_constant<int, T>{}, s + 1);
            if constexpr (!(LAST && T == 8)) {
                if constexpr (NEXT && T < G::D - 1) {  // only slice 0 can follow an epilogue
                    if (epi) wait_vmn<hc_wait_n<G, T, NEXT, LAST>() + HMT_EPI_STORES>();
                    else wait_vmn<hc_wait_n<G, T, NEXT, LAST>()>();
                } else {
                    wait_vmn<hc_wait_n<G, T, NEXT, LAST>()>();
                }
            }
            P8_LGKM0_;
            P8_BAR();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[4 + u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[u], acc[4 + u][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            P8_BAR();
        });
    };

#pragma unroll 1
    for (int t = 0; t < mt; ++t) {
        const int y0 = yb + t * G::TH;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        make_la(ln);
        if (t > 0) halo_setup(y0, ln);  // this tile's halo offsets again (not kept through the epilogue)
        if (t == 0) wait_vmn<(G::D - 1) * G::NBW>();  // halo 0 + weights of K-step 0
        else wait_vmn<(G::D - 1) * G::NBW + HMT_EPI_STORES>();
        P8_BAR();
        if (t == 0) EGG_STAMP(1);
        if (grp8 == 1) P8_BAR();  // wave-group stagger, realigned before the epilogue
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int s = 0; s < S - 1; ++s) slice(s, t > 0 && s == 0, std::true_type{}, std::false_type{});
        slice(S - 1, false, std::false_type{}, std::true_type{});
        if (grp8 == 0) P8_BAR();
        if (t == 0) EGG_STAMP(2);
        // everything lane-derived that the prefetch and the epilogue need is re-derived here from an opaque
        // copy of the lane id: hoisted out of the tile loop it would be spilled, and a scratch reload
        // waits vmcnt(0) — behind the next tile's prefetch DMAs, i.e. it serialises the two
        int lne = lane;
        asm volatile("" : "+v"(lne));
        if (t + 1 < mt) {
            // every wave has passed its last fragment read of this tile (the barrier above): halo
            // buffer 0 and the ring are free for the next tile
            prefetch(y0 + G::TH, lne);
        }
        const int64_t prow = ((int64_t)img * H + y0) * W + x0;  // output pixel of tile row 0
        auto row_of = [&](int r) -> int64_t { return prow + (int64_t)(r / G::TWD) * W + (r % G::TWD); };
        if (bias)
            lora_mfma_addend<0>(acc, lne, 0, n0, wm * 128, wn * 64, bias, nullptr, nullptr, 0, 0, 0.0f, 1 << 30, 1 << 30,
                                N);
        if constexpr (NORM) {
            u16x8 rv[4];  // pass 0's residual rows, in flight during the norm math
            load_res_rows<0, 4>(rv, res, lne, wm * 128, n0 + wn * 64, N, row_of);
            conv_rmsnorm_epilogue<1, WMW, WNW>(acc, red, wm, wn, lne, row_of, eps, nw, nb,
                                               (const unsigned short*)nullptr);
            store_tile_rows_c32<0, decltype(row_of), true>(acc, ctile, lne, wm * 128, n0 + wn * 64, Y, N, row_of, res,
                                                          rv);
        } else {
            u16x8 rv0[4];
            store_tile_rows_c32<ACT>(acc, ctile, lne, wm * 128, n0 + wn * 64, Y, N, row_of, nullptr, rv0);
        }
        if (t == 0) EGG_STAMP(3);
    }
    EGG_STAMP_DRAIN();
    EGG_STAMP(5);
    EGG_STAMP_RT(7);
}

}  // namespace eggroll

using namespace eggroll;

extern "C" {

#ifdef EGG_STAMPS
// diagnostic build only: copy the first n stamps (n <= 131072 * 8) to host memory
int eggroll_debug_stamps(unsigned long long* host, int64_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_egg_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? EGGROLL_OK
               : EGGROLL_ERR_LAUNCH;
}
#endif

int eggroll_lora_project(const void* X, int64_t ldx, const float* theta_pop, int64_t ld_theta, int64_t offA, int32_t r,
                         int64_t rows_per_member, int64_t M, int64_t K, float* T, void* stream) {
    EGG_CHECK_ARG(M >= 0 && K > 0 && K % 8 == 0 && ldx % 8 == 0 && ldx >= K, "lora_project: need K%%8==0, ldx%%8==0");
    EGG_CHECK_ARG(ld_theta % 4 == 0 && offA % 4 == 0, "lora_project: theta offsets must be 16-byte aligned");
    EGG_CHECK_ARG(rows_per_member > 0, "lora_project: rows_per_member must be > 0");
    if (M == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(X && theta_pop && T, "lora_project: NULL pointer");
    return project(X, ldx, theta_pop, ld_theta, offA, r, rows_per_member, M, K, T, as_stream(stream));
}

int eggroll_lora_project_multi(const void* X, int64_t ldx, const float* theta_pop, int64_t ld_theta,
                               const int64_t* offA_host, int32_t n_lin, int32_t r, int64_t rows_per_member, int64_t M,
                               int64_t K, float* T, void* stream) {
    EGG_CHECK_ARG(n_lin >= 1 && n_lin <= 4 && r >= 1 && n_lin * r <= 8,
                  "lora_project_multi: need 1 <= n_lin <= 4 and n_lin * r <= 8 (n_lin=%d r=%d)", n_lin, r);
    EGG_CHECK_ARG(M >= 0 && K >= 32 && K % 32 == 0 && K <= 4096, "lora_project_multi: need K %% 32 == 0, K <= 4096");
    EGG_CHECK_ARG(ldx % 8 == 0 && ldx >= K, "lora_project_multi: ldx must be a multiple of 8 and >= K");
    EGG_CHECK_ARG(rows_per_member > 0 && ld_theta % 4 == 0, "lora_project_multi: bad rows_per_member / ld_theta");
    if (M == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(X && theta_pop && T && offA_host, "lora_project_multi: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)X & 15) == 0 && ((uintptr_t)theta_pop & 15) == 0,
                  "lora_project_multi: X and theta_pop must be 16-byte aligned (16-byte vector loads)");
    int64_t off[4] = {0, 0, 0, 0};
    for (int l = 0; l < n_lin; ++l) {
        off[l] = offA_host[l];
        EGG_CHECK_ARG(off[l] >= 0 && off[l] % 4 == 0 && off[l] + (int64_t)r * K <= ld_theta,
                      "lora_project_multi: offA[%d] must be 16-byte aligned and inside a theta row", l);
    }
    const unsigned grid = (unsigned)((M + PM_ROWS_PER_BLOCK - 1) / PM_ROWS_PER_BLOCK);
    const size_t lds = (size_t)K * 32;
    hipStream_t st = as_stream(stream);
#define EGG_PM_CASE(nq)                                                                                          \
    case nq:                                                                                                     \
        hipLaunchKernelGGL(k_lora_project_mfma<nq>, dim3(grid), dim3(256), lds, st, (const unsigned short*)X, ldx, \
                           theta_pop, ld_theta, off[0], off[1], off[2], off[3], (int)r, rows_per_member, M, K, T); \
        break;
    switch (n_lin * r) {
        EGG_PM_CASE(1) EGG_PM_CASE(2) EGG_PM_CASE(3) EGG_PM_CASE(4)
        EGG_PM_CASE(5) EGG_PM_CASE(6) EGG_PM_CASE(7) EGG_PM_CASE(8)
        default: break;
    }
#undef EGG_PM_CASE
    EGG_CHECK_LAUNCH("lora_project_multi");
    return EGGROLL_OK;
}

int eggroll_lora_expand(const float* T, const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                        int64_t rows_per_member, int64_t M, int64_t N, void* Y, int64_t ldy, void* stream) {
    EGG_CHECK_ARG(M >= 0 && N > 0 && r >= 1 && r <= 16 && rows_per_member > 0 && ldy >= N, "lora_expand: bad sizes");
    if (M == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(T && theta_pop && Y, "lora_expand: NULL pointer");
    const int64_t work = M * ((N + 7) / 8);
    hipLaunchKernelGGL(k_lora_expand, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, as_stream(stream), T,
                       theta_pop, ld_theta, offB, r, scale, rows_per_member, M, N, (unsigned short*)Y, ldy);
    EGG_CHECK_LAUNCH("lora_expand");
    return EGGROLL_OK;
}

int eggroll_lora_delta_f32(const float* x, int64_t ldx, const float* A, int64_t lda_member, const float* B,
                           int64_t ldb_member, int32_t r, float scale, int64_t rows_per_member, int64_t M, int64_t N,
                           int64_t K, float* y, int64_t ldy, void* stream) {
    EGG_CHECK_ARG(r >= 1 && r <= 8, "lora_delta_f32: r=%d must be in [1, 8]", r);
    EGG_CHECK_ARG(M >= 0 && N > 0 && K > 0 && N < (1ll << 31) && K < (1ll << 31) && rows_per_member > 0,
                  "lora_delta_f32: bad sizes M=%lld N=%lld K=%lld rows_per_member=%lld", (long long)M, (long long)N,
                  (long long)K, (long long)rows_per_member);
    EGG_CHECK_ARG(ldx >= K && ldy >= N && lda_member >= 0 && ldb_member >= 0, "lora_delta_f32: bad strides");
    if (M == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && A && B && y, "lora_delta_f32: NULL pointer");
    const int64_t blocks = std::min<int64_t>((M + 3) / 4, 2048);
    hipStream_t st = as_stream(stream);
#define EGG_DELTA(RV)                                                                                            \
    case RV:                                                                                                     \
        hipLaunchKernelGGL(k_lora_delta_f32<RV>, dim3((unsigned)blocks), dim3(256), 0, st, x, ldx, A, lda_member, \
                           B, ldb_member, scale, rows_per_member, M, (int)N, (int)K, y, ldy);                    \
        break;
    switch (r) {
        EGG_DELTA(1) EGG_DELTA(2) EGG_DELTA(3) EGG_DELTA(4) EGG_DELTA(5) EGG_DELTA(6) EGG_DELTA(7) EGG_DELTA(8)
    }
#undef EGG_DELTA
    EGG_CHECK_LAUNCH("lora_delta_f32");
    return EGGROLL_OK;
}

// Kernel choice is a per-call argument (no process-global state: the C-ABI is thread-safe per
// stream).  0 = automatic: the 8-phase 256x256 kernel when the grid still fills the chip, else the
// 128x128 one-barrier tile.  8 / 9 = 8-phase with MFMA / VALU LoRA epilogue, 12 = as 8 with the
// projection fused (linear_pop only), 128 / 256 = one-barrier tiles.
static int lora_gemm_impl(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                          const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                          int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy,
                          int32_t kernel, void* stream) {
    EGG_CHECK_ARG(kernel == 0 || kernel == 8 || kernel == 9 || kernel == 10 || kernel == 12 || kernel == 128 ||
                      kernel == 256,
                  "lora_gemm: kernel must be 0 (auto), 8, 9, 10, 12, 128 or 256 (got %d)", kernel);
    EGG_CHECK_ARG(M >= 0 && N > 0 && K > 0, "lora_gemm: bad sizes M=%lld N=%lld K=%lld", (long long)M, (long long)N,
                  (long long)K);
    EGG_CHECK_ARG(K % 64 == 0, "lora_gemm: K=%lld must be a multiple of 64", (long long)K);
    EGG_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0 && ldx >= K && ldw >= K && ldy >= N, "lora_gemm: bad strides");
    EGG_CHECK_ARG(r >= 0 && r <= 16, "lora_gemm: r=%d out of range", r);
    EGG_CHECK_ARG(rows_per_member > 0, "lora_gemm: rows_per_member must be > 0");
    EGG_CHECK_ARG(M < (1ll << 31) && N < (1ll << 31) && rows_per_member < (1ll << 31), "lora_gemm: M/N too large");
    if (M == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(X && W && Y, "lora_gemm: NULL pointer");
    EGG_CHECK_ARG(r == 0 || (T && theta_pop), "lora_gemm: T / theta_pop NULL with r > 0");
    hipStream_t st = as_stream(stream);
    const int tsel = kernel ? kernel
                            : ((M / 256) * ((N + 255) / 256) >= 512 ? gemm8_auto(M, N, r, rows_per_member, EPI_NONE) : 128);
    if (tsel == 10 && gemm8n_ok(r, rows_per_member)) {   // else: kernel 8's VALU-epilogue path, as kernel 8 does
        EGG_CHECK_ARG(M * ldx * 2 < (1ll << 31) && N * ldw * 2 < (1ll << 31), "lora_gemm: operand > 2 GiB");
        return launch_gemm8n(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale, rows_per_member, M, N, K, Y,
                             ldy, EPI_NONE, EpiArgs{}, st);
    }
    if (tsel == 8 || tsel == 9 || tsel == 10 || tsel == 12) {
        EGG_CHECK_ARG(M * ldx * 2 < (1ll << 31) && N * ldw * 2 < (1ll << 31), "lora_gemm: operand > 2 GiB");
        const bool mf = tsel != 9 && r <= 2 && rows_per_member >= 256;
        return mf ? launch_gemm8<true>(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale,
                                       rows_per_member, M, N, K, Y, ldy, st)
                  : launch_gemm8<false>(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale,
                                        rows_per_member, M, N, K, Y, ldy, st);
    }
    return tsel == 256 ? launch_gemm<kT256>(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale,
                                            rows_per_member, M, N, K, Y, ldy, st)
                       : launch_gemm<kT128>(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale,
                                            rows_per_member, M, N, K, Y, ldy, st);
}

int eggroll_lora_gemm(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                      const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                      int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy, void* stream) {
    return lora_gemm_impl(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale, rows_per_member, M, N, K, Y,
                          ldy, 0, stream);
}

int eggroll_lora_gemm_sel(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                          const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                          int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy,
                          int32_t kernel, void* stream) {
    EGG_CHECK_ARG(kernel != 12, "lora_gemm_sel: kernel 12 fuses the projection (eggroll_lora_linear_pop_sel only)");
    return lora_gemm_impl(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale, rows_per_member, M, N, K, Y,
                          ldy, kernel, stream);
}

int64_t eggroll_lora_workspace_bytes(int64_t M, int64_t K, int32_t r, int64_t rows_per_member) {
    if (M <= 0 || r <= 0 || rows_per_member <= 0) return 0;
    const int64_t t_bytes = M * r * 4;
    const int64_t n_members = (M + rows_per_member - 1) / rows_per_member;
    const int64_t ak_bytes = n_members * 16 * K * 2;
    return t_bytes > ak_bytes ? t_bytes : ak_bytes;
}

int eggroll_lora_linear_pop_sel(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                                const float* theta_pop, int64_t ld_theta, int64_t offA, int64_t offB, int32_t r,
                                float scale, int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y,
                                int64_t ldy, float* T_ws, int32_t kernel, void* stream) {
    EGG_CHECK_ARG(kernel == 0 || kernel == 8 || kernel == 9 || kernel == 10 || kernel == 12 || kernel == 128 ||
                      kernel == 256,
                  "lora_linear_pop: kernel must be 0 (auto), 8, 9, 10, 12, 128 or 256 (got %d)", kernel);
    EGG_CHECK_ARG(K > 0 && K % 64 == 0, "lora_linear_pop: K=%lld must be a multiple of 64", (long long)K);
    EGG_CHECK_ARG(r >= 0 && r <= 16, "lora_linear_pop: r=%d out of range", r);
    if (M == 0) return EGGROLL_OK;
    if (r > 0 && fused_ok(kernel, r, K, rows_per_member)) {  // projection fused into the 8-phase GEMM
        EGG_CHECK_ARG(X && W && Y && theta_pop && T_ws, "lora_linear_pop: NULL pointer");
        EGG_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0 && ldx >= K && ldw >= K && ldy >= N, "lora_linear_pop: bad strides");
        EGG_CHECK_ARG(ld_theta % 4 == 0 && offA % 4 == 0, "lora_linear_pop: theta offsets must be 16-byte aligned");
        return launch_gemm8f(X, ldx, W, ldw, bias, theta_pop, ld_theta, offA, offB, r, scale, rows_per_member, M, N,
                             K, Y, ldy, T_ws, as_stream(stream));
    }
    if (r > 0) {
        EGG_CHECK_ARG(theta_pop && T_ws, "lora_linear_pop: theta_pop / T_ws NULL with r > 0");
        int rc = eggroll_lora_project(X, ldx, theta_pop, ld_theta, offA, r, rows_per_member, M, K, T_ws, stream);
        if (rc) return rc;
    }
    return lora_gemm_impl(X, ldx, W, ldw, bias, T_ws, theta_pop, ld_theta, offB, r, scale, rows_per_member, M, N, K, Y,
                          ldy, kernel == 12 ? 8 : kernel, stream);
}

// The epilogue GEMM with T = X A_k^T already computed (shared by linear_pop_epi and lora_gemm_epi).
static int gemm_epi_impl(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                         const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                         int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy, int32_t epi,
                         const void* res, int64_t ldr, const void* gate, int64_t gstride, int64_t rows_per_group,
                         int32_t kernel, void* stream) {
    const EpiArgs ea{(const unsigned short*)res, ldr, (const unsigned short*)gate, gstride, rows_per_group};
    const int64_t rpm = r ? rows_per_member : (M > 0 ? M : 1);
    if (kernel == 0) kernel = gemm8_auto(M, N, r, rpm, epi);
    if (kernel == 10)
        return launch_gemm8n(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale, rpm, M, N, K, Y, ldy, epi,
                             ea, as_stream(stream));
    return launch_gemm8_epi(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale, rpm, M, N, K, Y, ldy, epi,
                            ea, as_stream(stream));
}

static int epi_args_ok(const void* X, int64_t ldx, const void* W, int64_t ldw, int32_t r, int64_t rows_per_member,
                       int64_t M, int64_t N, int64_t K, const void* Y, int64_t ldy, int32_t epi, const void* res,
                       int64_t ldr, const void* gate, int64_t gstride, int64_t rows_per_group, int32_t kernel) {
    EGG_CHECK_ARG(kernel == 0 || kernel == 8 || kernel == 10, "lora_linear_pop_epi: kernel must be 0, 8 or 10");
    EGG_CHECK_ARG(epi >= EPI_SILU && epi <= EPI_GELU_ERF, "lora_linear_pop_epi: epi=%d unknown", epi);
    EGG_CHECK_ARG(r >= 0 && r <= 2, "lora_linear_pop_epi: r=%d (epilogue ops need r <= 2)", r);
    EGG_CHECK_ARG(r == 0 || rows_per_member >= 256, "lora_linear_pop_epi: rows_per_member must be >= 256 with r > 0");
    EGG_CHECK_ARG(M >= 0 && N > 0 && K > 0 && K % 64 == 0, "lora_linear_pop_epi: need K %% 64 == 0");
    EGG_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0 && ldx >= K && ldw >= K && ldy >= N, "lora_linear_pop_epi: bad strides");
    EGG_CHECK_ARG(M < (1ll << 31) && N < (1ll << 31) && rows_per_member < (1ll << 31), "lora_linear_pop_epi: M/N too large");
    EGG_CHECK_ARG(epi == EPI_SILU || epi == EPI_GELU || epi == EPI_GELU_ERF || (res && ldr >= N),
                  "lora_linear_pop_epi: res NULL or ldr < N");
    EGG_CHECK_ARG((epi != EPI_GATED && epi != EPI_GATED32) || (gate && gstride >= N && rows_per_group > 0),
                  "lora_linear_pop_epi: bad gate");
    if (M == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(X && W && (Y || epi == EPI_RES32 || epi == EPI_GATED32), "lora_linear_pop_epi: NULL pointer");
    EGG_CHECK_ARG(M * ldx * 2 < (1ll << 31) && N * ldw * 2 < (1ll << 31), "lora_linear_pop_epi: operand > 2 GiB");
    return EGGROLL_OK;
}

int eggroll_lora_linear_pop_epi_sel(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                                    const float* theta_pop, int64_t ld_theta, int64_t offA, int64_t offB, int32_t r,
                                    float scale, int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y,
                                    int64_t ldy, float* T_ws, int32_t epi, const void* res, int64_t ldr,
                                    const void* gate, int64_t gstride, int64_t rows_per_group, int32_t kernel,
                                    void* stream) {
    if (epi == EPI_NONE) {
        EGG_CHECK_ARG(kernel == 0 || kernel == 8 || kernel == 10, "lora_linear_pop_epi: kernel must be 0, 8 or 10");
        return eggroll_lora_linear_pop_sel(X, ldx, W, ldw, bias, theta_pop, ld_theta, offA, offB, r, scale,
                                           rows_per_member, M, N, K, Y, ldy, T_ws, kernel, stream);
    }
    const int rc0 = epi_args_ok(X, ldx, W, ldw, r, rows_per_member, M, N, K, Y, ldy, epi, res, ldr, gate, gstride,
                                rows_per_group, kernel);
    if (rc0 || M == 0) return rc0;
    if (r > 0) {
        EGG_CHECK_ARG(theta_pop && T_ws, "lora_linear_pop_epi: theta_pop / T_ws NULL with r > 0");
        int rc = eggroll_lora_project(X, ldx, theta_pop, ld_theta, offA, r, rows_per_member, M, K, T_ws, stream);
        if (rc) return rc;
    }
    return gemm_epi_impl(X, ldx, W, ldw, bias, T_ws, theta_pop, ld_theta, offB, r, scale, rows_per_member, M, N, K, Y,
                         ldy, epi, res, ldr, gate, gstride, rows_per_group, kernel, stream);
}

int eggroll_lora_gemm_epi_sel(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const float* T,
                              const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r, float scale,
                              int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y, int64_t ldy,
                              int32_t epi, const void* res, int64_t ldr, const void* gate, int64_t gstride,
                              int64_t rows_per_group, int32_t kernel, void* stream) {
    const int rc0 = epi_args_ok(X, ldx, W, ldw, r, rows_per_member, M, N, K, Y, ldy, epi, res, ldr, gate, gstride,
                                rows_per_group, kernel);
    if (rc0 || M == 0) return rc0;
    EGG_CHECK_ARG(r == 0 || (T && theta_pop), "lora_gemm_epi: T / theta_pop NULL with r > 0");
    return gemm_epi_impl(X, ldx, W, ldw, bias, T, theta_pop, ld_theta, offB, r, scale, rows_per_member, M, N, K, Y, ldy,
                         epi, res, ldr, gate, gstride, rows_per_group, kernel, stream);
}

int eggroll_lora_linear_pop_epi(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                                const float* theta_pop, int64_t ld_theta, int64_t offA, int64_t offB, int32_t r,
                                float scale, int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y,
                                int64_t ldy, float* T_ws, int32_t epi, const void* res, int64_t ldr, const void* gate,
                                int64_t gstride, int64_t rows_per_group, void* stream) {
    return eggroll_lora_linear_pop_epi_sel(X, ldx, W, ldw, bias, theta_pop, ld_theta, offA, offB, r, scale,
                                           rows_per_member, M, N, K, Y, ldy, T_ws, epi, res, ldr, gate, gstride,
                                           rows_per_group, 0, stream);
}

int eggroll_lora_linear_pop(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                            const float* theta_pop, int64_t ld_theta, int64_t offA, int64_t offB, int32_t r,
                            float scale, int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y,
                            int64_t ldy, float* T_ws, void* stream) {
    return eggroll_lora_linear_pop_sel(X, ldx, W, ldw, bias, theta_pop, ld_theta, offA, offB, r, scale,
                                       rows_per_member, M, N, K, Y, ldy, T_ws, 0, stream);
}

}  // extern "C"

// The halo-staged kernel takes 3x3 px-1 convs whose tiles are all full: H % 16 == 0, W % TWD == 0
// (TWD = 32 for the 512 x 128 tile, 16 for 256 x 256), N % BN == 0: 512 x 128 (N == 128) or 256 x 256
// (N % 256 == 0), one 8-wave workgroup per CU.  Variant v: 2 = padded halo rows (HC PAD), 3 = the
// round-2 unpadded layout (A/B), 4 = multi-tile (padded).
static bool halo_ok(int v, int64_t ks, int64_t px, int64_t H, int64_t W, int64_t Cin, int64_t N) {
    (void)v;
    if (ks != 3 || px != 1 || H % 16 || 18 * (W + 2) * Cin * 2 >= (1ll << 31)) return false;  // 32-bit halo offsets
    if (N == 128) return W % HC<4>::TWD == 0;
    return N % 256 == 0 && W % HC<2>::TWD == 0;
}

// kernel 4 (multi-tile): tiles per workgroup = the largest of 4, 2, 1 dividing the row bands H / 16
static int halo_mt_tiles(int64_t H) {
    const int64_t bands = H / 16;
    return bands % 4 == 0 ? 4 : bands % 2 == 0 ? 2 : 1;
}

template <int ACT, bool NORM, int WMW, int WNW>
static void launch_halo_mt_t(const void* x, const void* w, const void* bias, int64_t B, int64_t H, int64_t W,
                             int64_t Cin, int64_t N, void* y, float eps, const void* nw, const void* nb, const void* res,
                             hipStream_t st) {
    using G = HC<WMW, WNW>;
    const int mt = halo_mt_tiles(H);
    const int64_t groups = B * (H / 16 / mt) * (W / G::TWD), tn = N / G::BN;
    hipLaunchKernelGGL((k_conv3x3_halo_mt<ACT, NORM, WMW, WNW>), dim3((unsigned)(groups * tn)), dim3(64 * G::NW), 0, st,
                       (const unsigned short*)x, (const unsigned short*)w, (const unsigned short*)bias, (int)H, (int)W,
                       (int)Cin, (int)N, (int)tn, mt, (unsigned short*)y, eps, (const unsigned short*)nw,
                       (const unsigned short*)nb, (const unsigned short*)res);
}

template <int ACT, bool NORM, int WMW, int WNW, bool PAD>
static void launch_halo_t(const void* x, const void* w, const void* bias, int64_t B, int64_t H, int64_t W, int64_t Cin,
                          int64_t N, void* y, float eps, const void* nw, const void* nb, const void* res,
                          hipStream_t st) {
    using G = HC<WMW, WNW, PAD>;
    const int64_t tiles = B * (H / 16) * (W / G::TWD), tn = N / G::BN;
    hipLaunchKernelGGL((k_conv3x3_halo<ACT, NORM, WMW, WNW, PAD>), dim3((unsigned)(tiles * tn)), dim3(64 * G::NW), 0, st,
                       (const unsigned short*)x, (const unsigned short*)w, (const unsigned short*)bias, (int)H, (int)W,
                       (int)Cin, (int)N, (int)tn, (unsigned short*)y, eps, (const unsigned short*)nw,
                       (const unsigned short*)nb, (const unsigned short*)res);
}

template <int ACT, bool NORM>
static void launch_halo(int v, const void* x, const void* w, const void* bias, int64_t B, int64_t H, int64_t W,
                        int64_t Cin, int64_t N, void* y, float eps, const void* nw, const void* nb, const void* res,
                        hipStream_t st) {
    if (v == 4) {
        if (N == 128) launch_halo_mt_t<ACT, NORM, 4, 2>(x, w, bias, B, H, W, Cin, N, y, eps, nw, nb, res, st);
        else launch_halo_mt_t<ACT, NORM, 2, 4>(x, w, bias, B, H, W, Cin, N, y, eps, nw, nb, res, st);
        return;
    }
    if (v == 3 && N == 128) launch_halo_t<ACT, NORM, 4, 2, false>(x, w, bias, B, H, W, Cin, N, y, eps, nw, nb, res, st);
    else if (v == 3) launch_halo_t<ACT, NORM, 2, 4, false>(x, w, bias, B, H, W, Cin, N, y, eps, nw, nb, res, st);
    else if (N == 128) launch_halo_t<ACT, NORM, 4, 2, true>(x, w, bias, B, H, W, Cin, N, y, eps, nw, nb, res, st);
    else launch_halo_t<ACT, NORM, 2, 4, true>(x, w, bias, B, H, W, Cin, N, y, eps, nw, nb, res, st);
}

extern "C" {

/* Implicit-GEMM ks x ks conv, pad 1 (k_conv3x3_gemm8 / k_conv3x3_halo): see include/eggroll.h */
int eggroll_conv_nhwc(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H, int64_t W,
                      int64_t Cin, int64_t N, int32_t ks, int32_t px, int32_t act, void* y, void* stream) {
    return eggroll_conv_nhwc_sel(x, w_packed, bias, B, H, W, Cin, N, ks, px, act, y, 0, stream);
}

int eggroll_conv_nhwc_sel(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H, int64_t W,
                          int64_t Cin, int64_t N, int32_t ks, int32_t px, int32_t act, void* y, int32_t kernel,
                          void* stream) {
    EGG_CHECK_ARG(kernel >= 0 && kernel <= 4, "conv_nhwc: kernel must be 0 (auto), 1 (tap-staged), 2, 3 or 4 (halo)");
    EGG_CHECK_ARG(ks == 2 || ks == 3, "conv_nhwc: ks must be 2 or 3 (got %d)", ks);
    EGG_CHECK_ARG(px == 1 || px == 2, "conv_nhwc: px must be 1 or 2 (got %d)", px);
    EGG_CHECK_ARG(ks == 3 || px == 1, "conv_nhwc: px 2 needs ks 3");
    EGG_CHECK_ARG(act == 0 || act == 2, "conv_nhwc: act must be 0 (none) or 2 (silu) (got %d)", act);
    const int64_t Ho = H + 3 - ks, Wo = W + 3 - ks;
    EGG_CHECK_ARG(B > 0 && H > 0 && W > 0 && Wo % px == 0, "conv_nhwc: bad B/H/W (output width %% px == 0 required)");
    EGG_CHECK_ARG(Cin >= 64 && Cin <= 2048 && (Cin & (Cin - 1)) == 0,
                  "conv_nhwc: Cin=%lld must be a power of two in [64, 2048]", (long long)Cin);
    EGG_CHECK_ARG(N >= 64 && N % 64 == 0 && N <= 8192, "conv_nhwc: N=%lld must be a multiple of 64 (<= 8192)",
                  (long long)N);
    const int64_t Mp = B * Ho * (Wo / px);
    const int64_t K = ks * (px + ks - 1) * Cin;
    // Cout = 128 at px 1 (3x3): the 512 x 128 tile (no zero MACs); everything else 256 x 256
    const bool tall = ks == 3 && px == 1 && N == 128;
    const int64_t BM = tall ? 512 : 256, BN = tall ? 128 : 256;
    EGG_CHECK_ARG(Mp < (1ll << 31) && (BM * (px + 1) + 2 * W + 8) * Cin * 2 < (1ll << 30) && N * K * 2 < (1ll << 31),
                  "conv_nhwc: sizes exceed the kernel's 32-bit offsets");
    EGG_CHECK_ARG(x && w_packed && y, "conv_nhwc: NULL pointer");
    const int64_t tiles_m = (Mp + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    EGG_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "conv_nhwc: grid too large");
    const int hv = kernel == 0 ? 2 : kernel;
    const bool hok = halo_ok(hv, ks, px, H, W, Cin, N);
    EGG_CHECK_ARG(kernel < 2 || hok, "conv_nhwc: halo kernel %d needs ks 3, px 1, H %% 16 == 0 and W, N multiples of "
                  "the tile (see include/eggroll.h)", kernel);
    hipStream_t st = as_stream(stream);
    if (hok && kernel != 1) {
        if (act == 0) launch_halo<0, false>(hv, x, w_packed, bias, B, H, W, Cin, N, y, 0.0f, nullptr, nullptr, nullptr, st);
        else launch_halo<1, false>(hv, x, w_packed, bias, B, H, W, Cin, N, y, 0.0f, nullptr, nullptr, nullptr, st);
        EGG_CHECK_LAUNCH("conv_nhwc");
        return EGGROLL_OK;
    }
    int lcpt = 0;
    while ((64ll << lcpt) < Cin) ++lcpt;
    const dim3 grid((unsigned)(tiles_m * tiles_n));
#define EGG_CONV(PX_, ACT_, KS_, WMW_)                                                                          \
    hipLaunchKernelGGL((k_conv3x3_gemm8<PX_, ACT_, false, KS_, WMW_>), grid, dim3(512), 0, st,                  \
                       (const unsigned short*)x, (const unsigned short*)w_packed, (const unsigned short*)bias, \
                       (int)H, (int)W, (int)Cin, lcpt, (int)Mp, (int)N, (int)tiles_n, (unsigned short*)y, 0.0f,   \
                       nullptr, nullptr, nullptr)
    if (ks == 2) {
        if (act == 0) EGG_CONV(1, 0, 2, 2);
        else EGG_CONV(1, 1, 2, 2);
    } else if (tall && act == 0) EGG_CONV(1, 0, 3, 4);
    else if (tall) EGG_CONV(1, 1, 3, 4);
    else if (px == 1 && act == 0) EGG_CONV(1, 0, 3, 2);
    else if (px == 1) EGG_CONV(1, 1, 3, 2);
    else if (act == 0) EGG_CONV(2, 0, 3, 2);
    else EGG_CONV(2, 1, 3, 2);
#undef EGG_CONV
    EGG_CHECK_LAUNCH("conv_nhwc");
    return EGGROLL_OK;
}

int eggroll_conv2x2_subpixel_nhwc(const void* x, const void* w_packed, const void* bias, const void* src,
                                  int32_t src_f32, int64_t B, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                  void* out, void* shadow, void* stream) {
    EGG_CHECK_ARG(B > 0 && H > 0 && W > 0, "conv2x2_subpixel: bad B/H/W");
    EGG_CHECK_ARG(Cin >= 64 && Cin <= 2048 && (Cin & (Cin - 1)) == 0,
                  "conv2x2_subpixel: Cin=%lld must be a power of two in [64, 2048]", (long long)Cin);
    EGG_CHECK_ARG(Cout >= 64 && Cout % 64 == 0 && 4 * Cout <= 8192 && (4 * Cout) % Cin == 0,
                  "conv2x2_subpixel: Cout=%lld must be a multiple of 64 with 4*Cout a multiple of Cin", (long long)Cout);
    const int64_t rep = 4 * Cout / Cin;
    EGG_CHECK_ARG(rep == 1 || rep == 2 || rep == 4, "conv2x2_subpixel: 4*Cout/Cin = %lld unsupported (1, 2, 4)",
                  (long long)rep);
    EGG_CHECK_ARG(src_f32 == 0 || src_f32 == 1, "conv2x2_subpixel: src_f32 must be 0 or 1");
    EGG_CHECK_ARG(src_f32 || !shadow, "conv2x2_subpixel: shadow needs the fp32 form");
    const int64_t Mp = B * (H + 1) * (W + 1), N = 4 * Cout, K = 4 * Cin;
    EGG_CHECK_ARG(Mp < (1ll << 31) && (256 * 2 + 2 * W + 8) * Cin * 2 < (1ll << 30) && N * K * 2 < (1ll << 31) &&
                      B * 4 * H * W * Cout < (1ll << 31),
                  "conv2x2_subpixel: sizes exceed the kernel's offsets");
    EGG_CHECK_ARG(x && w_packed && src && out, "conv2x2_subpixel: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                      ((uintptr_t)shadow & 15) == 0 && ((uintptr_t)bias & 15) == 0,
                  "conv2x2_subpixel: pointers must be 16-byte aligned");
    const int64_t tiles_m = (Mp + 255) / 256, tiles_n = N / 256 + (N % 256 != 0);
    EGG_CHECK_ARG(tiles_m * tiles_n < (1ll << 31), "conv2x2_subpixel: grid too large");
    int lcpt = 0;
    while ((64ll << lcpt) < Cin) ++lcpt;
    const SubpixArgs spa{(const unsigned short*)bias, src, out, (unsigned short*)shadow, (int)H, (int)W, (int)Cin,
                         (int)Cout};
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)(tiles_m * tiles_n));
#define EGG_SPX(SP_, REP_)                                                                                      \
    hipLaunchKernelGGL((k_conv3x3_gemm8<1, 0, false, 2, 2, SP_, REP_>), grid, dim3(512), 0, st,                 \
                       (const unsigned short*)x, (const unsigned short*)w_packed, nullptr, (int)H, (int)W, (int)Cin, \
                       lcpt, (int)Mp, (int)N, (int)tiles_n, nullptr, 0.0f, nullptr, nullptr, nullptr, spa)
    if (src_f32) {
        if (rep == 1) EGG_SPX(2, 1);
        else if (rep == 2) EGG_SPX(2, 2);
        else EGG_SPX(2, 4);
    } else {
        if (rep == 1) EGG_SPX(1, 1);
        else if (rep == 2) EGG_SPX(1, 2);
        else EGG_SPX(1, 4);
    }
#undef EGG_SPX
    EGG_CHECK_LAUNCH("conv2x2_subpixel_nhwc");
    return EGGROLL_OK;
}

int eggroll_conv3x3_nhwc(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H, int64_t W,
                         int64_t Cin, int64_t N, int32_t px, int32_t act, void* y, void* stream) {
    return eggroll_conv_nhwc(x, w_packed, bias, B, H, W, Cin, N, 3, px, act, y, stream);
}

/* ResBlock conv2 + RMSNorm + residual in one launch: see include/eggroll.h */
int eggroll_conv3x3_rmsnorm_nhwc(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H,
                                 int64_t W, int64_t Cin, int64_t N, int32_t px, float eps, const void* norm_w,
                                 const void* norm_b, const void* res, void* y, void* stream) {
    return eggroll_conv3x3_rmsnorm_nhwc_sel(x, w_packed, bias, B, H, W, Cin, N, px, eps, norm_w, norm_b, res, y, 0,
                                            stream);
}

int eggroll_conv3x3_rmsnorm_nhwc_sel(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H,
                                     int64_t W, int64_t Cin, int64_t N, int32_t px, float eps, const void* norm_w,
                                     const void* norm_b, const void* res, void* y, int32_t kernel, void* stream) {
    EGG_CHECK_ARG(kernel >= 0 && kernel <= 4,
                  "conv3x3_rmsnorm_nhwc: kernel must be 0 (auto), 1 (tap-staged), 2, 3 or 4 (halo)");
    EGG_CHECK_ARG(px == 1 || px == 2, "conv3x3_rmsnorm_nhwc: px must be 1 or 2 (got %d)", px);
    EGG_CHECK_ARG(N == 256 || (N == 128 && px == 1),
                  "conv3x3_rmsnorm_nhwc: N = px * Cout must be 256, or 128 at px 1 (got %lld, px %d)", (long long)N, px);
    const bool tall = N == 128;  // 512 x 128 tile
    EGG_CHECK_ARG(B > 0 && H > 0 && W > 0 && W % px == 0, "conv3x3_rmsnorm_nhwc: bad B/H/W (W %% px == 0 required)");
    EGG_CHECK_ARG(Cin >= 64 && Cin <= 2048 && (Cin & (Cin - 1)) == 0,
                  "conv3x3_rmsnorm_nhwc: Cin=%lld must be a power of two in [64, 2048]", (long long)Cin);
    const int64_t Mp = B * H * (W / px);
    const int64_t BM = tall ? 512 : 256;
    EGG_CHECK_ARG(Mp < (1ll << 31) && (BM * (px + 1) + 2 * W + 8) * Cin * 2 < (1ll << 30),
                  "conv3x3_rmsnorm_nhwc: sizes exceed the kernel's 32-bit offsets");
    EGG_CHECK_ARG(x && w_packed && y && norm_w && res, "conv3x3_rmsnorm_nhwc: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)res & 7) == 0, "conv3x3_rmsnorm_nhwc: res must be 8-byte aligned");
    EGG_CHECK_ARG(res != y && x != y, "conv3x3_rmsnorm_nhwc: y may not alias x or res");
    const int hv = kernel == 0 ? 2 : kernel;
    const bool hok = halo_ok(hv, 3, px, H, W, Cin, N);
    EGG_CHECK_ARG(kernel < 2 || hok, "conv3x3_rmsnorm_nhwc: halo kernel %d needs px 1, H %% 16 == 0 and W a multiple "
                  "of the tile width (see include/eggroll.h)", kernel);
    hipStream_t st = as_stream(stream);
    if (hok && kernel != 1) {
        launch_halo<0, true>(hv, x, w_packed, bias, B, H, W, Cin, N, y, eps, norm_w, norm_b, res, st);
        EGG_CHECK_LAUNCH("conv3x3_rmsnorm_nhwc");
        return EGGROLL_OK;
    }
    int lcpt = 0;
    while ((64ll << lcpt) < Cin) ++lcpt;
    const dim3 grid((unsigned)((Mp + BM - 1) / BM));
#define EGG_CONVN(PX_, WMW_)                                                                                    \
    hipLaunchKernelGGL((k_conv3x3_gemm8<PX_, 0, true, 3, WMW_>), grid, dim3(512), 0, st, (const unsigned short*)x, \
                       (const unsigned short*)w_packed, (const unsigned short*)bias, (int)H, (int)W, (int)Cin, lcpt, \
                       (int)Mp, (int)N, 1, (unsigned short*)y, eps, (const unsigned short*)norm_w,              \
                       (const unsigned short*)norm_b, (const unsigned short*)res)
    if (tall) EGG_CONVN(1, 4);
    else if (px == 1) EGG_CONVN(1, 2);
    else EGG_CONVN(2, 2);
#undef EGG_CONVN
    EGG_CHECK_LAUNCH("conv3x3_rmsnorm_nhwc");
    return EGGROLL_OK;
}

}  // extern "C"
