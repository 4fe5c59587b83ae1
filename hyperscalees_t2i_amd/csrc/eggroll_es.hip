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
__device__ __forceinline__ void box_muller(uint32_t w0, uint32_t w1, float& z0, float& z1) {
#pragma clang fp contract(off)
    // 23-bit uniforms: exact in fp32.  u1 in (0,1), u2 in [0,1).
    const float u1 = ((float)(w0 >> 9) + 0.5f) * 1.1920928955078125e-07f;  // 2^-23
    const float u2 = (float)(w1 >> 9) * 1.1920928955078125e-07f;
    const float rr = sqrtf(-2.0f * logf(u1));
    float s, c;
    sincospif(2.0f * u2, &s, &c);
    z0 = rr * c;
    z1 = rr * s;
}

__global__ __launch_bounds__(256) void k_noise(uint32_t k0, uint32_t k1, int64_t base_lo,
                                               int64_t factor_len, int64_t ld, float* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t g0 = q * 4;
    if (g0 >= factor_len) return;
    const int64_t j = base_lo + blockIdx.y;
    u32x4 c{(uint32_t)q, (uint32_t)(q >> 32), (uint32_t)j, kNoiseTag};
    const u32x4 w = philox4x32_10(c, k0, k1);
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
    const u32x4 w = philox4x32_10(c, k0, k1);
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

__device__ __forceinline__ int find_mat(const eggroll_mat_t* __restrict__ mats, int n_mats, int64_t chunk) {
    int lo = 0, hi = n_mats - 1;
    while (lo < hi) {  // last i with chunk_off <= chunk
        const int mid = (lo + hi + 1) >> 1;
        if (mats[mid].chunk_off <= chunk) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// eps value of element e of matrix `mt` for base sample factor row `fj`
__device__ __forceinline__ float eps_value(const eggroll_mat_t& mt, const float* __restrict__ fj, int64_t e,
                                           int r, float sqrt_r) {
#pragma clang fp contract(off)
    if (mt.cols == 0) return fj[mt.factor_off + e];
    const int64_t row = e / mt.cols, col = e - row * mt.cols;
    const float* a = fj + mt.factor_off + row * r;
    const float* b = fj + mt.factor_off + mt.rows * r + col * r;
    float acc = a[0] * b[0];
    for (int q = 1; q < r; ++q) acc = acc + a[q] * b[q];
    return acc / sqrt_r;
}

// ------------------------------------------------------------------------------------
// perturb / materialise: out[k] = theta + sigma * s_k * E_j(k)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_perturb(const float* __restrict__ theta, const float* __restrict__ factors,
                                                 int64_t ld_f, const eggroll_mat_t* __restrict__ mats, int n_mats,
                                                 int r, float sqrt_r, int32_t pop, int32_t antithetic,
                                                 int64_t member_lo, float sigma, float* __restrict__ out,
                                                 int64_t ld_out) {
#pragma clang fp contract(off)
    const int64_t chunk = blockIdx.x;
    const int mi = find_mat(mats, n_mats, chunk);
    const eggroll_mat_t mt = mats[mi];
    const int64_t numel = mt.cols == 0 ? mt.rows : mt.rows * mt.cols;
    const int64_t e0 = (chunk - mt.chunk_off) * EGGROLL_CHUNK;
    const int64_t k = member_lo + blockIdx.y;
    int64_t j;
    float sgn;
    member_to_base(k, pop, antithetic, j, sgn);
    const float* fj = factors + j * ld_f;
    float* dst = out + (int64_t)blockIdx.y * ld_out + mt.theta_off;
#pragma unroll
    for (int u = 0; u < EGGROLL_CHUNK / 256; ++u) {
        const int64_t e = e0 + u * 256 + threadIdx.x;
        if (e >= numel) break;
        const float eps = sgn * eps_value(mt, fj, e, r, sqrt_r);
        float v;
        if (theta) {
            const float t = sigma * eps;
            v = theta[mt.theta_off + e] + t;
        } else {
            v = sigma * eps;
        }
        dst[e] = v;
    }
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
                                                  float* __restrict__ scores, float* __restrict__ mu,
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
            if (sb < 1e-8f) sb = 1e-8f;  // clamp_min keeps NaN
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
    const int64_t numel = mt.cols == 0 ? mt.rows : mt.rows * mt.cols;
    const int64_t e0 = (chunk - mt.chunk_off) * EGGROLL_CHUNK;
    double pdd = 0.0, poo = 0.0, ptd = 0.0, ptt = 0.0;
#pragma unroll
    for (int u = 0; u < EGGROLL_CHUNK / 256; ++u) {
        const int64_t e = e0 + u * 256 + tid;
        if (e >= numel) break;
        const float th = theta[mt.theta_off + e];
        float v = th;
        if (nf > 0) {
            float acc = 0.0f;
            for (int64_t j = 0; j < n_base; ++j) {
                const float ev = eps_value(mt, factors + j * ld_f, e, r, sqrt_r);
                acc = acc + s_c[j] * ev;
            }
            const float g = acc / (float)nf;
            const float t = lr * g;
            v = th + t;
        }
        out[mt.theta_off + e] = v;
        const double d = (double)v - (double)th;
        pdd += d * d;
        poo += (double)v * (double)v;
        ptd += (double)th * d;
        ptt += (double)th * (double)th;
    }
    pdd = wave_sum_d(pdd);
    poo = wave_sum_d(poo);
    ptd = wave_sum_d(ptd);
    ptt = wave_sum_d(ptt);
    const int w = tid >> 6, lane = tid & 63;
    if (lane == 0) {
        s_red[w][0] = pdd;
        s_red[w][1] = poo;
        s_red[w][2] = ptd;
        s_red[w][3] = ptt;
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
        int theta_on = (max_theta > 0.0f) && (tn > (double)max_theta);
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
    EGG_CHECK_ARG(total_chunks >= 1 && total_chunks < (1ll << 31), "perturb: bad total_chunks");
    if (member_hi == member_lo || D == 0) return EGGROLL_OK;
    const float sqrt_r = (float)sqrt((double)rank);
    dim3 grid((unsigned)total_chunks, (unsigned)(member_hi - member_lo));
    hipLaunchKernelGGL(k_perturb, grid, dim3(256), 0, as_stream(stream), theta, factors, ld_f, mats, n_mats, rank,
                       sqrt_r, pop, antithetic, member_lo, sigma, out, ld_out);
    EGG_CHECK_LAUNCH("perturb");
    return EGGROLL_OK;
}

int eggroll_fitness(const float* S, int32_t n, int32_t m, int32_t use_promptnorm, float* scores, float* mu,
                    float* stats, float* fitness, int32_t* finite, int32_t* order, void* stream) {
    EGG_CHECK_ARG(n >= 1 && n <= 4096 && m >= 1 && m <= 1024, "fitness: need 1<=n<=4096, 1<=m<=1024 (got %d,%d)", n, m);
    EGG_CHECK_ARG(S && scores && mu && stats && fitness && finite && order, "fitness: NULL pointer");
    hipLaunchKernelGGL(k_fitness, dim3(1), dim3(1024), 0, as_stream(stream), S, n, m, use_promptnorm, scores, mu,
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
    EGG_CHECK_ARG(total_chunks >= 1 && total_chunks < (1ll << 31), "update: bad total_chunks");
    EGG_CHECK_ARG(((uintptr_t)workspace & 15) == 0, "update: workspace must be 16-byte aligned");
    if (D == 0) return EGGROLL_OK;
    const float sqrt_r = (float)sqrt((double)rank);
    double* partials = reinterpret_cast<double*>(workspace);
    UpdScalars* sc = reinterpret_cast<UpdScalars*>(partials + total_chunks * 4);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_update_delta, dim3((unsigned)total_chunks), dim3(256), (size_t)n_base * sizeof(float), st,
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
