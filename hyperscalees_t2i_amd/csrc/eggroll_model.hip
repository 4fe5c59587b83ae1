// libeggroll — model-side fused ops used by the Sana / DC-AE host of the ES hot path (gfx950).
//
//   k_dwconv_nhwc    : channels-last depthwise KSxKS conv (stride 1, zero pad KS/2) with optional
//                      SiLU on the input, per-channel bias and optional GLU gate
//                      out[c] = conv[c] * silu(conv[c + C/2]); replaces the GLUMBConv middle of
//                      every Sana FFN and DC-AE EfficientViT block (MIOpen ran it as per-group
//                      grouped GEMMs at ~10% of HBM bandwidth).  LDS-tiled, HBM-bound.
//   k_rownorm        : RMS/Layer norm + affine / AdaLN modulation + act + residual (one pass)
//   k_gated_residual : x += gate[image] * y
//   k_upshortcut_add : DC-AE up-block pixel-shuffle shortcut, fused into the residual add
#include "common.h"

namespace eggroll {

typedef __attribute__((ext_vector_type(8))) unsigned short u16x8m;

__device__ __forceinline__ float b2f(unsigned short h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ unsigned short f2b(float f) {
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<unsigned short*>(&b);
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

// LDS-tiled depthwise conv.  Block = (image b, band of TH output rows, 32 output channels): the
// (TH+KS-1) x (W+KS-1) x 32-channel input tile (and the matching gate-channel tile for GLU) is
// staged into LDS once, SiLU applied once per element (bf16, as torch's silu output), then each
// thread convolves (pixel, 8-channel) outputs from LDS with ds_read_b128.  HBM traffic: input
// ~(TH+KS-1)/TH reads, output one write.
constexpr int DW_CS = 32;          // output channels per block
constexpr int DW_CH = DW_CS / 8;   // 16-B chunks per pixel per plane
constexpr int DW_LDS = 72 * 1024;  // max LDS per block

template <int KS, bool PRE_SILU, bool GLU>
__global__ __launch_bounds__(256, 2) void k_dwconv_nhwc(const unsigned short* __restrict__ in,
                                                     const unsigned short* __restrict__ wt,   // [KS*KS][Cin]
                                                     const unsigned short* __restrict__ bias, // [Cin] or null
                                                     int H, int W, int Cin, int TH, int bands, int cslices,
                                                     unsigned short* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int PLANES = GLU ? 2 : 1;
    constexpr int HALO = KS / 2;
    const int Cout = GLU ? Cin / 2 : Cin;
    const int tid = threadIdx.x;
    int bid = blockIdx.x;
    const int cs = bid % cslices;
    bid /= cslices;
    const int band = bid % bands;
    const int b = bid / bands;
    const int y0 = band * TH;
    const int c0 = cs * DW_CS;
    const int TW = W + KS - 1, TR = TH + KS - 1;
    const int tile_elems = TR * TW * DW_CH;  // 16-B units per plane
    const unsigned short* img = in + (int64_t)b * H * W * Cin;
    for (int u = tid; u < tile_elems * PLANES; u += 256) {
        const int plane = u / tile_elems;
        const int rem = u - plane * tile_elems;
        const int ch = rem % DW_CH;
        const int pix = rem / DW_CH;
        const int ty = pix / TW, tx = pix - ty * TW;
        const int gy = y0 + ty - HALO, gx = tx - HALO;
        u16x8m v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
            v = *reinterpret_cast<const u16x8m*>(img + ((int64_t)gy * W + gx) * Cin + plane * Cout + c0 + ch * 8);
            if (PRE_SILU) {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = f2b(silu(b2f(v[i])));
            }
        }
        *reinterpret_cast<u16x8m*>(lds + (size_t)u * 16) = v;
    }
    // weights [plane][tap][32 ch] after the input tile (the launcher sizes LDS for both)
    char* wlds = lds + (size_t)tile_elems * PLANES * 16;
    for (int u = tid; u < PLANES * KS * KS * DW_CH; u += 256) {
        const int ch = u % DW_CH, t = (u / DW_CH) % (KS * KS), pl = u / (DW_CH * KS * KS);
        *reinterpret_cast<u16x8m*>(wlds + (size_t)u * 16) =
            *reinterpret_cast<const u16x8m*>(wt + t * Cin + pl * Cout + c0 + ch * 8);
    }
    __syncthreads();
    const int ch = tid % DW_CH;
    float bsv[PLANES][8];
#pragma unroll
    for (int pl = 0; pl < PLANES; ++pl)
#pragma unroll
        for (int i = 0; i < 8; ++i) bsv[pl][i] = bias ? b2f(bias[pl * Cout + c0 + ch * 8 + i]) : 0.0f;
    const int npix = TH * W;
    for (int p = tid / DW_CH; p < npix; p += 256 / DW_CH) {
        const int py = p / W, px = p - py * W;
        if (y0 + py >= H) break;
        float acc[PLANES][8];
#pragma unroll
        for (int pl = 0; pl < PLANES; ++pl)
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[pl][i] = bsv[pl][i];
#pragma unroll
        for (int dy = 0; dy < KS; ++dy)
#pragma unroll
            for (int dx = 0; dx < KS; ++dx) {
                const int lp = (py + dy) * TW + (px + dx);
#pragma unroll
                for (int pl = 0; pl < PLANES; ++pl) {
                    const u16x8m v = *reinterpret_cast<const u16x8m*>(lds + ((size_t)pl * tile_elems + lp * DW_CH + ch) * 16);
                    const u16x8m wv = *reinterpret_cast<const u16x8m*>(wlds + ((size_t)(pl * KS * KS + dy * KS + dx) * DW_CH + ch) * 16);
#pragma unroll
                    for (int i = 0; i < 8; ++i) acc[pl][i] += b2f(v[i]) * b2f(wv[i]);
                }
            }
        u16x8m o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = f2b(GLU ? acc[0][i] * silu(acc[PLANES - 1][i]) : acc[0][i]);
        *reinterpret_cast<u16x8m*>(out + (((int64_t)b * H + y0 + py) * W + px) * Cout + c0 + ch * 8) = o;
    }
}

// ------------------------------------------------------------------------------------
// Fused row normalisation over the channel (last) dim of a [rows, C] bf16 tensor:
//   y = norm(x)                      RMS (x / sqrt(mean x^2 + eps)) or LayerNorm (centred)
//   y = y * w[c] (opt) * (1 + mscale[g, c]) (opt) + mshift[g, c] (opt) + b[c] (opt)
//   y = act(y)  (none / relu / silu);   y += res[r, c] (opt)
// g = row / rows_per_group (AdaLN: one modulation vector per image).  SEG lanes per row
// (16/32/64), up to NCH 16-byte chunks per lane, fp32 statistics.
// Covers DC-AE RMSNorm(+bias)(+residual)(+ReLU), Sana q/k/caption RMSNorm, and the Sana AdaLN
// "layer_norm(x) * (1 + scale) + shift" of every block and of norm_out.
// ------------------------------------------------------------------------------------
template <int SEG, int NCH>
__global__ __launch_bounds__(256) void k_rownorm(const unsigned short* __restrict__ x, int64_t rows, int C, float eps,
                                                 int layer, const unsigned short* __restrict__ w,
                                                 const unsigned short* __restrict__ b,
                                                 const unsigned short* __restrict__ mscale,
                                                 const unsigned short* __restrict__ mshift, int64_t mstride,
                                                 int64_t rows_per_group, int act,
                                                 const unsigned short* __restrict__ res,
                                                 unsigned short* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int seg_lane = lane % SEG;
    const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / SEG;
    const bool live = row < rows;
    const int nchunks = C / 8;
    const unsigned short* xr = x + (live ? row : 0) * C;
    float v[NCH][8];
    float s1 = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = seg_lane + t * SEG;
        if (live && ci < nchunks) {
            const u16x8m q = *reinterpret_cast<const u16x8m*>(xr + ci * 8);
#pragma unroll
            for (int i = 0; i < 8; ++i) { v[t][i] = b2f(q[i]); s1 += v[t][i]; }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[t][i] = 0.f;
        }
    }
#pragma unroll
    for (int o = SEG / 2; o > 0; o >>= 1) s1 += __shfl_xor(s1, o, 64);
    const float mean = layer ? s1 / C : 0.f;
    float s2 = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = seg_lane + t * SEG;
        if (ci < nchunks)
#pragma unroll
            for (int i = 0; i < 8; ++i) { const float d = v[t][i] - mean; s2 += d * d; }
    }
#pragma unroll
    for (int o = SEG / 2; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    const float rstd = rsqrtf(s2 / C + eps);
    if (!live) return;
    const int64_t g = row / rows_per_group;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = seg_lane + t * SEG;
        if (ci >= nchunks) continue;
        const int c0 = ci * 8;
        float y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = (v[t][i] - mean) * rstd;
        if (w) {
            const u16x8m q = *reinterpret_cast<const u16x8m*>(w + c0);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] *= b2f(q[i]);
        }
        if (mscale) {
            const u16x8m q = *reinterpret_cast<const u16x8m*>(mscale + g * mstride + c0);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] *= 1.0f + b2f(q[i]);
        }
        if (mshift) {
            const u16x8m q = *reinterpret_cast<const u16x8m*>(mshift + g * mstride + c0);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] += b2f(q[i]);
        }
        if (b) {
            const u16x8m q = *reinterpret_cast<const u16x8m*>(b + c0);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] += b2f(q[i]);
        }
        if (act == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] = y[i] > 0.f ? y[i] : 0.f;
        } else if (act == 2) {
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] = silu(y[i]);
        }
        if (res) {
            const u16x8m q = *reinterpret_cast<const u16x8m*>(res + row * C + c0);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] += b2f(q[i]);
        }
        u16x8m o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = f2b(y[i]);
        *reinterpret_cast<u16x8m*>(out + row * C + c0) = o;
    }
}

// x[r, c] += gate[g, c] * y[r, c]   (bf16, in place; g = r / rows_per_group)
__global__ __launch_bounds__(256) void k_gated_residual(unsigned short* __restrict__ x, const unsigned short* __restrict__ y,
                                                        const unsigned short* __restrict__ gate, int64_t gstride,
                                                        int64_t rows_per_group, int C, int64_t total_chunks) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total_chunks) return;
    const int nch = C / 8;
    const int64_t row = i / nch;
    const int c0 = (int)(i - row * nch) * 8;
    const u16x8m xv = *reinterpret_cast<const u16x8m*>(x + row * C + c0);
    const u16x8m yv = *reinterpret_cast<const u16x8m*>(y + row * C + c0);
    const u16x8m gv = *reinterpret_cast<const u16x8m*>(gate + (row / rows_per_group) * gstride + c0);
    u16x8m o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = f2b(b2f(xv[k]) + b2f(gv[k]) * b2f(yv[k]));
    *reinterpret_cast<u16x8m*>(x + row * C + c0) = o;
}

// y = act(bf16(y + bias[c])) in place (conv bias folded into the activation pass; torch's conv2d
// with bias on MIOpen runs the bias as its own add_ pass).  act: 0 none, 1 relu, 2 silu.
__global__ __launch_bounds__(256) void k_bias_act(unsigned short* __restrict__ y, const unsigned short* __restrict__ bias,
                                                  unsigned nch, int act, unsigned total_chunks) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total_chunks) return;
    const unsigned c0 = (i % nch) * 8;
    u16x8m yv = *reinterpret_cast<const u16x8m*>(y + (size_t)i * 8);
    const u16x8m bv = *reinterpret_cast<const u16x8m*>(bias + c0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float v = b2f(f2b(b2f(yv[k]) + b2f(bv[k])));
        if (act == 1) v = v > 0.f ? v : 0.f;
        else if (act == 2) v = v / (1.0f + __expf(-v));
        yv[k] = f2b(v);
    }
    *reinterpret_cast<u16x8m*>(y + (size_t)i * 8) = yv;
}

// DCUpBlock2d shortcut, NHWC: y[b, 2h+i, 2w+j, c] += x[b, h, w, (4c + 2i + j) / rep]
// (= pixel_shuffle(repeat_interleave(x, rep, channel), 2) without materialising it).
// One thread = one output pixel x 8 channels; 32-bit index math.
__global__ __launch_bounds__(256) void k_upshortcut_add(unsigned short* __restrict__ y, const unsigned short* __restrict__ x,
                                                        int H, int W, int Cin, int Cout, int rep, int pix_total) {
    const int groups = Cout >> 3;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int pix = t / groups;
    if (pix >= pix_total) return;
    const int c0 = (t - pix * groups) << 3;
    const int W2 = 2 * W, HW4 = 4 * H * W;
    const int bb = pix / HW4;
    const int r = pix - bb * HW4;
    const int Y = r / W2, X = r - Y * W2;
    const int k = 2 * (Y & 1) + (X & 1);
    const unsigned short* src = x + ((int64_t)(bb * H + (Y >> 1)) * W + (X >> 1)) * Cin;
    unsigned short* dst = y + (int64_t)pix * Cout + c0;
    u16x8m yv = *reinterpret_cast<const u16x8m*>(dst);
#pragma unroll
    for (int i = 0; i < 8; ++i) yv[i] = f2b(b2f(yv[i]) + b2f(src[(4 * (c0 + i) + k) / rep]));
    *reinterpret_cast<u16x8m*>(dst) = yv;
}

// Sub-pixel up-block output, NHWC: out[b, 2h+i, 2w+j, c] = y4[b, h+i, w+j, (2i+j)*Cout + c]
//                                                      + x[b, h, w, (4c + 2i + j) / rep]
// y4 = conv2d(x, W4, pad 1) with 2x2 phase kernels [B, H+1, W+1, 4*Cout]: equal to
// conv3x3(upsample_nearest_x2(x)) + pixel_shuffle(repeat_interleave(x)) (DCUpBlock2d).
__global__ __launch_bounds__(256) void k_subpixel_shortcut(const unsigned short* __restrict__ y4,
                                                           const unsigned short* __restrict__ x,
                                                           unsigned short* __restrict__ out, int H, int W, int Cin,
                                                           int Cout, int rep, int pix_total) {
    const int groups = Cout >> 3;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int pix = t / groups;
    if (pix >= pix_total) return;
    const int c0 = (t - pix * groups) << 3;
    const int W2 = 2 * W, HW4 = 4 * H * W;
    const int bb = pix / HW4;
    const int r = pix - bb * HW4;
    const int Y = r / W2, X = r - Y * W2;
    const int i = Y & 1, j = X & 1, h = Y >> 1, w = X >> 1;
    const int k = 2 * i + j;
    const unsigned short* src = x + ((int64_t)(bb * H + h) * W + w) * Cin;
    const u16x8m yv = *reinterpret_cast<const u16x8m*>(
        y4 + ((int64_t)(bb * (H + 1) + h + i) * (W + 1) + (w + j)) * (4 * Cout) + k * Cout + c0);
    u16x8m o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2b(b2f(yv[q]) + b2f(src[(4 * (c0 + q) + k) / rep]));
    *reinterpret_cast<u16x8m*>(out + (int64_t)pix * Cout + c0) = o;
}

// ------------------------------------------------------------------------------------
// ReLU linear attention, head dim 32 (SanaLinearAttnProcessor2_0 / DC-AE multiscale attention):
//   kv[i][j] = sum_n v[n,i] relu(k[n,j]),  ksum[j] = sum_n relu(k[n,j])     (per image, head)
//   out[n,i] = (sum_j relu(q[n,j]) kv[i][j]) / (sum_j relu(q[n,j]) ksum[j] + 1e-15)
// fp32 accumulation.  Pass 1: per (image*head, token chunk) partial kv/ksum -> workspace;
// pass 2: per (image*head, token chunk) fixed-order sum of the partials in LDS, then one token
// per thread.  q/k/v are strided views (row stride, head stride) of the projection outputs.
// ------------------------------------------------------------------------------------
constexpr int LA_D = 32;
constexpr int LA_PART = LA_D * LA_D + LA_D;   // kv + ksum floats per partial
constexpr int LA_T = 256;                     // tokens per chunk

__global__ __launch_bounds__(256) void k_la_kv(const unsigned short* __restrict__ k, const unsigned short* __restrict__ v,
                                               int64_t ld, int64_t hstride, int heads, int N, int nchunk, int relu,
                                               float* __restrict__ part) {
    __shared__ float sk[LA_T][LA_D + 1];
    __shared__ float sv[LA_T][LA_D + 1];
    const int bh = blockIdx.x / nchunk, c = blockIdx.x - bh * nchunk;
    const int b = bh / heads, h = bh - b * heads;
    const int n0 = c * LA_T;
    const int cnt = (N - n0) < LA_T ? (N - n0) : LA_T;
    const int tid = threadIdx.x;
    // stage LA_T tokens x 32 dims of k and v (16-B loads: 4 per token row per tensor)
    for (int u = tid; u < LA_T * 4; u += 256) {
        const int t = u >> 2, q4 = u & 3;
        float kf[8], vf[8];
        if (t < cnt) {
            const int64_t off = ((int64_t)b * N + n0 + t) * ld + (int64_t)h * hstride + q4 * 8;
            const u16x8m kv8 = *reinterpret_cast<const u16x8m*>(k + off);
            const u16x8m vv8 = *reinterpret_cast<const u16x8m*>(v + off);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float kk = b2f(kv8[i]);
                kf[i] = relu ? (kk > 0.f ? kk : 0.f) : kk;
                vf[i] = b2f(vv8[i]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) kf[i] = vf[i] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            sk[t][q4 * 8 + i] = kf[i];
            sv[t][q4 * 8 + i] = vf[i];
        }
    }
    __syncthreads();
    // thread -> row i = tid / 8, columns j0 = (tid % 8) * 4 .. +3 of kv; threads < 32 also do ksum
    const int i = tid >> 3, j0 = (tid & 7) * 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, ks = 0.f;
    for (int t = 0; t < cnt; ++t) {
        const float vi = sv[t][i];
        a0 += vi * sk[t][j0];
        a1 += vi * sk[t][j0 + 1];
        a2 += vi * sk[t][j0 + 2];
        a3 += vi * sk[t][j0 + 3];
        if (tid < LA_D) ks += sk[t][tid];
    }
    float* dst = part + (int64_t)blockIdx.x * LA_PART;
    dst[i * LA_D + j0] = a0;
    dst[i * LA_D + j0 + 1] = a1;
    dst[i * LA_D + j0 + 2] = a2;
    dst[i * LA_D + j0 + 3] = a3;
    if (tid < LA_D) dst[LA_D * LA_D + tid] = ks;
}

__global__ __launch_bounds__(256) void k_la_out(const unsigned short* __restrict__ q, int64_t ld, int64_t hstride,
                                                int heads, int N, int nchunk, int relu, const float* __restrict__ part,
                                                unsigned short* __restrict__ out, int64_t ldo) {
    __shared__ float skv[LA_PART];
    const int bh = blockIdx.x / nchunk, c = blockIdx.x - bh * nchunk;
    const int b = bh / heads, h = bh - b * heads;
    const int tid = threadIdx.x;
    for (int e = tid; e < LA_PART; e += 256) {
        float s = 0.f;
        for (int cc = 0; cc < nchunk; ++cc) s += part[((int64_t)bh * nchunk + cc) * LA_PART + e];
        skv[e] = s;
    }
    __syncthreads();
    const int n = c * LA_T + tid;
    if (n >= N) return;
    const int64_t row = (int64_t)b * N + n;
    float qv[LA_D];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
        const u16x8m q8 = *reinterpret_cast<const u16x8m*>(q + row * ld + (int64_t)h * hstride + q4 * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float x = b2f(q8[i]);
            qv[q4 * 8 + i] = relu ? (x > 0.f ? x : 0.f) : x;
        }
    }
    float den = 0.f;
#pragma unroll
    for (int j = 0; j < LA_D; ++j) den += qv[j] * skv[LA_D * LA_D + j];
    const float inv = 1.0f / (den + 1e-15f);
    unsigned short* o = out + row * ldo + h * LA_D;
#pragma unroll
    for (int i0 = 0; i0 < LA_D; i0 += 8) {
        u16x8m o8;
#pragma unroll
        for (int ii = 0; ii < 8; ++ii) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < LA_D; ++j) s += qv[j] * skv[(i0 + ii) * LA_D + j];
            o8[ii] = f2b(s * inv);
        }
        *reinterpret_cast<u16x8m*>(o + i0) = o8;
    }
}

}  // namespace eggroll

using namespace eggroll;

template <int SEG, int NCH>
static void launch_rownorm(const void* x, int64_t rows, int C, float eps, int layer, const void* w, const void* b,
                           const void* ms, const void* mh, int64_t mstride, int64_t rpg, int act, const void* res,
                           void* out, hipStream_t st) {
    const int64_t threads = rows * SEG;
    hipLaunchKernelGGL((k_rownorm<SEG, NCH>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                       (const unsigned short*)x, rows, C, eps, layer, (const unsigned short*)w,
                       (const unsigned short*)b, (const unsigned short*)ms, (const unsigned short*)mh, mstride, rpg,
                       act, (const unsigned short*)res, (unsigned short*)out);
}

extern "C" int eggroll_rownorm(const void* x, int64_t rows, int64_t C, float eps, int32_t layer, const void* w,
                               const void* b, const void* mscale, const void* mshift, int64_t mstride,
                               int64_t rows_per_group, int32_t act, const void* res, void* out, void* stream) {
    EGG_CHECK_ARG(rows >= 0 && C > 0 && C % 8 == 0 && C <= 8 * 64 * 8, "rownorm: need C %% 8 == 0, C <= 4096");
    EGG_CHECK_ARG(act >= 0 && act <= 2 && rows_per_group > 0, "rownorm: bad act / rows_per_group");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 && (!res || ((uintptr_t)res & 15) == 0),
                  "rownorm: pointers must be 16-byte aligned");
    EGG_CHECK_ARG(mstride % 8 == 0, "rownorm: modulation stride must be a multiple of 8");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && out, "rownorm: NULL pointer");
    hipStream_t st = as_stream(stream);
    const int nch = (int)(C / 8);
    if (nch <= 16) launch_rownorm<16, 1>(x, rows, (int)C, eps, layer, w, b, mscale, mshift, mstride, rows_per_group, act, res, out, st);
    else if (nch <= 32) launch_rownorm<32, 1>(x, rows, (int)C, eps, layer, w, b, mscale, mshift, mstride, rows_per_group, act, res, out, st);
    else if (nch <= 64) launch_rownorm<64, 1>(x, rows, (int)C, eps, layer, w, b, mscale, mshift, mstride, rows_per_group, act, res, out, st);
    else if (nch <= 128) launch_rownorm<64, 2>(x, rows, (int)C, eps, layer, w, b, mscale, mshift, mstride, rows_per_group, act, res, out, st);
    else if (nch <= 256) launch_rownorm<64, 4>(x, rows, (int)C, eps, layer, w, b, mscale, mshift, mstride, rows_per_group, act, res, out, st);
    else launch_rownorm<64, 8>(x, rows, (int)C, eps, layer, w, b, mscale, mshift, mstride, rows_per_group, act, res, out, st);
    EGG_CHECK_LAUNCH("rownorm");
    return EGGROLL_OK;
}

extern "C" int eggroll_gated_residual(void* x, const void* y, const void* gate, int64_t gstride, int64_t rows,
                                      int64_t C, int64_t rows_per_group, void* stream) {
    EGG_CHECK_ARG(rows >= 0 && C > 0 && C % 8 == 0 && gstride % 8 == 0 && rows_per_group > 0, "gated_residual: bad sizes");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && y && gate, "gated_residual: NULL pointer");
    const int64_t total = rows * (C / 8);
    hipLaunchKernelGGL(k_gated_residual, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (unsigned short*)x, (const unsigned short*)y, (const unsigned short*)gate, gstride,
                       rows_per_group, (int)C, total);
    EGG_CHECK_LAUNCH("gated_residual");
    return EGGROLL_OK;
}

extern "C" int eggroll_dwconv_nhwc(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H, int64_t W,
                                   int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out, void* stream) {
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && C > 0, "dwconv: bad sizes");
    const int64_t cout = glu ? C / 2 : C;
    EGG_CHECK_ARG((!glu || C % 2 == 0) && cout % DW_CS == 0, "dwconv: output channels must be a multiple of %d", DW_CS);
    EGG_CHECK_ARG(ks == 3 || ks == 5, "dwconv: ks=%d unsupported (3, 5)", ks);
    EGG_CHECK_ARG(((uintptr_t)in & 15) == 0 && ((uintptr_t)w_t & 15) == 0 && ((uintptr_t)out & 15) == 0,
                  "dwconv: pointers must be 16-byte aligned");
    EGG_CHECK_ARG(H * W * C < (1ll << 31), "dwconv: image too large");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(in && w_t && out, "dwconv: NULL pointer");
    const int planes = glu ? 2 : 1;
    auto lds_bytes = [&](int64_t th) { return ((th + ks - 1) * (W + ks - 1) + ks * ks) * DW_CH * 16 * planes; };
    int64_t TH = 256 / W;
    if (TH < 1) TH = 1;
    if (TH > H) TH = H;
    while (TH > 1 && lds_bytes(TH) > DW_LDS) --TH;
    EGG_CHECK_ARG(lds_bytes(TH) <= DW_LDS, "dwconv: W=%lld too wide for the LDS tile", (long long)W);
    const int64_t bands = (H + TH - 1) / TH, cslices = cout / DW_CS;
    const int64_t nblk = B * bands * cslices;
    EGG_CHECK_ARG(nblk < (1ll << 31), "dwconv: grid too large");
    const dim3 grid((unsigned)nblk);
    const size_t shm = (size_t)lds_bytes(TH);
    hipStream_t st = as_stream(stream);
    auto* i = (const unsigned short*)in;
    auto* w = (const unsigned short*)w_t;
    auto* bb = (const unsigned short*)bias;
    auto* o = (unsigned short*)out;
#define EGG_DW(KS_, PS_, GL_)                                                                                 \
    hipLaunchKernelGGL((k_dwconv_nhwc<KS_, PS_, GL_>), grid, dim3(256), shm, st, i, w, bb, (int)H, (int)W, (int)C, \
                       (int)TH, (int)bands, (int)cslices, o)
    if (ks == 3 && pre_silu && glu) EGG_DW(3, true, true);
    else if (ks == 3 && !pre_silu && glu) EGG_DW(3, false, true);
    else if (ks == 3 && pre_silu && !glu) EGG_DW(3, true, false);
    else if (ks == 3) EGG_DW(3, false, false);
    else if (ks == 5 && pre_silu && glu) EGG_DW(5, true, true);
    else if (ks == 5 && !pre_silu && glu) EGG_DW(5, false, true);
    else if (ks == 5 && pre_silu) EGG_DW(5, true, false);
    else EGG_DW(5, false, false);
#undef EGG_DW
    EGG_CHECK_LAUNCH("dwconv_nhwc");
    return EGGROLL_OK;
}

extern "C" int eggroll_upshortcut_add(void* y, const void* x, int64_t B, int64_t H, int64_t W, int64_t Cin,
                                      int64_t Cout, void* stream) {
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && (4 * Cout) % Cin == 0 && Cout % 8 == 0,
                  "upshortcut: bad sizes");
    EGG_CHECK_ARG(B * 4 * H * W * Cout < (1ll << 31) && B * H * W * Cin < (1ll << 31), "upshortcut: tensor too large");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && y, "upshortcut: NULL pointer");
    const int64_t pix = B * 4 * H * W;
    const int64_t threads = pix * (Cout / 8);
    hipLaunchKernelGGL(k_upshortcut_add, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (unsigned short*)y, (const unsigned short*)x, (int)H, (int)W, (int)Cin, (int)Cout,
                       (int)(4 * Cout / Cin), (int)pix);
    EGG_CHECK_LAUNCH("upshortcut_add");
    return EGGROLL_OK;
}

extern "C" int eggroll_subpixel_shortcut(const void* y4, const void* x, void* out, int64_t B, int64_t H, int64_t W,
                                         int64_t Cin, int64_t Cout, void* stream) {
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && (4 * Cout) % Cin == 0 && Cout % 8 == 0,
                  "subpixel_shortcut: bad sizes");
    EGG_CHECK_ARG(B * 4 * H * W * Cout < (1ll << 31) && B * (H + 1) * (W + 1) * 4 * Cout < (1ll << 31),
                  "subpixel_shortcut: tensor too large");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(y4 && x && out, "subpixel_shortcut: NULL pointer");
    const int64_t pix = B * 4 * H * W;
    const int64_t threads = pix * (Cout / 8);
    hipLaunchKernelGGL(k_subpixel_shortcut, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (const unsigned short*)y4, (const unsigned short*)x, (unsigned short*)out, (int)H, (int)W,
                       (int)Cin, (int)Cout, (int)(4 * Cout / Cin), (int)pix);
    EGG_CHECK_LAUNCH("subpixel_shortcut");
    return EGGROLL_OK;
}

extern "C" int64_t eggroll_linear_attention_workspace_bytes(int64_t B, int64_t N, int64_t heads) {
    const int64_t nchunk = (N + LA_T - 1) / LA_T;
    return B * heads * nchunk * LA_PART * (int64_t)sizeof(float);
}

extern "C" int eggroll_linear_attention(const void* q, const void* k, const void* v, int64_t ld, int64_t hstride,
                                        int64_t B, int64_t N, int64_t heads, int32_t relu_qk, void* out, int64_t ldo,
                                        void* workspace, void* stream) {
    EGG_CHECK_ARG(B >= 0 && N > 0 && heads > 0 && ld % 8 == 0 && hstride % 8 == 0 && ldo % 8 == 0,
                  "linear_attention: bad sizes/strides");
    EGG_CHECK_ARG(((uintptr_t)q & 15) == 0 && ((uintptr_t)k & 15) == 0 && ((uintptr_t)v & 15) == 0 &&
                  ((uintptr_t)out & 15) == 0, "linear_attention: pointers must be 16-byte aligned");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(q && k && v && out && workspace, "linear_attention: NULL pointer");
    const int64_t nchunk = (N + LA_T - 1) / LA_T;
    const int64_t blocks = B * heads * nchunk;
    EGG_CHECK_ARG(blocks < (1ll << 31), "linear_attention: grid too large");
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_la_kv, dim3((unsigned)blocks), dim3(256), 0, st, (const unsigned short*)k,
                       (const unsigned short*)v, ld, hstride, (int)heads, (int)N, (int)nchunk, relu_qk,
                       (float*)workspace);
    EGG_CHECK_LAUNCH("linear_attention_kv");
    hipLaunchKernelGGL(k_la_out, dim3((unsigned)blocks), dim3(256), 0, st, (const unsigned short*)q, ld, hstride,
                       (int)heads, (int)N, (int)nchunk, relu_qk, (const float*)workspace, (unsigned short*)out, ldo);
    EGG_CHECK_LAUNCH("linear_attention_out");
    return EGGROLL_OK;
}

extern "C" int eggroll_bias_act(void* y, const void* bias, int64_t rows, int64_t C, int32_t act, void* stream) {
    EGG_CHECK_ARG(rows >= 0 && C > 0 && C % 8 == 0 && act >= 0 && act <= 2, "bias_act: bad sizes/act");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(y && bias, "bias_act: NULL pointer");
    const int64_t total = rows * (C / 8);
    EGG_CHECK_ARG(total < (1ll << 32) - 256, "bias_act: tensor too large for 32-bit chunk index");
    hipLaunchKernelGGL(k_bias_act, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (unsigned short*)y, (const unsigned short*)bias, (unsigned)(C / 8), act, (unsigned)total);
    EGG_CHECK_LAUNCH("bias_act");
    return EGGROLL_OK;
}
