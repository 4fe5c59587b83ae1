// libeggroll — model-side fused ops used by the Sana / DC-AE host of the ES hot path (gfx950).
//
//   k_dwconv_nhwc : channels-last depthwise KSxKS conv (stride 1, zero pad KS/2) with optional
//                   SiLU applied to the input on load, per-channel bias, and optional GLU gate
//                   out[c] = conv[c] * silu(conv[c + C/2]).
// Replaces the GLUMBConv middle of every Sana FFN and DC-AE EfficientViT block
// (silu(conv_inverted) -> conv_depth -> chunk -> x * silu(gate)), which MIOpen runs as a
// per-group grouped-GEMM at ~10% of HBM bandwidth.  HBM-bound: one read of the input, one
// write of the output; the KS*KS neighbour re-reads are served from L1/L2.
#include "common.h"

namespace eggroll {

typedef __attribute__((ext_vector_type(8))) unsigned short u16x8m;

__device__ __forceinline__ float b2f(unsigned short h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ unsigned short f2b(float f) {
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<unsigned short*>(&b);
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

template <int KS, bool PRE_SILU, bool GLU>
__global__ __launch_bounds__(256) void k_dwconv_nhwc(const unsigned short* __restrict__ in,
                                                     const unsigned short* __restrict__ wt,   // [KS*KS][Cin]
                                                     const unsigned short* __restrict__ bias, // [Cin] or null
                                                     int H, int W, int Cin, int64_t total,
                                                     unsigned short* __restrict__ out) {
    const int Cout = GLU ? Cin / 2 : Cin;
    const int groups = Cout / 8;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int cg = (int)(idx % groups);
    const int64_t pix = idx / groups;
    const int x = (int)(pix % W);
    const int y = (int)((pix / W) % H);
    const int64_t b = pix / ((int64_t)W * H);
    const int c0 = cg * 8;
    float acc[8], accg[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        acc[i] = bias ? b2f(bias[c0 + i]) : 0.0f;
        accg[i] = (GLU && bias) ? b2f(bias[Cout + c0 + i]) : 0.0f;
    }
    const unsigned short* img = in + b * (int64_t)H * W * Cin;
#pragma unroll
    for (int dy = 0; dy < KS; ++dy) {
        const int yy = y + dy - KS / 2;
        if (yy < 0 || yy >= H) continue;
#pragma unroll
        for (int dx = 0; dx < KS; ++dx) {
            const int xx = x + dx - KS / 2;
            if (xx < 0 || xx >= W) continue;
            const unsigned short* p = img + ((int64_t)yy * W + xx) * Cin + c0;
            const u16x8m v = *reinterpret_cast<const u16x8m*>(p);
            const u16x8m wv = *reinterpret_cast<const u16x8m*>(wt + (dy * KS + dx) * Cin + c0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float a = b2f(v[i]);
                if (PRE_SILU) a = silu(a);
                acc[i] += a * b2f(wv[i]);
            }
            if (GLU) {
                const u16x8m vg = *reinterpret_cast<const u16x8m*>(p + Cout);
                const u16x8m wg = *reinterpret_cast<const u16x8m*>(wt + (dy * KS + dx) * Cin + Cout + c0);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    float g = b2f(vg[i]);
                    if (PRE_SILU) g = silu(g);
                    accg[i] += g * b2f(wg[i]);
                }
            }
        }
    }
    u16x8m o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f2b(GLU ? acc[i] * silu(accg[i]) : acc[i]);
    *reinterpret_cast<u16x8m*>(out + pix * Cout + c0) = o;
}

}  // namespace eggroll

using namespace eggroll;

extern "C" int eggroll_dwconv_nhwc(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H, int64_t W,
                                   int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out, void* stream) {
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && C > 0, "dwconv: bad sizes");
    EGG_CHECK_ARG(C % (glu ? 16 : 8) == 0, "dwconv: C=%lld must be a multiple of %d", (long long)C, glu ? 16 : 8);
    EGG_CHECK_ARG(ks == 3 || ks == 5, "dwconv: ks=%d unsupported (3, 5)", ks);
    EGG_CHECK_ARG(((uintptr_t)in & 15) == 0 && ((uintptr_t)w_t & 15) == 0 && ((uintptr_t)out & 15) == 0,
                  "dwconv: pointers must be 16-byte aligned");
    EGG_CHECK_ARG(H * W * C < (1ll << 31), "dwconv: image too large");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(in && w_t && out, "dwconv: NULL pointer");
    const int64_t cout = glu ? C / 2 : C;
    const int64_t total = B * H * W * (cout / 8);
    const dim3 grid((unsigned)((total + 255) / 256));
    hipStream_t st = as_stream(stream);
    auto* i = (const unsigned short*)in;
    auto* w = (const unsigned short*)w_t;
    auto* bb = (const unsigned short*)bias;
    auto* o = (unsigned short*)out;
#define EGG_DW(KS_, PS_, GL_) \
    hipLaunchKernelGGL((k_dwconv_nhwc<KS_, PS_, GL_>), grid, dim3(256), 0, st, i, w, bb, (int)H, (int)W, (int)C, total, o)
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
