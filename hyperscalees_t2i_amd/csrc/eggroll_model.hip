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
typedef __attribute__((ext_vector_type(8))) __bf16 la_bf16x8;  // MFMA 16x16x32 operand fragment
typedef __attribute__((ext_vector_type(4))) float la_f32x4;     // MFMA 16x16 accumulator fragment

__device__ __forceinline__ float b2f(unsigned short h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ unsigned short f2b(float f) {
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<unsigned short*>(&b);
}
// x * sigmoid(x) with the hardware reciprocal (v_rcp_f32, ~1 ulp) instead of an IEEE division
// (v_div_scale/fmas/fixup): every caller rounds the result to bf16.
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// LDS-tiled depthwise conv, register sliding window.  Block = (image b, band of DW_TH output rows,
// tile of DW_TW output columns, DW_CS channels per plane).  The (TH+KS-1) x (TW+KS-1) input tile of
// each plane (the value plane, and for GLU the gate plane) is staged into LDS once with SiLU applied
// once per element (bf16, as torch's silu output).  Thread = (4-channel group q, column x): it keeps
// its 4 channels' KS*KS fp32 weights in registers and walks the band's rows; for KS = 3 the 3x3 input
// window lives in registers too (one new input row per output row: 3 LDS reads instead of 9).  The
// previous kernel (8-channel threads, weights and every tap re-read from LDS, bf16->fp32 per use)
// ran the Sana FFN shape at 1.4 TB/s, VALU-bound on conversions.
// HBM traffic: input ~(TH+KS-1)/TH (halo rows, mostly L2 hits), output one write.
constexpr int DW_CS = 32;  // channels per plane per block (64 B per pixel: adjacent blocks share lines)
constexpr int DW_TW = 32;  // output columns per block
constexpr int DW_TH = 8;   // output rows per block
constexpr int DW_ORDER_AUTO = 0;
#ifndef EGG_DW5_DOT2  // 5x5 taps on v_dot2_f32_bf16 (1) or bf16 -> fp32 conversions + fp32 FMAs (0, the default):
// the dot2 form issues 100 instead of ~150 VALU per output row but measured SLOWER — 385 -> 412 us at
// 8 x 128^2 x 1536, 203 -> 222 at 8 x 64^2 x 3072 (profiles/r14b_dw5_dot2_ab.log; numerics within 1 bf16 ulp)
#define EGG_DW5_DOT2 0
#endif  // block order of kernel 0 (eggroll_dwconv_nhwc_sel: 1 = order 0, 2 = order 1)

typedef __attribute__((ext_vector_type(4))) unsigned short u16x4m;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2m;

// PW: the DC-AE multi-scale branch's grouped 1x1 conv (groups of DW_CS = 32 channels, the block's
// channel slice) fused behind the depthwise conv: the block's bf16-rounded conv tile [256 px][32 ch]
// goes to LDS and every wave multiplies its 64 pixels by pw[slice] [32 out][32 in] on MFMA (8 x
// 16x16x32), fp32 accumulate, one bf16 rounding — the torch.bmm it replaces rounds the same way.
template <int KS, bool PRE_SILU, bool GLU, bool PW = false>
__global__ __launch_bounds__(256) void k_dwconv_nhwc(const unsigned short* __restrict__ in,
                                                     const unsigned short* __restrict__ wt,   // [KS*KS][Cin]
                                                     const unsigned short* __restrict__ bias, // [Cin] or null
                                                     int H, int W, int Cin, int xtiles, int bands, int cslices,
                                                     unsigned short* __restrict__ out,
                                                     const unsigned short* __restrict__ pw = nullptr, int ord = 0,
                                                     int ldo = 0) {
    static_assert(!PW || (!GLU && DW_CS == 32 && DW_TH * DW_TW == 256), "PW: one 32-channel group per block");
    constexpr int PLANES = GLU ? 2 : 1;
    constexpr int HALO = KS / 2;
    constexpr int TR = DW_TH + KS - 1, TC = DW_TW + KS - 1;
    constexpr int PIXB = DW_CS * 2;  // bytes per staged pixel per plane
    constexpr int IN_BYTES = PLANES * TR * TC * PIXB;
    // PW: the conv tile [256 px][32 ch] bf16 gets its own region, written row by row as the band is
    // computed (no 8 x 4 result registers held to the end: 284 -> ~170 VGPRs, 1 -> 3 waves per SIMD)
    constexpr int PW_BYTES = PW ? DW_TH * DW_TW * 64 : 0;
    __shared__ __attribute__((aligned(16))) char lds[IN_BYTES + PW_BYTES];
    char* const pwt = lds + IN_BYTES;
    auto swz = [](uint32_t L) { return L ^ ((L >> 3) & 32u); };
    const int Cout = GLU ? Cin / 2 : Cin;
    // output row stride: ldo > Cout pads each pixel's row (the last channel slice's blocks zero the
    // <= 32 pad channels), so a following GEMM sees K = ldo, a multiple of its 64-wide k-step
    const int64_t ldo_ = ldo > 0 ? ldo : Cout;
    const int tid = threadIdx.x;
    // Block order on each XCD (xcd_remap: an XCD walks a contiguous range of ids, ~96 blocks in flight).
    // ord 0: channel slice fastest — adjacent slices share 128-B lines, but a band's vertical neighbour
    // (whose rows overlap its halo) is cslices ids away.  ord 1: column sweep — a pair of slices (one
    // 128-B line per pixel), then all bands of the column, then the tile column: both the shared lines
    // and the overlapping halo rows are read within a few neighbouring ids (L2 hits).
    int bid = xcd_remap(blockIdx.x, gridDim.x);
    int cs, xt, band;
    if (ord == 0) {
        cs = bid % cslices;
        bid /= cslices;
        xt = bid % xtiles;
        bid /= xtiles;
        band = bid % bands;
        bid /= bands;
    } else {
        const int cp = (cslices & 1) ? 1 : 2, chi = cslices / cp;
        const int clo = bid % cp;
        bid /= cp;
        band = bid % bands;
        bid /= bands;
        xt = bid % xtiles;
        bid /= xtiles;
        cs = (bid % chi) * cp + clo;
        bid /= chi;
    }
    const int b = bid;
    const int y0 = band * DW_TH, x0 = xt * DW_TW, c0 = cs * DW_CS;
    const char* img = reinterpret_cast<const char*>(in + (int64_t)b * H * W * Cin);
    const uint32_t cin2 = (uint32_t)Cin * 2, rowb = (uint32_t)W * cin2;
    // Stage the 16-byte units [plane][ty][tx][4 chunks] with buffer loads whose addresses cost no VALU
    // work (the address arithmetic of the previous form was ~40% of the kernel's VALU issue, and the
    // kernel is VALU-issue-bound: profiles/r09a_pmc_dwconv.json).  Main columns (tx in [HALO, HALO+32)):
    // thread = (row parity rp, column mc, chunk ch), one image row pair per pass; the row's buffer
    // descriptor (SGPRs: base = the row, size 0 when the row is outside the image) makes the zero padding
    // rows free, and a column past W gets an out-of-range offset (the load returns zeros).  The 2*HALO
    // halo columns: one unit per thread with its own index arithmetic.  Every load of the thread is issued
    // before the first is consumed.
    constexpr uint32_t OOR = 0x80000000u;  // out-of-range buffer offset (images are < 2 GiB: host check)
    const int rp = __builtin_amdgcn_readfirstlane(tid >> 7);  // wave-uniform
    const int mc = (tid >> 2) & 31, ch = tid & 3;
    const uint32_t mvoff = x0 + mc < W ? (uint32_t)(x0 + mc) * cin2 + (uint32_t)(c0 * 2 + ch * 16) : OOR;
    constexpr int MPASS = PLANES * TR / 2;  // TR is even for KS 3 and 5
    static_assert(TR % 2 == 0, "row pairs");
    u16x8m v[MPASS];
#pragma unroll
    for (int p = 0; p < MPASS; ++p) {
        const int pl = (2 * p) / TR, ty = (2 * p) % TR + rp;
        const int gy = y0 + ty - HALO;
        const bool ok = gy >= 0 && gy < H;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(img + (int64_t)(ok ? gy : 0) * rowb + pl * Cout * 2), (short)0, ok ? (int)rowb : 0, 0x00020000);
        v[p] = __builtin_bit_cast(u16x8m, __builtin_amdgcn_raw_buffer_load_b128(rs, mvoff, 0, 0));
    }
    constexpr int HC = 2 * HALO, HUNITS = PLANES * TR * HC * 4, HPER = (HUNITS + 255) / 256;
    const __amdgpu_buffer_rsrc_t rimg = __builtin_amdgcn_make_buffer_rsrc((void*)img, (short)0, (int)(H * rowb),
                                                                          0x00020000);
    u16x8m hv[HPER];
    uint32_t hlds[HPER];
#pragma unroll
    for (int k = 0; k < HPER; ++k) {
        const int u = tid + k * 256;
        const int hch = u & 3, hcol = (u >> 2) % HC, row = (u >> 2) / HC;
        const int pl = row / TR, ty = row - pl * TR;
        const int tx = hcol < HALO ? hcol : hcol + DW_TW;
        const int gy = y0 + ty - HALO, gx = x0 + tx - HALO;
        const bool ok = u < HUNITS && gy >= 0 && gy < H && gx >= 0 && gx < W;
        const uint32_t off = ok ? (uint32_t)(gy * W + gx) * cin2 + (uint32_t)((pl * Cout + c0) * 2 + hch * 16) : OOR;
        hv[k] = __builtin_bit_cast(u16x8m, __builtin_amdgcn_raw_buffer_load_b128(rimg, off, 0, 0));
        hlds[k] = u < HUNITS ? (uint32_t)(((pl * TR + ty) * TC + tx) * 64 + hch * 16) : 0xffffffffu;
    }
    auto pre = [](u16x8m& x) {
        if (PRE_SILU) {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = f2b(silu(b2f(x[i])));
        }
    };
    const uint32_t mlds = (uint32_t)((rp * TC + HALO + mc) * 64 + ch * 16);
#pragma unroll
    for (int p = 0; p < MPASS; ++p) {
        pre(v[p]);
        *reinterpret_cast<u16x8m*>(lds + mlds + (2 * p) * TC * 64) = v[p];
    }
#pragma unroll
    for (int k = 0; k < HPER; ++k) {
        if (hlds[k] != 0xffffffffu) {
            pre(hv[k]);
            *reinterpret_cast<u16x8m*>(lds + hlds[k]) = hv[k];
        }
    }
    __syncthreads();
    const int q = tid & 7, xs = tid >> 3;  // 4-channel group, column in the tile
    const int x = x0 + xs;
    const int cq = c0 + q * 4;
    auto rd = [&](int pl, int ty, int tx, float (&f)[4]) {
        const u16x4m v = *reinterpret_cast<const u16x4m*>(lds + ((pl * TR + ty) * TC + tx) * PIXB + q * 8);
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = b2f(v[i]);
    };
    // output: one buffer descriptor per image (rows past H: offset out of range, store dropped)
    const int64_t obase = (int64_t)b * H * W * ldo_;
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(out + obase), (short)0, (int)((int64_t)H * W * ldo_ * 2), 0x00020000);
    float res[DW_TH][4];  // value-plane results, gated by the second plane (GLU)
#pragma unroll 1
    for (int pl = 0; pl < PLANES; ++pl) {
        // DOT2 (5x5, EGG_DW5_DOT2): weights kept as bf16 pairs (w, 0) / (0, w) for v_dot2_f32_bf16 against the
        // raw bf16 channel pairs of a tap — no per-tap bf16 -> fp32 conversions (the 5x5 form's VALU bound)
        constexpr bool DOT2 = KS == 5 && EGG_DW5_DOT2;
        float w[DOT2 ? 1 : KS * KS][4], bs[4];
        uint32_t wd[DOT2 ? KS * KS : 1][4];
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(wt + pl * Cout), (short)0, (int)(KS * KS * cin2), 0x00020000);
#pragma unroll
        for (int t = 0; t < KS * KS; ++t) {
            const u16x4m wv = __builtin_bit_cast(u16x4m, __builtin_amdgcn_raw_buffer_load_b64(rw, (uint32_t)cq * 2,
                                                                                            t * (int)cin2, 0));
            if constexpr (DOT2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) wd[t][i] = (i & 1) ? ((uint32_t)wv[i] << 16) : (uint32_t)wv[i];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) w[t][i] = b2f(wv[i]);
            }
        }
        if (bias) {
            const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(bias + pl * Cout), (short)0,
                                                                                (int)cin2, 0x00020000);
            const u16x4m bv = __builtin_bit_cast(u16x4m, __builtin_amdgcn_raw_buffer_load_b64(rb, (uint32_t)cq * 2, 0, 0));
#pragma unroll
            for (int i = 0; i < 4; ++i) bs[i] = b2f(bv[i]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) bs[i] = 0.0f;
        }
        // one output row's result -> the PW tile in LDS, the GLU value plane, or the output
        auto emit = [&](int oy, const float (&acc)[4]) {
            if constexpr (PW) {
                // conv tile -> LDS [pixel oy*32+x][32 ch], 64-B rows with slot ^= 2*((pixel >> 2) & 1): the
                // 16x16x32 fragment reads (16 consecutive pixels, 4 chunks) are then bank-conflict-free
                u16x4m o;
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = f2b(acc[i]);
                *reinterpret_cast<u16x4m*>(pwt + swz((uint32_t)((oy * DW_TW + xs) * 64 + q * 8))) = o;
            } else if (pl == 0 && GLU) {
#pragma unroll
                for (int i = 0; i < 4; ++i) res[oy][i] = acc[i];
            } else {
                const int y = y0 + oy;
                u16x4m o;
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = f2b(GLU ? res[oy][i] * silu(acc[i]) : acc[i]);
                const uint32_t px = (uint32_t)(y * W + x) * (uint32_t)ldo_ * 2;
                const bool ok = y < H && x < W;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2m, o), rout,
                                                      ok ? px + (uint32_t)cq * 2 : OOR, 0, 0);
                if (ldo_ > Cout && cs == cslices - 1 && Cout + q * 4 < ldo_)
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2m{0u, 0u}, rout,
                                                          ok ? px + (uint32_t)(Cout + q * 4) * 2 : OOR, 0, 0);
            }
        };
        if constexpr (KS == 3) {
            // the 3x3 input window in registers, sliding down the band: one new input row (3 LDS reads,
            // 12 conversions) per output row instead of 9
            float win[KS][KS][4];
#pragma unroll
            for (int r = 0; r < KS - 1; ++r)
#pragma unroll
                for (int dx = 0; dx < KS; ++dx) rd(pl, r, xs + dx, win[r][dx]);
#pragma unroll
            for (int oy = 0; oy < DW_TH; ++oy) {
#pragma unroll
                for (int dx = 0; dx < KS; ++dx) rd(pl, oy + KS - 1, xs + dx, win[KS - 1][dx]);
                float acc[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = bs[i];
#pragma unroll
                for (int dy = 0; dy < KS; ++dy)
#pragma unroll
                    for (int dx = 0; dx < KS; ++dx)
#pragma unroll
                        for (int i = 0; i < 4; ++i) acc[i] += win[dy][dx][i] * w[dy * KS + dx][i];
#pragma unroll
                for (int r = 0; r < KS - 1; ++r)
#pragma unroll
                    for (int dx = 0; dx < KS; ++dx)
#pragma unroll
                        for (int i = 0; i < 4; ++i) win[r][dx][i] = win[r + 1][dx][i];
                emit(oy, acc);
            }
        } else {
            // KS = 5: every tap read from LDS and converted at its use.  A 5x5 fp32 register window
            // measured 11 % slower (2 vs 3 waves per SIMD, profiles/r05e_dw5_register_window_ab.log), and
            // row groups that convert each input row once for 2-4 output rows spill at 3 waves per SIMD
            // next to the 25 taps' fp32 weights (r09 build, 172-500 B of scratch per lane).  Staging the
            // tile as fp32 (one conversion per staged element, 71.7 KB LDS -> 2 blocks per CU) measured
            // 0.90x (366 -> 408 us at 8 x 128^2 x 1536, profiles/r10a_dw5_fp32_tile_ab.log).
#pragma unroll 1
            for (int oy = 0; oy < DW_TH; ++oy) {
                float acc[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = bs[i];
#pragma unroll
                for (int dy = 0; dy < KS; ++dy)
#pragma unroll
                    for (int dx = 0; dx < KS; ++dx) {
                        if constexpr (DOT2) {
                            typedef __attribute__((ext_vector_type(2))) __bf16 dw_bf2;
                            const u32x2m v = *reinterpret_cast<const u32x2m*>(
                                lds + ((pl * TR + oy + dy) * TC + xs + dx) * PIXB + q * 8);
                            // (the dwords through a plain array: hipcc miscompiles __builtin_bit_cast of an
                            // ext-vector subscript v[i >> 1] into element 0 for every i)
                            const uint32_t xw[2] = {v.x, v.y};
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                acc[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(dw_bf2, xw[i >> 1]),
                                                                         __builtin_bit_cast(dw_bf2, wd[dy * KS + dx][i]),
                                                                         acc[i], false);
                        } else {
                            float tap[4];
                            rd(pl, oy + dy, xs + dx, tap);
#pragma unroll
                            for (int i = 0; i < 4; ++i) acc[i] += tap[i] * w[dy * KS + dx][i];
                        }
                    }
                emit(oy, acc);
            }
        }
    }
    if constexpr (PW) {
        __syncthreads();  // the whole conv tile is in pwt
        const int lane = tid & 63, wv = tid >> 6, r16 = lane & 15, g4 = lane >> 4;
        const unsigned short* pg = pw + (int64_t)cs * (DW_CS * DW_CS);  // [o][c] of this channel group
        la_bf16x8 bo[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
            bo[j] = *reinterpret_cast<const la_bf16x8*>(pg + (16 * j + r16) * DW_CS + 8 * g4);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int p = wv * 64 + 16 * f + r16;  // tile pixel of this lane's fragment row
            const la_bf16x8 a = *reinterpret_cast<const la_bf16x8*>(pwt + swz((uint32_t)(p * 64 + g4 * 16)));
            const int y = y0 + (p >> 5), xx = x0 + (p & 31);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                // transposed product: lane holds pixel p, outputs 16j + 4 g4 .. +3
                const la_f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bo[j], a, la_f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                u16x4m o;
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = f2b(d[e]);
                const uint32_t off = y < H && xx < W ? ((uint32_t)(y * W + xx) * Cout + c0 + 16 * j + 4 * g4) * 2 : OOR;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2m, o), rout, off, 0, 0);
            }
        }
    }
}

// Sum over SEG-lane segments (16 / 32 / 64) without LDS round trips, as the xor butterfly
// __shfl_xor(·, SEG/2 ... 1) computes it — the same additions in the same order, so the same bits in every
// lane: xor 32 / xor 16 by v_permlane32_swap / v_permlane16_swap (gfx950; called on one register twice,
// the two results are each lane's own value and its partner's, and their sum is the butterfly step), xor 8
// by DPP row_ror:8; after that every value is symmetric under xor 8, so row_ror:4 reads the xor-4 partner;
// quad_perm does xor 2 and xor 1.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
template <int SEG>
__device__ __forceinline__ float seg_sum(float v) {
    static_assert(SEG == 16 || SEG == 32 || SEG == 64, "segment of 16, 32 or 64 lanes");
    if constexpr (SEG == 64) {
        const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                         false, false);
        v = __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
    }
    if constexpr (SEG >= 32) {
        const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                         false, false);
        v = __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
    }
    v += dpp_f<0x128>(v);  // row_ror:8 = xor 8
    v += dpp_f<0x124>(v);  // row_ror:4 = xor 4 here
    v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1] = xor 2
    v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2] = xor 1
    return v;
}

// Reductions over the 4 lane groups of 16 (xor 16, then xor 32) on v_permlane16_swap / v_permlane32_swap
// instead of two ds_bpermute shuffles (LDS round trips): each swap returns the lane's own value and its
// partner's, combined exactly as `v op __shfl_xor(v, 16)` then `op __shfl_xor(v, 32)` (+ and max are
// commutative, so the same bits).
__device__ __forceinline__ float g4_sum(float v) {
    auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
    v = __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
    r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
    return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ float g4_max(float v) {
    auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
    v = fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
    r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v), false, false);
    return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
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
// 8 consecutive values of a bf16 (f32 = 0) or fp32 (f32 = 1) vector as floats
__device__ __forceinline__ void load8f(const void* p, int f32, int64_t off, float (&o)[8]) {
    if (f32) {
        const float4 a0 = *reinterpret_cast<const float4*>((const float*)p + off);
        const float4 a1 = *reinterpret_cast<const float4*>((const float*)p + off + 4);
        o[0] = a0.x; o[1] = a0.y; o[2] = a0.z; o[3] = a0.w; o[4] = a1.x; o[5] = a1.y; o[6] = a1.z; o[7] = a1.w;
    } else {
        const u16x8m q = *reinterpret_cast<const u16x8m*>((const unsigned short*)p + off);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = b2f(q[i]);
    }
}

// XF: x is fp32 (the fp32 residual stream of the Sana blocks); mf32: the modulation
// vectors mscale / mshift are fp32 (the fp32 AdaLN modulation); rf32: res is fp32.  OF: the output
// is fp32 (the DC-AE fp32 residual stream: out = res + norm(x) in place of res) and `shadow` (optional)
// receives its bf16 copy; else the output is bf16 (a GEMM operand).
template <int SEG, int NCH, bool XF, bool OF>
__global__ __launch_bounds__(256) void k_rownorm(const void* __restrict__ x, int64_t rows, int C, float eps,
                                                 int layer, const unsigned short* __restrict__ w,
                                                 const unsigned short* __restrict__ b,
                                                 const void* __restrict__ mscale,
                                                 const void* __restrict__ mshift, int64_t mstride, int mf32,
                                                 int64_t rows_per_group, int act,
                                                 const void* __restrict__ res, int rf32,
                                                 void* __restrict__ out, unsigned short* __restrict__ shadow) {
    const int lane = threadIdx.x & 63;
    const int seg_lane = lane % SEG;
    const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / SEG;
    const bool live = row < rows;
    const int nchunks = C / 8;
    const int64_t xoff = (live ? row : 0) * C;
    float v[NCH][8];
    float s1 = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = seg_lane + t * SEG;
        if (live && ci < nchunks) {
            load8f(x, XF, xoff + ci * 8, v[t]);
#pragma unroll
            for (int i = 0; i < 8; ++i) s1 += v[t][i];
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[t][i] = 0.f;
        }
    }
    s1 = seg_sum<SEG>(s1);
    const float mean = layer ? s1 / C : 0.f;
    float s2 = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = seg_lane + t * SEG;
        if (ci < nchunks)
#pragma unroll
            for (int i = 0; i < 8; ++i) { const float d = v[t][i] - mean; s2 += d * d; }
    }
    s2 = seg_sum<SEG>(s2);
    const float rstd = rsqrtf(s2 / C + eps);
    if (!live) return;
    const int64_t g = row / rows_per_group;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = seg_lane + t * SEG;
        if (ci >= nchunks) continue;
        const int c0 = ci * 8;
        float y[8], q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = (v[t][i] - mean) * rstd;
        if (w) {
            load8f(w, 0, c0, q);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] *= q[i];
        }
        if (mscale) {
            load8f(mscale, mf32, g * mstride + c0, q);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] *= 1.0f + q[i];
        }
        if (mshift) {
            load8f(mshift, mf32, g * mstride + c0, q);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] += q[i];
        }
        if (b) {
            load8f(b, 0, c0, q);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] += q[i];
        }
        if (act == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] = y[i] > 0.f ? y[i] : 0.f;
        } else if (act == 2) {
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] = silu(y[i]);
        }
        if (res) {
            load8f(res, rf32, row * C + c0, q);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] += q[i];
        }
        if constexpr (OF) {
            float* o32 = reinterpret_cast<float*>(out) + row * C + c0;
            *reinterpret_cast<float4*>(o32) = float4{y[0], y[1], y[2], y[3]};
            *reinterpret_cast<float4*>(o32 + 4) = float4{y[4], y[5], y[6], y[7]};
        }
        if (!OF || shadow) {
            u16x8m o;
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = f2b(y[i]);
            *reinterpret_cast<u16x8m*>((OF ? shadow : reinterpret_cast<unsigned short*>(out)) + row * C + c0) = o;
        }
    }
}

// ------------------------------------------------------------------------------------
// fp32 residual stream + LayerNorm of the CLIP reward towers (clip_tower.py, fp32_residual):
//   h[r] += float(y[r])           (y bf16, optional: the block output just computed by a GEMM)
//   out[r] = bf16(LN(h[r]) * w + b) with fp32 statistics (mean, then the centred second moment)
// One 64-lane wave per row (h held in registers between the passes), 8 channels per lane-chunk.
// Replaces, per residual point, torch's bf16->fp32 copy, fp32 add, fp32 layer_norm and the bf16
// cast of its output (four passes over the row, three of them over the fp32 stream).
// ------------------------------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void k_resid_layernorm(float* __restrict__ h, int64_t ldh,
                                                         const unsigned short* __restrict__ y, int64_t ldy,
                                                         int64_t rows, int C, float eps,
                                                         const unsigned short* __restrict__ w,
                                                         const unsigned short* __restrict__ b,
                                                         unsigned short* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (row >= rows) return;  // whole waves: a row is one wave
    const int nchunks = C >> 3;
    float* hr = h + row * ldh;
    const unsigned short* yr = y ? y + row * ldy : nullptr;
    float v[NCH][8];
    float s1 = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = lane + t * 64;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[t][i] = 0.f;
        if (ci < nchunks) {
            const float4 a0 = *reinterpret_cast<const float4*>(hr + ci * 8);
            const float4 a1 = *reinterpret_cast<const float4*>(hr + ci * 8 + 4);
            v[t][0] = a0.x; v[t][1] = a0.y; v[t][2] = a0.z; v[t][3] = a0.w;
            v[t][4] = a1.x; v[t][5] = a1.y; v[t][6] = a1.z; v[t][7] = a1.w;
            if (yr) {
                const u16x8m q = *reinterpret_cast<const u16x8m*>(yr + ci * 8);
#pragma unroll
                for (int i = 0; i < 8; ++i) v[t][i] += b2f(q[i]);
                *reinterpret_cast<float4*>(hr + ci * 8) = float4{v[t][0], v[t][1], v[t][2], v[t][3]};
                *reinterpret_cast<float4*>(hr + ci * 8 + 4) = float4{v[t][4], v[t][5], v[t][6], v[t][7]};
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) s1 += v[t][i];
        }
    }
    s1 = seg_sum<64>(s1);
    const float mean = s1 / C;
    float s2 = 0.f;
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        if (lane + t * 64 < nchunks)
#pragma unroll
            for (int i = 0; i < 8; ++i) { const float d = v[t][i] - mean; s2 += d * d; }
    }
    s2 = seg_sum<64>(s2);
    const float rstd = rsqrtf(s2 / C + eps);
#pragma unroll
    for (int t = 0; t < NCH; ++t) {
        const int ci = lane + t * 64;
        if (ci >= nchunks) continue;
        const u16x8m qw = *reinterpret_cast<const u16x8m*>(w + ci * 8);
        const u16x8m qb = *reinterpret_cast<const u16x8m*>(b + ci * 8);
        u16x8m o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = f2b((v[t][i] - mean) * rstd * b2f(qw[i]) + b2f(qb[i]));
        *reinterpret_cast<u16x8m*>(out + row * C + ci * 8) = o;
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

// fp32 residual stream update (Sana blocks):  x[r, c] = fma(gate[g, c], y[r, c], x[r, c])
// (x fp32 in place, y bf16, gate bf16 or fp32 (g32) or NULL = 1: x += y), optionally also writing the
// bf16 shadow copy of x that the next GEMM reads.  The same expression as the fused GEMM epilogues
// EPI_RES32 / EPI_GATED32 of eggroll_lora.hip, so fused == unfused bit for bit.
__global__ __launch_bounds__(256) void k_gated_residual_f32(float* __restrict__ x, const unsigned short* __restrict__ y,
                                                            const void* __restrict__ gate, int g32, int64_t gstride,
                                                            int64_t rows_per_group, int C, int64_t total_chunks,
                                                            unsigned short* __restrict__ shadow) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total_chunks) return;
    const int nch = C / 8;
    const int64_t row = i / nch;
    const int c0 = (int)(i - row * nch) * 8;
    float xv[8], yv[8], gv[8];
    load8f(x, 1, row * C + c0, xv);
    load8f(y, 0, row * C + c0, yv);
    if (gate) {
        load8f(gate, g32, (row / rows_per_group) * gstride + c0, gv);
#pragma unroll
        for (int k = 0; k < 8; ++k) xv[k] = __builtin_fmaf(gv[k], yv[k], xv[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) xv[k] = xv[k] + yv[k];
    }
    *reinterpret_cast<float4*>(x + row * C + c0) = float4{xv[0], xv[1], xv[2], xv[3]};
    *reinterpret_cast<float4*>(x + row * C + c0 + 4) = float4{xv[4], xv[5], xv[6], xv[7]};
    if (shadow) {
        u16x8m o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = f2b(xv[k]);
        *reinterpret_cast<u16x8m*>(shadow + row * C + c0) = o;
    }
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
                                                           const unsigned short* __restrict__ bias,
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
    for (int q = 0; q < 8; ++q)
        o[q] = f2b(b2f(yv[q]) + (bias ? b2f(bias[c0 + q]) : 0.f) + b2f(src[(4 * (c0 + q) + k) / rep]));
    *reinterpret_cast<u16x8m*>(out + (int64_t)pix * Cout + c0) = o;
}

// Same output, one thread per LOW-resolution pixel (b, h, w) and 8 output channels c0..c0+7, all four
// phases (i, j): the shortcut source channels (4c + 2i + j) / REP of all phases lie in one
// 32/REP-channel window of x[b, h, w] starting at 4 c0 / REP, loaded as 16-byte vectors and indexed
// with compile-time positions (the per-output kernel above gathers them as 8 scalar 2-byte loads
// per output chunk).  REP = 4 Cout / Cin in {1, 2, 4}.
// F32: the DC-AE fp32 residual stream — x (the shortcut source) and out are fp32, and `shadow`
// (optional) receives bf16(out); the same arithmetic on the fp32 shortcut values.
template <int REP, bool F32 = false>
__global__ __launch_bounds__(256) void k_subpixel_shortcut4(const unsigned short* __restrict__ y4,
                                                            const void* __restrict__ x,
                                                            const unsigned short* __restrict__ bias,
                                                            void* __restrict__ out, int H, int W, int Cin,
                                                            int Cout, int lowpix_total,
                                                            unsigned short* __restrict__ shadow = nullptr) {
    constexpr int XW = 32 / REP;  // source window (channels)
    const int groups = Cout >> 3;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int lp = t / groups;
    if (lp >= lowpix_total) return;
    const int c0 = (t - lp * groups) << 3;
    const int HW = H * W;
    const int bb = lp / HW;
    const int r = lp - bb * HW;
    const int h = r / W, w = r - h * W;
    float xs[XW];
#pragma unroll
    for (int v = 0; v < XW / 8; ++v) {
        float q[8];
        load8f(x, F32, (int64_t)lp * Cin + 4 * c0 / REP + 8 * v, q);
#pragma unroll
        for (int e = 0; e < 8; ++e) xs[8 * v + e] = q[e];
    }
    float bv[8];
    if (bias) {
        const u16x8m q = *reinterpret_cast<const u16x8m*>(bias + c0);
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = b2f(q[e]);
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = 0.f;
    }
    u16x8m yv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = k >> 1, j = k & 1;
        yv[k] = *reinterpret_cast<const u16x8m*>(
            y4 + ((int64_t)(bb * (H + 1) + h + i) * (W + 1) + (w + j)) * (4 * Cout) + k * Cout + c0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = k >> 1, j = k & 1;
        const int64_t opix = ((int64_t)(bb * 2 * H + 2 * h + i) * (2 * W) + 2 * w + j) * Cout + c0;
        float f[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) f[q] = b2f(yv[k][q]) + bv[q] + xs[(4 * q + k) / REP];
        if constexpr (F32) {
            float* o32 = reinterpret_cast<float*>(out) + opix;
            *reinterpret_cast<float4*>(o32) = float4{f[0], f[1], f[2], f[3]};
            *reinterpret_cast<float4*>(o32 + 4) = float4{f[4], f[5], f[6], f[7]};
        }
        if (!F32 || shadow) {
            u16x8m o;
#pragma unroll
            for (int q = 0; q < 8; ++q) o[q] = f2b(f[q]);
            *reinterpret_cast<u16x8m*>((F32 ? shadow : reinterpret_cast<unsigned short*>(out)) + opix) = o;
        }
    }
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
#ifndef EGG_LA_HEAD_PAIRS
#define EGG_LA_HEAD_PAIRS 1
#endif
#ifndef EGG_LA_FOLD  // k_la_kv_fold for few chunks per head (A/B knob; 0 = k_la_kv + k_la_reduce)
#define EGG_LA_FOLD 1
#endif

// Pass 1 per (image*head, chunk of LA_T tokens) on MFMA: k (ReLU'd) and v staged into LDS token-major
// as bf16 (all 8 loads per thread in flight), then kv^T-free: C[i][j] = sum_n v[n][i] relu(k[n][j]) as
// 16x16x32 bf16 MFMAs with the TOKEN axis as K — both operands need 8 consecutive tokens of one
// feature per lane, which ds_read_b64_tr_b16 (gfx950 transpose read: per 16-lane group a 4-row x
// 16-column block delivered column-major) reads straight from the token-major image.  ksum[j] is one
// more MFMA with a row of ones as A.  Each wave covers 64 tokens (2 K-steps); the 4 waves' partials
// are summed in a fixed order through LDS.  Products of bf16 inputs are exact in fp32, as in the VALU
// form; only the accumulation order differs.
constexpr int LA_RS = LA_D + 8;  // bf16 LDS row stride (80 B: 8-B aligned rows for the transpose reads)
typedef __attribute__((ext_vector_type(4))) short la_s4;
typedef __attribute__((address_space(3))) la_s4 la_lds_s4;

__device__ __forceinline__ la_bf16x8 la_tr8(const unsigned short* base, int lane) {
    // rows base + 8g + {0..3} and {4..7} of the 16-lane group g; lane 4q+p addresses row q, columns 4p..4p+3
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const unsigned short* r0 = base + (8 * g + q) * LA_RS + 4 * p;
    const la_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((la_lds_s4*)(r0));
    const la_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((la_lds_s4*)(r0 + 4 * LA_RS));
    typedef __attribute__((ext_vector_type(8))) short s8;
    const s8 f = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(la_bf16x8, f);
}

// HP = 2 (contiguous heads, hstride == 32, even head count): a block stages one token chunk of a head
// PAIR, so every k / v load covers a whole 128-B line (a token's 64 B of two neighbouring heads) instead
// of relying on the neighbouring head's block to read the other half through L2; each head's MFMAs,
// per-wave token split and partial sums are those of HP = 1 (the same bits).
template <int HP>
__global__ __launch_bounds__(256) void k_la_kv(const unsigned short* __restrict__ k, const unsigned short* __restrict__ v,
                                               int64_t ld, int64_t hstride, int heads, int N, int nchunk, int relu,
                                               float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) unsigned short lds_kv[HP * 2 * LA_T * LA_RS];  // [head] sk | sv, then red
    float(*red)[LA_PART] = reinterpret_cast<float(*)[LA_PART]>(lds_kv);  // [head * 4 + wave], after the MFMAs
    static_assert(HP * 4 * LA_PART * 4 <= HP * 2 * LA_T * LA_RS * 2, "reduction buffer fits in the staging LDS");
    const int lb = xcd_remap(blockIdx.x, gridDim.x);  // adjacent heads share 128-B lines: same L2
    const int bhp = lb / nchunk, c = lb - bhp * nchunk;
    const int hg = heads / HP, b = bhp / hg, h0 = (bhp - b * hg) * HP;
    const int n0 = c * LA_T;
    const int cnt = (N - n0) < LA_T ? (N - n0) : LA_T;
    const int tid = threadIdx.x;
    constexpr int U = 4 * HP;  // 16-B units per token and tensor (HP heads x 64 B)
    u16x8m kr[U], vr[U];
#pragma unroll
    for (int it = 0; it < U; ++it) {  // LA_T tokens x U units per tensor
        const int u = tid + it * 256, t = u / U, q8 = u % U;
        kr[it] = vr[it] = u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
        if (t < cnt) {
            const int64_t off = ((int64_t)b * N + n0 + t) * ld + (int64_t)h0 * hstride + (q8 >> 2) * hstride + (q8 & 3) * 8;
            kr[it] = *reinterpret_cast<const u16x8m*>(k + off);
            vr[it] = *reinterpret_cast<const u16x8m*>(v + off);
        }
    }
#pragma unroll
    for (int it = 0; it < U; ++it) {
        const int u = tid + it * 256, t = u / U, q8 = u % U;
        unsigned short* sk = lds_kv + (q8 >> 2) * (2 * LA_T * LA_RS);
        unsigned short* sv = sk + LA_T * LA_RS;
        if (relu) {
#pragma unroll
            for (int i = 0; i < 8; ++i) kr[it][i] = (kr[it][i] & 0x8000) ? (unsigned short)0 : kr[it][i];  // bf16 ReLU (-0 -> +0)
        }
        *reinterpret_cast<u16x8m*>(sk + t * LA_RS + (q8 & 3) * 8) = kr[it];
        *reinterpret_cast<u16x8m*>(sv + t * LA_RS + (q8 & 3) * 8) = vr[it];
    }
    __syncthreads();
    const int lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
    la_bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (__bf16)(r16 == 0 ? 1.0f : 0.0f);  // A row 0 = ones -> ksum
    la_f32x4 acc[HP][2][2], ks[HP][2];
#pragma unroll
    for (int hh = 0; hh < HP; ++hh)
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            ks[hh][x] = la_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[hh][x][y] = la_f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
    for (int hh = 0; hh < HP; ++hh) {
        const unsigned short* sk = lds_kv + hh * (2 * LA_T * LA_RS);
        const unsigned short* sv = sk + LA_T * LA_RS;
#pragma unroll
        for (int s = 0; s < 2; ++s) {  // this wave's 64 tokens as 2 K-steps of 32
            const int t0 = w * 64 + s * 32;
            la_bf16x8 av[2], bk[2];
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                av[x] = la_tr8(sv + t0 * LA_RS + 16 * x, lane);  // A[i = 16x + r16][n]
                bk[x] = la_tr8(sk + t0 * LA_RS + 16 * x, lane);  // B[n][j = 16x + r16]
            }
#pragma unroll
            for (int x = 0; x < 2; ++x) {
#pragma unroll
                for (int y = 0; y < 2; ++y)
                    acc[hh][x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[x], bk[y], acc[hh][x][y], 0, 0, 0);
                ks[hh][x] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bk[x], ks[hh][x], 0, 0, 0);
            }
        }
    }
    __syncthreads();  // every wave is done reading sk / sv: reuse the staging LDS for the reduction
    // C layout: lane holds C[4g + e][r16]
#pragma unroll
    for (int hh = 0; hh < HP; ++hh) {
        float* rw = red[hh * 4 + w];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int e = 0; e < 4; ++e) rw[(16 * x + 4 * g + e) * LA_D + 16 * y + r16] = acc[hh][x][y][e];
        if (g == 0) {
#pragma unroll
            for (int y = 0; y < 2; ++y) rw[LA_D * LA_D + 16 * y + r16] = ks[hh][y][0];
        }
    }
    __syncthreads();
#pragma unroll
    for (int hh = 0; hh < HP; ++hh) {
        // slot bh * nchunk + c (bh = b * heads + h): k_la_reduce sums chunks in order
        float* dst = part + ((int64_t)b * heads + h0 + hh) * nchunk * LA_PART + (int64_t)c * LA_PART;
        const float(*r4)[LA_PART] = red + hh * 4;
        for (int e = tid; e < LA_PART; e += 256) dst[e] = ((r4[0][e] + r4[1][e]) + r4[2][e]) + r4[3][e];
    }
}

// Round 6: the kv pass with the chunk reduction folded in, for few chunks per head
// (N <= LA_FOLD_MAX * LA_T) on grids large enough to fill the chip with one block per head (group): the block
// walks its head's chunks in order, computes each chunk's partial exactly as k_la_kv does (same MFMAs, same
// ((w0 + w1) + w2) + w3 wave sum), and adds it into a per-thread running sum that starts at 0 as
// k_la_reduce's does — the same additions in the same order, so kvsum is bitwise k_la_kv + k_la_reduce's,
// without the partials' round trip through HBM or the reduce launch.  The next chunk's k / v loads are
// issued as soon as this chunk is in LDS, so they land under its MFMAs and reduction.
constexpr int LA_FOLD_MAX = 4;
template <int HP>
__global__ __launch_bounds__(256) void k_la_kv_fold(const unsigned short* __restrict__ k, const unsigned short* __restrict__ v,
                                                    int64_t ld, int64_t hstride, int heads, int N, int nchunk, int relu,
                                                    float* __restrict__ kvsum) {
    __shared__ __attribute__((aligned(16))) unsigned short lds_kv[HP * 2 * LA_T * LA_RS];
    float(*red)[LA_PART] = reinterpret_cast<float(*)[LA_PART]>(lds_kv);
    static_assert(HP * 4 * LA_PART * 4 <= HP * 2 * LA_T * LA_RS * 2, "reduction buffer fits in the staging LDS");
    constexpr int EPT = (LA_PART + 255) / 256;  // kvsum elements per thread per head
    const int bhp = xcd_remap(blockIdx.x, gridDim.x);
    const int hg = heads / HP, b = bhp / hg, h0 = (bhp - b * hg) * HP;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
    constexpr int U = 4 * HP;
    u16x8m kr[U], vr[U];
    auto load = [&](int c) {
        const int n0 = c * LA_T, cnt = (N - n0) < LA_T ? (N - n0) : LA_T;
#pragma unroll
        for (int it = 0; it < U; ++it) {
            const int u = tid + it * 256, t = u / U, q8 = u % U;
            kr[it] = vr[it] = u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
            if (t < cnt) {
                const int64_t off = ((int64_t)b * N + n0 + t) * ld + (int64_t)h0 * hstride + (q8 >> 2) * hstride + (q8 & 3) * 8;
                kr[it] = *reinterpret_cast<const u16x8m*>(k + off);
                vr[it] = *reinterpret_cast<const u16x8m*>(v + off);
            }
        }
    };
    la_bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (__bf16)(r16 == 0 ? 1.0f : 0.0f);
    float sum[HP][EPT];
#pragma unroll
    for (int hh = 0; hh < HP; ++hh)
#pragma unroll
        for (int q = 0; q < EPT; ++q) sum[hh][q] = 0.f;
    load(0);
#pragma unroll 1
    for (int c = 0; c < nchunk; ++c) {
        if (c > 0) __syncthreads();  // every thread is done reading the previous chunk's reduction table
#pragma unroll
        for (int it = 0; it < U; ++it) {
            const int u = tid + it * 256, t = u / U, q8 = u % U;
            unsigned short* sk = lds_kv + (q8 >> 2) * (2 * LA_T * LA_RS);
            unsigned short* sv = sk + LA_T * LA_RS;
            if (relu) {
#pragma unroll
                for (int i = 0; i < 8; ++i) kr[it][i] = (kr[it][i] & 0x8000) ? (unsigned short)0 : kr[it][i];
            }
            *reinterpret_cast<u16x8m*>(sk + t * LA_RS + (q8 & 3) * 8) = kr[it];
            *reinterpret_cast<u16x8m*>(sv + t * LA_RS + (q8 & 3) * 8) = vr[it];
        }
        if (c + 1 < nchunk) load(c + 1);  // in flight under this chunk's MFMAs
        __syncthreads();
        la_f32x4 acc[HP][2][2], ks[HP][2];
#pragma unroll
        for (int hh = 0; hh < HP; ++hh)
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                ks[hh][x] = la_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[hh][x][y] = la_f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
        for (int hh = 0; hh < HP; ++hh) {
            const unsigned short* sk = lds_kv + hh * (2 * LA_T * LA_RS);
            const unsigned short* sv = sk + LA_T * LA_RS;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int t0 = w * 64 + s * 32;
                la_bf16x8 av[2], bk[2];
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    av[x] = la_tr8(sv + t0 * LA_RS + 16 * x, lane);
                    bk[x] = la_tr8(sk + t0 * LA_RS + 16 * x, lane);
                }
#pragma unroll
                for (int x = 0; x < 2; ++x) {
#pragma unroll
                    for (int y = 0; y < 2; ++y)
                        acc[hh][x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[x], bk[y], acc[hh][x][y], 0, 0, 0);
                    ks[hh][x] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bk[x], ks[hh][x], 0, 0, 0);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int hh = 0; hh < HP; ++hh) {
            float* rw = red[hh * 4 + w];
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int e = 0; e < 4; ++e) rw[(16 * x + 4 * g + e) * LA_D + 16 * y + r16] = acc[hh][x][y][e];
            if (g == 0) {
#pragma unroll
                for (int y = 0; y < 2; ++y) rw[LA_D * LA_D + 16 * y + r16] = ks[hh][y][0];
            }
        }
        __syncthreads();
#pragma unroll
        for (int hh = 0; hh < HP; ++hh) {
            const float(*r4)[LA_PART] = red + hh * 4;
#pragma unroll
            for (int q = 0; q < EPT; ++q) {
                const int e = tid + 256 * q;
                if (e < LA_PART) sum[hh][q] += ((r4[0][e] + r4[1][e]) + r4[2][e]) + r4[3][e];
            }
        }
    }
#pragma unroll
    for (int hh = 0; hh < HP; ++hh) {
        float* dst = kvsum + ((int64_t)b * heads + h0 + hh) * LA_PART;
#pragma unroll
        for (int q = 0; q < EPT; ++q) {
            const int e = tid + 256 * q;
            if (e < LA_PART) dst[e] = sum[hh][q];
        }
    }
}

// Fixed-order sum of the nchunk partials of one (image, head) -> kvsum[bh], once per head: the
// k_la_out blocks then read 4 KiB each instead of every block re-summing all nchunk partials
// (O(nchunk) instead of O(nchunk^2) partial reads: 64 chunks per head at DC-AE's 128x128 stage).
__global__ __launch_bounds__(256) void k_la_reduce(const float* __restrict__ part, int nchunk,
                                                   float* __restrict__ kvsum) {
    const int64_t bh = blockIdx.x;
    const float* src = part + bh * nchunk * LA_PART;
    for (int e = threadIdx.x; e < LA_PART; e += 256) {
        float s = 0.f;
        int cc = 0;
        for (; cc + 8 <= nchunk; cc += 8) {  // 8 loads in flight, summed in chunk order
            float p[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) p[u] = src[(int64_t)(cc + u) * LA_PART + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += p[u];
        }
        for (; cc < nchunk; ++cc) s += src[(int64_t)cc * LA_PART + e];
        kvsum[bh * LA_PART + e] = s;
    }
}

// Many chunks (>= LA_RED_WIDE, DC-AE's 64^2 and 128^2 maps): one thread per element, one wave per 64
// elements (17 waves per head), a thread's partials loaded 16 at a time and summed in the same chunk
// order (bit-identical to k_la_reduce, which walks ~4 elements per thread one after another: 8 B x
// 16 K x 16 heads 0.226 -> 0.214 ms for the whole attention; at 4 chunks the 17x more workgroups cost
// more than they save)
constexpr int LA_RED_WAVES = (LA_PART + 63) / 64;
constexpr int LA_RED_WIDE = 16;
__global__ __launch_bounds__(64) void k_la_reduce_e(const float* __restrict__ part, int nchunk,
                                                    float* __restrict__ kvsum) {
    const int64_t bh = blockIdx.x / LA_RED_WAVES;
    const int e = (blockIdx.x % LA_RED_WAVES) * 64 + threadIdx.x;
    if (e >= LA_PART) return;
    const float* src = part + bh * nchunk * LA_PART + e;
    float s = 0.f;
    int cc = 0;
    for (; cc + 16 <= nchunk; cc += 16) {  // 16 loads in flight, summed in chunk order
        float p[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) p[u] = src[(int64_t)(cc + u) * LA_PART];
#pragma unroll
        for (int u = 0; u < 16; ++u) s += p[u];
    }
    for (; cc < nchunk; ++cc) s += src[(int64_t)cc * LA_PART];
    kvsum[bh * LA_PART + e] = s;
}

// Pass 3 on MFMA: out^T[i][t] = sum_j kv[i][j] relu(q[t][j]) as 16x16x32 bf16 MFMAs with kv as the A
// operand (row i, 8 consecutive j per lane — the natural [i][j] layout) and 16 tokens' q as the B
// operand (each lane's 16-B load is 8 consecutive features of one token), so the accumulator lane
// holds 4 consecutive output features of one token (one 8-byte store).  kv (fp32) enters as a bf16
// hi + lo pair (two MFMAs: ~2^-16 relative, fp32-class), and the denominator relu(q) . ksum is one
// more hi/lo MFMA pair with ksum as row 0 of a 16-row A tile.  The VALU form spent 1056 FMAs + as many
// LDS broadcast reads per token-head; this one is 6 MFMAs per 16 tokens and memory-bound.

__device__ __forceinline__ void la_split8(const float (&f)[8], la_bf16x8& hi, la_bf16x8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const __bf16 h = (__bf16)f[e];
        hi[e] = h;
        lo[e] = (__bf16)(f[e] - (float)h);
    }
}

// Round 5: the denominator row ksum is written into A rows 0, 4, 8 and 12 (each lane group g then holds
// den of its own token r16 as C[4g][r16] — the shuffle that broadcast row 0 is gone), a wave covers
// TPW tiles of 16 tokens (the kv hi/lo split amortised over twice the tokens, twice the q loads in
// flight), and q / out go through buffer descriptors (one per image, head offset in the base: 32-bit
// offsets, tokens past N out of range).  Same MFMAs, same operands: the same bits.
// TPW: 16-token tiles per wave (8; 16 at the DC-AE's 128^2 maps: 166 -> 154 us, r10c); HP = 2: a head
// pair per block as in k_la_kv (each q load / output row a whole 128-B line), per-head math unchanged.
template <int HP, int TPW>
__global__ __launch_bounds__(256) void k_la_out(const unsigned short* __restrict__ q, int64_t ld, int64_t hstride,
                                                int heads, int N, int nblk_tok, int relu, const float* __restrict__ kvsum,
                                                unsigned short* __restrict__ out, int64_t ldo) {
    constexpr int T = 4 * TPW * 16;  // tokens per block
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int bhp = lb / nblk_tok, c = lb - bhp * nblk_tok;
    const int hg = heads / HP, b = bhp / hg, h0 = (bhp - b * hg) * HP;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r16 = lane & 15, g = lane >> 4;
    const int n0 = c * T + wave * (T / 4);
    // q tiles first (the longest latency), then kv from L2
    constexpr uint32_t OOR = 0x80000000u;
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(q + (int64_t)b * N * ld + (int64_t)h0 * hstride), (short)0, (int)((int64_t)N * ld * 2), 0x00020000);
    u16x8m qr[TPW][HP];
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
        const int tok = n0 + tt * 16 + r16;
#pragma unroll
        for (int hh = 0; hh < HP; ++hh) {
            const uint32_t off = tok < N ? ((uint32_t)tok * (uint32_t)ld + (uint32_t)(hh * hstride) + 8 * g) * 2 : OOR;
            qr[tt][hh] = __builtin_bit_cast(u16x8m, __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, 0));
        }
    }
    la_bf16x8 akv[HP][2][2], aden[HP][2];  // [head][feature block][hi, lo]
#pragma unroll
    for (int hh = 0; hh < HP; ++hh) {
        const float* kvh = kvsum + ((int64_t)b * heads + h0 + hh) * LA_PART;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
            const float4 x0 = *reinterpret_cast<const float4*>(kvh + (16 * cb + r16) * LA_D + 8 * g);
            const float4 x1 = *reinterpret_cast<const float4*>(kvh + (16 * cb + r16) * LA_D + 8 * g + 4);
            const float f[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            la_split8(f, akv[hh][cb][0], akv[hh][cb][1]);
        }
        float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if ((r16 & 3) == 0) {  // A rows 0, 4, 8, 12 = ksum, the rest 0
            const float4 x0 = *reinterpret_cast<const float4*>(kvh + LA_D * LA_D + 8 * g);
            const float4 x1 = *reinterpret_cast<const float4*>(kvh + LA_D * LA_D + 8 * g + 4);
            f[0] = x0.x; f[1] = x0.y; f[2] = x0.z; f[3] = x0.w;
            f[4] = x1.x; f[5] = x1.y; f[6] = x1.z; f[7] = x1.w;
        }
        la_split8(f, aden[hh][0], aden[hh][1]);
    }
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(out + (int64_t)b * N * ldo + h0 * LA_D), (short)0, (int)((int64_t)N * ldo * 2), 0x00020000);
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
        const int tok = n0 + tt * 16 + r16;
#pragma unroll
        for (int hh = 0; hh < HP; ++hh) {
            u16x8m qv = qr[tt][hh];
            if (relu) {
#pragma unroll
                for (int e = 0; e < 8; ++e) qv[e] = (qv[e] & 0x8000) ? (unsigned short)0 : qv[e];  // bf16 ReLU
            }
            const la_bf16x8 bq = *reinterpret_cast<const la_bf16x8*>(&qv);
            la_f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, ad = a0;
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(akv[hh][0][0], bq, a0, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(akv[hh][0][1], bq, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(akv[hh][1][0], bq, a1, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(akv[hh][1][1], bq, a1, 0, 0, 0);
            ad = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aden[hh][0], bq, ad, 0, 0, 0);
            ad = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aden[hh][1], bq, ad, 0, 0, 0);
            const float inv = 1.0f / (ad[0] + 1e-15f);  // C[4g][r16] = den of token r16 in every lane group
            const uint32_t off = tok < N ? ((uint32_t)tok * (uint32_t)ldo + (uint32_t)(hh * LA_D) + 4 * g) * 2 : OOR;
            u16x4m o0, o1;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o0[e] = f2b(a0[e] * inv);
                o1[e] = f2b(a1[e] * inv);
            }
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2m, o0), ro, off, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2m, o1), ro, off + 32, 0, 0);
        }
    }
}

// ------------------------------------------------------------------------------------
// DC-AE decoder head, fused: y[p, o] = cb[o] + sum_{tap, c} a[p + tap, c] * Wc[o, tap, c]  (3x3, pad 1)
// with a = bf16(relu(rms_norm(x) * w + b)) (norm_out + ReLU + conv_out of the reference decoder).
// The unfused pair was a rownorm pass over x plus MIOpen's 128 -> 3 channel conv, which ran at 16 TF
// (3.6 ms per 8-image decode, reading 2 GB at 0.6 TB/s).  Block = 8 x 16 output pixels: the
// 10 x 18-pixel halo tile of x is loaded with every 16-B load in flight, RMS-normalised per pixel
// (16-lane shuffle reduction over 128 channels), written to LDS as bf16; then 36 MFMA k-steps
// (9 taps x 4 x 32 channels) of 16 pixels x 16 outputs (3 real) per output row.  HBM: x read once
// (+halo L2 hits), y written once — the conv is ~free on MFMA.  Round 4: a block walks EGG_HEAD_TPB
// bands down its tile column with the next band's loads in flight under the current band's conv:
// 1217 -> 1014 us at 8 x 1024^2 x 128, bitwise equal (profiles/r07i_dcae_head_band_walk_ab.jsonl).
// ------------------------------------------------------------------------------------
constexpr int HD_C = 128;                // input channels (the decoder's widths[0])
#ifndef EGG_HEAD_TPB
#define EGG_HEAD_TPB 8                   // output bands walked per block (A/B knob; 1 = the round-2 form)
#endif
constexpr int HD_TH = 8, HD_TW = 16;     // output tile
constexpr int HD_TR = HD_TH + 2, HD_TC = HD_TW + 2;
constexpr int HD_PSTR = HD_C * 2;        // LDS bytes per staged pixel: 16-B chunk c of pixel p sits at slot
                                         // c ^ (p & 15) (conflict-free b128 reads of 16 pixels, no padding:
                                         // 53 KB per block -> 3 blocks per CU instead of 2)
__device__ __forceinline__ int hd_slot(int pix, int c) { return pix * HD_PSTR + ((c ^ (pix & 15)) << 4); }

typedef __attribute__((ext_vector_type(8))) __bf16 hd_bf16x8;
typedef __attribute__((ext_vector_type(4))) float hd_f32x4;

__global__ __launch_bounds__(256, 3) void k_dcae_head(const unsigned short* __restrict__ x, int H, int W, float eps,
                                                   const unsigned short* __restrict__ nw,
                                                   const unsigned short* __restrict__ nb,
                                                   const unsigned short* __restrict__ wc,   // [3][3][3][C]
                                                   const unsigned short* __restrict__ cb,   // [3] or null
                                                   int xtiles, int bands, int tpb, unsigned short* __restrict__ y) {
    __shared__ __attribute__((aligned(16))) char tile[HD_TR * HD_TC * HD_PSTR];
    __shared__ __attribute__((aligned(16))) unsigned short wl[3 * 9 * HD_C];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-contiguous tile ranges: horizontally adjacent tiles (sharing 2 halo columns) on one L2.  A block
    // walks tpb bands down its tile column; the next band's halo loads are issued as soon as the current
    // band's raw values have been normalised into LDS, so they are in flight during its conv and stores
    // (the one-band form waited a full memory latency per tile with only 3 blocks per CU to cover it)
    const int bgroups = (bands + tpb - 1) / tpb;
    int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int xt = bid % xtiles;
    bid /= xtiles;
    const int bg = bid % bgroups;
    const int b = bid / bgroups;
    const int band_lo = bg * tpb, band_hi = min(bands, band_lo + tpb);
    const int x0 = xt * HD_TW;
    const char* img = reinterpret_cast<const char*>(x + (int64_t)b * H * W * HD_C);
    const uint32_t rowb = (uint32_t)W * HD_PSTR;
    // conv weights -> LDS (6.75 KiB), once per block
    for (int u = tid; u < 3 * 9 * HD_C / 8; u += 256)
        *reinterpret_cast<u16x8m*>(wl + u * 8) = *reinterpret_cast<const u16x8m*>(wc + u * 8);
    // Halo tile staging with buffer descriptors (round 5; the per-unit pixel division and 64-bit address
    // arithmetic of the previous form made this kernel VALU-issue-bound, profiles/r09d_epoch_census.txt).
    // Thread = (main column mc, 16-B chunk ch): the 16 main columns (tx 1..16) of every halo row, one row
    // descriptor per row (size 0 outside the image: zero rows), a column past W an out-of-range offset;
    // the 2 halo columns (tx 0, 17) x 10 rows x 16 chunks = 320 units take one or two indexed loads.  A
    // pixel's 16 chunks stay 16 consecutive lanes (its sum of squares is a 16-lane shuffle reduction).
    constexpr uint32_t OOR = 0x80000000u;
    const int ch = tid & 15, mc = tid >> 4;
    const bool mcol_ok = x0 + mc < W;
    const uint32_t mvoff = mcol_ok ? (uint32_t)(x0 + mc) * HD_PSTR + ch * 16 : OOR;
    constexpr int HU = HD_TR * 2 * 16, HPER = (HU + 255) / 256;   // 320 halo-column units
    u16x8m v[HD_TR], hv[HPER];
    bool hok[HPER];
    const __amdgpu_buffer_rsrc_t rimg = __builtin_amdgcn_make_buffer_rsrc((void*)img, (short)0, (int)(H * rowb),
                                                                          0x00020000);
    // halo-column unit k of rows rlo..HD_TR-1: row rlo + (hp >> 1), column 0 or 17
    auto hunit = [&](int k, int rlo, int& ty, int& tx) {
        const int u = tid + k * 256, hp = u >> 4;
        ty = rlo + (hp >> 1);
        tx = (hp & 1) ? HD_TC - 1 : 0;
        return u < (HD_TR - rlo) * 32;
    };
    // rows rlo..HD_TR-1 of the halo tile whose first row is image row y0 - 1 (rlo = 0: a block's first
    // band; 2: a later band, whose rows 0, 1 are the previous band's rows 8, 9, already in LDS)
    auto load = [&](int y0, int rlo) {
#pragma unroll
        for (int r = 0; r < HD_TR; ++r) {
            if (r < rlo) continue;
            const int gy = y0 + r - 1;
            const bool ok = gy >= 0 && gy < H;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(img + (int64_t)(ok ? gy : 0) * rowb), (short)0, ok ? (int)rowb : 0, 0x00020000);
            v[r] = __builtin_bit_cast(u16x8m, __builtin_amdgcn_raw_buffer_load_b128(rs, mvoff, 0, 0));
        }
#pragma unroll
        for (int k = 0; k < HPER; ++k) {
            int ty, tx;
            const bool in = hunit(k, rlo, ty, tx);
            const int gy = y0 + ty - 1, gx = x0 + tx - 1;
            hok[k] = in && gy >= 0 && gy < H && gx >= 0 && gx < W;
            const uint32_t off = hok[k] ? (uint32_t)(gy * W + gx) * HD_PSTR + ch * 16 : OOR;
            hv[k] = __builtin_bit_cast(u16x8m, __builtin_amdgcn_raw_buffer_load_b128(rimg, off, 0, 0));
        }
    };
    float wv[8], bv[8];
    {
        const u16x8m qw = *reinterpret_cast<const u16x8m*>(nw + ch * 8);
        const u16x8m qb = *reinterpret_cast<const u16x8m*>(nb + ch * 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) { wv[i] = b2f(qw[i]); bv[i] = b2f(qb[i]); }
    }
    // RMS-normalise one 16-B unit (8 channels of one pixel), affine, ReLU, bf16; zero where the halo pixel
    // is outside the image.  (f * rstd) * w + b per value as before: the packed pairs round each product
    // and sum exactly like the scalar ops, so the tile is bitwise unchanged.
    typedef __attribute__((ext_vector_type(2))) float f2;
    auto norm = [&](const u16x8m& q, bool ok) {
        float f[8], ss = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) { f[i] = b2f(q[i]); ss += f[i] * f[i]; }
        ss = seg_sum<16>(ss);
        const float rstd = __builtin_amdgcn_rsqf(ss / HD_C + eps);  // >= eps: never denormal
        u16x8m o8 = {0, 0, 0, 0, 0, 0, 0, 0};
        if (ok) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                f2 t = f2{f[i], f[i + 1]} * f2{rstd, rstd};
                t = t * f2{wv[i], wv[i + 1]};
                t = t + f2{bv[i], bv[i + 1]};
                o8[i] = f2b(t.x > 0.f ? t.x : 0.f);
                o8[i + 1] = f2b(t.y > 0.f ? t.y : 0.f);
            }
        }
        return o8;
    };
    const int n = lane & 15, g = lane >> 4;
    const float bias = (n < 3 && cb) ? b2f(cb[n]) : 0.f;
    // B operand column n = output channel n; columns 3..15 are computed and never stored, so their lanes
    // read a real channel's weights (no zero row, no branch: 52.9 KB of LDS, 3 blocks per CU)
    const int wrow = (n % 3) * 9 * HD_C + g * 8;
    // Rolling rows: tile row r of the j-th band a block walks sits in LDS row slot (8j + r) mod 10, so the
    // two rows a band shares with the next (its rows 8, 9 = the next band's rows 0, 1) are loaded and
    // normalised once (10 -> 8 rows per band after the first).
    auto slot = [](int j8, int r) { const int q = j8 + r; return q >= HD_TR ? q - HD_TR : q; };
    load(band_lo * HD_TH, 0);
    int j8 = 0;  // 8j mod 10
#pragma unroll 1
    for (int band = band_lo; band < band_hi; ++band) {
        const int y0 = band * HD_TH;
        const int rlo = band > band_lo ? 2 : 0;
        if (band > band_lo) __syncthreads();  // every wave's conv reads of the previous band are done
#pragma unroll
        for (int r = 0; r < HD_TR; ++r) {
            if (r < rlo) continue;
            const int gy = y0 + r - 1;
            const u16x8m o8 = norm(v[r], mcol_ok && gy >= 0 && gy < H);
            *reinterpret_cast<u16x8m*>(tile + hd_slot(slot(j8, r) * HD_TC + 1 + mc, ch)) = o8;
        }
#pragma unroll
        for (int k = 0; k < HPER; ++k) {
            int ty, tx;
            const bool in = hunit(k, rlo, ty, tx);
            const u16x8m o8 = norm(hv[k], hok[k]);
            if (in) *reinterpret_cast<u16x8m*>(tile + hd_slot(slot(j8, ty) * HD_TC + tx, ch)) = o8;
        }
        if (band + 1 < band_hi) load(y0 + HD_TH, 2);
        // conv A-fragment addresses: hd_slot(pix, cq*4 + g) = hd_slot(pix, g) ^ (cq << 6) (the chunk's low
        // two bits are g, cq only flips bits 2..3 of the slot): one base per (output row, tap), a XOR per k-step
        uint32_t abase[2][9];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
                abase[r][tap] = (uint32_t)hd_slot(slot(j8, wave * 2 + r + tap / 3) * HD_TC + n + tap % 3, g);
        __syncthreads();
        // conv: wave w computes output rows 2w, 2w+1 (one 16-pixel M-tile each)
        hd_f32x4 acc[2] = {hd_f32x4{0.f, 0.f, 0.f, 0.f}, hd_f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < 36; ++s) {
            const int tap = s >> 2, cq = s & 3;
            const hd_bf16x8 bf = *reinterpret_cast<const hd_bf16x8*>(wl + wrow + tap * HD_C + cq * 32);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const hd_bf16x8 af = *reinterpret_cast<const hd_bf16x8*>(tile + (abase[r][tap] ^ (uint32_t)(cq << 6)));
                acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[r], 0, 0, 0);
            }
        }
        // C[m = pixel 4g + e][col = output channel n]
        if (n < 3) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int yy = y0 + wave * 2 + r;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int xx = x0 + 4 * g + e;
                    if (yy < H && xx < W) y[(((int64_t)b * H + yy) * W + xx) * 3 + n] = f2b(acc[r][e] + bias);
                }
            }
        }
        j8 = slot(j8, HD_TH);
    }
}

}  // namespace eggroll

using namespace eggroll;

// ------------------------------------------------------------------------------------
// CLIP image preprocessing, bit-exact with transformers' CLIPImageProcessor (PIL backend) on the
// PIL image the reference would build from the decoder output (rewards.py:86-90, 133-147):
//   u8 = PixArt postprocess (mode 0: rint((x/2 + 0.5).clamp(0,1) * 255), Sana) or the VAR PIL
//        path (mode 1: fp16 ((x+1)*0.5).clamp(0,1) * 255 truncated, models/VAR.py:190, 245-259) or
//        Infinity's (mode 2: bf16 (x+1)/2*255 truncated);
//   Pillow BICUBIC resize in 8-bit fixed point (Resample.c: int32 taps of 22 fractional bits,
//   horizontal pass first, each pass rounded + clipped to 8 bits), center crop, then
//   (u8 / 255 - mean[c]) / std[c] in fp32 (IEEE division, as torch).
// Tap tables (host-built from Pillow's precompute_coeffs): int32 [out][1 + KT] = {first input
// index, KT weights (zero beyond the filter's support)}.  Pass 1 writes the horizontally resized
// rows of the crop's columns as uint8 [n][3][H][OW]; pass 2 the normalised [n][3][OH][OW] fp32.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int clip_u8_of(float x, int mode) {
    if (mode == 0) {
        float v = fminf(fmaxf(x * 0.5f + 0.5f, 0.0f), 1.0f);
        return (int)rintf(v * 255.0f);
    }
    if (mode == 2) {
        // Infinity (models/Infinity.py img postprocess under bf16 autocast): (x + 1) / 2 * 255, every op
        // rounded to bf16, clamped (the decoder output is in [-1, 1]), .to(uint8) truncates
        auto r = [](float v) { return b2f(f2b(v)); };
        float v = r(r(r(x + 1.0f) * 0.5f) * 255.0f);
        v = fminf(fmaxf(v, 0.0f), 255.0f);
        return (int)v;
    }
    // fp16 arithmetic of the reference's autocast output: every op rounded to half
    _Float16 h = (_Float16)x;
    h = (_Float16)(h + (_Float16)1.0f);
    h = (_Float16)(h * (_Float16)0.5f);
    h = h < (_Float16)0.0f ? (_Float16)0.0f : (h > (_Float16)1.0f ? (_Float16)1.0f : h);
    h = (_Float16)(h * (_Float16)255.0f);
    return (int)(float)h;  // .to(torch.uint8) truncates toward zero
}

__device__ __forceinline__ int pil_clip8(int ss) {
    ss >>= 22;  // arithmetic shift: floor, as Resample.c's clip8
    return ss < 0 ? 0 : (ss > 255 ? 255 : ss);
}

// Pass 1: one block per input row (image n, row y): the row's 3 x W pixels are converted to uint8
// once into LDS (coalesced loads), then the 3 x OW horizontal taps are summed from LDS.
constexpr int CLIP_MAXW = 4096;
__global__ __launch_bounds__(256) void k_clip_resize_h(const unsigned short* __restrict__ img, int64_t sn, int64_t sc,
                                                       int64_t sh, int64_t sw, int H, int W, int OW, int left,
                                                       int mode, const int* __restrict__ tab, int KT,
                                                       unsigned char* __restrict__ tmp) {
    __shared__ unsigned char row[3 * CLIP_MAXW];
    const int64_t n = blockIdx.x / H;
    const int y = (int)(blockIdx.x - n * H);
    const unsigned short* src = img + n * sn + (int64_t)y * sh;
    for (int t = threadIdx.x; t < 3 * W; t += 256) {
        const int x = t / 3, c = t - 3 * x;
        row[c * W + x] = (unsigned char)clip_u8_of(b2f(src[c * sc + (int64_t)x * sw]), mode);
    }
    __syncthreads();
    for (int o = threadIdx.x; o < 3 * OW; o += 256) {
        const int c = o / OW, xo = o - c * OW;
        const int* t = tab + (int64_t)(left + xo) * (KT + 1);
        const unsigned char* r = row + c * W + t[0];
        int ss = 1 << 21;
        for (int k = 0; k < KT; ++k) ss += (int)r[k] * t[1 + k];
        tmp[((n * 3 + c) * H + y) * OW + xo] = (unsigned char)pil_clip8(ss);
    }
}

__global__ __launch_bounds__(256) void k_clip_resize_v(const unsigned char* __restrict__ tmp, int H, int OW, int OH,
                                                       int top, const int* __restrict__ tab, int KT, float m0,
                                                       float m1, float m2, float s0, float s1, float s2,
                                                       int64_t total, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int xo = (int)(i % OW);
    int64_t r = i / OW;                    // (n, c, yo)
    const int yo = (int)(r % OH);
    const int64_t nc = r / OH;
    const int c = (int)(nc % 3);
    const int* t = tab + (int64_t)(top + yo) * (KT + 1);
    const int y0 = t[0];
    const unsigned char* col = tmp + nc * H * OW + xo;
    int ss = 1 << 21;
    for (int k = 0; k < KT; ++k) {
        const int w = t[1 + k];
        if (w != 0) ss += (int)col[(int64_t)(y0 + k) * OW] * w;
    }
    const float v = (float)pil_clip8(ss) / 255.0f;
    const float m = c == 0 ? m0 : (c == 1 ? m1 : m2), sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
    out[i] = (v - m) / sd;
}

// ------------------------------------------------------------------------------------
// Softmax cross-attention over a short key sequence (Sana attn2: 300 caption tokens, head dim 112),
// diffusers SanaAttnProcessor2_0 / F.scaled_dot_product_attention(q, k, v, attn_mask=bias, scale):
//   o[b, n, h, :] = softmax_j(scale * q[b,n,h,:] . k[u,j,h,:] + bias[u, j]) @ v[u, :, h, :],
//   u = enc_index[b] (the image's caption row: images of one prompt share k / v).
// One workgroup per (image, head): the caption's k and v ([L <= 320][112] bf16 each) are staged in
// LDS once and the 8 waves sweep the image's queries in blocks of 16.  Per block, on MFMA
// 16x16x32 bf16 with fp32 accumulation:
//   S^T = K Q^T   A = k rows (16 keys x 32 dims, 16-B LDS reads), B = q rows (16-B global reads);
//                 the C layout leaves each lane 4 consecutive keys of ONE query, so the softmax max /
//                 sum per query reduce over the lane's registers and the 4 lane groups (xor 16, 32);
//   O^T = V^T P^T B = exp(S^T - max) packed straight from the C registers: lane group g holds keys
//                 4g..4g+3 of each 16-key fragment, so a 32-key k-step uses the key order
//                 {4g..4g+3, 16+4g..16+4g+3} per group — A (V^T) reads exactly that order from the
//                 key-major V tile with ds_read_tr16_b64 (no data movement for P);
//   o = O / rowsum, written as 4 consecutive dims of one query per lane (8-B stores) in the q layout.
// Keys past L are excluded (-inf); the additive bias is the reference's attention mask.
// ------------------------------------------------------------------------------------
#ifndef EGG_XA_PREFETCH
#define EGG_XA_PREFETCH 1
#endif
constexpr int XA_LMAX = 320;          // keys per (caption, head) staged in LDS
constexpr int XA_LMAX_128 = 256;      // the same at head dim 128 (2 x 256 x 136 x 2 B of k / v)

template <int RS>
__device__ __forceinline__ la_bf16x8 xa_tr8_perm(const unsigned short* base, int lane) {
    // rows base + 4g + {0..3} and base + 16 + 4g + {0..3} of the 16-lane group g (lane 4q+p: row q, columns 4p..)
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const unsigned short* r0 = base + (4 * g + q) * RS + 4 * p;
    const la_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((la_lds_s4*)(r0));
    const la_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((la_lds_s4*)(r0 + 16 * RS));
    typedef __attribute__((ext_vector_type(8))) short s8;
    const s8 f = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(la_bf16x8, f);
}

// k / v rows of caption u, head h -> LDS (row stride HD + 8), rows >= L zero.  Every load of the thread
// is issued before the first store: the strided loop this replaces waited for each 16-B pair in turn (one
// memory latency per trip, ~9 trips with one workgroup per CU and nothing to overlap them).
template <int HD, int LM, int NT>
__device__ __forceinline__ void xa_stage_kv(const unsigned short* __restrict__ k, const unsigned short* __restrict__ v,
                                            int64_t ldkv, int u, int h, int L, int tid, unsigned short* sk,
                                            unsigned short* sv) {
    constexpr int RS = HD + 8, CH = HD / 8, NCH = LM * CH, IT = (NCH + NT - 1) / NT;
    u16x8m kr[IT], vr[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int c = tid + it * NT, r = c / CH, cc = c - r * CH;
        kr[it] = vr[it] = u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
        if (c < NCH && r < L) {
            const int64_t off = ((int64_t)u * L + r) * ldkv + (int64_t)h * HD + cc * 8;
            kr[it] = *reinterpret_cast<const u16x8m*>(k + off);
            vr[it] = *reinterpret_cast<const u16x8m*>(v + off);
        }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int c = tid + it * NT, r = c / CH, cc = c - r * CH;
        if (NCH % NT == 0 || c < NCH) {
            *reinterpret_cast<u16x8m*>(sk + r * RS + cc * 8) = kr[it];
            *reinterpret_cast<u16x8m*>(sv + r * RS + cc * 8) = vr[it];
        }
    }
}

template <int HD, int NWAVE, int QF, int LM = XA_LMAX>
__global__ __launch_bounds__(64 * NWAVE) void k_cross_attn(const unsigned short* __restrict__ q, int64_t ldq,
                                                    const unsigned short* __restrict__ k,
                                                    const unsigned short* __restrict__ v, int64_t ldkv,
                                                    const unsigned short* __restrict__ bias,
                                                    const int* __restrict__ enc_index, int heads, int N, int L,
                                                    int U, float scale, unsigned short* __restrict__ o, int64_t ldo) {
    // NWAVE waves sweep the image's queries in blocks of 16 * QF (QF query fragments share every k / v
    // fragment read from LDS)
    constexpr int RS = HD + 8, KSN = (HD + 31) / 32, DF = HD / 16;  // LDS row stride, Q.K k-steps, PV dim frags
    static_assert(HD % 16 == 0 && HD <= 128 && LM % 32 == 0, "head dim / key capacity");
    __shared__ __attribute__((aligned(16))) unsigned short sk[LM * RS];
    __shared__ __attribute__((aligned(16))) unsigned short sv[LM * RS];
    __shared__ float sb[LM];
    constexpr int NT = 64 * NWAVE;
    const int bh = xcd_remap(blockIdx.x, gridDim.x);
    const int b = bh / heads, h = bh - b * heads;
    const int u_in = enc_index ? enc_index[b] : b;
    const bool u_bad = u_in < 0 || u_in >= U;  // out-of-range caption row: NaN output, no out-of-bounds read
    const int u = u_bad ? 0 : u_in;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
    // stage k / v rows of caption u, head h: HD / 8 chunks of 16 B per row; rows >= L are zeros
    xa_stage_kv<HD, LM, NT>(k, v, ldkv, u, h, L, tid, sk, sv);
    for (int r = tid; r < LM; r += NT)
        sb[r] = u_bad ? __builtin_nanf("") : r < L ? (bias ? b2f(bias[(int64_t)u * L + r]) : 0.0f) : -INFINITY;
    __syncthreads();
    const int nkf = (L + 15) / 16, nkb = (L + 31) / 32;  // key fragments / 32-key PV steps in use
    const int nqb = (N + 16 * QF - 1) / (16 * QF);
    // B = Q^T fragments for the 4 k-steps (dims 32ks + 8g .. +7; dims >= 112 are zero).  EGG_XA_PREFETCH:
    // the next block's q fragments are loaded right after this block's S^T MFMAs are issued, so their
    // global-load latency runs under the softmax and PV instead of opening the next block.
    auto load_q = [&](int qb_, la_bf16x8 (&dst)[QF][KSN]) {
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            const int qrow = qb_ * 16 * QF + 16 * x + r16;
#pragma unroll
            for (int ks = 0; ks < KSN; ++ks) {
                const int d0 = 32 * ks + 8 * g;
                u16x8m t = u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
                if (d0 < HD && qrow < N)
                    t = *reinterpret_cast<const u16x8m*>(q + ((int64_t)b * N + qrow) * ldq + (int64_t)h * HD + d0);
                dst[x][ks] = __builtin_bit_cast(la_bf16x8, t);
            }
        }
    };
    la_bf16x8 bq[QF][KSN], bqn[QF][KSN];
    if (EGG_XA_PREFETCH && w < nqb) load_q(w, bqn);
    for (int qb = w; qb < nqb; qb += NWAVE) {
        if (EGG_XA_PREFETCH) {
#pragma unroll
            for (int x = 0; x < QF; ++x)
#pragma unroll
                for (int ks = 0; ks < KSN; ++ks) bq[x][ks] = bqn[x][ks];
        } else {
            load_q(qb, bq);
        }
        // S^T[key][query] for every key fragment
        la_f32x4 sf[QF][(LM / 16)];
        float mx[QF];
#pragma unroll
        for (int x = 0; x < QF; ++x) mx[x] = -INFINITY;
#pragma unroll
        for (int f = 0; f < (LM / 16); ++f) {
#pragma unroll
            for (int x = 0; x < QF; ++x) sf[x][f] = la_f32x4{0.f, 0.f, 0.f, 0.f};
            if (f < nkf) {
#pragma unroll
                for (int ks = 0; ks < KSN; ++ks) {
                    const int d0 = 32 * ks + 8 * g;
                    la_bf16x8 a;
                    if (d0 < HD) a = *reinterpret_cast<const la_bf16x8*>(sk + (16 * f + r16) * RS + d0);
                    else a = la_bf16x8{};
#pragma unroll
                    for (int x = 0; x < QF; ++x) sf[x][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[x][ks], sf[x][f], 0, 0, 0);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float bb = sb[16 * f + 4 * g + e];
#pragma unroll
                    for (int x = 0; x < QF; ++x) {
                        const float sv_ = sf[x][f][e] * scale + bb;
                        sf[x][f][e] = sv_;
                        mx[x] = fmaxf(mx[x], sv_);
                    }
                }
            }
        }
        if (EGG_XA_PREFETCH && qb + NWAVE < nqb) load_q(qb + NWAVE, bqn);
        float sum[QF];
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            mx[x] = g4_max(mx[x]);
            sum[x] = 0.0f;
        }
#pragma unroll
        for (int f = 0; f < (LM / 16); ++f) {
            if (f < nkf) {
#pragma unroll
                for (int x = 0; x < QF; ++x)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float pe = __expf(sf[x][f][e] - mx[x]);
                        sf[x][f][e] = pe;
                        sum[x] += pe;
                    }
            }
        }
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            sum[x] = g4_sum(sum[x]);
        }
        // O^T[dim][query] = sum_keys V^T[dim][key] P^T[key][query]
        la_f32x4 oc[QF][DF];
#pragma unroll
        for (int x = 0; x < QF; ++x)
#pragma unroll
            for (int d = 0; d < DF; ++d) oc[x][d] = la_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < (LM / 16) / 2; ++j) {
            if (j < nkb) {
                la_bf16x8 bp[QF];
#pragma unroll
                for (int x = 0; x < QF; ++x)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        bp[x][e] = (__bf16)sf[x][2 * j][e];
                        bp[x][4 + e] = (__bf16)sf[x][2 * j + 1][e];
                    }
#pragma unroll
                for (int d = 0; d < DF; ++d) {
                    const la_bf16x8 av = xa_tr8_perm<RS>(sv + (32 * j) * RS + 16 * d, lane);
#pragma unroll
                    for (int x = 0; x < QF; ++x) oc[x][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bp[x], oc[x][d], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            const int qrow = qb * 16 * QF + 16 * x + r16;
            if (qrow < N) {
                const float inv = 1.0f / sum[x];
                unsigned short* dst = o + ((int64_t)b * N + qrow) * ldo + (int64_t)h * HD + 4 * g;
#pragma unroll
                for (int d = 0; d < DF; ++d) {
                    u16x4m t;
#pragma unroll
                    for (int e = 0; e < 4; ++e) t[e] = f2b(oc[x][d][e] * inv);
                    *reinterpret_cast<u16x4m*>(dst + 16 * d) = t;
                }
            }
        }
    }
}

// Round 5: 32 queries per wave block (QF = 2 query fragments share every k / v fragment read from LDS:
// half the LDS bytes per query, the bound of the 16-query form), with the softmax taken online over two
// key halves so that only half the scores are live in registers (S for 2 x LM/2 keys: the QF = 2
// two-pass form needed 160 score registers and fell to 1 wave per SIMD).  After the first half
// (max m0, P0 = exp(S0 - m0), O = V0^T P0), the second rescales O and the running row sums by
// exp(m0 - m1) before adding its own keys — exact softmax up to fp32 rounding.
template <int HD, int NWAVE, int LM>
__global__ __launch_bounds__(64 * NWAVE) void k_cross_attn_h2(const unsigned short* __restrict__ q, int64_t ldq,
                                                       const unsigned short* __restrict__ k,
                                                       const unsigned short* __restrict__ v, int64_t ldkv,
                                                       const unsigned short* __restrict__ bias,
                                                       const int* __restrict__ enc_index, int heads, int N, int L,
                                                       int U, float scale, unsigned short* __restrict__ o, int64_t ldo) {
    constexpr int QF = 2;
    constexpr int RS = HD + 8, KSN = (HD + 31) / 32, DF = HD / 16;
    constexpr int FH = LM / 32;  // key fragments (of 16) per half
    static_assert(HD % 16 == 0 && HD <= 128 && LM % 64 == 0, "head dim / key capacity");
    __shared__ __attribute__((aligned(16))) unsigned short sk[LM * RS];
    __shared__ __attribute__((aligned(16))) unsigned short sv[LM * RS];
    __shared__ float sb[LM];
    constexpr int NT = 64 * NWAVE;
    const int bh = xcd_remap(blockIdx.x, gridDim.x);
    const int b = bh / heads, h = bh - b * heads;
    const int u_in = enc_index ? enc_index[b] : b;
    const bool u_bad = u_in < 0 || u_in >= U;  // out-of-range caption row: NaN output, no out-of-bounds read
    const int u = u_bad ? 0 : u_in;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
    xa_stage_kv<HD, LM, NT>(k, v, ldkv, u, h, L, tid, sk, sv);
    for (int r = tid; r < LM; r += NT)
        sb[r] = u_bad ? __builtin_nanf("") : r < L ? (bias ? b2f(bias[(int64_t)u * L + r]) : 0.0f) : -INFINITY;
    __syncthreads();
    const int nkf = (L + 15) / 16, nkb = (L + 31) / 32;
    const int nqb = (N + 16 * QF - 1) / (16 * QF);
    auto load_q = [&](int qb_, la_bf16x8 (&dst)[QF][KSN]) {
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            const int qrow = qb_ * 16 * QF + 16 * x + r16;
#pragma unroll
            for (int ks = 0; ks < KSN; ++ks) {
                const int d0 = 32 * ks + 8 * g;
                u16x8m t = u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
                if (d0 < HD && qrow < N)
                    t = *reinterpret_cast<const u16x8m*>(q + ((int64_t)b * N + qrow) * ldq + (int64_t)h * HD + d0);
                dst[x][ks] = __builtin_bit_cast(la_bf16x8, t);
            }
        }
    };
    // the next block's q fragments are loaded right after this block's first-half S^T MFMAs are issued
    // (their latency runs under the softmax and PV: EGG_XA_PREFETCH)
    la_bf16x8 bq[QF][KSN], bqn[QF][KSN];
    if (w < nqb) load_q(w, bqn);
#pragma unroll 1
    for (int qb = w; qb < nqb; qb += NWAVE) {
#pragma unroll
        for (int x = 0; x < QF; ++x)
#pragma unroll
            for (int ks = 0; ks < KSN; ++ks) bq[x][ks] = bqn[x][ks];
        float mx[QF], sum[QF];
        la_f32x4 oc[QF][DF];
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            mx[x] = -INFINITY;
            sum[x] = 0.0f;
#pragma unroll
            for (int d = 0; d < DF; ++d) oc[x][d] = la_f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int f0 = half * FH;
            if (f0 >= nkf) break;  // uniform: L <= LM / 2 keys
            la_f32x4 sf[QF][FH];
            float lm[QF];
#pragma unroll
            for (int x = 0; x < QF; ++x) lm[x] = -INFINITY;
#pragma unroll
            for (int f = 0; f < FH; ++f) {
#pragma unroll
                for (int x = 0; x < QF; ++x) sf[x][f] = la_f32x4{0.f, 0.f, 0.f, 0.f};
                if (f0 + f < nkf) {
#pragma unroll
                    for (int ks = 0; ks < KSN; ++ks) {
                        const int d0 = 32 * ks + 8 * g;
                        la_bf16x8 a;
                        if (d0 < HD) a = *reinterpret_cast<const la_bf16x8*>(sk + (16 * (f0 + f) + r16) * RS + d0);
                        else a = la_bf16x8{};
#pragma unroll
                        for (int x = 0; x < QF; ++x) sf[x][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[x][ks], sf[x][f], 0, 0, 0);
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float bb = sb[16 * (f0 + f) + 4 * g + e];
#pragma unroll
                        for (int x = 0; x < QF; ++x) {
                            const float sv_ = sf[x][f][e] * scale + bb;
                            sf[x][f][e] = sv_;
                            lm[x] = fmaxf(lm[x], sv_);
                        }
                    }
                }
            }
            if (half == 0 && qb + NWAVE < nqb) load_q(qb + NWAVE, bqn);
            float alpha[QF];
#pragma unroll
            for (int x = 0; x < QF; ++x) {
                lm[x] = g4_max(lm[x]);
                const float mn = fmaxf(mx[x], lm[x]);
                alpha[x] = half == 0 ? 0.0f : __expf(mx[x] - mn);
                mx[x] = mn;
            }
            if (half > 0) {
#pragma unroll
                for (int x = 0; x < QF; ++x) {
                    sum[x] *= alpha[x];
#pragma unroll
                    for (int d = 0; d < DF; ++d)
#pragma unroll
                        for (int e = 0; e < 4; ++e) oc[x][d][e] *= alpha[x];
                }
            }
#pragma unroll
            for (int f = 0; f < FH; ++f) {
                if (f0 + f < nkf) {
#pragma unroll
                    for (int x = 0; x < QF; ++x)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float pe = __expf(sf[x][f][e] - mx[x]);
                            sf[x][f][e] = pe;
                            sum[x] += pe;
                        }
                }
            }
#pragma unroll
            for (int j = 0; j < FH / 2; ++j) {
                const int jj = half * (FH / 2) + j;
                if (jj < nkb) {
                    la_bf16x8 bp[QF];
#pragma unroll
                    for (int x = 0; x < QF; ++x)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            bp[x][e] = (__bf16)sf[x][2 * j][e];
                            bp[x][4 + e] = (__bf16)sf[x][2 * j + 1][e];
                        }
#pragma unroll
                    for (int d = 0; d < DF; ++d) {
                        const la_bf16x8 av = xa_tr8_perm<RS>(sv + (32 * jj) * RS + 16 * d, lane);
#pragma unroll
                        for (int x = 0; x < QF; ++x) oc[x][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bp[x], oc[x][d], 0, 0, 0);
                    }
                }
            }
        }
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            sum[x] = g4_sum(sum[x]);
            const int qrow = qb * 16 * QF + 16 * x + r16;
            if (qrow < N) {
                const float inv = 1.0f / sum[x];
                unsigned short* dst = o + ((int64_t)b * N + qrow) * ldo + (int64_t)h * HD + 4 * g;
#pragma unroll
                for (int d = 0; d < DF; ++d) {
                    u16x4m t;
#pragma unroll
                    for (int e = 0; e < 4; ++e) t[e] = f2b(oc[x][d][e] * inv);
                    *reinterpret_cast<u16x4m*>(dst + 16 * d) = t;
                }
            }
        }
    }
}

template <int SEG, int NCH>
static void launch_rownorm(const void* x, int xf32, int64_t rows, int C, float eps, int layer, const void* w,
                           const void* b, const void* ms, const void* mh, int64_t mstride, int mf32, int64_t rpg,
                           int act, const void* res, int rf32, void* out, int of32, void* shadow, hipStream_t st) {
    const int64_t threads = rows * SEG;
    const dim3 grid((unsigned)((threads + 255) / 256));
#define EGG_RNK(XF_, OF_)                                                                                          \
    hipLaunchKernelGGL((k_rownorm<SEG, NCH, XF_, OF_>), grid, dim3(256), 0, st, x, rows, C, eps, layer,          \
                       (const unsigned short*)w, (const unsigned short*)b, ms, mh, mstride, mf32, rpg, act, res, rf32, \
                       out, (unsigned short*)shadow)
    if (xf32) EGG_RNK(true, false);
    else if (of32) EGG_RNK(false, true);
    else EGG_RNK(false, false);
#undef EGG_RNK
}

extern "C" int eggroll_rownorm_ex(const void* x, int32_t x_f32, int64_t rows, int64_t C, float eps, int32_t layer,
                                  const void* w, const void* b, const void* mscale, const void* mshift,
                                  int64_t mstride, int32_t mod_f32, int64_t rows_per_group, int32_t act,
                                  const void* res, int32_t res_f32, void* out, int32_t out_f32, void* shadow,
                                  void* stream) {
    EGG_CHECK_ARG(rows >= 0 && C > 0 && C % 8 == 0 && C <= 8 * 64 * 8, "rownorm: need C %% 8 == 0, C <= 4096");
    EGG_CHECK_ARG(act >= 0 && act <= 2 && rows_per_group > 0, "rownorm: bad act / rows_per_group");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 && (!res || ((uintptr_t)res & 15) == 0) &&
                      (!mscale || ((uintptr_t)mscale & 15) == 0) && (!mshift || ((uintptr_t)mshift & 15) == 0) &&
                      ((uintptr_t)shadow & 15) == 0,
                  "rownorm: pointers must be 16-byte aligned");
    EGG_CHECK_ARG(mstride % 8 == 0, "rownorm: modulation stride must be a multiple of 8");
    EGG_CHECK_ARG((x_f32 == 0 || x_f32 == 1) && (mod_f32 == 0 || mod_f32 == 1) && (res_f32 == 0 || res_f32 == 1) &&
                      (out_f32 == 0 || out_f32 == 1) && !(x_f32 && out_f32) && (out_f32 || !shadow),
                  "rownorm: dtype flags are 0 / 1; fp32 x with fp32 out, or a shadow without fp32 out, unsupported");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && out, "rownorm: NULL pointer");
    hipStream_t st = as_stream(stream);
    const int nch = (int)(C / 8);
#define EGG_RN(S_, N_) launch_rownorm<S_, N_>(x, x_f32, rows, (int)C, eps, layer, w, b, mscale, mshift, mstride, mod_f32, \
                                              rows_per_group, act, res, res_f32, out, out_f32, shadow, st)
    if (nch <= 16) EGG_RN(16, 1);
    else if (nch <= 32) EGG_RN(32, 1);
    else if (nch <= 64) EGG_RN(64, 1);
    else if (nch <= 128) EGG_RN(64, 2);
    else if (nch <= 256) EGG_RN(64, 4);
    // Sana's C = 2240 (280 chunks): 5 chunks per lane use 88 % of the slots (8: 55 %, 64 dead value
    // registers); a lane sums the same chunks in the same order either way, so the bits do not change
    else if (nch <= 320) EGG_RN(64, 5);
    else EGG_RN(64, 8);
#undef EGG_RN
    EGG_CHECK_LAUNCH("rownorm");
    return EGGROLL_OK;
}

// ------------------------------------------------------------------------------------
// Per-head RMS norm + rotary position embedding, in place (the Z-Image q / k, head dim 128):
//   y = x * rsqrt(mean_head(x^2) + eps) * w;   (y[2p], y[2p+1]) <- (y0 c - y1 s, y0 s + y1 c)
// with c, s = cos / sin[row % tab_rows][p] (fp32 tables, one row per token position of one member; the
// member copies of a population batch repeat them).  16 lanes per (token, head), 8 consecutive values =
// 4 rotation pairs per lane, fp32 throughout and one bf16 rounding.  Replaces the norm pass and torch's
// fp32 rotation (~10 full passes over q and k per attention).
// ------------------------------------------------------------------------------------
// out == NULL: in place on x.  Otherwise the result goes to out at row (row / rps) * out_bs + (row0 +
// row % rps) * out_ld (a KV cache [seq][ltot][C] slice), and vin (when given) is copied to vout at the same
// row (the values of the same tokens); hscale (optional, fp32 [heads]) multiplies head h's output.
__global__ __launch_bounds__(256) void k_qk_norm_rope(unsigned short* __restrict__ x, int64_t ldx, int heads,
                                                      float eps, const unsigned short* __restrict__ w,
                                                      const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                      int64_t tab_rows, int64_t segs, const float* __restrict__ hscale,
                                                      unsigned short* __restrict__ out, int64_t out_bs, int64_t out_ld,
                                                      int64_t rps, int64_t row0, const unsigned short* __restrict__ vin,
                                                      int64_t ldv, unsigned short* __restrict__ vout) {
    const int64_t seg = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int l = threadIdx.x & 15;
    const bool live = seg < segs;
    const int64_t row = live ? seg / heads : 0;
    const int h = live ? (int)(seg - row * heads) : 0;
    unsigned short* p = x + row * ldx + h * 128 + l * 8;
    u16x8m v = u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
    if (live) v = *reinterpret_cast<const u16x8m*>(p);
    float f[8], ss = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        f[i] = b2f(v[i]);
        ss += f[i] * f[i];
    }
    ss = seg_sum<16>(ss);   // within the 16-lane segment
    const float r = rsqrtf(ss / 128.f + eps);
    if (!live) return;
    const u16x8m wv = *reinterpret_cast<const u16x8m*>(w + l * 8);
    const int64_t tr = row % tab_rows;
    const float4 c4 = *reinterpret_cast<const float4*>(cosb + tr * 64 + l * 4);
    const float4 s4 = *reinterpret_cast<const float4*>(sinb + tr * 64 + l * 4);
    const float cs[4] = {c4.x, c4.y, c4.z, c4.w}, sn[4] = {s4.x, s4.y, s4.z, s4.w};
    const float hs = hscale ? hscale[h] : 1.0f;
    u16x8m o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float y0 = f[2 * j] * r * b2f(wv[2 * j]), y1 = f[2 * j + 1] * r * b2f(wv[2 * j + 1]);
        if (hscale) {
            o[2 * j] = f2b(b2f(f2b(y0 * cs[j] - y1 * sn[j])) * hs);
            o[2 * j + 1] = f2b(b2f(f2b(y0 * sn[j] + y1 * cs[j])) * hs);
        } else {
            o[2 * j] = f2b(y0 * cs[j] - y1 * sn[j]);
            o[2 * j + 1] = f2b(y0 * sn[j] + y1 * cs[j]);
        }
    }
    if (!out) {
        *reinterpret_cast<u16x8m*>(p) = o;
        return;
    }
    const int64_t orow = (row / rps) * out_bs + (row0 + row % rps) * out_ld + h * 128 + l * 8;
    *reinterpret_cast<u16x8m*>(out + orow) = o;
    if (vin) *reinterpret_cast<u16x8m*>(vout + orow) = *reinterpret_cast<const u16x8m*>(vin + row * ldv + h * 128 + l * 8);
}

extern "C" int eggroll_qk_norm_rope(void* x, int64_t ldx, int64_t rows, int32_t heads, int32_t head_dim, float eps,
                                    const void* w, const float* cos_tab, const float* sin_tab, int64_t tab_rows,
                                    void* stream) {
    EGG_CHECK_ARG(head_dim == 128, "qk_norm_rope: head_dim must be 128 (got %d)", head_dim);
    EGG_CHECK_ARG(rows >= 0 && heads > 0 && ldx >= (int64_t)heads * 128 && ldx % 8 == 0 && tab_rows > 0,
                  "qk_norm_rope: bad sizes / strides");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)cos_tab & 15) == 0 &&
                      ((uintptr_t)sin_tab & 15) == 0,
                  "qk_norm_rope: pointers must be 16-byte aligned");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && w && cos_tab && sin_tab, "qk_norm_rope: NULL pointer");
    const int64_t segs = rows * heads;
    EGG_CHECK_ARG(segs < (1ll << 31) / 16, "qk_norm_rope: too many rows");
    hipLaunchKernelGGL(k_qk_norm_rope, dim3((unsigned)((segs * 16 + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (unsigned short*)x, ldx, (int)heads, eps, (const unsigned short*)w, cos_tab, sin_tab, tab_rows,
                       segs, nullptr, nullptr, 0, 0, 1, 0, nullptr, 0, nullptr);
    EGG_CHECK_LAUNCH("qk_norm_rope");
    return EGGROLL_OK;
}

extern "C" int eggroll_qk_norm_rope_kv(void* x, int64_t ldx, int64_t rows, int32_t heads, int32_t head_dim, float eps,
                                       const void* w, const float* cos_tab, const float* sin_tab, int64_t tab_rows,
                                       const float* hscale, void* out, int64_t out_bs, int64_t out_ld,
                                       int64_t rows_per_seq, int64_t row0, const void* vin, int64_t ldv, void* vout,
                                       void* stream) {
    EGG_CHECK_ARG(head_dim == 128, "qk_norm_rope_kv: head_dim must be 128 (got %d)", head_dim);
    EGG_CHECK_ARG(rows >= 0 && heads > 0 && ldx >= (int64_t)heads * 128 && ldx % 8 == 0 && tab_rows > 0,
                  "qk_norm_rope_kv: bad sizes / strides");
    EGG_CHECK_ARG(!out || (rows_per_seq > 0 && row0 >= 0 && out_ld >= (int64_t)heads * 128 && out_ld % 8 == 0 &&
                           out_bs % 8 == 0 && out_bs >= (row0 + rows_per_seq) * out_ld),
                  "qk_norm_rope_kv: bad output geometry");
    EGG_CHECK_ARG(!vin || (out && vout && ldv >= (int64_t)heads * 128 && ldv % 8 == 0),
                  "qk_norm_rope_kv: the value copy needs out, vout and ldv");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)cos_tab & 15) == 0 &&
                      ((uintptr_t)sin_tab & 15) == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)vin & 15) == 0 &&
                      ((uintptr_t)vout & 15) == 0,
                  "qk_norm_rope_kv: pointers must be 16-byte aligned");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && w && cos_tab && sin_tab, "qk_norm_rope_kv: NULL pointer");
    const int64_t segs = rows * heads;
    EGG_CHECK_ARG(segs < (1ll << 31) / 16, "qk_norm_rope_kv: too many rows");
    hipLaunchKernelGGL(k_qk_norm_rope, dim3((unsigned)((segs * 16 + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (unsigned short*)x, ldx, (int)heads, eps, (const unsigned short*)w, cos_tab, sin_tab, tab_rows,
                       segs, hscale, (unsigned short*)out, out_bs, out_ld, out ? rows_per_seq : 1, row0,
                       (const unsigned short*)vin, ldv, (unsigned short*)vout);
    EGG_CHECK_LAUNCH("qk_norm_rope_kv");
    return EGGROLL_OK;
}

extern "C" int eggroll_rownorm(const void* x, int64_t rows, int64_t C, float eps, int32_t layer, const void* w,
                               const void* b, const void* mscale, const void* mshift, int64_t mstride,
                               int64_t rows_per_group, int32_t act, const void* res, void* out, void* stream) {
    return eggroll_rownorm_ex(x, 0, rows, C, eps, layer, w, b, mscale, mshift, mstride, 0, rows_per_group, act, res,
                              0, out, 0, nullptr, stream);
}

extern "C" int eggroll_resid_layernorm(float* h, int64_t ldh, const void* y, int64_t ldy, int64_t rows, int64_t C,
                                       float eps, const void* w, const void* b, void* out, void* stream) {
    EGG_CHECK_ARG(rows >= 0 && C > 0 && C % 8 == 0 && C <= 4096, "resid_layernorm: need C %% 8 == 0, C <= 4096");
    EGG_CHECK_ARG(ldh >= C && ldh % 4 == 0 && (!y || (ldy >= C && ldy % 8 == 0)),
                  "resid_layernorm: row strides must cover C and keep 16-byte rows");
    EGG_CHECK_ARG(((uintptr_t)h & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                      ((uintptr_t)w & 15) == 0 && ((uintptr_t)b & 15) == 0,
                  "resid_layernorm: pointers must be 16-byte aligned");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(h && w && b && out, "resid_layernorm: NULL pointer");
    EGG_CHECK_ARG(rows < (1ll << 31) / 4, "resid_layernorm: too many rows");
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)((rows + 3) / 4));
    const int nch = (int)(C / 8);
    auto* yy = (const unsigned short*)y;
    auto* ww = (const unsigned short*)w;
    auto* bb = (const unsigned short*)b;
    auto* oo = (unsigned short*)out;
#define EGG_RLN(N_) hipLaunchKernelGGL(k_resid_layernorm<N_>, grid, dim3(256), 0, st, h, ldh, yy, ldy, rows, (int)C, eps, \
                                       ww, bb, oo)
    if (nch <= 64) EGG_RLN(1);
    else if (nch <= 128) EGG_RLN(2);
    else if (nch <= 192) EGG_RLN(3);   // CLIP-H: C = 1280 (160 chunks)
    else if (nch <= 256) EGG_RLN(4);
    else EGG_RLN(8);
#undef EGG_RLN
    EGG_CHECK_LAUNCH("resid_layernorm");
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

extern "C" int eggroll_gated_residual_f32(float* x, const void* y, const void* gate, int32_t gate_f32, int64_t gstride,
                                          int64_t rows, int64_t C, int64_t rows_per_group, void* shadow, void* stream) {
    EGG_CHECK_ARG(rows >= 0 && C > 0 && C % 8 == 0 && gstride % 8 == 0 && rows_per_group > 0 &&
                      (gate_f32 == 0 || gate_f32 == 1),
                  "gated_residual_f32: bad sizes");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)gate & 15) == 0 &&
                      ((uintptr_t)shadow & 15) == 0,
                  "gated_residual_f32: pointers must be 16-byte aligned");
    if (rows == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && y, "gated_residual_f32: NULL pointer");
    const int64_t total = rows * (C / 8);
    hipLaunchKernelGGL(k_gated_residual_f32, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), x,
                       (const unsigned short*)y, gate, gate_f32, gstride, rows_per_group, (int)C, total,
                       (unsigned short*)shadow);
    EGG_CHECK_LAUNCH("gated_residual_f32");
    return EGGROLL_OK;
}

// block order (kernel argument `ord`, see k_dwconv_nhwc) for the automatic choice
static int dw_order(int kernel) { return kernel == 0 ? DW_ORDER_AUTO : kernel - 1; }

extern "C" int eggroll_dwconv_nhwc(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H, int64_t W,
                                   int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out, void* stream) {
    return eggroll_dwconv_nhwc_sel(in, w_t, bias, B, H, W, C, ks, pre_silu, glu, out, 0, stream);
}

extern "C" int eggroll_dwconv_nhwc_sel(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H,
                                       int64_t W, int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out,
                                       int32_t kernel, void* stream) {
    return eggroll_dwconv_nhwc_ex(in, w_t, bias, B, H, W, C, ks, pre_silu, glu, out, glu ? C / 2 : C, kernel, stream);
}

extern "C" int eggroll_dwconv_nhwc_ex(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H,
                                      int64_t W, int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out,
                                      int64_t ldo, int32_t kernel, void* stream) {
    EGG_CHECK_ARG(kernel >= 0 && kernel <= 2, "dwconv: kernel must be 0 (auto), 1 (channel-fastest) or 2 (column "
                  "sweep) (got %d)", kernel);
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && C > 0, "dwconv: bad sizes");
    const int64_t cout = glu ? C / 2 : C;
    EGG_CHECK_ARG((!glu || C % 2 == 0) && cout % DW_CS == 0, "dwconv: output channels must be a multiple of %d", DW_CS);
    EGG_CHECK_ARG(ldo >= cout && ldo - cout <= DW_CS && ldo % 8 == 0,
                  "dwconv: output row stride %lld must be in [%lld, %lld] and a multiple of 8", (long long)ldo,
                  (long long)cout, (long long)(cout + DW_CS));
    EGG_CHECK_ARG(ks == 3 || ks == 5, "dwconv: ks=%d unsupported (3, 5)", ks);
    EGG_CHECK_ARG(((uintptr_t)in & 15) == 0 && ((uintptr_t)w_t & 15) == 0 && ((uintptr_t)out & 15) == 0,
                  "dwconv: pointers must be 16-byte aligned");
    EGG_CHECK_ARG(H * W * C < (1ll << 30) && H * W * ldo < (1ll << 30), "dwconv: image too large (< 2 GiB per image)");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(in && w_t && out, "dwconv: NULL pointer");
    const int64_t bands = (H + DW_TH - 1) / DW_TH, xtiles = (W + DW_TW - 1) / DW_TW, cslices = cout / DW_CS;
    const int64_t nblk = B * bands * xtiles * cslices;
    EGG_CHECK_ARG(nblk < (1ll << 31), "dwconv: grid too large");
    const dim3 grid((unsigned)nblk);
    hipStream_t st = as_stream(stream);
    auto* i = (const unsigned short*)in;
    auto* w = (const unsigned short*)w_t;
    auto* bb = (const unsigned short*)bias;
    auto* o = (unsigned short*)out;
#define EGG_DW(KS_, PS_, GL_)                                                                                 \
    hipLaunchKernelGGL((k_dwconv_nhwc<KS_, PS_, GL_>), grid, dim3(256), 0, st, i, w, bb, (int)H, (int)W, (int)C,  \
                       (int)xtiles, (int)bands, (int)cslices, o, nullptr, dw_order(kernel), (int)ldo)
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

extern "C" int eggroll_dwconv_pw_nhwc(const void* in, const void* w_t, const void* pw, int64_t B, int64_t H, int64_t W,
                                      int64_t C, int32_t ks, void* out, void* stream) {
    return eggroll_dwconv_pw_nhwc_sel(in, w_t, pw, B, H, W, C, ks, out, 0, stream);
}

extern "C" int eggroll_dwconv_pw_nhwc_sel(const void* in, const void* w_t, const void* pw, int64_t B, int64_t H,
                                          int64_t W, int64_t C, int32_t ks, void* out, int32_t kernel, void* stream) {
    EGG_CHECK_ARG(kernel >= 0 && kernel <= 2, "dwconv_pw: kernel must be 0 (auto), 1 or 2 (got %d)", kernel);
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && C > 0 && C % DW_CS == 0, "dwconv_pw: C must be a multiple of %d", DW_CS);
    EGG_CHECK_ARG(ks == 3 || ks == 5, "dwconv_pw: ks=%d unsupported (3, 5)", ks);
    EGG_CHECK_ARG(((uintptr_t)in & 15) == 0 && ((uintptr_t)w_t & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                      ((uintptr_t)pw & 15) == 0,
                  "dwconv_pw: pointers must be 16-byte aligned");
    EGG_CHECK_ARG(H * W * C < (1ll << 30), "dwconv_pw: image too large (< 2 GiB per image)");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(in && w_t && pw && out && out != in, "dwconv_pw: NULL or aliased pointer");
    const int64_t bands = (H + DW_TH - 1) / DW_TH, xtiles = (W + DW_TW - 1) / DW_TW, cslices = C / DW_CS;
    const int64_t nblk = B * bands * xtiles * cslices;
    EGG_CHECK_ARG(nblk < (1ll << 31), "dwconv_pw: grid too large");
    auto* i = (const unsigned short*)in;
    auto* w = (const unsigned short*)w_t;
    auto* o = (unsigned short*)out;
    auto* p = (const unsigned short*)pw;
    hipStream_t st = as_stream(stream);
    if (ks == 5)
        hipLaunchKernelGGL((k_dwconv_nhwc<5, false, false, true>), dim3((unsigned)nblk), dim3(256), 0, st, i, w, nullptr,
                           (int)H, (int)W, (int)C, (int)xtiles, (int)bands, (int)cslices, o, p, dw_order(kernel));
    else
        hipLaunchKernelGGL((k_dwconv_nhwc<3, false, false, true>), dim3((unsigned)nblk), dim3(256), 0, st, i, w, nullptr,
                           (int)H, (int)W, (int)C, (int)xtiles, (int)bands, (int)cslices, o, p, dw_order(kernel));
    EGG_CHECK_LAUNCH("dwconv_pw_nhwc");
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

extern "C" int eggroll_subpixel_shortcut(const void* y4, const void* x, const void* bias, void* out, int64_t B,
                                         int64_t H, int64_t W, int64_t Cin, int64_t Cout, void* stream) {
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && (4 * Cout) % Cin == 0 && Cout % 8 == 0,
                  "subpixel_shortcut: bad sizes");
    EGG_CHECK_ARG(B * 4 * H * W * Cout < (1ll << 31) && B * (H + 1) * (W + 1) * 4 * Cout < (1ll << 31),
                  "subpixel_shortcut: tensor too large");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(y4 && x && out, "subpixel_shortcut: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)bias & 15) == 0, "subpixel_shortcut: bias must be 16-byte aligned");
    const int64_t rep = 4 * Cout / Cin;
    if ((rep == 1 || rep == 2 || rep == 4) && Cin % 8 == 0) {
        const int64_t lowpix = B * H * W;
        const int64_t threads = lowpix * (Cout / 8);
        const dim3 grid((unsigned)((threads + 255) / 256));
#define EGG_SP4(RP)                                                                                                  \
    hipLaunchKernelGGL(k_subpixel_shortcut4<RP>, grid, dim3(256), 0, as_stream(stream), (const unsigned short*)y4, \
                       (const unsigned short*)x, (const unsigned short*)bias, (unsigned short*)out, (int)H, (int)W,  \
                       (int)Cin, (int)Cout, (int)lowpix)
        if (rep == 1) EGG_SP4(1);
        else if (rep == 2) EGG_SP4(2);
        else EGG_SP4(4);
#undef EGG_SP4
        EGG_CHECK_LAUNCH("subpixel_shortcut");
        return EGGROLL_OK;
    }
    const int64_t pix = B * 4 * H * W;
    const int64_t threads = pix * (Cout / 8);
    hipLaunchKernelGGL(k_subpixel_shortcut, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, as_stream(stream),
                       (const unsigned short*)y4, (const unsigned short*)x, (const unsigned short*)bias,
                       (unsigned short*)out, (int)H, (int)W, (int)Cin, (int)Cout, (int)rep, (int)pix);
    EGG_CHECK_LAUNCH("subpixel_shortcut");
    return EGGROLL_OK;
}

extern "C" int eggroll_subpixel_shortcut_f32(const void* y4, const float* x, const void* bias, float* out,
                                             void* shadow, int64_t B, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                             void* stream) {
    const int64_t rep = Cin > 0 ? 4 * Cout / Cin : 0;
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && (4 * Cout) % Cin == 0 && Cout % 8 == 0 &&
                      (rep == 1 || rep == 2 || rep == 4) && Cin % 8 == 0,
                  "subpixel_shortcut_f32: bad sizes (4 Cout / Cin in {1, 2, 4})");
    EGG_CHECK_ARG(B * 4 * H * W * Cout < (1ll << 31) && B * (H + 1) * (W + 1) * 4 * Cout < (1ll << 31),
                  "subpixel_shortcut_f32: tensor too large");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(y4 && x && out, "subpixel_shortcut_f32: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)bias & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                      ((uintptr_t)shadow & 15) == 0,
                  "subpixel_shortcut_f32: pointers must be 16-byte aligned");
    const int64_t lowpix = B * H * W;
    const dim3 grid((unsigned)((lowpix * (Cout / 8) + 255) / 256));
#define EGG_SP4F(RP)                                                                                                  \
    hipLaunchKernelGGL((k_subpixel_shortcut4<RP, true>), grid, dim3(256), 0, as_stream(stream),                   \
                       (const unsigned short*)y4, (const void*)x, (const unsigned short*)bias, (void*)out, (int)H,  \
                       (int)W, (int)Cin, (int)Cout, (int)lowpix, (unsigned short*)shadow)
    if (rep == 1) EGG_SP4F(1);
    else if (rep == 2) EGG_SP4F(2);
    else EGG_SP4F(4);
#undef EGG_SP4F
    EGG_CHECK_LAUNCH("subpixel_shortcut_f32");
    return EGGROLL_OK;
}

extern "C" int64_t eggroll_linear_attention_workspace_bytes(int64_t B, int64_t N, int64_t heads) {
    const int64_t nchunk = (N + LA_T - 1) / LA_T;
    return B * heads * (nchunk + 1) * LA_PART * (int64_t)sizeof(float);  // partials, then per-head sums
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
    EGG_CHECK_ARG(N * ld < (1ll << 30) && N * ldo < (1ll << 30), "linear_attention: image too large (< 2 GiB per image)");
    const int64_t nchunk = (N + LA_T - 1) / LA_T;
    const int64_t blocks = B * heads * nchunk;
    EGG_CHECK_ARG(blocks < (1ll << 31), "linear_attention: grid too large");
    hipStream_t st = as_stream(stream);
    // head pairs per block when a head's 64 B and its neighbour's are one 128-B line (Sana's q / k / v,
    // the DC-AE's planar [Q | K | V]) and the grid stays large: Sana attn1 637 -> 615 us, the DC-AE's 128^2
    // maps 154 -> 152; at 8 x 64^2 / 32^2 x 32 heads (4096 / 1024 per-head blocks) the halved grid lost
    // 1-4 % (profiles/r10d_linear_attention_head_pairs_ab.log).  The reference-layout interleaved q | k | v
    // (hstride 96) stays per head.
    const int hp = hstride == LA_D && heads % 2 == 0 && blocks >= 8192 && EGG_LA_HEAD_PAIRS ? 2 : 1;
    float* kvsum = (float*)workspace + blocks * LA_PART;
    // few chunks per head on a grid that one block per head (group) still fills (Sana attn1: 128 x 35 head
    // pairs x 4 chunks): the reduction folded into the kv pass (k_la_kv_fold, the same bits)
    const bool fold = EGG_LA_FOLD && nchunk <= LA_FOLD_MAX && B * heads / hp >= 2048;
    if (fold) {
        if (hp == 2)
            hipLaunchKernelGGL(k_la_kv_fold<2>, dim3((unsigned)(B * heads / 2)), dim3(256), 0, st,
                               (const unsigned short*)k, (const unsigned short*)v, ld, hstride, (int)heads, (int)N,
                               (int)nchunk, relu_qk, kvsum);
        else
            hipLaunchKernelGGL(k_la_kv_fold<1>, dim3((unsigned)(B * heads)), dim3(256), 0, st, (const unsigned short*)k,
                               (const unsigned short*)v, ld, hstride, (int)heads, (int)N, (int)nchunk, relu_qk, kvsum);
        EGG_CHECK_LAUNCH("linear_attention_kv_fold");
    } else {
        if (hp == 2)
            hipLaunchKernelGGL(k_la_kv<2>, dim3((unsigned)(blocks / 2)), dim3(256), 0, st, (const unsigned short*)k,
                               (const unsigned short*)v, ld, hstride, (int)heads, (int)N, (int)nchunk, relu_qk,
                               (float*)workspace);
        else
            hipLaunchKernelGGL(k_la_kv<1>, dim3((unsigned)blocks), dim3(256), 0, st, (const unsigned short*)k,
                               (const unsigned short*)v, ld, hstride, (int)heads, (int)N, (int)nchunk, relu_qk,
                               (float*)workspace);
        EGG_CHECK_LAUNCH("linear_attention_kv");
        if (nchunk >= LA_RED_WIDE)
            hipLaunchKernelGGL(k_la_reduce_e, dim3((unsigned)(B * heads * LA_RED_WAVES)), dim3(64), 0, st,
                               (const float*)workspace, (int)nchunk, kvsum);
        else
            hipLaunchKernelGGL(k_la_reduce, dim3((unsigned)(B * heads)), dim3(256), 0, st, (const float*)workspace,
                               (int)nchunk, kvsum);
        EGG_CHECK_LAUNCH("linear_attention_reduce");
    }
    const bool big = N >= 8192;  // 16 tiles per wave at the DC-AE's 128^2 maps
    const int64_t tpb = 4 * 16 * (big ? 16 : 8);
    const int64_t oblk = (N + tpb - 1) / tpb;
    const dim3 og((unsigned)(B * (heads / hp) * oblk));
#define EGG_LAO(HP_, TPW_)                                                                                          \
    hipLaunchKernelGGL((k_la_out<HP_, TPW_>), og, dim3(256), 0, st, (const unsigned short*)q, ld, hstride, (int)heads, \
                       (int)N, (int)oblk, relu_qk, (const float*)kvsum, (unsigned short*)out, ldo)
    if (hp == 2 && big) EGG_LAO(2, 16);
    else if (hp == 2) EGG_LAO(2, 8);
    else if (big) EGG_LAO(1, 16);
    else EGG_LAO(1, 8);
#undef EGG_LAO
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

extern "C" int eggroll_dcae_head(const void* x, int64_t B, int64_t H, int64_t W, int64_t C, float eps,
                                 const void* norm_w, const void* norm_b, const void* conv_w, const void* conv_b,
                                 void* y, void* stream) {
    EGG_CHECK_ARG(B >= 0 && H > 0 && W > 0, "dcae_head: bad sizes");
    EGG_CHECK_ARG(C == HD_C, "dcae_head: C=%lld unsupported (%d)", (long long)C, HD_C);
    EGG_CHECK_ARG(H * W * C < (1ll << 30), "dcae_head: image too large (< 2 GiB per image: 32-bit buffer offsets)");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && norm_w && norm_b && conv_w && y, "dcae_head: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)norm_w & 15) == 0 && ((uintptr_t)norm_b & 15) == 0 &&
                  ((uintptr_t)conv_w & 15) == 0, "dcae_head: pointers must be 16-byte aligned");
    const int64_t bands = (H + HD_TH - 1) / HD_TH, xtiles = (W + HD_TW - 1) / HD_TW;
    // bands per block: enough blocks to fill 256 CUs x 3 many times over, the rest walked in-block
    const int64_t tpb = EGG_HEAD_TPB;
    const int64_t nblk = B * ((bands + tpb - 1) / tpb) * xtiles;
    EGG_CHECK_ARG(nblk < (1ll << 31), "dcae_head: grid too large");
    hipLaunchKernelGGL(k_dcae_head, dim3((unsigned)nblk), dim3(256), 0, as_stream(stream), (const unsigned short*)x,
                       (int)H, (int)W, eps, (const unsigned short*)norm_w, (const unsigned short*)norm_b,
                       (const unsigned short*)conv_w, (const unsigned short*)conv_b, (int)xtiles, (int)bands, (int)tpb,
                       (unsigned short*)y);
    EGG_CHECK_LAUNCH("dcae_head");
    return EGGROLL_OK;
}

extern "C" int eggroll_clip_preprocess(const void* img, int64_t n, int64_t H, int64_t W, int64_t sn, int64_t sc,
                                       int64_t sh, int64_t sw, int32_t mode, const int32_t* tab_w, const int32_t* tab_h,
                                       int32_t ktw, int32_t kth, int64_t RW, int64_t RH, int64_t out_size,
                                       const float* mean, const float* stdv, void* tmp, void* out, void* stream) {
    EGG_CHECK_ARG(n >= 0 && H > 0 && W > 0 && out_size > 0 && RW >= out_size && RH >= out_size, "clip_preprocess: bad sizes");
    EGG_CHECK_ARG(mode >= 0 && mode <= 2, "clip_preprocess: mode %d (0 PixArt round, 1 VAR fp16 trunc, 2 Infinity bf16 trunc)",
                  mode);
    EGG_CHECK_ARG(ktw > 0 && kth > 0 && ktw <= 64 && kth <= 64, "clip_preprocess: tap counts out of range");
    if (n == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(img && tab_w && tab_h && mean && stdv && tmp && out, "clip_preprocess: NULL pointer");
    const int left = (int)((RW - out_size) / 2), top = (int)((RH - out_size) / 2);
    const int64_t t2 = n * 3 * out_size * out_size;
    EGG_CHECK_ARG((t2 + 255) / 256 < (1ll << 31), "clip_preprocess: grid too large");
    hipStream_t st = as_stream(stream);
    EGG_CHECK_ARG(W <= CLIP_MAXW && n * H < (1ll << 31), "clip_preprocess: W=%lld > %d or too many rows",
                  (long long)W, CLIP_MAXW);
    hipLaunchKernelGGL(k_clip_resize_h, dim3((unsigned)(n * H)), dim3(256), 0, st, (const unsigned short*)img,
                       sn, sc, sh, sw, (int)H, (int)W, (int)out_size, left, (int)mode, tab_w, (int)ktw,
                       (unsigned char*)tmp);
    EGG_CHECK_LAUNCH("clip_resize_h");
    float m[3], sd[3];
    // mean / std are host pointers (3 floats each): passed by value to the kernel
    for (int k = 0; k < 3; ++k) { m[k] = mean[k]; sd[k] = stdv[k]; }
    hipLaunchKernelGGL(k_clip_resize_v, dim3((unsigned)((t2 + 255) / 256)), dim3(256), 0, st, (const unsigned char*)tmp,
                       (int)H, (int)out_size, (int)out_size, top, tab_h, (int)kth, m[0], m[1], m[2], sd[0], sd[1], sd[2],
                       t2, (float*)out);
    EGG_CHECK_LAUNCH("clip_resize_v");
    return EGGROLL_OK;
}

// ------------------------------------------------------------------------------------
// Flash attention, head dim 128 (Z-Image self-attention; Infinity's cosine attention over the KV cache):
//   o[b, n, h, :] = softmax_j(scale * q[b,n,h,:] . k[b,j,h,:]) @ v[b, :, h, :],  j < Lk, no mask.
// q / k / v / o: [B][rows][heads * 128] bf16 views with their own batch and row strides (a KV cache
// [B][ltot][C] is read in place).  Workgroup = (b, h, 128-query block), 4 waves x 32 queries; keys in
// blocks of 64 staged in LDS (k and v [64][136] bf16), the next block held in registers while this one
// computes.  Per key block and wave, MFMA 16x16x32 bf16, fp32 accumulation, the k_cross_attn layout:
//   S^T = K Q^T   (Q^T fragments stay in registers for the whole key sweep; each lane: 4 keys of ONE query)
//   online softmax in base 2: m' = max(m, rowmax), O *= 2^(m - m'), P = 2^(S - m'), per-lane partial row
//                 sums rescaled the same way and reduced over the 4 lane groups once at the end
//   O^T += V^T P^T  (P^T packed from the C registers, V^T read with ds_read_tr16_b64 in the matching key order)
// ------------------------------------------------------------------------------------
// LDS row stride 144 bf16 = 288 B = 72 dwords: consecutive rows start 8 banks apart, so the S^T k reads
// (ds_read_b128, lane groups {0-3,12-15,20-27}...: 8 rows x 2 chunks) and the V^T reads (ds_read_b64_tr_b16,
// 32-lane groups: 8 rows x 32 B) both cover 64 distinct banks; the first form's 136 (4 banks apart) left
// 38 % of the LDS cycles to bank conflicts (PMC SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)
constexpr int FA_HD = 128, FA_KB = 64, FA_RS = FA_HD + 16;
typedef float fa_f32x2 __attribute__((ext_vector_type(2)));

template <int QF>
__global__ __launch_bounds__(256, QF == 1 ? 3 : (QF == 2 ? 2 : 1)) void k_flash_attn(const unsigned short* __restrict__ q, int64_t q_bs, int64_t ldq,
                                                    const unsigned short* __restrict__ k, int64_t k_bs, int64_t ldk,
                                                    const unsigned short* __restrict__ v, int64_t v_bs, int64_t ldv,
                                                    int heads, int Nq, int Lk, int nqb, float scale_log2,
                                                    unsigned short* __restrict__ o, int64_t o_bs, int64_t ldo) {
    constexpr int QW = 16 * QF, KSN = FA_HD / 32, DF = FA_HD / 16, KF = FA_KB / 16, CH = FA_HD / 8;
    constexpr int UNITS = 2 * FA_KB * CH / 256;   // 16-B chunks of k + v per thread per key block (8)
    __shared__ __attribute__((aligned(16))) unsigned short sk[FA_KB * FA_RS];
    __shared__ __attribute__((aligned(16))) unsigned short sv[FA_KB * FA_RS];
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int qb = bid % nqb, bh = bid / nqb;
    const int b = bh / heads, h = bh - b * heads;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
    const unsigned short* kb_ = k + (int64_t)b * k_bs + (int64_t)h * FA_HD;
    const unsigned short* vb_ = v + (int64_t)b * v_bs + (int64_t)h * FA_HD;
    // Q^T fragments (B operand): dims 32 ks + 8 g .. +7 of query 16 x + r16 of this wave's 32
    la_bf16x8 bq[QF][KSN];
    const int q0 = qb * (4 * QW) + w * QW;
#pragma unroll
    for (int x = 0; x < QF; ++x) {
        const int qr = q0 + 16 * x + r16;
#pragma unroll
        for (int ks = 0; ks < KSN; ++ks) {
            u16x8m t = u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
            if (qr < Nq)
                t = *reinterpret_cast<const u16x8m*>(q + (int64_t)b * q_bs + (int64_t)qr * ldq + (int64_t)h * FA_HD +
                                                     32 * ks + 8 * g);
            bq[x][ks] = __builtin_bit_cast(la_bf16x8, t);
        }
    }
    u16x8m pre[UNITS];
    auto load_blk = [&](int key0) {
#pragma unroll
        for (int i = 0; i < UNITS; ++i) {
            const int c = tid + 256 * i;             // [k | v][row][chunk]
            const int kv = c / (FA_KB * CH), rc = c - kv * (FA_KB * CH);
            const int r = rc / CH, cc = rc - r * CH;
            // branch-free: rows past Lk read the last key (in bounds) and are zeroed by a select
            const int row = min(key0 + r, Lk - 1);
            const unsigned short* src = kv ? vb_ + (int64_t)row * ldv : kb_ + (int64_t)row * ldk;
            const u16x8m t = *reinterpret_cast<const u16x8m*>(src + cc * 8);
            pre[i] = key0 + r < Lk ? t : u16x8m{0, 0, 0, 0, 0, 0, 0, 0};
        }
    };
    auto store_blk = [&]() {
#pragma unroll
        for (int i = 0; i < UNITS; ++i) {
            const int c = tid + 256 * i;
            const int kv = c / (FA_KB * CH), rc = c - kv * (FA_KB * CH);
            const int r = rc / CH, cc = rc - r * CH;
            *reinterpret_cast<u16x8m*>((kv ? sv : sk) + r * FA_RS + cc * 8) = pre[i];
        }
    };
    la_f32x4 oc[QF][DF];
    float m[QF], l[QF];
#pragma unroll
    for (int x = 0; x < QF; ++x) {
        m[x] = -INFINITY;
        l[x] = 0.0f;
#pragma unroll
        for (int d = 0; d < DF; ++d) oc[x][d] = la_f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int nkb = (Lk + FA_KB - 1) / FA_KB;
    load_blk(0);
    for (int kb = 0; kb < nkb; ++kb) {
        __syncthreads();   // every wave is done reading the previous block
        store_blk();
        __syncthreads();
        if (kb + 1 < nkb) load_blk((kb + 1) * FA_KB);   // in flight under this block's MFMAs
        la_f32x4 sf[QF][KF];
        // k-step outer, key fragment inner: 4 x QF independent accumulations between two dependent MFMAs
        // (f outer put each chain's next MFMA right behind it: PMC issue stalls ~35 % of wave cycles)
#pragma unroll
        for (int ks = 0; ks < KSN; ++ks) {
#pragma unroll
            for (int f = 0; f < KF; ++f) {
                const la_bf16x8 a = *reinterpret_cast<const la_bf16x8*>(sk + (16 * f + r16) * FA_RS + 32 * ks + 8 * g);
                // the first k-step takes a literal zero accumulator (no per-block zeroing of 32 registers)
#pragma unroll
                for (int x = 0; x < QF; ++x)
                    sf[x][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[x][ks], ks ? sf[x][f] : la_f32x4{0.f, 0.f, 0.f, 0.f},
                                                                       0, 0, 0);
            }
        }
        const int key0 = kb * FA_KB;
        // the VALU side is the bound here (PMC: ~6 VALU instructions per MFMA), so the softmax runs on
        // raw scores: max of raw S (scale > 0 commutes with max), then p = 2^(s * scale_log2 - m) as one
        // packed FMA per pair + exp2; O is rescaled only when some lane's running max moved
        if (key0 + FA_KB > Lk) {   // the partial last block: keys >= Lk -> -inf (uniform branch)
#pragma unroll
            for (int f = 0; f < KF; ++f)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const bool ok = key0 + 16 * f + 4 * g + e < Lk;
#pragma unroll
                    for (int x = 0; x < QF; ++x) sf[x][f][e] = ok ? sf[x][f][e] : -INFINITY;
                }
        }
#pragma unroll
        for (int x = 0; x < QF; ++x) {
            float mb = fmaxf(fmaxf(sf[x][0][0], sf[x][0][1]), fmaxf(sf[x][0][2], sf[x][0][3]));
#pragma unroll
            for (int f = 1; f < KF; ++f)
                mb = fmaxf(fmaxf(mb, fmaxf(sf[x][f][0], sf[x][f][1])), fmaxf(sf[x][f][2], sf[x][f][3]));
            mb = g4_max(mb);
            const float mn = fmaxf(m[x], mb * scale_log2);
            if (__builtin_amdgcn_ballot_w64(mn != m[x])) {   // a running max moved: rescale this query set
                const float alpha = __builtin_amdgcn_exp2f(m[x] - mn);   // 0 on the first block (m = -inf)
                l[x] *= alpha;
#pragma unroll
                for (int d = 0; d < DF; ++d)
#pragma unroll
                    for (int e = 0; e < 4; ++e) oc[x][d][e] *= alpha;
                m[x] = mn;
            }
            const fa_f32x2 sc2 = {scale_log2, scale_log2}, nm2 = {-mn, -mn};
            fa_f32x2 acc2 = {0.f, 0.f};
#pragma unroll
            for (int f = 0; f < KF; ++f)
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
                    fa_f32x2 t = (fa_f32x2){sf[x][f][e], sf[x][f][e + 1]} * sc2 + nm2;
                    t.x = __builtin_amdgcn_exp2f(t.x);
                    t.y = __builtin_amdgcn_exp2f(t.y);
                    sf[x][f][e] = t.x;
                    sf[x][f][e + 1] = t.y;
                    acc2 = acc2 + t;
                }
            l[x] += acc2.x + acc2.y;
        }
#pragma unroll
        for (int j = 0; j < KF / 2; ++j) {
            la_bf16x8 bp[QF];
#pragma unroll
            for (int x = 0; x < QF; ++x)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    bp[x][e] = (__bf16)sf[x][2 * j][e];
                    bp[x][4 + e] = (__bf16)sf[x][2 * j + 1][e];
                }
#pragma unroll
            for (int d = 0; d < DF; ++d) {
                const la_bf16x8 av = xa_tr8_perm<FA_RS>(sv + (32 * j) * FA_RS + 16 * d, lane);
#pragma unroll
                for (int x = 0; x < QF; ++x) oc[x][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bp[x], oc[x][d], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int x = 0; x < QF; ++x) {
        float sum = l[x];
        sum = g4_sum(sum);
        const int qr = q0 + 16 * x + r16;
        if (qr < Nq) {
            const float inv = 1.0f / sum;
            unsigned short* dst = o + (int64_t)b * o_bs + (int64_t)qr * ldo + (int64_t)h * FA_HD + 4 * g;
#pragma unroll
            for (int d = 0; d < DF; ++d) {
                u16x4m t;
#pragma unroll
                for (int e = 0; e < 4; ++e) t[e] = f2b(oc[x][d][e] * inv);
                *reinterpret_cast<u16x4m*>(dst + 16 * d) = t;
            }
        }
    }
}

extern "C" int eggroll_flash_attention_sel(const void* q, int64_t q_bs, int64_t ldq, const void* k, int64_t k_bs,
                                           int64_t ldk, const void* v, int64_t v_bs, int64_t ldv, int64_t B,
                                           int64_t heads, int64_t Nq, int64_t Lk, int64_t head_dim, float scale, void* o,
                                           int64_t o_bs, int64_t ldo, int32_t qf, void* stream) {
    EGG_CHECK_ARG(qf == 0 || qf == 1 || qf == 2 || qf == 4, "flash_attention: qf must be 0 (auto), 1, 2 or 4");
    if (qf == 0) qf = 2;
    EGG_CHECK_ARG(head_dim == FA_HD, "flash_attention: head_dim %lld unsupported (128)", (long long)head_dim);
    EGG_CHECK_ARG(B >= 0 && heads > 0 && Nq >= 0 && Lk >= 1, "flash_attention: bad sizes");
    EGG_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0 && q_bs % 8 == 0 && k_bs % 8 == 0 &&
                  v_bs % 8 == 0 && o_bs % 4 == 0 && ldq >= heads * FA_HD && ldk >= heads * FA_HD &&
                  ldv >= heads * FA_HD && ldo >= heads * FA_HD, "flash_attention: bad strides");
    if (B == 0 || Nq == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(q && k && v && o, "flash_attention: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)q & 15) == 0 && ((uintptr_t)k & 15) == 0 && ((uintptr_t)v & 15) == 0 && ((uintptr_t)o & 7) == 0,
                  "flash_attention: q/k/v must be 16-byte aligned, o 8-byte aligned");
    EGG_CHECK_ARG(Nq < (1ll << 31) && Lk < (1ll << 31), "flash_attention: sequence too long");
    const int64_t qwg = 4 * 16 * qf, nqb = (Nq + qwg - 1) / qwg;
    EGG_CHECK_ARG(B * heads * nqb < (1ll << 31), "flash_attention: grid too large");
    auto* kern = qf == 4 ? k_flash_attn<4> : (qf == 1 ? k_flash_attn<1> : k_flash_attn<2>);
    hipLaunchKernelGGL(kern, dim3((unsigned)(B * heads * nqb)), dim3(256), 0, as_stream(stream),
                       (const unsigned short*)q, q_bs, ldq, (const unsigned short*)k, k_bs, ldk,
                       (const unsigned short*)v, v_bs, ldv, (int)heads, (int)Nq, (int)Lk, (int)nqb,
                       scale * 1.4426950408889634f, (unsigned short*)o, o_bs, ldo);
    EGG_CHECK_LAUNCH("flash_attention");
    return EGGROLL_OK;
}

extern "C" int eggroll_flash_attention(const void* q, int64_t q_bs, int64_t ldq, const void* k, int64_t k_bs,
                                       int64_t ldk, const void* v, int64_t v_bs, int64_t ldv, int64_t B, int64_t heads,
                                       int64_t Nq, int64_t Lk, int64_t head_dim, float scale, void* o, int64_t o_bs,
                                       int64_t ldo, void* stream) {
    return eggroll_flash_attention_sel(q, q_bs, ldq, k, k_bs, ldk, v, v_bs, ldv, B, heads, Nq, Lk, head_dim, scale, o,
                                       o_bs, ldo, 0, stream);
}

// ------------------------------------------------------------------------------------
// GroupNorm (+ SiLU) on NHWC bf16 activations (the FLUX / Infinity VAE decoders' GroupNorm(32)):
//   y[b, p, c] = act((x - mean[b, g]) * rstd[b, g] * w[c] + bias[c]),  g = c / (C / G),
// statistics over the H*W pixels and C/G channels of (b, g), biased variance, fp32 data path.
// Three launches: (1) per (image, pixel chunk) partial per-group sums / sums of squares (fp32 over at most
// 256 x C/G values, reduced in a fixed order), (2) per (image, group) the chunks combined in fp64 ->
// mean, rstd, (3) normalise + affine + act, 16-B loads / stores.  The torch form (an fp32 copy,
// Welford statistics, four elementwise passes) moved ~10x the bytes.
// ------------------------------------------------------------------------------------
constexpr int GN_PASSES = 16;   // pixel passes per block: pixels per chunk = (256 / (C / 8)) * GN_PASSES

__global__ __launch_bounds__(256) void k_gn_stats(const unsigned short* __restrict__ x, int64_t HW, int C, int G,
                                                  int ppc, int nch, float2* __restrict__ part) {
    __shared__ float red[256][17];
    __shared__ float chs[2048][2];
    const int tid = threadIdx.x, tpp = C / 8, pps = 256 / tpp;   // threads per pixel, pixels per pass
    const int b = blockIdx.x / nch, ch = blockIdx.x - b * nch;
    const int slot = tid % tpp, pl = tid / tpp;
    float s[8], q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = q[i] = 0.f;
    if (pl < pps) {
        const int64_t p0 = (int64_t)ch * ppc;
#pragma unroll 4
        for (int k = 0; k < GN_PASSES; ++k) {
            const int64_t p = p0 + (int64_t)k * pps + pl;
            if (p < HW) {
                const u16x8m v = *reinterpret_cast<const u16x8m*>(x + ((int64_t)b * HW + p) * C + slot * 8);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float f = b2f(v[i]);
                    s[i] += f;
                    q[i] += f * f;
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        red[tid][i] = s[i];
        red[tid][8 + i] = q[i];
    }
    __syncthreads();
    // channel c = 8 slot + i: sum over the pixel lanes pl (fixed order)
    for (int c = tid; c < C; c += 256) {
        const int sl = c >> 3, i = c & 7;
        float a = 0.f, a2 = 0.f;
        for (int l = 0; l < pps; ++l) {
            a += red[l * tpp + sl][i];
            a2 += red[l * tpp + sl][8 + i];
        }
        chs[c][0] = a;
        chs[c][1] = a2;
    }
    __syncthreads();
    const int cpg = C / G;
    for (int g = tid; g < G; g += 256) {
        float a = 0.f, a2 = 0.f;
        for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
            a += chs[c][0];
            a2 += chs[c][1];
        }
        part[((int64_t)b * nch + ch) * G + g] = float2{a, a2};
    }
}

__global__ __launch_bounds__(256) void k_gn_finalize(const float2* __restrict__ part, int G, int nch, double count,
                                                     float eps, float2* __restrict__ stats) {
    // one workgroup per (image, group): the chunk partials strided over the threads, then a fixed tree
    __shared__ double sa[256], sq[256];
    const int i = blockIdx.x, b = i / G, g = i - b * G, tid = threadIdx.x;
    double a = 0.0, a2 = 0.0;
    for (int c = tid; c < nch; c += 256) {
        const float2 v = part[((int64_t)b * nch + c) * G + g];
        a += v.x;
        a2 += v.y;
    }
    sa[tid] = a;
    sq[tid] = a2;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (tid < h) {
            sa[tid] += sa[tid + h];
            sq[tid] += sq[tid + h];
        }
        __syncthreads();
    }
    if (tid == 0) {
        const double mean = sa[0] / count;
        double var = sq[0] / count - mean * mean;
        var = var > 0.0 ? var : 0.0;
        stats[i] = float2{(float)mean, (float)(1.0 / sqrt(var + (double)eps))};
    }
}

template <int ACT>
__global__ __launch_bounds__(256) void k_gn_apply(const unsigned short* __restrict__ x, int64_t HW, int C, int G,
                                                  const float2* __restrict__ stats,
                                                  const unsigned short* __restrict__ w,
                                                  const unsigned short* __restrict__ bias, int64_t total8,
                                                  unsigned short* __restrict__ y) {
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;   // 8-channel unit
    if (u >= total8) return;
    const int tpp = C / 8, cpg = C / G;
    const int64_t pix = u / tpp;
    const int slot = (int)(u - pix * tpp);
    const int b = (int)(pix / HW);
    const u16x8m v = *reinterpret_cast<const u16x8m*>(x + u * 8);
    const u16x8m wv = *reinterpret_cast<const u16x8m*>(w + slot * 8);
    const u16x8m bv = *reinterpret_cast<const u16x8m*>(bias + slot * 8);
    u16x8m o;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int c = slot * 8 + i;
        const float2 st = stats[(int64_t)b * G + c / cpg];
        float t = (b2f(v[i]) - st.x) * st.y;
        t = t * b2f(wv[i]) + b2f(bv[i]);
        if (ACT == 1) t = silu(t);
        o[i] = f2b(t);
    }
    *reinterpret_cast<u16x8m*>(y + u * 8) = o;
}

static int64_t gn_chunks(int64_t HW, int C, int* ppc_out) {
    const int ppc = (256 / (C / 8)) * GN_PASSES;
    if (ppc_out) *ppc_out = ppc;
    return (HW + ppc - 1) / ppc;
}

extern "C" int64_t eggroll_group_norm_workspace_bytes(int64_t B, int64_t HW, int32_t C, int32_t G) {
    if (B < 0 || HW < 0 || C < 8 || C % 8 || G < 1 || C % G) return 0;
    return (B * gn_chunks(HW, C, nullptr) * G + B * G) * (int64_t)sizeof(float2);
}

extern "C" int eggroll_group_norm_nhwc(const void* x, int64_t B, int64_t HW, int32_t C, int32_t G, float eps,
                                       const void* w, const void* bias, int32_t act, void* y, void* workspace,
                                       void* stream) {
    EGG_CHECK_ARG(C >= 8 && C <= 2048 && C % 8 == 0 && G >= 1 && C % G == 0, "group_norm: need C %% 8 == 0, C <= 2048, "
                  "C %% G == 0 (C=%d G=%d)", C, G);
    EGG_CHECK_ARG(B >= 0 && HW >= 0 && act >= 0 && act <= 1, "group_norm: bad sizes / act");
    if (B == 0 || HW == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(x && w && bias && y && workspace, "group_norm: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)w & 15) == 0 &&
                  ((uintptr_t)bias & 15) == 0 && ((uintptr_t)workspace & 7) == 0, "group_norm: misaligned pointer");
    int ppc = 0;
    const int64_t nch = gn_chunks(HW, C, &ppc);
    EGG_CHECK_ARG(B * nch < (1ll << 31) && B * G < (1ll << 31) && B * HW * C / 8 / 256 < (1ll << 31),
                  "group_norm: grid too large");
    float2* part = reinterpret_cast<float2*>(workspace);
    float2* stats = part + B * nch * G;
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_gn_stats, dim3((unsigned)(B * nch)), dim3(256), 0, st, (const unsigned short*)x, HW, C, G, ppc,
                       (int)nch, part);
    hipLaunchKernelGGL(k_gn_finalize, dim3((unsigned)(B * G)), dim3(256), 0, st, part, G, (int)nch,
                       (double)HW * (double)(C / G), eps, stats);
    const int64_t total8 = B * HW * C / 8;
    auto* k = act ? k_gn_apply<1> : k_gn_apply<0>;
    hipLaunchKernelGGL(k, dim3((unsigned)((total8 + 255) / 256)), dim3(256), 0, st, (const unsigned short*)x, HW, C, G,
                       stats, (const unsigned short*)w, (const unsigned short*)bias, total8, (unsigned short*)y);
    EGG_CHECK_LAUNCH("group_norm");
    return EGGROLL_OK;
}

// variant: 0 = automatic (the 32-query two-half online-softmax k_cross_attn_h2), 1 = the 16-query two-pass
// k_cross_attn (one max / exp pass over all keys), 2 = k_cross_attn_h2 explicitly.  Both are exact softmax up
// to fp32 rounding; the selector lets the full-size rank test score the same epochs through each form.
extern "C" int eggroll_cross_attention_sel(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv,
                                           const void* bias, const int32_t* enc_index, int64_t B, int64_t N,
                                           int64_t heads, int64_t head_dim, int64_t L, int64_t U, float scale, void* o,
                                           int64_t ldo, int32_t variant, void* stream) {
    EGG_CHECK_ARG(variant >= 0 && variant <= 2, "cross_attention: variant must be 0 (auto), 1 (two-pass) or 2 (online)");
    EGG_CHECK_ARG(head_dim == 64 || head_dim == 80 || head_dim == 112 || head_dim == 128, "cross_attention: head_dim "
                  "%lld unsupported (64, 80, 112, 128)", (long long)head_dim);
    // head dim 128 (Infinity's text cross-attention) stages at most 256 keys: k + v at 320 would not fit 160 KiB
    const int64_t lmax = head_dim == 128 ? XA_LMAX_128 : XA_LMAX;
    EGG_CHECK_ARG(B >= 0 && N > 0 && heads > 0 && L > 0 && L <= lmax, "cross_attention: bad sizes (L <= %lld at head "
                  "dim %lld)", (long long)lmax, (long long)head_dim);
    EGG_CHECK_ARG(U > 0 && U * L < (1ll << 31) && (enc_index || U >= B),
                  "cross_attention: U=%lld caption rows (need U >= B without enc_index)", (long long)U);
    EGG_CHECK_ARG(ldq % 8 == 0 && ldkv % 8 == 0 && ldo % 4 == 0 && ldq >= heads * head_dim &&
                  ldkv >= heads * head_dim && ldo >= heads * head_dim, "cross_attention: bad strides");
    if (B == 0) return EGGROLL_OK;
    EGG_CHECK_ARG(q && k && v && o, "cross_attention: NULL pointer");
    EGG_CHECK_ARG(((uintptr_t)q & 15) == 0 && ((uintptr_t)k & 15) == 0 && ((uintptr_t)v & 15) == 0 && ((uintptr_t)o & 7) == 0,
                  "cross_attention: q/k/v must be 16-byte aligned, o 8-byte aligned");
    EGG_CHECK_ARG(B * heads < (1ll << 31), "cross_attention: grid too large");
    // 8 waves x 16-query blocks (164 VGPRs, 2 waves per SIMD): measured 0.80 ms at the Sana attn2 shape
    // (B 128, N 1024, 20 heads, L 300) vs 0.94 for 4 waves x 32 queries and 1.27 for 4 x 16 (SDPA on
    // the gathered k / v with the mask: 1.53 ms)
    // default: 32-query blocks with the two-half online softmax (k_cross_attn_h2)
#define EGG_XA(HD_, LM_)                                                                                         \
    hipLaunchKernelGGL(variant == 1 ? (k_cross_attn<HD_, 8, 1, LM_>) : (k_cross_attn_h2<HD_, 8, LM_>),           \
                       dim3((unsigned)(B * heads)), dim3(512), 0, as_stream(stream),                              \
                       (const unsigned short*)q, ldq, (const unsigned short*)k, (const unsigned short*)v, ldkv,    \
                       (const unsigned short*)bias, enc_index, (int)heads, (int)N, (int)L, (int)U, scale, (unsigned short*)o, \
                       ldo)
    if (head_dim == 112) EGG_XA(112, XA_LMAX);
    else if (head_dim == 128) EGG_XA(128, XA_LMAX_128);
    else if (head_dim == 80) EGG_XA(80, XA_LMAX);
    else EGG_XA(64, XA_LMAX);
#undef EGG_XA
    EGG_CHECK_LAUNCH("cross_attention");
    return EGGROLL_OK;
}

extern "C" int eggroll_cross_attention(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv,
                                       const void* bias, const int32_t* enc_index, int64_t B, int64_t N,
                                       int64_t heads, int64_t head_dim, int64_t L, int64_t U, float scale, void* o,
                                       int64_t ldo, void* stream) {
    return eggroll_cross_attention_sel(q, ldq, k, v, ldkv, bias, enc_index, B, N, heads, head_dim, L, U, scale, o, ldo,
                                       0, stream);
}
