// MFMA shape A/B on gfx950 ("try 32x32x16 for the power-limited main loops").
//
// Two LDS-fed bf16 main loops at the SAME wave output tile as k_conv3x3_halo / k_lora_gemm8n
// (128 x 64 per wave, 8 waves per workgroup = 2 per SIMD, K consumed 32 per step, operands re-read from
// LDS with ds_read_b128 every step, random data):
//   shape 0: 16x16x32 — per step 8 A + 4 B fragments, 32 MFMAs (8 x 4 accumulator tiles of 4 regs)
//   shape 1: 32x32x16 — per step 2 k-halves x (4 A + 2 B fragments), 16 MFMAs (4 x 2 tiles of 16 regs)
// Same FLOPs, same LDS bytes, same accumulator registers.  Prints TF/s by wall (hipEvents over many
// back-to-back launches) and, from a stamped run, the in-kernel clock (s_memtime / s_memrealtime).
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/mfma_shape_probe tools/mfma_shape_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int LDS_BYTES = 64 * 1024;   // 1024 rows x 64 B (32 bf16 of K per row)

__device__ __forceinline__ uint32_t swz(uint32_t L) { return L ^ ((L >> 3) & 32u); }

template <int SHAPE>
__global__ __launch_bounds__(512, 1) void k_probe(const unsigned short* __restrict__ src, int steps, float* out,
                                                  unsigned long long* stamps) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < LDS_BYTES / 16; i += 512)
        reinterpret_cast<uint4*>(smem)[i] = reinterpret_cast<const uint4*>(src)[(blockIdx.x * 97 + i) % (LDS_BYTES / 16)];
    __syncthreads();
    unsigned long long t0 = 0, r0 = 0;
    if (stamps && tid == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    // A rows: wave's 128 pixel rows at wave * 64; B rows: 64 channel rows at 512 + wave * 32 (mod 1024)
    const uint32_t abase = (uint32_t)(wave * 64) * 64, bbase = (uint32_t)(512 + wave * 32) * 64;
    if constexpr (SHAPE == 0) {
        f32x4 acc[8][4];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < steps; ++s) {
            const uint32_t sh = (uint32_t)(s & 7) * 4096u;
            bf16x8 a[8], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                b[j] = *reinterpret_cast<const bf16x8*>(
                    smem + (swz(bbase + ((16 * j + (lane & 15)) * 64) + (lane >> 4) * 16) + sh) % LDS_BYTES);
#pragma unroll
            for (int f = 0; f < 8; ++f)
                a[f] = *reinterpret_cast<const bf16x8*>(
                    smem + (swz(abase + ((16 * f + (lane & 15)) * 64) + (lane >> 4) * 16) + sh) % LDS_BYTES);
#pragma unroll
            for (int f = 0; f < 8; ++f)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[f], acc[f][j], 0, 0, 0);
        }
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
        out[blockIdx.x * 512 + tid] = t;
    } else {
        f32x16 acc[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        for (int s = 0; s < steps; ++s) {
            const uint32_t sh = (uint32_t)(s & 7) * 4096u;
#pragma unroll
            for (int kh = 0; kh < 2; ++kh) {
                bf16x8 a[4], b[2];
                // lane l: row l & 31, k chunk 8 (l >> 5) + 16 kh  (16-B chunk index 2 kh + (l >> 5))
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    b[j] = *reinterpret_cast<const bf16x8*>(
                        smem + (swz(bbase + ((32 * j + (lane & 31)) * 64) + (2 * kh + (lane >> 5)) * 16) + sh) % LDS_BYTES);
#pragma unroll
                for (int f = 0; f < 4; ++f)
                    a[f] = *reinterpret_cast<const bf16x8*>(
                        smem + (swz(abase + ((32 * f + (lane & 31)) * 64) + (2 * kh + (lane >> 5)) * 16) + sh) % LDS_BYTES);
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[f][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[f], acc[f][j], 0, 0, 0);
            }
        }
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) t += acc[i][j][e];
        out[blockIdx.x * 512 + tid] = t;
    }
    if (stamps && tid == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

// One wave per SIMD (4 waves per workgroup, 512-register budget): wave tile 128 x 128, K 32 per step.
// LDS bytes per MFMA-FLOP are 2/3 of the 128 x 64 tile's (16 fragment reads per 64 MFMAs instead of 12 per 32).
// SHAPE 0: 16x16x32 (8 x 8 accumulators of 4), SHAPE 1: 32x32x16 (4 x 4 of 16).
template <int SHAPE>
__global__ __launch_bounds__(256, 1) void k_probe_w1(const unsigned short* __restrict__ src, int steps, float* out,
                                                     unsigned long long* stamps) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < LDS_BYTES / 16; i += 256)
        reinterpret_cast<uint4*>(smem)[i] = reinterpret_cast<const uint4*>(src)[(blockIdx.x * 97 + i) % (LDS_BYTES / 16)];
    __syncthreads();
    unsigned long long t0 = 0, r0 = 0;
    if (stamps && tid == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    const uint32_t abase = (uint32_t)(wave * 128) * 64, bbase = 512u * 64;
    float t = 0.f;
    if constexpr (SHAPE == 0) {
        f32x4 acc[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < steps; ++s) {
            const uint32_t sh = (uint32_t)(s & 7) * 4096u;
            bf16x8 a[8], b[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                b[j] = *reinterpret_cast<const bf16x8*>(
                    smem + (swz(bbase + ((16 * j + (lane & 15)) * 64) + (lane >> 4) * 16) + sh) % LDS_BYTES);
#pragma unroll
            for (int f = 0; f < 8; ++f)
                a[f] = *reinterpret_cast<const bf16x8*>(
                    smem + (swz(abase + ((16 * f + (lane & 15)) * 64) + (lane >> 4) * 16) + sh) % LDS_BYTES);
#pragma unroll
            for (int f = 0; f < 8; ++f)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[f], acc[f][j], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    } else {
        f32x16 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        for (int s = 0; s < steps; ++s) {
            const uint32_t sh = (uint32_t)(s & 7) * 4096u;
#pragma unroll
            for (int kh = 0; kh < 2; ++kh) {
                bf16x8 a[4], b[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    b[j] = *reinterpret_cast<const bf16x8*>(
                        smem + (swz(bbase + ((32 * j + (lane & 31)) * 64) + (2 * kh + (lane >> 5)) * 16) + sh) % LDS_BYTES);
#pragma unroll
                for (int f = 0; f < 4; ++f)
                    a[f] = *reinterpret_cast<const bf16x8*>(
                        smem + (swz(abase + ((32 * f + (lane & 31)) * 64) + (2 * kh + (lane >> 5)) * 16) + sh) % LDS_BYTES);
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[f][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[f], acc[f][j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) t += acc[i][j][e];
    }
    out[blockIdx.x * 512 + tid] = t;
    if (stamps && tid == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 256 * 4;
    const int steps = argc > 2 ? atoi(argv[2]) : 4096;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    std::vector<unsigned short> h(LDS_BYTES / 2);
    unsigned s = 12345u;
    for (auto& v : h) {   // random bf16 in [-2, 2): sign, exponent 126..128, random mantissa
        s = s * 1664525u + 1013904223u;
        v = (unsigned short)(((s >> 16) & 0x8000u) | ((126u + (s >> 8) % 3u) << 7) | ((s >> 1) & 0x7Fu));
    }
    unsigned short* src;
    float* out;
    unsigned long long* st;
    CHECK(hipMalloc(&src, LDS_BYTES));
    CHECK(hipMalloc(&out, (size_t)grid * 512 * 4));
    CHECK(hipMalloc(&st, (size_t)grid * 16));
    CHECK(hipMemcpy(src, h.data(), LDS_BYTES, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double flops = 2.0 * 128 * 64 * 32 * 8 * (double)steps * grid;   // 8 waves x 128x64 tile x 32 K per step
    for (int round = 0; round < 3; ++round) {
        for (int shape = 0; shape < 4; ++shape) {
            auto kern = shape == 0 ? k_probe<0> : shape == 1 ? k_probe<1> : shape == 2 ? k_probe_w1<0> : k_probe_w1<1>;
            const int thr = shape < 2 ? 512 : 256;
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(thr), 0, 0, src, steps, out, nullptr);
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(thr), 0, 0, src, steps, out, nullptr);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(thr), 0, 0, src, steps, out, st);   // stamped run right after
            CHECK(hipDeviceSynchronize());
            std::vector<unsigned long long> hs(2 * grid);
            CHECK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> clk;
            for (int b = 0; b < grid; ++b)
                if (hs[2 * b + 1]) clk.push_back((double)hs[2 * b] / (double)hs[2 * b + 1] * 0.1);   // GHz (100 MHz ref)
            std::sort(clk.begin(), clk.end());
            const double us = 1e3 * ms / reps;
            printf("{\"round\": %d, \"shape\": \"%s\", \"grid\": %d, \"steps\": %d, \"us\": %.1f, \"tflops\": %.1f, "
                   "\"clock_GHz_median\": %.3f}\n",
                   round, shape == 0 ? "16x16x32 128x64/wave 2w/SIMD" : shape == 1 ? "32x32x16 128x64/wave 2w/SIMD"
                   : shape == 2 ? "16x16x32 128x128/wave 1w/SIMD" : "32x32x16 128x128/wave 1w/SIMD", grid, steps, us,
                   flops / (us * 1e6),
                   clk.empty() ? 0.0 : clk[clk.size() / 2]);
            fflush(stdout);
        }
    }
    return 0;
}
