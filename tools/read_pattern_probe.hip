// Read-pattern microbenchmark for the rank-4 ES update's factor stream (tools/read_pattern_probe.py).
// Each workgroup owns a 16-KiB column chunk and walks NROWS factor rows (2 rows per iteration, 8 float4
// loads in flight per thread, as k_update<4> does).  STRIDED: a thread's 64 contiguous bytes as 4 float4
// loads (lane stride 64 B: every load instruction touches 32 cache lines, 32 B of each); COALESCED: load
// c of lane i at 1024 c + 16 i (every instruction one contiguous KiB).  Same bytes, same loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <bool COALESCED>
__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ f, int64_t ld4, int nrows, int64_t nchunks,
                                              float* __restrict__ sink) {
    const int tid = threadIdx.x;
    const int64_t chunk = blockIdx.x;
    if (chunk >= nchunks) return;
    float acc = 0.0f;
    for (int j0 = 0; j0 < nrows; j0 += 2) {
        float4 X[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int64_t q = COALESCED ? (int64_t)(tid >> 6) * 256 + c * 64 + (tid & 63) : (int64_t)tid * 4 + c;
                X[t][c] = f[(int64_t)(j0 + t) * ld4 + chunk * 1024 + q];
            }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc += X[t][c].x * X[t][c].y + X[t][c].z * X[t][c].w;
    }
    if (acc == 1234.5f) sink[blockIdx.x * 256 + tid] = acc;
}

extern "C" int rp_read(const void* f, int64_t ld4, int nrows, int64_t nchunks, int coalesced, int lds_bytes,
                       void* sink, void* stream) {  // lds_bytes: dynamic LDS per workgroup, to cap occupancy
    if (coalesced)
        hipLaunchKernelGGL(k_read<true>, dim3((unsigned)nchunks), dim3(256), (unsigned)lds_bytes, (hipStream_t)stream,
                           (const float4*)f, ld4, nrows, nchunks, (float*)sink);
    else
        hipLaunchKernelGGL(k_read<false>, dim3((unsigned)nchunks), dim3(256), (unsigned)lds_bytes, (hipStream_t)stream,
                           (const float4*)f, ld4, nrows, nchunks, (float*)sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
