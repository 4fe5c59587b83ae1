// v_dot2_f32_bf16 semantics check (diagnostic): dot2((x0, x1), (w0, w1), acc) vs fma chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
typedef __attribute__((ext_vector_type(2))) __bf16 bf2;
__global__ void k(const unsigned* xs, const unsigned* ws, const float* accs, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, xs[i]), __builtin_bit_cast(bf2, ws[i]), accs[i], false);
}
static float b2f(unsigned short h) { unsigned u = (unsigned)h << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
    const int n = 1 << 16;
    unsigned *xs = (unsigned*)malloc(n * 4), *ws = (unsigned*)malloc(n * 4);
    float *acc = (float*)malloc(n * 4), *out = (float*)malloc(n * 4);
    srand(1);
    for (int i = 0; i < n; ++i) {
        float a = (rand() / (float)RAND_MAX - 0.5f) * 4, b = (rand() / (float)RAND_MAX - 0.5f) * 4, c = (rand() / (float)RAND_MAX - 0.5f);
        unsigned ua, ub; memcpy(&ua, &a, 4); memcpy(&ub, &b, 4);
        unsigned short x0 = ua >> 16, x1 = (ua >> 8) & 0xffff, w0 = ub >> 16;
        int mode = i % 3;  // 0: (w0, 0); 1: (0, w1); 2: both
        unsigned short wl = mode == 1 ? 0 : w0, wh = mode == 0 ? 0 : (unsigned short)(ub >> 12);
        xs[i] = x0 | ((unsigned)x1 << 16); ws[i] = wl | ((unsigned)wh << 16); acc[i] = c;
    }
    unsigned *dx, *dw; float *da, *dout;
    hipMalloc(&dx, n * 4); hipMalloc(&dw, n * 4); hipMalloc(&da, n * 4); hipMalloc(&dout, n * 4);
    hipMemcpy(dx, xs, n * 4, hipMemcpyHostToDevice); hipMemcpy(dw, ws, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(da, acc, n * 4, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, dw, da, dout, n);
    hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
    int bad[3] = {0, 0, 0}; double maxd[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
        float x0 = b2f(xs[i] & 0xffff), x1 = b2f(xs[i] >> 16), w0 = b2f(ws[i] & 0xffff), w1 = b2f(ws[i] >> 16);
        float ref = i % 3 == 0 ? fmaf(x0, w0, acc[i]) : i % 3 == 1 ? fmaf(x1, w1, acc[i]) : (float)((double)x0 * w0 + (double)x1 * w1 + acc[i]);
        if (memcmp(&ref, &out[i], 4)) { bad[i % 3]++; double d = fabs((double)ref - out[i]); if (d > maxd[i % 3]) maxd[i % 3] = d; }
        if (i < 6) printf("i=%d x=(%g,%g) w=(%g,%g) acc=%g -> %g ref %g\n", i, x0, x1, w0, w1, acc[i], out[i], ref);
    }
    printf("mismatch (w0,0): %d max %g | (0,w1): %d max %g | both vs fp64-sum rounded: %d max %g (of %d each)\n",
           bad[0], maxd[0], bad[1], maxd[1], bad[2], maxd[2], n / 3);
    return 0;
}
