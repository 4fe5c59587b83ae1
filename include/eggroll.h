/*
 * eggroll.h — C-ABI of the MI355X-native EGGROLL ES engine (libeggroll.so).
 *
 * This is the drop-in boundary for the reference's ES hot path
 * (amit154154/HyperscaleES_T2I, `unifed_es.py:89-314` es_step_unified on top of
 * `utills.py:14-136` EggRollNoiser, `utills.py:310-349` fitness shaping / caps, and the
 * PEFT LoRA linear injected at `es_backend.py:193-200`).  The reference is pure Python;
 * these entry points are what its `ctypes` binding would call.
 *
 * Conventions (all entry points):
 *   - every pointer is a caller-allocated DEVICE pointer unless the name ends in `_host`;
 *   - work is stream-ordered on `stream` (a hipStream_t, NULL = default stream);
 *   - no internal allocation, no host synchronisation (graph-capturable);
 *   - no process-global mutable state (kernel choices are per-call arguments): calls on
 *     different threads / streams are independent (thread-safe per stream);
 *   - return 0 on success, negative on error; eggroll_last_error() gives a message
 *     (thread-local);
 *   - deterministic: identical inputs give bit-identical outputs, independent of which
 *     rank/device evaluates which member (noise is a pure function of (seed, base member,
 *     factor element)).
 *
 * Noise model (reference `utills.py:43-106`): every parameter MATRIX P (m x n) gets
 *   E = a b^T / sqrt(r),  a in R^{m x r}, b in R^{n x r}, entries iid N(0,1);
 * 1-D parameters get dense iid N(0,1) noise (reference fallback `utills.py:63-66`).
 * Antithetic layout (`utills.py:88-105`): with h = pop/2, member k uses base sample
 *   j = k (k < h, sign +), j = k-h (h <= k < 2h, sign -), j = h (k = 2h, odd pop, sign +).
 * Non-antithetic: member k uses base sample k with sign +.
 */
#ifndef EGGROLL_H_
#define EGGROLL_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EGGROLL_OK 0
#define EGGROLL_ERR_ARG (-1)
#define EGGROLL_ERR_LAUNCH (-2)
#define EGGROLL_ERR_UNSUPPORTED (-3)

/* One trainable parameter inside the flat theta vector (reference `utills.py:141-162`:
 * theta = concat of module.parameters() with requires_grad, row-major views).
 * Passed to kernels as a DEVICE array of n_mats records (int64 fields).
 * Factor layout of one base sample (the noise kernel fills the whole padded vector): a matrix's
 * a [rows][r] starts at factor_off, its b [cols][r] at factor_off + pad4(rows*r) (pad4(x) = x
 * rounded up to a multiple of 4); a 1-D param's numel values start at factor_off.  Hosts place
 * every factor_off at a multiple of 4 (segments padded to 4 floats) so the kernels move factors
 * as 16-byte vectors; other offsets are accepted and run the per-element path.                 */
typedef struct eggroll_mat {
    int64_t rows;       /* m: first dim (or numel for a 1-D param)                    */
    int64_t cols;       /* n: second dim; 0 marks a 1-D param (dense Gaussian noise)  */
    int64_t theta_off;  /* element offset of this param in theta                       */
    int64_t factor_off; /* element offset of its factors in one base sample's factor   *
                         * vector (see the layout note above)                          */
    int64_t chunk_off;  /* informational: prefix count of EGGROLL_CHUNK-element chunks */
    int64_t reserved;
} eggroll_mat_t;

/* One workgroup's share of perturb / update: matrix `mat`, tile `index` inside it.  Built on the
 * host by eggroll_tile_table (depends on the mats records and the egg rank) and passed as a
 * DEVICE array: the kernels find their matrix with one load instead of a search.              */
typedef struct eggroll_tile {
    int32_t mat;
    int32_t index;
} eggroll_tile_t;

/* Host function (host pointers, no GPU work): writes the tile table of mats_host for egg rank
 * `rank` into tiles_host[0, capacity) and returns the tile count (call with tiles_host = NULL to
 * size it); negative on a bad argument.                                                        */
int64_t eggroll_tile_table(const eggroll_mat_t* mats_host, int32_t n_mats, int32_t rank,
                           eggroll_tile_t* tiles_host, int64_t capacity);

#define EGGROLL_CHUNK 1024

/* Library identification. */
const char* eggroll_version(void);
const char* eggroll_last_error(void);

/* (1) Noise factors — replaces `torch.randn` calls of `EggRollNoiser._sample_low_rank_block`
 * (utills.py:59-65).  Counter-based Philox4x32-10 keyed by `seed` (the epoch, as in
 * unifed_es.py:120-122), counter = (element/4, base member j, 0xE6606011).  Writes
 * out[(j - base_lo) * ld + g] = N(0,1) for j in [base_lo, base_hi), g in [0, factor_len).
 * ld >= factor_len, ld % 4 == 0.                                                        */
int eggroll_noise_factors(uint64_t seed, int64_t base_lo, int64_t base_hi, int64_t factor_len,
                          int64_t ld, float* out, void* stream);

/* Debug/parity: raw Philox4x32-10 words for (seed, j, quads [0, n_quads)). out: 4*n_quads u32. */
int eggroll_philox_words(uint64_t seed, int64_t j, int64_t n_quads, uint32_t* out, void* stream);

/* Perturb — replaces `theta_k = theta + sigma * eps[k]` (unifed_es.py:160) and, with
 * theta == NULL and sigma == 1, materialises eps rows (EggRollNoiser.sample_eps,
 * utills.py:70-106).  For members k in [member_lo, member_hi):
 *   out[(k - member_lo) * ld_out + d] = theta[d] + sigma * s_k * E_{j(k)}[d]
 * with E computed as (sum_q a[i,q] b[c,q]) / sqrt(r) in fp32 (reference op order).
 * factors: base samples [0, n_base) with row stride ld_f (as written by noise_factors,
 * base_lo = 0), 16-byte aligned, ld_f % 4 == 0.  mats: device array of n_mats records; tiles:
 * device array of the n_tiles records eggroll_tile_table built for (mats, rank); D = total theta
 * length.  16-byte aligned theta / out with ld_out % 4 == 0 take the vector path.               */
int eggroll_perturb(const float* theta, const float* factors, int64_t ld_f, int64_t n_base,
                    const eggroll_mat_t* mats, const eggroll_tile_t* tiles, int64_t n_tiles,
                    int64_t D, int32_t rank,
                    int32_t pop, int32_t antithetic, int64_t member_lo, int64_t member_hi,
                    float sigma, float* out, int64_t ld_out, void* stream);

/* Perturb with the noise REGENERATED in the kernel (north_star kernel (1)): the same result as
 * eggroll_noise_factors(seed, 0, n_base, ...) followed by eggroll_perturb on those factors, bit for
 * bit, but every factor value is recomputed (Philox4x32-10 + Box-Muller of its counter) where it is
 * consumed — no factor buffer is written or read.  Replaces torch.manual_seed(epoch) +
 * EggRollNoiser.sample_eps + theta + sigma * eps[k] (unifed_es.py:120-160).                     */
int eggroll_perturb_seeded(uint64_t seed, const float* theta, const eggroll_mat_t* mats,
                           const eggroll_tile_t* tiles, int64_t n_tiles, int64_t D, int32_t rank,
                           int32_t pop, int32_t antithetic, int64_t member_lo, int64_t member_hi,
                           float sigma, float* out, int64_t ld_out, void* stream);

/* (3) Fitness — replaces paper_prompt_normalized_scores (utills.py:310-330) or
 * S.mean(dim=1) (unifed_es.py:234), the finite mask (unifed_es.py:236-240,266),
 * standardize_fitness (utills.py:168-178) and the rank sort (unifed_es.py:244).
 * S: [n, m] fp32 row-major; promptnorm_eps = the `eps` of paper_prompt_normalized_scores
 * (sigma_bar.clamp_min(eps), reference default 1e-8).  Outputs (device):
 *   scores[n], mu[m] (promptnorm column means; S column means otherwise),
 *   stats[4] = {sigma_bar (NaN if promptnorm off), n_finite, mean_f, std_f},
 *   fitness[n] (z-scored over finite members; 0 for non-finite members),
 *   finite[n] (0/1), order[n] = stable ascending argsort of scores (NaN last).
 * Single workgroup; n <= 4096, m <= 1024.                                                 */
int eggroll_fitness(const float* S, int32_t n, int32_t m, int32_t use_promptnorm,
                    float promptnorm_eps, float* scores, float* mu, float* stats, float* fitness, int32_t* finite,
                    int32_t* order, void* stream);

/* (4) Update — replaces EggRollNoiser.do_update (utills.py:115-136) followed by
 * cap_step_norm and cap_theta_norm (utills.py:333-349, unifed_es.py:280-281):
 *   theta_out = theta + (lr_scale*sigma) * (1/N_f) * sum_k f_k eps_k
 * evaluated in factor form as a rank-(n_base*r) reduction per matrix (antithetic pairs
 * collapsed: c_j = f_j - f_{j+h}).  N_f is read from stats[1] (device, written by
 * eggroll_fitness); N_f == 0 leaves theta unchanged, caps included (unifed_es.py:237-240).
 * max_step_norm / theta_max_norm <= 0 disable the caps; with both disabled the update is ONE
 * launch, else a second launch reduces the per-tile norms in a fixed order and rescales only
 * if a cap triggers.  tiles / n_tiles as for eggroll_perturb.
 * workspace: >= eggroll_update_workspace_bytes(n_tiles) bytes, 16-byte aligned.
 * theta_out may not alias theta.                                                          */
int64_t eggroll_update_workspace_bytes(int64_t n_tiles);
int eggroll_update(const float* theta, const float* factors, int64_t ld_f, int64_t n_base,
                   const float* fitness, const float* stats, int32_t pop, int32_t antithetic,
                   const eggroll_mat_t* mats, const eggroll_tile_t* tiles, int64_t n_tiles,
                   int64_t D, int32_t rank, float lr, float max_step_norm, float theta_max_norm,
                   void* workspace, float* theta_out, void* stream);

/* Update with the noise regenerated in the kernel from `seed` (see eggroll_perturb_seeded): the
 * same result as eggroll_update on eggroll_noise_factors(seed, 0, n_base) bit for bit, n_base
 * derived from (pop, antithetic).  The factor read — 4 * n_base * factor_len bytes — is gone.      */
int eggroll_update_seeded(uint64_t seed, const float* theta, const float* fitness, const float* stats,
                          int32_t pop, int32_t antithetic, const eggroll_mat_t* mats,
                          const eggroll_tile_t* tiles, int64_t n_tiles, int64_t D, int32_t rank, float lr,
                          float max_step_norm, float theta_max_norm, void* workspace, float* theta_out,
                          void* stream);


/* eggroll_lora_linear_pop with one elementwise op fused into the GEMM epilogue, applied to the
 * bf16-rounded output y exactly as the separate torch / libeggroll op it replaces would:
 *   epi 1: Y = bf16(silu(y))                       GLUMBConv 1x1 conv -> SiLU (sana.py, dcae.py)
 *   epi 2: Y = bf16(res + y)                       x = x + attn2(...) (Sana block)
 *   epi 3: Y = bf16(res + gate[row/rpg, :] * y)    x += gate_msa * attn1(...) (eggroll_gated_residual)
 *   epi 4: res = res + y                           the same on the fp32 residual stream (res fp32)
 *   epi 5: res = fma(gate[row/rpg, :], y, res)     (res fp32, gate fp32; eggroll_gated_residual_f32)
 *   epi 6: Y = bf16(gelu_tanh(y))                  Infinity ffn fc1 -> GELU(tanh) (x * sigmoid(2k), <= 1 ulp)
 *   epi 7: Y = bf16(res * y)                       Z-Image SwiGLU silu(w1 x) * w3 x (res may alias Y)
 *   epi 8: Y = bf16(gelu(y))                       PickScore CLIP-H/14 mlp fc1 -> exact (erf) GELU (= torch bits)
 * res [M, ldr] bf16 may alias Y; gate rows gstride apart.  epi 4 / 5: res is an fp32 stream updated in
 * place and Y (may be NULL) receives bf16(res).  Requires r <= 2 (and rows_per_member >= 256 when
 * r > 0) and K % 64 == 0: always an MFMA-addend 8-phase kernel.  epi 0 = linear_pop.               */
int eggroll_lora_linear_pop_epi(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                                const float* theta_pop, int64_t ld_theta, int64_t offA, int64_t offB, int32_t r,
                                float scale, int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y,
                                int64_t ldy, float* T_ws, int32_t epi, const void* res, int64_t ldr, const void* gate,
                                int64_t gstride, int64_t rows_per_group, void* stream);
/* The same with an explicit kernel (A/B measurement): 0 = automatic, 8 = the 256x256 8-phase
 * kernel, 10 = the 256x320 8-phase kernel (bit-identical to 8).                                   */
int eggroll_lora_linear_pop_epi_sel(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                                    const float* theta_pop, int64_t ld_theta, int64_t offA, int64_t offB, int32_t r,
                                    float scale, int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y,
                                    int64_t ldy, float* T_ws, int32_t epi, const void* res, int64_t ldr,
                                    const void* gate, int64_t gstride, int64_t rows_per_group, int32_t kernel,
                                    void* stream);
/* The epilogue GEMM alone, with T = X A_k^T already computed (fp32 [M, r], e.g. by
 * eggroll_lora_project / eggroll_lora_project_multi): the second of linear_pop_epi's two launches,
 * bit-identical to it (bench.py times the two apart on the product path).                        */
int eggroll_lora_gemm_epi_sel(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                              const float* T, const float* theta_pop, int64_t ld_theta, int64_t offB, int32_t r,
                              float scale, int64_t rows_per_member, int64_t M, int64_t N, int64_t K, void* Y,
                              int64_t ldy, int32_t epi, const void* res, int64_t ldr, const void* gate,
                              int64_t gstride, int64_t rows_per_group, int32_t kernel, void* stream);
/* (2) Population-batched perturbed LoRA linear — replaces per-member
 * `unflatten_to_params` + PEFT lora.Linear.forward (peft: y = base(x) + B(A x) * alpha/r),
 * members evaluated sequentially in the reference (unifed_es.py:159-163).
 * Rows of X are stacked member-major: row -> member k = member_lo + row / rows_per_member.
 *   Y[row, n] = sum_k X[row,k] W[n,k] + bias[n] + scale * sum_q T[row,q] * Bk[n,q]
 *   T[row, q] = sum_k X[row,k] * Ak[q,k]            (fp32, full-K reduction)
 * Ak = theta_pop[k_local*ld_theta + offA] as [r][K]; Bk = theta_pop[... + offB] as [N][r]
 * (PEFT lora_A.weight / lora_B.weight row-major inside theta_k).
 * X, W, Y bf16 row-major (ldx, ldw, ldy in elements); bias bf16 or NULL; theta_pop fp32.
 * T_ws: workspace of >= eggroll_lora_workspace_bytes(M, K, r, rows_per_member) bytes,
 * 16-byte aligned (fp32 T [M, r] for the two-pass path; bf16 hi/lo A_k images [members][16][K]
 * when the projection is fused into the GEMM: tile 12 forced, r <= 2, rows_per_member >= 256).
 * Requires K % 64 == 0, r <= 16, ldx/ldw % 8 == 0.                                        */
int64_t eggroll_lora_workspace_bytes(int64_t M, int64_t K, int32_t r, int64_t rows_per_member);
int eggroll_lora_linear_pop(const void* X, int64_t ldx, const void* W, int64_t ldw,
                            const void* bias, const float* theta_pop, int64_t ld_theta,
                            int64_t offA, int64_t offB, int32_t r, float scale,
                            int64_t rows_per_member, int64_t M, int64_t N, int64_t K,
                            void* Y, int64_t ldy, float* T_ws, void* stream);

/* Pieces of (2), exported for A/B measurement and for hosts that run the base GEMM
 * elsewhere:  T = X Ak^T per member (fp32); the MFMA GEMM + fused epilogue given T
 * (T may be NULL when r == 0); and Y += scale * T Bk^T (bf16 in place).                  */
int eggroll_lora_gemm(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                      const float* T, const float* theta_pop, int64_t ld_theta, int64_t offB,
                      int32_t r, float scale, int64_t rows_per_member, int64_t M, int64_t N,
                      int64_t K, void* Y, int64_t ldy, void* stream);
/* The same two entry points with an explicit kernel choice (per call; no global state), for A/B
 * measurement: 0 = automatic (as above: the 8-phase 256x256 kernel when the grid fills the chip,
 * else 128x128); 8 = 8-phase with the MFMA LoRA epilogue, 9 = 8-phase with a VALU epilogue,
 * 10 = 8-phase 256x320 tile with the MFMA LoRA epilogue (r <= 2 with rows_per_member >= 256, or
 * r = 0; bit-identical to 8), 128 / 256 = one-barrier tiles; linear_pop_sel also takes 12 = 8-phase
 * with the projection fused into the GEMM (opt-in: slower than the two-pass path at the Sana shapes). */
int eggroll_lora_gemm_sel(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias,
                          const float* T, const float* theta_pop, int64_t ld_theta, int64_t offB,
                          int32_t r, float scale, int64_t rows_per_member, int64_t M, int64_t N,
                          int64_t K, void* Y, int64_t ldy, int32_t kernel, void* stream);
int eggroll_lora_linear_pop_sel(const void* X, int64_t ldx, const void* W, int64_t ldw,
                                const void* bias, const float* theta_pop, int64_t ld_theta,
                                int64_t offA, int64_t offB, int32_t r, float scale,
                                int64_t rows_per_member, int64_t M, int64_t N, int64_t K,
                                void* Y, int64_t ldy, float* T_ws, int32_t kernel, void* stream);
int eggroll_lora_project(const void* X, int64_t ldx, const float* theta_pop, int64_t ld_theta,
                         int64_t offA, int32_t r, int64_t rows_per_member, int64_t M, int64_t K,
                         float* T, void* stream);
/* T = X A^T for n_lin LoRA linears that read the same X (Sana attn1 to_q/to_k/to_v, attn2 to_k/to_v:
 * the PEFT lora_A products of es_backend.py:193-200 sharing one input), X read from HBM once:
 *   T[l*M*r + row*r + q] = sum_k X[row,k] * A_{k,l}[q,k],  A_{k,l} = theta_pop[kl*ld_theta + offA_host[l]]
 * as [r][K] (kl = row / rows_per_member).  MFMA with A split into bf16 hi + lo: each product carries
 * ~2^-16 relative error (the lo part's rounding; fp32 accumulation), so T agrees with the fp32 VALU
 * eggroll_lora_project to ~2^-16 * sum|x||a| per element, not to fp32 rounding and not bit for bit
 * (this is the default projection of the Sana attn1 q/k/v and attn2 k/v linears).
 * offA_host: HOST array of n_lin offsets (multiples of 4).  1 <= n_lin <= 4, n_lin * r <= 8,
 * K % 32 == 0, K <= 4096, ldx % 8 == 0, X and theta_pop 16-byte aligned (16-byte vector loads). */
int eggroll_lora_project_multi(const void* X, int64_t ldx, const float* theta_pop, int64_t ld_theta,
                               const int64_t* offA_host, int32_t n_lin, int32_t r, int64_t rows_per_member,
                               int64_t M, int64_t K, float* T, void* stream);
int eggroll_lora_expand(const float* T, const float* theta_pop, int64_t ld_theta, int64_t offB,
                        int32_t r, float scale, int64_t rows_per_member, int64_t M, int64_t N,
                        void* Y, int64_t ldy, void* stream);
/* The PEFT LoRA term in fp32 for the few small linears the host keeps in fp32 (time / guidance embedders,
 * AdaLN modulation, proj_out; es_backend.py:193-200 evaluated for all members at once):
 *   y[m, :] += scale * (x[m, :] A_k^T) B_k^T,   k = m / rows_per_member,
 * A_k = A + k * lda_member as [r][K] (lora_A), B_k = B + k * ldb_member as [N][r] (lora_B); member strides 0
 * apply one adapter to every row.  x [M][ldx] fp32, y [M][ldy] fp32 (the base x W^T + b, updated in place).
 * One wave per row: x A_k^T by a fixed-order wave reduction (a row's result does not depend on the member
 * count), then y + (T B_k^T) * scale.  1 <= r <= 8. */
int eggroll_lora_delta_f32(const float* x, int64_t ldx, const float* A, int64_t lda_member, const float* B,
                           int64_t ldb_member, int32_t r, float scale, int64_t rows_per_member, int64_t M,
                           int64_t N, int64_t K, float* y, int64_t ldy, void* stream);

/* Model-side fused op of the Sana / DC-AE host (not part of the reference ES interface):
 * channels-last depthwise ks x ks conv (stride 1, zero pad ks/2) of in [B,H,W,C] bf16 with
 * weights w_t [ks*ks][C] bf16 (tap-major), optional bias [C]; pre_silu applies SiLU to the
 * input on load; glu writes out[.., c] = y[c] * silu(y[c + C/2]) for c < C/2 (out [B,H,W,C/2]),
 * else out [B,H,W,C].  Replaces silu(conv_inverted) -> conv_depth -> chunk -> gate of the
 * reference's diffusers GLUMBConv (models/SanaSprint.py transformer FFN and DC-AE blocks).      */
int eggroll_dwconv_nhwc(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H,
                        int64_t W, int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out,
                        void* stream);
/* The DC-AE multi-scale aggregation (diffusers SanaMultiscaleAttentionProjection: depthwise ks x ks
 * conv, no bias, then a grouped 1x1 conv with groups of 32 channels) in one pass:
 *   d = bf16(dwconv(in, w_t)),  out[.., 32g + o] = bf16(sum_c pw[g][o][c] * d[.., 32g + c])
 * in / out [B,H,W,C] bf16 (C % 32 == 0, out may not alias in), pw [C/32][32][32] bf16.          */
int eggroll_dwconv_pw_nhwc(const void* in, const void* w_t, const void* pw, int64_t B, int64_t H,
                           int64_t W, int64_t C, int32_t ks, void* out, void* stream);
/* The two depthwise entries with an explicit block order (per call, for A/B measurement):
 * 0 = automatic, 1 = channel slice fastest, 2 = column sweep (a pair of 32-channel slices, then
 * every row band of the tile column: the halo rows and 128-B lines shared by neighbouring blocks
 * are read by blocks a few ids apart).                                                            */
int eggroll_dwconv_nhwc_sel(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H,
                            int64_t W, int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out,
                            int32_t kernel, void* stream);
int eggroll_dwconv_pw_nhwc_sel(const void* in, const void* w_t, const void* pw, int64_t B, int64_t H,
                               int64_t W, int64_t C, int32_t ks, void* out, int32_t kernel, void* stream);
/* eggroll_dwconv_nhwc_sel with an output row stride ldo (elements, cout <= ldo <= cout + 32,
 * ldo % 8 == 0; cout = glu ? C/2 : C): channels [cout, ldo) of every output pixel are written as
 * zeros.  The Sana FFN's GLU output (5600 channels) is written at ldo 5632 so the point-wise conv
 * runs on the LoRA GEMM (K % 64 == 0) against a zero-padded weight.                             */
int eggroll_dwconv_nhwc_ex(const void* in, const void* w_t, const void* bias, int64_t B, int64_t H,
                           int64_t W, int64_t C, int32_t ks, int32_t pre_silu, int32_t glu, void* out,
                           int64_t ldo, int32_t kernel, void* stream);

/* Model-side fused row normalisation of x [rows, C] bf16 (C % 8 == 0, C <= 4096):
 *   y = (x - mean·layer) * rsqrt(var + eps) [* w] [* (1 + mscale[g])] [+ mshift[g]] [+ b];
 *   y = act(y) (0 none, 1 relu, 2 silu); y += res (optional);  g = row / rows_per_group,
 *   modulation rows mstride elements apart.  Replaces RMSNorm / LayerNorm + AdaLN modulate /
 *   bias / residual chains of the Sana blocks and the DC-AE decoder.                         */
int eggroll_rownorm(const void* x, int64_t rows, int64_t C, float eps, int32_t layer, const void* w,
                    const void* b, const void* mscale, const void* mshift, int64_t mstride,
                    int64_t rows_per_group, int32_t act, const void* res, void* out, void* stream);
/* x[r, :] += gate[r / rows_per_group, :] * y[r, :]  (bf16, in place; gate rows gstride apart). */
int eggroll_gated_residual(void* x, const void* y, const void* gate, int64_t gstride, int64_t rows,
                           int64_t C, int64_t rows_per_group, void* stream);
/* Per-head RMS norm + rotary embedding of x [rows, >= heads*128] bf16 (row stride ldx), in place:
 * y = x * rsqrt(mean_head(x^2) + eps) * w[128], then every adjacent pair (2p, 2p+1) of a head rotated
 * by cos / sin[row % tab_rows][p] (fp32 tables [tab_rows][64]); fp32 math, one bf16 rounding.  The
 * Z-Image q / k path (diffusers ZImageTransformer2DModel: norm_q / norm_k then the 3-axis RoPE).    */
int eggroll_qk_norm_rope(void* x, int64_t ldx, int64_t rows, int32_t heads, int32_t head_dim, float eps,
                         const void* w, const float* cos_tab, const float* sin_tab, int64_t tab_rows, void* stream);
/* The same with (all optional) a per-head output multiplier hscale [heads] fp32, an output other than x —
 * row r of x goes to out[(r / rows_per_seq) * out_bs + (row0 + r % rows_per_seq) * out_ld], a KV-cache
 * slice [seq][ltot][C] — and vin row r (ldv apart) copied to vout at the same position (Infinity's cache
 * append of the tokens' keys and values).                                                              */
int eggroll_qk_norm_rope_kv(void* x, int64_t ldx, int64_t rows, int32_t heads, int32_t head_dim, float eps,
                            const void* w, const float* cos_tab, const float* sin_tab, int64_t tab_rows,
                            const float* hscale, void* out, int64_t out_bs, int64_t out_ld, int64_t rows_per_seq,
                            int64_t row0, const void* vin, int64_t ldv, void* vout, void* stream);
/* The same row normalisation with dtype options: x_f32 = 1: fp32 input x (the fp32 residual stream of
 * the Sana blocks); mod_f32 = 1: fp32 modulation vectors (the fp32 AdaLN modulation); res_f32 = 1: fp32
 * res; out_f32 = 1: fp32 output (the DC-AE fp32 residual stream, out = norm(x)·w + b + res, may alias
 * res) with `shadow` (optional) receiving bf16(out); else out is bf16 and shadow must be NULL.
 * x_f32 with out_f32 is not supported.                                                             */
int eggroll_rownorm_ex(const void* x, int32_t x_f32, int64_t rows, int64_t C, float eps, int32_t layer,
                       const void* w, const void* b, const void* mscale, const void* mshift, int64_t mstride,
                       int32_t mod_f32, int64_t rows_per_group, int32_t act, const void* res, int32_t res_f32,
                       void* out, int32_t out_f32, void* shadow, void* stream);
/* fp32 residual stream update: x = fma(gate[g], y, x) (gate bf16 or fp32 per gate_f32; NULL: x += y),
 * x fp32 [rows, C] in place, y bf16; shadow (optional) receives bf16(x).  The unfused form of the
 * EPI_RES32 / EPI_GATED32 GEMM epilogues (eggroll_lora_linear_pop_epi epi 4 / 5), bit-identical.   */
int eggroll_gated_residual_f32(float* x, const void* y, const void* gate, int32_t gate_f32, int64_t gstride,
                               int64_t rows, int64_t C, int64_t rows_per_group, void* shadow, void* stream);
/* fp32 residual stream + LayerNorm of the CLIP reward towers (one pass per residual point):
 *   h[r, :] += float(y[r, :])  (y bf16, rows ldy apart; y == NULL: no add, h is only read)
 *   out[r, :] = bf16(layer_norm(h[r, :]) * w + b)   fp32 statistics, w / b bf16 [C], out [rows, C]
 * h fp32 rows ldh apart (ldh % 4 == 0), C % 8 == 0, C <= 4096, 16-byte aligned pointers.
 * Replaces `h = h + linear(...).float(); F.layer_norm(h, ..., w.float(), b.float()).to(bf16)` of
 * transformers' CLIPEncoderLayer pre-norm residual (rewards.py:66-158 scorers).                   */
int eggroll_resid_layernorm(float* h, int64_t ldh, const void* y, int64_t ldy, int64_t rows, int64_t C,
                            float eps, const void* w, const void* b, void* out, void* stream);
/* DC-AE up-block shortcut, NHWC: y[b,2h+i,2w+j,c] += x[b,h,w,(4c+2i+j)/(4*Cout/Cin)]
 * (pixel_shuffle(repeat_interleave(x)) without materialising it).                            */
int eggroll_upshortcut_add(void* y, const void* x, int64_t B, int64_t H, int64_t W, int64_t Cin,
                           int64_t Cout, void* stream);

/* DC-AE up-block via sub-pixel phases, NHWC: out[b,2h+i,2w+j,c] = y4[b,h+i,w+j,(2i+j)*Cout+c]
 * (+ bias[c]) + x[b,h,w,(4c+2i+j)/(4*Cout/Cin)], where y4 [B,H+1,W+1,4*Cout] = conv2d(x, 2x2 phase
 * kernels, pad 1, no bias).  Equals conv3x3(nearest_upsample_x2(x)) + bias +
 * pixel_shuffle(repeat_interleave(x)) at 4/9 of the conv FLOPs and without the upsampled tensor
 * (reference DCUpBlock2d).  bias: [Cout] bf16 or NULL (the conv's own bias, added here in fp32 so
 * the phase conv runs without one).                                                            */
int eggroll_subpixel_shortcut(const void* y4, const void* x, const void* bias, void* out, int64_t B,
                              int64_t H, int64_t W, int64_t Cin, int64_t Cout, void* stream);
/* The same on the DC-AE fp32 residual stream: x (shortcut source) and out fp32, shadow (optional)
 * bf16(out); 4 Cout / Cin in {1, 2, 4}, Cin % 8 == 0.                                              */
int eggroll_subpixel_shortcut_f32(const void* y4, const float* x, const void* bias, float* out, void* shadow,
                                  int64_t B, int64_t H, int64_t W, int64_t Cin, int64_t Cout, void* stream);

/* DC-AE decoder head (norm_out + ReLU + conv_out of the reference AutoencoderDC decoder), NHWC:
 *   a[p, c] = bf16(relu(x[p, c] / sqrt(mean_c x[p, :]^2 + eps) * norm_w[c] + norm_b[c]))
 *   y[p, o] = bf16(conv_b[o] + sum_{ky,kx,c} a[p + (ky-1, kx-1), c] * conv_w[o, ky, kx, c])  (zero pad)
 * x [B,H,W,C] bf16 with C = 128; conv_w [3][3][3][C] bf16 (channels-last [Cout, Cin, 3, 3]);
 * conv_b [3] or NULL; y [B,H,W,3] bf16.                                                        */
int eggroll_dcae_head(const void* x, int64_t B, int64_t H, int64_t W, int64_t C, float eps, const void* norm_w,
                      const void* norm_b, const void* conv_w, const void* conv_b, void* y, void* stream);

/* y[row, c] = act(bf16(y[row, c] + bias[c])) in place; y bf16 [rows, C] contiguous, C % 8 == 0,
 * act 0 none / 1 relu / 2 silu.  (Conv bias + activation of the DC-AE ResBlock in one pass.)   */
int eggroll_bias_act(void* y, const void* bias, int64_t rows, int64_t C, int32_t act, void* stream);

/* Dense 3x3 conv, stride 1, zero pad 1, NHWC bf16, as an implicit GEMM on MFMA (DC-AE ResBlock
 * conv1/conv2 of the reference's AutoencoderDC decoder, models/SanaSprint.py:157-160):
 *   y[b, h, x, o] = act(bias[o] + sum_{ky,kx,c} x[b, h+ky-1, x+kx-1, c] * w[o, c, ky, kx])
 * computed on super-pixels of px (1 or 2) horizontally adjacent pixels: w_packed is
 * [N = px*Cout][3][px+2][Cin] bf16 with w_packed[p*Cout + o][ky][tx][c] = w[o, c, ky, tx - p]
 * (zero where tx - p is outside 0..2); bias [N] bf16 (the conv bias repeated px times) or NULL;
 * act 0 none / 2 silu (fp32, before the single bf16 rounding).  Cin a power of two in [64, 2048],
 * N % 64 == 0, W % px == 0.  x [B,H,W,Cin]; y [B,H,W,Cout] contiguous.                          */
int eggroll_conv3x3_nhwc(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H,
                         int64_t W, int64_t Cin, int64_t N, int32_t px, int32_t act, void* y, void* stream);
/* General form: ks x ks conv (ks 2 or 3), zero pad 1, output [B, H+3-ks, W+3-ks, N/px]:
 *   y[b, h, x, o] = act(bias[o] + sum_{ky,kx,c} x[b, h+ky-1, x+kx-1, c] * w[o, c, ky, kx])
 * w_packed [N = px*Cout][ks][px+ks-1][Cin] (px 2 only with ks 3).  ks = 2 is the sub-pixel
 * phase conv of the DC-AE up-blocks (see eggroll_subpixel_shortcut).                          */
int eggroll_conv_nhwc(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H, int64_t W,
                      int64_t Cin, int64_t N, int32_t ks, int32_t px, int32_t act, void* y, void* stream);
/* DC-AE up-block in one launch (round 5): the ks = 2 phase conv above with the sub-pixel interleave,
 * bias and pixel-shuffle shortcut in its epilogue (no [B, H+1, W+1, 4*Cout] intermediate):
 *   out[b, 2h+i, 2w+j, c] = bf16(y4[b, h+i, w+j, (2i+j)*Cout + c]) + bias[c] + src[b, h, w, (4c + 2i+j) / REP]
 * REP = 4*Cout/Cin in {1, 2, 4}; y4 the bias-free phase conv of x (w_packed as eggroll_conv_nhwc, ks 2).
 * src_f32 0: src [B,H,W,Cin] bf16 (= x), out bf16; 1: src fp32 (the DC-AE fp32 residual stream), out fp32
 * and shadow (optional) its bf16 copy.  Bitwise equal to eggroll_conv_nhwc + eggroll_subpixel_shortcut(_f32).
 * Cout % 64 == 0; pointers 16-byte aligned.                                                     */
int eggroll_conv2x2_subpixel_nhwc(const void* x, const void* w_packed, const void* bias, const void* src,
                                  int32_t src_f32, int64_t B, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                  void* out, void* shadow, void* stream);
/* Kernel choice per call: 0 auto, 1 the tap-staged implicit GEMM (any shape above), 2 the halo-
 * staged kernel (ks 3, px 1, H % 16 == 0, and W % 32 == 0 with N == 128 or W % 16 == 0 with
 * N % 256 == 0: the input halo of a 16-row tile is staged once per 32-channel slice instead of once
 * per tap).  Auto picks 2 whenever the shape allows it.  Results agree to fp32 summation order.  */
int eggroll_conv_nhwc_sel(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H, int64_t W,
                          int64_t Cin, int64_t N, int32_t ks, int32_t px, int32_t act, void* y, int32_t kernel,
                          void* stream);
/* The same conv with the ResBlock tail fused into its epilogue (conv2 -> RMSNorm -> + residual):
 *   y[p, c] = bf16(z[p, c] / sqrt(mean_c z[p, :]^2 + eps) * norm_w[c] (+ norm_b[c]) + res[p, c])
 * with z the fp32 conv output (+ bias); requires N = px * Cout = 256 (whole pixels per tile:
 * Cout 128 with px 2, Cout 256 with px 1), or Cout 128 at px 1.  res [B,H,W,Cout] bf16 (may not alias y).         */
int eggroll_conv3x3_rmsnorm_nhwc(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H,
                                 int64_t W, int64_t Cin, int64_t N, int32_t px, float eps, const void* norm_w,
                                 const void* norm_b, const void* res, void* y, void* stream);
int eggroll_conv3x3_rmsnorm_nhwc_sel(const void* x, const void* w_packed, const void* bias, int64_t B, int64_t H,
                                     int64_t W, int64_t Cin, int64_t N, int32_t px, float eps, const void* norm_w,
                                     const void* norm_b, const void* res, void* y, int32_t kernel, void* stream);

/* ReLU linear attention with head dim 32 (diffusers SanaLinearAttnProcessor2_0 and DC-AE
 * SanaMultiscaleLinearAttention): for every image b and head h over its N tokens,
 *   out[n, h*32+i] = sum_j q'[n,j] kv[i][j] / (sum_j q'[n,j] ksum[j] + 1e-15),
 *   kv[i][j] = sum_n v[n,i] k'[n,j],  ksum[j] = sum_n k'[n,j],  x' = relu(x) if relu_qk.
 * q/k/v: bf16 views, element (b*N + n, h, d) at ptr[(b*N+n)*ld + h*hstride + d]; out bf16 with
 * row stride ldo.  fp32 accumulation; workspace >= eggroll_linear_attention_workspace_bytes.   */
int64_t eggroll_linear_attention_workspace_bytes(int64_t B, int64_t N, int64_t heads);
int eggroll_linear_attention(const void* q, const void* k, const void* v, int64_t ld, int64_t hstride,
                             int64_t B, int64_t N, int64_t heads, int32_t relu_qk, void* out, int64_t ldo,
                             void* workspace, void* stream);

/* CLIP image preprocessing of decoder outputs for the reward towers, bit-exact with transformers'
 * CLIPImageProcessor (PIL backend) on the PIL image the reference builds (rewards.py:86-90,133-147):
 *   u8 = mode 0: rint((x/2 + 0.5).clamp(0,1) * 255)    (PixArtImageProcessor.postprocess, Sana)
 *        mode 1: fp16 ((x+1)*0.5).clamp(0,1) * 255, truncated  (models/VAR.py:190, 245-259)
 *        mode 2: bf16 (x+1)/2*255, clamped, truncated        (Infinity's image postprocess)
 *   Pillow BICUBIC 8-bit fixed-point resize to RH x RW (horizontal pass first, clip8 per pass),
 *   center crop out_size^2, out = (u8/255 - mean[c]) / std[c]  fp32 [n, 3, out, out].
 * img: bf16, element (i, c, y, x) at img[i*sn + c*sc + y*sh + x*sw]; tab_w [RW][1+ktw] / tab_h
 * [RH][1+kth] int32 device tables {first input index, taps}; mean / std: 3 floats (host);
 * tmp: device scratch of n*3*H*out_size bytes.                                                  */
int eggroll_clip_preprocess(const void* img, int64_t n, int64_t H, int64_t W, int64_t sn, int64_t sc, int64_t sh,
                            int64_t sw, int32_t mode, const int32_t* tab_w, const int32_t* tab_h, int32_t ktw,
                            int32_t kth, int64_t RW, int64_t RH, int64_t out_size, const float* mean,
                            const float* stdv, void* tmp, void* out, void* stream);

/* Softmax cross-attention over a short key sequence (Sana attn2: diffusers SanaAttnProcessor2_0,
 * F.scaled_dot_product_attention with the caption mask as an additive bias):
 *   o[b,n,h,:] = softmax_j(scale * q[b,n,h,:] . k[u,j,h,:] + bias[u,j]) @ v[u,:,h,:],  u = enc_index[b]
 * q / o bf16 rows b*N + n (head h at columns h*head_dim), k / v bf16 rows u*L + j (U caption rows); bias
 * bf16 [U][L] or NULL; enc_index int32 [B] or NULL (u = b, needs U >= B).  An enc_index entry outside
 * [0, U) gives that image NaN output (no out-of-bounds read).  head_dim 64 / 80 / 112 (112: Sana attn2;
 * 64 / 80: the CLIP towers' self-attention), L <= 320; head_dim 128 (Infinity's text cross-attention,
 * models/Infinity.py CrossAttention), L <= 256.  MFMA, fp32 softmax.                                  */
int eggroll_cross_attention(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv, const void* bias,
                            const int32_t* enc_index, int64_t B, int64_t N, int64_t heads, int64_t head_dim,
                            int64_t L, int64_t U, float scale, void* o, int64_t ldo, void* stream);
/* The same with the kernel form chosen (variant 0: automatic = 2; 1: 16-query blocks, two-pass softmax over all
 * keys; 2: 32-query blocks, online softmax over two key halves) — numerics / timing A/B.                */
int eggroll_cross_attention_sel(const void* q, int64_t ldq, const void* k, const void* v, int64_t ldkv,
                                const void* bias, const int32_t* enc_index, int64_t B, int64_t N, int64_t heads,
                                int64_t head_dim, int64_t L, int64_t U, float scale, void* o, int64_t ldo,
                                int32_t variant, void* stream);

/* GroupNorm over NHWC bf16 activations (+ SiLU when act = 1):
 *   y[b,p,c] = act((x[b,p,c] - mean[b,g]) * rstd[b,g] * w[c] + bias[c]),  g = c / (C / G)
 * statistics over the HW pixels x C/G channels of (b, g) (biased variance, fp32 partial sums combined in
 * fp64); x / y [B][HW][C] bf16 (16-byte aligned, C % 8 == 0, C <= 2048, C % G == 0), w / bias [C] bf16;
 * workspace of eggroll_group_norm_workspace_bytes(B, HW, C, G) bytes (8-byte aligned).  Three launches. */
int64_t eggroll_group_norm_workspace_bytes(int64_t B, int64_t HW, int32_t C, int32_t G);
int eggroll_group_norm_nhwc(const void* x, int64_t B, int64_t HW, int32_t C, int32_t G, float eps, const void* w,
                            const void* bias, int32_t act, void* y, void* workspace, void* stream);

/* Flash attention, head dim 128, no mask (Z-Image self-attention, Infinity's attention over its KV cache):
 *   o[b,n,h,:] = softmax_j(scale * q[b,n,h,:] . k[b,j,h,:]) @ v[b,:,h,:],  n < Nq, j < Lk
 * q / k / v / o bf16, element (b, row, h, d) at X[b * X_bs + row * ldX + h * 128 + d] (a KV cache read in
 * place through its batch stride).  Online softmax in fp32, P rounded to bf16 for the PV MFMA.         */
int eggroll_flash_attention(const void* q, int64_t q_bs, int64_t ldq, const void* k, int64_t k_bs, int64_t ldk,
                            const void* v, int64_t v_bs, int64_t ldv, int64_t B, int64_t heads, int64_t Nq,
                            int64_t Lk, int64_t head_dim, float scale, void* o, int64_t o_bs, int64_t ldo,
                            void* stream);
/* The same with the queries per wave chosen (qf 1: 16, 2: 32, 4: 64; 0: automatic) — A/B measurement. */
int eggroll_flash_attention_sel(const void* q, int64_t q_bs, int64_t ldq, const void* k, int64_t k_bs, int64_t ldk,
                                const void* v, int64_t v_bs, int64_t ldv, int64_t B, int64_t heads, int64_t Nq,
                                int64_t Lk, int64_t head_dim, float scale, void* o, int64_t o_bs, int64_t ldo, int32_t qf,
                                void* stream);

#ifdef __cplusplus
}
#endif
#endif /* EGGROLL_H_ */
