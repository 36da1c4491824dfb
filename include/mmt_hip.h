/*
 * mmt_hip.h — C ABI of libmmt_hip.so, the MI355X (gfx950) kernels behind the MixFormer RGB-T
 * tracking forward path.
 *
 * Conventions
 *   - every entry point is `extern "C"`, takes plain device pointers, sizes and a hipStream_t
 *     (passed as void*), allocates nothing, keeps no global state, and returns 0 on success or
 *     a negative status (-hipError_t, or MMT_EBADARG for a rejected shape);
 *   - `dtype` selects the compute/storage type of the matmul operands: MMT_F32 or MMT_BF16
 *     (bf16 operands, fp32 accumulation, fp32 softmax / norm statistics);
 *   - tensors are row-major and contiguous unless a stride argument says otherwise.
 *
 * What each entry replaces in the reference (LZ-QWQ/Multi-modal-Tracking):
 *   mmt_ms_deform_attn_forward  pybind `MultiScaleDeformableAttention.ms_deform_attn_forward`
 *       lib/models/mixformer_vit_rgbt/deformable_attention/ops/src/vision.cpp:13-16,
 *       ms_deform_attn_cuda.cu:20-80 (same tensor meaning; fp64/fp32/bf16)
 *   mmt_ms_deform_attn_backward pybind `MultiScaleDeformableAttention.ms_deform_attn_backward`
 *       (ops/src/vision.cpp:13-16, ms_deform_attn_cuda.cu:83-153, ms_deform_im2col_cuda.cuh:86-235)
 *   mmt_prroi_pool_forward      `_prroi_pooling.prroi_pooling_forward_cuda`
 *       external/PreciseRoIPooling/pytorch/prroi_pool/src/prroi_pooling_gpu.c:22-50,
 *       prroi_pooling_gpu_impl.cu:149-212, 388-400 (plus explicit feature strides)
 *   mmt_prroi_pool_backward / mmt_prroi_pool_coor_backward  `prroi_pooling_backward_cuda`,
 *       `prroi_pooling_coor_backward_cuda` (prroi_pooling_gpu.c:52-113, _impl.cu:214-378)
 *   mmt_gemm                    the eager nn.Linear / 1x1-conv / 3x3-conv (+BN+ReLU) / patch-embed
 *       calls of mixformer.py:26-76, :137-138, fusion_utils.py:252-278, deformable_encoder*.py,
 *       head.py:7-20,159-198, score_decoder.py (implicit GEMM, fused epilogues)
 *   mmt_gemm_multi              several independent mmt_gemm problems in one launch (the head's
 *       parallel conv chains head.py:159-197, the encoder's value / offset Linears)
 *   mmt_mam_attention           Attention.forward MAM softmax(QK^T)V, mixformer.py:52-78 /
 *       asymmetric_shared.py:55-104
 *   mmt_mam_attention_bwd       its autograd (training step, train_script_mixformer*.py)
 *   mmt_transpose_bf16          operand transposes of the Linear backward (nn.Linear autograd)
 *   mmt_adamw_step              gradient clipping + AdamW over every parameter (torch.optim.AdamW)
 *   mmt_layernorm / mmt_groupnorm  nn.LayerNorm / nn.GroupNorm on the hot path
 *   mmt_patch_im2col            PatchEmbed conv input staging, mixformer.py:29-34
 *   mmt_msda_bimodal            MSDeformAttn_Bimodal.forward middle part (offset/weight softmax,
 *       sampling locations, MSDA gather), ms_deform_attn_bimodal.py:97-128
 *   mmt_corner_softargmax       conv5 + pyramid adds + soft_argmax + box_xyxy_to_cxcywh,
 *       head.py:191-212, mixformer.py:419-432
 *   mmt_conv3x3_c1 / mmt_conv3x3_c1_pair  the 1-channel conv-BN-ReLU of adjust3/adjust4,
 *       head.py:115-120 (the pair form runs adjust3[2] and adjust4[1] in one launch)
 *   mmt_spm_attention           ScoreDecoder single-query attention, score_decoder.py:55-61
 *   mmt_ce_t2s_attention / mmt_ce_select / mmt_ce_gather / mmt_ce_recover  candidate elimination
 *       of asymmetric_shared_ce.py:22-102, :198-202, :426-447 (attn_t2s mean, sorted top-k, recover)
 *   mmt_sample_target           the trackers' host crop + preprocessing, processing_utils.py:15-77,
 *       tracker_utils.py:24-48 (cv2 crop/pad/resize, colour map, normalise)
 *   mmt_track_update            map_box_back + clip_box, lib/test/tracker/mixformer_vit_rgbt.py:92-95,
 *       :124-131, lib/utils/box_ops.py:155-164
 */
#ifndef MMT_HIP_H_
#define MMT_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMT_F32 0
#define MMT_BF16 1
#define MMT_F64 2
#define MMT_F16 3 /* fp16 operands, fp32 accumulation (the path of BASELINE config 5); taken by the
                     kernels of the forward plan (GEMM, MAM attention default kernels, norms,
                     patch staging, bimodal MSDA, head); the others return MMT_EBADARG */
#define MMT_EBADARG (-10000)
#define MMT_MAX_GROUPS 2

/* ---------------------------------------------------------------- GEMM / implicit-GEMM conv
 * C[g][m][n] = epi( sum_k A[g](m,k) * W[g][n][k] + bias[g][n] )
 * A addressing (GEMM mode, conv_h == 0):
 *   seg = m / a_seg_rows, A(m,k) = a[g] + (seg % a_segs_a)*a_stride_a + (seg / a_segs_a)*a_stride_b
 *                                  + (m % a_seg_rows)*lda + k        (k <  k_split, or k_split == 0)
 *                                  same with a1[g] and k - k_split       (k >= k_split)
 * A addressing (conv mode, conv_h > 0): NHWC implicit im2col of a 3x3/pad-1 (conv_k3=1) or 1x1
 *   conv producing a conv_h x conv_h map; the input map is conv_h/conv_up square, pixel stride
 *   lda (channels are contiguous, conv_cin of them), k = (ky*3+kx)*conv_cin + ci; consecutive
 *   input images a_stride_a pixels apart (0: packed, (conv_h/conv_up)^2).  conv_k3=2: the 3x3 taps
 *   read in reverse order (input pixel (y+1-ky, x+1-kx)), i.e. the convolution with the flipped
 *   kernel -- the data gradient of a 3x3 conv from its unflipped weights [Cin][ky][kx][Cout].
 * Epilogue: v = act(acc + bias) with act 0 none / 1 GELU(erf) / 2 ReLU / 5 GELU backward:
 *   v = (acc + bias) * GELU'(R) (R then not added; 16-bit LDS-DMA kernels);
 *   c2 == NULL: C = v (+ R if r != NULL);  c2 != NULL: C = v, C2 = v + R (c2_copy 1: C = v (+ R),
 *   C2 = the same values in `dtype`; c2_copy 2: C = v (+ R), C2 = acc + bias, the pre-activation, in
 *   `dtype`, no R needed -- the training step's fc1 keeps it for the GELU backward; c2_copy 3: a
 *   column split, output columns [0, N-8) to C with pitch ldc >= N-8 and the last 8 columns to C2
 *   [M][8] (pitch 8), N % 8 == 0, no R needed -- the training dW GEMM, whose last column is the
 *   bias gradient; c2_copy 4: as 3, but only column N-8 goes to C2, as a contiguous [M] vector (fp32
 *   C); 16-bit LDS-DMA kernels).
 *   R row index: r_mode 0 -> m, 1 -> m % r_p0, 2 -> conv map m=(b,y,x) of an r_p0 x r_p0 map read
 *   at (y / r_p1, x / r_p1) of an (r_p0/r_p1)^2 map.  R is fp32 (or dtype if r_t); C/C2 are fp32
 *   if c_f32 else dtype.
 */
typedef struct {
    const void* a[MMT_MAX_GROUPS];
    const void* a1[MMT_MAX_GROUPS];
    const void* w[MMT_MAX_GROUPS];
    const float* bias[MMT_MAX_GROUPS];
    const float* r[MMT_MAX_GROUPS];
    void* c[MMT_MAX_GROUPS];
    void* c2[MMT_MAX_GROUPS];
    int64_t lda, ldr, ldc;
    int64_t a_seg_rows, a_segs_a, a_stride_a, a_stride_b;
    int32_t M, N, K, k_split;
    int32_t act, c_f32;
    int32_t r_mode, r_p0, r_p1;
    int32_t conv_h, conv_up, conv_cin, conv_k3;
    int32_t groups;
    int32_t r_t;  /* 1: R is stored in `dtype` instead of fp32 */
    int32_t impl; /* kernel choice, results identical up to fp32 summation order: 0 auto;
                     -1 register-staged 64/128 tiles; LDS-DMA (bf16, K % 8 == 0): 1 128x128
                     (8 waves), 2 128x64 (K split over 2 wave groups), 3 64x64 (K split 2),
                     4 128x128 (4 waves), 5 256x128 / 6 128x256 (8 waves, large M), 7 256x256
                     (8 waves, plain GEMM mode only: no ln_fold / conv / split-K), 8 128x128 at two
                     workgroups per CU (64 KiB ring; same restrictions as 7; auto on big unsplit grids),
                     9 (A/B builds only, MMT_GEMM_AB) 256x256 at one wave per SIMD (4 waves of 128x128
                     with AGPR accumulators; plain GEMM mode, ln_fold 0 / 2, row_scale) */
    /* LayerNorm folded into the GEMM (bf16 LDS-DMA kernels, GEMM mode): A holds the raw rows x
     * (K = the LayerNorm width), W = W_lin * gamma (per column k), and the epilogue's v is
     *   rstd_m * (acc - mu_m * ln_colsum[g][n]) + bias[g][n],   mu / rstd over the K values of row m
     * with ln_colsum[n] = sum_k W[n][k] and bias = b_lin + W_lin beta, i.e. Linear(LayerNorm(x)).
     * ln_fold 1: statistics summed from the A fragments in the K loop; 2: read from ln_stats_in. */
    int32_t ln_fold;
    float ln_eps;
    const float* ln_colsum[MMT_MAX_GROUPS];
    /* 1: C2 receives a copy of C (the value C holds, in `dtype`) instead of C = v, C2 = v + R */
    int32_t c2_copy;
    /* Split-K over workgroups (bf16 LDS-DMA kernel, GEMM and conv modes, not with ln_fold): each
     * output tile's K-steps are cut into `splitk` slices computed by separate workgroups; each slice
     * draws an arrival ticket, every slice but the last-arriving one stores its fp32 partial tile in
     * sk_ws, and the last one sums the partials in slice order (bitwise deterministic) and runs the
     * epilogue.  splitk: 0 auto (cost model), 1 off, n >= 2 forced.  sk_ws: fp32 slab workspace of
     * sk_ws_floats floats; sk_cnt: sk_cnt_n uint32 counters (tickets in the first half, published
     * counts in the second), zero before the first launch and left zero by every launch.
     * Without both buffers (or when they are too small for the choice) no split is made. */
    int32_t splitk;
    float* sk_ws;
    int64_t sk_ws_floats;
    uint32_t* sk_cnt;
    int64_t sk_cnt_n;
    /* Output row map (GEMM mode): c_seg_rows > 0 stores logical row m at physical row
     * (m / c_seg_rows) * c_seg_pitch + m % c_seg_rows of C and C2, and reads R there when
     * r_mode == 0 -- e.g. the search rows [n_t, ntok) of every sequence of a [S][ntok] stream
     * (c, c2, r offset by n_t rows; c_seg_rows = ntok - n_t, c_seg_pitch = ntok). 0: identity. */
    int64_t c_seg_rows, c_seg_pitch;
    /* LayerNorm row statistics handed from producer to consumer (16-bit LDS-DMA kernels, GEMM mode):
     *   ln_stats_out[g] != NULL (producer, with c2_copy): for every stored row (output row map
     *     applied) and every 64-column group j of N, (sum, sum of squares) of the C2 values as
     *     stored (16-bit) go to ln_stats_out[g][row][j][0..1] (fp32, N/64 pairs per row);
     *   ln_fold == 2 (consumer): as ln_fold == 1, but mu / rstd of A row m come from
     *     ln_stats_in[g][m][0 .. K/64) (summed in order) instead of sums over the A fragments
     *     in the K loop; the A map must be the identity (one segment, k_split == 0). */
    float* ln_stats_out[MMT_MAX_GROUPS];
    const float* ln_stats_in[MMT_MAX_GROUPS];
    /* MN-major operands (16-bit LDS-DMA kernels, 128x128 tiles; plain GEMM mode: no conv, no LayerNorm
     * fold, identity A map, k_split 0), read with ds_read_b64_tr_b16 instead of a transposed copy:
     *   w_t 1: W given as W^T [K][ldw] (row k holds the N elements of contraction index k) -- the
     *          Linear backward's dX = dY W reads the weight [N_out][K_in] as it is;
     *   w_t 2: as 1 with N - 8 real columns, column N - 8 all ones and N - 7 .. N - 1 zero (with
     *          c2_copy 3: the dW GEMM's bias gradient as the last column block);
     *   a_t 1 (needs w_t): A given as A^T [K][lda] (M % 8 == 0, lda >= M) -- dW = dY^T X reads dY and
     *          X as they are.  K need not be a multiple of 64 (rows past K are zero). */
    int32_t a_t;
    int32_t w_t;
    int64_t ldw;
    /* row_scale != NULL (16-bit LDS-DMA kernels, impl 0 / 8 on the 128x128 two-per-CU tile, no conv / LayerNorm fold /
     * MN-major operands / split-K): v *= row_scale[m / row_scale_div] before R is added
     * (the training step's per-sample stochastic depth on a residual branch, x + keep_b / (1 - p) * f(x)) */
    const float* row_scale;
    int32_t row_scale_div;
    int32_t pad_;
} mmt_gemm_params;

int mmt_gemm(const mmt_gemm_params* p, int dtype, void* stream);

/* n (1..4) independent GEMMs / convolutions ps[0..n-1] (each as mmt_gemm; none may write what
 * another reads) in ONE launch when the 16-bit LDS-DMA kernel takes them all in one tile shape
 * (all GEMM or all conv mode, no folded LayerNorm, equal impl; split-K is not used), else one
 * launch each.  The tile shape is chosen for the union, so results equal mmt_gemm's up to the fp32
 * summation order of the tile shape (bit-identical for an equal forced impl).  The frame plan uses
 * it for the corner head's parallel conv chains (lib/models/mixformer_cvt/head.py:159-197: conv3
 * beside adjust3[0]; conv4 beside adjust4[0] and adjust3[1]) and the encoder's value / offset
 * Linears (ops/modules/ms_deform_attn_bimodal.py:103-110), which are independent and a few
 * workgroups each. */
int mmt_gemm_multi(const mmt_gemm_params* ps, int n, int dtype, void* stream);

/* ---------------------------------------------------------------- MAM attention
 * qkv: [S][ntok][3*C] (dtype) as produced by the fused qkv Linear (reshape(B,N,3,H,d) order);
 * out: [S][ntok][C].  Queries [0,n_t) attend keys [0,n_t) of their own sequence; queries
 * [n_t,ntok) attend all ntok keys (asym == 0) or [tmpl(V) | tmpl(I) | own search] (asym == 1;
 * sequence s of modality m = s / Bm, batch b = s % Bm).  Head dim C/H must be 64.
 */
typedef struct {
    const void* qkv;
    void* out;
    int32_t S, Bm, ntok, n_t, C, H, asym;
    float scale;
    int32_t impl; /* bf16 kernel choice (results equal within bf16 rounding): 0 auto (bf16: the
                     latency kernel 4 below ~200 throughput workgroups, 21 up to ~900, 22 from
                     there; the training forward (lse) 21 on large grids (round 6), fp16 8);
                     2 / 4 = latency kernel, key tiles split over 2 / 4 groups of 4 waves;
                     8 = running-maximum throughput kernel (128 queries per workgroup, 3 per CU);
                     9 = 8 with a 3-deep ring, 2 workgroups per CU; 10-12 = 32x32x16 variants of 8;
                     16-19 = range-checked exponent kernel variants, 17 = its MFMA row-sum form;
                     20 = persistent whole-pair kernel (ViT-B 128/320 shape only);
                     21 = 17 with its two key blocks per tile software-pipelined;
                     22 = 21's math with 64 queries per wave (bf16; writes no lse).
                     q may arrive pre-multiplied by scale*log2(e); then pass scale = 1/log2(e). */
    float* lse;   /* NULL, or [S][H][ntok] fp32: per query the log2-sum-exp2 of its pre-scaled scores
                     (training forward, bf16 only; impls 0 / 4 / 8 / 17 / 21) */
    int32_t q_part; /* 0: all queries; 1: template queries [0,n_t) only; 2: search queries
                       [n_t,ntok) only -- the template K/V cache: template rows of qkv computed
                       once per template update, only the search rows per frame.  Rows of `out`
                       outside the part are not written. */
    int32_t tok_pitch; /* rows between consecutive sequences in qkv / out; 0 = ntok.  Candidate
                       elimination keeps each sequence's rows at the original pitch and runs on
                       its first ntok (template + surviving search) rows (not with lse). */
    int32_t out_pitch; /* rows between consecutive sequences in out; 0 = as qkv (tok_pitch / ntok) */
    int32_t out_q0;    /* query stored at row 0 of a sequence's out rows (0: row = query index).  The
                          template K/V cache passes store compact activations: the template pass
                          (q_part 1) out_pitch n_t, out_q0 0; the search pass (q_part 2) out_pitch
                          ntok - n_t, out_q0 n_t.  Not with lse. */
} mmt_attn_params;

int mmt_mam_attention(const mmt_attn_params* p, int dtype, void* stream);

/* MAM attention backward (training, two-stream / shared layout: asym must be 0; bf16).  qkv / out
 * as in the forward (q NOT pre-scaled: pass the natural `scale`), dout = dL/dout [S][ntok][C], lse
 * from the forward with the same qkv and scale; delta: [S][H][ntok] fp32 workspace; dqkv:
 * [S][ntok][3C] = (dL/dq, dL/dk, dL/dv) in the qkv layout.  Deterministic (no atomics).
 * Replaces the autograd of Attention.forward, mixformer.py:52-78. */
typedef struct {
    const void* qkv;
    const void* out;
    const void* dout;
    const float* lse;
    float* delta;
    void* dqkv;
    int32_t S, Bm, ntok, n_t, C, H, asym;
    float scale;
} mmt_attn_bwd_params;

int mmt_mam_attention_bwd(const mmt_attn_bwd_params* p, int dtype, void* stream);

/* ---------------------------------------------------------------- norms / elementwise
 * LayerNorm over the last dim C (C % 256 == 0) of fp32 rows; x = in[row] (+ add[row % add_rows]);
 * gamma/beta chosen per group = (row / rows_per_group) % 2 (2 groups that alternate every
 * rows_per_group rows: the modality halves of a [2][...] stream, or of each sequence's [2][h*w]
 * token block in the fusion encoder).  Writes out_f32 and/or out_t (dtype) when non-NULL.
 */
int mmt_layernorm(const float* in, const float* add, int64_t add_rows, float* out_f32, void* out_t,
                  const float* gamma0, const float* beta0, const float* gamma1, const float* beta1,
                  int64_t rows, int64_t rows_per_group, int C, float eps, int dtype, void* stream);

/* LayerNorm backward (training step; forward = mmt_layernorm without `add`): x [rows][C] fp32 = the
 * LayerNorm input, dy [rows][C] in dy_dtype (bf16 / fp16 / fp32) = the output gradient, gamma per row
 * group as the forward ((row / rows_per_group) % 2; gamma1 NULL: one group).  dx [rows][C] fp32 = rstd * (g - mean(g) - xhat *
 * mean(g * xhat)), g = dy * gamma (statistics recomputed from x, eps as the forward).  dgb = fp32
 * [groups][2][C]: (dgamma, dbeta) of each group = column sums of dy * xhat and dy over its rows, summed
 * in a fixed order (bitwise reproducible), added to dgb if dgb_accumulate.  ws: fp32 workspace of
 * >= ceil(rows / 32) * 4 * C floats.  Replaces aten's layer_norm backward in the training step
 * (timm Block norm1 / norm2, mixformer.py:129-138; the per-modality norm*_v / norm*_i of the shared
 * backbone, mixformer_shared.py:143-159). */
int mmt_layernorm_bwd(const float* x, const void* dy, int dy_dtype, const float* gamma0, const float* gamma1,
                      float* dx, float* dgb, int dgb_accumulate, float* ws, int64_t ws_floats, int64_t rows,
                      int64_t rows_per_group, int C, float eps, void* stream);

/* mmt_layernorm_bwd with a second gradient of the LayerNorm input added in the same pass: dx = (the
 * LayerNorm backward as above) + dres, dres [rows][C] fp32 (may be dx itself).  The pre-LN block's residual
 * stream feeds the LayerNorm and the residual add (x + f(LN(x)), mixformer.py:136-139): its two gradients meet
 * here instead of in an extra elementwise pass over the stream. */
int mmt_layernorm_bwd_add(const float* x, const void* dy, int dy_dtype, const float* gamma0, const float* gamma1,
                          const float* dres, float* dx, float* dgb, int dgb_accumulate, float* ws, int64_t ws_floats,
                          int64_t rows, int64_t rows_per_group, int C, float eps, void* stream);

/* GroupNorm over [n_inst][P][Ctot] fp32 (channels-last, P positions, Ctot channels in `groups`
 * equal groups), per-instance affine set chosen by inst / inst_per_set (2 sets max).  Outputs
 * fp32 and/or dtype copies with the same layout. */
int mmt_groupnorm(const float* in, float* out_f32, void* out_t, const float* gamma0, const float* beta0,
                  const float* gamma1, const float* beta1, int n_inst, int inst_per_set, int P, int Ctot,
                  int groups, float eps, int dtype, void* stream);

/* GroupNorm backward (training step; forward = mmt_groupnorm with one affine set), channels-last fp32
 * [n_inst][P][Ctot] x (the GroupNorm input) and dy; dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) per
 * (instance, group), g = dy * gamma[c]; dgb = fp32 [2][Ctot] (dgamma, dbeta) = sums over instances and
 * positions of dy * xhat and dy (fixed order: bitwise reproducible), added to dgb if dgb_accumulate.
 * ws: >= n_inst * 2 * Ctot floats.  Limits: Ctot / groups a multiple of 4 and <= 256, P * Ctot / groups
 * <= 24576 (the group's x and dy in registers).  The fusion's adjust_v / adjust_i / adjust_cat GroupNorms (fusion_utils.py:252-279). */
int mmt_groupnorm_bwd(const float* x, const float* dy, const float* gamma, float* dx, float* dgb, int dgb_accumulate,
                      float* ws, int64_t ws_floats, int n_inst, int P, int Ctot, int groups, float eps, void* stream);

/* out_t[i] = (dtype) in[i] (+ add[i % add_n] if add) for n elements; also writes out_f32 = in+add
 * when out_f32 != NULL. */
int mmt_add_cast(const float* in, const float* add, int64_t add_n, float* out_f32, void* out_t, int64_t n,
                 int dtype, void* stream);

/* out[r][c] = (dtype) (in[r][c] * scale[r / rows_per]) over an fp32 [rows][cols] (cols % 8 == 0, 16-B aligned),
 * dtype MMT_BF16 / MMT_F16: the training step's residual-branch gradient under stochastic depth (the per-sample
 * DropPath scale, mixformer.py:136-139) cast to the GEMM operand type in one pass. */
int mmt_scale_rows_cast(const float* in, const float* scale, int64_t rows_per, void* out, int64_t rows, int64_t cols,
                        int dtype, void* stream);

/* Patch staging for the 16x16/s16 patch-embed conv: for each of S = 2*Bm sequences
 * (modality m = s / Bm, batch b = s % Bm) the row block [tmpl | online | search] of tokens, each row
 * = (c, ky, kx) flattened (3*P*P), from fp32 NCHW images img_t[m], img_o[m], img_s[m].  With
 * img_t1 = img_o1 = img_s1 = NULL: one modality, S = Bm (RGB-only MixFormer). */
int mmt_patch_im2col(const float* img_t0, const float* img_t1, const float* img_o0, const float* img_o1,
                     const float* img_s0, const float* img_s1, void* out, int Bm, int ht, int hs, int patch,
                     int dtype, void* stream);

/* ---------------------------------------------------------------- deformable attention
 * Reference-op replacement: value (N,S,M,D), spatial_shapes (L,2) int64, level_start (L) int64,
 * loc (N,Lq,M,L,P,2), attn (N,Lq,M,L,P) -> out (N,Lq,M*D); dtype MMT_F64 / MMT_F32 / MMT_BF16. */
int mmt_ms_deform_attn_forward(const void* value, const int64_t* spatial_shapes, const int64_t* level_start,
                               const void* sampling_loc, const void* attn_weight, void* out, int N, int S,
                               int M, int D, int Lq, int L, int P, int dtype, void* stream);

/* Reference-op replacement for `ms_deform_attn_backward` (ops/src/vision.cpp:13-16,
 * ms_deform_attn_cuda.cu:83-153): same tensors as the forward plus grad_output (N,Lq,M*D); writes
 * grad_value (N,S,M,D; zeroed here, then accumulated by atomics), grad_loc (N,Lq,M,L,P,2) and
 * grad_attn (N,Lq,M,L,P).  dtype MMT_F64 / MMT_F32 (the reference's dispatch). */
int mmt_ms_deform_attn_backward(const void* value, const int64_t* spatial_shapes, const int64_t* level_start,
                                const void* sampling_loc, const void* attn_weight, const void* grad_output,
                                void* grad_value, void* grad_loc, void* grad_attn, int N, int S, int M, int D,
                                int Lq, int L, int P, int dtype, void* stream);
/* mmt_ms_deform_attn_backward with the grad_value gather chosen: value_impl 0 auto, 1 the 64-pixel-chunk workgroups,
 * 2 one workgroup per (n, m, level) over the whole level (needs Lq * P <= 2048 and every level's H * W <= max_hw
 * <= 1024; auto takes it then).  Both sum each pixel's taps in (sample, tap) order: equal results.  max_hw: an
 * upper bound of the levels' H * W (the plain entry passes S). */
int mmt_ms_deform_attn_backward_impl(const void* value, const int64_t* spatial_shapes, const int64_t* level_start,
                                     const void* sampling_loc, const void* attn_weight, const void* grad_output,
                                     void* grad_value, void* grad_loc, void* grad_attn, int N, int S, int M, int D,
                                     int Lq, int L, int P, int max_hw, int value_impl, int dtype, void* stream);

/* ---------------------------------------------------------------- candidate elimination
 * asymmetric_shared_ce.py (CE_Block_Shared :228-282, candidate_elimination :52-102,
 * get_token_from_attn :22-46, _recover_search :426-447).  Token streams are [S][tok_pitch][C]
 * with S = 2*Bm sequences, modality-major; a stage keeps each sequence's first n_t + keep rows.
 *   mmt_ce_t2s_attention: partial[Bm][H][2*n_t/QB][2*n_s] (QB = 16 for MMT_BF16, 8 for MMT_F32)
 *     column sums of the template->search
 *     softmax (qkv [S][tok_pitch][3C], q/k in place; scale in natural-log units, i.e. 1/log2(e)
 *     when q carries scale*log2(e) already);
 *   mmt_ce_t2s_attention_masked: the same with ce_template_mask (candidate_elimination :81-89,
 *     lib/utils/ce_utils.py:14-38 generate_mask_cond): template_mask[Bm][2*n_t] bytes in the query
 *     order [q_mt_V ; q_mt_I] (nonzero = the query's softmax row enters the sums; NULL = all);
 *     mean_scale of mmt_ce_select is then 1 / (H * masked queries per frame);
 *   mmt_ce_select: sums the partials (into each frame's first partial row, so `partial` is
 *     overwritten) and ranks each modality's n_s tokens by the sum (desc, ties by index)
 *     and keeps `keep`: order[S][ns_full] (slot -> current row - n_t), gidx_out = original search
 *     positions (gidx_in NULL = identity), attn_mean[Bm][2*n_s] = sums * mean_scale (NULL = not
 *     written);
 *   mmt_ce_gather: xc rows [0, n_t + keep) of every sequence = x's template rows then the kept
 *     rows in order (xn, if not NULL, gets the same rows cast to xn_dtype);
 *   mmt_ce_recover: out rows [n_t, n_t + ns_full) = x's surviving rows (slots [0, keep) of the
 *     final gidx) at their original positions, zeros where pruned (dtype MMT_BF16 / MMT_F32). */
int mmt_ce_t2s_attention(const void* qkv, float* partial, int Bm, int tok_pitch, int n_t, int n_s, int C, int H,
                         float scale, int dtype, void* stream);
int mmt_ce_t2s_attention_masked(const void* qkv, float* partial, const unsigned char* template_mask, int Bm,
                                int tok_pitch, int n_t, int n_s, int C, int H, float scale, int dtype, void* stream);
int mmt_ce_select(float* partial, int nparts, int Bm, int n_s, int keep, int ns_full, const int* gidx_in,
                  int* gidx_out, int* order, float* attn_mean, float mean_scale, void* stream);
int mmt_ce_gather(const float* x, float* xc, void* xn, const int* order, int S, int tok_pitch, int n_t, int keep,
                  int ns_full, int C, int xn_dtype, void* stream);
int mmt_ce_recover(const float* x, const int* gidx, int keep, void* out, int S, int tok_pitch, int n_t, int ns_full,
                   int C, int dtype, void* stream);

/* Bimodal encoder layer core (ms_deform_attn_bimodal.py:97-128) for nq queries per modality on an
 * hw x hw map, 8 heads x 64 ch, 2 levels x 4 points: offw[b*nq+q][192] fp32 = [sampling_offsets
 * (128) | attention logits (64)] from the [q_v | q_i] Linear; value [2][B][nq][512] (dtype);
 * out[b*nq+q][512] (dtype) -- identical for both modalities, as in the reference. */
int mmt_msda_bimodal(const float* offw, const void* value, void* out, int B, int hw, int dtype, void* stream);
/* Training form of the bimodal MSDA middle (ms_deform_attn_bimodal.py:97-128 in the training step,
 * mmt_amd.train.fusion_forward; 8 heads x 2 levels x 4 points, 64 channels per head, levels hw x hw, nq = hw^2
 * <= 484), bf16 in and out: a = softmax(awl) per (query, head), loc = ref + off / hw, out = the sampled sum
 * (msda_generic_kernel's arithmetic).  value [B][2][nq][512], off [B][nq][128], awl [B][nq][64], ref fp32
 * [nq][2], out [B][nq][512]; off / awl rows (and grad_off / grad_awl rows) off_pitch / awl_pitch elements apart
 * (the [offsets | logits] columns of one Linear output: pitch 192).  Backward: grad_value (deterministic per-pixel gather), grad_off = gloc / hw,
 * grad_awl = the softmax backward of the per-sample weight gradients, all bf16. */
int mmt_msda_bimodal_train_fwd(const void* value, const void* off, int off_pitch, const void* awl, int awl_pitch,
                               const float* ref, void* out, int B, int hw, void* stream);
int mmt_msda_bimodal_train_bwd(const void* value, const void* off, int off_pitch, const void* awl, int awl_pitch,
                               const float* ref, const void* grad_out, void* grad_value, void* grad_off, void* grad_awl,
                               int B, int hw, void* stream);

/* ---------------------------------------------------------------- corner head / SPM
 * Cout=1 3x3/pad-1 conv (+bias, BN folded) + ReLU on NHWC input [G][B][h*h][cin] (pixel stride
 * in_stride) -> out fp32 [G][B][h*h]. */
int mmt_conv3x3_c1(const void* in, const void* w, const float* bias, float* out, int G, int B, int h,
                   int cin, int64_t in_stride, int dtype, void* stream);
/* mmt_conv3x3_c1 of two independent convolutions (same G, B, cin; own input, weights, size and
 * pixel stride) in one launch: the corner head's adjust3[2] and adjust4[1] (head.py:115-120). */
int mmt_conv3x3_c1_pair(const void* in0, const void* w0, const float* bias0, float* out0, int h0, int64_t in_stride0,
                        const void* in1, const void* w1, const float* bias1, float* out1, int h1, int64_t in_stride1,
                        int G, int B, int cin, int dtype, void* stream);

/* score(p) = x4[g][b][p] . w5[g] + b5[g] + a3[g][b][up4(p)] + a4[g][b][up2(p)] on an fh x fh map
 * (g = 0 top-left, 1 bottom-right), softmax over the map, expectation of stride*col / stride*row,
 * / (fh*stride).  score_maps: [2][B][fh*fh] fp32 workspace, left holding the two score maps.
 * boxes_cxcywh / boxes_xyxy: [B][4] fp32.  If rois != NULL also writes the score-head RoIs
 * [B][5] = (b, box_cxcywh_to_xyxy(cxcywh) * roi_scale) (asymmetric_shared_online.py:409,
 * score_decoder.py:38-44).  x4 channels c4 must be a multiple of 8 (bf16) / 4 (fp32). */
int mmt_corner_softargmax(const void* x4, const float* w5, const float* b5, const float* a3, const float* a4,
                          float* score_maps, float* boxes_cxcywh, float* boxes_xyxy, float* rois, float roi_scale,
                          int B, int fh, int c4, int stride, int dtype, void* stream);

/* Training (train.py _HipCornerScore; head.py:191-192): ONE corner branch's score map, with its backward.
 * score_map[b][p] fp32 = (x4[b][p] . w5 + b5) + a3[b][up4(p)] + a4[b][up2(p)]: x4 bf16 [B][fh*fh][c4] (NHWC
 * rows, c4 % 8 == 0), w5 [c4] / b5 [1] fp32 (conv5 in fp32), a3 / a4 bf16 1-channel maps of (fh/4)^2 /
 * (fh/2)^2 pixels at pixel strides s3 / s4 (elements).  The backward writes dx4 bf16 [B][fh*fh][c4], da3 /
 * da4 bf16 rows of p3 / p4 channels (1..8: channel 0 the gradient, the padding channels 0), dw5 [c4] / db5 [1] fp32 (deterministic: fixed-order partial sums through ws, which
 * holds mmt_corner_score_train_ws_floats(B, fh, c4) floats); fh <= 128, c4 < 64.  Replaces the reference
 * path's Conv2d(48, 1, 1) + two F.interpolate + adds (and aten's / hipBLASLt's kernels for them). */
int mmt_corner_score_train(const void* x4, const float* w5, const float* b5, const void* a3, int64_t s3,
                           const void* a4, int64_t s4, float* score_map, int B, int fh, int c4, void* stream);
int64_t mmt_corner_score_train_ws_floats(int B, int fh, int c4);
int mmt_corner_score_train_bwd(const float* dsm, const void* x4, const float* w5, void* dx4, void* da3, int p3,
                               void* da4, int p4, float* dw5, float* db5, float* ws, int B, int fh, int c4, void* stream);

/* PrRoIPool2D forward.  features fp32 with strides (batch, channel, y, x) in elements, rois
 * [R][5] = (batch, x0, y0, x1, y1); out element (r, c, ph, pw) at r*o_r + c*o_c + (ph*pw_+pw)*o_p
 * (the reference's [R][C][ph][pw] is o_r = C*ph*pw, o_c = ph*pw, o_p = 1). */
int mmt_prroi_pool_forward(const float* features, const float* rois, float* out, int R, int C, int H, int W,
                           int64_t s_b, int64_t s_c, int64_t s_h, int64_t s_w, int ph, int pw,
                           float spatial_scale, int64_t o_r, int64_t o_c, int64_t o_p, void* stream);

/* `prroi_pooling_backward_cuda` / `prroi_pooling_coor_backward_cuda` (prroi_pooling_gpu.c:52-107,
 * prroi_pooling_gpu_impl.cu:214-378): contiguous NCHW features (B,C,H,W) fp32, rois (R,5).
 * _backward zeroes grad_features (B,C,H,W) and accumulates it by atomics; _coor_backward writes
 * grad_rois (R,5) (column 0 = 0) from the forward's output `out` (R,C,ph,pw). */
int mmt_prroi_pool_backward(const float* rois, const float* grad_out, float* grad_features, int B, int R, int C, int H,
                            int W, int ph, int pw, float spatial_scale, void* stream);
int mmt_prroi_pool_coor_backward(const float* features, const float* rois, const float* out, const float* grad_out,
                                 float* grad_rois, int R, int C, int H, int W, int ph, int pw, float spatial_scale,
                                 void* stream);

/* ScoreDecoder attention: q [B][C] fp32 (one query per batch), kv [B][Lk][2C] fp32 (k | v),
 * H heads of C/H (= 64), scale; out [B][C] fp32 (dtype copy optional via out_t). */
int mmt_spm_attention(const float* q, int64_t q_stride, const float* kv, float* out, int B, int Lk, int C, int H,
                      float scale, void* stream);

/* ---------------------------------------------------------------- tracker pre/post-processing
 * mmt_sample_target replaces the per-frame host path of the RGB-T trackers
 *   sample_target (lib/train/data/processing_utils.py:15-77, cv2.copyMakeBorder + cv2.resize) +
 *   Preprocessor_wo_mask / Preprocessor_Multimodal.process (lib/test/tracker/tracker_utils.py:24-48)
 * for n (<= MMT_MAX_CROPS) crops of equal out_sz in one launch.  The crop box comes from the
 * device-resident box (x, y, w, h) in fp64, exactly as the tracker state: crop_sz =
 * ceil(sqrt(w*h)*factor), x1 = round-half-even(x + w/2 - crop_sz/2).  out: [3][out_sz][out_sz] fp32
 * = ((v / 255) - mean) / std of the resized uint8 crop v (after the colour map `lut` if non-NULL:
 * BGR2GRAY then lut[gray][c], the cv2.applyColorMap(COLORMAP_JET) step).  Optional: patch
 * [out_sz][out_sz][3] uint8 (sample_target's crop), crop [4] fp64 = (x1, y1, crop_sz,
 * resize_factor = out_sz / crop_sz).
 */
#define MMT_MAX_CROPS 4
typedef struct {
    const uint8_t* image; /* [H][W][3] uint8 frame (HWC, as the tracker receives it) */
    int32_t H, W;
    const double* box;  /* [4] x, y, w, h */
    double factor;      /* search_area_factor (template_factor / search_factor) */
    int32_t out_sz;     /* output_sz */
    const uint8_t* lut; /* NULL or [256][3] */
    float mean[3], std[3];
    float* out;
    uint8_t* patch;
    double* crop;
} mmt_crop_params;

int mmt_sample_target(const mmt_crop_params* p, int n, void* stream);

/* Box post-processing of the trackers (lib/test/tracker/mixformer_vit_rgbt.py:92-95, :124-131;
 * lib/utils/box_ops.py:155-164): for each of n trackers, pred = pred_cxcywh[i] * search_size /
 * resize_factor (fp32, as torch computes it), map_box_back against state[i] (fp64 x, y, w, h) and
 * crop[i][3] = resize_factor, clip_box(H, W, margin); the result replaces state[i]. */
int mmt_track_update(const float* pred_cxcywh, const double* crop, double* state, int n, int H, int W,
                     int search_size, double margin, void* stream);

/* ---------------------------------------------------------------- training-step helpers
 * bf16 transpose: out[b][c][r] = in[b][r][c] for a rows x cols matrix (leading dimensions ld_in /
 * ld_out in elements, `batch` matrices stride_in / stride_out elements apart).  Feeds the Linear
 * backward's dX = dY W and dW = dY^T X GEMMs (both contract over a non-contiguous dimension). */
int mmt_transpose_bf16(const void* in, void* out, int rows, int cols, int64_t ld_in, int64_t ld_out, int batch,
                       int64_t stride_in, int64_t stride_out, int fill, void* stream);
/* fill: 0 writes out[c][r] for r < rows only; 1 also zeros in the padding columns [rows, ld_out); 2 (batch 1)
 * as 1 plus 8 appended output rows, row `cols` = 1.0 over [0, rows) and the rest zero (the ones row of
 * the dW GEMM that also yields the bias gradient) -- the whole padded operand in one launch. */

/* 3x3 / pad-1 im2col of an NHWC bf16 map [B][H][W][C] (C % 8 == 0): out[(b*H + y)*W + x][(ky*3 + kx)*C + c]
 * = in[b][y+ky-1][x+kx-1][c], zero outside the map -- the implicit-GEMM conv's A layout, materialised for
 * the corner head's weight gradients in the training step (dW = dY^T im2col(X), one GEMM over pixels;
 * replaces the autograd of nn.Conv2d 3x3 in lib/models/mixformer_cvt/head.py:7-20). */
int mmt_im2col3x3_bf16(const void* in, void* out, int B, int H, int W, int C, void* stream);
/* The same of the nearest-upsampled (x up: 1, 2, 4 or 8) map of in [B][H/up][W/up][C]; H, W the upsampled sizes
 * (the training head's upsampling folded into its convolutions, head.py:187-189). */
int mmt_im2col3x3_up_bf16(const void* in, void* out, int B, int H, int W, int C, int up, void* stream);
/* The same with channel-major columns, out[pix][c * 9 + ky * 3 + kx] (PyTorch's Conv2d weight order, so the dW
 * GEMM against it writes the [Cout][Cin][3][3] gradient directly); up 1, 2, 4 or 8 as above. */
int mmt_im2col3x3_cm_bf16(const void* in, void* out, int B, int H, int W, int C, int up, void* stream);
/* The training head's 3x3 conv weights to the bf16 operand layouts of its convs, up to MMT_WPREP_MAX convs in
 * one launch (once per step, instead of two cast / permute copies per conv): w fp32 [cout][cin][3][3] ->
 * wf bf16 [cp][3][3][cin] (forward) and wb bf16 [cin][3][3][cp] (dX), co in [cout, cp) zero; bp (optional)
 * fp32 [cp] = b padded with zeros (b NULL: zeros). */
#define MMT_WPREP_MAX 24
typedef struct mmt_conv_wprep {
    const float* w;
    const float* b;
    void* wf;
    void* wb;
    float* bp;
    int32_t cout, cp, cin, pad_;
} mmt_conv_wprep;
typedef struct mmt_conv_wprep_batch {  /* kernel argument (by value) */
    mmt_conv_wprep item[MMT_WPREP_MAX];
    int32_t blk0[MMT_WPREP_MAX];
    int32_t n;
} mmt_conv_wprep_batch;
int mmt_conv3x3_wprep(const mmt_conv_wprep* items, int n, void* stream);

/* The training step's deformable-encoder glue (deformable_encoder_lnspecific.py:131-160,
 * ms_deform_attn_bimodal.py:97-128; mmt_amd.train.fusion_forward), one pass each, fp32 streams / bf16 branches:
 *   mmt_ft_query_prep: src [B][2][nq][d], lpos [2][nq][d] -> qbi [B][nq][2d] = bf16(src + lpos) of both halves
 *     side by side (the bimodal query), srcb = bf16(src); _bwd: dsrc = dthrough (optional) + unshuffle(dqbi) +
 *     dsrcb, dlpos [2][nq][d] = the batch sum of unshuffle(dqbi) (fixed order).
 *   mmt_ft_drop_residual: out [B][rows][d] = x + bf16(dropout(y)); dup: y [B][rows/2][d] on both halves;
 *     _bwd: dy = bf16(dropout'(bf16(dout))), dup: the halves' sum.
 *   mmt_ft_relu_drop: out = bf16(dropout(h)) (h >= 0, the ReLU epilogue's output); _bwd: dh = (h > 0) ?
 *     bf16(dropout'(dy)) : 0.
 * Dropout: keep with probability 1 - p (16-bit draws from a counter hash of rng = {seed, counter} on the device,
 * the call site's salt and the element index), survivors * 1 / (1 - p); rng NULL or p == 0: no dropout. */
/* The training step's corner read-out and box loss (head.py:176-177, :200-212; actors/mixformer_rgbt.py:127-168
 * with lib/utils/box_ops.py:100-152), fp32:
 *   mmt_corner_boxes: score_tl / score_br [B][fh*fh] -> xyxy [B][4] = the soft-argmax expectations (coordinates
 *     stride * (col, row)) times 1 / img_sz; stats [B][2][4] (max, sum of exp, E[x], E[y]) for the backward;
 *     _bwd: dscore = the softmax backward of d xyxy's expectation gradient.
 *   mmt_box_loss: pred cxcywh [B][4], gt xywh [B][4] -> out[4] = (iou_w mean(1 - CIoU) + l1_w mean|pred - gt|, the
 *     CIoU loss, the L1, the mean IoU) on xyxy boxes (gt clamped to [0, 1]); _bwd: dpred [B][4] from dloss[0]. */
int mmt_corner_boxes(const float* score_tl, const float* score_br, float* xyxy, float* stats, int B, int fh,
                     float stride, float img_sz, void* stream);
int mmt_corner_boxes_bwd(const float* score_tl, const float* score_br, const float* stats, const float* dxyxy,
                         float* dscore_tl, float* dscore_br, int B, int fh, float stride, float img_sz, void* stream);
int mmt_box_loss(const float* pred, const float* gt, float* out, int B, float iou_w, float l1_w, void* stream);
int mmt_box_loss_bwd(const float* pred, const float* gt, const float* dloss, float* dpred, int B, float iou_w,
                     float l1_w, void* stream);
/* mmt_ft_rows_cast: out [S][nrows][C] bf16 = the rows [row0, row0 + nrows) of x [S][rows][C] fp32 (the backbones'
 * search tokens as the fusion's adjust Linears read them, mixformer.py:256-259 -> fusion_utils.py:270-275); _bwd: dx
 * [S][rows][C] fp32 = dout on those rows, 0 elsewhere. */
int mmt_ft_rows_cast(const float* x, void* out, int S, int rows, int row0, int nrows, int C, void* stream);
int mmt_ft_rows_cast_bwd(const void* dout, float* dx, int S, int rows, int row0, int nrows, int C, void* stream);
int mmt_ft_query_prep(const float* src, const float* lpos, void* qbi, void* srcb, int B, int nq, int d, void* stream);
int mmt_ft_query_prep_bwd(const void* dqbi, const void* dsrcb, const float* dthrough, float* dsrc, float* dlpos, int B,
                          int nq, int d, void* stream);
int mmt_ft_drop_residual(const float* x, const void* y, float* out, const int64_t* rng, int salt, float p, int B,
                         int rows, int d, int dup, void* stream);
int mmt_ft_drop_residual_bwd(const float* dout, void* dy, const int64_t* rng, int salt, float p, int B, int rows, int d,
                             int dup, void* stream);
int mmt_ft_relu_drop(const void* h, void* out, const int64_t* rng, int salt, float p, int64_t n, void* stream);
int mmt_ft_relu_drop_bwd(const void* dy, const void* h, void* dh, const int64_t* rng, int salt, float p, int64_t n,
                         void* stream);
/* Backward of nearest upsampling x up on NHWC bf16: out [B][Hi][Wi][C] = the up x up block sums of in
 * [B][Hi*up][Wi*up][C] (fp32 sums in a fixed order, bf16 out). */
int mmt_upsample_sum_bf16(const void* in, void* out, int B, int Hi, int Wi, int C, int up, void* stream);
/* out [B][H][W][C] = bf16(up(a) + b), a [B][H/up][W/up][C], NHWC bf16 (the pyramid add up2(adjust2) + x3). */
int mmt_add_up_bf16(const void* a, const void* b, void* out, int B, int H, int W, int C, int up, void* stream);

/* BatchNorm2d (+ ReLU) of the corner head's conv() blocks in the training step (nn.BatchNorm2d -> nn.ReLU,
 * lib/models/mixformer_cvt/head.py:7-20) on an NHWC bf16 map x [M = B*H*W][pitch] with C valid channels
 * (pitch >= C a multiple of 8, <= 2048, 16-B aligned) -> y bf16 [M][pitch] = relu?((x - mean) * invstd *
 * gamma + beta), padding channels 0.  training: batch mean and
 * biased variance over the M rows (fixed-order sums: bitwise reproducible), and when running_mean /
 * running_var are given they are updated in place as nn.BatchNorm2d does (momentum, unbiased variance);
 * else (eval) the running statistics normalise.  save: fp32 [4][C] (mean, invstd, scale, shift), kept
 * for the backward.  ws: >= mmt_batchnorm_ws_floats(M, C) floats (training only).  gamma / beta may be
 * NULL (1 / 0). */
int64_t mmt_batchnorm_ws_floats(int64_t M, int C);
int mmt_batchnorm_relu(const void* x, void* y, int64_t M, int C, int pitch, const float* gamma, const float* beta,
                       float* running_mean, float* running_var, float momentum, float eps, int training, int relu,
                       float* save, float* ws, int64_t ws_floats, void* stream);
/* Its backward: dy bf16 [M][pitch] -> dx bf16 [M][pitch] (through the ReLU mask recomputed from x and save), dgb fp32
 * [2][C] = (dgamma, dbeta) (fixed order).  training: dx = gamma * invstd * (g - mean(g) - xhat *
 * mean(g * xhat)); eval: gamma * invstd * g.  ws: >= mmt_batchnorm_ws_floats(M, C) floats. */
int mmt_batchnorm_relu_bwd(const void* x, const void* dy, void* dx, int64_t M, int C, int pitch, const float* gamma,
                           const float* save, int training, int relu, float* dgb, float* ws, int64_t ws_floats,
                           void* stream);

/* AdamW update with global-norm gradient clipping (torch.nn.utils.clip_grad_norm_
 * + torch.optim.AdamW's fused form over the reference's parameter groups, train_script_mixformer.py:
 * 105-140, base_functions.py:362-400).  Device tables: one entry per fp32 parameter tensor (p, its
 * gradient g, the moments m / v, an optional bf16 shadow written with the updated p, the element
 * count n and its parameter group) and a list of chunks of mmt_adamw_chunk_elems() elements (the
 * entry and the chunk's first element), one workgroup each.
 *   mmt_adamw_step: with max_norm > 0, partial[i] = sum of g^2 over chunk i (nchunks floats of
 *     workspace); then the device state (32 B, zeroed before the first step) is advanced:
 *     state[0] = total L2 norm (partials summed in chunk order), state[1] = c = min(1, max_norm /
 *     (norm + 1e-6)) (1 without clipping), t = ++step (int32 at state[4]), state[2] = 1 - b1^t,
 *     state[3] = sqrt(1 - b2^t); then per element, g' = c g, group lr / wd (HOST arrays of ngroups
 *     values, copied into the launch):  p *= 1 - lr wd; m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2;
 *     p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps); zero_grad: g = 0 afterwards.
 *     No host-side state: a captured hipGraph of the step replays correct steps. */
#define MMT_ADAMW_MAX_GROUPS 8
typedef struct mmt_adamw_tensor {
    float* p;
    float* g;
    float* m;
    float* v;
    uint16_t* shadow; /* bf16 copy of p after the update, or NULL */
    int64_t n;
    int32_t group;
    int32_t pad_;
} mmt_adamw_tensor;
typedef struct mmt_adamw_chunk {
    int32_t tensor;
    int32_t pad_;
    int64_t offset;
} mmt_adamw_chunk;
int mmt_adamw_chunk_elems(void);
int mmt_adamw_step(const mmt_adamw_tensor* tensors, const mmt_adamw_chunk* chunks, int nchunks, float* partial,
                   float* state, const float* lr, const float* weight_decay, int ngroups, double beta1, double beta2,
                   double eps, float max_norm, int zero_grad, void* stream);

/* Library version string (for diagnostics). */
const char* mmt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MMT_HIP_H_ */
