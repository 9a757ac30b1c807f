/*
 * mmni.h — C ABI of the MI355X-native hot path of Transconnectome/multimodal_neuroimage.
 *
 * One shared library, libmmni.so (built for gfx950 by __graft_entry__.build()), exports
 * every entry point below.  The ABI is plain C: device pointers, sizes, strides and a
 * hipStream_t passed as void*.  No torch types cross it.  The library never allocates
 * or frees device memory; outputs, saved-for-backward tensors and gradient accumulators
 * are allocated by the caller (PyTorch on the Python side) and zeroed where documented.
 *
 * Error convention: every int-returning function returns
 *   0  on success,
 *  <0  for a bad argument (shape / stride / unsupported template combination),
 *  >0  a hipError_t from the launch.
 * mmni_last_error() returns a thread-local message describing the last failure.
 *
 * Streams: every launch goes to the caller's stream (torch.cuda.current_stream()).
 * Nothing synchronises the device; every entry point is graph-capturable.
 *
 * Reference interfaces each entry point replaces are cited per function
 * (paths relative to the reference repository root).
 */
#ifndef MMNI_H
#define MMNI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMNI_ABI_VERSION 8

/* ------------------------------------------------------------------------------------
 * Shifted-window attention.
 *
 * Token layout in HBM: channels-last (B, D, H, W, channels); token row
 *   row(b, z, y, x) = ((b*D + z)*H + y)*W + x.
 * The cyclic shift (torch.roll by -shift) and window partition of
 *   modules/swin_v2_module.py:35-46,278  and  modules/swinfusion_module.py:33-45,351
 * are folded into the kernels' addressing: window w = ((b*nWd + wz)*nWh + wy)*nWw + wx,
 * window-local token t = (i*wh + j)*ww + k reads row(b, (wz*wd+i+sd)%D, (wy*wh+j+sh)%H,
 * (wx*ww+k+sw)%W); outputs are written back to the same row, which is exactly the
 * reverse partition + reverse roll (swinfusion_module.py:366-373).
 * 2D reference shapes use D = 1, wd = 1, sd = 0.
 *
 * Element (row, head h, channel c) of q / k / v lives at  ptr[row*stride + h*head_dim + c];
 * a packed qkv projection (B*L, 3C) is passed as q = base, k = base + C, v = base + 2C
 * with all strides 3C; the cross-attention kv projection (B*L, 2C) as k = kv, v = kv + C.
 * ------------------------------------------------------------------------------------ */
typedef struct mmni_wattn_desc {
    int32_t B;                  /* volumes in the batch                                   */
    int32_t D, H, W;            /* spatial extents (D = 1 for the 2D reference shapes)    */
    int32_t C;                  /* channels = heads * head_dim                            */
    int32_t heads;
    int32_t wd, wh, ww;         /* window extent per axis                                 */
    int32_t sd, sh, sw;         /* cyclic shift per axis; 0 = unshifted (no mask)         */
    int32_t kind;               /* 0: SwinFusion scaled dot product + learned table bias
                                      (swinfusion_module.py:114-145, 213-246)
                                   1: Swin-V2 cosine attention, tau per head
                                      (swin_v2_module.py:138-178)                         */
    float   scale;              /* kind 0: q scale (head_dim^-0.5); ignored for kind 1    */
    int64_t q_stride;           /* elements between consecutive token rows of q           */
    int64_t k_stride;
    int64_t v_stride;
    int64_t o_stride;           /* output rows (and dq/dk/dv rows use q/k/v strides)      */
} mmni_wattn_desc;

/* Forward.  table: (Tsz, heads) row-major with Tsz = (2wd-1)(2wh-1)(2ww-1), indexed by
 *   idx = ((dz+wd-1)*(2wh-1) + (dy+wh-1))*(2ww-1) + (dx+ww-1),  d* = query - key coords
 *   (relative_position_index, swinfusion_module.py:93-103).  For kind 1 the caller passes
 *   the already-activated 16*sigmoid(cpb_mlp(relative_coords_table)) (swin_v2_module.py:158-162).
 * tau: kind 1 only, (heads) = exp(min(logit_scale, ln 100)) (swin_v2_module.py:154-156).
 * Shift mask: -100 between tokens of different shift regions (swinfusion_module.py:317-338),
 *   computed analytically from region ids, never materialised.
 * out: rows with o_stride; lse: (B*D*H*W, heads) natural-log softmax normaliser per row. */
int mmni_wattn_fwd(const mmni_wattn_desc* d,
                   const float* q, const float* k, const float* v,
                   const float* table, const float* tau,
                   float* out, float* lse, unsigned int* vmax, void* stream);

/* Backward (flash-style recompute from lse).  dq/dk/dv are fully overwritten (every token
 * belongs to exactly one window).  dtable (Tsz, heads) and dtau (heads) are ACCUMULATED
 * (dtable += grad): the caller zeroes them.  dtau may be NULL for kind 0.
 * workspace: >= mmni_wattn_bwd_workspace_bytes(d) bytes, 8-byte aligned, contents ignored
 * (the library initialises what it uses on the stream).  Either path makes dtable bitwise
 * deterministic:
 *   - row-broadcast path (kind 0, 6x6x6 windows, C == 2*heads): one fp32 partial table row per
 *     workgroup (its waves' private LDS copies summed in a fixed order), then a fixed-order
 *     column sum; vmax is not read;
 *   - every other shape: a 64-bit fixed-point table gradient with a max|dout|,max|v| bound.
 * vmax (both calls, nullable): one uint32 the caller zeroes before the forward; the forward raises
 * it to the float bits of max|v| over the call (folded into the K/V staging), and the backward
 * then scans only dout for the fixed-point bound instead of dout and v.  ABI v2 added it. */
size_t mmni_wattn_bwd_workspace_bytes(const mmni_wattn_desc* d);
int mmni_wattn_bwd(const mmni_wattn_desc* d,
                   const float* q, const float* k, const float* v,
                   const float* table, const float* tau,
                   const float* out, const float* dout, const float* lse,
                   float* dq, float* dk, float* dv,
                   float* dtable, float* dtau, void* workspace, const unsigned int* vmax,
                   void* stream);

/* Integer maps the attention kernels use, exported for bit-exact parity tests (row a0).
 *   mmni_window_rows:   rows[w*N + t] = source token row of window-local token t of window w
 *                       (N = wd*wh*ww, w over all B*nW windows)
 *   mmni_window_mask:   mask[w*N*N + i*N + j] in {0, -100} for the nW windows of ONE sample
 *                       (calculate_mask, swinfusion_module.py:317-338)
 *   mmni_relative_index: idx[i*N + j] (relative_position_index)                          */
int mmni_window_rows(const mmni_wattn_desc* d, int32_t* rows, void* stream);
int mmni_window_mask(const mmni_wattn_desc* d, float* mask, void* stream);
int mmni_relative_index(const mmni_wattn_desc* d, int32_t* idx, void* stream);

/* ------------------------------------------------------------------------------------
 * Crossmodal multi-head attention core:
 *   modules/multihead_attention.py:109-125 between in_proj and out_proj:
 *   dropout(softmax_fp32(q*scale @ k^T + mask)) @ v, mask = -inf where (j - i) >= causal_diag
 *   (buffered_future_mask, crossmodal_transformer.py:179-186, causal_diag = 1+|Tk-Tq|).
 * Time-major layout (T, B, E): element (t, b, h, c) at ptr[(t*B + b)*stride + h*head_dim + c].
 * head_dim 1..16, padded to 4 / 8 / 16.  The contractions run on the bf16 matrix cores with each
 * fp32 operand split into bf16 hi + lo and three products (hi*hi + hi*lo + lo*hi) accumulated in
 * fp32: ~2^-16 relative error per product, fp32-class results.  With dtype = 1 (bf16 storage,
 * SURVEY §8d C5) the operands are bf16 already and one product is taken (fp32 accumulation and
 * softmax; the probabilities enter P·V rounded to bf16).
 * Attention dropout (multihead_attention.py:123, F.dropout of the probabilities): dropout = p in
 * [0, 1); element (b, h, i, j) is kept iff a counter-based hash of (seed, (b*heads + h)*Tq + i, j)
 * falls below (1 - p) * 2^32, and kept probabilities are scaled by 1 / (1 - p).  The same seed in
 * the backward regenerates the same mask.  p = 0 is the exact no-dropout path.  (ABI v3 added
 * dropout and seed.)
 * Workspaces (ABI v4): >= mmni_mha_{fwd,bwd}_workspace_bytes(d) bytes, 256-byte aligned, contents
 * ignored; they hold the bf16 split images of the 64-row tiles (written by the call itself) and,
 * in the backward, delta = rowsum(dO * O).
 * ------------------------------------------------------------------------------------ */
typedef struct mmni_mha_desc {
    int32_t Tq, Tk, B, heads, head_dim;
    int32_t causal_diag;        /* <= 0: no mask                                          */
    float   scale;              /* head_dim^-0.5 (multihead_attention.py:22)              */
    int64_t q_stride, k_stride, v_stride, o_stride;
    float   dropout;            /* attention-probability dropout p (0: none)              */
    uint32_t seed;              /* dropout stream; forward and backward must agree         */
    int32_t dtype;              /* storage of q/k/v/out/dout/dq/dk/dv: 0 fp32, 1 bf16 (ABI v5);
                                   lse and the softmax are fp32 either way                   */
} mmni_mha_desc;

size_t mmni_mha_fwd_workspace_bytes(const mmni_mha_desc* d);
size_t mmni_mha_bwd_workspace_bytes(const mmni_mha_desc* d);
/* out: (Tq, B, E) rows with o_stride; lse: (B, heads, Tq) of the undropped softmax. */
int mmni_mha_fwd(const mmni_mha_desc* d, const void* q, const void* k, const void* v,
                 void* out, float* lse, void* workspace, void* stream);
/* dq/dk/dv overwritten. */
int mmni_mha_bwd(const mmni_mha_desc* d, const void* q, const void* k, const void* v,
                 const void* out, const void* dout, const float* lse,
                 void* dq, void* dk, void* dv, void* workspace, void* stream);
/* Head-averaged (dropped) attention probabilities (B, Tq, Tk) — the second return value of
 * MultiheadAttention.forward (multihead_attention.py:131-133). */
int mmni_mha_mean_probs(const mmni_mha_desc* d, const void* q, const void* k,
                        const float* lse, float* probs, void* stream);
/* The dropout multipliers (0 or 1/(1-p)) of every (b, h, i, j) as (B, heads, Tq, Tk) floats:
 * the mask the forward and backward apply, exported for tests. */
int mmni_mha_dropout_mask(const mmni_mha_desc* d, float* mask, void* stream);

/* ------------------------------------------------------------------------------------
 * 3D convolutions.  Channels-last activations (B, D, H, W, C).
 * Weights in PyTorch layout (Cout, Cin, kd, kh, kw); 2D convs pass kd = 1 on D = 1 volumes.
 * ------------------------------------------------------------------------------------ */
typedef struct mmni_conv3d_desc {
    int32_t B, D, H, W, Cin;    /* input (2D reference convs use D = 1, kd = 1, pd = 0)      */
    int32_t Cout;
    int32_t kd, kh, kw;         /* kernel extents                                         */
    int32_t sd, sh, sw;         /* strides: k==stride, pad 0 = patch-embed (swin_v2_module.py:483) */
    int32_t pd, ph, pw;         /* zero padding: k3 s1 p1 = GreenBlock conv (nvidia_blocks.py:43) */
    int32_t Do, Ho, Wo;         /* output extents                                         */
    float   slope;              /* fused LeakyReLU negative slope; 1.0 = identity         */
} mmni_conv3d_desc;

/* Input is read as (B, D, H, W, Cin) channels-last; output written (B, Do, Ho, Wo, Cout).
   w is (Cout, Cin, kd, kh, kw) contiguous; 8-byte aligned for the k3 s1 p1 case (< 0 otherwise). */
int mmni_conv3d_fwd(const mmni_conv3d_desc* d, const float* x, const float* w,
                    const float* bias, float* y, void* stream);
/* dx overwritten (may be NULL); dw (Cout*Cin*kd*kh*kw) and db (Cout, nullable) OVERWRITTEN.
 * y is the forward output, needed when slope != 1 to gate the LeakyReLU gradient.
 * workspace: >= mmni_conv3d_bwd_workspace_bytes(d) bytes, contents ignored: one row of partial
 * dW/db per persistent workgroup, reduced in a fixed order, so dw/db are bitwise deterministic
 * (ABI v3; v2 accumulated them with float atomics). */
size_t mmni_conv3d_bwd_workspace_bytes(const mmni_conv3d_desc* d);
int mmni_conv3d_bwd(const mmni_conv3d_desc* d, const float* x, const float* w,
                    const float* y, const float* dy, float* dx, float* dw, float* db,
                    void* workspace, void* stream);

/* ------------------------------------------------------------------------------------
 * Token-wise ops of the Swin blocks: LayerNorm over C = 12/24/48/96
 * channels (nn.LayerNorm semantics, swinfusion_module.py:300,306; swin_v2_module.py:233,240)
 * and the weight gradient of a token Linear (dW = dY^T X, db = colsum dY) for the tall-skinny
 * shapes of the qkv / proj / MLP layers.  Row-major (rows, C) / (rows, ld) tensors.
 * Workspaces: caller-allocated, sizes from the *_workspace_bytes queries, contents ignored.
 * dgamma / dbeta / dw / db are overwritten; reductions run in a fixed order (deterministic).
 * ------------------------------------------------------------------------------------ */
int mmni_layernorm_fwd(int64_t rows, int C, const float* x, const float* gamma, const float* beta,
                       float eps, float* y, float* mean, float* rstd, void* stream);
size_t mmni_layernorm_bwd_workspace_bytes(int64_t rows, int C);
int mmni_layernorm_bwd(int64_t rows, int C, const float* dy, const float* x, const float* gamma,
                       const float* mean, const float* rstd, float* dx, float* dgamma, float* dbeta,
                       void* workspace, void* stream);
size_t mmni_linear_dw_workspace_bytes(int N, int K);
int mmni_linear_dw(int64_t rows, int N, int K, const float* x, int64_t ldx, const float* dy,
                   int64_t lddy, float* dw, float* db, void* workspace, void* stream);

/* Token Linear forward / input-gradient (tokenlinear.hip): rows x K -> rows x N, one lane per row,
 * replacing hipBLASLt on the block Linears (swinfusion_module.py:25-31,104-110,203-205;
 * swin_v2_module.py:26-32) and fusing their epilogues:
 *   epi 0  y = x W^T (+ bias)
 *   epi 1  y = gelu(x W^T + bias)                          (Mlp fc1 + nn.GELU, exact erf)
 *   epi 2  y = (x W^T) * gelu'(aux W2^T + b2)               (Mlp backward: x = dY of fc2,
 *          W = fc2.weight^T, aux = fc1 input (rows x K2), W2/b2 = fc1 weight/bias)
 * residual (nullable, epi 0/1, same shape and row stride as y) is added last: the block's
 * `x + drop_path(proj(...))` / `x + drop_path(mlp(...))` with an inactive drop_path
 * (swinfusion_module.py:377-378). y may alias residual.
 * W(n, k) = w[n*w_sn + k*w_sk]: (w_sn, w_sk) = (K, 1) for an nn.Linear weight, (1, N) for its
 * transpose.  x / y / aux rows 16-byte aligned.  Returns -2 for a shape outside the compiled set
 * (mmni_token_linear_supported). */
typedef struct mmni_tlin_desc {
    int64_t rows;
    int32_t K, N, epi, K2;
    int64_t ldx, ldy, ldaux;
    int64_t w_sn, w_sk;
} mmni_tlin_desc;
int mmni_token_linear(const mmni_tlin_desc* d, const float* x, const float* w, const float* bias,
                      const float* aux, const float* w2, const float* b2, const float* residual, float* y,
                      void* stream);
int mmni_token_linear_supported(int K, int N, int epi, int K2);

/* Fused token MLP (mlp.hip): y = fc2(GELU(fc1(x))) (+ residual) with the hidden activation kept
 * in registers (Mlp / Mlp_fusion, swin_v2_module.py:16-32, swinfusion_module.py:14-30; nn.GELU
 * exact erf, dropout inactive), on the f32 MFMA.  Covers C = 12, hidden H = 48
 * (mmni_mlp_supported).  w1: fc1.weight (H, C), b1 (H) nullable, w2: fc2.weight (C, H), b2 (C)
 * nullable.  x / residual / y / dy / dx are contiguous (rows, C): ldx = ldy = C.
 * Backward recomputes the hidden activation: dx overwritten (row stride ldx), dw1 / db1 / dw2 /
 * db2 overwritten (fixed-order reduction, deterministic); the residual's gradient is dy itself and
 * stays with the caller. */
typedef struct mmni_mlp_desc {
    int64_t rows;
    int32_t C, H;
    int64_t ldx, ldy;
} mmni_mlp_desc;
int mmni_mlp_supported(int C, int H);
int mmni_mlp_fwd(const mmni_mlp_desc* d, const float* x, const float* w1, const float* b1,
                 const float* w2, const float* b2, const float* residual, float* y, void* stream);
size_t mmni_mlp_bwd_workspace_bytes(const mmni_mlp_desc* d);
int mmni_mlp_bwd(const mmni_mlp_desc* d, const float* x, const float* w1, const float* b1,
                 const float* w2, const float* dy, float* dx, float* dw1, float* db1, float* dw2,
                 float* db2, void* workspace, void* stream);

/* norm2 + MLP (+ residual) of a pre-norm block in one kernel per direction
 * (swinfusion_module.py:374-377): y = [x] + fc2(GELU(fc1(LN(x)))), residual_x selecting the
 * "+ x"; LN statistics are recomputed in the backward (nothing saved).  The backward writes
 * dx = LN_bwd(dMLP/dLN) (+ dy when residual_x), dgamma, dbeta and the fc gradients.  Same
 * shapes as mmni_mlp_*; the workspace is mmni_mlp_bwd_workspace_bytes. */
int mmni_ln_mlp_fwd(const mmni_mlp_desc* d, float eps, const float* x, const float* gamma, const float* beta,
                    const float* w1, const float* b1, const float* w2, const float* b2, int residual_x, float* y,
                    void* stream);
/* mmni_ln_mlp_fwd plus the identity skip of the residual group that ends with this block
 * (RSTB / CRSTB `residual_group(x) + x`, swinfusion_module.py:814,918-927):
 * y = [x] + fc2(GELU(fc1(LN(x)))) + skip.  skip is (rows, C) contiguous, 16-byte aligned and must
 * not alias y; its gradient is dy itself, so mmni_ln_mlp_bwd serves both forms. */
int mmni_ln_mlp_skip_fwd(const mmni_mlp_desc* d, float eps, const float* x, const float* gamma, const float* beta,
                         const float* w1, const float* b1, const float* w2, const float* b2, int residual_x,
                         const float* skip, float* y, void* stream);
int mmni_ln_mlp_bwd(const mmni_mlp_desc* d, float eps, const float* x, const float* gamma, const float* beta,
                    const float* w1, const float* b1, const float* w2, const float* dy, int residual_x, float* dx,
                    float* dgamma, float* dbeta, float* dw1, float* db1, float* dw2, float* db2, void* workspace,
                    void* stream);

/* Fused token ops around the window attention of a SwinFusion block (blockops.hip, C = 12, f32
 * MFMA), replacing norm1 + attn.qkv / attn.q / attn.kv and their backward with the block's
 * residual gradient (swinfusion_module.py:346,121,202-205,377), and the backward of attn.proj
 * (swinfusion_module.py:143).  Token rows contiguous and 16-byte aligned.
 *   ln_linear_fwd   y (rows, N) = LN(x) W^T + b, LN over C with gamma/beta/eps (nn.LayerNorm);
 *                   mean / rstd (rows) saved for the backward (the LN output is never stored).
 *   ln_linear_bwd   dx = LN_bwd(dy W) + dres (dres nullable), dw (N, C), db (N, nullable),
 *                   dgamma, dbeta (C): LN(x) recomputed from x, mean, rstd.  N = 12, 24, 36.
 *   linear_bwd      dx = dy W, dw = dy^T x, db = colsum dy for a C -> C Linear (N = C).
 * Gradients are overwritten; reductions run in a fixed order (deterministic). */
typedef struct mmni_tok_desc {
    int64_t rows;
    int32_t C, N;
    float eps;
} mmni_tok_desc;
int mmni_ln_linear_fwd(const mmni_tok_desc* d, const float* x, const float* gamma, const float* beta,
                       const float* w, const float* b, float* y, float* mean, float* rstd, void* stream);
size_t mmni_tok_bwd_workspace_bytes(const mmni_tok_desc* d);
int mmni_ln_linear_bwd(const mmni_tok_desc* d, const float* dy, const float* x, const float* mean,
                       const float* rstd, const float* gamma, const float* beta, const float* w,
                       const float* dres, float* dx, float* dw, float* db, float* dgamma,
                       float* dbeta, void* workspace, void* stream);
/* ln_linear_bwd with a second residual gradient: dx = LN_bwd(dy W) + dres + dres2 (each nullable).
 * dres2 carries the gradient of the identity skip of the residual group this block opens (RSTB /
 * CRSTB `residual_group(x) + x`, swinfusion_module.py:814,918-927), which would otherwise meet dx
 * in a separate full-size add. */
int mmni_ln_linear_bwd2(const mmni_tok_desc* d, const float* dy, const float* x, const float* mean,
                        const float* rstd, const float* gamma, const float* beta, const float* w,
                        const float* dres, const float* dres2, float* dx, float* dw, float* db, float* dgamma,
                        float* dbeta, void* workspace, void* stream);
int mmni_linear_bwd(const mmni_tok_desc* d, const float* dy, const float* x, const float* w,
                    float* dx, float* dw, float* db, void* workspace, void* stream);

/* Input preprocessing (preprocess.hip), replacing the per-subject host work
 * of the reference's Dataset.__getitem__:
 *   zscore          y = (x - mean) / std over each of n_arrays contiguous arrays of `count`
 *                   floats (scipy.stats.zscore(axis=None), ddof 0; datasets.py:416, 664), statistics
 *                   in double, deterministic; half_round != 0 rounds through float16 (.half()).
 *   fir_highpass    host: nitime FilterAnalyzer.fir high-pass taps (firwin hamming, spectral
 *                   inversion), cutoff as a fraction of Nyquist.
 *   fmri_band_split y (B, R, Lmax) series with lens[b] valid samples (device int32) ->
 *                   raw / low / ultralow (B, seq, R): zscore(x), zscore(fir(x)), zscore(x - fir(x))
 *                   over time, zero-padded to seq with (seq - L) / 2 in front (datasets.py:665-698).
 *                   fir = zero-phase filtfilt (odd extension 3 * ntaps) with the mean restored.
 *                   Needs 3 * ntaps < lens[b] <= Lmax <= seq <= 1024, ntaps odd <= 129. */
typedef struct mmni_bandsplit_desc {
    int32_t B, R;      /* subjects, ROIs */
    int32_t Lmax;      /* row stride of y (time samples) */
    int32_t seq;       /* padded output length (368 in the reference) */
    int32_t ntaps;     /* FIR length (nitime filt_order + 1 = 65) */
} mmni_bandsplit_desc;
size_t mmni_zscore_workspace_bytes(int64_t n_arrays);
int mmni_zscore(int64_t n_arrays, int64_t count, const float* x, float* y, int half_round, void* workspace,
                void* stream);
int mmni_fir_highpass_taps(int ntaps, double cutoff_frac, double* taps);
int mmni_fmri_band_split(const mmni_bandsplit_desc* d, const float* y, const int32_t* lens, const double* taps,
                         float* raw, float* low, float* ultralow, void* stream);

/* ------------------------------------------------------------------------------------
 * Crossmodal-encoder dense layers (ABI v6).  Token rows are the
 * time-major (T, B, E) activations seen as (T*B, E) rows of row stride ld*.
 *
 *   mmni_rowgemm     y[r][n] = epi( sum_k x'[r][k] * W(n, k) ),  W(n, k) = w[n*w_sn + k*w_sk]
 *                    (w_sk = 1: an nn.Linear weight (N, K); w_sn = 1: the transpose, for the
 *                    input gradient dX = dY W of a Linear (K_lin, N_lin) -> (N = K_lin, K = N_lin))
 *                    x' = LayerNorm_K(x) with gamma/beta/eps when ln (row mean / rstd written to
 *                    mean / rstd when those are non-null), else x.
 *                    epi: + bias[n] (nullable), ReLU when relu, * (aux[r][n] > 0) when aux is
 *                    non-null (the ReLU backward), + res[r][n] when res is non-null.
 *                    Replaces in one launch: layer_norms[i](x) -> F.linear -> F.relu -> + residual
 *                    (crossmodal_transformer.py:145-165), the in_proj slices and out_proj of
 *                    MultiheadAttention.forward (multihead_attention.py:71-84,129).
 *   mmni_rowgemm_dw  dw[n][k] = sum_r dy[r][n] * x'[r][k], db[n] = sum_r dy[r][n] (db nullable);
 *                    x' = LayerNorm recomputed from the forward's mean / rstd when ln.  Row
 *                    chunks reduced in a fixed order: deterministic.  dy rows of stride ldy.
 *   mmni_row_layernorm_fwd  y = LayerNorm(x) over rows of C <= 256 (+ mean, rstd for the backward):
 *                    the crossmodal encoder's layer_norms / final LayerNorm on the per-op paths
 *                    (crossmodal_transformer.py:145,159; the encoder's final norm :94).
 *   mmni_row_layernorm_bwd  dx = LayerNorm backward of dxn (+ dres), dgamma, dbeta over
 *                    rows of C <= 256 (fixed-order partial sums: deterministic).
 * All fp32.  Workspaces: mmni_rowgemm_dw_workspace_bytes / mmni_row_layernorm_bwd_workspace_bytes.
 * ------------------------------------------------------------------------------------ */
typedef struct mmni_rowgemm_desc {
    int64_t rows;
    int32_t K, N;
    int64_t ldx, ldy, ldres, ldaux;
    int64_t w_sn, w_sk;
    int32_t ln;        /* LayerNorm prologue over the K input columns */
    float eps;
    int32_t relu;      /* ReLU epilogue */
} mmni_rowgemm_desc;
int mmni_rowgemm(const mmni_rowgemm_desc* d, const float* x, const float* gamma, const float* beta, const float* w,
                 const float* bias, const float* aux, const float* res, float* y, float* mean, float* rstd,
                 void* stream);
size_t mmni_rowgemm_dw_workspace_bytes(const mmni_rowgemm_desc* d);
int mmni_rowgemm_dw(const mmni_rowgemm_desc* d, const float* x, const float* gamma, const float* beta,
                    const float* mean, const float* rstd, const float* dy, float* dw, float* db, void* workspace,
                    void* stream);
int mmni_row_layernorm_fwd(int64_t rows, int C, const float* x, int64_t ldx, const float* gamma, const float* beta,
                           float eps, float* y, int64_t ldy, float* mean, float* rstd, void* stream);
size_t mmni_row_layernorm_bwd_workspace_bytes(int64_t rows, int C);
int mmni_row_layernorm_bwd(int64_t rows, int C, const float* dxn, int64_t lddxn, const float* x, int64_t ldx,
                           const float* gamma, const float* mean, const float* rstd, const float* dres,
                           int64_t ldres, float* dx, int64_t lddx, float* dgamma, float* dbeta, void* workspace,
                           void* stream);
/* ABI v8: the same two with the LayerNorm output y (fwd) / input gradient dxn (bwd) stored as fp32
 * (dtype 0) or bf16 (dtype 1): the bf16 crossmodal head's pre-norms feed bf16 GEMMs directly
 * (torch autocast computes layer_norm in fp32 and the consuming Linear rounds it to bf16; the
 * kernel rounds the same fp32 value once). */
int mmni_row_layernorm_fwd_t(int64_t rows, int C, const float* x, int64_t ldx, const float* gamma, const float* beta,
                             float eps, void* y, int y_dtype, int64_t ldy, float* mean, float* rstd, void* stream);
int mmni_row_layernorm_bwd_t(int64_t rows, int C, const void* dxn, int dxn_dtype, int64_t lddxn, const float* x,
                             int64_t ldx, const float* gamma, const float* mean, const float* rstd, const float* dres,
                             int64_t ldres, float* dx, int64_t lddx, float* dgamma, float* dbeta, void* workspace,
                             void* stream);

/* ------------------------------------------------------------------------------------
 * Split-K weight-gradient reductions (ABI v8) of the crossmodal encoder's Linears
 * (crossmodal_transformer.py:189-194 Linear, multihead_attention.py in_proj / out_proj: the
 * backward of F.linear, whose weight gradient the host runs as one batched GEMM over S row chunks):
 *   dw[e] = sum_{c < S} part[c][e]   (e < NK = N * K; chunk order)
 *   db[n] = sum_{r < rows} dy[r][n]  (row stride ldy; fixed row slabs + fixed-order slab sum; db,
 *                                     dy nullable together)
 * part and dy are fp32 (dtype 0) or bf16 (dtype 1, the autocast head); sums and outputs fp32.
 * Bitwise deterministic.  Workspace: mmni_splitk_reduce_workspace_bytes(rows, N).
 * ------------------------------------------------------------------------------------ */
#define MMNI_CAST_MAX_SEGS 64
/* dst[i][e] = bf16(src[i][e]) (round to nearest even) for e < count[i], i < n <= 64, in one launch:
 * the per-step bf16 copies of the head's Linear weights and biases under autocast (torch casts each
 * one separately: ~8 launches per encoder layer).  src / dst / count are host arrays. */
int mmni_cast_bf16_multi(int n, const float* const* src, void* const* dst, const int64_t* count, void* stream);
size_t mmni_splitk_reduce_workspace_bytes(int64_t rows, int N);
int mmni_splitk_reduce(int S, int64_t NK, const void* part, int64_t rows, int N, const void* dy, int64_t ldy,
                       int dtype, float* dw, float* db, void* workspace, void* stream);

/* ------------------------------------------------------------------------------------
 * Swin-V2 continuous position bias table (ABI v7; replaces WindowAttention.cpb_mlp applied to
 * relative_coords_table and the 16 * sigmoid that follows, swin_v2_module.py:88-91,158-162):
 *   out[t][h] = 16 * sigmoid( sum_j w2[h][j] * relu( w1[j] . coords[t] + b1[j] ) )
 *   coords (tsz, nd), w1 (hidden, nd), b1 (hidden), w2 (heads, hidden), out (tsz, heads);
 *   nd <= 3, hidden <= 512, heads <= 32, fp32.
 *   mmni_cpb_bwd  dw1, db1, dw2 from dout and the forward's out (per-block partial rows, fixed-order
 *                 column sum: deterministic; the coordinate table is a constant buffer: no dcoords).
 * ------------------------------------------------------------------------------------ */
int mmni_cpb_fwd(int64_t tsz, int nd, int hidden, int heads, const float* coords, const float* w1, const float* b1,
                 const float* w2, float* out, void* stream);
size_t mmni_cpb_bwd_workspace_bytes(int64_t tsz, int nd, int hidden, int heads);
int mmni_cpb_bwd(int64_t tsz, int nd, int hidden, int heads, const float* coords, const float* w1, const float* b1,
                 const float* w2, const float* out, const float* dout, float* dw1, float* db1, float* dw2,
                 void* workspace, void* stream);

int mmni_version(void);
const char* mmni_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MMNI_H */
