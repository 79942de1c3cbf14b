/*
 * visionseg.h — C ABI of libvisionseg_hip.so, the MI355X (gfx950) kernels of the
 * Swin + Mask2Former training hot path.
 *
 * Boundary.  The reference (Wlsghdh/VISION-Instance-Seg) reaches this path only
 * through upstream Python/C++ extensions that are not vendored:
 *   - MSDeformAttn CUDA extension `MultiScaleDeformableAttention.ms_deform_attn_forward/
 *     backward(value, spatial_shapes, level_start_index, sampling_loc, attn_weight,
 *     im2col_step)` called by MaskDINO/Mask2Former `MSDeformAttnFunction`
 *     (upstream ops/functions/ms_deform_attn_func.py); in-container oracle equivalent
 *     HF:m2f:798-837 `multi_scale_deformable_attention`.
 *   - Swin `window_partition` / `window_reverse` + `torch.roll` + `F.pad`
 *     (HF:swin:486-505, 546-566, 609-626) and the window attention core
 *     (HF:swin:373-398, 401-468).
 *   - the mask head einsum + attention-mask derivation (HF:m2f:2040-2056).
 *   - the masked cross-attention core of `nn.MultiheadAttention` as the decoder calls
 *     it (HF:m2f:1644-1650, fully-blocked-row fix HF:m2f:1912-1914).
 * Callers: training/train_template.py `train_maskdino(...)` and
 * labeling_server/ai_segmentation.py `AISegmentationModel.predict(...)` reach these
 * entry points through the Python package `visionseg`.
 *
 * Conventions.
 *   - Every pointer named *without* a `_host` suffix is DEVICE memory; all tensors are
 *     dense row-major (C-contiguous) in the layout documented per function.
 *   - `dtype` selects the storage type of the activation tensors: VS_F32 or VS_BF16.
 *     Coordinates, attention weights, statistics and gradient accumulators are f32.
 *     Arithmetic is always f32 (MFMA accumulate in f32).
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  Every call is
 *     asynchronous on that stream; no call allocates device memory or synchronises,
 *     so calls are hipGraph-capturable.
 *   - Return value: VS_OK (0) or a negative error code; vs_last_error() returns a
 *     thread-local message for the last failure (mirrors TORCH_CHECK -> RuntimeError
 *     in the upstream extension).
 */
#ifndef VISIONSEG_H_
#define VISIONSEG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VS_ABI_VERSION 1

#if defined(__GNUC__)
#define VS_API __attribute__((visibility("default")))
#else
#define VS_API
#endif

enum vs_dtype { VS_F32 = 0, VS_BF16 = 1 };
enum vs_status { VS_OK = 0, VS_ERR_INVALID = -1, VS_ERR_HIP = -2, VS_ERR_UNSUPPORTED = -3 };

VS_API int vs_abi_version(void);
VS_API const char* vs_last_error(void);

/* ---- a8: multi-scale deformable attention sampling -------------------------------
 * value       [B, S, H, 32]            dtype      (S = sum_l H_l*W_l, head dim 32)
 * spatial_shapes_host  int64 [L, 2]    HOST       (H_l, W_l), L <= 4
 * level_start_host     int64 [L]       HOST       start of level l inside S
 * sampling_loc f32 [B, Q, H, L, P, 2]  (x, y) normalised to [0,1]
 * attn_weight  f32 [B, Q, H, L, P]
 * out         [B, Q, H*32]             dtype
 * Sampling: h = y*H_l - 0.5, w = x*W_l - 0.5, bilinear, zeros outside (upstream
 * ms_deform_attn_im2col_bilinear == grid_sample(align_corners=False, zeros)).
 * Replaces ms_deform_attn_forward.  im2col_step of the upstream API has no meaning
 * here (the whole batch is one launch) and is not part of the ABI. */
VS_API int vs_msda_forward(int dtype, const void* value, const int64_t* spatial_shapes_host,
                    const int64_t* level_start_host, const float* sampling_loc,
                    const float* attn_weight, void* out, int batch, int spatial_size,
                    int num_heads, int channels, int num_levels, int num_query,
                    int num_point, void* stream);

/* Replaces ms_deform_attn_backward.  grad_out [B, Q, H*32] dtype.  Outputs (all f32,
 * overwritten): grad_value [B, S, H, 32], grad_loc [B, Q, H, L, P, 2],
 * grad_attn [B, Q, H, L, P]. */
VS_API int vs_msda_backward(int dtype, const void* value, const int64_t* spatial_shapes_host,
                     const int64_t* level_start_host, const float* sampling_loc,
                     const float* attn_weight, const void* grad_out, float* grad_value,
                     float* grad_loc, float* grad_attn, int batch, int spatial_size,
                     int num_heads, int channels, int num_levels, int num_query,
                     int num_point, void* stream);

/* vs_msda_backward with a workspace (vs_msda_backward_workspace_bytes bytes, any content):
 * bf16 encoder problems (queries = the value grid, P = 4) then take the destination-tile
 * kernel -- every grad_value cell written once with plain stores, no memset, deterministic;
 * taps further than 4 cells from their query's reference point go through a far-tap list
 * and f32 atomics afterwards.  Other problems: as vs_msda_backward. */
VS_API long long vs_msda_backward_workspace_bytes(int B, int Q, int heads, int L, int P);
VS_API int vs_msda_backward_ex(int dtype, const void* value, const int64_t* spatial_shapes,
                               const int64_t* level_start, const float* loc, const float* attn,
                               const void* grad_out, float* grad_value, float* grad_loc, float* grad_attn,
                               void* workspace, int B, int S, int heads, int D, int L, int Q, int P,
                               void* stream);

/* Opt-in backward (VS_MSDA_BWD=tiled; replaces ms_deform_attn_backward like the others):
 * grad_value by destination tiles
 * (image, head, level, te x te cells), each owned by one wave that accumulates its
 * corner contributions with plain LDS read-modify-write -- no float atomics, no memset;
 * grad_value [B, S, H, 32] is written once, in the value dtype.  grad_loc / grad_attn as
 * in vs_msda_backward.  Any queries.  workspace >=
 * vs_msda_backward_tiled_workspace_bytes (spatial_shapes_host as below; -1 on bad sizes). */
VS_API long long vs_msda_backward_tiled_workspace_bytes(int batch, int num_heads, int num_levels, int num_query,
                                                        int num_point, const int64_t* spatial_shapes_host);
VS_API int vs_msda_backward_tiled(int dtype, const void* value, const int64_t* spatial_shapes_host,
                                  const int64_t* level_start_host, const float* sampling_loc,
                                  const float* attn_weight, const void* grad_out, void* grad_value,
                                  float* grad_loc, float* grad_attn, void* workspace, int batch, int spatial_size,
                                  int num_heads, int channels, int num_levels, int num_query, int num_point,
                                  void* stream);

/* ---- a7: MSDeformAttn prologue (csrc/msda_prep.hip) ---------------------------------
 * Replaces the reference path's `sampling_offsets(q) / offset_normalizer + reference_points`
 * and `softmax(attention_weights(q))` (HF:m2f:994-1002; upstream MSDeformAttn.forward,
 * reached from training/maskdino/train_full.py:308-310 through the pixel decoder):
 *   loc[b,q,h,l,p,:] = ref[b,q,l,:] + offsets[b,q,h,l,p,:] / (W_l, H_l)      (f32 out)
 *   attw[b,q,h,:]    = softmax_{L*P}(logits[b,q,h,:])                        (f32 out)
 * offsets [B,Q,H*L*P*2] / logits [B,Q,H*L*P] in dtype with row strides (elements) >= a
 * row (views of one fused projection allowed); ref f32 [B,Q,L,2] with rows contiguous
 * and batch stride ref_batch_stride (even; 0: shared by the batch); loc / attw contiguous;
 * ref, loc (and, backward, grad_loc) 8-byte aligned.
 * L <= 4, L*P <= 32. */
VS_API int vs_msda_prep_forward(int dtype, const void* offsets, long long offsets_row_stride, const void* logits,
                                long long logits_row_stride, const float* ref, long long ref_batch_stride,
                                const int64_t* spatial_shapes_host, float* loc, float* attw, int batch,
                                int num_query, int num_heads, int num_levels, int num_point, void* stream);
/* Adjoint: grad_offsets = grad_loc / (W_l, H_l), grad_logits = attw * (g - <g, attw>)
 * (attw = the forward's output), both rounded to dtype and written with the given row
 * strides. */
VS_API int vs_msda_prep_backward(int dtype, const float* grad_loc, const float* grad_attw, const float* attw,
                                 const int64_t* spatial_shapes_host, void* grad_offsets,
                                 long long grad_offsets_row_stride, void* grad_logits, long long grad_logits_row_stride,
                                 int batch, int num_query, int num_heads, int num_levels, int num_point, void* stream);

/* ---- a2: Swin pad + cyclic shift + window partition / its inverse ---------------
 * window_partition: x [B, H, W, C] -> windows [B*nWh*nWw, ws*ws, C] where
 * Hp = ceil(H/ws)*ws, nWh = Hp/ws (same for W); windows[(b,wy,wx), (ty,tx)] =
 * xpad[b, (wy*ws+ty+shift) % Hp, (wx*ws+tx+shift) % Wp] with zero padding.
 * Bit-exact data movement for any element size (esize = bytes per element).
 * window_reverse is the exact inverse on the un-padded region (crop) — it is also the
 * backward of window_partition, and window_partition is the backward of
 * window_reverse. */
VS_API int vs_window_partition(const void* x, void* windows, int esize, int batch, int height,
                        int width, int channels, int window, int shift, void* stream);
VS_API int vs_window_reverse(const void* windows, void* x, int esize, int batch, int height,
                      int width, int channels, int window, int shift, void* stream);


/* ---- a3/a4/a5: Swin (shifted-)window attention core ------------------------------
 * qkv   [Bw, N, 3, heads, 32] dtype   fused q;k;v projection of the partitioned windows
 *                                     (N = window^2, Bw = batch * nwin_h * nwin_w)
 * rel_table f32 [(2*window-1)^2, heads]   relative position bias table
 * out   [Bw, N, heads*32] dtype;  lse f32 [Bw, heads, N] (saved for backward)
 * S_ij = q_i.k_j*scale + table[rel(i,j)] + (shift>0 && region_i != region_j ? -100 : 0);
 * region ids are computed from the padded-grid position (nwin_h*window rows), exactly as
 * HF:swin:584-607 builds its mask.  f32 softmax. */
VS_API int vs_window_attn_forward(int dtype, const void* qkv, const float* rel_table, void* out,
                                  float* lse, int num_windows, int heads, int window, int shift,
                                  int nwin_h, int nwin_w, float scale, void* stream);

/* grad_out [Bw, N, heads*32] dtype -> grad_qkv [Bw, N, 3, heads, 32] dtype (overwritten),
 * grad_table_partial f32 [Bw, heads, (2*window-1)^2]: per-window partial sums of the
 * bias-table gradient; the caller reduces over Bw (deterministic, no global atomics). */
VS_API int vs_window_attn_backward(int dtype, const void* qkv, const float* rel_table,
                                   const void* out, const float* lse, const void* grad_out,
                                   void* grad_qkv, float* grad_table_partial, int num_windows,
                                   int heads, int window, int shift, int nwin_h, int nwin_w,
                                   float scale, void* stream);


/* ---- C5: fp8 (OCP e4m3) window attention ----------------------------------------
 * Same layouts and semantics as vs_window_attn_forward/backward with bf16 storage, for
 * window^2 <= 160.  The forward's logits S = q.k^T and product P.V run on the
 * block-scaled MX MFMA v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands and e8m0
 * power-of-two scales 2^floor(log2(448/amax)): one per q / k token (amax over its 32
 * channels), one per (window, head) for V, and a fixed 2^8 for P = exp(S - max) <= 1;
 * f32 softmax and accumulation.  The backward recomputes S from the same e4m3 values
 * (dequantised exactly to bf16, so exp(S - lse) is the forward's P) and forms dV, dP,
 * dQ, dK in bf16 from the bf16 operands (straight-through quantisation).  Replaces the
 * same upstream call sites as vs_window_attn_* (HF:swin:373-398) under BASELINE config
 * C5. */
VS_API int vs_window_attn_forward_fp8(const void* qkv, const float* rel_table, void* out, float* lse,
                                      int num_windows, int heads, int window, int shift, int nwin_h,
                                      int nwin_w, float scale, void* stream);
VS_API int vs_window_attn_backward_fp8(const void* qkv, const float* rel_table, const void* out,
                                       const float* lse, const void* grad_out, void* grad_qkv,
                                       float* grad_table_partial, int num_windows, int heads,
                                       int window, int shift, int nwin_h, int nwin_w, float scale,
                                       void* stream);

/* Image-layout variants: the window reverse (vs_window_reverse) folded into the attention
 * kernels.  out / grad_out are [batch, height, width, heads*32] in the un-shifted,
 * un-padded image layout (nwin_h * window >= height > (nwin_h - 1) * window, likewise the
 * width); qkv, grad_qkv, lse and the table partials keep the window layout.  bf16 only
 * (fp8 != 0: the C5 e4m3 kernels), window^2 <= 160.  The partition of grad_out that the
 * reverse's backward would run is folded into the backward's loads the same way (padded
 * tokens: zero output gradient).  Replace HF:swin:558-566 + the attention core. */
VS_API int vs_window_attn_forward_image(int dtype, int fp8, const void* qkv, const float* rel_table,
                                        void* out, float* lse, int num_windows, int heads, int window,
                                        int shift, int nwin_h, int nwin_w, int height, int width,
                                        float scale, void* stream);
VS_API int vs_window_attn_backward_image(int dtype, int fp8, const void* qkv, const float* rel_table,
                                         const void* out, const float* lse, const void* grad_out,
                                         void* grad_qkv, float* grad_table_partial, int num_windows,
                                         int heads, int window, int shift, int nwin_h, int nwin_w,
                                         int height, int width, float scale, void* stream);


/* LayerNorm forwards that also write their bf16 output as MX fp8 (e4m3 y_q [rows, C] + e8m0
 * y_qscales [rows, C/32], the bytes vs_mx_quantize would make of y) at the same rows: the
 * operand of the fp8 token GEMM that consumes y (config C5), without a quantisation pass.
 * bf16, C % 32 == 0; otherwise as vs_layer_norm_forward_rows / vs_add_layer_norm_forward(_rows)
 * (y_rows may be NULL for the add form: row-major output). */
VS_API int vs_layer_norm_forward_rows_q(const void* x, const void* w, const void* b, void* y, void* y_q,
                                        void* y_qscales, float* mean, float* rstd, int M, int C, float eps,
                                        const int* y_rows, void* stream);
VS_API int vs_add_layer_norm_forward_q(const void* x, const void* r, const void* w, const void* b, void* s,
                                       void* y, void* y_q, void* y_qscales, float* mean, float* rstd, int M,
                                       int C, float eps, const int* y_rows, void* stream);

/* The same LayerNorm forwards writing their bf16 output also as ROW-scaled e4m3 (y_q [rows, C]
 * + f32 y_scale [rows], y ~= q * scale with a power-of-two scale per row, the rule of
 * vs_row_quantize_fp8) at the same (window-layout) rows: the operand of the vendor rowwise
 * fp8 GEMM (config C5's fp8 Linears) without a quantisation pass.  bf16 only. */
VS_API int vs_layer_norm_forward_qr(const void* x, const void* w, const void* b, void* y, void* y_q, float* y_scale,
                                    float* mean, float* rstd, int M, int C, float eps, const int* y_rows,
                                    void* stream);
VS_API int vs_add_layer_norm_forward_qr(const void* x, const void* r, const void* w, const void* b, void* s,
                                        void* y, void* y_q, float* y_scale, float* mean, float* rstd, int M, int C,
                                        float eps, const int* y_rows, void* stream);

/* ---- a5 / a6: token GEMM (the Swin block's Linears) ----------------------------------
 * y[M, N] = x[M, K] w[N, K]^T + bias[N] (bf16 out, f32 accumulation), both operands
 * K-contiguous rows: the F.linear of HF:swin:418-468 (qkv, proj) and HF:swin:511-536
 * (fc1, fc2) over B * H * W tokens.  mode bits:
 *   VS_TGEMM_FP8  : x, w are e4m3 bytes with one e8m0 scale byte per 32 elements along K
 *                   (x_scales [M, K/32], w_scales [N, K/32], from vs_mx_quantize); the
 *                   block-scaled MX MFMA (config C5's fp8 path); K % 128 == 0.
 *                   Without it x, w are bf16 (K % 8 == 0).
 *   VS_TGEMM_GELU : y = gelu(x w^T + b) with the exact erf GELU of HF `gelu`, and y_pre =
 *                   the bf16 pre-activation (the input of the GELU's backward); the GELU is
 *                   taken of the rounded pre-activation.
 *   VS_TGEMM_QOUT : (with GELU) y also as MX fp8: y_q e4m3 [M, N] + y_qscales e8m0
 *                   [M, N/32], the same bytes as vs_mx_quantize(y) (the next GEMM's operand
 *                   without a quantisation pass); N % 32 == 0.
 *   VS_TGEMM_GELU_BWD : the MLP's GELU backward in the epilogue of fc2's input gradient
 *                   (x = dY, w = W2^T): y = bf16(x w^T) * gelu'(y_pre), each product rounded
 *                   once, y_pre the saved bf16 pre-activation (READ); bf16, no bias, N % 8 == 0.
 *                   Replaces the stored dH plus the activation backward's pass over it
 *                   (autograd's GeluBackward of HF:swin:511-536).
 *   VS_TGEMM_RELU_BWD : the same for a ReLU FFN (the pixel decoder's encoder layers,
 *                   HF:m2f:1080-1082): y_pre = the ReLU OUTPUT, y = bf16(x w^T) * [y_pre > 0].
 * bias may be NULL.  N % 4 == 0. */
#define VS_TGEMM_FP8 1
#define VS_TGEMM_GELU 2
#define VS_TGEMM_QOUT 4
#define VS_TGEMM_GELU_BWD 8
#define VS_TGEMM_RELU_BWD 16
VS_API int vs_token_gemm(int mode, const void* x, const void* x_scales, const void* w, const void* w_scales,
                         const void* bias, void* y, void* y_pre, void* y_q, void* y_qscales, int M, int N, int K,
                         void* stream);

/* bf16 rows x [rows, K] -> e4m3 bytes q [rows, K] and e8m0 scales [rows, K/32]: per block of
 * 32 elements the largest power of two 2^k with amax * 2^k <= 448 (scale byte 127 - k), the
 * elements rounded to nearest even at that scale.  K % 32 == 0. */
VS_API int vs_mx_quantize(const void* x, void* q, void* scales, int rows, int K, void* stream);

/* Row-wise e4m3 quantisation for the vendor (hipBLASLt) fp8 GEMM with one f32 scale per
 * operand row (torch._scaled_mm rowwise; config C5's fp8 Linears, csrc/fp8_rows.hip):
 * x bf16 [rows, K] -> q e4m3 bytes [rows, K] and scale f32 [rows], x ~= q * scale with
 * scale = 2^-k, k the largest exponent with amax(row) 2^k <= 448.  K % 8 == 0, K <= 8192;
 * x / y 16-B aligned, q 8-B aligned.  The gelu variant quantises y = gelu(h) (exact erf,
 * stored in bf16 to y) in the same pass: the Swin MLP's fc1 -> fc2 hand-off. */
VS_API int vs_row_quantize_fp8(const void* x, void* q, float* scale, int rows, int K, void* stream);
VS_API int vs_gelu_row_quantize_fp8(const void* h, void* y, void* q, float* scale, int rows, int K, void* stream);

/* ---- a11: mask head -----------------------------------------------------------------
 * logits f32 [B, Q, H*W] = E [B, Q, C] x P[b]^T, with the pixel embedding P
 * channels-last [B, H*W, C] (HF:m2f:2051 einsum 'bqc,bchw->bqhw').  dtype of E and P:
 * bf16 (v_mfma_f32_32x32x16_bf16) or f32 (v_mfma_f32_32x32x2_f32, exact f32 products). */
VS_API int vs_mask_head_forward(int dtype, const void* mask_embed, const void* pixel_embed_nhwc,
                                float* logits, int batch, int num_query, int channels, int height,
                                int width, void* stream);

/* Backward of vs_mask_head_forward, bf16 path (Q <= 128, C in {128, 256}):
 * grad_logits f32 [B, Q, H*W] -> grad_E [B, Q, C], grad_P [B, H*W, C] (bf16, overwritten).
 * workspace: vs_mask_head_backward_workspace_bytes(B, Q, C) bytes of device scratch
 * (per-workgroup f32 partials of grad_E, reduced in a fixed order: deterministic). */
VS_API long long vs_mask_head_backward_workspace_bytes(int batch, int num_query, int channels);
VS_API int vs_mask_head_backward(int dtype, const float* grad_logits, const void* mask_embed,
                                 const void* pixel_embed_nhwc, void* grad_mask_embed,
                                 void* grad_pixel_embed, void* workspace, int batch, int num_query,
                                 int channels, int height, int width, void* stream);
/* vs_mask_head_backward with accumulate_grad_P != 0: grad_P += dL^T.E (bf16, in place),
 * so the decoder's mask-head calls sum their pixel-embedding gradient into one buffer
 * (replaces autograd's accumulation of one [B, HW, C] gradient per call). */
VS_API int vs_mask_head_backward_ex(int dtype, const float* grad_logits, const void* E, const void* P, void* grad_E,
                                    void* grad_P, void* workspace, int batch, int num_queries, int channels,
                                    int height, int width, int accumulate_grad_P, void* stream);

/* vs_mask_head_forward (bf16, C in {128, 256}) with the logits rows stored in groups of
 * `group` rows: row (b, q) of the product goes to row ((q / group) * B + b) * group +
 * q % group of logits [Q / group, B, group, H*W] (Q % group == 0, Q * group < 2^20).
 * With E = the matched (step, target) embeddings of S steps x group targets per image
 * this writes the matched maps in (step, image, target) order from one launch. */
VS_API int vs_mask_head_forward_grouped(const void* mask_embed, const void* pixel_embed_nhwc, float* logits,
                                        int batch, int num_query, int channels, int height, int width, int group,
                                        void* stream);

/* Adjoint of the mask losses' point sampling (point_sample = grid_sample bilinear,
 * align_corners=False, zero padding; HF:m2f:245-275) for the matched (step, image, target)
 * pairs: grad_points f32 [S*B*K, n] (pair order (s, b, k)), grid f32 [S*B*K, n, 2] (the
 * sampling grid in [-1, 1], x then y) -> maps f32 [B, S*K, H, W] (pair order (b, s, k)),
 * every element written: maps[b, s*K + k] = sum over the pair's points of the point's
 * gradient times its bilinear corner weights (the same float formulas as
 * grid_sampler_2d_backward).  The maps feed vs_mask_head_backward as grad_logits with
 * num_queries = S*K, the pairs' mask embeddings gathered as E. */
VS_API int vs_point_scatter(const float* grad_points, const float* grid, float* maps, int S, int B, int K, int n,
                            int height, int width, void* stream);

/* Point gather for the mask losses' labels: out f32 [N, P] = bilinear sample (point_sample
 * = grid_sample, align_corners=False, zero padding; HF:m2f:245-275) of maps f32 [M, H, W]
 * row rows[n] (int64 [N], each in [0, M); or NULL: set n reads map n, N <= M) at coords f32
 * [N, P, 2] in [0, 1] (x, y). */
VS_API int vs_point_sample_rows(const float* maps, const long long* rows, const float* coords, float* out,
                                int num_maps, int height, int width, int num_sets, int num_points, void* stream);

/* The same bilinear point gather from bool target masks stored as u8 [M, H, W] (the
 * criterion's target labels: matcher HF:m2f:453-459, loss labels HF:m2f:700-724) without an
 * f32 copy of the masks.  rows: int64 [N] or NULL (set n reads mask n).  grid_space 0:
 * coords f32 [N, P, 2] in [0, 1]; grid_space 1: coords already in grid_sample's [-1, 1]
 * space, one [P, 2] point set per `sets_per_coord` consecutive sets (the matcher's points,
 * shared by an image's Kc targets). */
VS_API int vs_point_sample_masks(const unsigned char* masks, const long long* rows, const float* coords, float* out,
                                 int num_maps, int height, int width, int num_sets, int num_points, int grid_space,
                                 int sets_per_coord, void* stream);

/* Row-wise top-k indices for the importance sampling of the mask losses (the `topk` of
 * HF:m2f:689-724 sample_points_using_uncertainty, MaskDINO's copy of it): indices int64
 * [rows, k] = the positions of the k largest of values f32 [rows, n], per row, in ascending
 * index order (radix select, csrc/topk.hip).  The same set as torch.topk when the k-th
 * largest value is unique in its row; among ties at the threshold the lowest indices. */
VS_API int vs_topk_rows(const float* values, long long* indices, int rows, int n, int k, void* stream);

/* Attention bitmask of the next decoder layer (HF:m2f:2049-2055 + row fix 1912-1914):
 * bilinear (align_corners=False) resize of each logits row [H, W] to [th, tw], key k
 * blocked iff sigmoid(v) < 0.5, stored as bit k%32 of words[row, k/32]
 * (words u32 [rows, ceil(th*tw/32)], rows = B*Q); a row blocked at every key is
 * written all-zero (un-blocked). */
VS_API int vs_attn_bitmask(const float* logits, uint32_t* words, int rows, int height, int width,
                           int target_h, int target_w, void* stream);

/* ---- a10: masked cross-attention core ------------------------------------------------
 * q [B, Q, heads*32], k/v [B, S, heads*32] (dtype), words u32 [B, Q, ceil(S/32)] from
 * vs_attn_bitmask, out [B, Q, heads*32] dtype, lse f32 [B, heads, Q].
 * workspace: device scratch of vs_masked_attn_workspace_bytes(B, Q, S, heads) bytes. */
VS_API long long vs_masked_attn_workspace_bytes(int batch, int num_query, int num_keys, int heads);
VS_API int vs_masked_attn_forward(int dtype, const void* q, const void* k, const void* v,
                                  const uint32_t* words, void* out, float* lse, void* workspace,
                                  int batch, int num_query, int num_keys, int heads, float scale,
                                  void* stream);
/* grad_out [B, Q, heads*32] -> grad_q, grad_k, grad_v (dtype, overwritten). */
VS_API int vs_masked_attn_backward(int dtype, const void* q, const void* k, const void* v,
                                   const uint32_t* words, const void* out, const float* lse,
                                   const void* grad_out, void* grad_q, void* grad_k, void* grad_v,
                                   void* workspace, int batch, int num_query, int num_keys,
                                   int heads, float scale, void* stream);

/* ---- a10: decoder self-attention core (csrc/self_attn.hip) ---------------------------
 * Replaces the F.scaled_dot_product_attention of the decoder layers' self-attention
 * (HF:m2f:1659-1664, Mask2FormerAttention over the queries; MaskDINO's decoder with its
 * denoising-group mask, upstream dn_components, reached through training/train_template.py:104).
 * q [B, Q, heads*32], k / v [B, S, heads*32] bf16, words u32 [Q, ceil(S/32)] (word_bstride = 0:
 * shared by the batch) or [B, Q, ceil(S/32)] (word_bstride = Q*ceil(S/32)), bit j%32 of word
 * j/32 = key j blocked, or NULL (no mask); out [B, Q, heads*32] bf16 (+ its f32 copy out_f32, for
 * the backward; may be NULL), lse f32 [B, heads, Q]
 * (+inf and a zero output row for a row blocked at every key).  bf16 only (f32 inputs: the
 * vs_masked_attn_* kernels with explicit words). */
VS_API int vs_self_attn_forward(int dtype, const void* q, const void* k, const void* v, const uint32_t* words,
                                long long word_bstride, void* out, float* out_f32, float* lse, int batch,
                                int num_query, int num_keys, int heads, float scale, void* stream);
/* grad_out [B, Q, heads*32] -> grad_q, grad_k, grad_v (bf16, overwritten); one launch.  out_f32:
 * the forward's f32 copy of the output (D = rowsum(grad_out * out) is formed from it). */
VS_API int vs_self_attn_backward(int dtype, const void* q, const void* k, const void* v, const uint32_t* words,
                                 long long word_bstride, const float* out_f32, const float* lse, const void* grad_out,
                                 void* grad_q, void* grad_k, void* grad_v, int batch, int num_query, int num_keys,
                                 int heads, float scale, void* stream);

/* ---- Token-major LayerNorm and column sums (csrc/norm.hip) --------------------------
 * Replaces torch.nn.LayerNorm on the Swin blocks / patch merging / out-norms
 * (HF modeling_swin SwinLayer.layernorm_before/after, SwinPatchMerging.norm; reference
 * training/maskdino/train_full.py:166-175 builds that backbone) and the pixel-decoder
 * encoder norms (HF:m2f Mask2FormerPixelDecoderEncoderLayer.self_attn_layer_norm /
 * final_layer_norm), plus the bias gradient of their Linears.  Semantics of
 * torch.nn.functional.layer_norm over the last dim.  x, w, b, y in `dtype`; mean / rstd
 * f32 [M]; C a multiple of 8, <= 2048. */
VS_API int vs_layer_norm_forward(int dtype, const void* x, const void* weight, const void* bias, void* y,
                                 float* mean, float* rstd, int rows, int cols, float eps, void* stream);
/* Residual add fused into the LayerNorm that follows it (Swin blocks HF:swin:672-684,
 * pixel-decoder encoder layers HF:m2f:1016-1045): s = x + r rounded to dtype (written),
 * y = LN(s); replaces the separate torch add + layer_norm.  Same tensors as
 * vs_layer_norm_forward plus r [M, C] and s [M, C]. */
VS_API int vs_add_layer_norm_forward(int dtype, const void* x, const void* r, const void* w, const void* b, void* s,
                                     void* y, float* mean, float* rstd, int M, int C, float eps, void* stream);
/* vs_layer_norm_backward with dx += dres (the gradient reaching the LayerNorm input
 * through the residual path; autograd's separate accumulation add). */
VS_API int vs_layer_norm_backward_add(int dtype, const void* dy, const void* x, const void* w, const float* mean,
                                      const float* rstd, const void* dres, void* dx, void* dw, void* db, void* ws,
                                      int M, int C, void* stream);
VS_API long long vs_layer_norm_backward_workspace_bytes(int rows, int cols);
/* vs_layer_norm_backward(_add) (dres may be NULL) that also writes dx_colsum [C] (dtype,
 * may be NULL): the column sums of dx as stored -- the bias gradient of a Linear whose
 * output is the LayerNorm's residual input, with no second read of dx. */
VS_API int vs_layer_norm_backward_ex(int dtype, const void* grad_y, const void* x, const void* weight,
                                     const float* mean, const float* rstd, const void* grad_res, void* grad_x,
                                     void* grad_weight, void* grad_bias, void* dx_colsum, void* workspace,
                                     int rows, int cols, void* stream);
/* grad_y [M, C] -> grad_x [M, C], grad_weight / grad_bias [C] (dtype, overwritten). */
VS_API int vs_layer_norm_backward(int dtype, const void* grad_y, const void* x, const void* weight,
                                  const float* mean, const float* rstd, void* grad_x, void* grad_weight,
                                  void* grad_bias, void* workspace, int rows, int cols, void* stream);
/* Row-mapped variants: the Swin window partition (HF:swin:546-551: pad, roll, partition)
 * folded into the LayerNorm that precedes it.  y row m is written at row y_rows[m] of y
 * (the window-layout row of image token m; y has as many rows as the windows hold, the
 * padding rows are the caller's), and the backward reads grad_y row m from row
 * dy_rows[m].  Otherwise as vs_layer_norm_forward / vs_add_layer_norm_forward /
 * vs_layer_norm_backward_ex. */
VS_API int vs_layer_norm_forward_rows(int dtype, const void* x, const void* weight, const void* bias, void* y,
                                      float* mean, float* rstd, int rows, int cols, float eps, const int* y_rows,
                                      void* stream);
VS_API int vs_add_layer_norm_forward_rows(int dtype, const void* x, const void* r, const void* w, const void* b,
                                          void* s, void* y, float* mean, float* rstd, int M, int C, float eps,
                                          const int* y_rows, void* stream);
VS_API int vs_layer_norm_backward_rows(int dtype, const void* grad_y, const void* x, const void* weight,
                                       const float* mean, const float* rstd, const void* grad_res, void* grad_x,
                                       void* grad_weight, void* grad_bias, void* dx_colsum, void* workspace,
                                       int rows, int cols, const int* dy_rows, void* stream);
VS_API long long vs_column_sum_workspace_bytes(int rows, int cols);
/* out[n] = sum_m x[m, n] (f32 accumulation, fixed order); N a multiple of 8, <= 2048. */
VS_API int vs_column_sum(int dtype, const void* x, void* out, void* workspace, int rows, int cols,
                         void* stream);
/* a4: the relative-position-table gradient from the window-attention backward's per-window
 * partials part [P, heads, T] (f32, T = (2 ws - 1)^2) -> out [T, heads] (dtype VS_BF16 /
 * VS_F32: the table's own layout and dtype), summed in a fixed order (deterministic).  The
 * rows are folded F at a time so the column-sum width is a multiple of 8 (F = 1, 2, 4 or 8
 * by heads * T): P % F == 0.  Workspace from vs_rel_table_grad_workspace_bytes.  Replaces
 * the table gradient autograd forms for HF:swin's relative_position_bias_table gather. */
VS_API long long vs_rel_table_grad_workspace_bytes(int P, int heads, int T);
VS_API int vs_rel_table_grad(int dtype, const float* part, void* out, void* ws, int P, int heads, int T, void* stream);
VS_API long long vs_column_sum_segments_workspace_bytes(int batch, int cols, int nseg);
/* Per-segment column sums of x [B, S, N] (f32 out [nseg, N], fixed order): segment k =
 * rows [seg_start[k], seg_start[k+1]) of every image (host array of nseg + 1 ints,
 * nseg <= 8).  The level-embedding gradient of a multi-scale encoder: the encoder token
 * sequence is the levels concatenated (HF:m2f:1236-1290 level_embed + position). */
VS_API int vs_column_sum_segments(int dtype, const void* x, float* out, void* workspace, int batch, int rows,
                                  int cols, const int* seg_start, int nseg, void* stream);

/* ---- Fused optimiser step over flat buffers (csrc/optim.hip) --------------------------
 * Replaces detectron2's clipped optimiser step as the reference runs it
 * (training/maskdino/train_full.py:153-167 DefaultTrainer.build_optimizer -> torch SGD,
 * momentum 0.9, weight decay 0.05 / 0 on norm parameters; CLIP_GRADIENTS "norm" 0.01 =
 * clip_grad_norm_(p, 0.01) per parameter, :266-271), or upstream Mask2Former/MaskDINO's
 * AdamW.  All buffers are flat device arrays over the same element index:
 *   grad      [total] f32 or bf16 (grad_dtype), scaled by grad_scale (1/world: summed
 *             gradients -> mean) before clipping;
 *   master    [total] f32 weights, state1 [total] f32 (SGD momentum / Adam exp_avg),
 *   state2    [total] f32 (Adam exp_avg_sq; unused, may be NULL, for SGD);
 *   weights_bf16 [total] bf16 working weights written from the updated master (or NULL).
 * grad_flags [num_params] (grad_dtype, or NULL = every parameter has a gradient): > 0.5
 *             when the parameter got a gradient this step on some rank (the all-reduce sums
 *             them); a parameter without one is skipped entirely, as torch.optim skips a
 *             parameter whose .grad is None (no decay, no state update).
 * table: int32 [num_chunks][5] = {start (multiple of 8), len, first chunk of the
 * parameter, chunks of the parameter, parameter index}; hyper: f32 [num_chunks][2] = {lr
 * multiplier, weight decay}.  optimizer 0 = SGD (torch semantics: d = g + wd*p; buf = d on
 * the parameter's first step, else momentum*buf + d; p -= lr*buf), 1 = AdamW (torch
 * semantics, bias correction by the parameter's own step count).  clip 0 = none,
 * 1 = per parameter, 2 = one global norm; scale = min(1, clip_value / (norm + clip_eps)).
 * lr: device f32 scalar (base lr, scheduler-owned); step: device f32 counter, advanced by
 * one at the start of the call; param_steps: f32 [num_params], each flagged parameter's
 * count advanced by one (== 1 on its first step).  Deterministic; 2 launches (3 with the
 * global clip).  workspace: vs_flat_step_workspace_bytes(num_chunks) bytes. */
VS_API long long vs_flat_step_workspace_bytes(int num_chunks);
VS_API int vs_flat_step(int grad_dtype, const void* grad, const void* grad_flags, float grad_scale, float* master,
                        float* state1, float* state2, void* weights_bf16, const int* table, const float* hyper,
                        int num_chunks, int optimizer, int clip, float clip_value, float clip_eps, float momentum,
                        float beta1, float beta2, float eps, const float* lr, float* step, float* param_steps,
                        void* workspace, void* stream);

/* ---- In-graph external events (csrc/stream.hip) ----------------------------------------
 * For the gradient all-reduce overlapped with a graph-replayed backward (no reference
 * counterpart: the reference's DDP all-reduce is eager, detectron2 create_ddp_model).
 * vs_event_record_external records `event` on `stream` with hipEventRecordExternal: under
 * stream capture it becomes an event-record node of the graph, fired when the replay
 * reaches it; vs_stream_wait_event makes `stream` wait on the event's last record. */
VS_API int vs_event_create(void** event);
VS_API int vs_event_destroy(void* event);
VS_API int vs_event_record_external(void* event, void* stream);
VS_API int vs_stream_wait_event(void* stream, void* event);

/* ---- Hungarian matching on the device (csrc/match.hip) -------------------------------
 * Replaces scipy.optimize.linear_sum_assignment(cost.cpu()) of the set-criterion matcher
 * (HF:m2f:489-491; upstream Mask2Former/MaskDINO matcher.py), batched over decoder steps
 * and images.  cost: device f32 [steps, batch, queries, max_targets] (problem (s, b) uses
 * its first targets_per_image[b] target columns); targets_per_image: HOST int [batch].
 * assign: device int32 [steps, batch, max_targets] = the query matched to each target
 * (-1 past the image's target count).  Minimum-total-cost assignment of every target to
 * a distinct query (targets <= queries <= 1024).  vs_lsa_max_targets(Q) = the largest
 * per-image target count the kernel accepts for Q queries. */
VS_API int vs_lsa_max_targets(int num_queries);
VS_API int vs_lsa_batch(const float* cost, const int* targets_per_image, int num_steps, int batch,
                        int num_queries, int max_targets, int* assign, void* stream);
/* Same, with the per-image target counts in DEVICE memory (int32 [batch], clamped to
 * [0, max_targets]): the launch does not depend on the counts, so a captured HIP graph
 * serves every batch whose largest count is <= max_targets (padded targets, see
 * visionseg/criterion.py PaddedTargets). */
/* Matcher cost matrix for every decoder step at once (HungarianMatcher, HF:m2f:413-481,
 * replacing its point_sample + pair-wise sigmoid-BCE / dice matmuls + class cost):
 * mask_logits = host array of num_steps device pointers, each f32 [B, Q, H, W];
 * class_probs f32 [S, B, Q, C+1] (softmax); target_classes int64 [B, Kc] (padded);
 * points f32 [B, P, 2] in [-1, 1] (grid_sample order x, y; align_corners=False, zero
 * padding); target_point_labels f32 [B, Kc, P]  ->  cost f32 [S, B, Q, Kc]
 * (= wm * BCE + wc * (-prob) + wd * dice, clamped to +-1e10, NaN -> 0).  S <= 16, Kc <= 16. */
VS_API int vs_match_cost(const float* const* mask_logits, int num_steps, const float* class_probs,
                         int num_classes_plus1, const long long* target_classes, const float* points,
                         const float* target_point_labels, float* cost, int batch, int num_queries, int height,
                         int width, int num_points, int max_targets, float mask_weight, float class_weight,
                         float dice_weight, void* stream);

/* ---- Matcher from the mask head's factors (csrc/match_factors.hip) -------------------
 * The logits L_s[b, q, n] = E_s[b, q, :] . F[b, n, :] are never materialised at full
 * resolution for matching: bilinear resampling commutes with the product.
 * vs_feature_resize_hilo: F bf16 [B, H*W, C] -> out bf16 [B, th*tw, 2C], the bilinear
 *   (align_corners=False, PyTorch upsample_bilinear2d index rule) resize of F in f32 stored
 *   as hi = bf16(v) in channels [0, C) and lo = bf16(v - hi) in [C, 2C) (E . (hi + lo) =
 *   the resized logits to ~2^-17 relative; HF:m2f:2049-2055 resizes the logits).
 * vs_feature_sample_hilo: F at grid points f32 [B, P, 2] in [-1, 1] (grid_sample bilinear,
 *   zeros padding, align_corners=False; HF:m2f:245-275) -> out bf16 [B, P, 2C] (hi | lo).
 * vs_match_cost_factors: E bf16 [S, B, Q, C] (C in {64, 128, 256}), point_features from
 *   vs_feature_sample_hilo at the matcher's points, class_probs f32 [S, B, Q, C+1],
 *   target_classes int64 [B, Kc], target_point_labels f32 [B, Kc, P] -> cost f32
 *   [S, B, Q, Kc], the same cost as vs_match_cost over the logits E_s . F (HF:m2f:434-481).
 *   workspace: vs_match_cost_factors_workspace_bytes(S, B, Q, P, Kc) bytes of device
 *   scratch (per-point-range partial sums, reduced in a fixed order: deterministic). */
/* vs_level_bitmask_hilo: the attention bitmask (vs_attn_bitmask's format and rule,
 *   sigmoid(x) < 0.5 with the all-blocked row fix) of the logits E . (hi + lo) at a level of
 *   height x width keys, from E bf16 [B, Q, C] and level_features = vs_feature_resize_hilo's
 *   output [B, height*width, 2C]: words u32 [B, Q, ceil(height*width/32)]; the logits are
 *   never stored. */
VS_API int vs_level_bitmask_hilo(const void* mask_embed, const void* level_features, uint32_t* words, int batch,
                                 int num_queries, int channels, int height, int width, void* stream);
VS_API int vs_feature_resize_hilo(const void* features, void* out, int batch, int height, int width, int channels,
                                  int target_h, int target_w, void* stream);
VS_API int vs_feature_sample_hilo(const void* features, const float* grid, void* out, int batch, int height,
                                  int width, int channels, int num_points, void* stream);
VS_API long long vs_match_cost_factors_workspace_bytes(int num_steps, int batch, int num_queries, int num_points,
                                                       int max_targets);
VS_API int vs_match_cost_factors(const void* mask_embed, const void* point_features, int num_steps,
                                 const float* class_probs, int num_classes_plus1, const long long* target_classes,
                                 const float* target_point_labels, float* cost, void* workspace, int batch,
                                 int num_queries, int channels, int num_points, int max_targets, float mask_weight,
                                 float class_weight, float dice_weight, void* stream);

VS_API int vs_lsa_batch_device_counts(const float* cost, const int* targets_per_image_dev, int num_steps,
                                      int batch, int num_queries, int max_targets, int* assign, void* stream);

/* ---- GroupNorm over channels-last activations (csrc/groupnorm.hip) -------------------
 * The pixel decoder's Conv2d + GroupNorm(32) blocks (upstream MSDeformAttnPixelDecoder
 * input projections / lateral / output convs; HF:m2f Mask2FormerPixelDecoder) on MIOpen's
 * channels-last outputs.  x, y: [B, HW, C] (NHWC), groups of exactly 8 channels
 * (C = 8 G); weight/bias [C] in dtype; mean/rstd f32 [B, G]; relu != 0 fuses a ReLU
 * after the affine (the backward recomputes its mask from x).  torch.nn.functional.
 * group_norm semantics (biased variance). */
VS_API long long vs_group_norm_workspace_bytes(int batch, int hw, int channels, int groups);
VS_API int vs_group_norm_forward(int dtype, const void* x, const void* weight, const void* bias, void* y,
                                 float* mean, float* rstd, void* workspace, int batch, int hw, int channels,
                                 int groups, float eps, int relu, void* stream);
VS_API int vs_group_norm_backward(int dtype, const void* grad_y, const void* x, const void* weight,
                                  const void* bias, const float* mean, const float* rstd, void* grad_x,
                                  void* grad_weight, void* grad_bias, void* workspace, int batch, int hw,
                                  int channels, int groups, int relu, void* stream);

/* ---- GroupNorm over NCHW-contiguous activations (csrc/groupnorm.hip) ----------------
 * Same op as above for MIOpen's NCHW conv outputs (the 1/4-resolution lateral and output
 * ConvGN blocks of the pixel decoder, HF:m2f Mask2FormerPixelDecoder): x, y [B, C, HW],
 * any C % G == 0; each group is C/G contiguous channel planes, so no layout copies. */
VS_API long long vs_group_norm_nchw_workspace_bytes(int batch, int channels, int groups);
VS_API int vs_group_norm_nchw_forward(int dtype, const void* x, const void* weight, const void* bias, void* y,
                                      float* mean, float* rstd, void* workspace, int batch, int channels, int hw,
                                      int groups, float eps, int relu, void* stream);
VS_API int vs_group_norm_nchw_backward(int dtype, const void* grad_y, const void* x, const void* weight,
                                       const void* bias, const float* mean, const float* rstd, void* grad_x,
                                       void* grad_weight, void* grad_bias, void* workspace, int batch,
                                       int channels, int hw, int groups, int relu, void* stream);

/* ---- small-token Linear weight / bias gradient (csrc/small_linear.hip) ------------
 * Replaces the backward GEMM + bias reduction autograd runs for the masked-attention
 * decoder's Linears (HF:m2f Mask2FormerMaskedAttentionDecoderLayer q/k/v/out projections
 * and FFN, Mask2FormerMLPPredictionHead; B x Q = 400 tokens): grad_w[o, i] = sum_t
 * grad_y[t, o] x[t, i], grad_b[o] = sum_t grad_y[t, o] (grad_b may be NULL), f32
 * accumulation, bf16 in / out.  grad_y [tokens, out], x [tokens, in], grad_w [out, in],
 * out and in multiples of 64. */
VS_API int vs_small_linear_wgrad(int dtype, const void* grad_y, const void* x, void* grad_w, void* grad_b,
                                 int tokens, int out_features, int in_features, void* stream);

/* The same Linear's forward and whole backward, each one launch (bf16, f32 accumulation,
 * the reduction split over four waves and summed in a fixed order):
 *   forward:  y [tokens, out] = act(x' weight[out, in]^T (+ bias[out] when non-NULL)),
 *             x' = x [tokens, in] (+ pos when non-NULL: pos row t % pos_rows, the sum
 *             rounded to bf16 like torch's add), act = ReLU when relu != 0
 *   backward: g = grad_y, masked where relu_out (the forward's ReLU output; NULL: no
 *             ReLU) is not positive; grad_x [tokens, in] = g weight (skipped when grad_x is
 *             NULL; grad_pos, when non-NULL, receives the same per-token rows: the gradient
 *             of pos; added to what grad_pos holds when accumulate_pos != 0: several
 *             consumers of one position table sum into one buffer) and grad_w = g^T x',
 *             grad_b = colsum g; grad_res (may be NULL) is added to grad_x only: the
 *             residual-path gradient of x (one rounding instead of a separate add)
 *             (as vs_small_linear_wgrad; skipped when grad_w is NULL), both in one grid.
 * Replaces autograd's addmm forward, F.relu and its threshold_backward, and the mm input
 * gradient for the decoder Linears above (torch.nn.functional.linear / LinearBackward;
 * HF:m2f:1730-1745 with_pos_embed for the cross-attention query). */
VS_API int vs_small_linear_forward(int dtype, const void* x, const void* pos, int pos_rows, const void* weight,
                                   const void* bias, int relu, void* y, int tokens, int out_features,
                                   int in_features, void* stream);
VS_API int vs_small_linear_backward(int dtype, const void* grad_y, const void* x, const void* pos, int pos_rows,
                                    const void* weight, const void* relu_out, const void* grad_res, void* grad_x,
                                    void* grad_pos, int accumulate_pos, void* grad_w, void* grad_b, int tokens,
                                    int out_features, int in_features, void* stream);

/* The self-attention input projections of a masked-attention decoder layer (HF:m2f
 * Mask2FormerMaskedAttentionDecoderLayer.forward_post: q = k = hidden + query_pos,
 * v = hidden; Mask2FormerAttention q_proj / k_proj / v_proj), bf16, [tokens, dim] rows,
 * dim x dim weights, arrays of 3 pointers in q, k, v order:
 *   forward:  outs[0] = (h + pos) Wq^T + bq, outs[1] = (h + pos) Wk^T + bk,
 *             outs[2] = h Wv^T + bv                     -- one launch
 *   backward: grad_pos (+)= dq Wq + dk Wk (may be NULL; accumulated into when
 *             accumulate_pos != 0), grad_h = dq Wq + dk Wk + dv Wv (+ grad_res, the
 *             residual-path gradient of h, when non-NULL), and the three weight / bias
 *             gradients                                   -- one launch
 * pos row of token t is t % pos_rows (pos_rows = queries: the query-position table
 * broadcast over the batch; = tokens: a full tensor); grad_pos is per token [tokens, dim].
 * h + pos is rounded to bf16 before the products (torch's bf16 add).  Replaces the add,
 * three Linear forwards and their backwards plus autograd's gradient adds. */
VS_API int vs_self_attn_in_proj_forward(int dtype, const void* h, const void* pos, int pos_rows,
                                        const void* const* weights, const void* const* biases, void* const* outs,
                                        int tokens, int dim, void* stream);
VS_API int vs_self_attn_in_proj_backward(int dtype, const void* h, const void* pos, int pos_rows,
                                         const void* const* weights, const void* const* grad_outs,
                                         const void* grad_res, void* grad_h, void* grad_pos, int accumulate_pos,
                                         void* const* grad_weights, void* const* grad_biases, int tokens, int dim,
                                         void* stream);

/* ---- activation backward + bias gradient (csrc/norm.hip) ------------------------------
 * dx = dy * act'(x) for act 0 = ReLU, 1 = exact GELU (torch's F.gelu, approximate='none'),
 * x the activation's input, all [M, N] dtype; dx_colsum [N] dtype = column sums of dx as
 * stored (the bias gradient of the Linear that produced x: Swin MLP fc1, encoder FFN fc1).
 * workspace: vs_column_sum_workspace_bytes(M, N) bytes. */
VS_API int vs_act_backward_colsum(int dtype, int act, const void* grad_y, const void* x, void* grad_x,
                                  void* dx_colsum, void* workspace, int rows, int cols, void* stream);

/* ---- split-K epilogue (csrc/norm.hip) -------------------------------------------------
 * out[i] = sum_{s < num_parts} partials[s * n + i] (+ extra[i] when extra != NULL), f32
 * accumulation in a fixed order, out in dtype: the weight gradient of a token-major
 * Linear computed as a batched GEMM over token chunks (visionseg/linear.py).  n % 4 == 0. */
VS_API int vs_splitk_sum(int dtype, const float* partials, int num_parts, long long n, const float* extra,
                         void* out, void* stream);

/* ---- a9: pixel-decoder FPN merge ----------------------------------------------------
 * out[B, C, H, W] = cur + bilinear_upsample(src) (align_corners=False, HF:m2f:1405-1413),
 * cur / out NCHW, src token-major [B, Hs*Ws, C] with batch stride src_batch_stride
 * (elements; token stride C); upsampling factor in [1, 2], C % 32 == 0.  The upsampled
 * value is rounded to dtype before the add (as F.interpolate + add). */
VS_API int vs_upsample_add_forward(int dtype, const void* cur, const void* src, void* out, int batch, int channels,
                                   int height, int width, int src_height, int src_width, long long src_batch_stride,
                                   void* stream);
/* grad_src [B, Hs*Ws, C] (contiguous, overwritten) = adjoint of the upsample applied to
 * grad_out [B, C, H, W]; fixed-order gather, no atomics. */
VS_API int vs_upsample_backward(int dtype, const void* grad_out, void* grad_src, int batch, int channels, int height,
                                int width, int src_height, int src_width, void* stream);
/* Channels-last forms (the bf16 NHWC 1/4-resolution tail): cur / out / grad_out
 * [B, H, W, C] contiguous, src / grad_src token-major [B, Hs*Ws, C]; C % 8 == 0, operands
 * 16-B aligned.  Same arithmetic as the NCHW forms. */
VS_API int vs_upsample_add_forward_nhwc(int dtype, const void* cur, const void* src, void* out, int batch,
                                        int channels, int height, int width, int src_height, int src_width,
                                        long long src_batch_stride, void* stream);
VS_API int vs_upsample_backward_nhwc(int dtype, const void* grad_out, void* grad_src, int batch, int channels,
                                     int height, int width, int src_height, int src_width, void* stream);

/* ---- a5-a7: weight (+ bias) gradient of a token-major Linear ---------------------------
 * dw [N, K] (dtype VS_BF16 / VS_F32, overwritten) = sum_t grad_y[t, n] x[t, k] and, when db
 * is non-NULL, db [N] = sum_t grad_y[t, n]; bf16 operands with row strides ld_grad_y /
 * ld_x (elements, % 8 == 0), unit column stride, 16-B aligned; N % 8 == 0, K % 8 == 0,
 * 0 < tokens < 2^31.  f32 accumulation: per-split partials in workspace (size from
 * vs_token_wgrad_workspace_bytes), summed in a fixed order (deterministic, no atomics).
 * Replaces autograd's gy^T x of F.linear's backward (the reference's Linears, HF:swin /
 * HF:m2f) for the token-heavy Linears. */
VS_API long long vs_token_wgrad_workspace_bytes(long long tokens, int N, int K);
/* A GROUP of independent token-Linear weight gradients in one launch (plus one reduction
 * launch when some are split): the plan spreads the Linears' tiles over the CUs, so most run
 * unsplit and write dw / db directly.  Every problem as for vs_token_wgrad (db may be NULL;
 * dw / db 16-B aligned); dtype applies to all dw / db.  Workspace from
 * vs_token_wgrad_grouped_workspace_bytes(probs, n) (the same list). */
typedef struct {
  const void* grad_y;
  const void* x;
  void* dw;
  void* db;
  long long ld_grad_y, ld_x, tokens;
  int N, K;
} vs_wgrad_problem;
VS_API long long vs_token_wgrad_grouped_workspace_bytes(const vs_wgrad_problem* probs, int n);
VS_API int vs_token_wgrad_grouped(int dtype, const vs_wgrad_problem* probs, int n, void* workspace, void* stream);
VS_API int vs_token_wgrad(int dtype, const void* grad_y, long long ld_grad_y, const void* x, long long ld_x, void* dw,
                          void* db, void* workspace, long long tokens, int N, int K, void* stream);

/* ---- a5-a7: W^T copies for the token Linears' input gradient -------------------------
 * dst [cols, rows] = src [rows, cols]^T for a LIST of bf16 matrices (dtype VS_BF16) in one
 * launch per 64 matrices; rows % 8 == 0, cols % 8 == 0, src / dst contiguous and 16-B
 * aligned.  The dX = dY W GEMM of a token Linear (autograd's backward of F.linear, HF:swin /
 * HF:m2f) runs on vs_token_gemm with W^T as its K-contiguous operand; this replaces one
 * strided-copy launch per Linear. */
typedef struct {
  const void* src;
  void* dst;
  int rows, cols;
} vs_transpose_item;
VS_API int vs_transpose_batched(int dtype, const vs_transpose_item* items, int n, void* stream);

/* ---- a9: the FPN's 3 x 3 output conv on NHWC planes (replaces MIOpen's conv + layout
 * transposes under nn.Conv2d(256, 256, 3, padding=1, bias=False), HF:m2f:1394-1419).
 * Stride 1, padding 1, bf16, channels-last x [B, H, W, Ci], y [B, H, W, Co].
 * vs_conv3x3_forward: y = conv(x) (+ bias[Co] when non-NULL) with the weights in the layout
 * w_fwd [Co, 3, 3, Ci]; Ci % 64 == 0, Co % 8 == 0.  The input gradient is the same call on
 * grad_y with w_bwd [Ci, 3, 3, Co] (the flipped transpose: Ci and Co swap roles).
 * vs_conv3x3_weight_layouts: w [Co, Ci, 3, 3] (torch) -> w_fwd and/or w_bwd (either NULL).
 * vs_conv3x3_wgrad: dw [Co, Ci, 3, 3] (dtype VS_BF16 / VS_F32, overwritten) = sum over pixels
 * of grad_y (x) x-neighbourhood; f32 partial sums in workspace (size from
 * vs_conv3x3_wgrad_workspace_bytes, 0 = unsupported shape), reduced in a fixed order.
 * Ci % 128 == 0 and Co % 128 == 0. */
VS_API int vs_conv3x3_forward(const void* x, const void* w_fwd, const void* bias, void* y, int batch, int height,
                              int width, int in_channels, int out_channels, void* stream);
VS_API int vs_conv3x3_weight_layouts(const void* w, void* w_fwd, void* w_bwd, int out_channels, int in_channels,
                                     void* stream);
VS_API long long vs_conv3x3_wgrad_workspace_bytes(int batch, int height, int width, int in_channels,
                                                  int out_channels);
VS_API int vs_conv3x3_wgrad(int dtype, const void* grad_y, const void* x, void* dw, void* workspace, int batch,
                            int height, int width, int in_channels, int out_channels, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* VISIONSEG_H_ */
