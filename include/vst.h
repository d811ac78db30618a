/*
 * vst.h — C ABI of libvst_hip.so, the MI355X (gfx950) kernels behind the AnimateDiff-XL +
 * UnZipLoRA denoising path of tanmud/video_style_transfer.
 *
 * The reference is pure Python/PyTorch; its "FFI" for this path is the set of torch ops its
 * plug-in classes call.  Each entry point below replaces one of those call sites (cited as
 * reference file:line).  Conventions:
 *   - all tensors are device pointers (bf16 unless stated), caller-owned; no allocation inside
 *     except none at all — workspaces are caller-provided (see *_workspace_bytes);
 *   - activations are token-major NHWC: row = (frame * H*W + pixel), C contiguous;
 *   - `stream` is a hipStream_t; every call is asynchronous on it and graph-capturable;
 *   - return 0 (VST_OK) on success, 1 for a bad argument, 2 for a launch failure, 3 for a
 *     supported-shape refusal (vst_gemm_lora, vst_gemm_cross_attention).
 */
#ifndef VST_H
#define VST_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Dense projection C = A.W^T (+bias) (+row_bias[m/div]) (+R), fp32 accumulate.
 * A2 != NULL splits A along K: columns [0,K1) from A, [K1,K) from A2 (K1 % 64 == 0).
 * With A2 = x.Acat^T and W = [W_base | s.(B (.) merger)] this is the fused base + UnZipLoRA
 * projection: replaces LoRACompatibleLinear.forward (unziplora_unet/lora_linear.py:74-81) +
 * UnZipLoRALinearLayerInfer.forward (unziplora_unet/unziplora_linear_layer.py:298-346), and
 * TemporalLoRALinear.forward (animatediff/temporal_lora.py:29-32).
 * epilogue 0: plain; 1: GEGLU (diffusers GEGLU feed-forward, unziplora_unet/unzip_attention.py
 * ff path) with hidden/gate rows interleaved per 32-column block ([32 h | 32 g] per 64 rows), output width N/2; 2: GELU(erf) after
 * the bias, no residual / row bias (TemporalTransformerBlock.ffn, animatediff/temporal_transformer.py:53-59). */
int vst_gemm(const void* A, int lda, const void* A2, int lda2, int K1, const void* W, int ldw, int M, int N, int K,
             const float* bias, const float* row_bias, int row_bias_div, int ld_row_bias, const void* R, int ldr,
             void* C, int ldc, int epilogue, void* stream);
/* Same, with the tile (0 auto, 1 = 128x128, 2 = 128x64, 3 = 256x256, 4 = 256x128, 5 = skinny N <= 64
 * without epilogue: the UnZipLoRA down-projection) and split-K (0 auto, >= 1 forced) choice and a
 * caller-owned fp32 workspace for split-K slabs (NULL / too small disables split-K).  An A / A2 / R / C
 * whose byte extent passes 2^31 - 1 (the kernels' 32-bit buffer offsets) is run as equal row chunks, each row
 * with the bits of one launch. */
int vst_gemm_ex(const void* A, int lda, const void* A2, int lda2, int K1, const void* W, int ldw, int M, int N, int K,
                const float* bias, const float* row_bias, int row_bias_div, int ld_row_bias, const void* R, int ldr,
                void* C, int ldc, int epilogue, int tile, int splits, void* workspace, size_t ws_bytes,
                void* stream);
size_t vst_gemm_workspace_bytes(int M, int N, int K);

/* Fused base + LoRA projection with the LoRA down-projection computed INSIDE the GEMM:
 *   C = [x | bf16(x.Acat^T)] . W^T (+bias) (+R),  W = [W_base | V] of width ldw >= K + P,
 * where Acat [P][K] (row stride ld_acat, zero rows past the real rank) holds the stacked down
 * factors (UnZipLoRA: [A_c; A_s]) and V's column block [g*group_r, (g+1)*group_r) carries the up
 * factors (s.(B (.) merger)) of the output columns n with n / group_n == g (q/k/v stacked: group_n =
 * C, group_r = 2r).  The 8-phase kernel accumulates u = x.Acat^T from the x tiles it already
 * streams, rounds it to bf16 (the reference's rounding point of the down output) and adds u.V^T
 * as one extra k-step: no separate pass over x (replaces the down half of
 * UnZipLoRALinearLayerInfer.forward, unziplora_unet/unziplora_linear_layer.py:298-346, inside
 * LoRACompatibleLinear.forward, unziplora_unet/lora_linear.py:74-81).  Returns 3
 * (VST_ERR_UNSUPPORTED) when the shape is not on the 8-phase kernel or a tile would need u columns
 * outside one 16-aligned block; vst_gemm_lora_supported answers that without a launch (0, or the
 * tile width 256 / 192 / 320 it uses; 320-wide tiles are 128 rows high). */
int vst_gemm_lora(const void* x, int ldx, const void* Acat, int ld_acat, int P, int group_n, int group_r,
                  const void* W, int ldw, int M, int N, int K, const float* bias, const void* R, int ldr,
                  void* C, int ldc, void* stream);
int vst_gemm_lora_supported(int M, int N, int K, int P, int group_n, int group_r);
/* Test / A-B knob: force the 8-phase kernel's tile width (256, 192 or 320 where legal; 0 = automatic policy) for
 * every later GEMM of this process; returns the previous setting.  Not on the product path. */
int vst_p8_force_bn(int bn);
/* Test / A-B knob: 3x3 convs whose channel sources are multiples of 64 run on the 8-phase kernel (1) or the ring
 * kernel (0) for every later conv of this process (default: VST_P8_CONV, else 1); returns the previous setting. */
int vst_p8_conv(int on);
/* Test / A-B knob: the 8-phase kernel's persistent grid (one workgroup per CU walking the tiles, each tile's last
 * k-tiles streaming the next tile's first ones) for GEMMs of two or more tile rounds (1) or one workgroup per tile
 * (0), for every later GEMM of this process (default: VST_P8_PERSIST, else 1; not the convs); returns the previous
 * setting.  Same bits. */
int vst_p8_persist(int on);

/* The motion-module attention's q/k/v projection and its frame-axis self-attention as ONE launch:
 *   O[(c, f, p), 40h .. 40h+39] = softmax(q_h[c,.,p] k_h[c,.,p]^T * scale) v_h[c,.,p]  over the 16 frames of pixel p,
 *   [q | k | v] = x . W^T (+ bias) rounded to bf16,
 * x: [nclip * 16 * HW, K] rows (clip, frame, pixel); Wt: the q/k/v weight rows laid out per group of 256 / (3 d)
 * heads (two of 40: [q_2t k_2t v_2t q_2t+1 k_2t+1 v_2t+1]; one of 80: [q_t k_t v_t]) + zero rows up to 256, i.e.
 * [heads / hpt * 256, K] (bias alike, fp32 or NULL).  q/k/v never reach HBM.  Replaces to_q/to_k/to_v +
 * F.scaled_dot_product_attention of the motion modules' AttnProcessor2_0 (diffusers AnimateDiffTransformer3D;
 * animatediff/temporal_transformer.py:40-71) for head_dim 40 / 80 and 16 frames (the 64^2 and 32^2 levels of
 * configs[2]); returns 3 (VST_ERR_UNSUPPORTED) otherwise, _supported answers without a launch. */
int vst_gemm_temporal_attention(const void* x, int ldx, const void* Wt, int ldw, const float* bias, int M, int K,
                                int nclip, int F, int HW, int heads, int head_dim, float scale, void* O, int ldo,
                                void* stream);
int vst_gemm_temporal_attention_supported(int M, int K, int nclip, int F, int HW, int heads, int head_dim);

/* attn2 of a BasicTransformerBlock as ONE launch: the q projection (vst_gemm_lora when Acat != NULL, else
 * [x].[W]^T) with the cross-attention over the text tokens as its epilogue,
 *   O[m, 64h .. 64h+63] = softmax(q_h K_h^T * scale) V_h,  q = bf16(x.W^T (+bias) (+LoRA)),
 * K/V rows [(frame / kv_div) * Nk + key] (frame = m / Nq; nkv_rows rows in all, row stride ldkv, head h at
 * columns 64h).  q never reaches HBM.  Replaces to_q (lora_linear.py:74-81) + F.scaled_dot_product_attention
 * (animatediff/attention_processor.py:78-80) of AnimateDiffAttnProcessor2_0 with encoder_hidden_states.
 * Needs Nq % 256 == 0, Nk <= 80, N % 64 == 0 and the 8-phase kernel's 256x192 tiles for (M, N); returns 3
 * (VST_ERR_UNSUPPORTED) otherwise.  _supported answers without a launch (lora: Acat will be non-NULL). */
int vst_gemm_cross_attention(const void* x, int ldx, const void* Acat, int ld_acat, int P, int group_n, int group_r,
                             const void* W, int ldw, const float* bias, int M, int N, int K, const void* Kt,
                             const void* Vt, int ldkv, int nkv_rows, int Nq, int Nk, int kv_div, float scale, void* O,
                             int ldo, void* stream);
int vst_gemm_cross_attention_supported(int M, int N, int K, int lora, int P, int group_n, int group_r, int Nq,
                                       int Nk);

/* Diagnostics: short name of the kernel (tile shape, epilogue, split-K) that a vst_gemm_ex
 * (kind 0 linear, 1 GEGLU) or vst_conv3x3_ex (kind 2, kind 3 = Cin not a multiple of 64) call with
 * these sizes and policy would launch.  Used by bench.py to attribute per-launch timings. */
const char* vst_gemm_kernel_name(int M, int N, int K, int kind, int tile, int splits, size_t ws_bytes);

/* 3x3 conv, padding 1, NHWC, optional channel-concat second input, stride 1|2, fused nearest-2x
 * upsample; Wt = [Cout][3][3][C1+C2].  Replaces the per-frame torch conv2d calls of diffusers
 * ResnetBlock2D / Downsample2D / Upsample2D inside UNetMotionModel (called from
 * inference_animatediff.py:110-121); temb add fused as row_bias[frame][Cout]. */
int vst_conv3x3(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W, int stride, int upsample,
                const void* Wt, int Cout, const float* bias, const float* row_bias, int row_bias_div, const void* R,
                int ldr, void* out, int ldc, void* stream);
/* _ex: + tile / split-K policy and workspace (as vst_gemm_ex) and the row stride of row_bias (0 = Cout), so
 * the time-embedding projections of every ResnetBlock2D can come from ONE batched GEMM output.  Inputs /
 * outputs past 2^31 - 1 bytes run as chunks of whole images (row_bias then must be per image: row_bias_div =
 * OH * OW; VST_ERR_UNSUPPORTED otherwise). */
int vst_conv3x3_ex(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W, int stride, int upsample,
                   const void* Wt, int Cout, const float* bias, const float* row_bias, int row_bias_div,
                   int ld_row_bias, const void* R, int ldr, void* out, int ldc, int tile, int splits, void* workspace,
                   size_t ws_bytes, void* stream);
/* + the GroupNorm column statistics of the stored output, colstat [ceil(M/128)][Cout][2] fp32 (sum, sum of squares
 * per 128-row tile and channel) for vst_groupnorm_colstat; returns 3 (unsupported, nothing launched) unless the
 * conv runs on the 8-phase kernel's 128x320 tiles (Cout % 320 == 0). */
int vst_conv3x3_colstat(const void* x1, int C1, const void* x2, int C2, int nimg, int H, int W, int stride,
                        int upsample, const void* Wt, int Cout, const float* bias, const float* row_bias,
                        int row_bias_div, int ld_row_bias, const void* R, int ldr, void* out, int ldc,
                        float* colstat, void* stream);

/* Spatial SDPA, head_dim 64: replaces F.scaled_dot_product_attention in
 * AnimateDiffAttnProcessor2_0.__call__ (animatediff/attention_processor.py:78-80).  K/V row
 * batch = q batch / kv_div (replaces the repeat_interleave of text states, :63-66). */
int vst_spatial_attention(const void* q, int ldq, const void* k, const void* v, int ldkv, void* o, int ldo,
                          int nbatch, int heads, int Nq, int Nk, int kv_div, int head_dim, float scale, float* lse,
                          void* stream);  /* lse: NULL, or fp32 [nbatch*heads*Nq] log2-domain logsumexp (training) */
/* Self-attention over 64+ keys (kv_div 1) on sa_self_kernel (1, default: VST_SA_SELF, else 1) or on the general
 * spatial kernel (0), for every later vst_spatial_attention of this process; returns the previous setting.  Same
 * bits either way (tests / A/B). */
int vst_sa_self(int on);

/* Frame-axis attention (motion module / TemporalTransformerBlock, animatediff/temporal_transformer.py:66-68):
 * token (clip b, frame f, pixel p) at row (b*F + f)*HW + p; F <= 32; head_dim in {8,16,32,40,64,80,160}. */
int vst_temporal_attention(const void* q, const void* k, const void* v, int ldqkv, void* o, int ldo, int nclip,
                           int F, int HW, int heads, int head_dim, float scale, void* stream);

/* One attention half of a motion-module BasicTransformerBlock in ONE launch (the fused temporal block of SURVEY
 * §8(d)):  y = x + to_out(softmax_over_frames(q k^T * scale) v),  [q | k | v] = (LayerNorm(x) + pe[frame]) . wqkv^T
 * (+ bqkv), to_out = . wo^T + bo; token (clip b, frame f, pixel p) at row (b*F + f)*HW + p; pe: [F][C] fp32 or NULL.
 * Replaces norm1/norm2 (+ the sinusoidal PE, animatediff/temporal_transformer.py:11-27), attn1/attn2 with the default
 * processor and the residual add of the motion module's BasicTransformerBlock (unziplora_unet/unzip_attention.py:
 * 150-151, 196-197; core: temporal_transformer.py:66-68).  C = 320 (the 64x64 level), 8 heads, F = 16, HW % 8 == 0;
 * returns 3 (VST_ERR_UNSUPPORTED) otherwise, which _supported answers without a launch.  Out of place (y != x).
 * The UNet uses it only with VST_MOTION_FUSE=1: it measured slower than the four launches. */
int vst_motion_attention_block(const void* x, int ldx, int nclip, int F, int HW, int C, int heads, const float* gamma,
                               const float* beta, float eps, const float* pe, const void* wqkv, int ldw,
                               const float* bqkv, const void* wo, int ldwo, const float* bo, float scale, void* y,
                               int ldy, void* stream);
int vst_motion_attention_block_supported(int C, int F, int HW, int heads);

/* GroupNorm (+SiLU) over NHWC samples of rows_per_sample rows; optional 2-source channel concat. */
size_t vst_groupnorm_workspace_bytes(int nsamples, int rows_per_sample, int groups, int C);
int vst_groupnorm(const void* x1, int ld1, int C1, const void* x2, int ld2, int C2, int nsamples,
                  int rows_per_sample, int groups, float eps, const float* gamma, const float* beta, int silu_act,
                  void* y, int ldy, void* workspace, void* stream);
/* Column statistics of x [M, C] (C % 8 == 0) in the arithmetic of vst_conv3x3_colstat's epilogue, cs
 * [ceil(M/128)][C][2] fp32: for a GroupNorm input whose producer did not write them (same bits if it had). */
int vst_colstat(const void* x, int ldx, int M, int C, float* cs, void* stream);
/* vst_groupnorm with its statistics from the column statistics the producing conv wrote (vst_conv3x3_colstat;
 * cs2 for x2's channels), so the GroupNorm does not read x for them: rows_per_sample % 128 == 0. */
int vst_groupnorm_colstat(const void* x1, int ld1, int C1, const float* cs1, const void* x2, int ld2, int C2,
                          const float* cs2, int nsamples, int rows_per_sample, int groups, float eps,
                          const float* gamma, const float* beta, int silu_act, void* y, int ldy, void* workspace,
                          void* stream);

/* GroupNorm (+SiLU) over NHWC samples of rows_per_sample rows; a frame's statistics depend only on its own rows
 * (the chunking is a function of rows_per_sample, not of how many samples share the launch). */

/* Motion-module GroupNorm (diffusers AnimateDiffTransformer3D norm, built at animatediff/utils.py:31: statistics
 * over every frame of a clip), frame-sharded or not.  vst_groupnorm_frame_partials writes fp32 (sum, sumsq) chunk
 * partials per frame, [nframes][vst_groupnorm_frame_chunks(rows_per_frame)][groups][2]; a frame's partials depend
 * only on that frame.  vst_groupnorm_apply_partials merges the partials of every frame of each clip in one fixed
 * order (fp64) and normalises this rank's rows: `part` is the rank-major all-gather of every rank's partials,
 * [nranks][nclips][frames_local][chunks][groups][2] (nranks = 1: this process holds the whole clip), so a
 * frame-sharded forward gets bit-identical statistics to the unsharded one.  scale_shift: caller-owned fp32
 * [2 * nclips * C], 16-byte aligned. */
int vst_groupnorm_frame_chunks(int rows_per_frame);
int vst_groupnorm_frame_partials(const void* x1, int ld1, int C1, int nframes, int rows_per_frame, int groups,
                                 float* part, void* stream);
int vst_groupnorm_apply_partials(const void* x1, int ld1, int C1, int nclips, int frames_local, int rows_per_frame,
                                 int groups, const float* part, int nranks, float eps, const float* gamma,
                                 const float* beta, int silu_act, void* y, int ldy, float* scale_shift, void* stream);

/* LayerNorm over C (+ sinusoidal PE row pe[(row/pe_div)%pe_mod], temporal_transformer.py:6-27). */
int vst_layernorm(const void* x, int ldx, int C, int rows, const float* gamma, const float* beta, float eps,
                  const float* pe, int pe_div, int pe_mod, void* y, int ldy, void* stream);

/* LayerNorm fused with the UnZipLoRA down-projection of the projections that consume it: y = LN(x) and
 * u = y . A^T (A: [R, C] bf16, R <= 64, R % 16 == 0; C % 32 == 0, C <= 1280), x read once.  Replaces the
 * BasicTransformerBlock norm1/norm2 LayerNorm (unziplora_unet/unzip_attention.py:113-239) followed by the
 * lora_down half of UnZipLoRALinearLayerInfer.forward (unziplora_linear_layer.py:298-346) on q/k/v. */
int vst_layernorm_lora(const void* x, int ldx, int C, int rows, const float* gamma, const float* beta, float eps,
                       const void* A, int R, void* y, int ldy, void* u, int ldu, void* stream);

/* SDXL text encoders (encode_prompt, inference_animatediff.py:16-35 / train_animatediff.py:29-50; transformers
 * CLIPTextModel / CLIPTextModelWithProjection):
 * vst_embed_tokens: CLIPTextEmbeddings, y[r] = token_embedding[ids[r]] + position_embedding[r % L] (ids int32, in
 *   range: checked by the caller; y fp32, the towers' residual stream);
 * vst_residual_layernorm: the encoder layer's residual add in fp32 (h_out = h + y, y bf16 or NULL) fused with the
 *   next LayerNorm (n = LN(h_out), bf16): the reference's fp32 text towers under bf16 autocast keep the residual
 *   stream fp32 (CLIPEncoderLayer, layer_norm1/2 and final_layer_norm);
 * vst_causal_attention: CLIPAttention's softmax(q k^T * scale + causal mask) v over N tokens, head_dim 64;
 * vst_quick_gelu: the CLIP ViT-L/14 MLP activation x * sigmoid(1.702 x). */
int vst_embed_tokens(const int* ids, int rows, int L, const void* tok, const void* pos, int C, float* y, int ldy,
                     void* stream);
int vst_residual_layernorm(const float* h, int ldh, const void* y, int ldy, int rows, int C, const float* gamma,
                           const float* beta, float eps, float* h_out, int ldho, void* n, int ldn, void* stream);
int vst_causal_attention(const void* q, int ldq, const void* k, const void* v, int ldkv, void* o, int ldo, int nbatch,
                         int heads, int N, int head_dim, float scale, void* stream);
int vst_quick_gelu(const void* x, void* y, size_t n, void* stream);

/* Row-block permutation: rows of C bf16 indexed (i0,i1,i2,i3) over dims (d0..d3) in src; dst
 * axis k is src axis p_k.  Used for the frame-shard <-> pixel-shard exchange around the motion
 * module's frame-axis attention (the reference's (B*F,HW,C) <-> (B*HW,F,C) permutes of
 * AnimateDiffTransformer3D, here across ranks). */
int vst_permute_rows(const void* src, void* dst, int C, int d0, int d1, int d2, int d3, int p0, int p1, int p2,
                     int p3, void* stream);

/* y[row] = x[row] + table[(row / div) % mod] (fp32 table [mod][C]): the reference TemporalTransformer's
 * PositionalEncoding.forward (animatediff/temporal_transformer.py:20-27) on token rows (b*F + f)*HW + p. */
int vst_add_row_table(const void* x, int ldx, int C, int rows, const float* table, int div, int mod, void* y, int ldy,
                      void* stream);
/* bf16 token rows ((b*F + f)*HW + p, C) -> fp32 (B, C, F, HW): the 5-D output layout of
 * TemporalTransformer.forward (temporal_transformer.py:142-144) and UNetMotionModel.forward. */
int vst_unpack_tokens(const void* src, int B, int C, int F, int HW, float* out, void* stream);

/* Denoise-loop glue (inference_animatediff.py:104-131). */
int vst_timestep_embedding(const float* t, const int* step_idx, int n, int dim, int flip_sin_to_cos,
                           float downscale_freq_shift, void* out, int ld, int col0, int per_row, void* stream);
int vst_pack_latents(const float* lat, int B, int Cl, int F, int HW, const float* sigmas, const int* step_idx,
                     float fixed_scale, int ncopy, void* out, void* stream);
int vst_euler_cfg_step(const void* noise, int ncopy, float guidance, float* lat, int B, int Cl, int F, int HW,
                       const float* sigmas, const int* step_idx, void* stream);
int vst_step_advance(int* step_idx, int num_steps, void* stream);  // wraps to 0 at num_steps
int vst_silu(const void* x, void* y, size_t n, void* stream);
int vst_add(const void* a, const void* b, void* y, size_t n, void* stream);
int vst_copy2d(const void* x, int ldx, void* y, int ldy, int rows, int cols, void* stream);
/* bf16 transpose y[c][r] = x[r][c] (x: rows x cols, row stride ldx; y: cols x rows, row stride ldy).  Backward-pass
 * operand layout for dW = dY^T X and the temporal-LoRA factor gradients (no reference counterpart: torch.autograd
 * of train_animatediff.py:265-319 does it implicitly). */
int vst_transpose(const void* x, int ldx, int rows, int cols, void* y, int ldy, void* stream);

/* Training path (torch.autograd of train_animatediff.py:265-319 in the reference).
 * vst_layernorm_bwd: dx and (dgamma, dbeta) of BasicTransformerBlock LayerNorm (x, g = dL/dy: rows x C bf16), stats
 * recomputed; workspace of vst_layernorm_bwd_workspace_bytes(C, rows); dgamma = dbeta = NULL (frozen affine):
 * dx only, no workspace.  vst_geglu_bwd: dp of the GEGLU projection output p (32-interleaved [h | gate] blocks,
 * as the fused GEMM stores them) from g = dL/d(h * gelu(gate)) (M x Nh). */
size_t vst_layernorm_bwd_workspace_bytes(int C, int rows);
int vst_layernorm_bwd(const void* x, int ldx, const void* g, int ldg, int C, int rows, const float* gamma, float eps,
                      void* dx, int lddx, float* dgamma, float* dbeta, void* workspace, void* stream);
/* vst_groupnorm_bwd: dx, dgamma, dbeta of vst_groupnorm (single source, optional fused SiLU; statistics and the
 * affine recomputed); workspace of vst_groupnorm_bwd_workspace_bytes. */
size_t vst_groupnorm_bwd_workspace_bytes(int nsamples, int rows_per_sample, int groups, int C);
int vst_groupnorm_bwd(const void* x, int ldx, const void* g, int ldg, int C, int nsamples, int rows_per_sample,
                      int groups, float eps, const float* gamma, const float* beta, int silu_act, void* dx, int lddx,
                      float* dgamma, float* dbeta, void* workspace, void* stream);
/* vst_spatial_attention_bwd: gradients of vst_spatial_attention (head_dim 64; K/V shared by kv_div consecutive
 * batches, as for the per-clip text states) from dO, the forward output o and the forward's lse output (flash-
 * attention backward on MFMA, deterministic): dq (lddq), dk/dv (lddkv, one row per kv token: the gradient of text
 * K/V summed over the frames sharing it; both NULL when K/V are frozen, which skips that pass).  Replaces the
 * autograd backward of F.scaled_dot_product_attention (animatediff/attention_processor.py:78-80) that
 * accelerator.backward runs (train_animatediff.py:314).  Workspace: vst_spatial_attention_bwd_workspace_bytes. */
size_t vst_spatial_attention_bwd_workspace_bytes(int nbatch, int heads, int Nq, int Nk);
int vst_spatial_attention_bwd(const void* q, int ldq, const void* k, const void* v, int ldkv, const void* o, int ldo,
                              const void* dout, int lddo, const float* lse, void* dq, int lddq, void* dk, void* dv,
                              int lddkv, int nbatch, int heads, int Nq, int Nk, int kv_div, int head_dim, float scale,
                              void* workspace, void* stream);
/* Sampler data gradients (NHWC tokens, C % 8 == 0): vst_zero_insert writes x [nimg, h, w, C] onto the even
 * positions of a caller-zeroed [nimg, 2h, 2w, C] (Downsample2D stride-2 conv dgrad); vst_sumpool2x2 sums 2x2 blocks
 * of x [nimg, 2h, 2w, C] into y [nimg, h, w, C] (adjoint of Upsample2D's nearest-2x). */
int vst_zero_insert(const void* x, int nimg, int h, int w, int C, void* y, void* stream);
int vst_sumpool2x2(const void* x, int nimg, int h, int w, int C, void* y, void* stream);
/* vst_temporal_attention_bwd: gradients of vst_temporal_attention (same token layout and q/k/v views) from dO; dq/dk/dv
 * are written with row stride lddqkv (e.g. column views of one [tokens, 3C] buffer).  F <= 32, head_dim one of
 * 8/16/32/40/64/80/160 (the forward's set; SDXL motion modules: 40/80/160), MFMA tiles as the forward. */
int vst_temporal_attention_bwd(const void* q, const void* k, const void* v, int ldqkv, const void* dout, int lddo,
                               void* dq, void* dk, void* dv, int lddqkv, int nclip, int F, int HW, int heads,
                               int head_dim, float scale, void* stream);
int vst_geglu_bwd(const void* p, int ldp, const void* g, int ldg, int M, int Nh, void* dp, int lddp, void* stream);
/* vst_colsum: y[N] (fp32) = column sums of the bf16 [M, N] view x (the bias gradients db = g^T 1 of the trainable
 * linears / GEGLU projections; torch's g.float().sum(0) in autograd's Linear backward), N % 8 == 0.  Deterministic
 * two-pass reduction through a workspace of vst_colsum_workspace_bytes(M, N) bytes (no atomics, no memset). */
size_t vst_colsum_workspace_bytes(int M, int N);
int vst_colsum(const void* x, int ldx, int M, int N, float* y, void* workspace, void* stream);

/* ---- SDXL VAE (diffusers AutoencoderKL, fp32 in the reference: inference_animatediff.py:164-169) decode of the
 * denoised clip (inference_animatediff.py:137-144) and encode of training frames (train_animatediff.py:219-224),
 * SURVEY §8(f) rank 4.  Convs, GroupNorm(+SiLU) and the 1x1 projections reuse the entries above. */
/* vst_conv3x3_down_pad0: diffusers Downsample2D(padding=0) of DownEncoderBlock2D = F.pad(x, (0,1,0,1)) then a 3x3
 * stride-2 conv without padding.  Output [nimg, (H-2)/2+1, (W-2)/2+1, Cout], row stride ldc. */
int vst_conv3x3_down_pad0(const void* x, int C, int nimg, int H, int W, const void* Wt, int Cout, const float* bias,
                          void* out, int ldc, void* workspace, size_t ws_bytes, void* stream);
/* C[N][K] (bf16, row stride ldc) = A^T B with A [M][N] and B [M][K] row-major over M tokens: the training step's
 * weight gradients (dW = g^T x, dA = s v^T x, dB = s g^T u; autograd.py, the backward of train_animatediff.py:265-319)
 * without transposed copies of either operand.  fp32 accumulation; the token range splits over workgroups and the
 * fp32 partials (workspace of vst_gemm_tn_workspace_bytes, may be 0) are summed in a fixed order.  N, K, lda, ldb
 * multiples of 8. */
size_t vst_gemm_tn_workspace_bytes(int M, int N, int K);
int vst_gemm_tn(const void* A, int lda, const void* B, int ldb, int M, int N, int K, void* C, int ldc,
                void* workspace, size_t ws_bytes, void* stream);
/* vst_gemm_f32out: C[M][N] = A[M][K] . W[N][K]^T left in fp32 (row stride N).  The mid-block attention's scores
 * (one head of dim 512 over the latent's h*w tokens) feed vst_softmax_rows unrounded, as the fp32 reference's do. */
int vst_gemm_f32out(const void* A, int lda, const void* W, int ldw, int M, int N, int K, float* C, void* stream);
/* vst_softmax_rows: P[r][j] = softmax_j(scale * S[r][j]) (fp32 math, bf16 out) -- diffusers Attention.get_attention_scores
 * + softmax of the VAE mid-block (AttnProcessor2_0's SDPA math, scale = head_dim^-0.5). */
int vst_softmax_rows(const float* S, int lds, int rows, int n, float scale, void* P, int ldp, void* stream);
/* Layout at the fp32 NCHW tensor boundary of vae.decode / vae.encode:
 * vst_nchw_to_nhwc: dst[(i*HW+p)*ldd + c] = bf16(src[(i*C+c)*HW+p] * mul), channels C..ldd-1 zero-filled
 *   (decode input: latents / scaling_factor, inference_animatediff.py:137; encode input: frames in [-1, 1]);
 * vst_nhwc_to_nchw: bf16 NHWC (row stride ld) -> fp32 NCHW (DecoderOutput.sample);
 * vst_frames_to_u8: (x / 2 + 0.5).clamp(0, 1) * 255 truncated to uint8, HWC per frame (inference_animatediff.py:141-143);
 * vst_vae_sample: DiagonalGaussianDistribution(moments).sample() * mul (train_animatediff.py:222-223): moments NHWC
 *   [n*HW][ld] bf16 (mean = ch 0-3, logvar = ch 4-7 clamped to [-30, 20]), eps fp32 NCHW (null: the mode), out fp32
 *   NCHW (n, 4, HW). */
int vst_nchw_to_nhwc(const float* src, int n, int C, int HW, float mul, void* dst, int ldd, void* stream);
int vst_nhwc_to_nchw(const void* src, int ld, int n, int C, int HW, float* dst, void* stream);
int vst_frames_to_u8(const void* src, int ld, int n, int C, int HW, void* dst, void* stream);
int vst_vae_sample(const void* moments, int ld, int n, int HW, const float* eps, float mul, float* out, void* stream);

/* Ceiling probes (no reference counterpart; bench.py's measured peaks next to the vendor figures,
 * SURVEY §8(d)).  vst_probe_mfma: `grid` workgroups x 8 waves, each wave `iters` x 16 independent
 * 16x16x32 bf16 MFMAs (flops = grid*8*iters*16*16384).  vst_probe_hbm_read: streams `bytes` of `src`
 * with 16-B loads.  `out` receives nothing in practice (anti-dead-code sink, >= grid elements). */
int vst_probe_mfma(int grid, int iters, float* out, void* stream);
int vst_probe_hbm_read(const void* src, size_t bytes, int grid, unsigned* out, void* stream);
/* vst_probe_fetch: the per-CU operand fetch rate from an L2-resident `bytes` region (the GEMM loaders' path): `grid`
 * 512-thread workgroups, each wave moving `iters` 1-KiB pieces, 8 in flight; mode 0 buffer loads into VGPRs, 1 LDS-DMA
 * into an LDS ring (the 8-phase GEMM's loader), 2 buffer loads + ds_write_b128 (a register-staged loader). */
int vst_probe_fetch(int mode, const void* src, int bytes, int grid, int iters, unsigned* out, void* stream);
/* vst_probe_mix: what a loader costs an MFMA stream: `grid` 512-thread workgroups, each wave iterating {issue `pieces`
 * (0, 2, 4, 8) one-KiB pieces, 32 register-operand 16x16x32 bf16 MFMAs, land the pieces}; mode 1 LDS-DMA, 2 buffer
 * loads + ds_write_b128.  Time against pieces = 0 is the loader's cost to the matrix core. */
int vst_probe_mix(int mode, int pieces, const void* src, int bytes, int grid, int iters, float* out, void* stream);
const char* vst_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VST_H */
