/*
 * red_diffeq_unet.h — C ABI of the U-Net epsilon-predictor kernels (libred_diffeq_hip.so).
 *
 * Replaces the PyTorch/cuDNN arithmetic of the reference U-Net forward
 * (SimingShan/red-diffeq red_diffeq/models/diffusion.py:78-301) and the RED regulariser's
 * elementwise prologue/epilogue (diffusion.py:393-429, 516-519;
 * red_diffeq/regularization/diffusion.py:63-81).  fp32 NCHW tensors, caller-owned, stream-ordered,
 * 0 / negative error codes, deterministic (no floating-point atomics: the conv's arrival tickets
 * only pick which workgroup sums the split-K slabs, always in slab order).
 */
#ifndef RED_DIFFEQ_UNET_H
#define RED_DIFFEQ_UNET_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Logical conv input = the (B, cin1 + cin2, H, W) tensor formed from x (and x2) by `in_mode`:
 *   0 RDQ_IN_PLAIN      x (B,cin1,H,W) ++ x2 (B,cin2,H,W) along channels (torch.cat, diffusion.py:293-299)
 *   1 RDQ_IN_UPSAMPLE2  x (B,cin1,H/2,W/2) nearest-upsampled x2 (nn.Upsample, diffusion.py:79)
 *   2 RDQ_IN_UNSHUFFLE2 x (B,cin1/4,2H,2W), channel c*4+p1*2+p2 <- x[c][2h+p1][2w+p2]
 *                       (einops 'b c (h p1) (w p2) -> b (c p1 p2) h w', diffusion.py:82)        */
#define RDQ_IN_PLAIN 0
#define RDQ_IN_UPSAMPLE2 1
#define RDQ_IN_UNSHUFFLE2 2

typedef struct rdq_conv_desc {
    int32_t B, cin1, cin2, H, W, cout, kh, kw, pad, in_mode;
} rdq_conv_desc;

/* y = conv2d(input, w, bias, stride 1, padding pad) [+ residual]   (nn.Conv2d, implicit GEMM on
 * fp32 MFMA v_mfma_f32_16x16x4_f32).  w: [cout][cin1+cin2][kh][kw]; bias/residual nullable.
 * ws (nullable) holds split-K partial slabs: rdq_conv2d_ws_bytes(d) bytes let the kernel split the
 * reduction over enough workgroups to fill the chip; a smaller (or null) ws splits less (or not).
 * tickets (nullable): rdq_conv2d_tickets(d) uint32 words that are ZERO when the call is enqueued;
 * the launch leaves them zero again, so one zeroed pool serves every stream-ordered call (two
 * launches must not use the same words concurrently).  With tickets the split-K slabs are combined
 * inside the conv launch by the last-arriving workgroup of each output tile; without, by a second
 * launch.  Both sum the slabs in slab order (deterministic, identical results). */
size_t rdq_conv2d_ws_bytes(const rdq_conv_desc *d);
size_t rdq_conv2d_tickets(const rdq_conv_desc *d);
int rdq_conv2d(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
               const float *residual, float *y, void *ws, size_t ws_bytes, uint32_t *tickets, hipStream_t stream);

/* y = conv2d(RMSNorm(x)) [+ bias] [+ residual] for a 1x1 conv (LinearAttention / Attention to_qkv,
 * diffusion.py:184-186, 211-213): F.normalize(x, dim=1) * g * sqrt(C) formed as the conv gathers its
 * operand (per-pixel norms from one pass over the input channels).  1x1, pad 0, no concat, C <= 2048,
 * channel counts multiples of 64; ws / tickets as rdq_conv2d (rdq_conv2d_ws_bytes). */
int rdq_conv2d_rms(const rdq_conv_desc *d, const float *x, const float *g, const float *w, const float *bias,
                   const float *residual, float *y, void *ws, size_t ws_bytes, uint32_t *tickets, hipStream_t stream);

/* Block.forward in two launches (diffusion.py:142-149, + the identity shortcut of 168):
 *   y = SiLU(GroupNorm_G(conv2d(input) + bias) * (scale+1) + shift) [+ post_residual]
 * The conv (channel-chunk form) accumulates the GroupNorm statistics of its output tiles in its
 * epilogue (fp64 per tile, group and sample; summed in tile order by the normalise pass), replacing
 * rdq_conv2d + rdq_group_norm_silu's statistics launch (+ a residual add).  rdq_conv2d_gn_ws_bytes
 * returns 0 where this form does not apply (filters other than 3x3 / 1x1-pad-0, channel counts
 * not multiples of the chunk, H*W < 32, C/G outside {8,16,32,64}): use the separate calls there.
 * ws: conv split-K slabs + the conv output + the partial statistics.  tickets as rdq_conv2d (null:
 * no split-K). */
size_t rdq_conv2d_gn_ws_bytes(const rdq_conv_desc *d, int32_t G);
int rdq_conv2d_gn_silu(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                       int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                       const float *post_residual, float *y, void *ws, size_t ws_bytes, uint32_t *tickets,
                       hipStream_t stream);

/* ResnetBlock with a 1x1 shortcut (diffusion.py:160-168, the U-Net's up path and final block):
 *   y   = SiLU(GroupNorm_G(conv3x3(cat(x, x2)) + bias) * (scale+1) + shift)   (block1, as rdq_conv2d_gn_silu)
 *   y_s = conv1x1(cat(x, x2), w_s) + b_s                                      (res_conv, as rdq_conv2d)
 * in two launches instead of three: both convs of the same input run in ONE launch (disjoint tile
 * ranges), then the normalise pass.  Results are bit for bit those of the separate calls.  Applies
 * where rdq_conv2d_gn_sc_ws_bytes > 0 (d: the 3x3 conv, plain input mode; the 1x1 in the
 * channel-chunk form).  w_s [cout_s][cin1+cin2]; b_s nullable; tickets: rdq_conv2d_gn_sc_tickets
 * zeroed words (nullable: no split-K). */
size_t rdq_conv2d_gn_sc_ws_bytes(const rdq_conv_desc *d, int32_t G, int32_t cout_s);
size_t rdq_conv2d_gn_sc_tickets(const rdq_conv_desc *d, int32_t cout_s);
int rdq_conv2d_gn_silu_sc(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                          int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                          float *y, int32_t cout_s, const float *w_s, const float *b_s, float *y_s, void *ws,
                          size_t ws_bytes, uint32_t *tickets, hipStream_t stream);

/* The first ResnetBlock's block1 (as rdq_conv2d_gn_silu, plain input mode) with every ResnetBlock's
 * Linear(SiLU(t)) (as rdq_linear_silu_multi: n <= 32 linears of the (B, in) time embedding temb,
 * ly[j] (B, lout[j])) computed as a side job of the conv launch (Unet.forward, diffusion.py:280-283
 * with 160-165).  ss_index >= 0: ly[ss_index] is this block's scale_shift (lout = 2 cout); -1: none.
 * ws / tickets as rdq_conv2d_gn_silu. */
int rdq_conv2d_gn_silu_lsm(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                           int32_t G, float eps, const float *gamma, const float *beta, const float *post_residual,
                           float *y, void *ws, size_t ws_bytes, uint32_t *tickets, int32_t in, const float *temb,
                           int32_t n, const float *const *lw, const float *const *lb, const int32_t *lout,
                           float *const *ly, int32_t ss_index, hipStream_t stream);

/* The U-Net's tail (diffusion.py:299-301): yf = conv1x1(Block(x) [+ post_residual], wf) + bf with
 * Block = rdq_conv2d_gn_silu's SiLU(GroupNorm(conv(x)) * (scale+1) + shift) — final_res_block's block2
 * and final_conv — in two launches, the cout-channel block output never written.  nf <= 4 output
 * channels, wf [nf][cout], bf nullable, yf [B][nf][H][W]; cout % 4 == 0; ws / tickets as
 * rdq_conv2d_gn_silu. */
int rdq_conv2d_gn_silu_out(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                           int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                           const float *post_residual, int32_t nf, const float *wf, const float *bf, float *yf,
                           void *ws, size_t ws_bytes, uint32_t *tickets, hipStream_t stream);

/* The U-Net's first launch (diffusion.py:276-279): y = init_conv(x) (as rdq_conv2d: a conv NOT in the
 * channel-chunk form, 7x7 or 3x3, cout <= 64, no K split) and temb = Unet.time_mlp(t) (as
 * rdq_time_mlp) in ONE launch.  RDQ_E_INVALID when the shapes do not allow it. */
int rdq_unet_head(const rdq_conv_desc *d, const float *x, const float *w, const float *bias, float *y, int32_t dim,
                  float theta, const int64_t *t, const float *w1, const float *b1, int32_t hid, const float *w2,
                  const float *b2, int32_t out, float *temb, hipStream_t stream);

/* Unet.init_conv (Conv2d(1, 64, 7, padding=3), fp32) as a direct conv: one thread per output pixel and
 * all 64 channels (the batched bf16 U-Net's stem; the fp32 reference path keeps rdq_conv2d / the fused
 * head).  d: cin1 = 1, cin2 = 0, 7 x 7, pad 3, cout 64, plain mode, 64 <= W <= 72; RDQ_E_INVALID otherwise. */
int rdq_conv2d_stem(const rdq_conv_desc *d, const float *x, const float *w, const float *bias, float *y,
                    hipStream_t stream);

/* Mixed-precision conv2d (same input modes and epilogue): bf16 operands, fp32 accumulation on
 * v_mfma_f32_32x32x16_bf16.  The weights are packed once by rdq_conv2d_bf16_pack into
 * wp[cout][kh*kw][cinp] bf16 (round-to-nearest-even, cinp = cin1+cin2 rounded up to 32, zero-padded;
 * rdq_conv2d_bf16_wpack_bytes bytes); activations are rounded to bf16 as they are staged.
 * New behaviour for configs[4] (no reference counterpart; the reference U-Net runs in fp32). */
size_t rdq_conv2d_bf16_wpack_bytes(const rdq_conv_desc *d);
int rdq_conv2d_bf16_pack(const rdq_conv_desc *d, const float *w, void *wp, hipStream_t stream);
size_t rdq_conv2d_bf16_ws_bytes(const rdq_conv_desc *d);
/* Process-wide U-Net kernel options (test / A-B switches).  They choose kernels, and with them the
 * fp32 summation order, for every later call in the process: the values are atomics (never torn), but
 * a change does not reach hipGraphs captured before it, so every change bumps the counter returned by
 * rdq_unet_options_generation (the Python U-Net keys its captured graphs on it and recaptures).
 *   RDQ_UNET_OPT_BF16_PER_TAP = 1: rdq_conv2d_bf16 always runs the per-tap kernel instead of the
 *   halo-staged 3x3 kernel (the two share the operand rounding; tests/test_gpu_unet.py compares them).
 * Returns the previous value, or RDQ_E_INVALID for an unknown option or value. */
#define RDQ_UNET_OPT_BF16_PER_TAP 1
#define RDQ_UNET_OPT_CONV3_MIN_TILES 2   /* least (256-pixel x 64-channel) tiles for the halo-staged 3x3 conv (default 64) */
#define RDQ_UNET_OPT_BF16_RAW 3   /* rdq_conv2d_bf16_gn_*: hold the raw conv output as bf16 (default 1) */
#define RDQ_UNET_OPT_CONV3F_MIN_TILES 4   /* least tiles for the fp32 halo-staged 3x3 conv (0: never; default 192) */
#define RDQ_UNET_OPT_CC_MIN_STAGES 6   /* channel-chunk convs: least K stages per split-K piece (default 3) */
#define RDQ_UNET_OPT_CC_SPLIT2_STAGES 7   /* grids of 128..255 tiles split K in two from this many stages (default 12) */
int rdq_unet_set_option(int32_t option, int32_t value);
int rdq_unet_options_generation(void);
int rdq_conv2d_bf16(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp, const float *bias,
                    const float *residual, float *y, void *ws, size_t ws_bytes, hipStream_t stream);

/* Block.forward in two launches on the bf16 halo-staged conv (the batched, mixed-precision U-Net of
 * configs[4]): y = SiLU(GroupNorm_G(h) * (scale+1) + shift) [+ post_residual], h = bf16(conv3x3_bf16(input)
 * + bias): the raw conv output is held as bf16 between the two launches (half the bytes written and
 * re-read), and the GroupNorm statistics of h are reduced in the conv's epilogue (fp64, fixed trees)
 * instead of a separate statistics pass.  rdq_conv2d_bf16_gn_ws_bytes returns 0 where this form does not
 * apply (not the halo-staged conv: see rdq_conv2d_bf16; H*W < 256; C/G outside {8,16,32,64}).
 * wp: rdq_conv2d_bf16_pack's weights; ws: the conv output + the partial statistics. */
size_t rdq_conv2d_bf16_gn_ws_bytes(const rdq_conv_desc *d, int32_t G);
int rdq_conv2d_bf16_gn_silu(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp, const float *bias,
                            int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                            const float *post_residual, float *y, void *ws, size_t ws_bytes, hipStream_t stream);
/* The same Block for a ResnetBlock's block1, whose output feeds only block2's conv (diffusion.py:166-167):
 * y8 = bf16(SiLU(GroupNorm(conv3x3(cat(x, x2)))...)) stored as channel octets [B][cout / 8][H*W][8]
 * (cout % 8 == 0) -- the rounding block2's bf16 conv applies to its operands anyway, so the pair is
 * bit-identical to rdq_conv2d_bf16_gn_silu twice; ws: rdq_conv2d_bf16_gn_ws_bytes. */
int rdq_conv2d_bf16_gn_silu8(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp,
                             const float *bias, int32_t G, float eps, const float *gamma, const float *beta,
                             const float *scale_shift, void *y8, void *ws, size_t ws_bytes, hipStream_t stream);
/* block2 of that pair: rdq_conv2d_bf16_gn_silu on the octet input x8 (d: plain mode, cin2 = 0,
 * cin1 % 32 == 0). */
int rdq_conv2d_bf16_gn_silu_x8(const rdq_conv_desc *d, const void *x8, const void *wp, const float *bias, int32_t G,
                               float eps, const float *gamma, const float *beta, const float *scale_shift,
                               const float *post_residual, float *y, void *ws, size_t ws_bytes, hipStream_t stream);

/* rdq_conv2d_gn_silu_out's tail (final_res_block's block2 + final_conv, diffusion.py:299-301) on the bf16
 * halo-staged conv: yf = conv1x1(Block_bf16(x) [+ post_residual], wf) + bf; ws: rdq_conv2d_bf16_gn_ws_bytes. */
int rdq_conv2d_bf16_gn_silu_out(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp,
                                const float *bias, int32_t G, float eps, const float *gamma, const float *beta,
                                const float *scale_shift, const float *post_residual, int32_t nf, const float *wf,
                                const float *bf, float *yf, void *ws, size_t ws_bytes, hipStream_t stream);

/* GroupNorm(G) -> [x*(scale+1)+shift] -> SiLU  (Block.forward, diffusion.py:142-149).
 * scale_shift: nullable [B][2C] (first C = scale, next C = shift); ws: rdq_group_norm_ws_bytes (fp64
 * chunk partials of sum / sum of squares, then the per-(sample, group) mean and 1/std). */
size_t rdq_group_norm_ws_bytes(int32_t B, int32_t C, int32_t HW, int32_t G);
int rdq_group_norm_silu(int32_t B, int32_t C, int32_t HW, int32_t G, float eps, const float *x, const float *gamma,
                        const float *beta, const float *scale_shift, float *y, void *ws, hipStream_t stream);

/* RMSNorm: F.normalize(x, dim=1) * g * sqrt(C) [+ residual]  (diffusion.py:84-91). */
int rdq_rmsnorm(int32_t B, int32_t C, int32_t HW, const float *x, const float *g, const float *residual, float *y,
                hipStream_t stream);

/* y[b][o] = act_out( W[o] . act_in(x[b]) + bias[o] ); act_in: 0 none / 1 SiLU, act_out: 0 none / 1 GELU(erf). */
int rdq_linear(int32_t B, int32_t in, int32_t out, const float *x, const float *w, const float *bias,
               int32_t act_in, int32_t act_out, float *y, hipStream_t stream);

/* Unet.time_mlp in one launch (diffusion.py:255-258): y = W2 GELU(W1 SinusoidalPosEmb(t) + b1) + b2,
 * w1 [hid][dim], w2 [out][hid]; one workgroup per sample. */
int rdq_time_mlp(int32_t B, int32_t dim, float theta, const int64_t *t, const float *w1, const float *b1, int32_t hid,
                 const float *w2, const float *b2, int32_t out, float *y, hipStream_t stream);

/* n <= 32 linears sharing one input, in one launch: y_j[b] = W_j . SiLU(x[b]) + b_j  (every
 * ResnetBlock's time MLP, diffusion.py:157-165); w_j [out_j][in], y_j [B][out_j], b nullable. */
int rdq_linear_silu_multi(int32_t B, int32_t in, const float *x, int32_t n, const float *const *w,
                          const float *const *b, const int32_t *out, float *const *y, hipStream_t stream);

/* SinusoidalPosEmb (diffusion.py:93-107): y[b] = [sin(t_b f), cos(t_b f)], f_i = exp(-i ln(theta)/(half-1)). */
int rdq_sinusoidal_emb(int32_t B, int32_t dim, float theta, const int64_t *t, float *y, hipStream_t stream);

/* LinearAttention core (diffusion.py:182-194; dh <= 32), qkv = to_qkv(RMSNorm(x)) as (B, 3*heads*dh, n);
 * mem_kv (2, heads, dh, nmem); out (B, heads*dh, n) before to_out.  ws: rdq_linear_attention_ws_bytes
 * (per-256-token k row maxima / exp sums and partial contexts, combined in chunk order with the
 * softmax rescaling exp(m_chunk - m), + the combined context).  dh = 32 forms each partial context
 * on v_mfma_f32_32x32x2_f32. */
size_t rdq_linear_attention_ws_bytes(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem);
int rdq_linear_attention(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, float scale, const float *qkv,
                         const float *mem_kv, float *out, void *ws, hipStream_t stream);

/* LinearAttention.forward + residual in three launches (diffusion.py:182-195 with to_out =
 * Conv2d(heads*dh, dim, 1) + RMSNorm(dim), residual 286/297): the partial contexts, then ONE launch for
 * the chunk combine (in that launch when the image has <= 8 chunks of 256 tokens, else its own
 * launch), softmax(q) x context, the 1x1 to_out conv (+ b_out), RMSNorm(g_out) and + res.
 * dh = 32, heads = 4 (the U-Net's), dim in {64, 128, 256}; w_out [dim][heads*dh]; b_out, res nullable;
 * y (B, dim, n); ws: rdq_linear_attention_ws_bytes.  Replaces rdq_linear_attention + rdq_conv2d +
 * rdq_rmsnorm for the U-Net's linear-attention blocks. */
int rdq_linear_attention_block(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, float scale,
                               const float *qkv, const float *mem_kv, int32_t dim, const float *w_out,
                               const float *b_out, const float *g_out, const float *res, float *y, void *ws,
                               hipStream_t stream);

/* LinearAttention.forward(x) + x with bf16 operands and fp32 accumulation (the configs[4] batched U-Net;
 * reference diffusion.py:182-195 and the residual at 286 / 297): RMSNorm(x) (g_in), qkv = to_qkv,
 * softmax(q) over d, softmax(k) over the memory + pixel tokens, context, to_out conv (+ b_out) and
 * RMSNorm (g_out), + x, in two launches that never materialise qkv or the hidden tensor.
 * heads = 4, dim_head = 32; dim 64 / 128; x, y (B, dim, n) fp32, y != x; mem_kv (2, 4, 32, nmem);
 * wqkv / wout: rdq_conv2d_bf16_pack's packs of the (384, dim, 1, 1) / (dim, 128, 1, 1) weights;
 * ws: rdq_linear_attention_bf16_ws_bytes (per chunk partial contexts). */
size_t rdq_linear_attention_bf16_ws_bytes(int32_t B, int32_t dim, int32_t n);
int rdq_linear_attention_bf16(int32_t B, int32_t dim, int32_t n, int32_t nmem, float scale, const float *x,
                              const float *g_in, const void *wqkv, const float *mem_kv, const void *wout,
                              const float *b_out, const float *g_out, float *y, void *ws, size_t ws_bytes,
                              hipStream_t stream);
/* The same two-launch LinearAttention block in fp32 (the reference's arithmetic: v_mfma_f32_32x32x2_f32,
 * fp32 staging): wqkv / wout are the module's own fp32 weights (384, dim) / (dim, 128); dim 64 / 128;
 * ws: rdq_linear_attention_f32_ws_bytes. */
size_t rdq_linear_attention_f32_ws_bytes(int32_t B, int32_t dim, int32_t n);
int rdq_linear_attention_f32(int32_t B, int32_t dim, int32_t n, int32_t nmem, float scale, const float *x,
                             const float *g_in, const float *wqkv, const float *mem_kv, const float *wout,
                             const float *b_out, const float *g_out, float *y, void *ws, size_t ws_bytes,
                             hipStream_t stream);

/* Attention core with Attend(flash=False) (diffusion.py:209-217): softmax(q k^T dh^-1/2) v over
 * nmem memory keys + n pixels; mem_kv (2, heads, nmem, dh); out (B, heads*dh, n).  dh = 32; K/V of one
 * head staged in LDS (n + nmem <= ~1500). */
int rdq_full_attention(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, const float *qkv,
                       const float *mem_kv, float *out, hipStream_t stream);

/* RED prologue: x_t = sqrt(abar_t) x0 + sqrt(1-abar_t) eps  (q_sample, diffusion.py:516-519);
 * tables are the fp32 schedule buffers, t int64 [B], n elements per sample. */
int rdq_red_q_sample(int32_t B, int64_t n, const float *sqrt_ac, const float *sqrt_1mac, const int64_t *t,
                     const float *x0, const float *eps, float *xt, hipStream_t stream);
/* The same, also copying t to t_out [B] in the launch: x_t and t written straight into the static input
 * buffers of a captured U-Net forward (Unet.graph_io), so the replay needs no input copies. */
int rdq_red_q_sample_t(int32_t B, int64_t n, const float *sqrt_ac, const float *sqrt_1mac, const int64_t *t,
                       const float *x0, const float *eps, float *xt, int64_t *t_out, hipStream_t stream);
/* RED epilogue (pred_noise objective, clip_x_start + rederive_pred_noise, diffusion.py:393-419):
 *   x0_hat = clamp(sr[t] x_t - srm1[t] eps_hat, -1, 1);  eps' = (sr[t] x_t - x0_hat) / srm1[t];
 *   g = eps' - eps   (regularization/diffusion.py:74). */
int rdq_red_epilogue(int32_t B, int64_t n, const float *sqrt_recip_ac, const float *sqrt_recipm1_ac,
                     const int64_t *t, const float *xt, const float *eps_hat, const float *eps, float *g,
                     hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RED_DIFFEQ_UNET_H */
