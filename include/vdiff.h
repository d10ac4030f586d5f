/*
 * vdiff.h -- C-ABI of libvdiff.so, the MI355X (gfx950) kernels behind the
 * video-diffusion denoiser hot path of wdas03/lipreading-video-generation.
 *
 * The reference has no FFI: its boundary is the Python module API of
 * video-generation/diffusion (unet.py, unet_audio.py, utils.py,
 * linear_noise_scheduler.py, noise_scheduler.py).  Every entry point below
 * replaces the ATen op(s) that the reference calls at the cited line; the
 * Python drop-in (lipreading-video-generation_amd/video-generation/diffusion)
 * binds them through ctypes.
 *
 * Conventions
 *  - All tensor arguments are caller-owned DEVICE pointers.  The library never
 *    allocates device memory; kernels that need scratch take a workspace
 *    pointer whose size is returned by the matching *_workspace_size().
 *  - Activations are channels-last: a [B, C, T, H, W] tensor is stored as
 *    [B][T][H][W][C] (C fastest).  2-D tensors use T = 1.
 *  - `stream` is a hipStream_t passed as void* (0 = null stream).  Every call
 *    is asynchronous and stream-ordered; nothing synchronises the host.
 *  - Return 0 on success, otherwise a VD_E* code; vd_last_error() returns a
 *    thread-local message describing the last failure.
 *  - dtype: VD_F32 (parity mode, fp32 storage, exact-fp32 MFMA / VALU math) or
 *    VD_BF16 (throughput mode, bf16 storage, fp32 accumulate/statistics).
 */
#ifndef VDIFF_H
#define VDIFF_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VDIFF_ABI_VERSION 1

enum vd_status { VD_OK = 0, VD_EINVAL = 1, VD_EUNSUPPORTED = 2, VD_ELAUNCH = 3 };
enum vd_dtype { VD_F32 = 0, VD_BF16 = 1 };

/* ---- library ---------------------------------------------------------- */
int vd_version(void);
const char* vd_last_error(void);
/* Writes "name;gfx;CUs;HBM bytes" of the current device into buf. */
int vd_device_info(char* buf, int buflen);

/* ---- timestep embedding ------------------------------------------------
 * replaces utils.py:140-158 (timestep_embedding): out[b, i] =
 * cos(t_b * f_i) (i < dim/2), sin(t_b * f_{i-dim/2}) (i >= dim/2),
 * f_i = exp(-ln(max_period) * i / (dim/2)); zero column when dim is odd.
 * t: int64[B]; out: fp32[B, dim]. */
int vd_timestep_embedding(const int64_t* t, int B, int dim, float max_period,
                          float* out, void* stream);
/* Same, with the frequency table f[dim/2] (fp32, device) supplied by the caller -- the
 * reference computes it on the host (utils.py:150-152: torch CPU exp), so a caller that
 * builds it the same way gets the reference's bit-identical arguments t_b * f_i. */
int vd_timestep_embedding_tab(const int64_t* t, int B, int dim, const float* freqs,
                              float* out, void* stream);

/* ---- DDPM / DDIM scheduler math ----------------------------------------
 * Tables are fp32 device arrays of length num_timesteps; t is int64[B];
 * x tensors are [B][per_sample] in `dtype`.  z may be NULL where the
 * formula adds no noise.
 *
 * q_sample: linear_noise_scheduler.py:24-46 (add_noise)
 *   xt = sqrt_acp[t] * x0 + sqrt_1m_acp[t] * eps */
int vd_q_sample(const void* x0, const void* eps, void* xt, const int64_t* t,
                const float* sqrt_acp, const float* sqrt_1m_acp,
                int64_t B, int64_t per_sample, int dtype, void* stream);

/* ---- MSE loss (train.py:103 nn.MSELoss(), :130 loss = criterion(noise_pred, noise)) ----
 * out[0] = mean((pred - target)^2) over n elements of `dtype`, fp32, in a FIXED order:
 * per-block partial sums of fixed ranges into the caller's workspace
 * (vd_mse_loss_workspace_size(n) bytes), then one block sums them in block order.  Two
 * launches, no semaphore and no memset, so the value is identical eager and replayed from
 * a HIP graph.  pred / target 16-B aligned.
 * vd_mse_loss_bwd: grad_pred = 2 (pred - target) / n * grad_loss[0] (grad_loss: device fp32
 * scalar, the autograd seed; MSELoss.backward). */
size_t vd_mse_loss_workspace_size(int64_t n);
int vd_mse_loss(const void* pred, const void* target, int64_t n, int dtype, float* out,
                void* workspace, size_t workspace_bytes, void* stream);
int vd_mse_loss_bwd(const void* pred, const void* target, const float* grad_loss, int64_t n,
                    int dtype, void* grad_pred, void* stream);

/* p_sample V1: linear_noise_scheduler.py:48-76 (LinearNoiseScheduler.
 * sample_prev_timestep).  x0 = clamp((xt - s1m[t] eps) / sqrt(acp[t])),
 * mean = (xt - beta[t] eps / s1m[t]) / sqrt(alpha[t]); t == 0 returns mean,
 * else mean + sqrt((1-acp[t-1])/(1-acp[t]) * beta[t]) * z. */
int vd_p_sample_v1(const void* xt, const void* eps, const void* z,
                   void* x_prev, void* x0, const int64_t* t,
                   const float* betas, const float* alphas, const float* acp,
                   const float* sqrt_1m_acp, int64_t B, int64_t per_sample,
                   int dtype, void* stream);

/* p_sample V2: linear_noise_scheduler.py:91-101 (LinearNoiseSchedulerV2).
 * mean = xt - s1m[t] eps / sqrt(alpha[t]); sigma = sqrt((1-acp[t]) beta[t]);
 * x_prev = mean + sigma z (also at t == 0); x0 = clamp((xt - s1m[t] eps)/sa[t]). */
int vd_p_sample_v2(const void* xt, const void* eps, const void* z,
                   void* x_prev, void* x0, const int64_t* t,
                   const float* betas, const float* alphas, const float* acp,
                   const float* sqrt_acp, const float* sqrt_1m_acp,
                   int64_t B, int64_t per_sample, int dtype, void* stream);

/* p_sample cosine: noise_scheduler.py:13-29 (CosineNoiseScheduler).
 * mean = (xt - s1m[t] eps) / sa[t]; t > 0: x_prev = mean + sigma z with
 * sigma = sqrt(acp[t-1] (1-acp[t]) / (1-acp[t-1])); t == 0: x_prev = mean.
 * Second output is `mean` (the reference returns (sampled, mean)). */
int vd_p_sample_cosine(const void* xt, const void* eps, const void* z,
                       void* x_prev, void* mean_out, const int64_t* t,
                       const float* acp, const float* sqrt_acp,
                       const float* sqrt_1m_acp, int64_t B, int64_t per_sample,
                       int dtype, void* stream);

/* DDIM step (build extension, no reference oracle beyond the acp tables):
 * x0 = (xt - sqrt(1-a_t) eps)/sqrt(a_t) [clamped to [-1,1] if clip];
 * sigma = eta sqrt((1-a_p)/(1-a_t) (1 - a_t/a_p));
 * x_prev = sqrt(a_p) x0 + sqrt(1-a_p-sigma^2) eps + sigma z, a_p = acp[t_prev]
 * or 1 when t_prev < 0.  t, t_prev: int64[B]. */
int vd_ddim_step(const void* xt, const void* eps, const void* z, void* x_prev,
                 void* x0, const int64_t* t, const int64_t* t_prev,
                 const float* acp, float eta, int clip, int64_t B,
                 int64_t per_sample, int dtype, void* stream);

/* ---- GroupNorm (+SiLU) -------------------------------------------------
 * replaces GroupNorm32 (utils.py:54-56, fp32 statistics) followed by nn.SiLU
 * (unet.py:194-198, 218-225, 297, 624-628).  x, y: [B][S][C] channels-last,
 * S = T*H*W; gamma/beta fp32[C]; mean/rstd fp32[B*G] (saved for backward).
 * (The ResBlock emb-add that precedes out_layers' GN is fused into the
 * producing conv's epilogue via vd_conv3d_fwd's chan_add.) */
/* drop_p > 0 also fuses the train-mode nn.Dropout that follows the SiLU in
 * ResBlock.out_layers (unet.py:218-225): element i is kept with probability
 * 1 - drop_p (scaled by 1/(1-drop_p)) by a counter-based hash of (seed, i);
 * the backward regenerates the same mask from the same seed. */
/* counter (device memory, or NULL = off): while set, every GroupNorm launch
 * with drop_p > 0 also takes this pointer and mixes the uint64 it reads at run
 * time into its seed.  A train step captured as a HIP graph (vdiff.engine.
 * Trainer(graph=True)) freezes the host seed in the launch arguments; bumping
 * the counter before each replay gives every step a fresh mask, the forward
 * and backward of one step the same one.  Host-side setting; no GPU call. */
void vd_set_dropout_counter(const uint64_t* counter);
/* Pixel rows whose loads each GroupNorm thread keeps in flight (1, 2 default, 4); the sums are
 * added in the same order for every value (bit-identical).  Process-wide A/B hook; returns the
 * previous value or -2.  No reference counterpart. */
int vd_groupnorm_set_unroll(int u);
size_t vd_groupnorm_workspace_size(int B, int64_t S, int C, int G);
int vd_groupnorm_silu_fwd(const void* x, const float* gamma, const float* beta,
                          void* y, float* mean, float* rstd, int B, int64_t S,
                          int C, int G, float eps, int silu, float drop_p,
                          uint64_t seed, int dtype, void* workspace,
                          void* stream);
/* dx = d/dx of dropout(silu(GN(x))); dgamma/dbeta are fp32[C], OVERWRITTEN. */
int vd_groupnorm_silu_bwd(const void* x, const void* dy, const float* gamma,
                          const float* beta, const float* mean,
                          const float* rstd, void* dx, float* dgamma,
                          float* dbeta, int B, int64_t S, int C, int G,
                          int silu, float drop_p, uint64_t seed, int dtype,
                          void* workspace, void* stream);
/* The same with dx += dadd (dadd in x's layout and dtype, or NULL): x's gradient from its
 * other consumer -- the residual branch of ResBlock (unet.py:268, skip_connection(x) + h) and
 * AttentionBlock (unet.py:317, x + h) -- added in fp32 before dx is rounded, instead of the
 * separate elementwise add autograd would run to accumulate the two gradients. */
int vd_groupnorm_silu_bwd_add(const void* x, const void* dy, const void* dadd,
                              const float* gamma, const float* beta, const float* mean,
                              const float* rstd, void* dx, float* dgamma, float* dbeta,
                              int B, int64_t S, int C, int G, int silu, float drop_p,
                              uint64_t seed, int dtype, void* workspace, void* stream);

/* ---- SiLU on flat tensors (time-embedding MLP, ResBlock.emb_layers:
 * unet.py:483-487, 211-217).  bwd: dx = dy * silu'(x). */
int vd_silu(const void* x, void* y, int64_t n, int dtype, void* stream);
int vd_silu_bwd(const void* x, const void* dy, void* dx, int64_t n, int dtype,
                void* stream);

/* ---- UNetAudio conditioning concat (unet_audio.py:52-61) -------------
 * out[b][t][y][x][:] = [ image[b][t][y][x][0:Cx] | imc[b][ys][xs][0:Ci] |
 *                        audio[b][t][0:Ca] | zeros up to out_cstride ]
 * with (ys, xs) the torch "nearest" source of (y, x) for an (h, w) -> (H, W)
 * resize (the 1x1 cond conv commutes with it and runs at (h, w)).  imc is
 * broadcast over T (one reference image per clip) and audio over (H, W).
 * bwd: d_imc[b][h][w][Ci] and d_audio[b][T][Ca] (fp32) are OVERWRITTEN, with fixed-order
 * sums (bit-reproducible; d_audio through a caller workspace of
 * vd_cond_concat_bwd_workspace_size bytes). */
int vd_cond_concat(const void* image, const void* imc, const void* audio,
                   void* out, int B, int T, int H, int W, int Cx, int h, int w,
                   int Ci, int Ca, int out_cstride, int dtype, void* stream);
size_t vd_cond_concat_bwd_workspace_size(int B, int T, int H, int W, int Ca);
int vd_cond_concat_bwd(const void* dout, float* d_imc, float* d_audio, int B,
                       int T, int H, int W, int Cx, int h, int w, int Ci,
                       int Ca, int out_cstride, int dtype, void* workspace,
                       void* stream);

/* ---- Upsample (nearest, x2 on H and W) --------------------------------
 * replaces unet.py:112-122 F.interpolate(..., mode="nearest") with the
 * dims=3 size (T, 2H, 2W) (and dims=2 scale_factor=2 with T=1).
 * x: [B][T][H][W][C] -> y: [B][T][2H][2W][C]; bwd sums the 4 children. */
int vd_upsample_nearest_hw(const void* x, void* y, int B, int T, int H, int W,
                           int C, int dtype, void* stream);
int vd_upsample_nearest_hw_bwd(const void* dy, void* dx, int B, int T, int H,
                               int W, int C, int dtype, void* stream);

/* ---- Convolution (implicit GEMM on MFMA) ------------------------------
 * replaces conv_nd (utils.py:59-69) at unet.py:110,143-145,197,223,231,234,
 * 494,627 and the 1x1 Conv1d of AttentionBlock (unet.py:298,306).
 * Weight layouts (packed by the caller from the torch [Co][Ci][kt][kh][kw]):
 *   fwd      : w_fwd [Co][taps][Ci]      (K = taps*Ci contiguous per Co)
 *   bwd_data : w_bwd [Ci][taps][Co]
 *   bwd_wgt  : dw    [Co][taps][Ci] fp32, ACCUMULATED into (zero it first)
 * Epilogue of fwd: y = conv + bias[co] + chan_add[b][co] + residual.
 * Any of bias / chan_add / residual may be NULL.  bias/chan_add are fp32;
 * residual has the activation dtype and y's shape.
 * Ci must be a multiple of 8 (bf16) or 4 (fp32); pad channels otherwise. */
typedef struct vd_conv_desc {
  int B;
  int Ti, Hi, Wi, Ci;  /* input  */
  int To, Ho, Wo, Co;  /* output */
  int kt, kh, kw;      /* kernel taps */
  int st, sh, sw;      /* stride */
  int pt, ph, pw;      /* zero padding */
  int x_cstride;       /* elements between input pixels (>= Ci), 0 = Ci */
  int y_cstride;       /* elements between output pixels (>= Co), 0 = Co */
  int dtype;
} vd_conv_desc;

int vd_conv3d_fwd(const vd_conv_desc* d, const void* x, const void* w_fwd,
                  const float* bias, const float* chan_add,
                  const void* residual, void* y, void* stream);
/* dx[B][Ti][Hi][Wi][Ci] = conv^T(dy); overwrites dx. */
int vd_conv3d_bwd_data(const vd_conv_desc* d, const void* dy,
                       const void* w_bwd, void* dx, void* stream);
/* dw[Co][taps][Ci] += sum over output pixels of dy (x) x  (fp32) */
int vd_conv3d_bwd_weight(const vd_conv_desc* d, const void* x, const void* dy,
                         float* dw, void* stream);
/* Deterministic weight gradient (the default of the Python ops since round 4): every pixel
 * split writes its fp32 partial dW into its own slice of `workspace`
 * (vd_conv3d_bwd_weight_workspace_size bytes), then one pass adds the slices in a fixed
 * order and WRITES dw in the torch layout [Co_out][Ci_out][taps] (Co_out <= d->Co and
 * Ci_out <= d->Ci drop the channel padding).  Bit-reproducible run to run; no zero fill
 * and no layout permute are needed.  Replaces the weight half of conv_nd's autograd
 * (utils.py:59-69) as vd_conv3d_bwd_weight does. */
size_t vd_conv3d_bwd_weight_workspace_size(const vd_conv_desc* d);
int vd_conv3d_bwd_weight_det(const vd_conv_desc* d, const void* x, const void* dy, float* dw,
                             int Co_out, int Ci_out, void* workspace, size_t workspace_bytes,
                             void* stream);

/* Which 3x3x3 stride-1 bf16 convs (fwd / bwd-data) take the halo-tile kernel: 0 none (the
 * gathered tiles), 1 and 2 (default) every eligible shape (W % 16 == 0, pad 1) on 4-wave
 * 2x4x16 tiles, 3 on 8-wave 2x8x16 tiles, 4 the 4-wave tiles with the compiler's fragment-read
 * placement, 5 the forward without early next-step halo pieces.  Modes 1-5 are bit-identical;
 * 0 agrees up to fp32 summation order.
 * Process-wide; returns the previous mode, or -2 for an invalid one.  Initial value from env
 * VDIFF_CONV_HALO.  No reference counterpart: an A/B and test hook. */
/* Which kernel computes the kw-strip (3x3x3 / 3x3 stride-1 bf16) and 1x1 weight gradients:
 * 1 (default) the round-6 kernel with the ring stages unrolled and early fragment reads, 2 the
 * same with the compiler's read placement, 0 the round-5 kernel; same tiles and summation
 * order (bit-identical results).  Returns the previous mode, or -2 (A/B, tests). */
int vd_conv_set_wgrad(int mode);
int vd_conv_set_halo(int mode);

/* ---- Conv glue ---------------------------------------------------------
 * vd_channel_sums: out[b][c] = sum over the S pixels of x[b][s][c] (fp32; x channels-last
 * with pixel stride cstride, 0 = C; C % 8 == 0; deterministic two-stage reduction through
 * a caller workspace of vd_channel_sums_workspace_size bytes).  One pass gives both the conv bias
 * gradient (sum over b) and the chan_add gradient of the ResBlock emb-add -- the autograd
 * of conv_nd's bias (utils.py:59-69) and of `h = h + emb_out` (unet.py:255-258).
 * vd_conv_pack_weight: torch fp32 weight [Co][Ci][taps] -> the w_fwd [Co][taps][Cip]
 * (transpose 0) or w_bwd [Cip][taps][Cop] (transpose 1) operand above, zero-padded. */
size_t vd_channel_sums_workspace_size(int B, int C);
int vd_channel_sums(const void* x, int B, int64_t S, int C, int cstride, int dtype,
                    float* out, void* workspace, void* stream);
int vd_conv_pack_weight(const float* w, int Co, int Ci, int taps, int Cip, int Cop,
                        int transpose, int dtype, void* out, void* stream);
/* vd_conv_pack_weights: n vd_conv_pack_weight jobs in ONE launch (a training step's conv
 * operands, re-packed once per optimizer step -- the weights that train.py:128-134's
 * optimizer.step() just updated).  `descs` is a DEVICE array of n descriptors with
 * start = the job's first element in the concatenation of all outputs (ascending, start[0]
 * = 0) and `total` the concatenation's length; every output is in `dtype`.  n <= 1024. */
typedef struct {
  const float* w;
  void* out;
  int Co, Ci, taps, Cip, Cop, transpose;
  int64_t start;
} vd_pack_desc;
int vd_conv_pack_weights(const vd_pack_desc* descs, int n, int64_t total, int dtype,
                         void* stream);

/* ---- Flash attention --------------------------------------------------
 * replaces QKVAttentionLegacy.forward (unet.py:349-366) + the fp32 softmax
 * (unet.py:364) and, with heads split by strides, QKVAttention (unet.py:
 * 388-401).  One "sequence" = `seq_len` tokens of one head; sequence i
 * starts at element (i / groups) * batch_stride + (i % groups) * group_stride
 * of q/k/v (and of o with the o_* strides); consecutive tokens are
 * token_stride apart.  joint: groups 1; spatial (per frame): groups T;
 * temporal (per pixel): groups H*W, token_stride H*W*row.
 * softmax(scale * q k^T) v, fp32 softmax statistics; lse fp32[nseq][seq_len]
 * (natural log of the row sum of exp(scale*s)) is saved for backward. */
typedef struct vd_attn_desc {
  int nseq, seq_len, head_dim, groups;
  int64_t batch_stride, group_stride, token_stride;       /* q/k/v */
  int64_t o_batch_stride, o_group_stride, o_token_stride; /* o and dout */
  float scale;
  int dtype;
} vd_attn_desc;

int vd_attention_fwd(const vd_attn_desc* d, const void* q, const void* k,
                     const void* v, void* o, float* lse, void* stream);
/* Same, with a workspace: where the query grid would leave CUs idle (bf16, e.g. head_dim 256
 * at N = 16384) the keys are split over grid.z and the fp32 partials merged by a second
 * kernel (flash-decoding style).  workspace_bytes < vd_attention_fwd_workspace_size(d)
 * (which is 0 for shapes that do not split) falls back to vd_attention_fwd. */
size_t vd_attention_fwd_workspace_size(const vd_attn_desc* d);
int vd_attention_fwd_ws(const vd_attn_desc* d, const void* q, const void* k,
                        const void* v, void* o, float* lse, void* workspace,
                        size_t workspace_bytes, void* stream);
/* Backward workspace: the row constants, plus the KV-split dQ partials for shapes that split. */
size_t vd_attention_bwd_workspace_size(const vd_attn_desc* d);
/* Kernel shape used for bf16 (no effect on results beyond fp32 summation order):
 * -1 per-kernel default, 0 base (4 waves x 32 rows), 1 two 32-row blocks per wave,
 * 2 eight waves, 3 / 4 software-pipelined with 8 / 4 waves, 5 / 6 the deferred-check
 * head_dim-64 forward with / without staggered wave halves, 7 the same with 4 waves and
 * two workgroups per CU, 8 the paired-wave head_dim-128 dK/dV, 9 the pipelined head_dim-64
 * backward with 4 waves x 2 blocks, 10 the role-split head_dim-256 dK/dV, 11 the
 * fragment-pipelined head_dim-64 backward, 12 the hand-scheduled head_dim-64 dQ (one wave
 * per SIMD, asm/gen_attn_asm.py) (shapes a kernel does not take keep their default).
 * Process-wide; returns the previous setting, or -2 for an invalid cfg (vd_last_error says
 * why).  Initial value from env VDIFF_ATTN_CFG
 * (base|nb2|w8|p8|p4|d8|d8n|d4|pair|p4n2|role|sp|asm).  No reference counterpart: an A/B
 * and test hook. */
int vd_attention_set_config(int cfg);
/* Short sequences (bf16, seq_len <= 32, head_dim 32/64/128/256, 16-B aligned rows: the
 * temporal attention of the spatial_temporal mode, T = 16 / 25 frames per pixel, and the
 * ViViT encoder's 9 tokens) run on dedicated kernels, one wave per sequence with 16x16 MFMA
 * tiles: vd_attention_fwd / _fwd_ws, and vd_attention_bwd as ONE fused dQ / dK / dV kernel
 * (no workspace used; it takes delta = rowsum(P dP) from the scores it holds, so its `o`
 * argument is not read there).  vd_attention_short_path(d) says whether d takes that path;
 * vd_attention_set_short(0) (or env VDIFF_ATTN_SHORT=0) routes such shapes to the flash
 * kernels instead (A/B and test hook; returns the previous setting).  No reference
 * counterpart: the reference materialises T x T scores (unet.py:361-365 per regrouped
 * sequence). */
int vd_attention_short_path(const vd_attn_desc* d);
/* The backward's decision on the real buffers: 1 when vd_attention_bwd will run the fused short
 * kernel for these pointers (every buffer 16-B aligned), 0 when it takes the flash dQ + dK/dV
 * kernels, which need the workspace of vd_attention_bwd_workspace_size. */
int vd_attention_bwd_short_path(const vd_attn_desc* d, const void* q, const void* k,
                                const void* v, const void* o, const void* dout, const void* dq,
                                const void* dk, const void* dv);
int vd_attention_set_short(int on);
/* dout uses the o_* strides; dq/dk/dv use the q/k/v strides (so they can be
 * written straight into a d(qkv) buffer) and are OVERWRITTEN. */
int vd_attention_bwd(const vd_attn_desc* d, const void* q, const void* k,
                     const void* v, const void* o, const void* dout,
                     const float* lse, void* dq, void* dk, void* dv,
                     void* workspace, void* stream);
/* The two halves of vd_attention_bwd (same arguments), for per-kernel timing:
 * _dq writes the per-row constants -rowsum(dO * O) and -lse*log2(e) into the
 * workspace and computes dq; _dkdv reads them and computes dk, dv.  Call _dq first. */
int vd_attention_bwd_dq(const vd_attn_desc* d, const void* q, const void* k,
                        const void* v, const void* o, const void* dout,
                        const float* lse, void* dq, void* workspace,
                        void* stream);
int vd_attention_bwd_dkdv(const vd_attn_desc* d, const void* q, const void* k,
                          const void* v, const void* dout, const float* lse,
                          void* dk, void* dv, void* workspace, void* stream);

/* ---- audio cross-attention (north_star build extension; no reference counterpart: the
 * reference conditions on audio by channel concatenation only, unet_audio.py:52-61).
 * Video tokens attend to audio tokens: softmax(scale * q k^T) v with q / o addressed by
 * `q` (as vd_attn_desc: nseq, seq_len = N_q, head_dim, groups, q and o strides, scale,
 * dtype) and k / v rows by the kv_* fields: sequence i's K/V rows start at
 * (i / q.groups) * kv_batch_stride + (i % q.groups) * kv_group_stride, kv_token_stride
 * apart, kv_len of them (N_kv may differ from N_q).  lse fp32 [nseq][N_q] as above.  The
 * backward has the self-attention contract (dq in the q strides, dk / dv in the kv
 * strides, overwritten); where the K/V grid leaves CUs idle (bf16, few audio tokens) the
 * queries are split and the fp32 dK / dV partials summed by a second kernel, inside the
 * workspace. */
typedef struct vd_xattn_desc {
  vd_attn_desc q;
  int kv_len;
  int64_t kv_batch_stride, kv_group_stride, kv_token_stride;
} vd_xattn_desc;

size_t vd_cross_attention_fwd_workspace_size(const vd_xattn_desc* x);
int vd_cross_attention_fwd(const vd_xattn_desc* x, const void* q, const void* k,
                           const void* v, void* o, float* lse, void* workspace,
                           size_t workspace_bytes, void* stream);
size_t vd_cross_attention_bwd_workspace_size(const vd_xattn_desc* x);
int vd_cross_attention_bwd_dq(const vd_xattn_desc* x, const void* q, const void* k,
                              const void* v, const void* o, const void* dout,
                              const float* lse, void* dq, void* workspace, void* stream);
int vd_cross_attention_bwd_dkdv(const vd_xattn_desc* x, const void* q, const void* k,
                                const void* v, const void* dout, const float* lse,
                                void* dk, void* dv, void* workspace, void* stream);

/* ---- data path (video-generation/dataset.py:68-139) ----------------
 * Frames: the reference's ToPILImage -> Resize((S, S)) -> ToTensor -> Normalize(0.5, 0.5)
 * (train.py:70-75, dataset.py:109-111) = PIL's antialiased bilinear resample.
 * vd_resize_plan (HOST, no GPU) computes one axis of PIL's plan (libImaging/Resample.c
 * precompute_coeffs + normalize_coeffs_8bpc): bounds int[out][2] (first tap, taps) and
 * 22-bit fixed-point coefficients int[out][ksize], ksize = 2 * ceil(in / out) + 1 (<= cap).
 * vd_frames_resize_normalize (GPU): uint8 frames [n][H][W][3] -> horizontal pass into tmp
 * (uint8 [n][H][OW][3]) -> vertical pass -> (v / 255 - 0.5) / 0.5 in `dtype`, frame f at
 * out + f * frame_stride as [3][OH][OW] (channels_last = 0) or [OH][OW][3]; the uint8
 * values equal PIL's bit for bit.  Plans are device int arrays. */
int vd_resize_plan(int in_size, int out_size, int* bounds, int* coef, int ksize_cap);
int vd_frames_resize_normalize(const uint8_t* frames, int64_t n, int H, int W, int OH, int OW,
                               const int* xbounds, const int* xcoef, int xksize,
                               const int* ybounds, const int* ycoef, int yksize, uint8_t* tmp,
                               void* out, int dtype, int64_t frame_stride, int channels_last,
                               void* stream);
/* HOST (no GPU): the audio window of one output frame, dataset.py:113-130 -- samples
 * [int(sr * max(0, (out_frame - buffer_frames) / fps)), int(sr * out_frame / fps)) of the
 * track wave fp32 [channels][n]; torchaudio highpass_biquad(300 Hz, Q 0.707) with lfilter's
 * clamp to [-1, 1]; (x - mean) / std (unbiased, all channels); process_audio (:51-66):
 * resample to target_sr (bug_compatible = 1: from orig_freq = channels, as the reference's
 * size(0) comparison does; 0: from sr, identity when sr == target_sr; torchaudio's
 * sinc_interp_hann kernel, width 6, rolloff 0.99), zero-pad / trim to target_len; then the
 * Wav2Vec2 processor's (x - mean) / sqrt(var + 1e-7) per channel.  out fp32
 * [channels][target_len]. */
int vd_audio_window(const float* wave, int channels, int64_t n, int sr, double fps,
                    int out_frame, int buffer_frames, int target_len, int target_sr,
                    int bug_compatible, float* out);

/* ---- ViViT lipreading encoder ops (lipreading/huggingface_vivit_model.py:18-33
 * over transformers' VivitModel: VivitLayer.layernorm_before/_after, final layernorm, VivitMLP
 * with hidden_act "gelu_fast").
 * vd_layernorm_fwd: rows of C contiguous elements (C % 8 == 0, C <= 2048); fp32 affine w, b;
 * writes y and the fp32 per-row mean / rstd the backward reads.
 * vd_layernorm_bwd: dx (overwritten), dw = sum(dy * xhat), db = sum(dy) over rows (fp32,
 * overwritten, deterministic), through a workspace of vd_layernorm_workspace_size bytes.
 * vd_gelu_tanh(_bwd): y = 0.5 x (1 + tanh(0.7978845608 x (1 + 0.044715 x^2))) on n elements
 * (n % 8 == 0); bwd: dx = dy * y'(x). */
size_t vd_layernorm_workspace_size(int rows, int C);
int vd_layernorm_fwd(const void* x, const float* w, const float* b, void* y, float* mean,
                     float* rstd, int rows, int C, float eps, int dtype, void* stream);
int vd_layernorm_bwd(const void* dy, const void* x, const float* w, const float* mean,
                     const float* rstd, void* dx, float* dw, float* db, int rows, int C,
                     int dtype, void* workspace, size_t workspace_bytes, void* stream);
int vd_gelu_tanh(const void* x, void* y, int64_t n, int dtype, void* stream);
int vd_gelu_tanh_bwd(const void* x, const void* dy, void* dx, int64_t n, int dtype,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VDIFF_H */
