/*
 * rdunet_hip.h — C ABI of librdunet_hip.so, the MI355X (gfx950) kernels of the
 * diffusion-RDUNet denoising hot path.
 *
 * Every entry point takes plain device pointers, element strides and sizes plus
 * a hipStream_t (passed as void*), launches asynchronously on that stream and
 * returns 0 on success or a negative RDN_E* code; rdn_last_error() returns a
 * thread-local message for the last failure on the calling thread.  The library
 * never allocates, frees or synchronises, so every call is hipGraph-capture safe.
 * Caller-owned workspaces are sized by the *_workspace_size queries.
 *
 * Layouts: activations NHWC with an explicit pixel stride (elements between two
 * pixels) and a channel offset, so a conv can read/write a channel slice of a
 * dense-block buffer (this is how the reference's torch.cat disappears).
 * Weights stay in the reference's OIHW (Conv2d) / IOHW (ConvTranspose2d) fp32
 * layout in the state_dict and are packed per call site by rdn_pack_weights.
 *
 * Reference interfaces replaced (file:line under pierregab/VUB_Image_denoising):
 *   rdn_conv_fwd      nn.Conv2d 3x3 p1 + nn.PReLU (+ residual add, + torch.cat)
 *                     diffusion_denoising/Unet/Unet_model.py:48-55,60-67,72-89,35-43;
 *                     nn.Conv2d k2 s2 + PReLU  Unet_model.py:26-30;
 *                     nn.ConvTranspose2d k2 s2 + PReLU  Unet_model.py:36-42;
 *                     and (with packed transposed weights) their input gradients
 *                     (aten convolution_backward, grad_input).
 *   rdn_conv_wgrad /  aten convolution_backward grad_weight for the same convs.
 *   rdn_wgrad_reduce
 *   rdn_conv_dgrad_wgrad  both of the above for one gated level-0 conv in one pass.
 *   rdn_dense3_fwd    conv_0..conv_2 (+ PReLU, + torch.cat) of a level-0 / level-1 DenoisingBlock
 *                     in one pass, Unet_model.py:81-87.
 *   rdn_prelu_bwd     aten _prelu_kernel_backward (dx, dalpha) + conv grad_bias.
 *   rdn_interp        x = a*noisy + (1-a)*clean, diffusion_RDUnet.py:90-100, :33-36.
 *   rdn_pack_input    torch.cat((inputs, t.expand(...)), 1), Unet_model.py:135-136.
 *   rdn_charbonnier_fwd/bwd  charbonnier_loss/combined_loss, diffusion_RDUnet.py:57-65.
 *   rdn_sqnorm / rdn_clip_scale  torch.nn.utils.clip_grad_norm_, diffusion_RDUnet.py:113.
 *   rdn_adam_step     torch.optim.Adam / AdamW step, diffusion_RDUnet.py:264-268,127.
 *   rdn_sampling_combine  the x_t update of improved_sampling, diffusion_RDUnet.py:45-49.
 *   rdn_synth_batch   CustomDataset/CustomSIDD_Dataset.__getitem__ + transforms
 *                     (dataset_creation/custom_dataset.py:64-100, SIDD_dataset.py:74-97).
 *   rdn_image_metrics skimage peak_signal_noise_ratio / structural_similarity,
 *                     evaluate_SIDD/evaluate_SIDD.py:63-64.
 */
#ifndef RDUNET_HIP_H
#define RDUNET_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { RDN_OK = 0, RDN_E_ARG = -1, RDN_E_SHAPE = -2, RDN_E_LAUNCH = -3 };

/* element type of activations / packed weights; master weights and weight
   gradients are always fp32 */
enum { RDN_F32 = 0, RDN_BF16 = 1 };

/* how GEMM row m (a pixel of the row grid n,h,w) gathers its K = taps*cin inputs */
enum {
  RDN_G_CONV3 = 0, /* 3x3, stride 1, pad 1: src (y+ky-1, x+kx-1), taps 9     */
  RDN_G_S2 = 1,    /* 2x2, stride 2: src (2y+dy, 2x+dx) of a 2h x 2w grid, taps 4 */
  RDN_G_PIX = 2    /* 1 tap, src (y, x): a plain per-pixel GEMM                */
};

/* epilogue flags of rdn_conv_fwd, applied in this order */
enum {
  RDN_EPI_BIAS = 1,      /* v += bias[c]                                     */
  RDN_EPI_STORE_PRE = 2, /* pre[pix, c] = v (PReLU input kept for backward)  */
  RDN_EPI_PRELU = 4,     /* v = v > 0 ? v : alpha[c] * v                     */
  RDN_EPI_RESID = 8,     /* v += res[pix, res_c0 + c] for c < res_climit     */
  RDN_EPI_ACCUM = 16,    /* v += out[pix, out_c0 + c] (gradient accumulation) */
  RDN_EPI_SCATTER2 = 32, /* column j = tap*cout + c lands on pixel (2y+dy, 2x+dx) */
  RDN_EPI_OUT_NCHW = 64, /* write fp32 NCHW out_nchw (residual from res_nchw)  */
  RDN_EPI_GOUT_KEEP = 128 /* with gout (rdn_conv_dgrad_wgrad only): the gated columns'
                             dY is stored to out as well (the finished layer's own
                             residual epilogue reads it)                     */
};

typedef struct rdn_conv_desc {
  int32_t dtype, gather, flags;
  int32_t n, h, w;       /* GEMM row grid: M = n*h*w                          */
  int32_t hin, win;      /* source image size                                 */
  int32_t cin;           /* channels per tap; K = taps*cin; multiple of 8     */
  const void* x; int64_t x_ps; int32_t x_c0;
  const void* wp; int32_t kp;  /* packed weights [rows >= ncols padded to 128][kp] */
  int32_t ncols;         /* valid GEMM columns                                */
  int32_t cout;          /* channels per output pixel (scatter: ncols/4)      */
  const float* bias; const float* alpha;
  void* out; int64_t out_ps; int32_t out_c0;
  void* pre; int64_t pre_ps;
  const void* res; int64_t res_ps; int32_t res_c0; int32_t res_climit;
  float* out_nchw; const float* res_nchw;
  int32_t bm, bn;        /* tile override, 0 = automatic                      */
  /* optional PReLU-backward gate on the INPUT (RDN_G_CONV3 only): the gathered
     x[p][c] becomes x[p][c] * (gate[p][c] > 0 ? 1 : gate_alpha[c]), i.e. the conv
     consumes dYpre computed on the fly from dY and the saved PReLU input
     (aten _prelu_kernel_backward fused into the input-gradient conv) */
  const void* gate; int64_t gate_ps; const float* gate_alpha;
  /* channel-blocked ("planar") operands.  With *_pl == 0 an operand is plain NHWC:
     channel c of pixel p sits at p*ps + c.  With *_pl > 0 its channels come in
     blocks of ps, each block one contiguous [pixels][ps] plane, planes *_pl
     elements apart: channel c of pixel p sits at (c/ps)*pl + p*ps + c%ps.  A conv
     that reads or writes a channel slice of such a buffer then touches only the
     planes of that slice (the dense-block buffers of Unet_model.py:81-89 are laid
     out this way so conv_0..conv_2 do not drag the whole pixel row through HBM).
     Channel offsets (x_c0, ...) count across planes; ps % (16 B / elem) == 0. */
  int64_t x_pl, out_pl, pre_pl, res_pl, gate_pl;
  /* optional PReLU backward fused into an INPUT-GRADIENT epilogue ("gate out",
     RDN_G_CONV3 only): with gout != NULL the output columns [gout_c0, ncols) are
     the complete gradient dY of the layer whose PReLU output is that input slice
     (this conv is its last consumer in backward order, e.g. conv_k+1 for the
     dense slice out_k, Unet_model.py:81-87).  Instead of storing dY there, the
     epilogue writes that layer's dYpre (aten _prelu_kernel_backward):
       gout[p][c'] = dY[p][c'] * (gout_pre[p][c'] > 0 ? 1 : gout_alpha[c']),
       c' = c - gout_c0 (plain NHWC, strides gout_ps / gout_pre_ps),
     and per-tile channel partials of its dalpha / conv-bias gradients
       gout_part[row][0][c'] = sum_{pre<=0} pre*dY, gout_part[row][1][c'] = sum dYpre
     over rdn_conv_gate_rows(d) rows (summed by rdn_wgrad_reduce, fixed order). */
  void* gout; int64_t gout_ps; const void* gout_pre; int64_t gout_pre_ps;
  const float* gout_alpha; float* gout_part; int32_t gout_c0;
} rdn_conv_desc;

/* Implicit-GEMM convolution (MFMA) with the fused epilogue above. */
int rdn_conv_fwd(const rdn_conv_desc* d, void* stream);
/* Split-K form of rdn_conv_fwd for 3x3 convs whose pixel grid is too small to fill the
   device (a batch-1 forward's deep levels, UNet/RDUNet_model.py:157-186): the input
   channels are walked in `splits` slices by separate blocks, each storing raw fp32 sums to
   ws (rdn_conv_fwd_splitk_workspace_size bytes), then one launch sums the slices in slice
   order (deterministic) and applies d's epilogue.  splits must equal rdn_conv_fwd_splits(d)
   (0: not split -- rdn_conv_fwd); no input gate / gate-out / scatter, ncols % 4 == 0. */
int32_t rdn_conv_fwd_splits(const rdn_conv_desc* d);
int64_t rdn_conv_fwd_splitk_workspace_size(const rdn_conv_desc* d, int32_t splits);
int rdn_conv_fwd_splitk(const rdn_conv_desc* d, int32_t splits, float* ws, void* stream);
/* partial rows the gate-out epilogue of d writes (d->gout set; nothing is
   launched); 0 when the kernel rdn_conv_fwd picks for d has no gate-out form
   (launch the separate rdn_prelu_bwd instead) */
int rdn_conv_gate_rows(const rdn_conv_desc* d);
/* name of the kernel instantiation rdn_conv_fwd would launch for d (nothing is
   launched); for profiles and per-kernel timing */
int rdn_conv_kernel_name(const rdn_conv_desc* d, char* buf, int32_t len);

typedef struct rdn_wgrad_desc {
  int32_t dtype, gather;   /* gather of the B operand: RDN_G_CONV3 or RDN_G_S2 */
  int32_t n, h, w;         /* pixel grid of operand A (reduction length n*h*w) */
  int32_t hin, win;        /* grid of operand B                                */
  const void* a; int64_t a_ps; int32_t a_c0; int32_t mdim;  /* rows of dW (A channels; A
                           buffer zero padded to a multiple of 8 channels)     */
  const void* b; int64_t b_ps; int32_t b_c0; int32_t ndim;  /* per-tap columns, multiple of 8 */
  float* ws;               /* [splits][mdim][taps*ndim] partial sums           */
  int32_t splits;          /* 0 = automatic (see rdn_wgrad_splits)             */
  /* optional PReLU-backward gate on operand A (RDN_G_CONV3 only), as in
     rdn_conv_desc; with `part` non-NULL the kernel also writes per-split channel
     partials part[split][0][m] = sum_{gate<=0} gate*A, part[split][1][m] = sum
     gated A (dalpha / conv-bias gradients, summed by rdn_wgrad_reduce) */
  const void* a_gate; int64_t a_gate_ps; const float* a_gate_alpha; float* part;
  int64_t a_pl, b_pl, a_gate_pl;   /* channel-blocked operands, as in rdn_conv_desc */
} rdn_wgrad_desc;

/* dW[m][tap][nd] partials = sum over pixels p of A[p][m] * B[gather(p,tap)][nd] */
int rdn_conv_wgrad(const rdn_wgrad_desc* d, void* stream);
/* name of the kernel instantiation rdn_conv_wgrad would launch for d */
int rdn_wgrad_kernel_name(const rdn_wgrad_desc* d, char* buf, int32_t len);
/* split count the automatic mode would use, and the workspace it needs (bytes) */
int rdn_wgrad_splits(const rdn_wgrad_desc* d);
/* input-channel chunks (grid.y) of the 3x3 weight-gradient kernel: operand A is
   read once per chunk, so the PReLU gate on A pays off only with 1 chunk */
int rdn_wgrad_chunks(const rdn_wgrad_desc* d);
int64_t rdn_wgrad_workspace_size(const rdn_wgrad_desc* d);
/* grad[(m*ndim_real+nd)*taps+tap] (+)= sum_s ws[s][m][tap*ndim+nd] for nd < ndim_real:
   the reference's OIHW (Conv2d) / IOHW (ConvTranspose2d) order.  With `part`
   non-NULL also dalpha[m] += sum_s part[s][0][m], dbias[m] += sum_s part[s][1][m]
   over s < part_splits (0: = splits) -- the partials of a gated rdn_conv_wgrad or
   of rdn_prelu_bwd run without dalpha/dbias (fixed summation order: deterministic). */
int rdn_wgrad_reduce(const float* ws, int32_t splits, int32_t mdim, int32_t ndim, int32_t ndim_real,
                     int32_t taps, float* grad, int32_t accumulate,
                     const float* part, int32_t part_splits, float* dalpha, float* dbias, void* stream);
/* the same for slabs that hold a slice of the input channels: grad[(m*grad_ci_total +
   grad_ci0 + nd)*taps + tap] (+)= sum_s ws[s][m][tap*ndim + nd] for nd < ndim (the column
   halves of rdn_conv_dgrad_wgrad, rdn_conv_dgrad_wgrad_cols) */
int rdn_wgrad_reduce_cols(const float* ws, int32_t splits, int32_t mdim, int32_t ndim, int32_t taps, float* grad,
                          int32_t grad_ci_total, int32_t grad_ci0, int32_t accumulate, const float* part,
                          int32_t part_splits, float* dalpha, float* dbias, void* stream);
/* Up to RDN_REDUCE_BATCH_MAX of these reductions in ONE launch (round 4: the fused
   layers' reduces on the compute stream are latency-bound, one launch each).  A job
   is rdn_wgrad_reduce_cols's arguments (ndim_real <= ndim: rdn_wgrad_reduce's
   ndim_real with gstride = ndim_real, gci0 = 0); sl / blocks / pblocks are filled in
   by the call.  Results bit-identical to the single launches. */
#define RDN_REDUCE_BATCH_MAX 8
typedef struct rdn_reduce_job {
  const float* ws; float* grad; const float* part; float* dalpha; float* dbias;
  int32_t splits, mdim, ndim, ndim_real, taps, gstride, gci0, accumulate, part_splits;
  int32_t sl, blocks, pblocks;   /* (set by rdn_wgrad_reduce_batch) */
} rdn_reduce_job;
int rdn_wgrad_reduce_batch(const rdn_reduce_job* jobs, int32_t n, void* stream);

/* Fused input gradient + weight gradient of one gated 3x3 conv (the narrow level-0
   layers: dgrad->cin = 16|32 dY channels, dgrad->ncols = wgrad->ndim = 32..80 input
   channels; and, in two column halves, the level-1 conv_1 / conv_2 with 32 dY and 96 /
   128 input channels; full 8x16 tiles, bf16): ONE pass over the gated dY (dgrad->gate must be
   set and equal wgrad->a_gate; wgrad->a must be dgrad->x) computes
   rdn_conv_fwd(dgrad) and rdn_conv_wgrad(wgrad) together, i.e. aten
   convolution_backward's grad_input and grad_weight of Unet_model.py:72-89 with
   _prelu_kernel_backward fused.  wgrad->splits must equal
   rdn_conv_dgrad_wgrad_splits(); sum with rdn_wgrad_reduce as usual.
   Returns 0 (launched), 1 (pair not served: launch the two separately) or < 0. */
int rdn_conv_dgrad_wgrad(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad, void* stream);
/* split count (weight-gradient slabs) the fused kernel writes for the pair; 0 = not served */
int rdn_conv_dgrad_wgrad_splits(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad);
/* input channels per weight-gradient slab: wgrad->ndim, or ndim/2 for the column-half
   launches, whose slabs [h*splits/2, (h+1)*splits/2) hold channels [h*ndim/2, ...) (sum
   each half with rdn_wgrad_reduce_cols; the dalpha/dbias partials are in half 0's rows,
   half 1's are zero); 0 = not served */
int rdn_conv_dgrad_wgrad_cols(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad);
/* gate-out on the fused pair (dgrad->gout set, as for rdn_conv_fwd; round 4): the
   shapes of up_0.conv (96 columns in halves) and the level-1 conv_0 (64 columns), no
   residual, 0 <= gout_c0 < ncols.  Each block writes one partial row (zeros in the
   columns of the other half): rows = this value (= the split count); 0 = not served */
int rdn_conv_dgrad_wgrad_gate_rows(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad);
/* name of the fused kernel instantiation (1 = not served) */
int rdn_conv_dgrad_wgrad_kernel_name(const rdn_conv_desc* dgrad, const rdn_wgrad_desc* wgrad, char* buf, int32_t len);

/* Fused forward of conv_0..conv_2 of a level-0 DenoisingBlock with base_filters 32
   (Unet_model.py:81-87: x 32 channels, growth 16, bf16): the same results as the three
   rdn_conv_fwd launches (bias, PReLU-input store, PReLU), in one pass that reads x once
   and keeps out_0 / out_1 on chip.  x: the block buffer's first plane (channels 0-15;
   channels 16-31 x_pl elements further; channel-blocked, 16-channel planes);
   out[k]: the plane receiving conv_k's output (pixel stride 16); pre[k]: its PReLU
   input, plain [pixels][16]; wp[k]: packed forward weights (rdn_pack_weights with
   ck = cin, kp[k] columns).  H % 8 == 0, W % 16 == 0.
   x_c = 64 (round 6): the level-1 block (x 64 channels, growth 32, 32-channel planes:
   x channels 32-63 x_pl elements after 0-31, out[k] pixel stride 32, pre[k] plain
   [pixels][32], wp[k] packed by rdn_pack_weights CONV_FWD with the rdn_conv3_chunk
   K order of cin = 64 / 96 / 128: kp >= 576 / 896 / 1152); H % 16 == 0, W % 16 == 0.
   x_c = 0 or 32: the level-0 form above.
   pre[k] may be NULL (a forward-only caller that keeps no PReLU input): nothing is
   stored for it. */
typedef struct rdn_dense3_desc {
  int32_t n, h, w;
  const void* x; int64_t x_pl;
  void* out[3]; void* pre[3];
  const void* wp[3]; int32_t kp[3];
  const float* bias[3]; const float* alpha[3];
  int32_t x_c;
} rdn_dense3_desc;
int rdn_dense3_fwd(const rdn_dense3_desc* d, void* stream);
/* name of the instantiation (tile geometry: 8x16, 16x16 or 8x32 output pixels, env
   RDN_DENSE_TILE) rdn_dense3_fwd launches for d; nothing is launched */
int rdn_dense3_kernel_name(const rdn_dense3_desc* d, char* buf, int32_t len);

/* PReLU backward (+ conv bias gradient) over a pixel grid of `pixels` pixels:
   dyp[p, c] = dy[p, c] * (pre[p, c] > 0 ? 1 : alpha[c])   (c < C; 0 for C <= c < cpad)
   dalpha[c] += sum_{pre<=0} pre*dy ; dbias[c] += sum dyp.
   dy is NHWC (dy_ps, dy_c0, channel-blocked when dy_pl > 0) or, when dy_nchw != NULL, fp32
   NCHW of the (n,h,w) grid. */
int rdn_prelu_bwd(int32_t dtype, int64_t pixels, int32_t n, int32_t h, int32_t w, int32_t C, int32_t cpad,
                  const void* dy, int64_t dy_ps, int32_t dy_c0, int64_t dy_pl, const float* dy_nchw,
                  const void* pre, int64_t pre_ps, const float* alpha,
                  void* dyp, float* dalpha, float* dbias, float* ws, void* stream);
/* per-block channel partials (deterministic, no atomics): bytes of `ws` needed */
int64_t rdn_prelu_bwd_workspace_size(int32_t dtype, int64_t pixels, int32_t C, int32_t cpad);
/* number of [2][C] partial rows rdn_prelu_bwd leaves in ws; with dalpha and dbias
   both NULL it stops there and rdn_wgrad_reduce (part_splits = this) sums them */
int32_t rdn_prelu_bwd_blocks(int32_t dtype, int64_t pixels, int32_t cpad);

/* x[b] = a_b*noisy[b] + (1-a_b)*clean[b], a_b = tnorm[b]; fp32 NCHW, `per` elements per image */
int rdn_interp(const float* clean, const float* noisy, const float* tnorm, int32_t batch, int64_t per,
               float* x, void* stream);

/* NHWC input image [n,h,w,cpad]: channels 0..c-1 from fp32 NCHW x, channel c from t
   (t[b*t_sb + y*t_sh + x*t_sw], strides may be 0 to broadcast) when has_t, rest 0 */
int rdn_pack_input(int32_t dtype, const float* x, int32_t n, int32_t c, int32_t h, int32_t w,
                   const float* t, int64_t t_sb, int64_t t_sh, int64_t t_sw, int32_t has_t,
                   void* out, int32_t cpad, void* stream);

/* fp32 OIHW/IOHW weight -> packed GEMM operand [rows_pad][kp] of `dtype`. */
enum {
  RDN_PACK_CONV_FWD = 0,  /* W[co][ci][ky][kx] -> P[co][tap*cin_p + ci]               */
  RDN_PACK_CONV_DGRAD = 1,/* W[co][ci][ky][kx] -> P[ci][tap'*cout_p + co], tap' flipped */
  RDN_PACK_GEMM_T = 2     /* W[a][b][dy][dx] (a = K side) -> P[tap*d1 + b][a]          */
};
/* CONV_FWD packs W[a][b][t] -> P[a][tap*pad1 + b] (pad1 >= d1, zero fill), which also
   serves ConvTranspose2d's input gradient in conv-s2 form (a = ci, b = co).
   CONV_DGRAD packs P[b][tap'*pad0 + a] with tap' the 180-degree rotated tap.
   GEMM_T packs the per-pixel GEMM of ConvTranspose2d forward / Conv2d-s2 dgrad;
   its K (= d0) is zero padded to pad0. */
int rdn_pack_weights(int32_t mode, int32_t dtype, const float* w, int32_t d0, int32_t d1, int32_t kh, int32_t kw,
                     int32_t pad0, int32_t pad1, void* out, int32_t rows_pad, int32_t kp, int32_t ck, void* stream);
/* ck > 0 (CONV_FWD / CONV_DGRAD of a 3x3 conv): chunked K order for the halo kernel,
   k = chunk*KC + tap*ck + ci, KC = roundup(9*ck, 128 B / elem size).  ck must be
   rdn_conv3_chunk(K-side channels, dtype); rdn_conv3_packed_k gives the kp to use. */
int rdn_conv3_chunk(int32_t cin, int32_t dtype);
int rdn_conv3_packed_k(int32_t cin, int32_t dtype);
/* output-channel tile the 3x3 kernel uses for `ncols` columns (16..128) */
int rdn_conv3_pick_bn(int32_t ncols);

/* Many packs in one launch: `items` is a DEVICE array of n rdn_pack_item, each with
   kp a multiple of 64 and rows_pad * kp < 2^31 (as the engine allocates them). */
typedef struct rdn_pack_item {
  const float* w; void* out;
  int32_t mode, d0, d1, kh, kw, pad0, pad1, rows_pad, kp, ck;
} rdn_pack_item;
int rdn_pack_weights_batched(const rdn_pack_item* items, int32_t n, int32_t dtype, void* stream);

/* Charbonnier (+MSE) over `count` fp32 elements.  ws >= rdn_reduce_workspace_size(count).
   out[0] = mean(sqrt(d^2+eps^2)), out[1] = mean(d^2). */
int64_t rdn_reduce_workspace_size(int64_t count);
int rdn_charbonnier_fwd(const float* pred, const float* target, int64_t count, float eps,
                        float* ws, float* out, void* stream);
/* dpred = gout[0] * (wc * d/sqrt(d^2+eps^2) + wm * 2d) / count */
int rdn_charbonnier_bwd(const float* pred, const float* target, int64_t count, float eps,
                        float wc, float wm, const float* gout, float* dpred, void* stream);

/* out[0] = sqrt(sum g^2) over a flat fp32 buffer; out[1] = min(max_norm/(out[0]+1e-6), 1) */
int rdn_sqnorm(const float* g, int64_t count, float max_norm, float* ws, float* out, void* stream);
/* the same for pre_scale*g without scaling g (pre_scale > 0: the data-parallel 1/world
 * average folded into the clip): out[0] = norm of pre_scale*g, out[1] = pre_scale *
 * min(max_norm/(out[0]+1e-6), 1); rdn_clip_scale with out+1 then leaves the averaged,
 * clipped gradient.  Bit-identical to averaging first when pre_scale is a power of two. */
int rdn_sqnorm_scaled(const float* g, int64_t count, float max_norm, float pre_scale, float* ws, float* out,
                      void* stream);
/* g *= coef[0] (device scalar; no host sync) */
int rdn_clip_scale(float* g, int64_t count, const float* coef, void* stream);

/* torch.optim.Adam(W) step over flat fp32 buffers.  decoupled = 1 -> AdamW
   (p *= 1 - lr*wd), 0 -> Adam L2 (g += wd*p).  Hyperparameters come in double and
   every derived scalar (1-beta, lr/(1-beta1^t), sqrt(1-beta2^t), 1-lr*wd) is rounded
   to fp32 from double, as torch's single-tensor Adam does.  `step` (>= 1) is the
   step number t; when step_dev != NULL it is read from device memory instead (a
   graph-replayable optimizer step; advance it with rdn_counter_inc).  grad_scale
   multiplies g first (e.g. 1/world_size). */
int rdn_adam_step(float* p, const float* g, float* m, float* v, int64_t count,
                  double lr, double beta1, double beta2, double eps, double wd, int32_t decoupled,
                  int64_t step, const int64_t* step_dev, float grad_scale, void* stream);
/* *counter += 1 on the device (one thread; stream-ordered) */
int rdn_counter_inc(int64_t* counter, void* stream);
/* buf[slot] = the device wall clock (constant rate, rdn_wall_clock_khz ticks per ms) when
   this launch starts on `stream`: stream-ordered timestamps that survive hipGraph capture
   (the exposed all-reduce time of the replayed data-parallel step; no reference
   counterpart -- the reference has no data parallelism) */
int rdn_stamp(uint64_t* buf, int32_t slot, void* stream);
/* ticks per millisecond of rdn_stamp's clock (hipDeviceAttributeWallClockRate, kHz), < 0 on error */
int64_t rdn_wall_clock_khz(void);

/* improved_sampling update: x = x - (c1*f1 + a*y) + (c2*f2 + ap*y), with c1 = 1-a and
   c2 = 1-ap rounded on the host exactly as the reference's Python scalars are */
int rdn_sampling_combine(float* x, const float* f1, const float* f2, const float* y, int64_t count,
                         float c1, float a, float c2, float ap, void* stream);

/* dense layout converters (fp32 NCHW <-> NHWC slice of `dtype`, channel-blocked when *_pl > 0) */
int rdn_nchw_to_nhwc(int32_t dtype, const float* src, int32_t n, int32_t c, int32_t h, int32_t w,
                     void* dst, int64_t dst_ps, int32_t dst_c0, int64_t dst_pl, int32_t accumulate, void* stream);
int rdn_nhwc_to_nchw(int32_t dtype, const void* src, int64_t src_ps, int32_t src_c0, int64_t src_pl,
                     int32_t n, int32_t c, int32_t h, int32_t w, float* dst, int32_t accumulate, void* stream);

/* fill a [pixels][cols] NHWC slice with zeros */
int rdn_zero_slice(int32_t dtype, void* dst, int64_t pixels, int64_t ps, int32_t c0, int32_t cols, void* stream);

/* GPU data synthesis: replaces CustomDataset.__getitem__ (dataset_creation/custom_dataset.py:64-100)
   and CustomSIDD_Dataset.__getitem__ (dataset_creation/SIDD_dataset.py:74-97) + the torchvision
   transforms of data_loader.py:35-46 for a whole batch.  One item = one P x P patch of a uint8 HWC
   image resident in device memory. */
typedef struct rdn_synth_item {
  int64_t clean_off;   /* byte offset of the patch's (0,0) pixel in clean_pool                  */
  int64_t noisy_off;   /* same in noisy_pool (real noisy/gt pairs); unused with synthetic noise */
  uint64_t seed;       /* key of the device noise stream                                       */
  int32_t row_stride;  /* bytes between two rows of the source image (width * channels)         */
  float sigma;         /* Gaussian sigma on the 0..255 scale (custom_dataset.py:83-85); 0: none */
  int32_t flip;        /* RandomHorizontalFlip fired (data_loader.py:42)                        */
  int32_t rotate;      /* RandomRotation fired: affine[] holds Pillow's 16.16 fixed-point       */
  int32_t affine[6];   /*   output->input coefficients of Image.rotate(angle, NEAREST) (:43)    */
} rdn_synth_item;
/* out_noisy / out_clean: fp32 NCHW [n][channels][patch][patch] in [-1, 1] (ToTensor +
   Normalize(0.5, 0.5)).  noisy_pool != NULL: the noisy image is read (paired data).  Otherwise
   noisy = clip(float32(clean + noise)) -> uint8 with noise[n][patch][patch][channels] (float64,
   e.g. the reference's np.random.normal draws) when noise != NULL, else a counter-based
   N(0, sigma) draw on the device.  items is a DEVICE array. */
int rdn_synth_batch(const rdn_synth_item* items, int32_t n, int32_t channels, int32_t patch,
                    const uint8_t* clean_pool, const uint8_t* noisy_pool, const double* noise,
                    float* out_noisy, float* out_clean, void* stream);

/* SIDD evaluation metrics (evaluate_SIDD/evaluate_SIDD.py:63-64, scikit-image 0.22
   peak_signal_noise_ratio / structural_similarity(channel_axis, win_size 7, uniform
   window, sample covariance)) for a batch of n fp32 NCHW image pairs: psnr[n] and
   ssim[n] (float64, device; either may be NULL).  ws: rdn_image_metrics_workspace_size
   bytes.  Images must be at least 7x7. */
int64_t rdn_image_metrics_workspace_size(int32_t n, int32_t c, int32_t h, int32_t w);
int rdn_image_metrics(const float* gt, const float* x, int32_t n, int32_t c, int32_t h, int32_t w,
                      float data_range, double* ws, double* psnr, double* ssim, void* stream);

const char* rdn_version(void);
const char* rdn_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RDUNET_HIP_H */
