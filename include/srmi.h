/* srmi -- MI355X-native (gfx950) engine for the RCAN / EDSR tiled
 * super-resolution hot path of nasa-nccs-hpda/super-resolution-climate.
 *
 * C ABI: plain pointers, sizes and a hipStream_t (passed as void*).  No torch
 * types.  All device memory is owned by the caller (PyTorch's caching
 * allocator on the Python side) and handed in as workspace; the library's only
 * allocation is host-side: the srmi_engine object (plan, workspace layout, pack
 * tables), created by srmi_engine_create and released by srmi_engine_destroy.
 * It creates no streams and no events: every launch goes to the caller's stream
 * (group events for a bucketed all-reduce are the caller's).  Every entry point returns 0
 * on success or a negative status (SRMI_ERR_*, or -hipError_t), which the
 * Python binding raises as RuntimeError (the reference raises Python
 * exceptions; sres/controller/dual_trainer.py:557 @exception_handled).
 *
 * Reference interface each group replaces (paths relative to the reference):
 *   srmi_param_*, srmi_engine_*  -> sres/model/manager.py:93-96 get_model plugin
 *                                   + sres/model/common/common.py:22-48 FModule
 *   srmi_forward                 -> RCAN.forward sres/model/rcan/network.py:22-27,
 *                                   EDSR.forward sres/model/edsr/network.py:27-32
 *   srmi_backward                -> autograd of the above (dual_trainer.py:322)
 *   srmi_rmse_*, srmi_loss_*     -> l2loss sres/controller/stats.py:5-8
 *   srmi_charbonnier_partial     -> ModelTrainer.charbonnier dual_trainer.py:196-198
 *   srmi_downsample/_upsample    -> sres/base/util/array.py:72-76 / :84-87
 *   srmi_interpolate             -> the same with torch_interp_mode, array.py:37-41
 *   srmi_adam_step               -> torch.optim.Adam, dual_trainer.py:126,323
 *   srmi_conv3x3* / srmi_wgrad*  -> nn.Conv2d of default_conv
 *                                   sres/model/common/cnn.py:8-9 (op level)
 *   srmi_ca_*                    -> CALayer sres/model/rcan/network.py:31-47
 *   srmi_region_to_tiles         -> get_tiles + 'lnorm' norm
 *                                   sres/base/source/swot/raw.py:216-233, :169-181
 *   srmi_batch_prep              -> norm 'lnorm' (swot/raw.py:169-181) + xyflip
 *                                   sres/base/source/batch.py:37-49 + downsample
 *   srmi_llc_*, srmi_tiles_*     -> SWOTRawDataLoader.load_file + get_tiles
 *                                   sres/base/source/swot/raw.py:133-145, :216-233
 *   srmi_tiles_to_region         -> denorm + assemble_images
 *                                   sres/controller/dual_trainer.py:67-77, :482-512
 */
#ifndef SRMI_H
#define SRMI_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRMI_OK 0
#define SRMI_ERR_ARG (-10001)
#define SRMI_ERR_SHAPE (-10002)
#define SRMI_ERR_WORKSPACE (-10003)
#define SRMI_ERR_UNSUPPORTED (-10004)

#define SRMI_ARCH_RCAN 0
#define SRMI_ARCH_EDSR 1

/* operand type of the engine (srmi_model_config.dtype, and the op-level entry
 * points' dtype argument):
 *   SRMI_DTYPE_BF16: activations / gradient maps / filter packs in bf16, fp32
 *     accumulation (v_mfma_f32_16x16x32_bf16), fp32 residual stream and master
 *     weights -- BASELINE configs 2, 3, 5;
 *   SRMI_DTYPE_F32: everything fp32, exact f32 MFMA (v_mfma_f32_16x16x4_f32) --
 *     the reference's own arithmetic (array2tensor fp32, sres/base/util/array.py:70;
 *     nn.Conv2d fp32, sres/model/common/cnn.py:8-9), BASELINE config 4. */
#define SRMI_DTYPE_BF16 0
#define SRMI_DTYPE_F32 1

typedef struct srmi_model_config {
  int arch;          /* SRMI_ARCH_RCAN | SRMI_ARCH_EDSR                     */
  int nchannels_in;  /* len(task.input_variables)   (1..4)                  */
  int nchannels_out; /* len(task.target_variables)  (1..4)                  */
  int nfeatures;     /* model.nfeatures (64)                                */
  int nlayers;       /* RCAN residual groups / EDSR resblocks               */
  int nblocks;       /* RCAN RCABs per group (ignored for EDSR)             */
  int reduction;     /* RCAN model.cbottleneck (channel-attention reduction): 64 / reduction
                        in 4 .. 32 and a multiple of 4 (else SRMI_ERR_UNSUPPORTED) */
  int scale;         /* prod(model.downscale_factors): 2, 4 or 8            */
  float res_scale;   /* EDSR model.res_scale                                */
  int batch;         /* max tiles per call (workspace capacity)             */
  int lr_h, lr_w;    /* LR tile size, e.g. 48 x 48                          */
  int cu_budget;     /* CUs one launch should fill (0 = the whole GPU); two
                        engines on two streams each take half the chip     */
  int dtype;         /* SRMI_DTYPE_BF16 | SRMI_DTYPE_F32                    */
  int flags;         /* SRMI_FLAG_* (0 = defaults)                           */
} srmi_model_config;
/* flags (bits 0 and 3 are retired: the CA-backward fold and the separate CA-scale
 * launch, both measured slower on MI355X and removed) */
/* SRMI_FLAG_NO_RCAB_INFER: inference engines run each RCAB as three launches (conv1,
 * conv2 + pool, CA) instead of one launch with a workgroup per image (A/B, tests) */
#define SRMI_FLAG_NO_RCAB_INFER 2
/* training forward (A/B, tests): SRMI_FLAG_CA_PASS runs each RCAB's channel attention as
 * a pass of its own after conv2 (conv1, conv2 + pool writing u, CA pass) instead of inside
 * conv2's launch */
#define SRMI_FLAG_CA_PASS 4
/* training backward (A/B, tests): SRMI_FLAG_DU_PASS has the CA backward write du = g s +
   dm / HW to memory for the conv2 backward to read (round 6), instead of the fused conv2
   backward forming du from the bf16 gradient stream in LDS (the same values, bit for bit) */
#define SRMI_FLAG_DU_PASS 16

typedef struct srmi_param_info {
  long long offset; /* element offset in the flat fp32 parameter buffer     */
  long long numel;
  int ndim;
  int shape[4];
} srmi_param_info;

typedef struct srmi_engine srmi_engine;

int srmi_version(void);

/* parameters, in state_dict order (identical keys to the reference model) */
int srmi_param_count(const srmi_model_config* cfg, long long* n_params, int* n_tensors);
int srmi_param_table(const srmi_model_config* cfg, srmi_param_info* out, int cap);

/* workspace for `train` (saves activations) or inference */
int srmi_workspace_size(const srmi_model_config* cfg, int train, size_t* bytes);
int srmi_engine_create(const srmi_model_config* cfg, void* workspace, size_t ws_bytes, int train,
                       srmi_engine** out);
int srmi_engine_destroy(srmi_engine* e);

/* fp32 master weights -> MFMA filter packs of the engine's dtype (call after every update) */
int srmi_pack_weights(srmi_engine* e, const float* params, void* stream);

/* lr: NCHW fp32 [n][Cin][lr_h][lr_w] -> sr: NCHW fp32 [n][Cout][lr_h*s][lr_w*s] */
int srmi_forward(srmi_engine* e, const float* params, const float* lr, float* sr, int n, void* stream);

/* backward of the last forward (train engines).  Either
 *   dy != NULL : upstream gradient NCHW fp32 like sr, or
 *   dy == NULL : RMSE gradient (sr - hr) * loss4[2] formed on the fly.
 * Writes every parameter gradient into grads (flat, state_dict order).
 * One event per residual group is recorded into group_events[g] (if not NULL,
 * hipEvent_t*) as soon as that group's gradients are final -- the hook for
 * bucketed all-reduce overlapped with the rest of backward. */
int srmi_backward(srmi_engine* e, const float* params, const float* lr, const float* sr, const float* hr,
                  const float* loss4, const float* dy, float* grads, void** group_events, void* stream);

/* the same backward in stages, so that a caller can enqueue work between them (a
 * residual group's gradient all-reduce right behind that group, srmi.trainer): stages
 * 0 = tail conv, upsamplers and body tail; 1 .. nlayers = residual groups nlayers-1 ..
 * 0; nlayers + 1 = head (RCAN; EDSR has one stage).  srmi_backward_stages runs stages
 * first .. last (in order, each exactly once per backward); group_events as above.
 * The engine tracks the next stage: `first` must be it (0 after a forward or a
 * completed backward), else SRMI_ERR_ARG and nothing is enqueued; srmi_backward is
 * refused while a staged backward is half-way through. */
int srmi_backward_stage_count(srmi_engine* e);
int srmi_backward_stages(srmi_engine* e, const float* params, const float* lr, const float* sr, const float* hr,
                         const float* loss4, const float* dy, float* grads, void** group_events, int first, int last,
                         void* stream);

/* diagnostic (bench roofline): re-issue `reps` times on `stream` the fused backward
 * launch of RCAB (0, 2) exactly as srmi_backward issues it (same shapes, CU split,
 * row chunks) -- which = 1: dgrad of conv1 accumulating into the gradient stream
 * (+ CA sums) beside conv1's filter gradient; which = 2: the ReLU-mask dgrad of
 * conv2 beside conv2's filter gradient -- on the buffers of the last backward
 * (their contents are overwritten).  RCAN train engines; which = 3: an RCAN
 * inference engine's one-launch RCAB (0, 2) on the buffers of the last forward;
 * which = 4 (nothing launched, reps ignored): 1 if the engine's backward runs the CA
 * backward inside the fused conv2 backward (du formed from the bf16 gradient stream),
 * 0 if as a launch of its own (SRMI_FLAG_DU_PASS, exact fp32, unfusable shapes). */
int srmi_engine_probe(srmi_engine* e, int which, int reps, void* stream);

/* RMSE (l2loss, squared=False).  loss4[0] = sum of squares (this rank),
 * loss4[1] = global element count; after the optional all-reduce of loss4[0],
 * srmi_rmse_finalize sets loss4[3] = L = sqrt(S/count), loss4[2] = 1/(count L). */
int srmi_rmse_partial(srmi_engine* e, const float* pred, const float* target, size_t n, double count_global,
                      float* loss4, void* stream);
int srmi_rmse_finalize(float* loss4, void* stream);

/* Charbonnier loss (model.loss_fn 'charbonnier', ModelTrainer.charbonnier
 * sres/controller/dual_trainer.py:196-198): loss4[0] = sum sqrt(d^2 + eps) (this
 * rank), loss4[1] = count_global; dy (optional, like pred) = d / sqrt(d^2 + eps) /
 * count_global -- the upstream gradient srmi_backward takes.  Finalise with
 * srmi_loss_finalize(loss4, SRMI_LOSS_MEAN): loss4[3] = loss4[0] / loss4[1].
 * loss4 NULL (dy required): dy only, no loss sums (the trainer takes the loss from
 * srmi_tile_loss_parts). */
#define SRMI_LOSS_RMSE 0
#define SRMI_LOSS_MEAN 1
int srmi_charbonnier_partial(srmi_engine* e, const float* pred, const float* target, size_t n, double count_global,
                             float eps, float* loss4, float* dy, void* stream);
int srmi_loss_finalize(float* loss4, int kind, void* stream);
/* per-batch losses of process_image / evaluate (dual_trainer.py:417-446, :509-532):
 * pred/target [ntiles][tile_elems] scored in batches of batch_size tiles (the last
 * one may be short), loss of a batch over all its elements (kind RMSE or MEAN =
 * Charbonnier with eps); out[0] = mean of the batch losses, out[1 + b] = batch b's
 * loss (at most 1024 batches); work: ntiles floats */
int srmi_batch_losses(const float* pred, const float* target, int ntiles, long long tile_elems, int batch_size,
                      int kind, float eps, float* work, float* out, void* stream);
/* the second half of srmi_batch_losses on per-tile sums already formed (its `work`
 * output, e.g. gathered from the ranks of a multi-rank tiled inference, srmi.inference):
 * out[0] = mean of the batch losses, out[1 + b] = batch b's loss, the same arithmetic
 * (process_image's np.array(batch_losses).mean(), dual_trainer.py:443-446) */
int srmi_batch_loss_means(const float* sums, int ntiles, long long tile_elems, int batch_size, int kind, float* out,
                          void* stream);
/* loss sums that do not depend on how a batch is split over calls / micro-batch
 * engines: srmi_tile_loss_parts writes parts[ntiles][16] (per tile, 16 fixed slices,
 * fixed reduction order; kind RMSE: (p - t)^2, MEAN: sqrt((p - t)^2 + eps)) -- each
 * call writes its tiles' rows of one batch-wide array; srmi_loss_from_parts then sums
 * the ntiles x 16 parts in order (fp64) into loss4 ([0] = S, [1] = count_global) and
 * finalises it as `kind` (-1: not finalised, before a data-parallel all-reduce) */
int srmi_tile_loss_parts(const float* pred, const float* target, int ntiles, long long tile_elems, int kind,
                         float eps, float* parts, void* stream);
int srmi_loss_from_parts(const float* parts, int ntiles, double count_global, int kind, float* loss4, void* stream);
/* loss4 = the sum over nparts micro-batch records parts4[k][4] (S summed in a fixed
 * order, the count of part 0), then finalised as `kind` (-1: not finalised, e.g.
 * before a data-parallel all-reduce of loss4[0]) */
int srmi_loss_combine(float* loss4, const float* parts4, int nparts, int kind, void* stream);

/* interp baseline / data path */
int srmi_downsample(const float* hr, int N, int C, int H, int W, int scale, float* lr, void* stream);
int srmi_upsample(const float* lr, int N, int C, int h, int w, int scale, float* hr, void* stream);
/* torch.nn.functional.interpolate(x, scale_factor=f, mode) with align_corners=False,
 * any factor: the downsample / upsample of array.py:72-76 / :84-87 under
 * task.downsample_mode / upsample_mode (torch_interp_mode, array.py:37-41: 'linear'
 * -> SRMI_INTERP_BILINEAR, 'cubic' -> SRMI_INTERP_BICUBIC) and data_downsample's
 * factors (dual_trainer.py:561-563).  x NCHW [N][C][H][W] -> y [N][C][Ho][Wo] with
 * Ho = floor(H f), Wo = floor(W f) chosen by the caller and rh = rw = (float)(1 / f),
 * the source-coordinate scale ATen uses (UpSample.h area_pixel_compute_scale) */
#define SRMI_INTERP_BILINEAR 1
#define SRMI_INTERP_BICUBIC 2
int srmi_interpolate(const float* x, int N, int C, int H, int W, int Ho, int Wo, float rh, float rw, int mode, float* y,
                     void* stream);

/* Adam on flat buffers, step counted from 1 */
int srmi_adam_step(float* p, const float* g, float* m, float* v, size_t n, int step, float lr, float beta1,
                   float beta2, float eps, float weight_decay, void* stream);

/* y += a * x (flat fp32; sums micro-batch gradients) */
int srmi_axpy(float* y, const float* x, float a, size_t n, void* stream);

/* ---- op-level entry points (kernel parity tests, custom graphs) ---------- */
/* dtype: SRMI_DTYPE_BF16 (x / yb / aux / packs bf16) or SRMI_DTYPE_F32 (fp32) */
/* forward conv: x NHWC [N][H][W][Cin], packed filters (srmi_pack_conv),
 * epi: 0 relu, 1 + channel sums (part[N][strips][64]), 2 alpha*(y+b)+r1
 * -> yf fp32 (opt) + yb, 3 PixelShuffle(2), 4 dgrad * (aux > 0), 5 dgrad + r1 + r2
 * + r3 -> yf (+ sums of g, g*aux), 6 plain (+ bias).  (The engine's own epilogues
 * 7-13 -- the CA forward, the bf16 in-group gradient stream -- take operands this
 * entry point does not pass; they are reached through srmi_forward / _backward.)  */
int srmi_conv3x3(const void* x, const void* wpack, const float* bias, int N, int H, int W, int Cin, int Cout,
                 int in_unshuffle, int epi, void* yb, float* yf, const float* r1, const float* r2, const float* r3,
                 const void* aux, float* part, float alpha, int dtype, void* stream);
int srmi_conv3x3_nstrips(int H, int W);
/* diagnostic: record s_memtime phase stamps of the Cin=64 conv kernel into buf
 * (64 x u64 per workgroup); NULL turns it off */
int srmi_debug_conv_stamps(void* buf);
int srmi_debug_wgrad_stamps(void* buf);
/* fp32 torch filter [Cout][Cin][3][3] -> packs of dtype: fwd [Cin/64][9][Cout][64],
 * dgrad [Cout/64][9][Cin][64] (flipped), bias [Cout]; ps != 0 permutes the
 * PixelShuffle channel order (packed c'' = 64q + c <- torch 4c + q)         */
int srmi_pack_conv(const float* w, const float* b, int Cout, int Cin, int ps, void* fpack, void* dpack, float* pbias,
                   int dtype, void* stream);
/* filter + bias gradient of a 3x3 conv (nn.Conv2d backward, weight half):
 * x NHWC [N][H][W][64], dy NHWC [N][H][W][Cout] (or, dy_unshuffle,
 * the PixelShuffle output [N][2H][2W][64] with Cout = 256); slab: workspace of
 * N*rs*Cout*577 floats; gw torch layout [Cout][64][3][3], gb [Cout] (both NULL:
 * leave the per-chunk partial slabs, skip the reduction) */
int srmi_wgrad3x3(const void* x, const void* dy, int N, int H, int W, int Cout, int dy_unshuffle, int row_splits,
                  float* slab, size_t slab_bytes, int ps, float alpha, float* gw, float* gb, int dtype, void* stream);
int srmi_ca_forward(const void* u, const float* part, int nstrips, const float* w1, const float* b1, const float* w2,
                    const float* b2, int N, int HW, int C, int R, const float* h_in, float* h_out, void* hb_out,
                    float* rec, int dtype, void* stream);
/* the same CALayer forward on the bf16 engine's residual-stream pair: h = h_in
 * (fp32, when non-NULL) or the pair hi_in (bf16) + lo_in (int8 remainder); out, for
 * the fp32 bit pattern A of h + s*u: hi = (A + 0x8000) >> 16 (bf16, rounded half away
 * from zero), lo = byte 1 of A; the pair's value has the bits ((hi << 16) | 0x80) +
 * (sext8(lo) << 8), i.e. h + s*u to within 128 fp32 steps (16 significant bits) (in
 * place allowed: lo_out == lo_in) */
int srmi_ca_forward_pair(const void* u, const float* part, int nstrips, const float* w1, const float* b1,
                         const float* w2, const float* b2, int N, int HW, int C, int R, const float* h_in,
                         const void* hi_in, const void* lo_in, void* hi_out, void* lo_out, float* rec, void* stream);
/* brec: N*(2C + C/R) floats (dz2 | dz1 | conv2 bias grad per image) followed by
 * N*C floats of dm (gradient of the pooled mean) -- N*(3C + C/R) in total */
int srmi_ca_backward(const float* g, const float* part, int nstrips, const float* rec, const float* w1,
                     const float* w2, int N, int HW, int C, int R, void* du, float* brec, int dtype, void* stream);
int srmi_head_forward(const float* lr, const float* w, const float* b, int N, int C, int H, int W, float* x0f,
                      void* x0b, int dtype, void* stream);
int srmi_tail_forward(const void* x, const float* w, const float* b, int N, int C, int H, int W, float* y, int dtype,
                      void* stream);

/* ---- tiled-region inference data path --------------------------------- */
/* region [C][H][W] fp32 -> floor grid gy = H/ty, gx = W/tx; tiles
 * [gy*gx][C][ty][tx] normalised per tile and channel ((x - mean) / std over the
 * tile, ddof 0); mean/std [gy*gx][C]; bad[gy*gx] (optional) = 1 where the tile
 * holds a non-finite value (the reference drops those tiles) */
int srmi_region_to_tiles(const float* region, int C, int H, int W, int ty, int tx, float* tiles, float* mean,
                         float* std, int* bad, void* stream);
/* tiles [n][C][ty][tx] -> out [C][gy*ty][gx*tx]: x * std + mean (mean == NULL:
 * no denorm); inv[gy*gx] = tile index of each grid cell or -1 (NaN cell);
 * inv == NULL: tile i is cell i */
int srmi_tiles_to_region(const float* tiles, const float* mean, const float* std, const int* inv, int C, int ty,
                         int tx, int gy, int gx, float* out, void* stream);

/* ---- training batch preparation ------------------ */
/* raw [B][C][T][T] fp32 tiles (select_batch, sres/base/source/swot/raw.py:160-166)
 * -> hr [B][C][T][T] = xyflip(lnorm(raw)) (norm 'lnorm' raw.py:169-181: per tile
 * and channel (x - mean) / std, ddof 0; xyflip sres/base/source/batch.py:37-49
 * with the drawn flip_index 0..7), lr [B][C][T/scale][T/scale] = downsample(hr)
 * (array.py:72-76; NULL: skipped), mean/std [B][C] (norm's ncstats attrs; NULL:
 * skipped).  T even. */
int srmi_batch_prep(const float* raw, int B, int C, int T, int flip_index, int scale, float* hr, float* lr,
                    float* mean, float* std, void* stream);

/* ---- on-disk LLC4320 source -> tiles --------------- */
/* Replaces SWOTRawDataLoader.load_file (sres/base/source/swot/raw.py:133-145):
 * template_be = the raw bytes of the '>f4' mask template (13 nx^2 words, 0 =
 * land), data_be = the raw bytes of a '>f4' wet-value file.  The index map of
 * the ROI [y0, y0+ys) x [x0, x0+xs) of the east | west.T[::-1] image (mds2d,
 * swot/util.py:3-7; subset_roi raw.py:38-45) is built once per template:
 * idx_map[ys*xs] = wet-value index or -1; *n_wet (device) = wet cell count.
 * workspace: srmi_llc_index_map_workspace bytes (n_template int32 ranks + scan). */
int srmi_llc_index_map_workspace(long long n_template, size_t* bytes);
int srmi_llc_index_map(const void* template_be, long long n_template, int nx, int y0, int ys, int x0, int xs,
                       int* idx_map, long long* n_wet, void* workspace, size_t workspace_bytes, void* stream);
/* out[p] = decoded data[idx_map[p]], NaN for land: one time slice of one variable */
int srmi_llc_gather(const void* data_be, long long n_values, const int* idx_map, long long npix, float* out,
                    void* stream);
/* get_tiles (raw.py:216-233): bad[c*gy*gx + t] = 1 where tile t of channel c of
 * region [C][H][W] holds a non-finite value (floor grid gy = H/ty, gx = W/tx) */
int srmi_tiles_nonfinite(const float* region, int C, int H, int W, int ty, int tx, int* bad, void* stream);
/* out[m] (ty x tx plane m of the [n/C][C][ty][tx] result) = tile plane src[m]
 * (= c*gy*gx + t of the channel-major flattening) */
int srmi_tiles_gather(const float* region, int C, int H, int W, int ty, int tx, const int* src, int nslots,
                      float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SRMI_H */
