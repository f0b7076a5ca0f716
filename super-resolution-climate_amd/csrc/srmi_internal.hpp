// Internal (C++) interface between the kernel translation units and the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/srmi.h"
#include "tuning.hpp"

namespace srmi {

typedef uint16_t bf16_t;

enum InMode { IN_PLAIN = 0, IN_UNSHUF = 1 };

enum Epi {
  EPI_RELU_BF16 = 0,   // y = relu(acc + b)                       -> bf16
  EPI_POOL_BF16 = 1,   // y = acc + b  (+ per-strip channel sums)   -> bf16
  EPI_RESID = 2,       // y = alpha*(acc + b) + r1                  -> fp32 (opt) + bf16
  EPI_PS_BF16 = 3,     // y = acc + b, PixelShuffle(2) scatter      -> bf16 [2H][2W][64]
  EPI_DG_RELUMASK = 4, // dz = acc * (aux > 0)                      -> bf16
  EPI_DG_ACC = 5,      // g = acc + r1 + r2 + r3 (+ sums of g, g*aux) -> fp32 + bf16; r1 may be the
                       // bf16 r1b instead, and yf may be null (bf16 yb only: the sums then use
                       // the rounded bf16 g, the stream's stored value)
  EPI_PLAIN_BF16 = 6,  // y = acc (+ b)                              -> bf16
  EPI_DG_ACC_CA = 7,   // g = acc + r1, sums of g and g*aux; r1/aux/part non-null, no yb/r2/r3
                       // (the hot RCAB case of EPI_DG_ACC, specialised: no runtime operand checks)
  // the inference RCAB (rcab_infer.hip), 64-channel non-deferred body only:
  EPI_RELU_POOL = 8,   // t = relu(acc + b) -> bf16, + per-strip channel sums of t
  EPI_CA_RESID = 9,    // h' = h + s[c] (acc + b): h in as fp32 r1 or the pair r1h / r1l,
                       // h' out as the pair yph / ypl, s = escale[n * escale_stride + c]
  // the training RCAB's conv2 (the CA forward without a pass of its own):
  EPI_CA_RESID_U = 10, // u = acc + b -> bf16 yb (saved for backward), h' = h + s[c] bf16(u) as
                       // in EPI_CA_RESID; s computed after the first strip's MFMAs (cas_on,
                       // ca_scale.hpp: from conv1's partial means, or from t) or read from escale
  // the bf16 engine's in-group gradient stream (the hot RCAB conv1 dgrad, F1):
  EPI_DG_ACC_CA16 = 11, // g = bf16(acc + r1b) -> bf16 yb (in place over r1b allowed), sums of
                        // that bf16 g and g*aux; r1b / aux / part / yb non-null, no yf / r1 / r2 / r3
  EPI_DG_CA16 = 12,     // the same without r1b: g = bf16(acc) (the group tail's dgrad starts the stream)
  EPI_DG_ACC_G1 = 13,   // the group's first RCAB (the stream's end): g = acc + r1b + r2 (+ r3) -> fp32 yf
                        // + its bf16 copy yb (in place over r1b allowed); no CA sums
};

// The CA scale of an RCAB from its conv1 output t (ca_scale.hpp): mean(u) of u =
// conv2(t) + b2 from t's statistics and conv2's bf16 filter image, then the MLP.
struct CaScale {
  const bf16_t* t;    // conv1 output [N][H][W][64] bf16
  const float* part;  // conv1's per-strip channel sums of t [N][nstrips][64] (EPI_RELU_POOL)
  int nstrips;
  const float *w1, *b1, *w2, *b2;  // conv_du.0 [CR][64] + [CR], conv_du.2 [64][CR] + [64]
  const float* bc2;   // conv2's bias [64]
  int CR;
  float* rec;         // out: m | z1 | s per image [N][128 + CR]
  unsigned long long* stamps;  // diagnostic build only: phase stamps of ca_scale_finish (null)
  // Partial means (training, SRMI_CA_MPART): conv1 (EPI_RELU_POOL with cas_on) writes, per
  // workgroup (run) of an image, the matvec of its rows' share of S_tap (ca_matvec) into
  // mpart [N][nruns][64]; conv2 then sums them instead of computing the scale from t.
  float* mpart;
  int nruns;           // workgroups per image of conv1's launch (conv64_runs_per_image)
  const bf16_t* wimg;  // conv2's packed bf16 filter image (conv1 loads it for the matvec)
};

// The CALayer backward of an RCAB (reference network.py:31-47, 61-64) as the fused conv2
// backward runs it (ca_bwd.hpp): the MLP backward of each image from the producer's
// per-strip sums, then du = bf16(g s[c] + dm[c] / HW) formed from the bf16 gradient stream
// g on the launch's input rings in LDS (null rec = off: x / dy is read as it is)
struct CaBwdIn {
  const float* part;   // sum_p g | sum_p g u per strip [N][nstrips][128] (F1's CA sums)
  int nstrips;
  const float* rec;    // the forward record m | z1 | s [N][128 + CR]
  const float* w1;     // conv_du.0 weight [CR][64]
  const float* w2;     // conv_du.2 weight [64][CR]
  int CR;
  float* brec;         // out, one workgroup per image: dz2 | dz1 | dbconv2 [N][128 + CR], then dm [N][64]
  int N;
  float inv_hw;        // 1 / (H W)
  int mlp;             // 1: every workgroup runs its image's MLP (ca_bwd_mlp; the first dgrad run
                       // of the image writes brec); 0: s and dm are read (rec, brec: an MLP launch ran)
};

struct ConvParams {
  const bf16_t* x;     // input (logical NHWC [N][H][W][Cin])
  const bf16_t* w;     // packed filters [Cin/64][9][Cout][64]
  const float* bias;   // [Cout] packed order (may be null for dgrad)
  int N, H, W, Cin, Cout;
  int in_mode;
  bf16_t* yb;          // bf16 output
  float* yf;           // fp32 output
  const float* r1;
  const bf16_t* r1b;   // (DG_ACC_CA16, DG_ACC) the gradient-stream operand in bf16 instead of r1
  const float* r2;
  const float* r3;
  const bf16_t* aux;   // relu output t (RELUMASK) / CA input u (DG_ACC sums)
  float* part;         // per-strip channel sums
  int part_stride;
  float alpha;
  const void* zeros;   // >= 16 zero bytes in global memory (DMA padding source)
  unsigned long long* stamps;  // diagnostic s_memtime stamps (null in production)
  int cu_budget;               // CUs a launch should fill (0 = all 256)
  int f32;                     // exact-fp32 mode: x, w, yb, aux point at fp32 data
                               // (the bf16_t* fields are plain addresses then)
  // EPI_CA_RESID: the residual stream as the pair (bf16 hi + lo8 remainder, common.hpp)
  const bf16_t* r1h;
  const uint8_t* r1l;
  bf16_t* yph;
  uint8_t* ypl;
  const float* escale;         // per-image channel scale s [N][escale_stride]
  int escale_stride;
  // EPI_CA_RESID_U with cas_on: every workgroup computes its image's s in the prologue
  // (and the first one of the image writes cas.rec); cas_on = 0: s from escale
  CaScale cas;
  int cas_on;
  // (EPI_DG_RELUMASK, the deferred 8-wave body) x is the bf16 gradient stream g and the
  // conv reads the CALayer backward's du formed from it on the input ring (CaBwdIn)
  CaBwdIn gx;
};

void conv3x3_set_debug_stamps(unsigned long long* buf);
unsigned long long* conv3x3_debug_stamps();  // (null unless a diagnostic run set it)
unsigned long long* conv3x3_stamps_for(int epi);  // (diagnostic build: SRMI_STAMP_EPI selects one epilogue)
int conv3x3_launch(const ConvParams& p, int epi, hipStream_t st);  // dispatches p.f32
int conv3x3_f32_launch(const ConvParams& p, int epi, hipStream_t st);
int conv3x3_nstrips(int H, int W);
int conv64_runs_per_image(const ConvParams& p);  // workgroups per image of a 48-wide v2 launch

struct ReduceSet {  // one slab reduction: slabs -> torch-layout dW (and db)
  const float* slab;   // (slab16: bf16 slabs at this address)
  const float* bslab;
  int nslab, Cout, ps, layout;
  float alpha;
  float* gw;
  float* gb;
  int slab16;          // the weight slabs are bf16 (WgradParams.slab16); the bias slabs stay fp32
};

// weight gradient of a 3x3 conv: slab[s][Cout][9][64] + bias slab[s][Cout]
struct WgradParams {
  const bf16_t* x;     // forward input NHWC [N][H][W][64]
  const bf16_t* dy;    // output grad: plain [N][H][W][Cout] or PS [N][2H][2W][64] (Cout = 256)
  int N, H, W, Cout;
  int dy_mode;         // IN_PLAIN / IN_UNSHUF
  int imgs_per_wg;     // images per workgroup
  int row_splits;      // H split into this many row groups
  float* slab;         // [nslab][Cout][9][64]
  float* bslab;        // [nslab][Cout]
  const void* zeros;   // >= 16 zero bytes in global memory (DMA source for padding)
  unsigned long long* stamps;  // diagnostic (null in production)
  int f32;             // exact-fp32 mode: x, dy point at fp32 data
  int slab16;          // (wgrad48 body) weight slabs stored as bf16 at `slab` (the RCAB filter
                       // gradients of the bf16 engine: half the slab bytes); bias slabs fp32
  // (wgrad48 body, IN_PLAIN, Cout == 64) dy is g and the filter gradient takes du formed
  // from it in LDS, as ConvParams.gx
  CaBwdIn gx;
};
void wgrad3x3_set_debug_stamps(unsigned long long* buf);
int wgrad3x3_launch(const WgradParams& p, hipStream_t st);  // dispatches p.f32
int wgrad_f32_launch(const WgradParams& p, hipStream_t st);
int wgrad3x3_nslabs(const WgradParams& p);
// order of the partial slabs the launch writes: 0 = [tap][ci][Cout], 1 = wgrad48's
// MFMA-native [Cout/64][wave][9][4][lane][4]
int wgrad3x3_slab_layout(const WgradParams& p);
// slab reduction into the torch-layout grad [Cout][64][3][3] (+ bias [Cout]);
// ps != 0 un-permutes the packed PixelShuffle channel order (c'' = 64q + c -> 4c + q)

int wgrad_reduce2_launch(const ReduceSet& r0, const ReduceSet& r1, hipStream_t st);
// n independent slab reductions (equal Cout) in one launch (blockIdx.y selects the set)
int wgrad_reduce_sets_launch(const ReduceSet* sets, int n, hipStream_t st);
// fused RCAB backward launch: dgrad conv (epi RELUMASK / DG_ACC_CA / DG_ACC, its runs
// sized for conv_cus CUs) beside the filter gradient wp of the same conv (wgrad48)
int rcab_bwd_fusable(const ConvParams& cp, const WgradParams& wp);
int rcab_bwd_launch(const ConvParams& cp, int epi, int conv_cus, const WgradParams& wp, hipStream_t st);
// the fused conv2 backward (EPI_DG_RELUMASK) of this build forms du from g (ConvParams gx_*)
bool rcab_bwd_du_from_g();
int wgrad_reduce_launch(const float* slab, const float* bslab, int nslab, int Cout, int ps, int layout, float alpha,
                        float* gw, float* gb, hipStream_t st, int slab16 = 0);

// small-channel kernels (head / tail), bicubic resampling, loss, CA, Adam, packing
// f32 != 0: the operand-type outputs / inputs below are fp32 (exact-fp32 engine mode)
int head_fwd_launch(const float* lr, const float* w, const float* b, int N, int C, int H, int W, float* x0f,
                    void* x0b, int f32, hipStream_t st);
int head_wgrad_launch(const float* lr, const float* g, int N, int C, int H, int W, float* slab, int* nslab,
                      hipStream_t st);
int head_wgrad_reduce_launch(const float* slab, int nslab, int C, float* gw, float* gb, hipStream_t st);

int tail_fwd_launch(const void* x, const float* w, const float* b, int N, int C, int H, int W, float* y, int f32,
                    hipStream_t st);
// dy is formed on the fly: dy = (y - hr) * scale, scale from loss[2]
int tail_dgrad_launch(const float* y, const float* hr, const float* loss, const float* w, int N, int C, int H,
                      int W, void* dx, int f32, hipStream_t st);
int tail_wgrad_launch(const float* y, const float* hr, const float* loss, const void* x, int N, int C, int H,
                      int W, float* slab, int* nslab, int f32, hipStream_t st);
int tail_wgrad_reduce_launch(const float* slab, int nslab, int C, float* gw, float* gb, hipStream_t st);

int downsample_launch(const float* hr, int N, int C, int H, int W, int scale, float* lr, hipStream_t st);
int upsample_launch(const float* lr, int N, int C, int h, int w, int scale, float* hr, hipStream_t st);
int interp_launch(const float* x, int N, int C, int H, int W, int Ho, int Wo, float rh, float rw, int mode, float* y,
                  hipStream_t st);
// loss[0] = sum (y-t)^2 (this rank), loss[1] = element count (global after all-reduce)
int sqerr_partial_launch(const float* y, const float* t, size_t n, float* partial, int nblk, hipStream_t st);
int sqerr_finish_launch(const float* partial, int nblk, double count, float* loss, hipStream_t st);
enum LossKind { LOSS_RMSE = 0, LOSS_MEAN = 1 };
int loss_finalize_launch(float* loss, int kind, hipStream_t st);
int loss_combine_launch(float* loss, const float* parts, int nparts, int kind, hipStream_t st);
int batch_losses_launch(const float* y, const float* t, int ntiles, long long tile_elems, int bs, int kind, float eps,
                        float* work, float* out, hipStream_t st);
int batch_loss_means_launch(const float* sums, int ntiles, long long tile_elems, int bs, int kind, float* out,
                            hipStream_t st);
// split-invariant loss sums (small.hip): parts[tile][kTileSub] of every tile, then S in
// fixed order (fp64) into loss4, finalised as kind (>= 0)
constexpr int kTileSub = 16;
int tile_loss_parts_launch(const float* y, const float* t, int ntiles, long long tile_elems, int kind, float eps,
                           float* parts, hipStream_t st);
int loss_from_parts_launch(const float* parts, int nparts, double count, int kind, float* loss, hipStream_t st);
int charb_partial_launch(const float* y, const float* t, size_t n, float eps, double count, float* dy,
                         float* partial, int nblk, hipStream_t st);

// channel attention
// residual stream: fp32 h_in / h_out, or (bf16 engine) as a bf16 hi + lo pair: lo_out
// non-null -> hi goes to hb_out, lo to lo_out; input from h_in (fp32) or, h_in null,
// from the pair hi_in + lo_in
int ca_fwd_launch(const void* u, const float* part, int nstrips, const float* w1, const float* b1,
                  const float* w2, const float* b2, int N, int HW, int C, int R, const float* h_in, float* h_out,
                  void* hb_out, float* rec, int f32, hipStream_t st, const void* hi_in = nullptr,
                  const void* lo_in = nullptr, void* lo_out = nullptr);
// red0/red1 (both or neither): two slab reductions carried in the same launch
// g: fp32, or (g16) the bf16 engine's in-group gradient stream in bf16
int ca_bwd_du_launch(const void* g, int g16, const float* part, int nstrips, const float* rec, const float* w1,
                     const float* w2, int N, int HW, int C, int R, void* du, float* brec, int f32, hipStream_t st,
                     const ReduceSet* red0 = nullptr, const ReduceSet* red1 = nullptr);
// inference RCAB, one launch with a workgroup per image (rcab_infer.hip): c1 = conv1
// (yb = t), c2 = conv2 (its bias = the CA's bc2); t's per-strip sums into part, the CA
// scale into rec, h' = h + s u into the pair hi_out / lo_out (h from h_in or the pair)
int rcab_infer_launch(const ConvParams& c1, const ConvParams& c2, const float* part, int nstrips, const float* w1,
                      const float* b1, const float* w2, const float* b2, int CR, const float* h_in, const void* hi_in,
                      const void* lo_in, void* hi_out, void* lo_out, float* rec, hipStream_t st);
// records of consecutive RCABs Ncap images apart (the engine capacity), N summed
int ca_param_grads_batched_launch(const float* recs, const float* brecs, int nblocks, int N, size_t rstride,
                                  size_t bstride, int C, int R, const long long* offs, float* grads, hipStream_t st);

int adam_launch(float* p, const float* g, float* m, float* v, size_t n, float lr, float b1, float b2, float eps,
                float wd, float step_size, float bc2_sqrt, hipStream_t st);

struct PackEntry {
  long long w_off;   // offset of the fp32 weight [Cout][Cin][3][3] in the param buffer
  long long b_off;   // offset of the fp32 bias [Cout]
  long long f_off;   // offset (elements) of the forward pack in the bf16 pack buffer
  long long d_off;   // offset of the dgrad pack
  long long pb_off;  // offset of the packed bias in the fp32 packed-bias buffer
  int Cout, Cin, ps, pad;
};
// max_cob / max_cib: the largest Cout / 64 and Cin / 64 over the entries
int pack_launch(const float* params, const PackEntry* dev_entries, int nentries, int max_cob, int max_cib,
                void* packs, float* pbias, int f32, hipStream_t st);

int pack_one_launch(const float* w, const float* b, int Cout, int Cin, int ps, void* fpack, void* dpack,
                    float* pbias, int f32, hipStream_t st);

int scale_add_launch(float* y, const float* x, float a, size_t n, hipStream_t st);

// tiled-region data path (tiles.hip)
int region_to_tiles_launch(const float* region, int C, int H, int W, int ty, int tx, float* tiles, float* mean,
                           float* stdv, int* bad, hipStream_t st);
int tiles_to_region_launch(const float* tiles, const float* mean, const float* stdv, const int* inv, int C, int ty,
                           int tx, int gy, int gx, float* out, hipStream_t st);
int llc_index_map_workspace(long long n, size_t* bytes);
int llc_index_map_launch(const uint32_t* tmpl, long long n, int nx, int y0, int ys, int x0, int xs, int* idx,
                         long long* n_wet, void* ws, size_t ws_bytes, hipStream_t st);
int llc_gather_launch(const uint32_t* data, long long nvals, const int* idx, long long np, float* out,
                      hipStream_t st);
int tiles_nonfinite_launch(const float* region, int C, int H, int W, int ty, int tx, int* bad, hipStream_t st);
int tiles_gather_launch(const float* region, int C, int H, int W, int ty, int tx, const int* src, int nslots,
                        float* out, hipStream_t st);
int batch_prep_launch(const float* raw, int B, int C, int T, int flip, int scale, float* hr, float* lr, float* mean,
                      float* stdv, hipStream_t st);

}  // namespace srmi
