// Memory-bound / small-channel kernels of the RCAN hot path on gfx950:
//  * head conv C->64 (sres/model/rcan/network.py:13) fwd + weight grad
//  * tail conv 64->C (network.py:16) fwd, data grad (with the RMSE gradient
//    formed on the fly) and weight grad
//  * bicubic 1/scale downsample (sres/base/util/array.py:72-76) and xscale
//    upsample (array.py:84-87, the interp baseline)
//  * RMSE loss partial sums (sres/controller/stats.py:5-8)
//  * channel attention forward (CALayer, network.py:31-47 + RCAB skip :61-64)
//    and backward, fused with the residual stream
//  * Adam (torch.optim.Adam defaults, dual_trainer.py:126,323)
//  * fp32 -> bf16 filter packing for the MFMA conv kernels
#include <math.h>
#include <stdlib.h>

#include "common.hpp"
#include "srmi_internal.hpp"
#include "wgrad_reduce.hpp"
#include "ca_bwd.hpp"

namespace srmi {

// =========================================================================== head
// x0[n][y][x][co] = b[co] + sum_{c,tap} lr[n][c][y+ky-1][x+kx-1] * w[co][c][tap]
// One workgroup per (image, row): lane = co, the 4 waves split the row's pixels.
// (Four rows per workgroup gave 384 workgroups at C2 -- 1.5 waves per SIMD for a
// store-bound pass: 31 us for 28 MB.)
constexpr int kHeadFwdRows = 1;
template <typename T>
__global__ void __launch_bounds__(256) head_fwd_kernel(const float* __restrict__ lr, const float* __restrict__ w,
                                                       const float* __restrict__ b, int C, int H, int W,
                                                       float* __restrict__ x0f, T* __restrict__ x0b) {
  constexpr int RB = kHeadFwdRows, HR = RB + 2;
  extern __shared__ float hs[];  // [C][HR][W+2] halo
  const int n = blockIdx.y, y0 = blockIdx.x * RB, tid = threadIdx.x;
  const int Wp = W + 2;
  float* halo = hs;
  const int hsz = C * HR * Wp;
  for (int i = tid; i < hsz; i += 256) {
    const int c = i / (HR * Wp), r = (i / Wp) % HR, xx = i % Wp;
    const int y = y0 - 1 + r, x = xx - 1;
    halo[i] = (y >= 0 && y < H && x >= 0 && x < W) ? lr[(((size_t)n * C + c) * H + y) * W + x] : 0.f;
  }
  const int co = tid & 63, grp = tid >> 6;
  float wr[36];
#pragma unroll
  for (int k = 0; k < 36; ++k) wr[k] = (k < 9 * C) ? w[co * 9 * C + k] : 0.f;
  const float bb = b[co];
  __syncthreads();
  for (int px = grp; px < RB * W; px += 4) {
    const int r = px / W, x = px - r * W;
    float s = bb;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < C) {
#pragma unroll
        for (int t = 0; t < 9; ++t)
          s += halo[(c * HR + r + t / 3) * Wp + x + t % 3] * wr[c * 9 + t];
      }
    }
    const size_t o = (((size_t)n * H + y0 + r) * W + x) * 64 + co;
    x0f[o] = s;
    x0b[o] = from_f32<T>(s);
  }
}

int head_fwd_launch(const float* lr, const float* w, const float* b, int N, int C, int H, int W, float* x0f,
                    void* x0b, int f32, hipStream_t st) {
  if (C < 1 || C > 4 || H % 4) return SRMI_ERR_SHAPE;
  const int smem = C * (kHeadFwdRows + 2) * (W + 2) * 4;
  const dim3 grid(H / kHeadFwdRows, N);
  if (f32)
    hipLaunchKernelGGL(head_fwd_kernel<float>, grid, dim3(256), smem, st, lr, w, b, C, H, W, x0f,
                       static_cast<float*>(x0b));
  else
    hipLaunchKernelGGL(head_fwd_kernel<bf16_t>, grid, dim3(256), smem, st, lr, w, b, C, H, W, x0f,
                       static_cast<bf16_t*>(x0b));
  SRMI_CHECK_LAUNCH();
  return 0;
}

// Deterministic slab reduction shared by the head / tail weight gradients:
// block = 16 outputs x 16 slab slices (slice q sums slabs q, q+16, ...), then the
// 16 slice sums are added in a fixed order.  MODE 0: head layout [co][9C+1];
// MODE 1: tail layout [c][577].
template <int MODE>
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, int nslab, int per, int C,
                                                          float* __restrict__ gw, float* __restrict__ gb) {
  __shared__ float red[16][17];
  const int oi = threadIdx.x & 15, q = threadIdx.x >> 4;
  const int o = blockIdx.x * 16 + oi;
  // 8 slabs' loads in flight per step into 8 partial sums (two at a time waited an
  // L2 latency per pair: 22 us for the 1536 tail slabs of a B=32 engine)
  float ps[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) ps[u] = 0.f;
  if (o < per) {
    int k = q;
    for (; k + 7 * 16 < nslab; k += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(size_t)(k + 16 * u) * per + o];
#pragma unroll
      for (int u = 0; u < 8; ++u) ps[u] += v[u];
    }
    for (; k < nslab; k += 16) ps[0] += slab[(size_t)k * per + o];
  }
  red[q][oi] = ((ps[0] + ps[1]) + (ps[2] + ps[3])) + ((ps[4] + ps[5]) + (ps[6] + ps[7]));
  __syncthreads();
  if (q == 0 && o < per) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][oi];
    if (MODE == 0) {
      const int nj = 9 * C + 1, co = o / nj, j = o % nj;
      if (j < nj - 1)
        gw[co * 9 * C + j] = s;
      else
        gb[co] = s;
    } else {
      const int c = o / 577, j = o % 577;
      if (j < 576)
        gw[c * 576 + j] = s;  // [c][ci][tap] == torch [C][64][3][3]
      else
        gb[c] = s;
    }
  }
}

// dW[co][c][tap] = sum_p g[p][co] * lr[c][p+off];  db[co] = sum_p g[p][co]
// One workgroup per (image, 2-row band); lane = co, the 4 waves split the band's
// pixels and each keeps ALL 9C + 1 accumulators, so every (coalesced, 256-byte)
// gradient load feeds 9C + 1 FMAs; loads are issued 4 pixels at a time.  The
// 4 waves' partials are added in LDS (fixed order) -> slab [co][9C + 1].
constexpr int kHeadRows = 2;
__global__ void __launch_bounds__(256) head_wgrad_kernel(const float* __restrict__ lr, const float* __restrict__ g,
                                                         int C, int H, int W, float* __restrict__ slab) {
  extern __shared__ float hs[];  // [C][kHeadRows + 2][W + 2], then red[4][64 * 37]
  const int n = blockIdx.y, y0 = blockIdx.x * kHeadRows, tid = threadIdx.x;
  const int co = tid & 63, wave = tid >> 6;
  const int Wp = W + 2, HR = kHeadRows + 2;
  const int hsz = C * HR * Wp;
  for (int i = tid; i < hsz; i += 256) {
    const int c = i / (HR * Wp), r = (i / Wp) % HR, xx = i % Wp;
    const int y = y0 - 1 + r, x = xx - 1;
    hs[i] = (y >= 0 && y < H && x >= 0 && x < W) ? lr[(((size_t)n * C + c) * H + y) * W + x] : 0.f;
  }
  __syncthreads();
  const int nj = 9 * C + 1;  // last = bias
  float acc[37];
#pragma unroll
  for (int k = 0; k < 37; ++k) acc[k] = 0.f;
  for (int r = 0; r < kHeadRows; ++r) {
    const float* grow = g + (((size_t)n * H + y0 + r) * W) * 64 + co;
    for (int x0 = wave; x0 < W; x0 += 16) {  // this wave's pixels x0, x0+4, x0+8, x0+12
      float gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) gv[u] = grow[(size_t)min(x0 + 4 * u, W - 1) * 64];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int x = x0 + 4 * u;
        if (x >= W) break;  // uniform
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c < C) {
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[c * 9 + t] += gv[u] * hs[(c * HR + r + t / 3) * Wp + x + t % 3];
          }
        }
        acc[36] += gv[u];
      }
    }
  }
  float* red = hs + hsz;
#pragma unroll
  for (int k = 0; k < 36; ++k)
    if (k < nj - 1) red[(wave * 64 + co) * 37 + k] = acc[k];
  red[(wave * 64 + co) * 37 + 36] = acc[36];
  __syncthreads();
  float* out = slab + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 64 * nj;
  for (int i = tid; i < 64 * nj; i += 256) {
    const int c2 = i / nj, j = i - c2 * nj, k = (j == nj - 1) ? 36 : j;
    out[i] = (red[(0 * 64 + c2) * 37 + k] + red[(1 * 64 + c2) * 37 + k]) +
             (red[(2 * 64 + c2) * 37 + k] + red[(3 * 64 + c2) * 37 + k]);
  }
}

int head_wgrad_launch(const float* lr, const float* g, int N, int C, int H, int W, float* slab, int* nslab,
                      hipStream_t st) {
  if (C < 1 || C > 4 || H % kHeadRows) return SRMI_ERR_SHAPE;
  const int smem = (C * (kHeadRows + 2) * (W + 2) + 4 * 64 * 37) * 4;
  hipLaunchKernelGGL(head_wgrad_kernel, dim3(H / kHeadRows, N), dim3(256), smem, st, lr, g, C, H, W, slab);
  SRMI_CHECK_LAUNCH();
  *nslab = N * (H / kHeadRows);
  return 0;
}

int head_wgrad_reduce_launch(const float* slab, int nslab, int C, float* gw, float* gb, hipStream_t st) {
  const int per = 64 * (9 * C + 1);
  hipLaunchKernelGGL(slab_reduce_kernel<0>, dim3((per + 15) / 16), dim3(256), 0, st, slab, nslab, per, C, gw, gb);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// =========================================================================== tail
// workgroup barrier ordering LDS only: prefetched global loads stay in flight
__device__ __forceinline__ void tail_fwd_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
// y[n][c][yy][xx] = b[c] + sum_{tap,ci} x[n][yy+ky-1][xx+kx-1][ci] * w[c][ci][tap]
// As an MFMA implicit GEMM with A = filters (16 output-channel
// rows, only the C < 16 real ones ever written or stored), B = halo pixels,
// K = 9 taps x 64 ci, v_mfma_f32_16x16x32_bf16.  Workgroup = 4 output rows x TW
// pixels (wave w = row w), halo and bf16 filters staged in LDS with the conv
// kernels' chunk swizzle.  The VALU form above spent ~1 K FMAs per pixel with
// per-FMA weight loads; this one is bound by reading the 64-channel input once.
//
// Persistent: a workgroup converts the filters once and walks strips s = blockIdx.x,
// + gridDim.x, ...; the next strip's halo is loaded into registers while the current
// strip's MFMAs and stores run and committed to LDS behind LDS-only barriers (one
// strip per workgroup waited one memory latency per 24 KiB of output work).
template <int TW>
__global__ void __launch_bounds__(256) tail_fwd_mfma_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ b, int C, int H, int W, int N,
                                                            float* __restrict__ y) {
  constexpr int NPT = TW / 16, WP = TW + 2, HALO = 6 * WP;
  constexpr int NL = (HALO * 8 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char tsm[];
  char* halo = tsm;               // [6][WP] px x 128 B
  char* wl = tsm + HALO * 128;    // [9 taps][16 co rows] x 128 B
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, fr = lane & 15, fk = lane >> 4;
  const int sx = W / TW, sy = H / 4, nstrips = sx * sy * N;
  uint4 hv[NL];
  auto issue = [&](int st) {  // every load of the thread in flight at once (clamped)
    const int n = st / (sx * sy), rem = st - n * sx * sy, y0 = (rem / sx) * 4, x0 = (rem % sx) * TW;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int i = min(tid + j * 256, HALO * 8 - 1);
      const int q = i >> 3, c = i & 7;
      const int hy = q / WP, hx = q - hy * WP;
      const int yy = min(max(y0 - 1 + hy, 0), H - 1), xx = min(max(x0 - 1 + hx, 0), W - 1);
      hv[j] = *reinterpret_cast<const uint4*>(x + (((size_t)n * H + yy) * W + xx) * 64 + c * 8);
    }
  };
  int s = blockIdx.x;
  if (s >= nstrips) return;
  issue(s);
  // filters w[co][ci][tap] (fp32, torch layout) -> bf16 rows co < C of [tap][co][ci];
  // rows >= C stay unwritten: they only feed output rows that are never stored
  for (int i = tid; i < C * 576; i += 256) {
    const int co = i / 576, ci = (i / 9) % 64, tap = i % 9;
    *reinterpret_cast<bf16_t*>(wl + tap * 2048 + swz128(co, ci >> 3) + (ci & 7) * 2) = f2bf(w[i]);
  }
  float bias[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias[i] = i < C ? b[i] : 0.f;
  for (; s < nstrips; s += gridDim.x) {
    const int n = s / (sx * sy), rem = s - n * sx * sy, y0 = (rem / sx) * 4, x0 = (rem % sx) * TW;
    tail_fwd_lds_barrier();  // the previous strip's halo readers are done
#pragma unroll
    for (int j = 0; j < NL; ++j) {  // commit (padding zeroed)
      const int i = tid + j * 256;
      if (i < HALO * 8) {
        const int q = i >> 3, c = i & 7;
        const int hy = q / WP, hx = q - hy * WP;
        const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
        const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
        *reinterpret_cast<uint4*>(halo + swz128(q, c)) = ok ? hv[j] : make_uint4(0, 0, 0, 0);
      }
    }
    tail_fwd_lds_barrier();
    if (s + (int)gridDim.x < nstrips) issue(s + gridDim.x);
    f32x4 acc[NPT];
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) acc[pt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 a = lds_frag(wl, tap * 2048 + swz128(fr, kk * 4 + fk));
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt)
          acc[pt] = mfma16(a, lds_frag(halo, swz128((wave + ky) * WP + pt * 16 + fr + kx, kk * 4 + fk)), acc[pt]);
      }
    }
    // lane (fr, fk) holds output channels 4 fk + i of pixel pt * 16 + fr
    if (fk == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < C) {
#pragma unroll
          for (int pt = 0; pt < NPT; ++pt)
            y[(((size_t)n * C + i) * H + y0 + wave) * W + x0 + pt * 16 + fr] = acc[pt][i] + bias[i];
        }
    }
  }
}

// Exact-fp32 form (fp32 engine mode) on the VALU (C <= 4 outputs per pixel: an MFMA
// form would waste 12 of its 16 output rows at 1/16 of the bf16 rate).  A workgroup
// = 4 rows x 32 px of one image with ALL 64 channels of its 6 x 34 halo staged once,
// pixel-major (whole 256-byte pixel rows per load; pitch 68 floats).  Thread = (row,
// 4-pixel group, 8-channel group): per filter row it reads its 6-pixel x 8-channel
// window (12 ds_read_b128) and the taps' filters for all C outputs as float4
// broadcasts, issues 8 ch x 3 kx x 4 px x 4 co FMAs, and the 8 channel groups (8
// consecutive lanes) are summed by xor shuffles in a fixed order.  (The former form
// staged 8-channel slices of 256-px rows: every 128-byte line of x was fetched for 4
// slices at different times -- 731 us at EDSR x8 for a 1.07 GB input.)
constexpr int kTfTX = 32, kTfP = 68;  // px per row per workgroup, LDS pixel pitch (floats)
__global__ void __launch_bounds__(256) tail_fwd_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ b, int C, int H, int W,
                                                           float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float hs[6][kTfTX + 2][kTfP];
  __shared__ float4 wl[64][9];  // [ci][tap] -> co 0..3 (zero beyond C)
  const int n = blockIdx.z, y0 = blockIdx.y * 4, x0 = blockIdx.x * kTfTX, tid = threadIdx.x;
  constexpr int NI = 6 * (kTfTX + 2) * 16, NL = (NI + 255) / 256;  // float4 chunks of the halo
  float4 hv[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) {  // every load of the thread in flight at once (clamped)
    const int i = min(tid + j * 256, NI - 1);
    const int q = i >> 4, c4 = i & 15;
    const int hy = q / (kTfTX + 2), hx = q - hy * (kTfTX + 2);
    const int yy = min(max(y0 - 1 + hy, 0), H - 1), xx = min(max(x0 - 1 + hx, 0), W - 1);
    hv[j] = *reinterpret_cast<const float4*>(x + (((size_t)n * H + yy) * W + xx) * 64 + c4 * 4);
  }
  for (int i = tid; i < 64 * 9; i += 256) {
    const int ci = i / 9, tap = i % 9;
    float v[4];
#pragma unroll
    for (int co = 0; co < 4; ++co) v[co] = co < C ? w[((size_t)co * 64 + ci) * 9 + tap] : 0.f;
    wl[ci][tap] = make_float4(v[0], v[1], v[2], v[3]);
  }
#pragma unroll
  for (int j = 0; j < NL; ++j) {  // padding zeroed
    const int i = tid + j * 256;
    if (i < NI) {
      const int q = i >> 4, c4 = i & 15;
      const int hy = q / (kTfTX + 2), hx = q - hy * (kTfTX + 2);
      const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      *reinterpret_cast<float4*>(&hs[hy][hx][c4 * 4]) = ok ? hv[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  const int cg = tid & 7, pg = (tid >> 3) & 7, r = tid >> 6;  // channels 8cg.., pixels 4pg.., row r
  float acc[4][4];                                            // [co][px]
#pragma unroll
  for (int co = 0; co < 4; ++co)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[co][j] = 0.f;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    float xw[6][8];
#pragma unroll
    for (int p = 0; p < 6; ++p) {
      const float4 u0 = *reinterpret_cast<const float4*>(&hs[r + ky][4 * pg + p][8 * cg]);
      const float4 u1 = *reinterpret_cast<const float4*>(&hs[r + ky][4 * pg + p][8 * cg + 4]);
      xw[p][0] = u0.x; xw[p][1] = u0.y; xw[p][2] = u0.z; xw[p][3] = u0.w;
      xw[p][4] = u1.x; xw[p][5] = u1.y; xw[p][6] = u1.z; xw[p][7] = u1.w;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float4 wv = wl[8 * cg + k][ky * 3 + kx];
        const float wc[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
        for (int co = 0; co < 4; ++co)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[co][j] = fmaf(xw[j + kx][k], wc[co], acc[co][j]);
      }
  }
  // sum over the 8 channel groups (lanes 8m .. 8m+7), fixed order
#pragma unroll
  for (int co = 0; co < 4; ++co)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = acc[co][j];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      acc[co][j] = v;
    }
  if (cg != 0) return;
  const int xo = x0 + 4 * pg;
#pragma unroll
  for (int co = 0; co < 4; ++co) {
    if (co < C) {
      const float bb = b[co];
      float* dst = y + (((size_t)n * C + co) * H + y0 + r) * W + xo;
      if (xo + 3 < W && (W & 3) == 0) {
        *reinterpret_cast<float4*>(dst) = make_float4(acc[co][0] + bb, acc[co][1] + bb, acc[co][2] + bb, acc[co][3] + bb);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (xo + j < W) dst[j] = acc[co][j] + bb;
      }
    }
  }
}

constexpr int kTailFwdBlocks = SRMI_TAIL_FWD_BLOCKS;

int tail_fwd_launch(const void* xv, const float* w, const float* b, int N, int C, int H, int W, float* y, int f32,
                    hipStream_t st) {
  if (C < 1 || C > 4 || H % 4) return SRMI_ERR_SHAPE;
  if (f32) {
    hipLaunchKernelGGL(tail_fwd_f32_kernel, dim3((W + kTfTX - 1) / kTfTX, H / 4, N), dim3(256), 0, st,
                       static_cast<const float*>(xv), w, b, C, H, W, y);
    SRMI_CHECK_LAUNCH();
    return 0;
  }
  const bf16_t* x = static_cast<const bf16_t*>(xv);
  // persistent grid: two workgroups per CU (the LDS image + filters take 57 KiB)
  if (W % 48 == 0) {
    const int ns = (W / 48) * (H / 4) * N;
    hipLaunchKernelGGL(tail_fwd_mfma_kernel<48>, dim3(std::min(ns, kTailFwdBlocks)), dim3(256),
                       6 * 50 * 128 + 9 * 2048, st, x, w, b, C, H, W, N, y);
  } else if (W % 32 == 0) {
    const int ns = (W / 32) * (H / 4) * N;
    hipLaunchKernelGGL(tail_fwd_mfma_kernel<32>, dim3(std::min(ns, kTailFwdBlocks)), dim3(256),
                       6 * 34 * 128 + 9 * 2048, st, x, w, b, C, H, W, N, y);
  } else {
    return SRMI_ERR_SHAPE;
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

// dx[n][yy][xx][ci] = sum_{tap,c} dy[n][c][yy-ky+1][xx-kx+1] * w[c][ci][tap],
// dy = (y - hr) * loss[2]   (gradient of the RMSE, stats.py:5-8)
template <int TWT, typename T>
__global__ void __launch_bounds__(256) tail_dgrad_kernel(const float* __restrict__ yv, const float* __restrict__ hr,
                                                        const float* __restrict__ loss, const float* __restrict__ w,
                                                        int C, int H, int W, T* __restrict__ dx) {
  extern __shared__ __attribute__((aligned(16))) float tds[];
  constexpr int WP = TWT + 2;
  const int n = blockIdx.z, y0 = blockIdx.y * 4, x0 = blockIdx.x * TWT, tid = threadIdx.x;
  float* dyl = tds;                   // [C][6][WP]
  float* wl = tds + 4 * 6 * WP;       // [C][9][64]  (tap-major, ci contiguous)
  const float sc = loss ? loss[2] : 1.f;
  {  // every load of the thread in flight at once (clamped, padding zeroed after)
    constexpr int LD = (4 * 6 * WP + 255) / 256;
    const int nd = C * 6 * WP;
    float yd[LD], hd[LD];
#pragma unroll
    for (int j = 0; j < LD; ++j) {
      const int i = min(tid + j * 256, nd - 1);
      const int c = i / (6 * WP), r = (i / WP) % 6, xx = i % WP;
      const int yy = min(max(y0 - 1 + r, 0), H - 1), xg = min(max(x0 - 1 + xx, 0), W - 1);
      const size_t o = (((size_t)n * C + c) * H + yy) * W + xg;
      yd[j] = yv[o];
      hd[j] = hr ? hr[o] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < LD; ++j) {
      const int i = tid + j * 256;
      if (i < nd) {
        const int r = (i / WP) % 6, xx = i % WP;
        const int yy = y0 - 1 + r, xg = x0 - 1 + xx;
        dyl[i] = (yy >= 0 && yy < H && xg >= 0 && xg < W) ? (yd[j] - hd[j]) * sc : 0.f;
      }
    }
  }
  for (int i = tid; i < C * 576; i += 256) {
    const int c = i / 576, t = (i / 64) % 9, ci = i % 64;
    wl[i] = w[((size_t)c * 64 + ci) * 9 + t];
  }
  __syncthreads();
  // a thread: 8 input channels (ck) of 4 consecutive pixels of one row; per (c, ky)
  // the 6-pixel dy window is read once and each tap's 8 filters once (96 FMAs per 8
  // LDS reads; one pixel per thread read 3 per 8 FMAs)
  const int ck = tid & 7;
  // the thread's channels: bf16 8ck .. 8ck+7 (one 16-byte store; 8 lanes = a 128-byte
  // pixel row); fp32 4ck .. 4ck+3 and 32+4ck .. 32+4ck+3, so that each of the two
  // 16-byte stores of the 8 lanes covers one contiguous 128-byte half of the pixel
  // row (8ck .. 8ck+7 left every store instruction writing 16 B pieces 16 B apart)
  const int c_lo = sizeof(T) == 2 ? 8 * ck : 4 * ck, c_hi = sizeof(T) == 2 ? 8 * ck + 4 : 32 + 4 * ck;
  const auto rdx = wt_rsrc(dx, (uint32_t)((size_t)gridDim.z * H * W * 64 * sizeof(T)));
  constexpr int QPR = TWT / 4;  // 4-pixel groups per row
  for (int pg = tid >> 3; pg < 4 * QPR; pg += 32) {
    const int r = pg / QPR, xq = 4 * (pg - r * QPR);
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
    for (int c = 0; c < C; ++c) {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        // output px xq + j, tap (ky, kx) reads dy at column xq + j + 2 - kx (halo-relative)
        const float* drow = dyl + (c * 6 + r + 2 - ky) * WP + xq;
        float dv[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dv[i] = drow[i];
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int t = ky * 3 + kx;
          const float4 w0 = *reinterpret_cast<const float4*>(wl + (c * 9 + t) * 64 + c_lo);
          const float4 w1 = *reinterpret_cast<const float4*>(wl + (c * 9 + t) * 64 + c_hi);
          const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = dv[j + 2 - kx];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[j][e] += d * wv[e];
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t e = (((size_t)n * H + y0 + r) * W + x0 + xq + j) * 64;
      if constexpr (sizeof(T) == 2) {
        uint4 o;
        o.x = pack2(acc[j][0], acc[j][1]); o.y = pack2(acc[j][2], acc[j][3]);
        o.z = pack2(acc[j][4], acc[j][5]); o.w = pack2(acc[j][6], acc[j][7]);
        // 8 lanes per pixel: 128-byte lines, written through (common.hpp)
        st_wt16(rdx, dx, (uint32_t)((e + c_lo) * 2), o);
      } else {
        st_wt16(rdx, dx, (uint32_t)((e + c_lo) * 4), make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]));
        st_wt16(rdx, dx, (uint32_t)((e + c_hi) * 4), make_float4(acc[j][4], acc[j][5], acc[j][6], acc[j][7]));
      }
    }
  }
}

template <typename T>
static int tail_dgrad_t(const float* y, const float* hr, const float* loss, const float* w, int N, int C, int H, int W,
                        T* dx, hipStream_t st) {
  if (W % 64 == 0) {
    const int smem = (4 * 6 * 66 + 4 * 576) * 4;
    hipLaunchKernelGGL((tail_dgrad_kernel<64, T>), dim3(W / 64, H / 4, N), dim3(256), smem, st, y, hr, loss, w, C, H,
                       W, dx);
  } else if (W % 32 == 0) {
    const int smem = (4 * 6 * 34 + 4 * 576) * 4;
    hipLaunchKernelGGL((tail_dgrad_kernel<32, T>), dim3(W / 32, H / 4, N), dim3(256), smem, st, y, hr, loss, w, C, H,
                       W, dx);
  } else {
    return SRMI_ERR_SHAPE;
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

int tail_dgrad_launch(const float* y, const float* hr, const float* loss, const float* w, int N, int C, int H, int W,
                      void* dx, int f32, hipStream_t st) {
  if (C < 1 || C > 4 || H % 4) return SRMI_ERR_SHAPE;
  return f32 ? tail_dgrad_t(y, hr, loss, w, N, C, H, W, static_cast<float*>(dx), st)
             : tail_dgrad_t(y, hr, loss, w, N, C, H, W, static_cast<bf16_t*>(dx), st);
}

// dW[c][ci][tap] = sum_p dy[c][p] * x[p+off][ci];  db[c] = sum_p dy[c][p]
// dy = (y - hr) * loss[2] is formed on the fly (RMSE gradient, stats.py:5-8).
constexpr int kTailRows = 4;
// Per segment of SEG pixels (64 bf16 / 32 fp32) the workgroup stages the 6 input
// rows its 4 waves need (SEG+2 px x 64 ch) and the RMSE gradient of its 4 rows;
// lane = ci reads the x window from LDS (one row per wave read, conflict-free) and
// the pixel's dy by LDS broadcast.  The cross-wave reduction reuses the x buffer.
template <int CC, typename T>
__global__ void __launch_bounds__(256) tail_wgrad_lds_kernel(const float* __restrict__ yv,
                                                            const float* __restrict__ hr,
                                                            const float* __restrict__ loss, const T* __restrict__ x,
                                                            int H, int W, float* __restrict__ slab) {
  constexpr int SEG = sizeof(T) == 2 ? 64 : 32, SP = SEG + 2;
  constexpr int XS_BYTES = 6 * SP * 64 * (int)sizeof(T), RED_BYTES = 4 * CC * 577 * 4;
  __shared__ __attribute__((aligned(16))) char sbuf[XS_BYTES > RED_BYTES ? XS_BYTES : RED_BYTES];
  __shared__ float dyl[CC][kTailRows][SEG];
  T* xs = reinterpret_cast<T*>(sbuf);                       // [row][px][ci]
  float(*red)[CC * 577] = reinterpret_cast<float(*)[CC * 577]>(sbuf);
  const int n = blockIdx.y, band = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int y0 = band * kTailRows;
  const float sc = loss ? loss[2] : 1.f;
  constexpr int VPC = 16 / (int)sizeof(T);                // elements per 16-byte chunk
  float acc[9][CC], bacc[CC];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < CC; ++c) acc[t][c] = 0.f;
#pragma unroll
  for (int c = 0; c < CC; ++c) bacc[c] = 0.f;
  for (int x0 = 0; x0 < W; x0 += SEG) {
    const int nx = min(SEG, W - x0);
    __syncthreads();  // previous segment's readers are done
    {  // every load of the thread in flight at once (clamped, padding zeroed after)
      constexpr int NX = 6 * SP * (64 / VPC), LX = (NX + 255) / 256;
      constexpr int ND = CC * kTailRows * SEG, LD = (ND + 255) / 256;
      uint4 xv[LX];
      float yd[LD], hd[LD];
#pragma unroll
      for (int j = 0; j < LX; ++j) {
        const int i = min(tid + j * 256, NX - 1);
        const int q = i / (64 / VPC), ch = i % (64 / VPC), r = q / SP, px = q - r * SP;
        const int yy = min(max(y0 - 1 + r, 0), H - 1), xx = min(max(x0 - 1 + px, 0), W - 1);
        xv[j] = *reinterpret_cast<const uint4*>(x + (((size_t)n * H + yy) * W + xx) * 64 + ch * VPC);
      }
#pragma unroll
      for (int j = 0; j < LD; ++j) {
        const int i = min(tid + j * 256, ND - 1);
        const int c = i / (kTailRows * SEG), r = (i / SEG) % kTailRows, px = min(i % SEG, nx - 1);
        const size_t o = (((size_t)n * CC + c) * H + y0 + r) * W + x0 + px;
        yd[j] = yv[o];
        hd[j] = hr ? hr[o] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < LX; ++j) {
        const int i = tid + j * 256;
        if (i < NX) {
          const int q = i / (64 / VPC), ch = i % (64 / VPC), r = q / SP, px = q - r * SP;
          const int yy = y0 - 1 + r, xx = x0 - 1 + px;
          const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W && px <= nx + 1;
          *reinterpret_cast<uint4*>(xs + q * 64 + ch * VPC) = ok ? xv[j] : make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < LD; ++j) {
        const int i = tid + j * 256;
        if (i < ND) {
          const int c = i / (kTailRows * SEG), r = (i / SEG) % kTailRows, px = i % SEG;
          dyl[c][r][px] = px < nx ? (yd[j] - hd[j]) * sc : 0.f;
        }
      }
    }
    __syncthreads();
    float win[3][3];
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      win[rr][0] = to_f32(xs[((wave + rr) * SP + 0) * 64 + lane]);
      win[rr][1] = to_f32(xs[((wave + rr) * SP + 1) * 64 + lane]);
    }
    for (int j = 0; j < nx; ++j) {
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) win[rr][2] = to_f32(xs[((wave + rr) * SP + j + 2) * 64 + lane]);
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        const float dd = dyl[c][wave][j];
        bacc[c] += dd;
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t][c] += dd * win[t / 3][t % 3];
      }
#pragma unroll
      for (int rr = 0; rr < 3; ++rr) {
        win[rr][0] = win[rr][1];
        win[rr][1] = win[rr][2];
      }
    }
  }
  __syncthreads();  // every wave is done with xs: red reuses its bytes
#pragma unroll
  for (int c = 0; c < CC; ++c) {
#pragma unroll
    for (int t = 0; t < 9; ++t) red[wave][c * 577 + lane * 9 + t] = acc[t][c];
    if (lane == 0) red[wave][c * 577 + 576] = bacc[c];  // every lane holds the same sum
  }
  __syncthreads();
  float* out = slab + ((size_t)n * gridDim.x + band) * CC * 577;
  for (int i = tid; i < CC * 577; i += 256) out[i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

template <typename T>
static void tail_wgrad_t(const float* y, const float* hr, const float* loss, const T* x, int N, int C, int H, int W,
                         float* slab, hipStream_t st) {
  const dim3 grid(H / kTailRows, N);
  switch (C) {
    case 1: hipLaunchKernelGGL((tail_wgrad_lds_kernel<1, T>), grid, dim3(256), 0, st, y, hr, loss, x, H, W, slab); break;
    case 2: hipLaunchKernelGGL((tail_wgrad_lds_kernel<2, T>), grid, dim3(256), 0, st, y, hr, loss, x, H, W, slab); break;
    case 3: hipLaunchKernelGGL((tail_wgrad_lds_kernel<3, T>), grid, dim3(256), 0, st, y, hr, loss, x, H, W, slab); break;
    default: hipLaunchKernelGGL((tail_wgrad_lds_kernel<4, T>), grid, dim3(256), 0, st, y, hr, loss, x, H, W, slab); break;
  }
}

int tail_wgrad_launch(const float* y, const float* hr, const float* loss, const void* x, int N, int C, int H,
                      int W, float* slab, int* nslab, int f32, hipStream_t st) {
  if (C < 1 || C > 4 || H % kTailRows) return SRMI_ERR_SHAPE;
  if (f32)
    tail_wgrad_t(y, hr, loss, static_cast<const float*>(x), N, C, H, W, slab, st);
  else
    tail_wgrad_t(y, hr, loss, static_cast<const bf16_t*>(x), N, C, H, W, slab, st);
  SRMI_CHECK_LAUNCH();
  *nslab = N * (H / kTailRows);
  return 0;
}

int tail_wgrad_reduce_launch(const float* slab, int nslab, int C, float* gw, float* gb, hipStream_t st) {
  const int per = C * 577;
  hipLaunchKernelGGL(slab_reduce_kernel<1>, dim3((per + 15) / 16), dim3(256), 0, st, slab, nslab, per, C, gw, gb);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// ====================================================================== resampling
// bicubic (A = -0.75, align_corners = False) at 1/scale: the source coordinate
// scale*d + (scale-1)/2 is half-way between samples -> separable [-3,19,19,-3]/32
// grid (ceil(h w / 256), min(NC, 65535)), planes blockIdx.y, + gridDim.y, ...: 32-bit
// index arithmetic within one plane (64-bit divisions of a flat index cost more than
// the loads), any number of planes
constexpr int kMaxGridY = 65535;
__global__ void downsample_kernel(const float* __restrict__ hr, int NC, int H, int W, int scale,
                                  float* __restrict__ lr) {
  const int h = H / scale, w = W / scale;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= h * w) return;
  const int x = i % w, y = i / w;
  const float k[4] = {-3.f / 32.f, 19.f / 32.f, 19.f / 32.f, -3.f / 32.f};
  const int sy = y * scale + scale / 2 - 2, sx = x * scale + scale / 2 - 2;
  for (size_t nc = blockIdx.y; nc < (size_t)NC; nc += gridDim.y) {
    const float* src = hr + nc * H * W;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int yy = min(max(sy + i, 0), H - 1);
      float rsum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int xx = min(max(sx + j, 0), W - 1);
        rsum += k[j] * src[(size_t)yy * W + xx];
      }
      acc += k[i] * rsum;
    }
    lr[nc * h * w + i] = acc;
  }
}

int downsample_launch(const float* hr, int N, int C, int H, int W, int scale, float* lr, hipStream_t st) {
  if (scale < 2 || H % scale || W % scale || N < 1 || C < 1) return SRMI_ERR_SHAPE;
  const int plane = (H / scale) * (W / scale);
  const int gy = N * C < kMaxGridY ? N * C : kMaxGridY;
  hipLaunchKernelGGL(downsample_kernel, dim3((plane + 255) / 256, gy), dim3(256), 0, st, hr, N * C, H, W, scale, lr);
  SRMI_CHECK_LAUNCH();
  return 0;
}

__device__ __forceinline__ void cubic_w(float t, float* c) {
  const float A = -0.75f;
  float x1 = t + 1.f;
  c[0] = ((A * x1 - 5.f * A) * x1 + 8.f * A) * x1 - 4.f * A;
  float x = t;
  c[1] = ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
  x = 1.f - t;
  c[2] = ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
  float x2 = 2.f - t;
  c[3] = ((A * x2 - 5.f * A) * x2 + 8.f * A) * x2 - 4.f * A;
}

__global__ void upsample_kernel(const float* __restrict__ lr, int NC, int h, int w, int scale,
                                float* __restrict__ hr) {
  const int H = h * scale, W = w * scale;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // grid as downsample_kernel's
  if (i >= H * W) return;
  const int X = i % W, Y = i / W;
  const float inv = 1.f / (float)scale;
  const float sy = inv * (Y + 0.5f) - 0.5f, sx = inv * (X + 0.5f) - 0.5f;
  const int iy = (int)floorf(sy), ix = (int)floorf(sx);
  float wy[4], wx[4];
  cubic_w(sy - iy, wy);
  cubic_w(sx - ix, wx);
  for (size_t nc = blockIdx.y; nc < (size_t)NC; nc += gridDim.y) {
    const float* src = lr + nc * h * w;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int yy = min(max(iy - 1 + i, 0), h - 1);
      float rsum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int xx = min(max(ix - 1 + j, 0), w - 1);
        rsum += wx[j] * src[(size_t)yy * w + xx];
      }
      acc += wy[i] * rsum;
    }
    hr[nc * H * W + i] = acc;
  }
}

int upsample_launch(const float* lr, int N, int C, int h, int w, int scale, float* hr, hipStream_t st) {
  if (scale < 1 || N < 1 || C < 1) return SRMI_ERR_SHAPE;
  const int plane = h * scale * w * scale;
  const int gy = N * C < kMaxGridY ? N * C : kMaxGridY;
  hipLaunchKernelGGL(upsample_kernel, dim3((plane + 255) / 256, gy), dim3(256), 0, st, lr, N * C, h, w, scale, hr);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// F.interpolate(x, scale_factor, mode, align_corners=False) at any factor, the form
// downsample / upsample take with task.downsample_mode / upsample_mode 'linear' ->
// bilinear, 'cubic' -> bicubic (torch_interp_mode, array.py:37-41, :72-76, :84-87) and
// data_downsample's non-even factors (dual_trainer.py:561-563).  As ATen computes it
// (UpSample.h): source coordinate r (d + 0.5) - 0.5 in fp32 with r = 1 / scale_factor;
// bilinear clamps it at 0, index i0 = min(floor, n - 1), weight lambda = clamp(src - i0,
// 0, 1) on i0 and min(i0 + 1, n - 1); bicubic (A = -0.75) reads i0 - 1 .. i0 + 2 clamped
// to the edge with the cubic weights of lambda.  One thread per output element.
__device__ __forceinline__ void interp_axis(float r, int d, int n, int mode, int* idx, float* wt) {
  float src = r * ((float)d + 0.5f) - 0.5f;
  if (mode == 1 && src < 0.f) src = 0.f;
  const int i0 = min((int)floorf(src), n - 1);
  const float t = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  if (mode == 1) {
    idx[0] = i0;
    idx[1] = min(i0 + 1, n - 1);
    wt[0] = 1.f - t;
    wt[1] = t;
  } else {
    cubic_w(t, wt);
#pragma unroll
    for (int i = 0; i < 4; ++i) idx[i] = min(max(i0 - 1 + i, 0), n - 1);
  }
}

__global__ void interp_kernel(const float* __restrict__ x, int NC, int H, int W, int Ho, int Wo, float rh, float rw,
                              int mode, float* __restrict__ y) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)NC * Ho * Wo) return;
  const int ox = idx % Wo, oy = (idx / Wo) % Ho;
  const size_t nc = idx / ((size_t)Wo * Ho);
  int iy[4], ix[4];
  float wy[4], wx[4];
  interp_axis(rh, oy, H, mode, iy, wy);
  interp_axis(rw, ox, W, mode, ix, wx);
  const float* src = x + nc * H * W;
  const int taps = mode == 1 ? 2 : 4;
  float acc = 0.f;
  for (int i = 0; i < taps; ++i) {
    float rsum = 0.f;
    for (int j = 0; j < taps; ++j) rsum += wx[j] * src[(size_t)iy[i] * W + ix[j]];
    acc += wy[i] * rsum;
  }
  y[idx] = acc;
}

int interp_launch(const float* x, int N, int C, int H, int W, int Ho, int Wo, float rh, float rw, int mode, float* y,
                  hipStream_t st) {
  if (!x || !y || (mode != 1 && mode != 2)) return SRMI_ERR_ARG;
  if (N < 1 || C < 1 || H < 1 || W < 1 || Ho < 1 || Wo < 1 || !(rh > 0.f) || !(rw > 0.f)) return SRMI_ERR_SHAPE;
  const size_t tot = (size_t)N * C * Ho * Wo;
  hipLaunchKernelGGL(interp_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, x, N * C, H, W, Ho, Wo, rh, rw, mode,
                     y);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// ============================================================================ loss
__global__ void __launch_bounds__(256) sqerr_partial_kernel(const float* __restrict__ y, const float* __restrict__ t,
                                                            size_t n, float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  const size_t n4 = n / 4;
  const float4* y4 = reinterpret_cast<const float4*>(y);
  const float4* t4 = reinterpret_cast<const float4*>(t);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 a = y4[i], b = t4[i];
    const float d0 = a.x - b.x, d1 = a.y - b.y, d2 = a.z - b.z, d3 = a.w - b.w;
    s += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
  }
  if (blockIdx.x == 0)
    for (size_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
      const float d = y[i] - t[i];
      s += d * d;
    }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

int sqerr_partial_launch(const float* y, const float* t, size_t n, float* partial, int nblk, hipStream_t st) {
  hipLaunchKernelGGL(sqerr_partial_kernel, dim3(nblk), dim3(256), 0, st, y, t, n, partial);
  SRMI_CHECK_LAUNCH();
  return 0;
}

__global__ void sqerr_finish_kernel(const float* __restrict__ partial, int nblk, double count, float* loss) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 256) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = (float)red[0];
    loss[1] = (float)count;
  }
}

int sqerr_finish_launch(const float* partial, int nblk, double count, float* loss, hipStream_t st) {
  hipLaunchKernelGGL(sqerr_finish_kernel, dim3(1), dim3(256), 0, st, partial, nblk, count, loss);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// Charbonnier loss of ModelTrainer.charbonnier (sres/controller/dual_trainer.py:196-198):
// L = mean(sqrt(d^2 + eps)), d = y - t; partial sums like sqerr_partial_kernel and,
// when dy != NULL, the elementwise gradient dL/dy = d / sqrt(d^2 + eps) / count.
__global__ void __launch_bounds__(256) charb_partial_kernel(const float* __restrict__ y, const float* __restrict__ t,
                                                            size_t n, float eps, float inv_count,
                                                            float* __restrict__ dy, float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float d = y[i] - t[i];
    const float r = sqrtf(d * d + eps);
    s += r;
    if (dy) dy[i] = d / r * inv_count;
  }
  if (!partial) return;  // dy only (uniform branch: no barrier is skipped by part of the block)
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

int charb_partial_launch(const float* y, const float* t, size_t n, float eps, double count, float* dy,
                         float* partial, int nblk, hipStream_t st) {
  hipLaunchKernelGGL(charb_partial_kernel, dim3(nblk), dim3(256), 0, st, y, t, n, eps, (float)(1.0 / count), dy,
                     partial);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// kind LOSS_RMSE: loss[3] = L = sqrt(S / count), loss[2] = dL/dy scale = 1 / (count * L);
// kind LOSS_MEAN (Charbonnier): loss[3] = S / count, loss[2] = 1 / count
__device__ __forceinline__ void loss_finalize_one(float* loss, int kind) {
  if (kind == LOSS_MEAN) {
    loss[3] = loss[0] / loss[1];
    loss[2] = 1.f / loss[1];
  } else {
    const float L = sqrtf(loss[0] / loss[1]);
    loss[3] = L;
    loss[2] = 1.f / (loss[1] * L);
  }
}

__global__ void loss_finalize_kernel(float* loss, int kind) { loss_finalize_one(loss, kind); }

int loss_finalize_launch(float* loss, int kind, hipStream_t st) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(1), 0, st, loss, kind);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// loss4 of a whole batch from the loss4 records of its micro-batches (parts[k][4]):
// sums of S in a fixed order, the (global) count of part 0; finalised when kind >= 0
__global__ void loss_combine_kernel(float* loss, const float* __restrict__ parts, int nparts, int kind) {
  float s = 0.f;
  for (int k = 0; k < nparts; ++k) s += parts[4 * k];
  loss[0] = s;
  loss[1] = parts[1];
  if (kind >= 0) loss_finalize_one(loss, kind);
}

int loss_combine_launch(float* loss, const float* parts, int nparts, int kind, hipStream_t st) {
  hipLaunchKernelGGL(loss_combine_kernel, dim3(1), dim3(1), 0, st, loss, parts, nparts, kind);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// Per-batch losses of ModelTrainer.process_image / evaluate (sres/controller/
// dual_trainer.py:417-446, :509-532): the tiles are scored in batches of
// task.batch_size (TileBatchIterator, sres/data/tiles.py:48-74; the last batch may
// be short), each batch's loss is the loss over all its elements, and the
// reported loss is the mean of the batch losses.  Pass 1: one block per tile sums
// its elements' (p - t)^2 (RMSE) or sqrt((p - t)^2 + eps) (Charbonnier) in a fixed
// order; pass 2 (one block) forms the batch losses and their mean in fp64.
__global__ void __launch_bounds__(256) tile_loss_sums_kernel(const float* __restrict__ y,
                                                             const float* __restrict__ t, long long tile_elems,
                                                             int kind, float eps, float* __restrict__ sums) {
  __shared__ float red[4];
  const size_t base = (size_t)blockIdx.x * (size_t)tile_elems;
  float s = 0.f;
  for (long long i = threadIdx.x; i < tile_elems; i += 256) {
    const float d = y[base + i] - t[base + i];
    s += kind == LOSS_MEAN ? sqrtf(d * d + eps) : d * d;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) sums[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// the same with 1024 threads and float4 loads, 4 in flight per thread (tile_elems % 4
// == 0, 16-byte aligned operands): the 256-thread scalar form above is latency bound
// at one workgroup per tile (C5: 441 tiles of 36864 elements, 78 us)
__global__ void __launch_bounds__(1024) tile_loss_sums_v4_kernel(const float4* __restrict__ y,
                                                                  const float4* __restrict__ t, long long tile_v4,
                                                                  int kind, float eps, float* __restrict__ sums) {
  __shared__ float red[16];
  const size_t base = (size_t)blockIdx.x * (size_t)tile_v4;
  auto term = [&](float d) { return kind == LOSS_MEAN ? sqrtf(d * d + eps) : d * d; };
  float s = 0.f;
  long long i = threadIdx.x;
  for (; i + 3 * 1024 < tile_v4; i += 4 * 1024) {
    float4 a[4], c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = y[base + i + u * 1024];
      c[u] = t[base + i + u * 1024];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      s += (term(a[u].x - c[u].x) + term(a[u].y - c[u].y)) + (term(a[u].z - c[u].z) + term(a[u].w - c[u].w));
  }
  for (; i < tile_v4; i += 1024) {
    const float4 a = y[base + i], c = t[base + i];
    s += (term(a.x - c.x) + term(a.y - c.y)) + (term(a.z - c.z) + term(a.w - c.w));
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < 16; k += 2) r += red[k] + red[k + 1];
    sums[blockIdx.x] = r;
  }
}

__global__ void __launch_bounds__(256) batch_loss_mean_kernel(const float* __restrict__ sums, int ntiles,
                                                              long long tile_elems, int bs, int kind,
                                                              float* __restrict__ out) {
  __shared__ double bl[1024];
  const int nb = (ntiles + bs - 1) / bs;
  for (int b = threadIdx.x; b < nb; b += 256) {
    const int t0 = b * bs, t1 = min(ntiles, t0 + bs);
    double s = 0.0;
    for (int k = t0; k < t1; ++k) s += sums[k];
    const double mean = s / ((double)(t1 - t0) * (double)tile_elems);
    const double l = kind == LOSS_MEAN ? mean : sqrt(mean);
    bl[b] = l;
    out[1 + b] = (float)l;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = 0.0;
    for (int b = 0; b < nb; ++b) m += bl[b];
    out[0] = (float)(m / nb);
  }
}

int batch_losses_launch(const float* y, const float* t, int ntiles, long long tile_elems, int bs, int kind, float eps,
                        float* work, float* out, hipStream_t st) {
  if (ntiles < 1 || tile_elems < 1 || bs < 1 || (ntiles + bs - 1) / bs > 1024) return SRMI_ERR_SHAPE;
  if (tile_elems % 4 == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)t & 15) == 0)
    hipLaunchKernelGGL(tile_loss_sums_v4_kernel, dim3(ntiles), dim3(1024), 0, st, reinterpret_cast<const float4*>(y),
                       reinterpret_cast<const float4*>(t), tile_elems / 4, kind, eps, work);
  else
    hipLaunchKernelGGL(tile_loss_sums_kernel, dim3(ntiles), dim3(256), 0, st, y, t, tile_elems, kind, eps, work);
  SRMI_CHECK_LAUNCH();
  hipLaunchKernelGGL(batch_loss_mean_kernel, dim3(1), dim3(256), 0, st, work, ntiles, tile_elems, bs, kind, out);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// Loss sums invariant to how the batch is split over micro-batch engines (and over
// calls): every tile's elements are summed by kTileSub blocks over fixed slices with a
// fixed reduction tree, into parts[tile][kTileSub]; the whole batch's S is then the sum
// of all parts in tile order, in fp64 (loss_from_parts).  So one engine of B tiles and
// two of B/2 give a bit-identical loss -- and loss scale 1/(count L), which the bf16
// gradient maps would otherwise turn from a 1-ulp difference into 1e-5-level noise.
__global__ void __launch_bounds__(256) tile_loss_parts_kernel(const float* __restrict__ y, const float* __restrict__ t,
                                                              long long tile_elems, int kind, float eps,
                                                              float* __restrict__ parts) {
  __shared__ float red[4];
  const int sub = blockIdx.x, tile = blockIdx.y;
  const long long per = (tile_elems + kTileSub - 1) / kTileSub;
  const long long i0 = (long long)sub * per, i1 = min(tile_elems, i0 + per);
  const size_t base = (size_t)tile * (size_t)tile_elems;
  float s = 0.f;
  for (long long i = i0 + threadIdx.x; i < i1; i += 256) {
    const float d = y[base + i] - t[base + i];
    s += kind == LOSS_MEAN ? sqrtf(d * d + eps) : d * d;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) parts[(size_t)tile * kTileSub + sub] = (red[0] + red[1]) + (red[2] + red[3]);
}

int tile_loss_parts_launch(const float* y, const float* t, int ntiles, long long tile_elems, int kind, float eps,
                           float* parts, hipStream_t st) {
  if (ntiles < 1 || tile_elems < 1) return SRMI_ERR_SHAPE;
  hipLaunchKernelGGL(tile_loss_parts_kernel, dim3(kTileSub, ntiles), dim3(256), 0, st, y, t, tile_elems, kind, eps,
                     parts);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// loss4 from the parts of loss_from_parts' tiles: [0] = S (fp64 sum in part order),
// [1] = count; finalised as `kind` when kind >= 0 (-1: before a data-parallel
// all-reduce of loss4[0])
__global__ void __launch_bounds__(256) loss_from_parts_kernel(const float* __restrict__ parts, int nparts, double count,
                                                              int kind, float* loss) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const int per = (nparts + 255) / 256, i0 = tid * per, i1 = min(nparts, i0 + per);
  double a = 0.0;
  for (int i = i0; i < i1; ++i) a += parts[i];
  red[tid] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) {
    loss[0] = (float)red[0];
    loss[1] = (float)count;
    if (kind >= 0) loss_finalize_one(loss, kind);
  }
}

int loss_from_parts_launch(const float* parts, int nparts, double count, int kind, float* loss, hipStream_t st) {
  if (nparts < 1 || count <= 0) return SRMI_ERR_ARG;
  hipLaunchKernelGGL(loss_from_parts_kernel, dim3(1), dim3(256), 0, st, parts, nparts, count, kind, loss);
  SRMI_CHECK_LAUNCH();
  return 0;
}

int batch_loss_means_launch(const float* sums, int ntiles, long long tile_elems, int bs, int kind, float* out,
                            hipStream_t st) {
  if (ntiles < 1 || tile_elems < 1 || bs < 1 || (ntiles + bs - 1) / bs > 1024) return SRMI_ERR_SHAPE;
  hipLaunchKernelGGL(batch_loss_mean_kernel, dim3(1), dim3(256), 0, st, sums, ntiles, tile_elems, bs, kind, out);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// =============================================================== channel attention
// Channel attention (CALayer, reference sres/model/rcan/network.py:31-47):
//   m = avgpool(u); z1 = W1 m + b1; s = sigmoid(W2 relu(z1) + b2); h += s * u
// rec per image: m[C] | z1[CR] | s[C]   (C = 64, CR = C / R <= 32)
//
// One launch per direction: every block of the elementwise pass first issues its
// own stream loads, then recomputes the image's tiny MLP (4 K MACs) from the
// producer's per-strip pool partials while those loads are in flight -- no
// separate per-image MLP launch and no launch-to-launch bubble on the critical
// chain.  Weights are read straight into registers (L2 hits); every dot product
// is split over 8 (4) lanes and finished with a fixed-order butterfly; the pool
// partials are summed in a fixed order, so all blocks of an image agree bit for
// bit and block 0 of the image writes the record the backward pass reads.

// workgroup barrier that orders LDS only: global loads stay in flight across it
// (__syncthreads' release fence would drain vmcnt)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// 4-channel units of an activation map in either storage type: raw loads kept
// packed (bf16: one dword pair) until use, written through as one store
template <typename T>
struct Unit4;
template <>
struct Unit4<bf16_t> {
  using raw = uint2;
  static __device__ __forceinline__ raw ld(const bf16_t* p) { return *reinterpret_cast<const uint2*>(p); }
  static __device__ __forceinline__ float get(const raw& v, int i) {
    const uint32_t w = i < 2 ? v.x : v.y;
    return bf2f((i & 1) ? (w >> 16) : (w & 0xFFFF));
  }
  static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, bf16_t* base, size_t e, const float (&o)[4]) {
    st_wt8(r, base, (uint32_t)(e * 2), make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3])));
  }
};
template <>
struct Unit4<float> {
  using raw = float4;
  static __device__ __forceinline__ raw ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ float get(const raw& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
  static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, float* base, size_t e, const float (&o)[4]) {
    st_wt16(r, base, (uint32_t)(e * 4), make_float4(o[0], o[1], o[2], o[3]));
  }
};

// elementwise passes: each thread handles kCaVec groups of 8 channels (4: the
// per-block MLP is amortised over 2x the data of the former 2; 18 blocks per
// 48x48 image, every block resident at once; ca_fwd 22.6 -> 20.0 us, ca_bwd
// 15.1 -> 13.7 us against the former separate MLP launches)
constexpr int kCaVec = SRMI_CA_VEC;

// h_out = u * s + h_in; grid (chunks, N).  Residual-stream forms (MODE):
//   CA_F32   fp32 h in, fp32 h + operand-type copy out (the exact-fp32 engine mode)
//   CA_F32LO fp32 h in (the group input), h out as a pair hi + lo
//   CA_LO    pair in and out
// The pair (common.hpp pair_encode4 / pair_decode4): hi = bf16(h) -- the next conv's
// operand, stored anyway -- and an 8-bit remainder lo, h to 16 significant bits, while
// the pass moves 8 B per element (u 2 + hi 2 + lo 1 in, hi 2 + lo 1 out) instead of 12
// with an fp32 stream.
enum CaMode { CA_F32 = 0, CA_F32LO = 1, CA_LO = 2 };
#define CA_DEC4 pair_decode4
#define CA_ENC4 pair_encode4

template <typename T, int MODE>
__global__ void __launch_bounds__(256) ca_fwd_kernel(const T* __restrict__ u, const float* __restrict__ part,
                                                     int nstrips, int HW, const float* __restrict__ w1,
                                                     const float* __restrict__ b1, const float* __restrict__ w2,
                                                     const float* __restrict__ b2, int C, int CR,
                                                     const float* __restrict__ h_in, const bf16_t* __restrict__ hi_in,
                                                     const uint8_t* __restrict__ lo_in, float* __restrict__ h_out,
                                                     T* __restrict__ hb_out, uint8_t* __restrict__ lo_out,
                                                     float* __restrict__ rec) {
  __shared__ float red[4][64], m[64], z1[32], s[64];
  const int n = blockIdx.y, tid = threadIdx.x;
  // 1. the MLP operands (L2 hits), issued first so that waiting for them does not
  //    wait for the stream loads behind them (vmcnt retires in order): W1 row
  //    slice (z1 lane group j, 8 lanes), W2 row slice (s lane group c, 4 lanes),
  //    biases, the pool partials.
  const int j = tid >> 3, pj = tid & 7;
  const int c4 = tid >> 2, p4 = tid & 3, per = CR / 4;
  // (unconditional loads at clamped indices -- no divergent branches, so the
  //  compiler's vmcnt accounting stays exact across the stream loads below)
  float pa = 0.f;
  {  // (the strip records issued at once, as in ca_bwd_du_kernel)
    constexpr int KU = 4;
    float pv[KU];
    const float* pp = part + (size_t)n * nstrips * C + (tid & 63);
#pragma unroll
    for (int i = 0; i < KU; ++i) pv[i] = pp[(size_t)min((tid >> 6) + 4 * i, nstrips - 1) * C];
#pragma unroll
    for (int i = 0; i < KU; ++i)
      if ((tid >> 6) + 4 * i < nstrips) pa += pv[i];
    for (int k = (tid >> 6) + 4 * KU; k < nstrips; k += 4) pa += pp[(size_t)k * C];
  }
  const int jc = min(j, CR - 1);
  float wa[8], wb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) wa[i] = w1[jc * C + pj * 8 + i];
#pragma unroll
  for (int i = 0; i < 8; ++i) wb[i] = w2[c4 * CR + p4 * per + min(i, per - 1)];
  const float bj = b1[jc];
  const float bc = b2[c4];
  __builtin_amdgcn_sched_barrier(0);
  // 2. this thread's stream loads (independent of s), in flight during the MLP.
  //    Units of 4 channels, consecutive lanes on consecutive units: every load and
  //    store instruction covers one contiguous run (1 KiB fp32 / 512 B bf16).
  constexpr int NU = 2 * kCaVec;
  const size_t base = (size_t)n * HW * C;
  const size_t nq = (size_t)HW * C / 4;
  const size_t q0 = ((size_t)blockIdx.x * NU) * blockDim.x + tid;
  typename Unit4<T>::raw uu[NU];
  float4 hh[NU];
#pragma unroll
  for (int k = 0; k < NU; ++k) {  // clamped, unconditional (tail lanes store nothing)
    const size_t e = base + min(q0 + (size_t)k * blockDim.x, nq - 1) * 4;
    uu[k] = Unit4<T>::ld(u + e);
    if constexpr (MODE == CA_LO) {  // the pair's raw bits: decoded after the MLP, so that these loads stay
                                    // in flight under it (a decode here waits for them first)
      const uint2 hb = *reinterpret_cast<const uint2*>(hi_in + e);
      const uint32_t lb = *reinterpret_cast<const uint32_t*>(lo_in + e);
      hh[k] = make_float4(__uint_as_float(hb.x), __uint_as_float(hb.y), __uint_as_float(lb), 0.f);
    } else {
      hh[k] = *reinterpret_cast<const float4*>(h_in + e);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // 3. the MLP (LDS-only barriers: the stream loads stay in flight)
  red[tid >> 6][tid & 63] = pa;
  lds_barrier();
  if (tid < C) m[tid] = (red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid]) / (float)HW;
  lds_barrier();
  {  // z1[j] = b1[j] + sum_c W1[j][c] m[c]
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += wa[i] * m[pj * 8 + i];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (j < CR && pj == 0) z1[j] = a + bj;
  }
  lds_barrier();
  {  // s[c] = sigmoid(b2[c] + sum_j W2[c][j] relu(z1[j]))
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) a += wb[i] * fmaxf(z1[p4 * per + i], 0.f);
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (p4 == 0) s[c4] = 1.f / (1.f + expf(-(a + bc)));
  }
  lds_barrier();
  if (blockIdx.x == 0) {
    float* r = rec + (size_t)n * (2 * C + CR);
    if (tid < C) {
      r[tid] = m[tid];
      r[C + CR + tid] = s[tid];
    }
    if (tid < CR) r[C + tid] = z1[tid];
  }
  // 4. elementwise; lane-contiguous runs written through (common.hpp): the
  //    boundary after this launch then has no dirty residual stream to flush
  [[maybe_unused]] const auto rh = wt_rsrc(h_out, (uint32_t)((size_t)gridDim.y * HW * C * 4));
  const auto rhb = wt_rsrc(hb_out, (uint32_t)((size_t)gridDim.y * HW * C * sizeof(T)));
  [[maybe_unused]] const auto rlo = wt_rsrc(lo_out, (uint32_t)((size_t)gridDim.y * HW * C));
#pragma unroll
  for (int k = 0; k < NU; ++k) {
    const size_t q = q0 + (size_t)k * blockDim.x;
    if (q >= nq) continue;
    const size_t e = base + q * 4;
    const int c0 = (int)((q * 4) % C);
    if constexpr (MODE == CA_LO)
      hh[k] = CA_DEC4(make_uint2(__float_as_uint(hh[k].x), __float_as_uint(hh[k].y)), __float_as_uint(hh[k].z));
    float o[4];
    o[0] = Unit4<T>::get(uu[k], 0) * s[c0 + 0] + hh[k].x;
    o[1] = Unit4<T>::get(uu[k], 1) * s[c0 + 1] + hh[k].y;
    o[2] = Unit4<T>::get(uu[k], 2) * s[c0 + 2] + hh[k].z;
    o[3] = Unit4<T>::get(uu[k], 3) * s[c0 + 3] + hh[k].w;
    if constexpr (MODE == CA_F32) {
      st_wt16(rh, h_out, (uint32_t)(e * 4), make_float4(o[0], o[1], o[2], o[3]));
      Unit4<T>::st(rhb, hb_out, e, o);
    } else {
      uint2 hi;
      const uint32_t lo = CA_ENC4(o[0], o[1], o[2], o[3], hi);
      st_wt8(rhb, hb_out, (uint32_t)(e * 2), hi);
      st_wt4(rlo, lo_out, (uint32_t)e, lo);
    }
  }
}

static int ca_grid_x(int HW, int C) {
  const int nv = HW * C / 8;
  int gx = (nv + 256 * kCaVec - 1) / (256 * kCaVec);
  return gx < 1 ? 1 : gx;
}

int ca_fwd_launch(const void* u, const float* part, int nstrips, const float* w1, const float* b1, const float* w2,
                  const float* b2, int N, int HW, int C, int R, const float* h_in, float* h_out, void* hb_out,
                  float* rec, int f32, hipStream_t st, const void* hi_in, const void* lo_in, void* lo_out) {
  if (C != 64 || C % R || (C / R) > 32 || (C / R) % 4 || (HW * C) % 8) return SRMI_ERR_SHAPE;
  const dim3 grid(ca_grid_x(HW, C), N);
  const bf16_t* hi = static_cast<const bf16_t*>(hi_in);
  const uint8_t* lo = static_cast<const uint8_t*>(lo_in);
  uint8_t* lout = static_cast<uint8_t*>(lo_out);
  if (f32) {
    if (!h_in || !h_out || lo_out || hi_in) return SRMI_ERR_ARG;
    hipLaunchKernelGGL((ca_fwd_kernel<float, CA_F32>), grid, dim3(256), 0, st, static_cast<const float*>(u), part,
                       nstrips, HW, w1, b1, w2, b2, C, C / R, h_in, hi, lo, h_out, static_cast<float*>(hb_out), lout,
                       rec);
  } else if (!lo_out) {
    if (!h_in || !h_out) return SRMI_ERR_ARG;
    hipLaunchKernelGGL((ca_fwd_kernel<bf16_t, CA_F32>), grid, dim3(256), 0, st, static_cast<const bf16_t*>(u), part,
                       nstrips, HW, w1, b1, w2, b2, C, C / R, h_in, hi, lo, h_out, static_cast<bf16_t*>(hb_out), lout,
                       rec);
  } else if (h_in) {
    hipLaunchKernelGGL((ca_fwd_kernel<bf16_t, CA_F32LO>), grid, dim3(256), 0, st, static_cast<const bf16_t*>(u),
                       part, nstrips, HW, w1, b1, w2, b2, C, C / R, h_in, hi, lo, h_out,
                       static_cast<bf16_t*>(hb_out), lout, rec);
  } else {
    if (!hi || !lo) return SRMI_ERR_ARG;
    hipLaunchKernelGGL((ca_fwd_kernel<bf16_t, CA_LO>), grid, dim3(256), 0, st, static_cast<const bf16_t*>(u), part,
                       nstrips, HW, w1, b1, w2, b2, C, C / R, h_in, hi, lo, h_out, static_cast<bf16_t*>(hb_out), lout,
                       rec);
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

// CA backward.  part[n][strip][2C] holds sum_p g (0..C-1) and sum_p g*u
// (C..2C-1) from the producer of g.  Every block recomputes the image's MLP
// backward while its g loads are in flight; block 0 of the image writes
// brec per image: dz2[C] dz1[CR] dbconv2[C]; followed (after all N images) by
// dm[N][C] = W1^T dz1 (the gradient of the pooled mean).
// du = g * s + dm / HW  (operand type T); g fp32, or (TG = bf16_t) the bf16 engine's
// in-group gradient stream.  DU = false (du null): the MLP backward and brec only, one
// block per image -- the next fused backward launch forms du from g itself (ConvParams
// gx_*, du_from_g8: the same fma and rounding)
//
// Rows blockIdx.y >= N of the grid (nred > 0) carry the fixed-order slab
// reductions of the previous RCAB's two filter gradients (r0, r1: nred blocks
// each, 256-thread wgrad_reduce_body): both are memory-bound passes of many small
// blocks, so the reduction rides in this launch instead of a launch of its own.
template <typename T, typename TG, bool DU = true>
__global__ void __launch_bounds__(256) ca_bwd_du_kernel(const TG* __restrict__ g, const float* __restrict__ part,
                                                        int nstrips, const float* __restrict__ rec,
                                                        const float* __restrict__ w1, const float* __restrict__ w2,
                                                        int N, int HW, int C, int CR, T* __restrict__ du,
                                                        float* __restrict__ brec, ReduceSet r0, ReduceSet r1,
                                                        int nred) {
  if ((int)blockIdx.y >= N) {
    const int id = ((int)blockIdx.y - N) * (int)gridDim.x + (int)blockIdx.x;
    if (id < nred)
      wgrad_reduce_body<16>(r0, id);
    else if (id < 2 * nred)
      wgrad_reduce_body<16>(r1, id - nred);
    return;
  }
  __shared__ float sm[kCaBwdScratch];
  const int n = blockIdx.y, tid = threadIdx.x;
  const CaBwdIn cb{part, nstrips, rec, w1, w2, CR, brec, N, 1.f / (float)HW};
  CaBwdPre q;  // the MLP operands first (ca_bwd.hpp), then the stream's loads behind them
  ca_bwd_load(cb, n, tid, q);
  __builtin_amdgcn_sched_barrier(0);
  const size_t base = (size_t)n * HW * C;
  const size_t nv = (size_t)HW * C / 8;
  const size_t v0 = ((size_t)blockIdx.x * kCaVec) * blockDim.x + tid;
  float4 g0[kCaVec], g1[kCaVec];
  [[maybe_unused]] uint4 gq[kCaVec];
#pragma unroll
  for (int k = 0; k < (DU ? kCaVec : 0); ++k) {  // clamped, unconditional (tail lanes store nothing)
    const size_t e = base + min(v0 + (size_t)k * blockDim.x, nv - 1) * 8;
    if constexpr (sizeof(TG) == 2) {
      gq[k] = *reinterpret_cast<const uint4*>(g + e);  // 8 bf16, decoded where used
    } else {
      g0[k] = *reinterpret_cast<const float4*>(g + e);
      g1[k] = *reinterpret_cast<const float4*>(g + e + 4);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  ca_bwd_mlp(cb, n, tid, q, sm, blockIdx.x == 0);
  const float* s = sm + kCaBwdS;
  const float* dm = sm + kCaBwdDm;
  if constexpr (!DU) return;
  const auto rdu = wt_rsrc(du, (uint32_t)((size_t)gridDim.y * HW * C * sizeof(T)));  // lane-contiguous: write-through
#pragma unroll
  for (int k = 0; k < kCaVec; ++k) {
    const size_t v = v0 + (size_t)k * blockDim.x;
    if (v >= nv) continue;
    const int c0 = (int)((v * 8) % C);
    float dmh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) dmh[i] = dm[c0 + i] * (1.f / (float)HW);
    if constexpr (sizeof(TG) == 2) {
      g0[k] = make_float4(bf2f(gq[k].x & 0xFFFFu), bf2f(gq[k].x >> 16), bf2f(gq[k].y & 0xFFFFu), bf2f(gq[k].y >> 16));
      g1[k] = make_float4(bf2f(gq[k].z & 0xFFFFu), bf2f(gq[k].z >> 16), bf2f(gq[k].w & 0xFFFFu), bf2f(gq[k].w >> 16));
    }
    const float o[8] = {fmaf(g0[k].x, s[c0 + 0], dmh[0]), fmaf(g0[k].y, s[c0 + 1], dmh[1]),
                        fmaf(g0[k].z, s[c0 + 2], dmh[2]), fmaf(g0[k].w, s[c0 + 3], dmh[3]),
                        fmaf(g1[k].x, s[c0 + 4], dmh[4]), fmaf(g1[k].y, s[c0 + 5], dmh[5]),
                        fmaf(g1[k].z, s[c0 + 6], dmh[6]), fmaf(g1[k].w, s[c0 + 7], dmh[7])};
    if constexpr (sizeof(T) == 2) {
      const uint4 ob = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
      st_wt16(rdu, du, (uint32_t)((base + v * 8) * 2), ob);
    } else {
      st_wt16(rdu, du, (uint32_t)((base + v * 8) * 4), make_float4(o[0], o[1], o[2], o[3]));
      st_wt16(rdu, du, (uint32_t)((base + v * 8) * 4 + 16), make_float4(o[4], o[5], o[6], o[7]));
    }
  }
}

int ca_bwd_du_launch(const void* g, int g16, const float* part, int nstrips, const float* rec, const float* w1,
                     const float* w2, int N, int HW, int C, int R, void* du, float* brec, int f32, hipStream_t st,
                     const ReduceSet* red0, const ReduceSet* red1) {
  if (f32 && g16) return SRMI_ERR_ARG;
  if (C != 64 || C % R || (C / R) > 32 || (C / R) % 4 || (HW * C) % 8) return SRMI_ERR_SHAPE;
  if ((red0 == nullptr) != (red1 == nullptr)) return SRMI_ERR_ARG;
  if (red0 && (red0->Cout != red1->Cout)) return SRMI_ERR_SHAPE;
  // (a set with neither gw nor gb -- the group tail's single reduction -- adds no blocks)
  const bool two = red1 && (red1->gw || red1->gb);
  if (!du && (f32 || !g16)) return SRMI_ERR_ARG;  // (du from g: the bf16 stream only)
  const int gx = du ? ca_grid_x(HW, C) : 1;
  const ReduceSet none{};
  const int nred = red0 ? wgrad_reduce_blocks(red0->Cout) : 0;
  const dim3 grid(gx, N + ((two ? 2 : 1) * nred + gx - 1) / gx);
  const ReduceSet& a = red0 ? *red0 : none;
  const ReduceSet& b = red1 ? *red1 : none;
  if (f32)
    hipLaunchKernelGGL((ca_bwd_du_kernel<float, float>), grid, dim3(256), 0, st, static_cast<const float*>(g), part,
                       nstrips, rec, w1, w2, N, HW, C, C / R, static_cast<float*>(du), brec, a, b, nred);
  else if (g16 && !du)
    hipLaunchKernelGGL((ca_bwd_du_kernel<bf16_t, bf16_t, false>), grid, dim3(256), 0, st, static_cast<const bf16_t*>(g),
                       part, nstrips, rec, w1, w2, N, HW, C, C / R, static_cast<bf16_t*>(du), brec, a, b, nred);
  else if (g16)
    hipLaunchKernelGGL((ca_bwd_du_kernel<bf16_t, bf16_t>), grid, dim3(256), 0, st, static_cast<const bf16_t*>(g),
                       part, nstrips, rec, w1, w2, N, HW, C, C / R, static_cast<bf16_t*>(du), brec, a, b, nred);
  else
    hipLaunchKernelGGL((ca_bwd_du_kernel<bf16_t, float>), grid, dim3(256), 0, st, static_cast<const float*>(g), part,
                       nstrips, rec, w1, w2, N, HW, C, C / R, static_cast<bf16_t*>(du), brec, a, b, nred);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// CA parameter grads of `nblocks` RCABs (summed over images, fixed order), plus
// the conv2 bias grad.  offs[k*5 + {0..4}] = grad offsets of
// conv_du.0.weight, conv_du.0.bias, conv_du.2.weight, conv_du.2.bias, conv2.bias
__global__ void __launch_bounds__(256) ca_param_grads_kernel(const float* __restrict__ recs,
                                                             const float* __restrict__ brecs, int N, size_t rstride,
                                                             size_t bstride, int C, int CR,
                                                             const long long* __restrict__ offs,
                                                             float* __restrict__ grads) {
  // blockIdx.y < 2*C*CR/256: one weight gradient per thread; the last y slice
  // does the biases.  Image sums run in a fixed order (deterministic).  The
  // records of consecutive RCABs are rstride / bstride floats apart (the engine's
  // slots: capacity x the widest record, whatever CR is); the first N images are summed.
  const int k = blockIdx.x;
  const int rs = 2 * C + CR;
  const float* rec = recs + (size_t)k * rstride;
  const float* brec = brecs + (size_t)k * bstride;  // [N][rs] then dm[N][C]
  const int nw = 2 * C * CR;
  const int o = blockIdx.y * 256 + threadIdx.x;
  if ((int)blockIdx.y * 256 < nw) {
    if (o >= nw) return;
    // a product per image, 8 images' loads in flight per step (a two-accumulator
    // loop waited one L2 latency per image pair: 14.5 us per launch), summed into 8
    // partial sums by image index mod 8 and combined in a fixed order
    const bool w2 = o < C * CR;
    const int oo = w2 ? o : o - C * CR;
    const int ia = w2 ? oo / CR : C + oo / C;   // brec operand: dz2[c] | dz1[j]
    const int ib = w2 ? C + oo % CR : oo % C;   // rec operand: relu(z1[j]) | m[c]
    float ps[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) ps[u] = 0.f;
    for (int n0 = 0; n0 < N; n0 += 8) {
      float a[8], bb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int n = min(n0 + u, N - 1);
        a[u] = brec[n * rs + ia];
        bb[u] = rec[n * rs + ib];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (n0 + u < N) ps[u] += a[u] * (w2 ? fmaxf(bb[u], 0.f) : bb[u]);
    }
    const float sum = ((ps[0] + ps[1]) + (ps[2] + ps[3])) + ((ps[4] + ps[5]) + (ps[6] + ps[7]));
    grads[offs[k * 5 + (w2 ? 2 : 0)] + oo] = sum;
    return;
  }
  for (int q = threadIdx.x; q < rs; q += 256) {
    float ps[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) ps[u] = 0.f;
    for (int n0 = 0; n0 < N; n0 += 8) {
      float a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = brec[min(n0 + u, N - 1) * rs + q];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (n0 + u < N) ps[u] += a[u];
    }
    const float s = ((ps[0] + ps[1]) + (ps[2] + ps[3])) + ((ps[4] + ps[5]) + (ps[6] + ps[7]));
    if (q < C)
      grads[offs[k * 5 + 3] + q] = s;
    else if (q < C + CR)
      grads[offs[k * 5 + 1] + q - C] = s;
    else
      grads[offs[k * 5 + 4] + q - C - CR] = s;
  }
}

int ca_param_grads_batched_launch(const float* recs, const float* brecs, int nblocks, int N, size_t rstride,
                                  size_t bstride, int C, int R, const long long* offs, float* grads, hipStream_t st) {
  const int CR = C / R;
  if (N < 1 || (size_t)N * (2 * C + CR) > rstride || (size_t)N * (3 * C + CR) > bstride) return SRMI_ERR_ARG;
  const int ny = (2 * C * CR + 255) / 256 + 1;
  hipLaunchKernelGGL(ca_param_grads_kernel, dim3(nblocks, ny), dim3(256), 0, st, recs, brecs, N, rstride, bstride, C, CR, offs,
                     grads);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// ============================================================================ Adam
// torch.optim.Adam (foreach path): m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, size_t n, float b1, float b2, float eps, float wd,
                            float step_size, float bc2_sqrt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    const float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi - step_size * (mi / (sqrtf(vi) / bc2_sqrt + eps));
  }
}

int adam_launch(float* p, const float* g, float* m, float* v, size_t n, float lr, float b1, float b2, float eps,
                float wd, float step_size, float bc2_sqrt, hipStream_t st) {
  (void)lr;
  size_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, st, p, g, m, v, n, b1, b2, eps, wd, step_size,
                     bc2_sqrt);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// ========================================================================= packing
// forward pack [Cin/64][9][Cout][64]; dgrad pack [Cout/64][9][Cin][64] with the
// taps flipped (dgrad == forward conv of dY with W'[ci][co][8-tap]); PixelShuffle
// convs store output channel c'' = 64q + c for torch channel 4c + q, so each
// 64-wide output block is one sub-pixel position.
template <typename T>
__device__ __forceinline__ void pack_elem(const float* __restrict__ W, const float* __restrict__ B, int Cout, int Cin,
                                          int ps, int which, long long idx, T* __restrict__ fpack,
                                          T* __restrict__ dpack, float* __restrict__ pbias) {
  if (which == 0) {
    const int ci_l = idx & 63;
    long long rest = idx >> 6;
    const int cop = rest % Cout;
    rest /= Cout;
    const int tap = rest % 9, cc = (int)(rest / 9);
    const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
    fpack[idx] = from_f32<T>(W[((size_t)cot * Cin + cc * 64 + ci_l) * 9 + tap]);
  } else if (which == 1) {
    const int co_l = idx & 63;
    long long rest = idx >> 6;
    const int ci = rest % Cin;
    rest /= Cin;
    const int tapd = rest % 9, ccd = (int)(rest / 9);
    const int cop = ccd * 64 + co_l;
    const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
    dpack[idx] = from_f32<T>(W[((size_t)cot * Cin + ci) * 9 + (8 - tapd)]);
  } else if (idx < Cout) {
    const int cop = (int)idx;
    const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
    pbias[cop] = B[cot];
  }
}

// One workgroup per (64-output-channel block, 64-input-channel block, conv): the
// block's filters W[cot][cc*64 .. +63][9] (64 contiguous 2304-byte rows, cot the
// torch channel of packed channel cop) are read coalesced into LDS in the pack's
// element type, then both packs are written as full 128-byte rows (forward: 64 ci
// of one (tap, cop); dgrad: 64 co of one (tap, ci)).  The element-wise form read W
// with a 36 B (forward) / 2.3 KB (dgrad) lane stride: 262 us per step.
// 8 consecutive pack elements (16-byte aligned: seg * 8 elements into a 64-element row)
// as one 16-byte store (bf16) or two (fp32) instead of 8 element stores
template <typename T>
__device__ __forceinline__ void store8(T* d, const T (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)v[2 * k] | ((uint32_t)v[2 * k + 1] << 16);
    *reinterpret_cast<uint4*>(d) = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) pack_tile_kernel(const float* __restrict__ params,
                                                        const PackEntry* __restrict__ ents, T* __restrict__ packs,
                                                        float* __restrict__ pbias) {
  extern __shared__ __attribute__((aligned(16))) char smem_pack[];
  T* wl = reinterpret_cast<T*>(smem_pack);  // [64 l][64 ci_l][9]
  const PackEntry e = ents[blockIdx.z];
  const int cb = blockIdx.x, cc = blockIdx.y;
  if (cb * 64 >= e.Cout || cc * 64 >= e.Cin) return;
  const int Cout = e.Cout, Cin = e.Cin, tid = threadIdx.x;
  const float* W = params + e.w_off;
  auto cot_of = [&](int cop) { return e.ps ? 4 * (cop & 63) + (cop >> 6) : cop; };
  // 1. 64 rows x 576 floats (144 float4 each = 36 per thread), in batches of 12 loads
  //    in flight (a load-then-store loop waited one memory latency per float4: 88 us)
  static_assert(64 * 144 == 36 * 256, "36 float4 per thread");
#pragma unroll
  for (int b0 = 0; b0 < 36; b0 += 12) {
    float4 v[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const int i = tid + (b0 + j) * 256, l = i / 144, q = i - l * 144;
      v[j] = *reinterpret_cast<const float4*>(W + ((size_t)cot_of(cb * 64 + l) * Cin + cc * 64) * 9 + q * 4);
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const int i = tid + (b0 + j) * 256, l = i / 144, q = i - l * 144;
      T* d = wl + l * 576 + q * 4;
      if constexpr (sizeof(T) == 2)  // one ds_write_b64 (a bf16 element at a time: four ds_write_b16)
        *reinterpret_cast<uint2*>(d) = make_uint2(pack2(v[j].x, v[j].y), pack2(v[j].z, v[j].w));
      else
        *reinterpret_cast<float4*>(d) = v[j];
    }
  }
  __syncthreads();
  // 2. forward pack rows (tap, cop): [cc][tap][cop][ci_l]; 8 lanes per row, 8 ci each
  T* fp = packs + e.f_off;
  for (int i = tid; i < 9 * 64 * 8; i += 256) {
    const int seg = i & 7, r = i >> 3, l = r & 63, tap = r >> 6;
    T v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = wl[l * 576 + (seg * 8 + k) * 9 + tap];
    store8(fp + (((size_t)cc * 9 + tap) * Cout + cb * 64 + l) * 64 + seg * 8, v);
  }
  // 3. dgrad pack rows (tapd, ci): [cb][tapd][ci][co_l] = W[cot][ci][8 - tapd]
  T* dp = packs + e.d_off;
  for (int i = tid; i < 9 * 64 * 8; i += 256) {
    const int seg = i & 7, r = i >> 3, ci_l = r & 63, tapd = r >> 6;
    T v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = wl[(seg * 8 + k) * 576 + ci_l * 9 + (8 - tapd)];
    store8(dp + (((size_t)cb * 9 + tapd) * Cin + cc * 64 + ci_l) * 64 + seg * 8, v);
  }
  if (cc == 0 && tid < 64) pbias[e.pb_off + cb * 64 + tid] = params[e.b_off + cot_of(cb * 64 + tid)];
}

int pack_launch(const float* params, const PackEntry* dev_entries, int nentries, int max_cob, int max_cib, void* packs,
                float* pbias, int f32, hipStream_t st) {
  const dim3 grid((unsigned)max_cob, (unsigned)max_cib, (unsigned)nentries);
  if (f32)
    hipLaunchKernelGGL(pack_tile_kernel<float>, grid, dim3(256), 64 * 576 * sizeof(float), st, params, dev_entries,
                       static_cast<float*>(packs), pbias);
  else
    hipLaunchKernelGGL(pack_tile_kernel<bf16_t>, grid, dim3(256), 64 * 576 * sizeof(bf16_t), st, params,
                       dev_entries, static_cast<bf16_t*>(packs), pbias);
  SRMI_CHECK_LAUNCH();
  return 0;
}

template <typename T>
__global__ void pack_one_kernel(const float* __restrict__ W, const float* __restrict__ B, int Cout, int Cin, int ps,
                                T* __restrict__ fpack, T* __restrict__ dpack, float* __restrict__ pbias) {
  const long long total = (long long)Cout * Cin * 9;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x)
    pack_elem(W, B, Cout, Cin, ps, blockIdx.y, idx, fpack, dpack, pbias);
}

int pack_one_launch(const float* w, const float* b, int Cout, int Cin, int ps, void* fpack, void* dpack,
                    float* pbias, int f32, hipStream_t st) {
  if (Cout % 64 || Cin % 64) return SRMI_ERR_SHAPE;
  if (ps && Cout != 256) return SRMI_ERR_SHAPE;  // the PixelShuffle(2) permutation spans 4 x 64 channels
  long long bx = ((long long)Cout * Cin * 9 + 255) / 256;
  if (bx > 1024) bx = 1024;
  if (f32)
    hipLaunchKernelGGL(pack_one_kernel<float>, dim3((unsigned)bx, 3), dim3(256), 0, st, w, b, Cout, Cin, ps,
                       static_cast<float*>(fpack), static_cast<float*>(dpack), pbias);
  else
    hipLaunchKernelGGL(pack_one_kernel<bf16_t>, dim3((unsigned)bx, 3), dim3(256), 0, st, w, b, Cout, Cin, ps,
                       static_cast<bf16_t*>(fpack), static_cast<bf16_t*>(dpack), pbias);
  SRMI_CHECK_LAUNCH();
  return 0;
}

__global__ void scale_add_kernel(float* y, const float* x, float a, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] += a * x[i];
}

int scale_add_launch(float* y, const float* x, float a, size_t n, hipStream_t st) {
  size_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(scale_add_kernel, dim3(blocks), dim3(256), 0, st, y, x, a, n);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
