// Region <-> tile data path of tiled inference, device side.
//
// region_to_tiles replaces the floor tiling of get_tiles (reference
// sres/base/source/swot/raw.py:216-233) fused with the per-tile, per-channel
// 'lnorm' normalisation of norm() (raw.py:169-181: mean and std over (x, y),
// ddof 0, x' = (x - mean) / std).  One workgroup per (tile, channel): the 2-pass
// statistics are reduced in a fixed order, so the result is deterministic.
//
// batch_prep replaces the training-batch preparation: the
// 'lnorm' branch of norm() (raw.py:169-181) on a selected tile batch, xyflip
// (sres/base/source/batch.py:37-49, applied by load_batch :301) and the
// apply_network input downsample (array.py:72-76) -- one pass over HBM.
//
// tiles_to_region replaces denorm (dual_trainer.py:67-77: x * std + mean) fused
// with assemble_images (dual_trainer.py:482-512: tile id -> grid cell
// (tid / gx, tid % gx), cells without a tile are NaN).
#include <math.h>

#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const float s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

// grid (C, ntiles): tile t = grid cell t (row-major over gy x gx)
__global__ void __launch_bounds__(256) region_to_tiles_kernel(const float* __restrict__ region, int C, int H, int W,
                                                              int ty, int tx, int gx, float* __restrict__ tiles,
                                                              float* __restrict__ mean, float* __restrict__ stdv,
                                                              int* __restrict__ bad) {
  __shared__ float red[4];
  const int c = blockIdx.x, t = blockIdx.y;
  const int y0 = (t / gx) * ty, x0 = (t % gx) * tx;
  const float* src = region + (size_t)c * H * W + (size_t)y0 * W + x0;
  const int n = ty * tx;
  float s = 0.f;
  int nonfinite = 0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = src[(size_t)(i / tx) * W + (i % tx)];
    s += v;
    nonfinite |= !isfinite(v);
  }
  const float m = block_sum256(s, red) / (float)n;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float d = src[(size_t)(i / tx) * W + (i % tx)] - m;
    q += d * d;
  }
  const float sd = sqrtf(block_sum256(q, red) / (float)n);
  const float inv = 1.f / sd;
  float* dst = tiles + ((size_t)t * C + c) * n;
  for (int i = threadIdx.x; i < n; i += 256) dst[i] = (src[(size_t)(i / tx) * W + (i % tx)] - m) * inv;
  const int anybad = __syncthreads_or(nonfinite);
  if (threadIdx.x == 0) {
    mean[(size_t)t * C + c] = m;
    stdv[(size_t)t * C + c] = sd;
    if (bad && anybad) atomicOr(&bad[t], 1);  // the reference drops tiles whose mean is not finite
  }
}

int region_to_tiles_launch(const float* region, int C, int H, int W, int ty, int tx, float* tiles, float* mean,
                           float* stdv, int* bad, hipStream_t st) {
  if (C < 1 || ty < 1 || tx < 1 || H < ty || W < tx) return SRMI_ERR_SHAPE;
  const int gy = H / ty, gx = W / tx;
  if (bad) {
    const hipError_t e = hipMemsetAsync(bad, 0, sizeof(int) * gy * gx, st);
    if (e != hipSuccess) return -(int)e;
  }
  hipLaunchKernelGGL(region_to_tiles_kernel, dim3(C, gy * gx), dim3(256), 0, st, region, C, H, W, ty, tx, gx, tiles,
                     mean, stdv, bad);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// out[c][Y][X] = tiles[inv[cell]][c][y][x] * std + mean, NaN where inv[cell] < 0
// (inv == NULL: tile i is grid cell i).  grid (ceil(gx*tx / 256), gy*ty, C)
__global__ void __launch_bounds__(256) tiles_to_region_kernel(const float* __restrict__ tiles,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ stdv,
                                                              const int* __restrict__ inv, int C, int ty, int tx,
                                                              int gx, float* __restrict__ out) {
  const int X = blockIdx.x * 256 + threadIdx.x, Y = blockIdx.y, c = blockIdx.z;
  const int Wo = gx * tx;
  if (X >= Wo) return;
  const int cell = (Y / ty) * gx + X / tx;
  const int t = inv ? inv[cell] : cell;
  float v = __int_as_float(0x7fc00000);  // NaN
  if (t >= 0) {
    const float z = tiles[(((size_t)t * C + c) * ty + (Y % ty)) * tx + (X % tx)];
    v = mean ? z * stdv[(size_t)t * C + c] + mean[(size_t)t * C + c] : z;
  }
  out[((size_t)c * gridDim.y + Y) * Wo + X] = v;
}

int tiles_to_region_launch(const float* tiles, const float* mean, const float* stdv, const int* inv, int C, int ty,
                           int tx, int gy, int gx, float* out, hipStream_t st) {
  if (C < 1 || ty < 1 || tx < 1 || gy < 1 || gx < 1) return SRMI_ERR_SHAPE;
  hipLaunchKernelGGL(tiles_to_region_kernel, dim3((gx * tx + 255) / 256, gy * ty, C), dim3(256), 0, st, tiles, mean,
                     stdv, inv, C, ty, tx, gx, out);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ batch prep
// One workgroup (1024 threads) per (channel, tile).  The raw tile is read from
// HBM once (float4) into LDS with a padded row pitch (T + 1: the transposed
// reads of flip index >= 4 walk columns without bank conflicts); mean and the
// 2-pass std (ddof 0) are fixed-order block reductions (deterministic) carried
// in fp64, and x - mean is formed in fp64: an fp32 mean of climate fields
// (|mean| ~ 300, ulp 3e-5) would shift a whole normalised tile by ~1e-5.  The
// normalised, flipped HR tile and its bicubic 1/scale LR are written from LDS.
// Tiles too large for LDS (T > 192, e.g. the EDSR x8 256^2 tiles) re-read the
// raw tile through L2 instead.
constexpr int kPrepThreads = 1024;

__device__ __forceinline__ double block_sum1024(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kPrepThreads / 64; ++i) s += red[i];
  __syncthreads();
  return s;
}

// output pixel (y, x) of xyflip(...) reads source pixel (sy, sx) (square tiles):
// swap (bit 2) first, then flip y (bit 1), then flip x (bit 0) -- the inverse of
// the reference's flip-x, flip-y, transpose sequence.
__device__ __forceinline__ void flip_src(int f, int T, int y, int x, int& sy, int& sx) {
  sy = (f & 4) ? x : y;
  sx = (f & 4) ? y : x;
  if (f & 2) sy = T - 1 - sy;
  if (f & 1) sx = T - 1 - sx;
}

template <bool kLds>
__global__ void __launch_bounds__(kPrepThreads) batch_prep_kernel(const float* __restrict__ raw, int C, int T,
                                                                  int flip, int scale, float* __restrict__ hr,
                                                                  float* __restrict__ lr, float* __restrict__ mean,
                                                                  float* __restrict__ stdv) {
  extern __shared__ float tile[];  // [T][T + 1] when kLds
  __shared__ double red[kPrepThreads / 64];
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int n = T * T, P = kLds ? T + 1 : T;
  const float* src = raw + ((size_t)b * C + c) * n;
  const float* buf = kLds ? tile : src;
  double s = 0.0;
  for (int i = 4 * tid; i < n; i += 4 * kPrepThreads) {  // T even -> n % 4 == 0
    const float4 v = *reinterpret_cast<const float4*>(src + i);
    s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
    if (kLds) {
      const int y = i / T, x = i - y * T;  // a float4 straddles two rows only if T % 4 == 2
      float* d = tile + y * P + x;
      if (x + 3 < T) {
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      } else {
        const float vv[4] = {v.x, v.y, v.z, v.w};
        for (int e = 0; e < 4; ++e) {
          const int ye = (i + e) / T, xe = (i + e) - ye * T;
          tile[ye * P + xe] = vv[e];
        }
      }
    }
  }
  const double m = block_sum1024(s, red) / (double)n;  // (also orders the LDS stores)
  double q = 0.0;
  for (int i = tid; i < n; i += kPrepThreads) {
    const int y = i / T, x = i - y * T;
    const double d = (double)buf[y * P + x] - m;
    q += d * d;
  }
  const double sd = sqrt(block_sum1024(q, red) / (double)n);
  const double inv = 1.0 / sd;
  auto norm = [&](int y, int x) __attribute__((always_inline)) {
    int sy, sx;
    flip_src(flip, T, y, x, sy, sx);
    return (float)(((double)buf[sy * P + sx] - m) * inv);
  };
  float* dst = hr + ((size_t)b * C + c) * n;
  for (int i = 4 * tid; i < n; i += 4 * kPrepThreads) {
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int y = (i + e) / T, x = (i + e) - y * T;
      o[e] = norm(y, x);
    }
    *reinterpret_cast<float4*>(dst + i) = make_float4(o[0], o[1], o[2], o[3]);
  }
  if (lr) {
    // downsample_kernel's arithmetic (small.hip) on the normalised, flipped tile
    const int t = T / scale;
    const float k[4] = {-3.f / 32.f, 19.f / 32.f, 19.f / 32.f, -3.f / 32.f};
    float* ldst = lr + ((size_t)b * C + c) * t * t;
    for (int i = tid; i < t * t; i += kPrepThreads) {
      const int y = i / t, x = i - y * t;
      const int y0 = y * scale + scale / 2 - 2, x0 = x * scale + scale / 2 - 2;
      float acc = 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int yy = min(max(y0 + a, 0), T - 1);
        float rsum = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) rsum += k[j] * norm(yy, min(max(x0 + j, 0), T - 1));
        acc += k[a] * rsum;
      }
      ldst[i] = acc;
    }
  }
  if (tid == 0) {
    if (mean) mean[(size_t)b * C + c] = (float)m;
    if (stdv) stdv[(size_t)b * C + c] = (float)sd;
  }
}

int batch_prep_launch(const float* raw, int B, int C, int T, int flip, int scale, float* hr, float* lr, float* mean,
                      float* stdv, hipStream_t st) {
  if (B < 1 || C < 1 || T < 2 || T % 2 || flip < 0 || flip > 7) return SRMI_ERR_SHAPE;
  if (lr && (scale < 2 || T % scale)) return SRMI_ERR_SHAPE;
  if (!raw || !hr) return SRMI_ERR_ARG;
  const size_t lds = (size_t)T * (T + 1) * sizeof(float);
  if (lds <= 150 * 1024) {
    hipLaunchKernelGGL(batch_prep_kernel<true>, dim3(C, B), dim3(kPrepThreads), lds, st, raw, C, T, flip, scale, hr,
                       lr, mean, stdv);
  } else {
    hipLaunchKernelGGL(batch_prep_kernel<false>, dim3(C, B), dim3(kPrepThreads), 0, st, raw, C, T, flip, scale, hr,
                       lr, mean, stdv);
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
