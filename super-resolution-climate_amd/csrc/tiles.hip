// Region <-> tile data path of tiled inference, device side.
//
// region_to_tiles replaces the floor tiling of get_tiles (reference
// sres/base/source/swot/raw.py:216-233) fused with the per-tile, per-channel
// 'lnorm' normalisation of norm() (raw.py:169-181: mean and std over (x, y),
// ddof 0, x' = (x - mean) / std).  One workgroup per (tile, channel): the 2-pass
// statistics are reduced in a fixed order, so the result is deterministic.
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

}  // namespace srmi
