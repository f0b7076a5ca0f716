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
// llc_* replace SWOTRawDataLoader.load_file (swot/raw.py:133-145, mds2d
// swot/util.py:3-7, subset_roi raw.py:38-45) and tiles_nonfinite/tiles_gather
// the tiling of get_tiles (raw.py:216-233) -- SURVEY.md §8f row 3, see below.
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

// The same with the tile held in registers: 1024 threads, float4 loads, every region
// element read once (the form above reads it three times with scalar loads: 157 us
// for the C5 region, 0.84 TB/s).  Needs tx, W multiples of 4 and ty * tx / 4 <= 1024 * KR.
constexpr int kR2tKR = 12;
__device__ __forceinline__ float block_sum1024(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; i += 2) s += red[i] + red[i + 1];
  __syncthreads();
  return s;
}
__global__ void __launch_bounds__(1024) region_to_tiles_reg_kernel(const float* __restrict__ region, int C, int H,
                                                                   int W, int ty, int tx, int gx,
                                                                   float* __restrict__ tiles, float* __restrict__ mean,
                                                                   float* __restrict__ stdv, int* __restrict__ bad) {
  __shared__ float red[16];
  const int c = blockIdx.x, t = blockIdx.y;
  const int y0 = (t / gx) * ty, x0 = (t % gx) * tx;
  const float* src = region + (size_t)c * H * W + (size_t)y0 * W + x0;
  const int tx4 = tx >> 2, n4 = ty * tx4, n = ty * tx;
  float4 v[kR2tKR];
  float s = 0.f;
  int nonfinite = 0;
#pragma unroll
  for (int j = 0; j < kR2tKR; ++j) {
    const int i = threadIdx.x + j * 1024;
    v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n4) {
      const int r = i / tx4, q = i - r * tx4;
      v[j] = *reinterpret_cast<const float4*>(src + (size_t)r * W + 4 * q);
      s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
      nonfinite |= !(isfinite(v[j].x) && isfinite(v[j].y) && isfinite(v[j].z) && isfinite(v[j].w));
    }
  }
  const float m = block_sum1024(s, red) / (float)n;
  float qs = 0.f;
#pragma unroll
  for (int j = 0; j < kR2tKR; ++j) {
    if (threadIdx.x + j * 1024 < n4) {
      const float a = v[j].x - m, b = v[j].y - m, cc = v[j].z - m, d = v[j].w - m;
      qs += (a * a + b * b) + (cc * cc + d * d);
    }
  }
  const float sd = sqrtf(block_sum1024(qs, red) / (float)n);
  const float inv = 1.f / sd;
  float4* dst = reinterpret_cast<float4*>(tiles + ((size_t)t * C + c) * n);
#pragma unroll
  for (int j = 0; j < kR2tKR; ++j) {
    const int i = threadIdx.x + j * 1024;
    if (i < n4) dst[i] = make_float4((v[j].x - m) * inv, (v[j].y - m) * inv, (v[j].z - m) * inv, (v[j].w - m) * inv);
  }
  const int anybad = __syncthreads_or(nonfinite);
  if (threadIdx.x == 0) {
    mean[(size_t)t * C + c] = m;
    stdv[(size_t)t * C + c] = sd;
    if (bad && anybad) atomicOr(&bad[t], 1);
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
  const bool reg = tx % 4 == 0 && W % 4 == 0 && (size_t)ty * (tx / 4) <= (size_t)1024 * kR2tKR &&
                   ((uintptr_t)region & 15) == 0 && ((uintptr_t)tiles & 15) == 0;
  if (reg)
    hipLaunchKernelGGL(region_to_tiles_reg_kernel, dim3(C, gy * gx), dim3(1024), 0, st, region, C, H, W, ty, tx, gx,
                       tiles, mean, stdv, bad);
  else
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

// the same, four pixels of one tile row per thread (tx % 4 == 0, 16-byte aligned):
// grid (ceil(gx tx / 1024), gy ty, C)
__global__ void __launch_bounds__(256) tiles_to_region_v4_kernel(const float* __restrict__ tiles,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ stdv,
                                                                 const int* __restrict__ inv, int C, int ty, int tx,
                                                                 int gx, float* __restrict__ out) {
  const int X = (blockIdx.x * 256 + threadIdx.x) * 4, Y = blockIdx.y, c = blockIdx.z;
  const int Wo = gx * tx;
  if (X >= Wo) return;
  const int cell = (Y / ty) * gx + X / tx;
  const int t = inv ? inv[cell] : cell;
  const float nan = __int_as_float(0x7fc00000);
  float4 v = make_float4(nan, nan, nan, nan);
  if (t >= 0) {
    v = *reinterpret_cast<const float4*>(tiles + (((size_t)t * C + c) * ty + (Y % ty)) * tx + (X % tx));
    if (mean) {
      const float sd = stdv[(size_t)t * C + c], m = mean[(size_t)t * C + c];
      v = make_float4(v.x * sd + m, v.y * sd + m, v.z * sd + m, v.w * sd + m);
    }
  }
  *reinterpret_cast<float4*>(out + ((size_t)c * gridDim.y + Y) * Wo + X) = v;
}

int tiles_to_region_launch(const float* tiles, const float* mean, const float* stdv, const int* inv, int C, int ty,
                           int tx, int gy, int gx, float* out, hipStream_t st) {
  if (C < 1 || ty < 1 || tx < 1 || gy < 1 || gx < 1) return SRMI_ERR_SHAPE;
  if (tx % 4 == 0 && ((uintptr_t)tiles & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(tiles_to_region_v4_kernel, dim3((gx * tx / 4 + 255) / 256, gy * ty, C), dim3(256), 0, st,
                       tiles, mean, stdv, inv, C, ty, tx, gx, out);
    SRMI_CHECK_LAUNCH();
    return 0;
  }
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

// ------------------------------------------------------------ LLC4320 source
// The reference expands a '>f4' wet-value file through a '>f4' mask template
// (13 nx^2 cells, 0 = land) on the host, then cuts the east | flipped-west
// image and the ROI.  Device version: the template -> ROI index map is built
// ONCE (the template is static): per-cell wet flags, a 3-kernel exclusive scan
// (block counts, one-block scan of the counts, block-local ranks), then each ROI
// pixel looks up the rank of its LLC cell.  Every time slice is then ONE
// gather: out[p] = bswap(data[idx[p]]) or NaN -- HBM-bound byte work.
constexpr int kScanThreads = 1024, kScanPer = 16, kScanBlk = kScanThreads * kScanPer;

__device__ __forceinline__ bool llc_wet(uint32_t be_word) {
  // file bytes are big-endian float32; "template != 0" (+-0 are land, NaN is wet)
  return (__builtin_bswap32(be_word) & 0x7fffffffu) != 0u;
}

__global__ void __launch_bounds__(kScanThreads) llc_count_kernel(const uint32_t* __restrict__ tmpl, long long n,
                                                                 int* __restrict__ blkcnt) {
  __shared__ int red[kScanThreads / 64];
  const long long base = (long long)blockIdx.x * kScanBlk + (long long)threadIdx.x * kScanPer;
  int c = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) c += (base + k < n) && llc_wet(tmpl[base + k]);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int i = 0; i < kScanThreads / 64; ++i) t += red[i];
    blkcnt[blockIdx.x] = t;
  }
}

// one block: blkoff[b] = sum_{i<b} blkcnt[i]; *total = sum
__global__ void __launch_bounds__(kScanThreads) llc_scan_counts_kernel(const int* __restrict__ blkcnt, int nb,
                                                                       long long* __restrict__ blkoff,
                                                                       long long* __restrict__ total) {
  __shared__ long long wsum[kScanThreads / 64];
  const int per = (nb + kScanThreads - 1) / kScanThreads;
  const int b0 = threadIdx.x * per;
  long long s = 0;
  for (int i = 0; i < per; ++i)
    if (b0 + i < nb) s += blkcnt[b0 + i];
  // exclusive scan of s over the block: wave inclusive scan + wave offsets
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long long inc = s;
  for (int o = 1; o < 64; o <<= 1) {
    const long long t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  long long woff = 0;
  for (int i = 0; i < w; ++i) woff += wsum[i];
  long long run = woff + inc - s;
  for (int i = 0; i < per; ++i)
    if (b0 + i < nb) {
      blkoff[b0 + i] = run;
      run += blkcnt[b0 + i];
    }
  if (threadIdx.x == kScanThreads - 1) *total = run;
}

// rank[i] = number of wet cells before i (wet i), -1 for land
__global__ void __launch_bounds__(kScanThreads) llc_rank_kernel(const uint32_t* __restrict__ tmpl, long long n,
                                                                const long long* __restrict__ blkoff,
                                                                int* __restrict__ rank) {
  __shared__ int wsum[kScanThreads / 64];
  const long long base = (long long)blockIdx.x * kScanBlk + (long long)threadIdx.x * kScanPer;
  uint32_t bits = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) bits |= (uint32_t)((base + k < n) && llc_wet(tmpl[base + k])) << k;
  const int c = __builtin_popcount(bits);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = c;
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int woff = 0;
  for (int i = 0; i < w; ++i) woff += wsum[i];
  long long r = blkoff[blockIdx.x] + woff + inc - c;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (base + k < n) {
      const bool wet = (bits >> k) & 1u;
      rank[base + k] = wet ? (int)r : -1;
      r += wet;
    }
  }
}

// ROI pixel (y, x) of the [3nx, 4nx] east | west.T[::-1] image -> LLC cell
__device__ __forceinline__ long long llc_cell(int Y, int X, int nx) {
  const long long n2 = (long long)nx * nx;
  if (X < nx) return (long long)Y * nx + X;
  if (X < 2 * nx) return 3 * n2 + (long long)Y * nx + (X - nx);
  return 7 * n2 + (long long)(X - 2 * nx) * 3 * nx + (3 * nx - 1 - Y);
}

__global__ void __launch_bounds__(256) llc_map_kernel(const int* __restrict__ rank, int nx, int y0, int ys, int x0,
                                                      int xs, int* __restrict__ idx) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long long)ys * xs) return;
  const int y = (int)(p / xs), x = (int)(p - (long long)y * xs);
  idx[p] = rank[llc_cell(y0 + y, x0 + x, nx)];
}

int llc_index_map_workspace(long long n, size_t* bytes) {
  if (n < 1) return SRMI_ERR_SHAPE;
  const long long nb = (n + kScanBlk - 1) / kScanBlk;
  *bytes = (size_t)n * 4 + (size_t)nb * 4 + (size_t)nb * 8 + 64;
  return 0;
}

int llc_index_map_launch(const uint32_t* tmpl, long long n, int nx, int y0, int ys, int x0, int xs, int* idx,
                         long long* n_wet, void* ws, size_t ws_bytes, hipStream_t st) {
  if (nx < 1 || n != 13LL * nx * nx || ys < 1 || xs < 1 || y0 < 0 || x0 < 0 || y0 + ys > 3 * nx ||
      x0 + xs > 4 * nx)
    return SRMI_ERR_SHAPE;
  size_t need = 0;
  llc_index_map_workspace(n, &need);
  if (!tmpl || !idx || !n_wet || !ws || ws_bytes < need) return SRMI_ERR_ARG;
  const long long nb = (n + kScanBlk - 1) / kScanBlk;
  char* w = static_cast<char*>(ws);
  int* rank = reinterpret_cast<int*>(w);
  long long* blkoff = reinterpret_cast<long long*>(w + (((size_t)n * 4 + 7) & ~(size_t)7));
  int* blkcnt = reinterpret_cast<int*>(reinterpret_cast<char*>(blkoff) + (size_t)nb * 8);
  hipLaunchKernelGGL(llc_count_kernel, dim3((unsigned)nb), dim3(kScanThreads), 0, st, tmpl, n, blkcnt);
  hipLaunchKernelGGL(llc_scan_counts_kernel, dim3(1), dim3(kScanThreads), 0, st, blkcnt, (int)nb, blkoff, n_wet);
  hipLaunchKernelGGL(llc_rank_kernel, dim3((unsigned)nb), dim3(kScanThreads), 0, st, tmpl, n, blkoff, rank);
  const long long np = (long long)ys * xs;
  hipLaunchKernelGGL(llc_map_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, rank, nx, y0, ys, x0, xs,
                     idx);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// out[p] = float(bswap(data[idx[p]])), NaN for land (idx < 0) or idx >= nvals
__global__ void __launch_bounds__(256) llc_gather_kernel(const uint32_t* __restrict__ data, long long nvals,
                                                         const int* __restrict__ idx, long long np,
                                                         float* __restrict__ out) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= np) return;
  const int i = idx[p];
  out[p] = (i >= 0 && i < nvals) ? __uint_as_float(__builtin_bswap32(data[i])) : __int_as_float(0x7fc00000);
}

int llc_gather_launch(const uint32_t* data, long long nvals, const int* idx, long long np, float* out,
                      hipStream_t st) {
  if (np < 1 || nvals < 0) return SRMI_ERR_SHAPE;
  if (!data || !idx || !out) return SRMI_ERR_ARG;
  hipLaunchKernelGGL(llc_gather_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, data, nvals, idx, np,
                     out);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// get_tiles' keep mask: bad[c * gy*gx + t] = 1 when tile t of channel c holds a
// non-finite value (its mean is then not finite).  grid (gy*gx, C)
__global__ void __launch_bounds__(256) tiles_nonfinite_kernel(const float* __restrict__ region, int H, int W, int ty,
                                                              int tx, int gx, int* __restrict__ bad) {
  const int t = blockIdx.x, c = blockIdx.y;
  const int y0 = (t / gx) * ty, x0 = (t % gx) * tx;
  const float* src = region + (size_t)c * H * W + (size_t)y0 * W + x0;
  int nf = 0;
  for (int i = threadIdx.x; i < ty * tx; i += 256) nf |= !isfinite(src[(size_t)(i / tx) * W + (i % tx)]);
  nf = __syncthreads_or(nf);
  if (threadIdx.x == 0) bad[(size_t)c * gridDim.x + t] = nf;
}

int tiles_nonfinite_launch(const float* region, int C, int H, int W, int ty, int tx, int* bad, hipStream_t st) {
  if (C < 1 || ty < 1 || tx < 1 || H < ty || W < tx) return SRMI_ERR_SHAPE;
  if (!region || !bad) return SRMI_ERR_ARG;
  hipLaunchKernelGGL(tiles_nonfinite_kernel, dim3((H / ty) * (W / tx), C), dim3(256), 0, st, region, H, W, ty, tx,
                     W / tx, bad);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// out plane m (= [m / C][m % C] of the [n/C][C][ty][tx] result) <- tile plane
// src[m] = c * gy*gx + t of the channel-major flattening.  grid (ceil(ty*tx/1024), nslots)
__global__ void __launch_bounds__(256) tiles_gather_kernel(const float* __restrict__ region, int H, int W, int ty,
                                                           int tx, int gx, int ntile, const int* __restrict__ src,
                                                           float* __restrict__ out) {
  const int m = blockIdx.y, j = src[m];
  const int c = j / ntile, t = j - c * ntile;
  const int y0 = (t / gx) * ty, x0 = (t % gx) * tx;
  const float* s = region + (size_t)c * H * W + (size_t)y0 * W + x0;
  float* d = out + (size_t)m * ty * tx;
  for (int i = blockIdx.x * 1024 + threadIdx.x; i < min(ty * tx, (int)(blockIdx.x + 1) * 1024); i += 256)
    d[i] = s[(size_t)(i / tx) * W + (i % tx)];
}

int tiles_gather_launch(const float* region, int C, int H, int W, int ty, int tx, const int* src, int nslots,
                        float* out, hipStream_t st) {
  if (C < 1 || ty < 1 || tx < 1 || H < ty || W < tx || nslots < 0) return SRMI_ERR_SHAPE;
  if (nslots == 0) return 0;
  if (!region || !src || !out) return SRMI_ERR_ARG;
  const int gx = W / tx, ntile = (H / ty) * gx;
  hipLaunchKernelGGL(tiles_gather_kernel, dim3((ty * tx + 1023) / 1024, nslots), dim3(256), 0, st, region, H, W, ty,
                     tx, gx, ntile, src, out);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
