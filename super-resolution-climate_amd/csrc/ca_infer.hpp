// The CA forward of one image from its conv1 output t (CALayer, sres/model/rcan/
// network.py:31-47), for a 512-thread workgroup: mean(u) of u = conv2(t) + b2 from t's
// statistics (linearity, rcab_infer.hip), then the MLP -> s.  Shared by the one-launch
// inference RCAB and the training conv2 launch (EPI_CA_RESID_U).  CA: any struct with
// part, nstrips, w1, b1, w2, b2, CR, wc2, bc2, rec.
#pragma once
#include "common.hpp"

namespace srmi {

constexpr int kCaScaleFloats = 1600;  // LDS scratch of ca_scale_from_t
constexpr int kCaScaleS = 1504;       // where it leaves s[64]

// the CA MLP of image n from m (LDS) -> z1, s (LDS) and the record (512 threads)
template <class CA>
__device__ __forceinline__ void ca_mlp(const CA& c, int n, float* m, float* z1, float* s) {
  constexpr int C = 64;
  const int tid = threadIdx.x, CR = c.CR, per = CR / 4;
  if (tid < 256) {  // z1[j] = b1[j] + W1[j] . m  (8 lanes per j)
    const int j = tid >> 3, pj = tid & 7, jc = min(j, CR - 1);
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += c.w1[jc * C + pj * 8 + i] * m[pj * 8 + i];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (j < CR && pj == 0) z1[j] = a + c.b1[j];
  }
  __syncthreads();
  if (tid < 256) {  // s[c] = sigmoid(b2[c] + W2[c] . relu(z1))  (4 lanes per c)
    const int c4 = tid >> 2, p4 = tid & 3;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) a += c.w2[c4 * CR + p4 * per + i] * fmaxf(z1[p4 * per + i], 0.f);
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (p4 == 0) s[c4] = 1.f / (1.f + expf(-(a + c.b2[c4])));
  }
  __syncthreads();
  if (c.rec) {
    float* r = c.rec + (size_t)n * (2 * C + CR);
    if (tid < C) {
      r[tid] = m[tid];
      r[C + CR + tid] = s[tid];
    }
    if (tid < CR) r[C + tid] = z1[tid];
  }
}

// v2 phase S for image n (512 threads, sm >= 1600 floats): mean(u) from t's statistics
// (the header), then the MLP; s lands in the record, where conv2's epilogue reads it
// wl: conv2's forward filter image in LDS ([9 taps][64 out rows][64 in] bf16, swz128
// chunks, as conv64_body loads it) for the matvec -- the weights conv2 itself uses --
// or null for the fp32 weights c.wc2 from global memory
template <class CA>
__device__ __forceinline__ void ca_scale_from_t(const CA& c, const bf16_t* t, int n, int H, int W, float* sm,
                                                const char* wl = nullptr) {
  constexpr int C = 64;
  const int tid = threadIdx.x, HW = H * W;
  float* red = sm;          // [4][64] strip-phase partials of T
  float* T = sm + 256;      // [64]
  float* bs = sm + 320;     // [4][64] sums of row 0, row H-1, column 0, column W-1
  float* cn = sm + 576;     // [4][64] corners (0,0) (0,W-1) (H-1,0) (H-1,W-1)
  float* St = sm + 832;     // [9][64]
  float* m = sm + 1408;     // [64]
  float* z1 = m + 64;       // [32]
  float* s = z1 + 32;       // [64]
  const bf16_t* tn = t + (size_t)n * HW * C;
  if (tid < 256) {  // T: conv1's per-strip sums, 4 strip phases, fixed order
    const int ch = tid & 63, ph = tid >> 6;
    float a = 0.f;
    for (int k = ph; k < c.nstrips; k += 4) a += c.part[((size_t)n * c.nstrips + k) * C + ch];
    red[ph * 64 + ch] = a;
    // corners
    const int y = (ph & 2) ? H - 1 : 0, x = (ph & 1) ? W - 1 : 0;
    cn[ph * 64 + ch] = bf2f(tn[((size_t)y * W + x) * C + ch]);
  }
  {  // border lines: line l = tid >> 7, channel group g (8 channels), positions j, j + 16, ...
    const int l = tid >> 7, g = (tid >> 4) & 7, j = tid & 15;
    const int len = l < 2 ? W : H;
    float a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.f;
    for (int q = j; q < len; q += 16) {
      const int y = l == 0 ? 0 : l == 1 ? H - 1 : q;
      const int x = l < 2 ? q : l == 2 ? 0 : W - 1;
      const uint4 v = *reinterpret_cast<const uint4*>(tn + ((size_t)y * W + x) * C + g * 8);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[2 * e] += bf2f(w[e] & 0xFFFFu);
        a[2 * e + 1] += bf2f(w[e] >> 16);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] += __shfl_xor(a[e], 1, 64);
      a[e] += __shfl_xor(a[e], 2, 64);
      a[e] += __shfl_xor(a[e], 4, 64);
      a[e] += __shfl_xor(a[e], 8, 64);
    }
    if (j == 0)
#pragma unroll
      for (int e = 0; e < 8; ++e) bs[l * 64 + g * 8 + e] = a[e];
  }
  __syncthreads();
  if (tid < C) T[tid] = (red[tid] + red[64 + tid]) + (red[128 + tid] + red[192 + tid]);
  __syncthreads();
  for (int i = tid; i < 9 * C; i += 512) {  // S_tap: tap (dy, dx) reads t[y + dy][x + dx]
    const int tap = i >> 6, ci = i & 63, dy = tap / 3 - 1, dx = tap % 3 - 1;
    float v = T[ci];
    if (dy == -1) v -= bs[64 + ci];   // row H-1 is never read
    if (dy == 1) v -= bs[ci];         // row 0
    if (dx == -1) v -= bs[192 + ci];  // column W-1
    if (dx == 1) v -= bs[128 + ci];   // column 0
    if (dy != 0 && dx != 0) v += cn[((dy == -1) ? 2 : 0) * 64 + ((dx == -1) ? 1 : 0) * 64 + ci];
    St[i] = v;
  }
  if (wl) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the caller's filter-image DMA (not compiler-tracked)
  __syncthreads();
  {  // m[c] = b2[c] + (1/HW) sum_{ci, tap} W2[c][ci][tap] S_tap[ci]: 8 lanes per c, 8 ci each
    const int co = tid >> 3, pc = tid & 7;
    float a = 0.f;
    if (wl) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const uint4 q = *reinterpret_cast<const uint4*>(wl + tap * 8192 + swz128(co, pc));
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
        const float* sv = St + tap * 64 + pc * 8;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a += bf2f(w[e] & 0xFFFFu) * sv[2 * e];
          a += bf2f(w[e] >> 16) * sv[2 * e + 1];
        }
      }
    } else {
      const float* wr = c.wc2 + ((size_t)co * C + pc * 8) * 9;  // 72 contiguous floats
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) a += wr[k * 9 + tap] * St[tap * 64 + pc * 8 + k];
    }
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (pc == 0) m[co] = c.bc2[co] + a / (float)HW;
  }
  __syncthreads();
  ca_mlp(c, n, m, z1, s);
}


}  // namespace srmi
