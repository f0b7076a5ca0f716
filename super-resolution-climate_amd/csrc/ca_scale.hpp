// The CA forward of one image from its conv1 output t (CALayer, sres/model/rcan/
// network.py:31-47), for a 512-thread workgroup: mean(u) of u = conv2(t) + b2 from t's
// statistics, then the MLP -> s.  By linearity
//   mean_p u[p][c] = b2[c] + (1/HW) sum_{tap, ci} W2[c][ci][tap] S_tap[ci],
//   S_tap[ci] = sum over the input pixels tap (dy, dx) reaches of t[.][ci]
//             = T[ci] - (row excluded by dy) - (column excluded by dx) + (their corner),
// so s is known before conv2 runs.  T comes from conv1's RELU_POOL epilogue, which sums
// the bf16-rounded t conv2 reads; the border lines and corners are read from the stored
// t; the matvec uses conv2's bf16 filter image in LDS -- the operands conv2's MFMAs
// use -- so m equals the mean of conv2's fp32 output up to fp32 summation order.
// Shared by the one-launch inference RCAB (rcab_infer.hip) and the training conv2
// launch (conv64_body EPI_CA_RESID_U, which computes its image's s in its prologue).
#pragma once
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

constexpr int kCaScaleFloats = 1600;  // LDS scratch of ca_scale_finish
constexpr int kCaScaleS = 1504;       // where it leaves s[64]
constexpr int kCaPreStrips = 4;       // strip sums per phase and ...
constexpr int kCaPreLine = 4;         // ... border pieces per lane held in registers

// one thread's global operands of the scale, issued ahead (before a conv prologue's
// DMA wait) so that their latency hides under it
struct CaScalePre {
  float tp[kCaPreStrips];  // tid < 256: strip sums k = ph, ph + 4, ... of channel tid & 63
  uint32_t cnr;            // tid < 256: corner ph of channel tid & 63 (bf16 bits)
  uint4 bl[kCaPreLine];    // border line l = tid >> 7, 8 channels, positions j, j + 16, ...
  float w1[8], w2[8];      // MLP weight slices (ca_scale_finish's lane groups)
  float b1, b2, bc2;
};

// (unconditional loads at clamped indices: no divergent branches around them, so the
//  compiler's vmcnt accounting stays exact)
__device__ __forceinline__ void ca_scale_load(const CaScale& c, int n, int H, int W, CaScalePre& q) {
  constexpr int C = 64;
  const int tid = threadIdx.x, ch = tid & 63, ph = (tid >> 6) & 3, CR = c.CR, per = CR / 4;
  const float* pp = c.part + (size_t)n * c.nstrips * C + ch;
#pragma unroll
  for (int i = 0; i < kCaPreStrips; ++i) q.tp[i] = pp[(size_t)min(ph + 4 * i, c.nstrips - 1) * C];
  const bf16_t* tn = c.t + (size_t)n * H * W * C;
  {
    const int y = (ph & 2) ? H - 1 : 0, x = (ph & 1) ? W - 1 : 0;
    q.cnr = tn[((size_t)y * W + x) * C + ch];
  }
  {
    const int l = tid >> 7, g = (tid >> 4) & 7, j = tid & 15, len = l < 2 ? W : H;
#pragma unroll
    for (int i = 0; i < kCaPreLine; ++i) {
      const int pos = min(j + 16 * i, len - 1);
      const int y = l == 0 ? 0 : l == 1 ? H - 1 : pos, x = l < 2 ? pos : l == 2 ? 0 : W - 1;
      q.bl[i] = *reinterpret_cast<const uint4*>(tn + ((size_t)y * W + x) * C + g * 8);
    }
  }
  const int jc = min(tid >> 3, CR - 1), pj = tid & 7;  // z1 lane group (8 lanes per j)
  const int c4 = (tid >> 2) & 63, p4 = tid & 3;        // s lane group (4 lanes per c)
#pragma unroll
  for (int i = 0; i < 8; ++i) q.w1[i] = c.w1[jc * C + pj * 8 + i];
#pragma unroll
  for (int i = 0; i < 8; ++i) q.w2[i] = c.w2[c4 * CR + p4 * per + min(i, per - 1)];
  q.b1 = c.b1[jc];
  q.b2 = c.b2[c4];
  q.bc2 = c.bc2[(tid >> 3) & 63];
}

// The scale of image n from the preloaded operands, 512 threads (sm >= kCaScaleFloats
// floats of LDS scratch, s left at sm + kCaScaleS).  wl: conv2's forward filter image in
// LDS ([9 taps][64 out rows][64 in] bf16, chunk-swizzled as the conv body loads it:
// swz128, or swz128t with TSW), landed and published by the caller's barrier.  The
// record m | z1 | s goes to c.rec[n] when `write_rec`.
template <bool TSW = false>
__device__ __forceinline__ void ca_scale_finish(const CaScale& c, const CaScalePre& q, int n, int H, int W, float* sm,
                                                const char* wl, bool write_rec) {
  constexpr int C = 64;
  const int tid = threadIdx.x, HW = H * W, CR = c.CR, per = CR / 4;
  float* red = sm;          // [4][64] strip-phase partials of T
  float* T = sm + 256;      // [64]
  float* bs = sm + 320;     // [4][64] sums of row 0, row H-1, column 0, column W-1
  float* cn = sm + 576;     // [4][64] corners (0,0) (0,W-1) (H-1,0) (H-1,W-1)
  float* St = sm + 832;     // [9][64]
  float* m = sm + 1408;     // [64]
  float* z1 = m + 64;       // [32]
  float* s = z1 + 32;       // [64]
  const bf16_t* tn = c.t + (size_t)n * HW * C;
  if (tid < 256) {  // T: conv1's per-strip sums, 4 strip phases, fixed order
    const int ch = tid & 63, ph = tid >> 6;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < kCaPreStrips; ++i)
      if (ph + 4 * i < c.nstrips) a += q.tp[i];
    for (int k = ph + 4 * kCaPreStrips; k < c.nstrips; k += 4) a += c.part[((size_t)n * c.nstrips + k) * C + ch];
    red[ph * 64 + ch] = a;
    cn[ph * 64 + ch] = bf2f((bf16_t)q.cnr);
  }
  {  // border lines: line l = tid >> 7, channel group g (8 channels), positions j, j + 16, ...
    const int l = tid >> 7, g = (tid >> 4) & 7, j = tid & 15;
    const int len = l < 2 ? W : H;
    float a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.f;
    auto add = [&](const uint4& v) __attribute__((always_inline)) {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[2 * e] += bf2f(w[e] & 0xFFFFu);
        a[2 * e + 1] += bf2f(w[e] >> 16);
      }
    };
#pragma unroll
    for (int i = 0; i < kCaPreLine; ++i)
      if (j + 16 * i < len) add(q.bl[i]);
    for (int pos = j + 16 * kCaPreLine; pos < len; pos += 16) {
      const int y = l == 0 ? 0 : l == 1 ? H - 1 : pos, x = l < 2 ? pos : l == 2 ? 0 : W - 1;
      add(*reinterpret_cast<const uint4*>(tn + ((size_t)y * W + x) * C + g * 8));
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
  __syncthreads();
  {  // m[c] = b2[c] + (1/HW) sum_{ci, tap} W2[c][ci][tap] S_tap[ci]: 8 lanes per c, 8 ci each
    const int co = tid >> 3, pc = tid & 7;
    float a = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const uint32_t off = TSW ? swz128t(co, pc) : swz128(co, pc);
      const uint4 v = *reinterpret_cast<const uint4*>(wl + tap * 8192 + off);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const float* sv = St + tap * 64 + pc * 8;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a += bf2f(w[e] & 0xFFFFu) * sv[2 * e];
        a += bf2f(w[e] >> 16) * sv[2 * e + 1];
      }
    }
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (pc == 0) m[co] = q.bc2 + a / (float)HW;
  }
  __syncthreads();
  if (tid < 256) {  // z1[j] = b1[j] + W1[j] . m  (8 lanes per j)
    const int j = tid >> 3, pj = tid & 7;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += q.w1[i] * m[pj * 8 + i];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (j < CR && pj == 0) z1[j] = a + q.b1;
  }
  __syncthreads();
  if (tid < 256) {  // s[c] = sigmoid(b2[c] + W2[c] . relu(z1))  (4 lanes per c)
    const int c4 = tid >> 2, p4 = tid & 3;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) a += q.w2[i] * fmaxf(z1[p4 * per + i], 0.f);
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (p4 == 0) s[c4] = 1.f / (1.f + expf(-(a + q.b2)));
  }
  __syncthreads();
  if (write_rec) {
    float* r = c.rec + (size_t)n * (2 * C + CR);
    if (tid < C) {
      r[tid] = m[tid];
      r[C + CR + tid] = s[tid];
    }
    if (tid < CR) r[C + tid] = z1[tid];
  }
}

}  // namespace srmi
