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
// (conv1 writing the border sums into its strip records instead measured -2 % in C5:
// its epilogue grew by ~1 K cycles per strip, more than the border reads cost here.)
// Shared by the one-launch inference RCAB (rcab_infer.hip) and the training conv2
// launch (conv64_body EPI_CA_RESID_U, which computes its image's s in its prologue).
#pragma once
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

#ifdef SRMI_STAMPS
#define CSTAMP(i)                                                                                           \
  do {                                                                                                      \
    if (c.stamps && threadIdx.x == 0) c.stamps[blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memtime();       \
  } while (0)
#else
#define CSTAMP(i) \
  do {            \
  } while (0)
#endif

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
  float w1[32];            // W1 rows j = 8 r + (lane >> 3), r < 4, inputs 8 (lane & 7) .. + 7 (z1)
  float b1[4];             // b1 of those rows
  float w2[8];             // W2 row c = tid >> 2, its quarter tid & 3 of the CR inputs (s)
  float b2, bc2;
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
  const int lane = tid & 63, jj = lane >> 3, pj = lane & 7;  // z1 lanes: 8 per row, 8 rows per round
  const int c4 = (tid >> 2) & 63, p4 = tid & 3;             // s lanes (4 per c)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = min(8 * r + jj, CR - 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) q.w1[8 * r + i] = c.w1[j * C + pj * 8 + i];
    q.b1[r] = c.b1[j];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) q.w2[i] = c.w2[c4 * CR + p4 * per + min(i, per - 1)];
  q.b2 = c.b2[c4];
  q.bc2 = c.bc2[(tid >> 3) & 63];
}

// sum over the 8 lanes of an aligned group (DPP: quad swaps, then the half-row mirror)
__device__ __forceinline__ float sum8(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  return v;
}

// The scale of image n from the preloaded operands, 512 threads (sm >= kCaScaleFloats
// floats of LDS scratch, s left at sm + kCaScaleS).  wl: conv2's forward filter image in
// LDS ([9 taps][64 out rows][64 in] bf16, chunk-swizzled as the conv body loads it:
// swz128, or swz128t with TSW), landed and published by the caller's barrier.  The
// record m | z1 | s goes to c.rec[n] when `write_rec`.  Three workgroup barriers:
//   1. T's strip-phase partials, the border-line sums (DPP) and the corners -> LDS
//   2. every lane (co, 8 ci): S_tap of its 8 ci from those, the matvec slice on the
//      filter image, summed over the 8 lanes of co -> m[co]
//   3. waves 0-3 each: all of z1 = W1 m + b1 (8 lanes per j, 8 rows per round), then
//      s for its 16 channels (4 lanes per c) -- wave-local, no barrier in between -> s
template <bool TSW = false>
__device__ __forceinline__ void ca_scale_finish(const CaScale& c, const CaScalePre& q, int n, int H, int W, float* sm,
                                                const char* wl, bool write_rec) {
  constexpr int C = 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, HW = H * W, CR = c.CR, per = CR / 4;
  float* red = sm;          // [4][64] strip-phase partials of T
  float* bs = sm + 256;     // [4][64] sums of row 0, row H-1, column 0, column W-1
  float* cn = sm + 512;     // [4][64] corners (0,0) (0,W-1) (H-1,0) (H-1,W-1)
  float* m = sm + 768;      // [64]
  float* z1w = sm + 832;    // [4 waves][32]
  float* s = sm + kCaScaleS;  // [64]
  static_assert(kCaScaleS >= 832 + 128 && kCaScaleS + 64 <= kCaScaleFloats, "scale scratch");
  const bf16_t* tn = c.t + (size_t)n * HW * C;
  CSTAMP(0);
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
    for (int e = 0; e < 8; ++e) a[e] = sum16(a[e]);  // over j (the lane's 16-lane DPP row)
    if (j == 0) {
      float4* d = reinterpret_cast<float4*>(bs + l * 64 + g * 8);
      d[0] = make_float4(a[0], a[1], a[2], a[3]);
      d[1] = make_float4(a[4], a[5], a[6], a[7]);
    }
  }
  CSTAMP(1);
  __syncthreads();
  CSTAMP(2);
  {  // m[co] = b2[co] + (1/HW) sum_{ci, tap} W2[co][ci][tap] S_tap[ci]: 8 lanes per co, 8 ci each
    const int co = tid >> 3, pc = tid & 7;
    float T[8], b[4][8], k[4][8];  // T; border sums of row 0, row H-1, column 0, column W-1; corners
    auto ld8 = [&](const float* src, float (&d)[8]) __attribute__((always_inline)) {
      const float4 x = *reinterpret_cast<const float4*>(src), y = *reinterpret_cast<const float4*>(src + 4);
      d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w; d[4] = y.x; d[5] = y.y; d[6] = y.z; d[7] = y.w;
    };
    auto sum4 = [&](const float* src, float (&d)[8]) __attribute__((always_inline)) {  // the 4 phases, fixed order
      float r[4][8];
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) ld8(src + ph * 64 + pc * 8, r[ph]);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = (r[0][e] + r[1][e]) + (r[2][e] + r[3][e]);
    };
    sum4(red, T);
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      ld8(bs + l * 64 + pc * 8, b[l]);
      ld8(cn + l * 64 + pc * 8, k[l]);
    }
    float a = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {  // tap (dy, dx) reads t[y + dy][x + dx]
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const uint32_t off = TSW ? swz128t(co, pc) : swz128(co, pc);
      const uint4 v = *reinterpret_cast<const uint4*>(wl + tap * 8192 + off);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float sv = T[e];
        if (dy == -1) sv -= b[1][e];  // row H-1 is never read
        if (dy == 1) sv -= b[0][e];   // row 0
        if (dx == -1) sv -= b[3][e];  // column W-1
        if (dx == 1) sv -= b[2][e];   // column 0
        if (dy != 0 && dx != 0) sv += k[(dy == -1 ? 2 : 0) + (dx == -1 ? 1 : 0)][e];
        const float wv = (e & 1) ? bf2f(w[e >> 1] >> 16) : bf2f(w[e >> 1] & 0xFFFFu);
        a += wv * sv;
      }
    }
    a = sum8(a);
    if (pc == 0) m[co] = q.bc2 + a / (float)HW;
  }
  CSTAMP(3);
  __syncthreads();
  CSTAMP(4);
  if (wave < 4) {  // the CA MLP, wave-local: all of z1 in every wave, then its 16 channels of s
    const int jj = lane >> 3, pj = lane & 7;
    const float4 m0 = *reinterpret_cast<const float4*>(m + pj * 8);
    const float4 m1 = *reinterpret_cast<const float4*>(m + pj * 8 + 4);
    const float mv[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    float* z = z1w + wave * 32;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) a += q.w1[8 * r + i] * mv[i];
      a = sum8(a);
      if (pj == 0 && 8 * r + jj < CR) z[8 * r + jj] = a + q.b1[r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's z1 writes before its reads
    const int p4 = lane & 3;  // s[c], c = tid >> 2: quarter p4 of the CR inputs
    float b = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) b += q.w2[i] * fmaxf(z[p4 * per + i], 0.f);
    b += dpp_mov<0xB1>(b);
    b += dpp_mov<0x4E>(b);
    if (p4 == 0) s[tid >> 2] = 1.f / (1.f + expf(-(b + q.b2)));
  }
  CSTAMP(5);
  __syncthreads();
  CSTAMP(6);
  if (write_rec) {
    float* r = c.rec + (size_t)n * (2 * C + CR);
    if (tid < C) {
      r[tid] = m[tid];
      r[C + CR + tid] = s[tid];
    }
    if (tid < CR) r[C + tid] = z1w[tid];
  }
}

}  // namespace srmi
