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
// launch (conv64_body EPI_CA_RESID_U, which computes its image's s between its first
// strip's MFMAs and epilogue).
#pragma once
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

#if defined(SRMI_STAMPS) && !defined(SRMI_NO_CSTAMP)  // (SRMI_NO_CSTAMP: the body's stamps only)
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

// one thread's global operands of the scale, issued ahead so that their latency hides
// under other work (the inference RCAB: its prologue's DMA wait; the training conv2:
// its first strip's MFMAs)
struct CaScalePre {
  float tp[kCaPreStrips];  // tid < 256: strip sums k = ph, ph + 4, ... of channel tid & 63
  uint32_t cnr;            // tid < 256: corner ph of channel tid & 63 (bf16 bits)
  uint4 bl[kCaPreLine];    // border line l = tid >> 7, 8 channels, positions j, j + 16, ...
  float w1[4];             // W1 row j = tid >> 4, inputs 4 (tid & 15) .. + 3 (z1)
  float b1;                // b1[j]
  float w2[4];             // W2 row c = tid >> 3, inputs (tid & 7) + 8 i (s)
  float b2, bc2;
  float bcm;               // (the partial-mean path) conv2's bias of channel tid & 63
};

// (unconditional loads at clamped indices: no divergent branches around them, so the
//  compiler's vmcnt accounting stays exact)
// The operands in two parts: what conv1 wrote (strip sums, border lines, corners: the
// latency that matters) and the CA parameters (L2-resident, read by every workgroup).
__device__ __forceinline__ void ca_scale_load_t(const CaScale& c, int n, int H, int W, CaScalePre& q) {
  constexpr int C = 64;
  const int tid = threadIdx.x, ch = tid & 63, ph = (tid >> 6) & 3;
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
}
// (an opaque copy of the thread index: the lane-dependent offsets derived from it stay
//  where they are used instead of being hoisted out of the conv body's strip loop,
//  where they would hold registers across every strip's MFMAs)
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ void ca_scale_load_params(const CaScale& c, CaScalePre& q) {
  constexpr int C = 64;
  const int tid = opaque_tid(), CR = c.CR;
  const int j = min(tid >> 4, CR - 1), i4 = 4 * (tid & 15);  // z1 lanes: 16 per row j
  const int c8 = tid >> 3, q8 = tid & 7;                     // s lanes: 8 per channel c
#pragma unroll
  for (int i = 0; i < 4; ++i) q.w1[i] = c.w1[j * C + i4 + i];
  q.b1 = c.b1[j];
#pragma unroll
  for (int i = 0; i < 4; ++i) q.w2[i] = c.w2[c8 * CR + min(q8 + 8 * i, CR - 1)];
  q.b2 = c.b2[c8];
  q.bc2 = c.bc2[c8];
}

// The partial-mean path (training, SRMI_CA_MPART): conv1's workgroups leave their share of
// the matvec in c.mpart [N][nruns][64]; conv2 issues the first kCaPreStrips of them (and
// its bias) ahead, in q.tp / q.bcm (channel tid & 63)
__device__ __forceinline__ void ca_mpart_load(const CaScale& c, int n, CaScalePre& q) {
  const int ch = threadIdx.x & 63;
  const float* mp = c.mpart + (size_t)n * c.nruns * 64 + ch;
#pragma unroll
  for (int i = 0; i < kCaPreStrips; ++i) q.tp[i] = mp[(size_t)min(i, c.nruns - 1) * 64];
  q.bcm = c.bc2[ch];
}

// sum over the 8 lanes of an aligned group (DPP: quad swaps, then the half-row mirror)
__device__ __forceinline__ float sum8(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  return v;
}

// sum_{ci, tap} W2[co][ci][tap] S_tap[ci], co = tid >> 3 (8 lanes per co, 8 ci each, in
// two halves of 4 ci: the training conv2 runs this with a strip's accumulators live, a
// half's operands are 36 registers), summed over those 8 lanes.  S_tap from T (four
// partials, summed in fixed order), the border-line sums bs (row 0, row H-1, column 0,
// column W-1) and the corners cn ((0,0) (0,W-1) (H-1,0) (H-1,W-1)), each [64] in LDS;
// wv: the lane's slices of conv2's bf16 filter image (ca_matvec_load_w), in registers.
// (conv1's run end: its share of the mean, SRMI_CA_MPART)
__device__ __forceinline__ void ca_matvec_load_w(const bf16_t* wimg, int tid, uint2 (&wv)[2][9]) {
  const int co = tid >> 3, pc = tid & 7;  // W2[co][ci][tap] at wimg[(tap * 64 + co) * 64 + ci]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
      wv[h][tap] = *reinterpret_cast<const uint2*>(wimg + ((size_t)(tap * 64 + co)) * 64 + pc * 8 + 4 * h);
}
__device__ __forceinline__ float ca_matvec(const float* red, const float* bs, const float* cn,
                                           const uint2 (&wv)[2][9], int tid) {
  {
    const int pc = tid & 7;
    float a = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c0 = pc * 8 + 4 * h;
      float T[4], b[4][4], k[4][4];  // T; border sums of row 0, row H-1, column 0, column W-1; corners
      auto ld4 = [&](const float* src, float (&d)[4]) __attribute__((always_inline)) {
        const float4 x = *reinterpret_cast<const float4*>(src);
        d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
      };
      {
        float r[4][4];  // the 4 phases, fixed order
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) ld4(red + ph * 64 + c0, r[ph]);
#pragma unroll
        for (int e = 0; e < 4; ++e) T[e] = (r[0][e] + r[1][e]) + (r[2][e] + r[3][e]);
      }
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        ld4(bs + l * 64 + c0, b[l]);
        ld4(cn + l * 64 + c0, k[l]);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {  // tap (dy, dx) reads t[y + dy][x + dx]
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const uint32_t w[2] = {wv[h][tap].x, wv[h][tap].y};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sv = T[e];
          if (dy == -1) sv -= b[1][e];  // row H-1 is never read
          if (dy == 1) sv -= b[0][e];   // row 0
          if (dx == -1) sv -= b[3][e];  // column W-1
          if (dx == 1) sv -= b[2][e];   // column 0
          if (dy != 0 && dx != 0) sv += k[(dy == -1 ? 2 : 0) + (dx == -1 ? 1 : 0)][e];
          const float we = (e & 1) ? bf2f(w[e >> 1] >> 16) : bf2f(w[e >> 1] & 0xFFFFu);
          a += we * sv;
        }
      }
    }
    return sum8(a);
  }
}

// z1 = W1 m + b1 (16 lanes per row j, 4 inputs each, DPP row sum), a barrier, then
// s = sigmoid(W2 relu(z1) + b2) (8 lanes per channel c): m, z1, s in LDS, q's MLP slices
__device__ __forceinline__ void ca_mlp(const CaScale& c, const CaScalePre& q, const float* m, float* z1, float* s,
                                       int tid) {
  const int CR = c.CR;
  {
    const int j = tid >> 4, i4 = 4 * (tid & 15);
    const float4 mv = *reinterpret_cast<const float4*>(m + i4);
    float a = q.w1[0] * mv.x + q.w1[1] * mv.y + q.w1[2] * mv.z + q.w1[3] * mv.w;
    a = sum16(a);
    if ((tid & 15) == 0 && j < CR) z1[j] = a + q.b1;
  }
  CSTAMP(5);
  __syncthreads();
  {
    const int q8 = tid & 7;
    float b = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (q8 + 8 * i < CR) b += q.w2[i] * fmaxf(z1[q8 + 8 * i], 0.f);
    b = sum8(b);
    if (q8 == 0) s[tid >> 3] = 1.f / (1.f + expf(-(b + q.b2)));
  }
}

// The scale of image n from conv1's partial means (q from ca_mpart_load and
// ca_scale_load_params): m = b2 + (1/HW) sum over the runs in run order, then the MLP;
// three barriers, s left at sm + kCaScaleS, the record m | z1 | s when `write_rec`.
__device__ __forceinline__ void ca_scale_from_mpart(const CaScale& c, const CaScalePre& q0, int n, int HW, float* sm,
                                                    bool write_rec) {
  CaScalePre q = q0;  // (opaque: see ca_scale_finish)
#pragma unroll
  for (int i = 0; i < kCaPreStrips; ++i) asm volatile("" : "+v"(q.tp[i]));
  asm volatile("" : "+v"(q.bcm));
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(q.w1[i]), "+v"(q.w2[i]));
  asm volatile("" : "+v"(q.b1), "+v"(q.b2));
  constexpr int C = 64;
  const int tid = opaque_tid(), CR = c.CR;
  float* m = sm + 768;
  float* z1 = sm + 832;
  float* s = sm + kCaScaleS;
  CSTAMP(0);
  if (tid < C) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < kCaPreStrips; ++i)
      if (i < c.nruns) a += q.tp[i];
    for (int r = kCaPreStrips; r < c.nruns; ++r) a += c.mpart[((size_t)n * c.nruns + r) * C + tid];
    m[tid] = q.bcm + a / (float)HW;
  }
  CSTAMP(3);
  __syncthreads();
  CSTAMP(4);
  ca_mlp(c, q, m, z1, s, tid);
  CSTAMP(6);
  __syncthreads();
  CSTAMP(7);
  if (write_rec) {
    float* r = c.rec + (size_t)n * (2 * C + CR);
    if (tid < C) {
      r[tid] = m[tid];
      r[C + CR + tid] = s[tid];
    }
    if (tid < CR) r[C + tid] = z1[tid];
  }
}

// The scale of image n from the preloaded operands, 512 threads (sm >= kCaScaleFloats
// floats of LDS scratch, s left at sm + kCaScaleS).  wl: conv2's forward filter image in
// LDS ([9 taps][64 out rows][64 in] bf16, chunk-swizzled as the conv body loads it:
// swz128, or swz128t with TSW), landed and published by the caller's barrier.  The
// record m | z1 | s goes to c.rec[n] when `write_rec`.  Four workgroup barriers:
//   1. T's strip-phase partials, the border-line sums (DPP) and the corners -> LDS
//   2. every lane (co, 8 ci): S_tap of its 8 ci from those, the matvec slice on the
//      filter image, summed over the 8 lanes of co -> m[co]
//   3. z1 = W1 m + b1 (16 lanes per j, 4 inputs each, DPP row sum)
//   4. s = sigmoid(W2 relu(z1) + b2) (8 lanes per c) -> s
// (every phase on all 512 lanes, a few operand registers each: the training conv2 runs
//  this between its first strip's MFMAs and epilogue, with the accumulators live)
template <bool TSW = false>
__device__ __forceinline__ void ca_scale_finish(const CaScale& c, const CaScalePre& q0, int n, int H, int W, float* sm,
                                                const char* wl, bool write_rec) {
  // (the preloaded t operands pass through an empty asm here: the compiler would
  //  otherwise hoist their first uses -- and the wait for them -- out of the training
  //  conv2's strip loop, to the point where they are issued)
  CaScalePre q = q0;
#pragma unroll
  for (int i = 0; i < kCaPreStrips; ++i) asm volatile("" : "+v"(q.tp[i]));
  asm volatile("" : "+v"(q.cnr));
#pragma unroll
  for (int i = 0; i < kCaPreLine; ++i) asm volatile("" : "+v"(q.bl[i].x), "+v"(q.bl[i].y), "+v"(q.bl[i].z), "+v"(q.bl[i].w));
  constexpr int C = 64;
  const int tid = opaque_tid(), HW = H * W, CR = c.CR;
  float* red = sm;          // [4][64] strip-phase partials of T
  float* bs = sm + 256;     // [4][64] sums of row 0, row H-1, column 0, column W-1
  float* cn = sm + 512;     // [4][64] corners (0,0) (0,W-1) (H-1,0) (H-1,W-1)
  float* m = sm + 768;      // [64]
  float* z1 = sm + 832;     // [32]
  float* s = sm + kCaScaleS;  // [64]
  static_assert(kCaScaleS >= 832 + 32 && kCaScaleS + 64 <= kCaScaleFloats, "scale scratch");
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
  {  // m[co] = b2[co] + (1/HW) sum_{ci, tap} W2[co][ci][tap] S_tap[ci]: 8 lanes per co, 8 ci
     // each, in two halves of 4 ci (the training conv2 runs this with a strip's
     // accumulators live: a half's operands are 36 registers)
    const int co = tid >> 3, pc = tid & 7;
    const uint32_t off = TSW ? swz128t(co, pc) : swz128(co, pc);
    float a = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c0 = pc * 8 + 4 * h;
      float T[4], b[4][4], k[4][4];  // T; border sums of row 0, row H-1, column 0, column W-1; corners
      auto ld4 = [&](const float* src, float (&d)[4]) __attribute__((always_inline)) {
        const float4 x = *reinterpret_cast<const float4*>(src);
        d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
      };
      {
        float r[4][4];  // the 4 phases, fixed order
#pragma unroll
        for (int ph = 0; ph < 4; ++ph) ld4(red + ph * 64 + c0, r[ph]);
#pragma unroll
        for (int e = 0; e < 4; ++e) T[e] = (r[0][e] + r[1][e]) + (r[2][e] + r[3][e]);
      }
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        ld4(bs + l * 64 + c0, b[l]);
        ld4(cn + l * 64 + c0, k[l]);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {  // tap (dy, dx) reads t[y + dy][x + dx]
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const uint2 v = *reinterpret_cast<const uint2*>(wl + tap * 8192 + off + 8 * h);
        const uint32_t w[2] = {v.x, v.y};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
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
    }
    a = sum8(a);
    if (pc == 0) m[co] = q.bc2 + a / (float)HW;
  }
  CSTAMP(3);
  __syncthreads();
  CSTAMP(4);
  {  // z1 = W1 m + b1: 16 lanes per row j (4 inputs each), summed over the lane's DPP row
    const int j = tid >> 4, i4 = 4 * (tid & 15);
    const float4 mv = *reinterpret_cast<const float4*>(m + i4);
    float a = q.w1[0] * mv.x + q.w1[1] * mv.y + q.w1[2] * mv.z + q.w1[3] * mv.w;
    a = sum16(a);
    if ((tid & 15) == 0 && j < CR) z1[j] = a + q.b1;
  }
  CSTAMP(5);
  __syncthreads();
  {  // s = sigmoid(W2 relu(z1) + b2): 8 lanes per channel c, inputs q + 8 i
    const int q8 = tid & 7;
    float b = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (q8 + 8 * i < CR) b += q.w2[i] * fmaxf(z1[q8 + 8 * i], 0.f);
    b = sum8(b);
    if (q8 == 0) s[tid >> 3] = 1.f / (1.f + expf(-(b + q.b2)));
  }
  CSTAMP(6);
  __syncthreads();
  CSTAMP(7);
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
