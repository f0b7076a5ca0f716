// The CALayer backward's MLP of one image (reference sres/model/rcan/network.py:31-47,
// differentiated): from sum_p g and sum_p g u over the image (the per-strip sums F1 wrote)
// and the forward record m | z1 | s,
//   ds = sum_p g u,  dz2 = ds s (1 - s),  dz1 = relu'(z1) W2^T dz2,  dm = W1^T dz1,
// so that du = g s + dm / HW.  Shared by the CA backward launch (small.hip ca_bwd_du_kernel)
// and the fused conv2 backward that forms du from g itself (conv64_body_defer, wgrad48_body):
// one thread mapping, summation order and arithmetic, hence the same dm bit for bit.
//
// MLP threads t = 0..255 (any 4 waves of the block: t & 63 must be the lane); every
// thread of the block calls ca_bwd_mlp (it holds 4 barriers), t < 0 for the others.
#pragma once
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

// LDS scratch of ca_bwd_mlp (floats): red [2][128] | s [64] | dz2 [64] | dz1 [32] | dm [64]
constexpr int kCaBwdS = 256, kCaBwdDz2 = 320, kCaBwdDz1 = 384, kCaBwdDm = 416, kCaBwdScratch = 480;
constexpr int kCaBwdKU = 8;  // strip records loaded at once per thread (more: loaded in the finish)

struct CaBwdPre {
  float pv[kCaBwdKU];  // the strip records of channel sum t & 127, strips (t >> 7) + 2 i
  float wa[8], wb[8];  // W2 column slice (dz1 lane group t >> 3), W1 column slice (dm lane group t >> 2)
  float zj, svl;
};

__device__ __forceinline__ void ca_bwd_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// the operands of MLP thread t of image n (issued at once, consumed by ca_bwd_mlp)
__device__ __forceinline__ void ca_bwd_load(const CaBwdIn& c, int n, int t, CaBwdPre& q) {
  constexpr int C = 64;
  const int CR = c.CR, per = CR / 4;
  const int j = t >> 3, pj = t & 7, c4 = t >> 2, p4 = t & 3, jc = min(j, CR - 1);
  const float* pp = c.part + (size_t)n * c.nstrips * (2 * C) + (t & 127);
#pragma unroll
  for (int i = 0; i < kCaBwdKU; ++i) q.pv[i] = pp[(size_t)min((t >> 7) + 2 * i, c.nstrips - 1) * (2 * C)];
#pragma unroll
  for (int i = 0; i < 8; ++i) q.wa[i] = c.w2[(pj * 8 + i) * CR + jc];
#pragma unroll
  for (int i = 0; i < 8; ++i) q.wb[i] = c.w1[(p4 * per + min(i, per - 1)) * C + c4];
  const float* r = c.rec + (size_t)n * (2 * C + CR);
  q.zj = r[C + jc];
  q.svl = r[C + CR + (t & 63)];
}

// The MLP; sm = LDS scratch (kCaBwdScratch floats): on return (after its last barrier)
// sm + kCaBwdS holds s and sm + kCaBwdDm holds dm of the image.  wr: this block writes the
// image's brec record (dz2 | dz1 | sum_p du) and dm.
__device__ __forceinline__ void ca_bwd_mlp(const CaBwdIn& c, int n, int t, const CaBwdPre& q, float* sm, bool wr) {
  constexpr int C = 64;
  const int CR = c.CR, per = CR / 4;
  const bool on = t >= 0 && t < 256;
  const int j = t >> 3, pj = t & 7, c4 = t >> 2, p4 = t & 3;
  float* red = sm;
  float* s = sm + kCaBwdS;
  float* dz2 = sm + kCaBwdDz2;
  float* dz1 = sm + kCaBwdDz1;
  float* dm = sm + kCaBwdDm;
  if (on) {  // G[c] = sum_p g, ds[c] = sum_p g u: strips of one parity in order, then the two parities
    float pa = 0.f;
#pragma unroll
    for (int i = 0; i < kCaBwdKU; ++i)
      if ((t >> 7) + 2 * i < c.nstrips) pa += q.pv[i];
    const float* pp = c.part + (size_t)n * c.nstrips * (2 * C) + (t & 127);
    for (int k = (t >> 7) + 2 * kCaBwdKU; k < c.nstrips; k += 2) pa += pp[(size_t)k * (2 * C)];
    red[(t >> 7) * 128 + (t & 127)] = pa;
    s[t & 63] = q.svl;
  }
  ca_bwd_lds_barrier();
  float G = 0.f, sv = 0.f;
  if (on && t < C) {
    G = red[t] + red[128 + t];
    const float ds = red[C + t] + red[128 + C + t];
    sv = s[t];
    dz2[t] = ds * sv * (1.f - sv);
  }
  ca_bwd_lds_barrier();
  if (on) {  // dz1[j] = relu'(z1[j]) sum_c W2[c][j] dz2[c]
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += q.wa[i] * dz2[pj * 8 + i];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (j < CR && pj == 0) dz1[j] = (q.zj > 0.f) ? a : 0.f;
  }
  ca_bwd_lds_barrier();
  if (on) {  // dm[c] = sum_j W1[j][c] dz1[j]
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) a += q.wb[i] * dz1[p4 * per + i];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (p4 == 0) dm[c4] = a;
  }
  ca_bwd_lds_barrier();
  if (wr && on) {
    float* br = c.brec + (size_t)n * (2 * C + CR);
    if (t < C) {
      br[t] = dz2[t];
      c.brec[(size_t)c.N * (2 * C + CR) + (size_t)n * C + t] = dm[t];
      br[C + CR + t] = sv * G + dm[t];  // conv2 bias grad: sum_p du
    }
    if (t < CR) br[C + t] = dz1[t];
  }
}

}  // namespace srmi
