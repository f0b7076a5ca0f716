// The consumer side of the CA-backward fold (srmi_internal.hpp CaFold): the image's
// channel-attention MLP backward, recomputed by every workgroup of the conv2
// backward launch that needs it, and the dgrad's border-class correction table.
// Included by conv64_body.hpp (conv3x3.hip, wgrad3x3.hip).
#pragma once
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

// LDS scratch of the fold, in floats, placed after the conv body's own LDS:
// red[2][128] | s[64] | dz2[64] | dz1[32] | G[64] | dm[64] | c[64] | corr[9][64]
constexpr int kFoldRed = 0, kFoldS = 256, kFoldDz2 = 320, kFoldDz1 = 384, kFoldG = 416, kFoldDm = 480,
              kFoldC = 544, kFoldCorr = 608;
constexpr int kFoldFloats = kFoldCorr + 9 * 64;
constexpr int kFoldBytes = kFoldFloats * 4;

// workgroup barrier ordering LDS only (global loads and LDS-DMA stay in flight)
__device__ __forceinline__ void fold_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// CALayer backward of image n (sres/model/rcan/network.py:44-47), C = 64:
//   G[c] = sum_p g, ds[c] = sum_p g u (the producer's per-strip sums, fixed order)
//   dz2 = ds s (1 - s); dz1 = relu'(z1) W2^T dz2; dm = W1^T dz1; c = dm / HW
// into sm[kFoldC ..]; write_brec: the image's backward record (dz2 | dz1 | the conv2
// bias gradient sum_p du = s G + dm, then dm) as ca_bwd_du writes it.  Every thread of
// the workgroup calls this (it holds barriers); threads 0..255 compute.  Same
// arithmetic and order as ca_bwd_du_kernel (small.hip).
struct CaFoldRegs {  // the MLP's global operands of one thread (threads 0..255)
  float pa, zj, svl;
  float wa[8], wb[8];
};

// the global loads of ca_fold_mlp, issued on their own so that a caller can put them
// in flight ahead of its LDS-DMA prologue (their latency then hides under it)
__device__ __forceinline__ void ca_fold_mlp_load(const CaFold& f, int n, CaFoldRegs& r) {
  constexpr int C = 64;
  const int tid = threadIdx.x, CR = f.CR, per = CR / 4;
  const int j = tid >> 3, pj = tid & 7, c4 = (tid >> 2) & 63, p4 = tid & 3;
  const int jc = min(j & 31, CR - 1);
  r.pa = 0.f;
  r.zj = r.svl = 0.f;
  if (tid < 256) {  // (wave-uniform)
    for (int k = tid >> 7; k < f.nstrips; k += 2) r.pa += f.part[((size_t)n * f.nstrips + k) * (2 * C) + (tid & 127)];
#pragma unroll
    for (int i = 0; i < 8; ++i) r.wa[i] = f.w2[(pj * 8 + i) * CR + jc];
#pragma unroll
    for (int i = 0; i < 8; ++i) r.wb[i] = f.w1[(p4 * per + min(i, per - 1)) * C + c4];
    const float* rr = f.rec + (size_t)n * (2 * C + CR);
    r.zj = rr[C + jc];
    r.svl = rr[C + CR + (tid & 63)];
  }
}

__device__ __forceinline__ void ca_fold_mlp_compute(const CaFold& f, int n, int N, int HW, float* sm, bool write_brec,
                                                    const CaFoldRegs& r) {
  constexpr int C = 64;
  const int tid = threadIdx.x, CR = f.CR, per = CR / 4;
  const bool act = tid < 256;  // (wave-uniform)
  const int j = tid >> 3, pj = tid & 7, c4 = (tid >> 2) & 63, p4 = tid & 3;
  if (act) {
    sm[kFoldRed + (tid >> 7) * 128 + (tid & 127)] = r.pa;
    if (tid < C) sm[kFoldS + tid] = r.svl;
  }
  fold_barrier();
  if (tid < C) {
    const float G = sm[kFoldRed + tid] + sm[kFoldRed + 128 + tid];
    const float ds = sm[kFoldRed + C + tid] + sm[kFoldRed + 128 + C + tid];
    const float sv = sm[kFoldS + tid];
    sm[kFoldDz2 + tid] = ds * sv * (1.f - sv);
    sm[kFoldG + tid] = G;
  }
  fold_barrier();
  if (act) {  // dz1[j] = relu'(z1[j]) sum_c W2[c][j] dz2[c]
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += r.wa[i] * sm[kFoldDz2 + pj * 8 + i];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (j < CR && pj == 0) sm[kFoldDz1 + j] = (r.zj > 0.f) ? a : 0.f;
  }
  fold_barrier();
  if (act) {  // dm[c] = sum_j W1[j][c] dz1[j]
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < per) a += r.wb[i] * sm[kFoldDz1 + p4 * per + i];
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (p4 == 0) {
      sm[kFoldDm + c4] = a;
      sm[kFoldC + c4] = a * (1.f / (float)HW);
    }
  }
  fold_barrier();
  if (write_brec && tid < C) {
    float* br = f.brec + (size_t)n * (2 * C + CR);
    const float dm = sm[kFoldDm + tid];
    br[tid] = sm[kFoldDz2 + tid];
    f.brec[(size_t)N * (2 * C + CR) + (size_t)n * C + tid] = dm;
    br[C + CR + tid] = sm[kFoldS + tid] * sm[kFoldG + tid] + dm;
    if (tid < CR) br[C + tid] = sm[kFoldDz1 + tid];
  }
}

__device__ __forceinline__ void ca_fold_mlp(const CaFold& f, int n, int N, int HW, float* sm, bool write_brec) {
  CaFoldRegs r;
  ca_fold_mlp_load(f, n, r);
  ca_fold_mlp_compute(f, n, N, HW, sm, write_brec, r);
}

// The dgrad of the constant field c (zero outside the image) through the dgrad
// filter image in LDS (wl: [9 taps][64 out rows][64 in] bf16, swz128t chunks; tap
// (ky, kx) reads input pixel (y + ky - 1, x + kx - 1)): per border class
// (cy, cx) in {top / inner / bottom} x {left / inner / right}
//   corr[cy][cx][co] = sum over the taps valid there of sum_ci W[tap][co][ci] c[ci]
// Needs sm[kFoldC] (ca_fold_mlp) and the filter image landed; all threads call it.
__device__ __forceinline__ void ca_fold_corr(const char* wl, float* sm) {
  const int tid = threadIdx.x;
  if (tid < 512) {  // (wave-uniform) row co = tid >> 3, input chunk j = tid & 7
    const int co = tid >> 3, j = tid & 7;
    float cc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) cc[e] = sm[kFoldC + 8 * j + e];
    float v[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const uint4 q = *reinterpret_cast<const uint4*>(wl + t * 8192 + swz128t(co, j));
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
      float a = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a += __uint_as_float(w[e] << 16) * cc[2 * e];
        a += __uint_as_float(w[e] & 0xFFFF0000u) * cc[2 * e + 1];
      }
      a += __shfl_xor(a, 1, 64);
      a += __shfl_xor(a, 2, 64);
      a += __shfl_xor(a, 4, 64);
      v[t] = a;
    }
    // lane j writes class j (and lane 0 class 8 too)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int cls = k == 0 ? j : 8;
      if (k == 1 && j != 0) break;
      const int cy = cls / 3, cx = cls % 3;
      float a = 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t % 3;
        const bool ok = !(cy == 0 && ky == 0) && !(cy == 2 && ky == 2) && !(cx == 0 && kx == 0) && !(cx == 2 && kx == 2);
        a += ok ? v[t] : 0.f;
      }
      sm[kFoldCorr + cls * 64 + co] = a;
    }
  }
  fold_barrier();
}

}  // namespace srmi
