// The deterministic slab reduction of the filter gradients (wgrad3x3.hip), shared
// with the CA-backward launch of small.hip (which carries reductions in the SRMI_F2_MLP 0
// variant) and the group-end multi-set launch.
#pragma once
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

// -------------------------------------------------------------------- reduce
// block = kRedQ output quads (4*kRedQ consecutive outputs, float4 loads) x kRedPh
// slab phases (512 threads); phase q sums slabs q, q+kRedPh, ... with 4
// independent accumulators (4 loads in flight), then the kRedPh x 4 partials are
// combined in a fixed 2-level order (deterministic).  64 outputs per block -> 576
// blocks for a 64->64 conv (the former 256-output blocks left 112 CUs idle).
// The bias slab ([nslab][Cout]) is handled by the last block(s).
constexpr int kRedQ = 16, kRedPh = 32;
// blocks of one slab reduction (Cout * 576 weights + Cout biases, kRedQ quads each)
inline int wgrad_reduce_blocks(int Cout, int Q = kRedQ) { return Cout * 576 / (4 * Q) + (Cout + 4 * Q - 1) / (4 * Q); }

// PH = slab phases per block (blockDim = kRedQ * PH: 32 -> 512 threads, 16 -> 256);
// bid = this block's index within the reduction's wgrad_reduce_blocks(Cout)
// slab16: the weight slabs are bf16 (4 values per 8-byte load), summed in fp32
// (Q = output quads per block: kRedQ, or more quads and fewer phases for long runs of
//  reductions, wgrad_reduce_sets_kernel)
template <int PH, int Q = kRedQ>
__device__ __forceinline__ void wgrad_reduce_body(const ReduceSet& rs, int bid) {
  const float* __restrict__ slab = rs.slab;
  const float* __restrict__ bslab = rs.bslab;
  const int nslab = rs.nslab, Cout = rs.Cout, ps = rs.ps, layout = rs.layout;
  const float alpha = rs.alpha;
  float* __restrict__ gw = rs.gw;
  float* __restrict__ gb = rs.gb;
  __shared__ float4 red[PH][Q], red2[4][Q];
  const int per = Cout * 576;
  const int nwb = per / (4 * Q);  // weight blocks (per % (4 Q) == 0: Cout % 64 == 0, Q | 576)
  const int qd = threadIdx.x % Q, ph = threadIdx.x / Q;
  const bool is_w = bid < nwb;
  const float* src;
  int stride, o4, valid;
  if (is_w) {
    if (!gw) return;
    o4 = bid * (4 * Q) + qd * 4;
    src = slab + o4;
    stride = per;
    valid = 1;
  } else {
    if (!gb) return;
    o4 = (bid - nwb) * (4 * Q) + qd * 4;
    src = bslab + o4;
    stride = Cout;
    valid = o4 < Cout;
  }
  float4 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid && is_w && rs.slab16) {  // (uniform) bf16 weight slabs: the same order and sums
    const uint16_t* src16 = reinterpret_cast<const uint16_t*>(slab) + o4;
    constexpr int U = 4;
    for (int k = ph; k < nslab; k += U * PH) {
      uint2 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int sl = k + j * PH;
        v[j] = *reinterpret_cast<const uint2*>(src16 + (size_t)min(sl, nslab - 1) * stride);
        if (sl >= nslab) v[j] = make_uint2(0u, 0u);  // (bf16 +0)
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        a[j].x += bf2f(v[j].x & 0xFFFFu); a[j].y += bf2f(v[j].x >> 16);
        a[j].z += bf2f(v[j].y & 0xFFFFu); a[j].w += bf2f(v[j].y >> 16);
      }
    }
  } else if (valid) {
    // phase ph sums slabs ph, ph + PH, ... -- U loads in flight per round,
    // clamped + zeroed past the end (adding 0.f is exact; no divergent branch)
    constexpr int U = 4;
    for (int k = ph; k < nslab; k += U * PH) {
      float4 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int sl = k + j * PH;
        v[j] = *reinterpret_cast<const float4*>(src + (size_t)min(sl, nslab - 1) * stride);
        if (sl >= nslab) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        a[j].x += v[j].x; a[j].y += v[j].y; a[j].z += v[j].z; a[j].w += v[j].w;
      }
    }
  }
  red[ph][qd] = make_float4((a[0].x + a[1].x) + (a[2].x + a[3].x), (a[0].y + a[1].y) + (a[2].y + a[3].y),
                            (a[0].z + a[1].z) + (a[2].z + a[3].z), (a[0].w + a[1].w) + (a[2].w + a[3].w));
  __syncthreads();
  // fixed-order 2-level combine of the PH phase partials
  constexpr int L1 = 4, PER = PH / L1;
  if (ph < L1) {
    float4 r = red[ph][qd];
#pragma unroll
    for (int q = 1; q < PER; ++q) {
      const float4 t = red[ph + q * L1][qd];
      r.x += t.x; r.y += t.y; r.z += t.z; r.w += t.w;
    }
    red2[ph][qd] = r;
  }
  __syncthreads();
  if (ph != 0 || !valid) return;
  float4 r = red2[0][qd];
#pragma unroll
  for (int q = 1; q < L1; ++q) {
    const float4 t = red2[q][qd];
    r.x += t.x; r.y += t.y; r.z += t.z; r.w += t.w;
  }
  const float s4[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int o = o4 + e;
    if (is_w) {
      int cop, ci, tap;
      if (layout == 1) {  // wgrad48 native order [cb][wave][t][ct][lane][4]
        const int cb = o / (64 * 576), l = o - cb * (64 * 576);
        const int r = l & 3, lane = (l >> 2) & 63, ct = (l >> 8) & 3, wt = l >> 10;
        const int wave = wt / 9, j = wt;  // j = 9 * wave + t
        tap = j >> 2;
        ci = (j & 3) * 16 + (lane & 15);
        cop = cb * 64 + ((ct + wave) & 3) * 16 + 4 * (lane >> 4) + r;
      } else {  // [tap][ci][Cout]
        cop = o % Cout;
        ci = (o / Cout) & 63;
        tap = o / (Cout * 64);
      }
      const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
      gw[((size_t)cot * 64 + ci) * 9 + tap] = alpha * s4[e];
    } else if (o < Cout) {
      const int cot = ps ? (4 * (o & 63) + (o >> 6)) : o;
      gb[cot] = alpha * s4[e];
    }
  }
}

}  // namespace srmi
