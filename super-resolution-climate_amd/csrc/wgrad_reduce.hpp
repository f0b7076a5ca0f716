// The deterministic slab reduction of the filter gradients (wgrad3x3.hip), shared
// with the fused CA-backward + reduction launch of small.hip.
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
inline int wgrad_reduce_blocks(int Cout) { return Cout * 576 / (4 * kRedQ) + (Cout + 4 * kRedQ - 1) / (4 * kRedQ); }

// PH = slab phases per block (blockDim = kRedQ * PH: 32 -> 512 threads, 16 -> 256);
// bid = this block's index within the reduction's wgrad_reduce_blocks(Cout)
template <int PH>
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ slab, const float* __restrict__ bslab,
                                                  int nslab, int Cout, int ps, int layout, float alpha,
                                                  float* __restrict__ gw, float* __restrict__ gb, int bid) {
  __shared__ float4 red[PH][kRedQ], red2[4][kRedQ];
  const int per = Cout * 576;
  const int nwb = per / (4 * kRedQ);  // weight blocks (per % 64 == 0 since Cout % 64 == 0)
  const int qd = threadIdx.x % kRedQ, ph = threadIdx.x / kRedQ;
  const bool is_w = bid < nwb;
  const float* src;
  int stride, o4, valid;
  if (is_w) {
    if (!gw) return;
    o4 = bid * (4 * kRedQ) + qd * 4;
    src = slab + o4;
    stride = per;
    valid = 1;
  } else {
    if (!gb) return;
    o4 = (bid - nwb) * (4 * kRedQ) + qd * 4;
    src = bslab + o4;
    stride = Cout;
    valid = o4 < Cout;
  }
  float4 a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
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

// The share `part` of `nparts` of nred (1 or 2) slab reductions of 64->64 convs
// (wgrad48 layout 1, no pixel-shuffle permutation), run by ONE 512-thread workgroup
// inside another launch: the fused RCAB backward's filter-gradient workgroups reduce
// the previous RCAB's slabs after their own chunk (no reduction launch of its own).
// Output quads of the concatenated sets are split evenly over the parts; per round a
// thread sums one quad over half of the slabs (up to 32 loads in flight, clamped and
// zeroed past the end), the two halves are combined in LDS in a fixed order:
// deterministic, independent of placement.  The conv1 bias (r.gb) is reduced by the
// last part.  lds: >= 512 float4 scratch.  Every thread of the workgroup calls this.
__device__ __forceinline__ void slab_reduce_share(const ReduceSet& ra, const ReduceSet& rb, int nred, int part,
                                                  int nparts, float4* lds) {
  constexpr int PERQ = 64 * 576 / 4;  // output quads per set
  // QR quads per round x NPH slab phases, up to NL loads in flight per thread
  constexpr int NL = 16, NPH = 4, QR = 512 / NPH;
  const int tid = threadIdx.x, qi = tid % QR, ph = tid / QR;
  const int total = nred * PERQ;
  const int q0 = (int)((long long)total * part / nparts), q1 = (int)((long long)total * (part + 1) / nparts);
  for (int qb = q0; qb < q1; qb += QR) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the previous round's (or the caller's) LDS reads are done
    const int q = min(qb + qi, q1 - 1);
    const int set = q >= PERQ;
    const float* slab = set ? rb.slab : ra.slab;
    const int nslab = set ? rb.nslab : ra.nslab;
    const int o4 = (q - set * PERQ) * 4;
    const int S = (nslab + NPH - 1) / NPH, s0 = ph * S, s1 = min(nslab, s0 + S);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int sb = s0; sb < s1; sb += NL) {
      float4 v[NL];
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const int sl = sb + i;
        v[i] = *reinterpret_cast<const float4*>(slab + (size_t)min(sl, nslab - 1) * (64 * 576) + o4);
        if (sl >= s1) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w;
      }
    }
    lds[ph * QR + qi] = acc;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ph == 0 && qb + qi < q1) {
      float4 r = lds[qi];
#pragma unroll
      for (int k = 1; k < NPH; ++k) {
        const float4 t = lds[k * QR + qi];
        r.x += t.x; r.y += t.y; r.z += t.z; r.w += t.w;
      }
      const float alpha = set ? rb.alpha : ra.alpha;
      float* gw = set ? rb.gw : ra.gw;
      const float s4[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // layout 1: [wave][t][ct][lane][4] (wgrad_reduce_body)
        const int l = o4 + e;
        const int rr = l & 3, lane = (l >> 2) & 63, ct = (l >> 8) & 3, wt = l >> 10;
        const int wave = wt / 9, tap = wt >> 2, ci = (wt & 3) * 16 + (lane & 15);
        const int co = ((ct + wave) & 3) * 16 + 4 * (lane >> 4) + rr;
        gw[((size_t)co * 64 + ci) * 9 + tap] = alpha * s4[e];
      }
    }
  }
  if (part == nparts - 1) {  // the biases: 64 outputs x 8 slab phases
    float* lf = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k >= nred) break;
      const ReduceSet& r = k ? rb : ra;
      if (!r.gb) continue;  // (uniform)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int c = tid & 63, bp = tid >> 6, S = (r.nslab + 7) >> 3, s0 = bp * S, s1 = min(r.nslab, s0 + S);
      float a = 0.f;
      for (int sb = s0; sb < s1; sb += 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int sl = sb + i;
          v[i] = r.bslab[(size_t)min(sl, r.nslab - 1) * 64 + c];
          if (sl >= s1) v[i] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) a += v[i];
      }
      lf[bp * 64 + c] = a;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (tid < 64) {
        float b = lf[tid];
#pragma unroll
        for (int k2 = 1; k2 < 8; ++k2) b += lf[k2 * 64 + tid];
        r.gb[tid] = r.alpha * b;
      }
    }
  }
}

}  // namespace srmi
