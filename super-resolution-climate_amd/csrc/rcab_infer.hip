// Inference RCAB as ONE launch, one workgroup per image (RCAB, sres/model/rcan/
// network.py:50-64; CALayer :31-47).  In inference an image is one run of the conv
// body anyway (run_len = all strips at the C5 batch), so an RCAB needs no other
// workgroup and no launch boundary inside it.
//
// v2 (default): u = conv2(t) + b2 is never stored.  The CA pool needs only mean(u),
// and by linearity
//   mean_p u[p][c] = b2[c] + (1/HW) sum_{tap, ci} W2[c][ci][tap] S_tap[ci],
//   S_tap[ci] = sum over the input pixels tap (dy, dx) reaches of t[.][ci]
//             = T[ci] - (row excluded by dy) - (column excluded by dx) + (their corner),
// so s = sigmoid(W2' relu(W1' mean(u) + c1) + c2) is known before conv2 runs:
//   phase A  t = relu(conv1(h) + b1), + per-strip channel sums T   conv64_body<RELU_POOL>
//   phase S  border rows / columns / corners of t, S_tap, mean(u), the CA MLP -> s
//   phase B  h' = h + s (conv2(t) + b2) in conv2's epilogue          conv64_body<CA_RESID>
// against v1's three passes (conv1; conv2 + pool writing u; the CA pass reading u, h
// and writing h'): per image 0.6 MB less traffic and no elementwise pass, and u enters
// h' in fp32 instead of rounded to bf16.  The sums differ from the pooled fp32 u only
// in summation order and in conv2's bf16 weights (the mean uses the fp32 weights).
// v1 (SRMI_INFER_V=1): bit-identical to the three training-path launches.
#ifndef SRMI_INFER_V
#define SRMI_INFER_V 2
#endif
// v2: the mean's matvec from conv2's bf16 filter image in LDS (1) or the fp32 weights (0)
#ifndef SRMI_INFER_WLDS
#define SRMI_INFER_WLDS 1
#endif
// plain (write-back) stores for this launch's outputs: t is re-read by the workgroup
// that wrote it, and the pair by the next launch (+1 % C5 against write-through)
#ifndef SRMI_INFER_WT
#define SRMI_INFER_WT 0
#endif
// deferred conv epilogues (conv64_body.hpp SRMI_DEFER) for this launch's convs: an
// image is one run of 12 strips here, not 3 as in training.  23 = v1's RELU / POOL
// (1, 2) and v2's RELU_POOL (16); v2's CA_RESID epilogue (32) measured 5 % slower
// deferred (its pair codec then competes with the next strip's MFMA issue)
#ifndef SRMI_INFER_DEFER
#define SRMI_INFER_DEFER 23
#endif
// diagnostic builds only (wrong results): 1 skips the CA pass (v2: the scale), 2 conv2, 4 conv1
#ifndef SRMI_INFER_DIAG
#define SRMI_INFER_DIAG 0
#endif
#define SRMI_WT SRMI_INFER_WT
#define SRMI_DEFER SRMI_INFER_DEFER
#include "conv64_body.hpp"
#include "ca_infer.hpp"
#include "srmi_internal.hpp"

namespace srmi {

__device__ __forceinline__ void stw8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint2 v) {  // write-through (sc1)
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 16);
}
__device__ __forceinline__ void stw4(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 16);
}

struct CaInfer {
  const bf16_t* u;      // conv2 output [N][HW][64] bf16
  const float* part;    // pool partials [N][nstrips][64]
  int nstrips;
  const float *w1, *b1, *w2, *b2;
  int CR;
  const float* h_in;    // fp32 group input (first RCAB of a group), or null
  const bf16_t* hi_in;  // else the pair hi + lo
  const uint8_t* lo_in;
  bf16_t* hi_out;       // the pair out (hi = the next conv1's operand)
  uint8_t* lo_out;
  float* rec;           // m | z1 | s per image (v1: optional; v2: s is conv2's scale)
  const float* wc2;     // v2: conv2's fp32 weight [64][64][3][3] and bias [64] (the mean)
  const float* bc2;
  const bf16_t* t;      // v2: conv1's output
};

// phase C for image n, 512 threads: the MLP in LDS scratch (sm >= 64 + 64 + 32 + 64 floats),
// then the elementwise pair update, 8 units of 4 channels in flight per thread
template <bool F32IN>
__device__ __forceinline__ void ca_image_body(const CaInfer& c, int n, int HW, float* sm) {
  constexpr int C = 64;
  const int tid = threadIdx.x;
  float* red = sm;            // [4][64]
  float* m = sm + 512;        // [64]
  float* z1 = m + 64;         // [32]
  float* s = z1 + 32;         // [64]
  if (tid < 256) {  // pool: 4 strip phases x 64 channels, the order of ca_fwd_kernel (bit-identical)
    const int ch = tid & 63, ph = tid >> 6;
    float a = 0.f;
    for (int k = ph; k < c.nstrips; k += 4) a += c.part[((size_t)n * c.nstrips + k) * C + ch];
    red[ph * 64 + ch] = a;
  }
  __syncthreads();
  if (tid < C) m[tid] = (red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid]) / (float)HW;
  __syncthreads();
  ca_mlp(c, n, m, z1, s);
  // elementwise: units of 4 channels, consecutive lanes on consecutive units
  const size_t base = (size_t)n * HW * C;
  const int nq = HW * C / 4;
  const auto rhb = wt_rsrc(c.hi_out, (uint32_t)((size_t)(n + 1) * HW * C * 2));
  const auto rlo = wt_rsrc(c.lo_out, (uint32_t)((size_t)(n + 1) * HW * C));
  constexpr int NU = 8;
  for (int q0 = tid; q0 < nq; q0 += 512 * NU) {
    uint2 uu[NU];
    float4 hh[NU];
#pragma unroll
    for (int k = 0; k < NU; ++k) {  // clamped, unconditional loads (the tail stores nothing)
      const size_t e = base + (size_t)min(q0 + k * 512, nq - 1) * 4;
      uu[k] = *reinterpret_cast<const uint2*>(c.u + e);
      if constexpr (F32IN) {
        hh[k] = *reinterpret_cast<const float4*>(c.h_in + e);
      } else {
        hh[k] = pair_decode4(*reinterpret_cast<const uint2*>(c.hi_in + e), *reinterpret_cast<const uint32_t*>(c.lo_in + e));
      }
    }
#pragma unroll
    for (int k = 0; k < NU; ++k) {
      const int q = q0 + k * 512;
      if (q >= nq) continue;
      const size_t e = base + (size_t)q * 4;
      const int c0 = (q * 4) & 63;
      const float o0 = bf2f(uu[k].x & 0xFFFFu) * s[c0 + 0] + hh[k].x;
      const float o1 = bf2f(uu[k].x >> 16) * s[c0 + 1] + hh[k].y;
      const float o2 = bf2f(uu[k].y & 0xFFFFu) * s[c0 + 2] + hh[k].z;
      const float o3 = bf2f(uu[k].y >> 16) * s[c0 + 3] + hh[k].w;
      uint2 hi;
      const uint32_t lo = pair_encode4(o0, o1, o2, o3, hi);
      stw8(rhb, (uint32_t)(e * 2), hi);
      stw4(rlo, (uint32_t)e, lo);
    }
  }
}

// the workgroup's own global stores visible to its own later loads (LDS-DMA included)
__device__ __forceinline__ void own_stores_visible() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  asm volatile("buffer_inv sc0" ::: "memory");  // this CU's L1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool F32IN>
__global__ void __launch_bounds__(512, 1) rcab_infer_kernel(ConvParams c1, ConvParams c2, CaInfer ca) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = blockIdx.x;
  const int nsy = c1.H / kTH;
  if (!(SRMI_INFER_DIAG & 4)) conv64_body<48, EPI_RELU_BF16, 8>(c1, nsy, n, smem);  // the whole image: one run
  own_stores_visible();
  if (!(SRMI_INFER_DIAG & 2)) conv64_body<48, EPI_POOL_BF16, 8>(c2, nsy, n, smem);
  own_stores_visible();
  if (!(SRMI_INFER_DIAG & 1)) ca_image_body<F32IN>(ca, n, c1.H * c1.W, reinterpret_cast<float*>(smem));
}

__global__ void __launch_bounds__(512, 1) rcab_infer2_kernel(ConvParams c1, ConvParams c2, CaInfer ca) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = blockIdx.x;
  const int nsy = c1.H / kTH;
  if (!(SRMI_INFER_DIAG & 4)) conv64_body<48, EPI_RELU_POOL, 8>(c1, nsy, n, smem);  // t and its per-strip sums
  own_stores_visible();
  if (!(SRMI_INFER_DIAG & 1)) {
#if SRMI_INFER_WLDS
    // conv2's filter image into the filter slot (conv1 is done with it): the mean's
    // matvec reads it there, with the weights conv2 computes with; scratch in the ring
    {
      const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t wbase = lds_u32(smem);
      for (int i = wv; i < 72; i += 8) {
        const int tap = i >> 3, row = 8 * (i & 7) + (lane >> 3), ch = (lane & 7) ^ (row & 7);
        glds16(c2.w + ((size_t)(tap * 64 + row)) * 64 + ch * 8, wbase + (uint32_t)i * 1024u);
      }
    }
    ca_scale_from_t(ca, c1.yb, n, c1.H, c1.W, reinterpret_cast<float*>(smem + Conv2Smem<48>::WB), smem);
#else
    ca_scale_from_t(ca, c1.yb, n, c1.H, c1.W, reinterpret_cast<float*>(smem));  // s
#endif
  }
  own_stores_visible();
  // h' = h + s (conv2(t) + b2); with WLDS its filter image is resident from the scale phase
  if (!(SRMI_INFER_DIAG & 2))
    conv64_body<48, EPI_CA_RESID, 8, false, SRMI_INFER_WLDS && !(SRMI_INFER_DIAG & 1)>(c2, nsy, n, smem);
}

int rcab_infer_launch(const ConvParams& c1, const ConvParams& c2, const float* part, int nstrips, const float* w1,
                      const float* b1, const float* w2, const float* b2, int CR, const float* h_in, const void* hi_in,
                      const void* lo_in, void* hi_out, void* lo_out, float* rec, hipStream_t st, const float* wc2,
                      const float* bc2) {
  if (c1.f32 || c2.f32 || c1.W != 48 || c1.H % kTH || c1.Cin != 64 || c1.Cout != 64 || c2.Cin != 64 ||
      c2.Cout != 64 || c1.N != c2.N || c1.H != c2.H || c1.W != c2.W || c1.in_mode != IN_PLAIN)
    return SRMI_ERR_SHAPE;
  if (!c1.yb || !part || !hi_out || !lo_out || (!h_in && (!hi_in || !lo_in)) || CR < 4 || CR > 32 || CR % 4 ||
      nstrips != (c1.H / kTH))
    return SRMI_ERR_ARG;
  const bool v2 = SRMI_INFER_V == 2 && wc2 && bc2 && rec;
  if (!v2 && (!c2.yb || !c2.part)) return SRMI_ERR_ARG;
  if ((size_t)c1.N * c1.H * c1.W * 64 * 2 >= ((size_t)1 << 32)) return SRMI_ERR_SHAPE;
  CaInfer ca{};
  ca.u = c2.yb;
  ca.part = part;
  ca.nstrips = nstrips;
  ca.w1 = w1;
  ca.b1 = b1;
  ca.w2 = w2;
  ca.b2 = b2;
  ca.CR = CR;
  ca.h_in = h_in;
  ca.hi_in = static_cast<const bf16_t*>(hi_in);
  ca.lo_in = static_cast<const uint8_t*>(lo_in);
  ca.hi_out = static_cast<bf16_t*>(hi_out);
  ca.lo_out = static_cast<uint8_t*>(lo_out);
  ca.rec = rec;
  ConvParams a = c1, b = c2;
  a.stamps = b.stamps = nullptr;
  const dim3 grid(c1.N);
  if (v2) {
    ca.wc2 = wc2;
    ca.bc2 = bc2;
    ca.t = c1.yb;
    a.part = const_cast<float*>(part);  // conv1's per-strip sums of t
    a.part_stride = 64;
    b.yb = nullptr;  // u is never stored
    b.part = nullptr;
    b.yf = nullptr;
    b.r1 = h_in;
    b.r1h = h_in ? nullptr : static_cast<const bf16_t*>(hi_in);
    b.r1l = h_in ? nullptr : static_cast<const uint8_t*>(lo_in);
    b.yph = static_cast<bf16_t*>(hi_out);
    b.ypl = static_cast<uint8_t*>(lo_out);
    b.escale = rec + 64 + CR;  // s of the record m | z1 | s
    b.escale_stride = 128 + CR;
    hipLaunchKernelGGL(rcab_infer2_kernel, grid, dim3(512), Conv2Smem<48>::TOTAL, st, a, b, ca);
    SRMI_CHECK_LAUNCH();
    return 0;
  }
  if (h_in)
    hipLaunchKernelGGL((rcab_infer_kernel<true>), grid, dim3(512), Conv2Smem<48>::TOTAL, st, a, b, ca);
  else
    hipLaunchKernelGGL((rcab_infer_kernel<false>), grid, dim3(512), Conv2Smem<48>::TOTAL, st, a, b, ca);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
