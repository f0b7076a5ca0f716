// Inference RCAB as ONE launch, one workgroup per image (RCAB, sres/model/rcan/
// network.py:50-64; CALayer :31-47):
//   phase A  t = relu(conv1(h) + b1)        conv64_body<RELU>, the whole image as one run
//   phase B  u = conv2(t) + b2, pool sums   conv64_body<POOL>, likewise
//   phase C  s = sigmoid(W2 relu(W1 mean(u) + c1) + c2); h' = h + s u   (residual pair)
// Training keeps the three launches (t, u and the CA record are saved for backward and
// an image there is split over several workgroups); in inference an image is one run
// anyway (run_len = all strips at the C5 batch), so the image's three passes need no
// other workgroup: no launch boundaries between them, the MLP once per image instead
// of once per elementwise block, and t / u re-read by the workgroup that just wrote
// them (L2 / Infinity-Cache hits instead of HBM).
// t and u are re-read by this workgroup within the launch: plain stores keep their
// lines in the XCD's L2 (write-through ones drop them); conv2 runs its strips last to
// first so that it starts on the t rows conv1 wrote last, and the CA pass starts on the
// u rows conv2 wrote last.  The residual pair stays write-through (stw_* below).
#ifndef SRMI_INFER_WT
#define SRMI_INFER_WT 0
#endif
#ifndef SRMI_INFER_REV
#define SRMI_INFER_REV 1
#endif
// deferred conv epilogues (conv64_body.hpp SRMI_DEFER) for this launch's convs: an
// image is one run of 12 strips here, not 3 as in training
#ifndef SRMI_INFER_DEFER
#define SRMI_INFER_DEFER 7
#endif
// diagnostic builds only (wrong results): 1 skips the CA pass, 2 conv2, 4 conv1
#ifndef SRMI_INFER_DIAG
#define SRMI_INFER_DIAG 0
#endif
#define SRMI_WT SRMI_INFER_WT
#define SRMI_DEFER SRMI_INFER_DEFER
#include "conv64_body.hpp"
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
  float* rec;           // optional: m | z1 | s per image
};

// phase C for image n, 512 threads: the MLP in LDS scratch (sm >= 64 + 64 + 32 + 64 floats),
// then the elementwise pair update, 8 units of 4 channels in flight per thread
template <bool F32IN>
__device__ __forceinline__ void ca_image_body(const CaInfer& c, int n, int HW, float* sm) {
  constexpr int C = 64;
  const int tid = threadIdx.x, CR = c.CR, per = CR / 4;
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
  constexpr bool kRev = SRMI_INFER_REV && !(SRMI_INFER_DEFER & 2);  // (reversal: the non-deferred body)
  if (!(SRMI_INFER_DIAG & 2)) conv64_body<48, EPI_POOL_BF16, 8, false, kRev>(c2, nsy, n, smem);
  own_stores_visible();
  if (!(SRMI_INFER_DIAG & 1)) ca_image_body<F32IN>(ca, n, c1.H * c1.W, reinterpret_cast<float*>(smem));
}

int rcab_infer_launch(const ConvParams& c1, const ConvParams& c2, const float* part, int nstrips, const float* w1,
                      const float* b1, const float* w2, const float* b2, int CR, const float* h_in, const void* hi_in,
                      const void* lo_in, void* hi_out, void* lo_out, float* rec, hipStream_t st) {
  if (c1.f32 || c2.f32 || c1.W != 48 || c1.H % kTH || c1.Cin != 64 || c1.Cout != 64 || c2.Cin != 64 ||
      c2.Cout != 64 || c1.N != c2.N || c1.H != c2.H || c1.W != c2.W || c1.in_mode != IN_PLAIN)
    return SRMI_ERR_SHAPE;
  if (!c1.yb || !c2.yb || !c2.part || !part || !hi_out || !lo_out || (!h_in && (!hi_in || !lo_in)) || CR < 4 ||
      CR > 32 || CR % 4 || nstrips != (c1.H / kTH))
    return SRMI_ERR_ARG;
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
  if (h_in)
    hipLaunchKernelGGL((rcab_infer_kernel<true>), grid, dim3(512), Conv2Smem<48>::TOTAL, st, a, b, ca);
  else
    hipLaunchKernelGGL((rcab_infer_kernel<false>), grid, dim3(512), Conv2Smem<48>::TOTAL, st, a, b, ca);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
