// Inference RCAB as ONE launch, one workgroup per image (RCAB, sres/model/rcan/
// network.py:50-64; CALayer :31-47).  In inference an image is one run of the conv
// body anyway (run_len = all strips at the C5 batch), so an RCAB needs no other
// workgroup and no launch boundary inside it.  u = conv2(t) + b2 is never stored: the
// CA pool needs only mean(u), which follows from t's statistics (ca_scale.hpp), so s is
// known before conv2 runs:
//   phase A  t = relu(conv1(h) + b1), + per-strip channel sums of the bf16 t   conv64_body<RELU_POOL>
//   phase B  h' = h + s (conv2(t) + b2) in conv2's epilogue                    conv64_body<CA_RESID>
//            with s computed inside it after its first strip's MFMAs (as the training
//            conv2 does): border rows / columns / corners of t, S_tap, mean(u) with
//            conv2's bf16 filter image in LDS, the CA MLP                      ca_scale_finish
// against the three launches of the training forward (conv1; conv2 + pool writing u;
// the CA pass reading u, h and writing h'): per image 0.6 MB less traffic and no
// elementwise pass.  It differs from them in summation order only (m from t's
// statistics instead of the pooled u): like them it rounds u to bf16 before
// h' = h + s * bf16(u) (SRMI_INFER_BF16U=1, the default; the =0 variant adds the fp32 u
// instead), within bf16 noise of the fp64 oracle
// (test_fused_inference_rcab_matches_three_launches_and_oracle).
// (write-back stores and the deferred conv1 epilogue: tuning.hpp SRMI_INFER_*)
#define SRMI_TU_INFER 1
#include "conv64_body.hpp"
#include "ca_scale.hpp"
#include "srmi_internal.hpp"

namespace srmi {

// the workgroup's own global stores visible to its own later loads (LDS-DMA included)
__device__ __forceinline__ void own_stores_visible() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  asm volatile("buffer_inv sc0" ::: "memory");  // this CU's L1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// diagnostic build (SRMI_STAMPS): the launch's phase stamps after the two conv bodies'
#ifdef SRMI_STAMPS
#define ISTAMP(i)                                                                                    \
  do {                                                                                               \
    if (c1.stamps && threadIdx.x == 0)                                                               \
      c1.stamps[(size_t)2 * gridDim.x * 64 + blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memtime();  \
  } while (0)
#else
#define ISTAMP(i) \
  do {            \
  } while (0)
#endif

__global__ void __launch_bounds__(512, 1) rcab_infer_kernel(ConvParams c1, ConvParams c2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = blockIdx.x;
  const int nsy = c1.H / kTH;
  ISTAMP(0);
  conv64_body<48, EPI_RELU_POOL, 8>(c1, nsy, n, smem);  // t and its per-strip sums: the whole image, one run
  ISTAMP(1);
  own_stores_visible();
  ISTAMP(2);
  // h' = h + s (conv2(t) + b2), s from t inside the body (c2.cas_on)
  conv64_body<48, EPI_CA_RESID, 8>(c2, nsy, n, smem);
  ISTAMP(3);
}

int rcab_infer_launch(const ConvParams& c1, const ConvParams& c2, const float* part, int nstrips, const float* w1,
                      const float* b1, const float* w2, const float* b2, int CR, const float* h_in, const void* hi_in,
                      const void* lo_in, void* hi_out, void* lo_out, float* rec, hipStream_t st) {
  if (c1.f32 || c2.f32 || c1.W != 48 || c1.H % kTH || c1.Cin != 64 || c1.Cout != 64 || c2.Cin != 64 ||
      c2.Cout != 64 || c1.N != c2.N || c1.H != c2.H || c1.W != c2.W || c1.in_mode != IN_PLAIN)
    return SRMI_ERR_SHAPE;
  if (!c1.yb || !part || !hi_out || !lo_out || (!h_in && (!hi_in || !lo_in)) || CR < 4 || CR > 32 || CR % 4 ||
      nstrips != (c1.H / kTH) || !rec || !c2.bias || !w1 || !b1 || !w2 || !b2)
    return SRMI_ERR_ARG;
  if ((size_t)c1.N * c1.H * c1.W * 64 * 2 >= ((size_t)1 << 32)) return SRMI_ERR_SHAPE;
  CaScale ca{};
  ca.t = c1.yb;
  ca.part = part;
  ca.nstrips = nstrips;
  ca.w1 = w1;
  ca.b1 = b1;
  ca.w2 = w2;
  ca.b2 = b2;
  ca.bc2 = c2.bias;
  ca.CR = CR;
  ca.rec = rec;
  ConvParams a = c1, b = c2;
  // (diagnostic: [3][N][64] stamps -- conv1's body, conv2's body, the launch's phases)
  a.stamps = conv3x3_debug_stamps();
  b.stamps = a.stamps ? a.stamps + (size_t)c1.N * 64 : nullptr;
  ca.stamps = a.stamps ? a.stamps + (size_t)3 * c1.N * 64 : nullptr;
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
  b.cas = ca;  // conv2 computes its s (and the record m | z1 | s) itself
  b.cas_on = 1;
  hipLaunchKernelGGL(rcab_infer_kernel, dim3(c1.N), dim3(512), Conv2Smem<48>::TOTAL + kCaScaleFloats * sizeof(float),
                     st, a, b);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
