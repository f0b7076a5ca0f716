// Weight (and bias) gradient of a 3x3 "same" conv as an MFMA GEMM on gfx950.
//
// Replaces the filter-gradient half of nn.Conv2d backward for default_conv
// (reference sres/model/common/cnn.py:8-9; all 64->64 and 64->256 convs of
// sres/model/rcan/network.py and blocks.py:64-65):
//     dW[co][ci][tap] = sum_{n,p} dY[n][p][co] * X[n][p + off(tap)][ci]
//     db[co]          = sum_{n,p} dY[n][p][co]
// M = 64 output channels (one co block), N = 9 taps x 64 input channels,
// K = pixels.  One workgroup = 9 waves, wave w owns tap w (a 64x64 f32 tile in
// 64 accumulator VGPRs).  Per stage (2 rows x TW columns) the dY tile and the
// (4 x TW+2) input halo are staged in LDS and read with ds_read_b64_tr_b16 so
// that both MFMA operands come out K(pixel)-major; every wave re-reads the same
// dY fragments and a tap-shifted window of the same halo.  Stages are
// double-buffered (register-staged global loads issued before the MFMAs).
// Each workgroup writes one partial slab; wgrad_reduce sums slabs in a fixed
// order (deterministic) straight into the torch-layout gradient.
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

constexpr int kWThreads = 576;

template <int TW>
struct WgSmem {
  static constexpr int DY_PIX = 2 * TW;
  static constexpr int X_PIX = 4 * (TW + 2);
  static constexpr int DY_BYTES = DY_PIX * 128;
  static constexpr int X_BYTES = X_PIX * 128;
  static constexpr int STAGE = DY_BYTES + X_BYTES;
  static constexpr int CHUNKS = (DY_PIX + X_PIX) * 8;
  static constexpr int PER_THREAD = (CHUNKS + kWThreads - 1) / kWThreads;
  static constexpr int TOTAL = 2 * STAGE + 9 * 64 * 4;  // + bias-sum scratch
};

template <int TW>
__global__ void __launch_bounds__(kWThreads, 1) wgrad3x3_kernel(WgradParams p) {
  using S = WgSmem<TW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, tap = tid >> 6;
  const int ky = tap / 3, kx = tap - 3 * (tap / 3);
  const int rs = blockIdx.x % p.row_splits, gi = blockIdx.x / p.row_splits;
  const int cb = blockIdx.y;
  const int Hr = p.H / p.row_splits;
  const int nxb = p.W / TW, nrp = Hr / 2;
  const int nst = p.imgs_per_wg * nrp * nxb;
  const int slab_id = blockIdx.x;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  uint4 stg[S::PER_THREAD];

  auto issue = [&](int st) {
    const int xb = st % nxb;
    const int rest = st / nxb;
    const int rp = rest % nrp;
    const int n = gi * p.imgs_per_wg + rest / nrp;
    const int y0 = rs * Hr + 2 * rp, x0 = xb * TW;
#pragma unroll
    for (int k = 0; k < S::PER_THREAD; ++k) {
      const int i = tid + k * kWThreads;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (i < S::CHUNKS) {
        const int q = i >> 3, c = i & 7;
        if (q < S::DY_PIX) {
          const int r = q / TW, xx = x0 + q - r * TW, y = y0 + r;
          const bf16_t* src;
          if (p.dy_mode == IN_PLAIN)
            src = p.dy + ((size_t)((size_t)n * p.H + y) * p.W + xx) * p.Cout + cb * 64 + c * 8;
          else
            src = p.dy + ((size_t)((size_t)n * 2 * p.H + 2 * y + (cb >> 1)) * (2 * p.W) + 2 * xx + (cb & 1)) * 64 + c * 8;
          v = *reinterpret_cast<const uint4*>(src);
        } else {
          const int qq = q - S::DY_PIX;
          const int hr = qq / (TW + 2), hx = qq - hr * (TW + 2);
          const int y = y0 - 1 + hr, xx = x0 - 1 + hx;
          if (y >= 0 && y < p.H && xx >= 0 && xx < p.W)
            v = *reinterpret_cast<const uint4*>(p.x + ((size_t)((size_t)n * p.H + y) * p.W + xx) * 64 + c * 8);
        }
      }
      stg[k] = v;
    }
  };
  auto commit = [&](int buf) {
    char* base = smem + buf * S::STAGE;
#pragma unroll
    for (int k = 0; k < S::PER_THREAD; ++k) {
      const int i = tid + k * kWThreads;
      if (i < S::CHUNKS) {
        const int q = i >> 3, c = i & 7;
        if (q < S::DY_PIX)
          *reinterpret_cast<uint4*>(base + swz128t(q, c)) = stg[k];
        else
          *reinterpret_cast<uint4*>(base + S::DY_BYTES + swz128t(q - S::DY_PIX, c)) = stg[k];
      }
    }
  };

  // lane coordinates for the transposed reads
  const int g = lane >> 4, li = lane & 15, lq = li >> 2, lp = li & 3;
  const int prow = g >> 1;                    // row of the 2-row stage
  const int pcol = 8 * (g & 1) + lq;          // + 16*kb + 4*s

  issue(0);
  commit(0);
  __syncthreads();
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) issue(st + 1);
    const char* dyl = smem + (st & 1) * S::STAGE;
    const char* xl = dyl + S::DY_BYTES;
#pragma unroll
    for (int kb = 0; kb < TW / 16; ++kb) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int chunk = 2 * ct + (lp >> 1);
        const uint32_t off = (lp & 1) * 8;
        const int px0 = prow * TW + kb * 16 + pcol;
        a[ct] = cat_tr(lds_tr(dyl, swz128t(px0, chunk) + off), lds_tr(dyl, swz128t(px0 + 4, chunk) + off));
        const int hq0 = (prow + ky) * (TW + 2) + kb * 16 + pcol + kx;
        b[ct] = cat_tr(lds_tr(xl, swz128t(hq0, chunk) + off), lds_tr(xl, swz128t(hq0 + 4, chunk) + off));
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int it = 0; it < 4; ++it) acc[ct][it] = mfma16(a[ct], b[it], acc[ct][it]);
    }
    // bias gradient: lane = channel, pixels strided over the 9 waves
    for (int px = tap; px < S::DY_PIX; px += 9) {
      const bf16_t v = *reinterpret_cast<const bf16_t*>(dyl + swz128t(px, lane >> 3) + (lane & 7) * 2);
      bsum += bf2f(v);
    }
    if (st + 1 < nst) commit((st + 1) & 1);
    __syncthreads();
  }

  // epilogue: partial slab [slab][Cout][9][64]
  float* slab = p.slab + (size_t)slab_id * p.Cout * 576;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int it = 0; it < 4; ++it)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cb * 64 + ct * 16 + 4 * (lane >> 4) + r;
        const int ci = it * 16 + (lane & 15);
        slab[((size_t)co * 9 + tap) * 64 + ci] = acc[ct][it][r];
      }
  float* red = reinterpret_cast<float*>(smem + 2 * S::STAGE);
  red[tap * 64 + lane] = bsum;
  __syncthreads();
  if (tid < 64) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 9; ++w) s += red[w * 64 + tid];
    p.bslab[(size_t)slab_id * p.Cout + cb * 64 + tid] = s;
  }
}

int wgrad3x3_nslabs(const WgradParams& p) { return (p.N / p.imgs_per_wg) * p.row_splits; }

int wgrad3x3_launch(const WgradParams& p, hipStream_t st) {
  if (p.Cout % 64 || p.N % p.imgs_per_wg || p.H % p.row_splits || (p.H / p.row_splits) % 2) return SRMI_ERR_SHAPE;
  if (p.dy_mode == IN_UNSHUF && p.Cout != 256) return SRMI_ERR_SHAPE;
  dim3 grid(wgrad3x3_nslabs(p), p.Cout / 64);
  if (p.W % 48 == 0) {
    hipLaunchKernelGGL(wgrad3x3_kernel<48>, grid, dim3(kWThreads), WgSmem<48>::TOTAL, st, p);
  } else if (p.W % 32 == 0) {
    hipLaunchKernelGGL(wgrad3x3_kernel<32>, grid, dim3(kWThreads), WgSmem<32>::TOTAL, st, p);
  } else {
    return SRMI_ERR_SHAPE;
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

// -------------------------------------------------------------------- reduce
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ bslab, int nslab,
                                    int Cout, int ps, float alpha, float* __restrict__ gw, float* __restrict__ gb) {
  const int per = Cout * 576;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < per) {
    float s = 0.f;
    for (int k = 0; k < nslab; ++k) s += slab[(size_t)k * per + idx];
    const int ci = idx & 63, tap = (idx >> 6) % 9, cop = idx / 576;
    const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
    gw[((size_t)cot * 64 + ci) * 9 + tap] = alpha * s;
  } else if (gb && idx < per + Cout) {
    const int cop = idx - per;
    float s = 0.f;
    for (int k = 0; k < nslab; ++k) s += bslab[(size_t)k * Cout + cop];
    const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
    gb[cot] = alpha * s;
  }
}

int wgrad_reduce_launch(const float* slab, const float* bslab, int nslab, int Cout, int ps, float alpha, float* gw,
                        float* gb, hipStream_t st) {
  const int total = Cout * 576 + Cout;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, slab, bslab, nslab, Cout, ps,
                     alpha, gw, gb);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
