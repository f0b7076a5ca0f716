// Weight (and bias) gradient of a 3x3 "same" conv as an MFMA GEMM on gfx950.
//
// Replaces the filter-gradient half of nn.Conv2d backward for default_conv
// (reference sres/model/common/cnn.py:8-9; all 64->64 and 64->256 convs of
// sres/model/rcan/network.py and blocks.py:64-65):
//     dW[co][ci][ky][kx] = sum_{n,p} dY[n][p][co] * X[n][p + (ky-1,kx-1)][ci]
//     db[co]             = sum_{n,p} dY[n][p][co]
//
// GEMM view: M = 64 output channels (one co block), N = 3 taps (one kernel row
// ky) x 64 input channels, K = pixels of one chunk (an image, or a band of rows).
// Workgroup = 4 waves (one per SIMD), one (chunk, ky, co-block); wave w owns 3 of
// the 12 16-wide N tiles (48 f32 accumulator VGPRs).  The three ky workgroups of
// a chunk are launched 1 XCD apart in blockIdx (bid = ky*nchunks + chunk) so the
// second and third reads of the chunk's dY / X come from the same L2.
//
// Data movement: per 2-row stage the dY tile (2 x TW px) and the 2 input rows
// the stage needs for this ky (2 x TW+2 px, zero-padded) are DMA'd straight
// into LDS with global_load_lds_dwordx4 (swizzle applied on the SOURCE address,
// LDS image lane-linear), 4 stages in flight, counted s_waitcnt vmcnt + raw
// s_barrier -- no VGPR staging.  Both MFMA operands are read K(pixel)-major
// with ds_read_b64_tr_b16 (v_mfma_f32_16x16x32_bf16).
// Each workgroup writes one partial slab; wgrad_reduce sums the slabs in a fixed
// order (deterministic) into the torch-layout gradient.
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

template <int TW>
struct Wg2 {
  static constexpr int DY_PIX = 2 * TW;
  static constexpr int X_PIX = 2 * (TW + 2);
  static constexpr int DY_BYTES = DY_PIX * 128;
  static constexpr int X_BYTES = X_PIX * 128;
  static constexpr int RAW = DY_BYTES + X_BYTES;
  static constexpr int NI = ((RAW + 4095) / 4096) * 4;     // 1 KiB DMA instructions per stage (multiple of 4)
  static constexpr int NIW = NI / 4;                        // per wave
  static constexpr int STAGE = NI * 1024;
  static constexpr int NSTG = 4;
  static constexpr int TOTAL = NSTG * STAGE + 4 * 64 * 4;   // + bias-sum scratch
};

// LDS-DMA of 16 bytes per lane: LDS[lds_base + 16*lane] <- *src.  Issued through
// inline asm so that hipcc does not treat the in-flight DMA as aliasing every later
// ds_read (it would drain the whole ring with vmcnt(0)); completion is ordered by
// our own counted s_waitcnt vmcnt + s_barrier (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_base)
      : "memory");
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int TW>
__global__ void __launch_bounds__(256, 1) wgrad3x3_kernel(WgradParams p) {
  using S = Wg2<TW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nchunks = gridDim.x / 3;
  const int ky = blockIdx.x / nchunks, chunk = blockIdx.x - ky * nchunks;
  const int cb = blockIdx.y;
  const int Hr = p.H / p.row_splits;
  const int n = chunk / p.row_splits, ybase = (chunk % p.row_splits) * Hr;
  const int nxb = p.W / TW;
  const int nst = (Hr / 2) * nxb;

  // ---------------------------------------------------------------- DMA issue
  // stage st -> rows (ybase + 2*(st / nxb)) .. +1, columns x0 .. x0+TW-1
  auto issue = [&](int st) {
    const int y0 = ybase + 2 * (st / nxb), x0 = (st % nxb) * TW;
    const uint32_t base = lds_u32(smem) + (st % S::NSTG) * S::STAGE;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
    for (int j = 0; j < S::NIW; ++j) {
      const int i = wv + 4 * j;                   // instruction index within the stage (wave-uniform)
      const int b = i * 1024 + lane * 16;          // destination byte (lane-linear)
      const void* src = p.zeros;
      if (b < S::DY_BYTES) {
        const int q = b >> 7, c = ((b >> 4) & 7) ^ ((((q >> 1) & 1) << 1) | (((q >> 3) & 1) << 2));
        const int r = q / TW, xx = x0 + q - r * TW, y = y0 + r;
        if (p.dy_mode == IN_PLAIN)
          src = p.dy + ((size_t)((size_t)n * p.H + y) * p.W + xx) * p.Cout + cb * 64 + c * 8;
        else
          src = p.dy + ((size_t)((size_t)n * 2 * p.H + 2 * y + (cb >> 1)) * (2 * p.W) + 2 * xx + (cb & 1)) * 64 + c * 8;
      } else if (b < S::DY_BYTES + S::X_BYTES) {
        const int bb = b - S::DY_BYTES;
        const int q = bb >> 7, c = ((bb >> 4) & 7) ^ ((((q >> 1) & 1) << 1) | (((q >> 3) & 1) << 2));
        const int r = q / (TW + 2), hx = q - r * (TW + 2);
        const int y = y0 + r + ky - 1, xx = x0 - 1 + hx;
        if (y >= 0 && y < p.H && xx >= 0 && xx < p.W)
          src = p.x + ((size_t)((size_t)n * p.H + y) * p.W + xx) * 64 + c * 8;
      }
      glds16(src, (uint32_t)__builtin_amdgcn_readfirstlane(base + i * 1024));
    }
  };

  f32x4 acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  // lane coordinates for the transposed reads
  const int g = lane >> 4, li = lane & 15, lq = li >> 2, lp = li & 3;
  const int prow = g >> 1;
  const int pcol = 8 * (g & 1) + lq;
  const uint32_t half = (lp & 1) * 8;
  // this wave's 3 N tiles: j = 3*wave + t -> (kx, ci tile)
  int nkx[3], nit[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int j = 3 * wave + t;
    nkx[t] = j >> 2;
    nit[t] = j & 3;
  }

  // prologue: NSTG-1 stages in flight
#pragma unroll
  for (int s = 0; s < S::NSTG - 1; ++s)
    if (s < nst) issue(s);

#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const int ahead = min(nst - 1, st + S::NSTG - 2) - st;   // stages issued after st
    if (ahead >= 2)
      wait_vm<2 * S::NIW>();
    else if (ahead == 1)
      wait_vm<S::NIW>();
    else
      wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // keep LDS reads and the next DMA below the barrier
    if (st + S::NSTG - 1 < nst) issue(st + S::NSTG - 1);
    const char* dyl = smem + (st % S::NSTG) * S::STAGE;
    const char* xl = dyl + S::DY_BYTES;
    // K-steps of 32 pixels; fragments double-buffered in registers so that step
    // kb+1's transposed reads are in flight while step kb's 12 MFMAs run
    bf16x8 A[2][4], B[2][3];
    auto load_step = [&](int kb, bf16x8 (&a)[4], bf16x8 (&b)[3]) {
      const int px0 = prow * TW + kb * 16 + pcol;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int chunk = 2 * ct + (lp >> 1);
        a[ct] = cat_tr(lds_tr(dyl, swz128t(px0, chunk) + half), lds_tr(dyl, swz128t(px0 + 4, chunk) + half));
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int chunk = 2 * nit[t] + (lp >> 1);
        const int hq0 = prow * (TW + 2) + kb * 16 + pcol + nkx[t];
        b[t] = cat_tr(lds_tr(xl, swz128t(hq0, chunk) + half), lds_tr(xl, swz128t(hq0 + 4, chunk) + half));
      }
    };
    load_step(0, A[0], B[0]);
#pragma unroll
    for (int kb = 0; kb < TW / 16; ++kb) {
      if (kb + 1 < TW / 16) load_step(kb + 1, A[(kb + 1) & 1], B[(kb + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[ct][t] = mfma16(A[kb & 1][ct], B[kb & 1][t], acc[ct][t]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (ky == 0) {  // bias gradient: lane = channel, pixels strided over the 4 waves
      for (int px = wave; px < S::DY_PIX; px += 4) {
        const bf16_t v = *reinterpret_cast<const bf16_t*>(dyl + swz128t(px, lane >> 3) + (lane & 7) * 2);
        bsum += bf2f(v);
      }
    }
  }

  // epilogue: partial slab [chunk][Cout][9][64]
  float* slab = p.slab + (size_t)chunk * p.Cout * 576;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cb * 64 + ct * 16 + 4 * (lane >> 4) + r;
        const int ci = nit[t] * 16 + (lane & 15);
        slab[((size_t)co * 9 + ky * 3 + nkx[t]) * 64 + ci] = acc[ct][t][r];
      }
  if (ky == 0) {
    float* red = reinterpret_cast<float*>(smem + S::NSTG * S::STAGE);
    red[wave * 64 + lane] = bsum;
    __syncthreads();
    if (tid < 64) p.bslab[(size_t)chunk * p.Cout + cb * 64 + tid] = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid];
  }
}

int wgrad3x3_nslabs(const WgradParams& p) { return p.N * p.row_splits; }

int wgrad3x3_launch(const WgradParams& p, hipStream_t st) {
  if (p.Cout % 64 || p.H % p.row_splits || (p.H / p.row_splits) % 2 || !p.zeros) return SRMI_ERR_SHAPE;
  if (p.dy_mode == IN_UNSHUF && p.Cout != 256) return SRMI_ERR_SHAPE;
  dim3 grid(3 * wgrad3x3_nslabs(p), p.Cout / 64);
  if (p.W % 48 == 0) {
    hipLaunchKernelGGL(wgrad3x3_kernel<48>, grid, dim3(256), Wg2<48>::TOTAL, st, p);
  } else if (p.W % 32 == 0) {
    hipLaunchKernelGGL(wgrad3x3_kernel<32>, grid, dim3(256), Wg2<32>::TOTAL, st, p);
  } else {
    return SRMI_ERR_SHAPE;
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

// -------------------------------------------------------------------- reduce
// one block = 64 consecutive outputs x 4 slab lanes; fixed summation order
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab,
                                                           const float* __restrict__ bslab, int nslab, int Cout,
                                                           int ps, float alpha, float* __restrict__ gw,
                                                           float* __restrict__ gb) {
  __shared__ float red[4][64];
  const int per = Cout * 576;
  const int o = blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  const bool is_w = o < per;
  const bool is_b = !is_w && gb && o < per + Cout;
  float s0 = 0.f, s1 = 0.f;
  if (is_w) {
    int k = q;
    for (; k + 4 < nslab; k += 8) {
      s0 += slab[(size_t)k * per + o];
      s1 += slab[(size_t)(k + 4) * per + o];
    }
    if (k < nslab) s0 += slab[(size_t)k * per + o];
  } else if (is_b) {
    for (int k = q; k < nslab; k += 4) s0 += bslab[(size_t)k * Cout + (o - per)];
  }
  red[q][threadIdx.x & 63] = s0 + s1;
  __syncthreads();
  if (q == 0 && (is_w || is_b)) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (is_w) {
      const int ci = o & 63, tap = (o >> 6) % 9, cop = o / 576;
      const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
      gw[((size_t)cot * 64 + ci) * 9 + tap] = alpha * s;
    } else {
      const int cop = o - per;
      const int cot = ps ? (4 * (cop & 63) + (cop >> 6)) : cop;
      gb[cot] = alpha * s;
    }
  }
}

int wgrad_reduce_launch(const float* slab, const float* bslab, int nslab, int Cout, int ps, float alpha, float* gw,
                        float* gb, hipStream_t st) {
  const int total = Cout * 576 + Cout;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 63) / 64), dim3(256), 0, st, slab, bslab, nslab, Cout, ps,
                     alpha, gw, gb);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
