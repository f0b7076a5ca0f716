// 3x3 "same" convolution as an MFMA implicit GEMM on gfx950 (CDNA4).
//
// Replaces nn.Conv2d(k=3, padding=1) built by default_conv
// (reference sres/model/common/cnn.py:8-9) for every 64->64 / 64->256 conv of
// RCAN (sres/model/rcan/network.py:13-16,55,71; blocks.py:64-65) and EDSR,
// forward AND data-gradient (dgrad = the same conv on dY with the flipped,
// transposed filter bank packed by pack.hip).
//
// Layout: activations NHWC bf16, 64 channels per 128-byte pixel row.
// One workgroup = 4 waves = one strip of TH=4 output rows x TW (32|48) columns of
// one image, one 64-wide block of output channels.  Per 64-channel input chunk
// the (TH+2)x(TW+2) halo is staged once in LDS (swizzled, conflict-free
// ds_read_b128); the 9 per-tap [64 co][64 ci] filter slices stream through a
// double-buffered LDS ring.  Wave w computes output row w:  A = filters
// (M = co), B = halo pixels (N = px), K = ci, with v_mfma_f32_16x16x32_bf16, so
// each lane ends up owning 4 consecutive channels of one pixel -> vectorised,
// fused epilogues (bias, ReLU, channel-attention pooling, residual add,
// PixelShuffle scatter, ReLU-mask for dgrad, residual-stream gradient add with
// the CA reductions).
#include <stdlib.h>

#include <algorithm>

#include <cstdlib>

#include "common.hpp"
#include "conv64_body.hpp"
#include "srmi_internal.hpp"

namespace srmi {

static unsigned long long* g_debug_stamps = nullptr;
void conv3x3_set_debug_stamps(unsigned long long* buf) { g_debug_stamps = buf; }
unsigned long long* conv3x3_debug_stamps() { return g_debug_stamps; }
// diagnostic build: SRMI_STAMP_EPI=<epilogue> stamps only that epilogue's launches
unsigned long long* conv3x3_stamps_for(int epi) {
#ifdef SRMI_STAMPS
  const char* only = std::getenv("SRMI_STAMP_EPI");
  if (only && std::atoi(only) != epi) return nullptr;
#endif
  (void)epi;
  return g_debug_stamps;
}

template <int TW>
struct ConvSmem {
  static constexpr int HALO_PIX = (kTH + 2) * (TW + 2);
  static constexpr int HALO_BYTES = HALO_PIX * 128;
  static constexpr int W_BYTES = 64 * 128;  // one tap slice [64 co][64 ci]
  static constexpr int TOTAL = HALO_BYTES + 2 * W_BYTES;
};

// every load of the thread in flight at once (clamped addresses, padding selected
// to zero afterwards): a load-wait-store loop serialised one memory latency per
// 16-byte chunk
template <int NPIX>
struct HaloRegs {
  static constexpr int NCH = NPIX * 8, NL = (NCH + kThreads - 1) / kThreads;
  uint4 v[NL];
};

// issue: every 16-B chunk of this thread's share of the chunk-cc halo into registers
template <int NPIX>
__device__ __forceinline__ void halo_issue(HaloRegs<NPIX>& hr, const bf16_t* __restrict__ x, int mode, int n, int H,
                                           int W, int Cin, int cc, int y0, int x0, int TWp2) {
  const int tid = threadIdx.x;
  constexpr int NCH = HaloRegs<NPIX>::NCH, NL = HaloRegs<NPIX>::NL;
  uint4* hv = hr.v;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = min(tid + j * kThreads, NCH - 1);
    const int q = i >> 3, c = i & 7;
    const int hy = q / TWp2, hx = q - hy * TWp2;
    const int y = min(max(y0 - 1 + hy, 0), H - 1), xx = min(max(x0 - 1 + hx, 0), W - 1);
    const bf16_t* src = mode == IN_PLAIN
                            ? x + ((size_t)((size_t)n * H + y) * W + xx) * Cin + cc * 64 + c * 8
                            // IN_UNSHUF: logical [H][W][4*64] view of a physical [2H][2W][64] map
                            : x + ((size_t)((size_t)n * 2 * H + 2 * y + (cc >> 1)) * (2 * W) + 2 * xx + (cc & 1)) * 64 + c * 8;
    hv[j] = *reinterpret_cast<const uint4*>(src);
  }
}

// workgroup barrier ordering LDS only (__syncthreads' release fence drains vmcnt,
// which would wait for the prefetched slices and halo)
__device__ __forceinline__ void lds_only_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// commit: the registers into the swizzled LDS halo, padding zeroed
template <int NPIX>
__device__ __forceinline__ void halo_commit(char* halo, const HaloRegs<NPIX>& hr, int H, int W, int y0, int x0,
                                            int TWp2) {
  const int tid = threadIdx.x;
  constexpr int NCH = HaloRegs<NPIX>::NCH, NL = HaloRegs<NPIX>::NL;
  const uint4* hv = hr.v;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    const int i = tid + j * kThreads;
    if (i < NCH) {
      const int q = i >> 3, c = i & 7;
      const int hy = q / TWp2, hx = q - hy * TWp2;
      const int y = y0 - 1 + hy, xx = x0 - 1 + hx;
      const bool ok = y >= 0 && y < H && xx >= 0 && xx < W;
      *reinterpret_cast<uint4*>(halo + swz128(q, c)) = ok ? hv[j] : make_uint4(0, 0, 0, 0);
    }
  }
}

// Fused epilogue shared by both conv kernels.  acc[pt][ct]: lane owns channels
// ct*16 + 4*(lane>>4) + {0..3} of pixel (y, x0 + pt*16 + (lane&15)).
template <int NPT, int EPI>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, f32x4 (&acc)[NPT][4], int n, int cb, int y, int x0,
                                              int strip, int nstrips, float* red, int fr, int fk, int wave, int tid) {
  const int HW = p.H * p.W;
  constexpr bool kPart1 = (EPI == EPI_POOL_BF16);
  constexpr bool kPart2 = (EPI == EPI_DG_ACC || EPI == EPI_DG_ACC_CA);
  float ps0[4][4], ps1[4][4];  // per (ct, r) partial sums over this lane's pixels
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) ps0[ct][r] = ps1[ct][r] = 0.f;

#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) {
    const int xx = x0 + pt * 16 + fr;
    const size_t pix = (size_t)n * HW + (size_t)y * p.W + xx;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int col = ct * 16 + fk * 4;           // channel within the 64-block
      const int co = cb * 64 + col;               // packed output channel
      f32x4 v = acc[pt][ct];
      if constexpr (EPI == EPI_RELU_BF16 || EPI == EPI_POOL_BF16 || EPI == EPI_RESID || EPI == EPI_PS_BF16) {
        const float4 bb = *reinterpret_cast<const float4*>(p.bias + co);
        v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      } else if constexpr (EPI == EPI_PLAIN_BF16) {
        if (p.bias) {
          const float4 bb = *reinterpret_cast<const float4*>(p.bias + co);
          v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
        }
      }
      if constexpr (EPI == EPI_RELU_BF16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if constexpr (EPI == EPI_RESID) {
        const size_t o = pix * p.Cout + co;
        const float4 rr = *reinterpret_cast<const float4*>(p.r1 + o);
        v[0] = p.alpha * v[0] + rr.x; v[1] = p.alpha * v[1] + rr.y;
        v[2] = p.alpha * v[2] + rr.z; v[3] = p.alpha * v[3] + rr.w;
        if (p.yf) *reinterpret_cast<float4*>(p.yf + o) = make_float4(v[0], v[1], v[2], v[3]);
      }
      if constexpr (EPI == EPI_DG_RELUMASK) {
        const size_t o = pix * p.Cout + co;
        const uint2 tt = *reinterpret_cast<const uint2*>(p.aux + o);
        v[0] = (tt.x & 0xFFFFu) && !(tt.x & 0x8000u) ? v[0] : 0.f;
        v[1] = (tt.x >> 16) && !(tt.x & 0x80000000u) ? v[1] : 0.f;
        v[2] = (tt.y & 0xFFFFu) && !(tt.y & 0x8000u) ? v[2] : 0.f;
        v[3] = (tt.y >> 16) && !(tt.y & 0x80000000u) ? v[3] : 0.f;
        v[0] *= p.alpha; v[1] *= p.alpha; v[2] *= p.alpha; v[3] *= p.alpha;
      }
      if constexpr (EPI == EPI_DG_ACC) {
        const size_t o = pix * p.Cout + co;
        if (p.r1) {
          const float4 rr = *reinterpret_cast<const float4*>(p.r1 + o);
          v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
        }
        if (p.r2) {
          const float4 rr = *reinterpret_cast<const float4*>(p.r2 + o);
          v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
        }
        if (p.r3) {
          const float4 rr = *reinterpret_cast<const float4*>(p.r3 + o);
          v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
        }
        *reinterpret_cast<float4*>(p.yf + o) = make_float4(v[0], v[1], v[2], v[3]);
        if (p.part) {
          const uint2 uu = *reinterpret_cast<const uint2*>(p.aux + o);
          ps0[ct][0] += v[0]; ps0[ct][1] += v[1]; ps0[ct][2] += v[2]; ps0[ct][3] += v[3];
          ps1[ct][0] += v[0] * bf2f(uu.x & 0xFFFFu);
          ps1[ct][1] += v[1] * bf2f(uu.x >> 16);
          ps1[ct][2] += v[2] * bf2f(uu.y & 0xFFFFu);
          ps1[ct][3] += v[3] * bf2f(uu.y >> 16);
        }
      }
      if constexpr (kPart1) {
        ps0[ct][0] += v[0]; ps0[ct][1] += v[1]; ps0[ct][2] += v[2]; ps0[ct][3] += v[3];
      }
      // bf16 store
      uint2 packed = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      if constexpr (EPI == EPI_PS_BF16) {
        // PixelShuffle(2): packed channel block cb = 2i+j -> output pixel (2y+i, 2x+j)
        const int oy = 2 * y + (cb >> 1), ox = 2 * xx + (cb & 1);
        const size_t o = ((size_t)n * (2 * p.H) + oy) * (size_t)(2 * p.W) + ox;
        *reinterpret_cast<uint2*>(p.yb + o * 64 + col) = packed;
      } else {
        if (p.yb) *reinterpret_cast<uint2*>(p.yb + pix * p.Cout + co) = packed;
      }
    }
  }

  if constexpr (kPart1 || kPart2) {
    // reduce over the 16 pixel-lanes, then over the 4 waves via LDS
    __syncthreads();
    if (!kPart2 || p.part) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float s0 = sum16(ps0[ct][r]);
          float s1 = 0.f;
          if constexpr (kPart2) s1 = sum16(ps1[ct][r]);
          if (fr == 0) {
            red[(wave * 2 + 0) * 64 + ct * 16 + fk * 4 + r] = s0;
            if constexpr (kPart2) red[(wave * 2 + 1) * 64 + ct * 16 + fk * 4 + r] = s1;
          }
        }
    }
    __syncthreads();
    if (!kPart2 || p.part) {
      if (tid < 64) {
        const float s = red[0 * 128 + tid] + red[1 * 128 + tid] + red[2 * 128 + tid] + red[3 * 128 + tid];
        p.part[((size_t)n * nstrips + strip) * p.part_stride + cb * 64 + tid] = s;
      } else if (kPart2 && tid < 128) {
        const int c = tid - 64;
        const float s = red[0 * 128 + 64 + c] + red[1 * 128 + 64 + c] + red[2 * 128 + 64 + c] + red[3 * 128 + 64 + c];
        p.part[((size_t)n * nstrips + strip) * p.part_stride + 64 + c] = s;
      }
    }
  }
}

template <int TW, int EPI>
__global__ void __launch_bounds__(kThreads, 2) conv3x3_kernel(ConvParams p) {
  using S = ConvSmem<TW>;
  constexpr int NPT = TW / 16;  // 16-pixel tiles per row
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* halo = smem;
  char* wbuf = smem + S::HALO_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int strips_x = p.W / TW;
  const int sy = blockIdx.x / strips_x, sx = blockIdx.x - sy * strips_x;
  const int y0 = sy * kTH, x0 = sx * TW;
  const int cb = blockIdx.y, n = blockIdx.z;
  const int nchunks = p.Cin >> 6;
  const bf16_t* __restrict__ wsrc = p.w;

  f32x4 acc[NPT][4];
#pragma unroll
  for (int i = 0; i < NPT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // lane-constant fragment coordinates
  const int fr = lane & 15;   // A row (co within tile) / B column (pixel within tile)
  const int fk = lane >> 4;   // 8-wide k group

  // The K dimension as one stream of nchunks*9 filter slices s = (cc, tap), each
  // [64 co][64 ci] = 8 KiB.  A slice's global load is issued three slices before
  // its use (register ring of 3, stored to the LDS double buffer one slice
  // ahead), and the next chunk's halo is loaded into registers while the current
  // chunk's nine taps run: a slice's compute (24 MFMAs per wave) is far shorter
  // than one global latency, so loading one slice ahead left every tap waiting.
  const int nslices = nchunks * 9;
  auto slice_src = [&](int s) {
    return wsrc + ((size_t)s * p.Cout + cb * 64) * 64;  // (cc*9 + tap) slices are consecutive
  };
  auto slice_issue = [&](uint4& r0, uint4& r1, int s) {
    const bf16_t* ws = slice_src(min(s, nslices - 1));  // clamped, unconditional
    r0 = *reinterpret_cast<const uint4*>(ws + (tid >> 3) * 64 + (tid & 7) * 8);
    r1 = *reinterpret_cast<const uint4*>(ws + ((tid + kThreads) >> 3) * 64 + (tid & 7) * 8);
  };
  auto slice_commit = [&](const uint4& r0, const uint4& r1, int buf) {
    char* wn = wbuf + buf * S::W_BYTES;
    *reinterpret_cast<uint4*>(wn + swz128(tid >> 3, tid & 7)) = r0;
    *reinterpret_cast<uint4*>(wn + swz128((tid + kThreads) >> 3, tid & 7)) = r1;
  };

  // register ring of three slices (named, so that it stays in registers)
  HaloRegs<S::HALO_PIX> hr;
  uint4 ra0, ra1, rb0, rb1, rc0, rc1;
  halo_issue<S::HALO_PIX>(hr, p.x, p.in_mode, n, p.H, p.W, p.Cin, 0, y0, x0, TW + 2);
  slice_issue(ra0, ra1, 0);
  slice_issue(rb0, rb1, 1);
  slice_issue(rc0, rc1, 2);
  halo_commit<S::HALO_PIX>(halo, hr, p.H, p.W, y0, x0, TW + 2);
  slice_commit(ra0, ra1, 0);
  lds_only_barrier();

  // one slice: reload slot (q0, q1) (slice s, committed at the end of slice s - 1)
  // with s + 3, run the 24 MFMAs, commit slot (n0, n1) = slice s + 1
  auto step = [&](const int cc, const int tap, uint4& q0, uint4& q1, const uint4& n0, const uint4& n1) {
    const int s = cc * 9 + tap;
    slice_issue(q0, q1, s + 3);
    const char* wb = wbuf + (s & 1) * S::W_BYTES;
    const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fk;
      bf16x8 a[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) a[ct] = lds_frag(wb, swz128(ct * 16 + fr, chunk));
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) {
        const int q = (wave + ky) * (TW + 2) + pt * 16 + fr + kx;
        const bf16x8 b = lds_frag(halo, swz128(q, chunk));
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[pt][ct] = mfma16(a[ct], b, acc[pt][ct]);
      }
    }
    if (s + 1 < nslices) {
      // buffer (s+1)&1 was last read by slice s-1, behind the previous barrier
      slice_commit(n0, n1, (s + 1) & 1);
      if (tap == 8) {  // the next chunk's halo, issued before the barrier that frees the LDS halo
        halo_issue<S::HALO_PIX>(hr, p.x, p.in_mode, n, p.H, p.W, p.Cin, cc + 1, y0, x0, TW + 2);
        lds_only_barrier();
        halo_commit<S::HALO_PIX>(halo, hr, p.H, p.W, y0, x0, TW + 2);
      }
    }
    // LDS-only barrier: the prefetched slices and halo stay in flight across it
    lds_only_barrier();
  };

#pragma unroll 1
  for (int cc = 0; cc < nchunks; ++cc) {
    step(cc, 0, ra0, ra1, rb0, rb1);
    step(cc, 1, rb0, rb1, rc0, rc1);
    step(cc, 2, rc0, rc1, ra0, ra1);
    step(cc, 3, ra0, ra1, rb0, rb1);
    step(cc, 4, rb0, rb1, rc0, rc1);
    step(cc, 5, rc0, rc1, ra0, ra1);
    step(cc, 6, ra0, ra1, rb0, rb1);
    step(cc, 7, rb0, rb1, rc0, rc1);
    step(cc, 8, rc0, rc1, ra0, ra1);
  }

  // ------------------------------------------------------------------ epilogue
  conv_epilogue<NPT, EPI>(p, acc, n, cb, y0 + wave, x0, blockIdx.x, gridDim.x, reinterpret_cast<float*>(smem), fr, fk,
                          wave, tid);
}

template <int TW, int EPI>
static int launch_tw(const ConvParams& p, hipStream_t st) {
  if (p.Cin == 64 && p.in_mode == IN_PLAIN) {
    // v2: persistent runs; ~1 workgroup per CU (LDS-limited), each a run of strips
    const int run_len = conv64_run_len(p, TW, p.cu_budget > 0 ? p.cu_budget : 256);
    dim3 grid(conv64_blocks(p, TW, run_len));
    ConvParams q = p;
    q.stamps = conv3x3_stamps_for(EPI);
    // 8 waves (two per SIMD, a wave per row and channel half) at TW = 48
    constexpr int NW = TW == 48 ? 8 : 4;
    hipLaunchKernelGGL((conv64_kernel<TW, EPI, NW>), grid, dim3(NW * 64), Conv2Smem<TW>::TOTAL, st, q, run_len);
  } else if constexpr (EPI == EPI_DG_ACC_CA16 || EPI == EPI_DG_CA16 || EPI == EPI_DG_ACC_G1) {
    return SRMI_ERR_SHAPE;  // (the bf16 gradient stream: the persistent-run body only)
  } else {
    // v1 handles the general form, without the bf16 gradient stream
    if (EPI == EPI_DG_ACC && (p.r1b || !p.yf)) return SRMI_ERR_SHAPE;
    constexpr int E1 = EPI == EPI_DG_ACC_CA ? EPI_DG_ACC : EPI;
    dim3 grid((p.H / kTH) * (p.W / TW), p.Cout / 64, p.N);
    hipLaunchKernelGGL((conv3x3_kernel<TW, E1>), grid, dim3(kThreads), ConvSmem<TW>::TOTAL, st, p);
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

// the epilogues only the 8-wave persistent-run body has (48-wide tiles, Cin = 64):
// conv1 with t's per-strip sums and the training conv2 with the CA residual update
template <int EPI>
static int launch_v2_only(const ConvParams& p, hipStream_t st) {
  if (p.Cin != 64 || p.Cout != 64 || p.in_mode != IN_PLAIN || p.W % 48 || p.H % kTH)
    return SRMI_ERR_SHAPE;
  const int run_len = conv64_run_len(p, 48, p.cu_budget > 0 ? p.cu_budget : 256);
  ConvParams q = p;
  q.stamps = conv3x3_stamps_for(EPI);
  size_t lds = Conv2Smem<48>::TOTAL;
  // (diagnostic: the scale's phase stamps after the body's, [grid][64] each)
  if (q.stamps && EPI == EPI_CA_RESID_U) q.cas.stamps = q.stamps + (size_t)conv64_blocks(p, 48, run_len) * 64;
  if (EPI == EPI_CA_RESID_U && p.cas_on) lds += kCaScaleFloats * sizeof(float);  // the scale's scratch
  if (EPI == EPI_RELU_POOL && p.cas_on) {  // conv1's partial CA means: the matvec's scratch
    if (!p.cas.mpart || !p.cas.wimg || p.cas.nruns != conv64_runs_per_image(p)) return SRMI_ERR_ARG;
    lds += kCaScaleFloats * sizeof(float);
  }
  hipLaunchKernelGGL((conv64_kernel<48, EPI, 8>), dim3(conv64_blocks(p, 48, run_len)), dim3(512), lds, st, q, run_len);
  SRMI_CHECK_LAUNCH();
  return 0;
}

template <int EPI>
static int launch_epi(const ConvParams& p, hipStream_t st) {
  if (p.W % 48 == 0 && p.H % kTH == 0) return launch_tw<48, EPI>(p, st);
  if (p.W % 32 == 0 && p.H % kTH == 0) return launch_tw<32, EPI>(p, st);
  return SRMI_ERR_SHAPE;
}

int conv3x3_tw(const ConvParams& p) {
  if (p.W % 48 == 0) return 48;
  if (p.W % 32 == 0) return 32;
  return 0;
}

int conv3x3_launch(const ConvParams& p, int epi, hipStream_t st) {
  if (p.Cin % 64 || p.Cout % 64 || p.N <= 0 || p.H % kTH) return SRMI_ERR_SHAPE;
  // operands each epilogue dereferences unconditionally: refuse, never fault
  if (!p.x || !p.w) return SRMI_ERR_ARG;
  if (p.gx.rec) return SRMI_ERR_ARG;  // (du formed from g: the fused backward launch only)
  if (epi == EPI_DG_ACC_CA && (!p.r1 || !p.aux || !p.part || p.yb || p.r2 || p.r3 || !p.yf || p.r1b))
    return SRMI_ERR_ARG;
  if (epi == EPI_DG_ACC_CA16 && (!p.r1b || !p.aux || !p.part || !p.yb || p.r1 || p.r2 || p.r3 || p.yf || p.f32))
    return SRMI_ERR_ARG;
  if (epi == EPI_DG_CA16 && (!p.aux || !p.part || !p.yb || p.r1 || p.r1b || p.r2 || p.r3 || p.yf || p.f32))
    return SRMI_ERR_ARG;
  if (epi == EPI_DG_ACC_G1 && (!p.r1b || !p.r2 || !p.yf || !p.yb || p.r1 || p.aux || p.part || p.f32))
    return SRMI_ERR_ARG;
  if (epi != EPI_DG_ACC && epi != EPI_DG_ACC_CA16 && epi != EPI_DG_ACC_G1 && p.r1b) return SRMI_ERR_ARG;
  switch (epi) {
    case EPI_PS_BF16:
      if (!p.yb) return SRMI_ERR_ARG;
      break;
    case EPI_POOL_BF16:
      if (!p.part) return SRMI_ERR_ARG;
      break;
    case EPI_RESID:
      if (!p.r1) return SRMI_ERR_ARG;
      break;
    case EPI_DG_RELUMASK:
      if (!p.aux) return SRMI_ERR_ARG;
      break;
    case EPI_DG_ACC:  // (yf may be null with a bf16 yb: the bf16 stream; r1 or r1b, not both)
      if ((!p.yf && !p.yb) || (p.part && !p.aux) || (p.r1 && p.r1b) || (p.f32 && (p.r1b || !p.yf)))
        return SRMI_ERR_ARG;
      break;
    case EPI_RELU_POOL:
      if (!p.yb || !p.part || p.f32) return SRMI_ERR_ARG;
      break;
    case EPI_CA_RESID_U:
      if (!p.yb || !p.yph || !p.ypl || (!p.r1 && (!p.r1h || !p.r1l)) || p.f32) return SRMI_ERR_ARG;
      if (p.cas_on) {
        if (!p.cas.w1 || !p.cas.b1 || !p.cas.w2 || !p.cas.b2 || !p.cas.bc2 || !p.cas.rec || p.cas.CR < 4 ||
            p.cas.CR > 32 || p.cas.CR % 4)
          return SRMI_ERR_ARG;
        // SRMI_CA_MPART: s from conv1's partial means; else from t's border lines
        if (SRMI_CA_MPART ? (!p.cas.mpart || p.cas.nruns < 1)
                          : (!p.cas.t || !p.cas.part || p.cas.nstrips != conv3x3_nstrips(p.H, p.W)))
          return SRMI_ERR_ARG;
      } else if (!p.escale) {
        return SRMI_ERR_ARG;
      }
      break;
    default:
      break;
  }
  if (epi == EPI_PS_BF16 && p.Cout != 256) return SRMI_ERR_SHAPE;
  if (p.in_mode == IN_UNSHUF && p.Cin != 256) return SRMI_ERR_SHAPE;
  // outputs are stored through buffer resources whose byte range is 32-bit: an
  // output map of 2^32 bytes or more would wrap num_records and drop its stores.
  // Sized from the bytes each output actually holds: yb 2 B (bf16) or 4 B (f32
  // engine) per element, yf always 4 B -- the same quantity init_engine checks.
  {
    const size_t elems = (size_t)p.N * p.H * p.W * p.Cout;
    if (p.yb && elems * (p.f32 ? 4 : 2) >= (1ull << 32)) return SRMI_ERR_SHAPE;
    if (p.yf && elems * 4 >= (1ull << 32)) return SRMI_ERR_SHAPE;
  }
  if (p.f32) return conv3x3_f32_launch(p, epi, st);
  switch (epi) {
    case EPI_RELU_BF16: return launch_epi<EPI_RELU_BF16>(p, st);
    case EPI_POOL_BF16: return launch_epi<EPI_POOL_BF16>(p, st);
    case EPI_RESID: return launch_epi<EPI_RESID>(p, st);
    case EPI_PS_BF16: return launch_epi<EPI_PS_BF16>(p, st);
    case EPI_DG_RELUMASK: return launch_epi<EPI_DG_RELUMASK>(p, st);
    case EPI_DG_ACC: return launch_epi<EPI_DG_ACC>(p, st);
    case EPI_PLAIN_BF16: return launch_epi<EPI_PLAIN_BF16>(p, st);
    case EPI_DG_ACC_CA: return launch_epi<EPI_DG_ACC_CA>(p, st);
    case EPI_DG_ACC_CA16: return launch_epi<EPI_DG_ACC_CA16>(p, st);
    case EPI_DG_CA16: return launch_epi<EPI_DG_CA16>(p, st);
    case EPI_DG_ACC_G1: return launch_epi<EPI_DG_ACC_G1>(p, st);
    case EPI_RELU_POOL: return launch_v2_only<EPI_RELU_POOL>(p, st);
    case EPI_CA_RESID_U: return launch_v2_only<EPI_CA_RESID_U>(p, st);
    default: return SRMI_ERR_ARG;
  }
}

int conv64_runs_per_image(const ConvParams& p) {
  const int run_len = conv64_run_len(p, 48, p.cu_budget > 0 ? p.cu_budget : 256);
  return (p.W / 48) * ((p.H / kTH + run_len - 1) / run_len);
}

int conv3x3_nstrips(int H, int W) {
  const int tw = (W % 48 == 0) ? 48 : 32;
  return (H / kTH) * (W / tw);
}

}  // namespace srmi
