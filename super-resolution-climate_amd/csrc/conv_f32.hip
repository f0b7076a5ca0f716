// Exact-fp32 3x3 convolution (forward / dgrad) and filter gradient on gfx950's
// f32-input matrix cores (v_mfma_f32_16x16x4_f32: f32 operands, f32 accumulate,
// 64 FLOP/clk/SIMD = 157 TF chip-wide, bitwise an fmaf chain).
//
// The fp32 engine mode (srmi_model_config.dtype = SRMI_DTYPE_F32) replaces the
// reference's fp32 nn.Conv2d arithmetic (default_conv, sres/model/common/cnn.py:8-9;
// array2tensor fp32, sres/base/util/array.py:70) with no bf16 rounding anywhere:
// activations and gradients are NHWC fp32 (256 B per 64-channel pixel row), the
// filter packs are fp32.  At 1/16 of the bf16 MFMA rate a 64->64 conv is firmly
// MFMA-bound (10.9 GFLOP / 157 TF = 69 us at B=64 against 9.4 us of HBM traffic),
// so these kernels aim at keeping one MFMA chain per SIMD fed, nothing more.
//
// MFMA lane maps (16x16x4 f32): A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15],
// D[row 4 (l >> 4) + r][col l & 15].
#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

namespace {

static __device__ float4 kZerosF[16];  // zero page: LDS-DMA source of padding pixels

__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 16-byte chunk c (channels 4c..4c+3) of pixel row q lives at slot c ^ (q & 15) of
// the 256-byte LDS row: ds_read_b128 of 16 consecutive rows at one chunk (A: 16
// output channels; B: 16 consecutive pixels) hits 16 distinct slots.
__device__ __forceinline__ uint32_t swz256(uint32_t q, uint32_t c) { return q * 256u + ((c ^ (q & 15u)) << 4); }

constexpr int kTH = 4;  // output rows per workgroup (one per wave)

template <int TW>
struct CF32Smem {
  static constexpr int HALO_PIX = (kTH + 2) * (TW + 2);
  static constexpr int HALO_BYTES = HALO_PIX * 256;
  static constexpr int W_BYTES = 64 * 256;  // one tap slice [64 co][64 ci] fp32
  static constexpr int TOTAL = HALO_BYTES + 2 * W_BYTES;
};

// fused epilogue (same semantics as the bf16 kernels' conv_epilogue, fp32 outputs)
// (a wave holds row `row` of the strip, output-channel tiles ct0 .. ct0+NCT-1)
template <int NPT, int EPI, int NCT = 4>
__device__ __forceinline__ void epilogue_f32(const ConvParams& p, f32x4 (&acc)[NPT][NCT], int n, int cb, int y, int x0,
                                             int strip, int nstrips, float* red, int fr, int fk, int row, int ct0,
                                             int tid) {
  const size_t HW = (size_t)p.H * p.W;
  float* yb = reinterpret_cast<float*>(p.yb);
  const float* aux = reinterpret_cast<const float*>(p.aux);
  constexpr bool kPart1 = (EPI == EPI_POOL_BF16);
  constexpr bool kPart2 = (EPI == EPI_DG_ACC);
  float ps0[NCT][4], ps1[NCT][4];
#pragma unroll
  for (int c = 0; c < NCT; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) ps0[c][r] = ps1[c][r] = 0.f;
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) {
    const int xx = x0 + pt * 16 + fr;
    const size_t pix = (size_t)n * HW + (size_t)y * p.W + xx;
#pragma unroll
    for (int c = 0; c < NCT; ++c) {
      const int ct = ct0 + c;
      const int col = ct * 16 + fk * 4;
      const int co = cb * 64 + col;
      const size_t o = pix * p.Cout + co;
      f32x4 v = acc[pt][c];
      if constexpr (EPI == EPI_RELU_BF16 || EPI == EPI_POOL_BF16 || EPI == EPI_RESID || EPI == EPI_PS_BF16 ||
                    EPI == EPI_PLAIN_BF16) {
        if (EPI != EPI_PLAIN_BF16 || p.bias) {
          const float4 bb = *reinterpret_cast<const float4*>(p.bias + co);
          v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
        }
      }
      if constexpr (EPI == EPI_RELU_BF16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if constexpr (EPI == EPI_RESID) {
        const float4 rr = *reinterpret_cast<const float4*>(p.r1 + o);
        v[0] = p.alpha * v[0] + rr.x; v[1] = p.alpha * v[1] + rr.y;
        v[2] = p.alpha * v[2] + rr.z; v[3] = p.alpha * v[3] + rr.w;
        if (p.yf) *reinterpret_cast<float4*>(p.yf + o) = make_float4(v[0], v[1], v[2], v[3]);
      }
      if constexpr (EPI == EPI_DG_RELUMASK) {
        const float4 t = *reinterpret_cast<const float4*>(aux + o);
        v[0] = t.x > 0.f ? p.alpha * v[0] : 0.f;
        v[1] = t.y > 0.f ? p.alpha * v[1] : 0.f;
        v[2] = t.z > 0.f ? p.alpha * v[2] : 0.f;
        v[3] = t.w > 0.f ? p.alpha * v[3] : 0.f;
      }
      if constexpr (EPI == EPI_DG_ACC) {
        const float* rs[3] = {p.r1, p.r2, p.r3};
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (rs[k]) {
            const float4 rr = *reinterpret_cast<const float4*>(rs[k] + o);
            v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
          }
        *reinterpret_cast<float4*>(p.yf + o) = make_float4(v[0], v[1], v[2], v[3]);
        if (p.part) {
          const float4 uu = *reinterpret_cast<const float4*>(aux + o);
          ps0[c][0] += v[0]; ps0[c][1] += v[1]; ps0[c][2] += v[2]; ps0[c][3] += v[3];
          ps1[c][0] += v[0] * uu.x; ps1[c][1] += v[1] * uu.y;
          ps1[c][2] += v[2] * uu.z; ps1[c][3] += v[3] * uu.w;
        }
      }
      if constexpr (kPart1) {
        ps0[c][0] += v[0]; ps0[c][1] += v[1]; ps0[c][2] += v[2]; ps0[c][3] += v[3];
      }
      const float4 ov = make_float4(v[0], v[1], v[2], v[3]);
      if constexpr (EPI == EPI_PS_BF16) {
        // PixelShuffle(2): packed channel block cb = 2i+j -> output pixel (2y+i, 2x+j)
        const int oy = 2 * y + (cb >> 1), ox = 2 * xx + (cb & 1);
        const size_t op = ((size_t)n * (2 * p.H) + oy) * (size_t)(2 * p.W) + ox;
        *reinterpret_cast<float4*>(yb + op * 64 + col) = ov;
      } else {
        if (yb) *reinterpret_cast<float4*>(yb + o) = ov;
      }
    }
  }
  if constexpr (kPart1 || kPart2) {
    __syncthreads();  // every wave is past its last LDS read of the K loop
    const bool on = !kPart2 || p.part;
    if (on) {
#pragma unroll
      for (int c = 0; c < NCT; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ct = ct0 + c;
          const float s0 = sum16(ps0[c][r]);
          float s1 = 0.f;
          if constexpr (kPart2) s1 = sum16(ps1[c][r]);
          if (fr == 0) {
            red[(row * 2 + 0) * 64 + ct * 16 + fk * 4 + r] = s0;
            if constexpr (kPart2) red[(row * 2 + 1) * 64 + ct * 16 + fk * 4 + r] = s1;
          }
        }
    }
    __syncthreads();
    if (on) {
      if (tid < 64) {
        const float s = red[tid] + red[128 + tid] + red[256 + tid] + red[384 + tid];
        p.part[((size_t)n * nstrips + strip) * p.part_stride + cb * 64 + tid] = s;
      } else if (kPart2 && tid < 128) {
        const int c = tid - 64;
        const float s = red[64 + c] + red[192 + c] + red[320 + c] + red[448 + c];
        p.part[((size_t)n * nstrips + strip) * p.part_stride + 64 + c] = s;
      }
    }
  }
}

// One workgroup = 4 waves = a strip of 4 output rows x TW columns of one image and
// one 64-wide block of output channels.  Per 64-channel input chunk the
// (TH+2) x (TW+2) halo is staged in LDS; the 9 per-tap [64 co][64 ci] filter slices
// stream through a double-buffered LDS ring (next tap held in registers during the
// MFMAs).  Wave w computes output row w; per tap and 16-channel group g a lane reads
// ONE float4 per A tile (filter row) and per B tile (pixel) -- K index k of MFMA s
// is channel 16g + 4k + s -- and issues 16 x NPT MFMAs with them.
//
// NW = 8: two waves per SIMD, a wave per row and output-channel half (the 16x16x4
// f32 MFMA's 32-cycle issue interval leaves one wave's LDS reads and waits exposed).
template <int TW, int EPI, int NW>
__global__ void __launch_bounds__(NW * 64, 1) conv3x3_f32_kernel(ConvParams p) {
  using S = CF32Smem<TW>;
  constexpr int NPT = TW / 16;
  constexpr int NT = NW * 64, NCT = NW == 8 ? 2 : 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* halo = smem;
  char* wbuf = smem + S::HALO_BYTES;
  const float* X = reinterpret_cast<const float*>(p.x);
  const float* Wp = reinterpret_cast<const float*>(p.w);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = wave & 3, ct0 = NCT * (wave >> 2);
  const int fr = lane & 15, fk = lane >> 4;
  const int strips_x = p.W / TW;
  const int sy = blockIdx.x / strips_x, sx = blockIdx.x - sy * strips_x;
  const int y0 = sy * kTH, x0 = sx * TW;
  const int cb = blockIdx.y, n = blockIdx.z;
  const int nchunks = p.Cin >> 6;

  f32x4 acc[NPT][NCT];
#pragma unroll
  for (int i = 0; i < NPT; ++i)
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int cc = 0; cc < nchunks; ++cc) {
    if (cc) __syncthreads();
    // halo chunk: (TH+2)(TW+2) pixels x 16 float4, every load of the thread in
    // flight at once (clamped addresses, padding selected to zero afterwards): a
    // load-wait-store loop serialised one memory latency per float4
    {
      constexpr int NH = (S::HALO_PIX * 16 + NT - 1) / NT;
      float4 hv[NH];
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        const int i = min(tid + j * NT, S::HALO_PIX * 16 - 1);
        const int q = i >> 4, c = i & 15;
        const int hy = q / (TW + 2), hx = q - hy * (TW + 2);
        const int yy = min(max(y0 - 1 + hy, 0), p.H - 1), xx = min(max(x0 - 1 + hx, 0), p.W - 1);
        const float* src = p.in_mode == IN_PLAIN
                               ? X + ((size_t)((size_t)n * p.H + yy) * p.W + xx) * p.Cin + cc * 64 + c * 4
                               // IN_UNSHUF: logical [H][W][256] view of the PixelShuffle output [2H][2W][64]
                               : X + ((size_t)((size_t)n * 2 * p.H + 2 * yy + (cc >> 1)) * (2 * p.W) + 2 * xx + (cc & 1)) * 64 +
                                     c * 4;
        hv[j] = *reinterpret_cast<const float4*>(src);
      }
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        const int i = tid + j * NT;
        if (i < S::HALO_PIX * 16) {
          const int q = i >> 4, c = i & 15;
          const int hy = q / (TW + 2), hx = q - hy * (TW + 2);
          const int yy = y0 - 1 + hy, xx = x0 - 1 + hx;
          const bool ok = yy >= 0 && yy < p.H && xx >= 0 && xx < p.W;
          *reinterpret_cast<float4*>(halo + swz256(q, c)) = ok ? hv[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    // tap 0 filter slice [64 co][64 ci]
    {
      const float* ws = Wp + ((size_t)(cc * 9 + 0) * p.Cout + cb * 64) * 64;
#pragma unroll
      for (int r = 0; r < 1024 / NT; ++r) {
        const int i = tid + r * NT, wr = i >> 4, c = i & 15;
        *reinterpret_cast<float4*>(wbuf + swz256(wr, c)) = *reinterpret_cast<const float4*>(ws + wr * 64 + c * 4);
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      // next tap's slice into registers (unconditional, clamped: keeps them in VGPRs)
      float4 nxt[1024 / NT];
      {
        const float* ws = Wp + ((size_t)(cc * 9 + min(tap + 1, 8)) * p.Cout + cb * 64) * 64;
#pragma unroll
        for (int r = 0; r < 1024 / NT; ++r) {
          const int i = tid + r * NT;
          nxt[r] = *reinterpret_cast<const float4*>(ws + (i >> 4) * 64 + (i & 15) * 4);
        }
      }
      const char* wb = wbuf + (tap & 1) * S::W_BYTES;
      const int ky = tap / 3, kx = tap - ky * 3;
      const int qrow = (row + ky) * (TW + 2) + fr + kx;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int chunk = 4 * g + fk;
        f32x4 a[NCT], b[NPT];
#pragma unroll
        for (int c = 0; c < NCT; ++c) a[c] = *reinterpret_cast<const f32x4*>(wb + swz256((ct0 + c) * 16 + fr, chunk));
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) b[pt] = *reinterpret_cast<const f32x4*>(halo + swz256(qrow + pt * 16, chunk));
        // s outermost: consecutive MFMAs update different accumulators (16x16x4 f32 has
        // a 40-cycle dependent latency against a 32-cycle issue interval)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
            for (int c = 0; c < NCT; ++c) acc[pt][c] = mfma4(a[c][s], b[pt][s], acc[pt][c]);
      }
      if (tap < 8) {
        char* wn = wbuf + ((tap + 1) & 1) * S::W_BYTES;
#pragma unroll
        for (int r = 0; r < 1024 / NT; ++r) {
          const int i = tid + r * NT;
          *reinterpret_cast<float4*>(wn + swz256(i >> 4, i & 15)) = nxt[r];
        }
      }
      __syncthreads();
    }
  }
  epilogue_f32<NPT, EPI, NCT>(p, acc, n, cb, y0 + row, x0, blockIdx.x, gridDim.x, reinterpret_cast<float*>(smem), fr,
                              fk, row, ct0, tid);
}

constexpr int kF32NW = SRMI_F32_NW;  // waves per workgroup of the fp32 conv

template <int TW, int EPI>
int launch_f32(const ConvParams& p, hipStream_t st) {
  dim3 grid((p.H / kTH) * (p.W / TW), p.Cout / 64, p.N);
  hipLaunchKernelGGL((conv3x3_f32_kernel<TW, EPI, kF32NW>), grid, dim3(kF32NW * 64), CF32Smem<TW>::TOTAL, st, p);
  SRMI_CHECK_LAUNCH();
  return 0;
}

template <int EPI>
int launch_f32_epi(const ConvParams& p, hipStream_t st) {
  if (p.W % 48 == 0) return launch_f32<48, EPI>(p, st);
  if (p.W % 32 == 0) return launch_f32<32, EPI>(p, st);
  return SRMI_ERR_SHAPE;
}

// ---------------------------------------------------------------------------
// filter (+ bias) gradient:  dW[co][ci][tap] = sum_p dY[p][co] X[p + off][ci]
// GEMM M = 64 co (one co block), N = 9 taps x 64 ci, K = the pixels of a chunk of
// rows of one image.  Stage = 2 output rows x TW columns: dY [2][TW] and X rows
// y0-1 .. y0+2 [4][TW + 4] (pitch a multiple of 4 px, zero padded) land in LDS by
// LDS-DMA (global_load_lds_dwordx4: 4 pixels = 1 KiB per wave instruction, double
// buffered).  K-step = 4 consecutive pixels of one row; wave w owns N tiles 9w ..
// 9w+8 (144 accumulators per lane); operands are single floats (ds_read_b32):
// channel c of pixel q sits at word c ^ (16 (q & 1)), so the two pixels a
// 32-lane half reads fall in opposite bank halves.  Wave 0 also sums dY for the
// bias gradient.  One partial slab [tap][ci][Cout] per chunk (wgrad_reduce, layout 0).
template <int TW>
struct WgF32 {
  static constexpr int XP = TW + 4;                 // X row pitch (px)
  static constexpr int DYPIX = 2 * TW, XPIX = 4 * XP;
  static constexpr int STAGE = (DYPIX + XPIX) * 256;
  static constexpr int NG = (DYPIX + XPIX) / 4;     // 1 KiB DMA groups per stage
  static constexpr int KSTEPS = DYPIX / 4;
};

//
// NW = 8 (two waves per SIMD): the 36 N tiles split 4 / 5 between waves WV and
// WV + 4 (the same SIMD: 16 + 20 MFMAs per K-step, as one 4-wave wave's 36); the
// DMA groups are dealt over all 8 waves.  The body is instantiated per wave (WV):
// its N tiles are compile-time.
template <int TW, int NW, int WV>
__device__ __forceinline__ void wgrad_f32_body(const WgradParams& p, char* smem) {
  using S = WgF32<TW>;
  constexpr int NT = NW == 4 ? 9 : (WV < 4 ? 4 : 5);                       // N tiles of this wave
  constexpr int J0 = NW == 4 ? 9 * WV : (WV < 4 ? 4 * WV : 16 + 5 * (WV - 4));  // its first N tile
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr int wave = WV, wave_s = WV;
  const int chunk = blockIdx.x, cb = blockIdx.y;
  const int Hr = p.H / p.row_splits;
  const int n = chunk / p.row_splits, ybase = (chunk % p.row_splits) * Hr;
  const int nrp = Hr / 2, nxb = p.W / TW, nst = nrp * nxb;
  const bool plain = p.dy_mode == IN_PLAIN;
  const float* DY = reinterpret_cast<const float*>(p.dy);
  const float* X = reinterpret_cast<const float*>(p.x);
  const float* dyn = plain ? DY + (size_t)n * p.H * p.W * p.Cout + cb * 64 : DY + (size_t)n * 4 * p.H * p.W * 64;
  const float* xn = X + (size_t)n * p.H * p.W * 64;
  const uint32_t lds0 = lds_u32(smem);
  const void* const zpage = uniform_ptr(kZerosF);
  // DMA lane roles: pixel dq = lane >> 4 of the group's 4, LDS slot ls = lane & 15,
  // source chunk ls ^ (4 (pixel & 1)) (the word swizzle above, in chunk units)
  const int dq = lane >> 4, ls = lane & 15;
  auto dma_group = [&](int st, int buf, int k) __attribute__((always_inline)) {
    const int xb = st / nrp, rp = st - xb * nrp;
    const int y0 = ybase + 2 * rp, x0 = xb * TW;
    const uint32_t dst = lds0 + (uint32_t)(buf * S::STAGE + k * 1024);
    const int q = 4 * k + dq;  // stage pixel index
    const void* src;
    if (q < S::DYPIX) {
      const int r = q / TW, px = q - r * TW;
      const int c = ls ^ (4 * (q & 1));
      const int y = y0 + r, xx = x0 + px;
      src = plain ? (const void*)(dyn + ((size_t)y * p.W + xx) * p.Cout + c * 4)
                  : (const void*)(dyn + ((size_t)(2 * y + (cb >> 1)) * (2 * p.W) + 2 * xx + (cb & 1)) * 64 + c * 4);
    } else {
      const int qx = q - S::DYPIX, r = qx / S::XP, hx = qx - r * S::XP;
      const int c = ls ^ (4 * (qx & 1));
      const int y = y0 - 1 + r, xx = x0 - 1 + hx;
      const bool ok = hx < TW + 2 && y >= 0 && y < p.H && xx >= 0 && xx < p.W;
      src = ok ? (const void*)(xn + ((size_t)y * p.W + xx) * 64 + c * 4) : zpage;
    }
    glds16(src, dst);
  };
  constexpr int NGW = (S::NG + NW - 1) / NW;  // groups per wave
  auto dma_stage = [&](int st, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < NGW; ++m) {
      const int k = wave_s + NW * m;
      if (k < S::NG) dma_group(st, buf, k);
    }
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};

  // lane-constant read offsets: A = dY[pixel k][co = 16 ct + (l & 15)],
  // B = X[pixel k + kx (row + ky)][ci = 16 it + (l & 15)] for the wave's 9 N tiles
  const int lk = lane >> 4, li = lane & 15;
  int bky[NT], bkx[NT], bci[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = J0 + t, tap = j >> 2, it = j & 3;
    bky[t] = tap / 3;
    bkx[t] = tap % 3;
    bci[t] = it * 16 + li;
  }
  auto wofs = [](int q, int c) -> uint32_t { return (uint32_t)(q * 256 + ((c ^ (16 * (q & 1))) << 2)); };

  dma_stage(0, 0);
  wait_vm<0>();
  __syncthreads();
#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) dma_stage(st + 1, (st + 1) & 1);  // lands while this stage computes
    const char* sb = smem + (st & 1) * S::STAGE;
#pragma unroll 2
    for (int ks = 0; ks < S::KSTEPS; ++ks) {
      const int r = ks / (TW / 4), px = 4 * (ks % (TW / 4)) + lk;  // this lane's K pixel
      const int qa = r * TW + px;
      float a[4], b[NT];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) a[ct] = *reinterpret_cast<const float*>(sb + wofs(qa, ct * 16 + li));
#pragma unroll
      for (int t = 0; t < NT; ++t)
        b[t] = *reinterpret_cast<const float*>(sb + S::DYPIX * 256 + wofs((r + bky[t]) * S::XP + px + bkx[t], bci[t]));
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct][t] = mfma4(a[ct], b[t], acc[ct][t]);
      if constexpr (wave == 0) {
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) bsum[ct] += a[ct];
      }
    }
    wait_vm<0>();  // the next stage has landed (this wave's part)
    __syncthreads();
  }

  // partial slab [chunk][tap][ci][Cout]: lane owns co rows 4 (l >> 4) + r of tile ct,
  // ci column l & 15 of N tile j
  float* slab = p.slab + (size_t)chunk * p.Cout * 576;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = J0 + t, tap = j >> 2, it = j & 3;
    const int ci = it * 16 + li;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int co = cb * 64 + ct * 16 + 4 * lk;
      *reinterpret_cast<float4*>(slab + ((size_t)tap * 64 + ci) * p.Cout + co) =
          make_float4(acc[ct][t][0], acc[ct][t][1], acc[ct][t][2], acc[ct][t][3]);
    }
  }
  if constexpr (wave == 0) {
    // lanes l, l+16, l+32, l+48 hold partial sums of co 16 ct + (l & 15)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      float v = bsum[ct];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) p.bslab[(size_t)chunk * p.Cout + cb * 64 + ct * 16 + lane] = v;
    }
  }
}

template <int TW, int NW>
__global__ void __launch_bounds__(NW * 64, 1) wgrad_f32_kernel(WgradParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: wgrad_f32_body<TW, NW, 0>(p, smem); break;
    case 1: wgrad_f32_body<TW, NW, 1>(p, smem); break;
    case 2: wgrad_f32_body<TW, NW, 2>(p, smem); break;
    case 3: wgrad_f32_body<TW, NW, 3>(p, smem); break;
    default:
      if constexpr (NW == 8) {
        switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
          case 4: wgrad_f32_body<TW, NW, 4>(p, smem); break;
          case 5: wgrad_f32_body<TW, NW, 5>(p, smem); break;
          case 6: wgrad_f32_body<TW, NW, 6>(p, smem); break;
          default: wgrad_f32_body<TW, NW, 7>(p, smem); break;
        }
      }
      break;
  }
}

}  // namespace

int conv3x3_f32_launch(const ConvParams& p, int epi, hipStream_t st) {
  if (p.Cin % 64 || p.Cout % 64 || p.N <= 0 || p.H % kTH) return SRMI_ERR_SHAPE;
  switch (epi) {
    case EPI_RELU_BF16: return launch_f32_epi<EPI_RELU_BF16>(p, st);
    case EPI_POOL_BF16: return launch_f32_epi<EPI_POOL_BF16>(p, st);
    case EPI_RESID: return launch_f32_epi<EPI_RESID>(p, st);
    case EPI_PS_BF16: return launch_f32_epi<EPI_PS_BF16>(p, st);
    case EPI_DG_RELUMASK: return launch_f32_epi<EPI_DG_RELUMASK>(p, st);
    case EPI_DG_ACC:
    case EPI_DG_ACC_CA: return launch_f32_epi<EPI_DG_ACC>(p, st);
    case EPI_PLAIN_BF16: return launch_f32_epi<EPI_PLAIN_BF16>(p, st);
    default: return SRMI_ERR_ARG;
  }
}

int wgrad_f32_launch(const WgradParams& p, hipStream_t st) {
  if (p.Cout % 64 || p.H % p.row_splits || (p.H / p.row_splits) % 2) return SRMI_ERR_SHAPE;
  if (p.dy_mode == IN_UNSHUF && p.Cout != 256) return SRMI_ERR_SHAPE;
  dim3 grid(p.N * p.row_splits, p.Cout / 64);
  if (p.W % 48 == 0) {
    hipLaunchKernelGGL((wgrad_f32_kernel<48, kF32NW>), grid, dim3(kF32NW * 64), 2 * WgF32<48>::STAGE, st, p);
  } else if (p.W % 32 == 0) {
    hipLaunchKernelGGL((wgrad_f32_kernel<32, kF32NW>), grid, dim3(kF32NW * 64), 2 * WgF32<32>::STAGE, st, p);
  } else {
    return SRMI_ERR_SHAPE;
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
