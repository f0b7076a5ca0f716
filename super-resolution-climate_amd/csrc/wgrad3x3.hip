// Weight (and bias) gradient of a 3x3 "same" conv as an MFMA GEMM on gfx950.
//
// Replaces the filter-gradient half of nn.Conv2d backward for default_conv
// (reference sres/model/common/cnn.py:8-9; all 64->64 and 64->256 convs of
// sres/model/rcan/network.py and blocks.py:64-65):
//     dW[co][ci][ky][kx] = sum_{n,p} dY[n][p][co] * X[n][p + (ky-1,kx-1)][ci]
//     db[co]             = sum_{n,p} dY[n][p][co]
//
// GEMM view: M = 64 output channels (one co block), N = 9 taps x 64 input
// channels, K = the pixels of one chunk (a band of rows of one image).
// Workgroup = 4 waves (one per SIMD), one (chunk, co block); wave w owns 9 of the
// 36 16-wide N tiles -> 144 f32 accumulators per lane.  Per 4-row stage the dY
// tile (4 x TW px) and the 6 input rows it needs (6 x TW+2 px, zero padded) are
// DMA'd into LDS (global_load_lds, issued ahead of the MFMAs of the previous
// stage), double buffered.  Both MFMA operands are read
// K(pixel)-major with ds_read_b64_tr_b16; the LDS row pitches are multiples of 16
// pixels so the swizzle (swz128t) is invariant across K-steps and every
// transposed read is a precomputed per-lane offset + an immediate.
// The bias gradient rides along as one extra MFMA per K-step against a ones
// fragment.  Each workgroup writes one partial slab; wgrad_reduce sums the slabs
// in a fixed order (deterministic) into the torch-layout gradient.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "conv64_body.hpp"
#include "srmi_internal.hpp"
#include "wgrad_reduce.hpp"

namespace srmi {

static __device__ uint4 kZerosW[4];  // zero page for halo lanes of the stage DMA
static unsigned long long* g_wg_stamps = nullptr;
void wgrad3x3_set_debug_stamps(unsigned long long* buf) { g_wg_stamps = buf; }
#ifdef SRMI_STAMPS
#define WSTAMP(i)                                                                                     \
  do {                                                                                                \
    if (p.stamps && tid == 0) p.stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 64 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define WSTAMP(i) \
  do {            \
  } while (0)
#endif

template <int TW>
struct Wg3 {
  static constexpr int SR = 4;                      // output rows per stage
  static constexpr int XP = (TW == 48) ? 64 : 48;   // X row pitch (px), multiple of 16, >= TW + 2
  static constexpr int DY_BYTES = SR * TW * 128;
  static constexpr int X_BYTES = (SR + 2) * XP * 128;
  static constexpr int STAGE = DY_BYTES + X_BYTES;
  static constexpr int KSTEPS = SR * TW / 32;
  static constexpr int TOTAL = 2 * STAGE;
};

template <int TW>
__global__ void __launch_bounds__(256, 1) wgrad3x3_kernel(WgradParams p) {
  using S = Wg3<TW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);  // SGPR copy for the DMA bases
  const int chunk = blockIdx.x, cb = blockIdx.y;
  const int Hr = p.H / p.row_splits;
  const int n = chunk / p.row_splits, ybase = (chunk % p.row_splits) * Hr;
  const int nrp = Hr / S::SR, nxb = p.W / TW;
  const int nst = nrp * nxb;
  WSTAMP(0);

  const bf16_t* dyn = p.dy_mode == IN_PLAIN ? p.dy + (size_t)n * p.H * p.W * p.Cout + cb * 64
                                             : p.dy + (size_t)n * 4 * p.H * p.W * 64;
  const bf16_t* xn = p.x + (size_t)n * p.H * p.W * 64;

  // Stage fill by LDS-DMA (global_load_lds_dwordx4): one wave instruction moves one
  // group of 8 pixels x 128 B into a contiguous kilobyte of LDS, so the swizzle is
  // applied on the source side -- lane (q = lane >> 3, slot = lane & 7) fetches the
  // logical chunk slot ^ f(q) of its pixel.  Halo / padding lanes read a zero page.
  // Stage st covers column block xb = st / nrp, rows y0 .. y0+3 (column-major order).
  constexpr int GD = TW / 8, GX = (TW + 2 + 7) / 8, NDY = S::SR * GD, NG = NDY + (S::SR + 2) * GX;
  const uint32_t lds0 = lds_u32(smem);
  const int dq = lane >> 3, ls = lane & 7;
  auto fsw = [](int q) { return (((q >> 1) & 1) << 1) | (((q >> 3) & 1) << 2); };
  // DMA group m (0 .. NGW-1) of this wave for stage st into buffer buf
  constexpr int NGW = (NG + 3) / 4;
  auto dma_group = [&](int st, int buf, int m) {
    const int xb = st / nrp, rp = st - xb * nrp;
    const int y0 = ybase + S::SR * rp, x0 = xb * TW;
    const uint32_t base = lds0 + buf * S::STAGE;
    const int k = wave_s + 4 * m;
    if (k < NDY) {
      const int r = k / GD, px = 8 * (k % GD) + dq;
      const int c = ls ^ fsw(r * TW + px);
      const int y = y0 + r, xx = x0 + px;
      const bf16_t* src;
      if (p.dy_mode == IN_PLAIN)
        src = dyn + ((size_t)y * p.W + xx) * p.Cout + c * 8;
      else
        src = dyn + ((size_t)(2 * y + (cb >> 1)) * (2 * p.W) + 2 * xx + (cb & 1)) * 64 + c * 8;
      glds16(src, base + (uint32_t)(r * TW + 8 * (k % GD)) * 128u);
    } else if (k < NG) {
      const int kk = k - NDY, r = kk / GX, hx = 8 * (kk % GX) + dq;
      const int c = ls ^ fsw(r * S::XP + hx);
      const int y = y0 - 1 + r, xx = x0 - 1 + hx;
      const bool ok = hx < TW + 2 && y >= 0 && y < p.H && xx >= 0 && xx < p.W;
      const void* src = ok ? (const void*)(xn + ((size_t)y * p.W + xx) * 64 + c * 8) : (const void*)kZerosW;
      glds16(src, base + (uint32_t)(S::DY_BYTES + (r * S::XP + 8 * (kk % GX)) * 128));
    }
  };
  auto dma_stage = [&](int st, int buf) {
#pragma unroll
    for (int m = 0; m < NGW; ++m) dma_group(st, buf, m);
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 bacc = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  // transposed-read lane coordinates.  K-step kb covers output rows 2*(kb / nkc)
  // .. +1 and columns 16*(kb % nkc) .. +15 of the stage; lane group g takes row
  // g>>1, columns 8*(g&1) + 4*s + q.
  const int g = lane >> 4, li = lane & 15, lq = li >> 2, lp = li & 3;
  const int prow = g >> 1, pcol = 8 * (g & 1) + lq;
  const uint32_t half = (lp & 1) * 8;
  uint32_t aoff[4][2], boff[9][2];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int h = 0; h < 2; ++h) aoff[ct][h] = swz128t(prow * TW + pcol + 4 * h, 2 * ct + (lp >> 1)) + half;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int j = 9 * wave + t, tap = j >> 2, it = j & 3, ky = tap / 3, kx = tap % 3;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      boff[t][h] = S::DY_BYTES + swz128t((prow + ky) * S::XP + pcol + kx + 4 * h, 2 * it + (lp >> 1)) + half;
  }
  constexpr int NKC = TW / 16;
  constexpr int DPS = (NGW + S::KSTEPS - 1) / S::KSTEPS;

  dma_stage(0, 0);
  wait_vm<0>();
  __syncthreads();
  WSTAMP(1);

#pragma unroll 1
  for (int st = 0; st < nst; ++st) {
    const bool pf = st + 1 < nst;
    [[maybe_unused]] const int sj = 2 + 3 * min(st, 19);
    WSTAMP(sj);
    const char* sb = smem + (st & 1) * S::STAGE;
    bf16x8 A[2][4], B[2][9];
    auto load_step = [&](int kb, bf16x8 (&a)[4], bf16x8 (&b)[9]) {
      const uint32_t da = (uint32_t)((2 * (kb / NKC) * TW + 16 * (kb % NKC)) * 128);
      const uint32_t db = (uint32_t)((2 * (kb / NKC) * S::XP + 16 * (kb % NKC)) * 128);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) a[ct] = cat_tr(lds_tr(sb, aoff[ct][0] + da), lds_tr(sb, aoff[ct][1] + da));
#pragma unroll
      for (int t = 0; t < 9; ++t) b[t] = cat_tr(lds_tr(sb, boff[t][0] + db), lds_tr(sb, boff[t][1] + db));
    };
    load_step(0, A[0], B[0]);
    WSTAMP(sj + 1);
#pragma unroll
    for (int kb = 0; kb < S::KSTEPS; ++kb) {
      // the next stage's DMA, spread over the K-steps (DPS groups per step) so the
      // wave stalls on a full memory queue between MFMA groups, not ahead of them
      if (pf) {
#pragma unroll
        for (int i = 0; i < DPS; ++i)
          if (kb * DPS + i < NGW) dma_group(st + 1, (st + 1) & 1, kb * DPS + i);
      }
      if (kb + 1 < S::KSTEPS) load_step(kb + 1, A[(kb + 1) & 1], B[(kb + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct][t] = mfma16(A[kb & 1][ct], B[kb & 1][t], acc[ct][t]);
      bf16x8 aw = A[kb & 1][0];
      if (wave == 1) aw = A[kb & 1][1];
      if (wave == 2) aw = A[kb & 1][2];
      if (wave == 3) aw = A[kb & 1][3];
      bacc = mfma16(aw, ones, bacc);
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_vm<0>();
    WSTAMP(sj + 2);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // epilogue: partial slab [chunk][9][64 ci][Cout] -- a lane's 4 accumulators are 4
  // consecutive output channels, so every store is 16 B
  float* slab = p.slab + (size_t)chunk * p.Cout * 576;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int j = 9 * wave + t, tap = j >> 2, it = j & 3;
    const int ci = it * 16 + (lane & 15);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int co = cb * 64 + ct * 16 + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(slab + ((size_t)tap * 64 + ci) * p.Cout + co) =
          make_float4(acc[ct][t][0], acc[ct][t][1], acc[ct][t][2], acc[ct][t][3]);
    }
  }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      p.bslab[(size_t)chunk * p.Cout + cb * 64 + wave * 16 + 4 * (lane >> 4) + r] = bacc[r];
  }
  WSTAMP(63);
}

// ---------------------------------------------------------------------------
// v4 for W == 48 (the 64->64 convs of every RCAB / group tail / body, and the
// first upsampler conv via IN_UNSHUF): row-pair granularity with rings.
//   * K-step = 2 output rows x 16 columns; a row pair = 3 K-steps.
//   * dY rows live in an RD-slot ring (6 KiB each), input rows in an RX-slot ring
//     (pitch 64 px, 8 KiB each): every input row is fetched once per chunk (v3
//     fetched 6 rows per 4), i.e. 26 DMA groups (26 KiB) per row pair.
//   * PF row pairs are in flight; the DMA for pair j+PF is spread over pair j's
//     K-steps and completion is tracked with a counted vmcnt (no vmcnt(0)
//     sawtooth), then one barrier per pair.
// Slot reuse: pair j+PF writes the dY slots and input rows last read by pair j-1,
// which every wave finished before the barrier that ended pair j-1.
namespace v4 {
constexpr int TW = 48, XP = 64, PF = 3, RD = 2 * (PF + 1), RX = 2 * PF + 4;
constexpr int DSLOT = TW * 128, XSLOT = XP * 128;
constexpr int DY_RING = RD * DSLOT, LDS = DY_RING + RX * XSLOT;  // 48 + 80 KiB
constexpr int GD = TW / 8, GX = 7;                               // 8-px groups per row
constexpr int NGP = 2 * GD + 2 * GX;                             // groups per pair (26)
}  // namespace v4



// The body is instantiated once per wave (WV = wave index): the wave's DMA groups,
// taps and tile rotation are compile-time constants (no SGPR pressure, no branches).
//
// NW = 8 (two waves per SIMD): the 36 N tiles are split 4 / 5 between waves WV and
// WV + 4 (the same SIMD: 17 + 20 MFMAs per K-step, as one 4-wave wave's 37); waves
// 0-3 also issue the DMA (the 4-wave schedule) and the bias gradient; every wave
// keeps all four output-channel tiles and writes its partial slab in the 4-wave
// layout, so wgrad_reduce is unchanged.
// DUG: the instantiation that may form du from g (p.gx, the fused conv2 backward only): the
// others carry none of its code (F1's launch had 20 SGPR spills with it compiled in)
template <int WV, int NW = 4, bool DUG = false>
__device__ __forceinline__ void wgrad48_body(const WgradParams& p, char* smem, int chunk, int cb) {
  using namespace v4;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int NCA = 4;  // output-channel (A) tiles of every wave
  // N tiles of this wave and its first one (8 waves: the younger half, waves 4-7, takes 5)
  constexpr int NT = NW == 4 ? 9 : (WV < 4 ? 4 : 5);
  constexpr int J0 = NW == 4 ? 9 * WV : (WV < 4 ? 4 * WV : 16 + 5 * (WV - 4));
  constexpr bool kMain = WV < 4;  // DMA + bias gradient
  constexpr bool kBias = kMain;
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr int wave = WV & 3, wave_s = WV & 3;
  // chunk = (image, row band, 48-column block): W may be any multiple of 48 (the
  // upsampler's second stage runs at 96); Wd = the row stride in pixels
  const int Hr = p.H / p.row_splits, Wd = p.W, nxb = Wd / TW;
  const int xb = chunk % nxb, cr = chunk / nxb, x0 = xb * TW;
  const int n = cr / p.row_splits, ybase = (cr % p.row_splits) * Hr;
  const int np = Hr / 2;
  const int H = p.H, Cout = p.Cout;
  const bool plain = p.dy_mode == IN_PLAIN;
  WSTAMP(0);
  const bf16_t* dyn = plain ? p.dy + ((size_t)n * H * Wd + x0) * Cout + cb * 64
                            : p.dy + ((size_t)n * 4 * H * Wd + 2 * x0) * 64;
  const bf16_t* xn = p.x + ((size_t)n * H * Wd + x0) * 64;
  const uint32_t lds0 = lds_u32(smem);
  const void* const zpage = uniform_ptr(kZerosW);
  const int dq = lane >> 3, ls = lane & 7;
  // source chunk of this lane inside its pixel: the swizzle bits of q = 8g + dq
  // are bit 1 of dq and bit 0 of g (row and slot bases are multiples of 16 px)
  const int cl0 = ls ^ (((dq >> 1) & 1) << 1);   // g even
  const int cl1 = cl0 ^ 4;                         // g odd

  // one DMA group: k < 2*GD -> dY row 2P + k / GD; else input row 2P + 1 + rr
  // (pre = true: input rows -1 and 0 of the chunk, k < 2*GX)
  auto dma = [&](int P, int k, bool pre) __attribute__((always_inline)) {
    if (!pre && k < 2 * GD) {
      const int rr = k / GD, g = k - rr * GD;
      const int r = 2 * P + rr, y = ybase + r, xx = 8 * g + dq;
      const int c = (g & 1) ? cl1 : cl0;
      const bf16_t* src = plain
                              ? dyn + ((size_t)y * Wd + xx) * Cout + c * 8
                              : dyn + ((size_t)(2 * y + (cb >> 1)) * (2 * Wd) + 2 * xx + (cb & 1)) * 64 + c * 8;
      glds16(src, lds0 + (uint32_t)((r % RD) * DSLOT + g * 1024));
    } else {
      const int kk = pre ? k : k - 2 * GD, rr = kk / GX, g = kk - rr * GX;
      const int r = pre ? rr - 1 : 2 * P + 1 + rr;  // chunk-relative input row
      const int y = ybase + r, hx = 8 * g + dq, xx = hx - 1;
      const bool ok = hx < TW + 2 && y >= 0 && y < H && x0 + xx >= 0 && x0 + xx < Wd;
      const int c = (g & 1) ? cl1 : cl0;
      const void* src = ok ? (const void*)(xn + ((ptrdiff_t)y * Wd + xx) * 64 + c * 8) : zpage;
      glds16(src, lds0 + (uint32_t)(DY_RING + ((r + 1) % RX) * XSLOT + g * 1024));
    }
  };
  // Pair DMA with precomputed per-lane offsets: group m of this wave is k = wave + 4m
  // (m < 7: waves 0,1 own 7 groups of a pair, waves 2,3 own 6).  Everything that
  // does not change from pair to pair -- the lane's pixel, chunk and x validity --
  // is computed once; per pair only a uniform base pointer and one add remain.
  int loff[7];
  uint32_t okx = 0;
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    const int k = wave_s + 4 * m;
    loff[m] = 0;
    if (k < 2 * GD) {
      const int rr = k / GD, g = k - rr * GD, xx = 8 * g + dq;
      const int c = (g & 1) ? cl1 : cl0;
      loff[m] = plain ? (rr * Wd + xx) * Cout + c * 8 : (2 * rr * (2 * Wd) + 2 * xx) * 64 + c * 8;
    } else if (k < NGP) {
      const int kk = k - 2 * GD, rr = kk / GX, g = kk - rr * GX, hx = 8 * g + dq, xx = hx - 1;
      const int c = (g & 1) ? cl1 : cl0;
      const bool ok = hx < TW + 2 && x0 + xx >= 0 && x0 + xx < Wd;
      okx |= ok ? (1u << m) : 0u;
      loff[m] = (rr * Wd + (ok ? xx : 0)) * 64 + c * 8;
    }
  }
  auto dma_pair_part = [&](int P, int m0, int m1) __attribute__((always_inline)) {
    const bf16_t* dyb = plain ? dyn + (size_t)(ybase + 2 * P) * Wd * Cout
                              : dyn + ((size_t)(2 * (ybase + 2 * P) + (cb >> 1)) * (2 * Wd) + (cb & 1)) * 64;
    const bf16_t* xb = xn + (ptrdiff_t)(ybase + 2 * P + 1) * Wd * 64;
    const bool yv0 = ybase + 2 * P + 1 < H, yv1 = ybase + 2 * P + 2 < H;
#pragma unroll
    for (int m = m0; m < m1; ++m) {
      const int k = wave_s + 4 * m;
      if (k < 2 * GD) {
        const int rr = k / GD, g = k - rr * GD;
        glds16(dyb + loff[m], lds0 + (uint32_t)(((2 * P + rr) & (RD - 1)) * DSLOT + g * 1024));
      } else if (k < NGP) {
        const int kk = k - 2 * GD, rr = kk / GX, g = kk - rr * GX;
        const bool ok = ((okx >> m) & 1u) && (rr ? yv1 : yv0);
        const void* src = ok ? (const void*)(xb + loff[m]) : zpage;
        int slot = 2 * P + 2 + rr;  // input row 2P+1+rr -> slot (row + 1) % RX
        slot = slot % RX;
        glds16(src, lds0 + (uint32_t)(DY_RING + slot * XSLOT + g * 1024));
      }
    }
  };

  f32x4 acc[NCA][NT];
#pragma unroll
  for (int i = 0; i < NCA; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the output-channel tile of A slot ct: rotated by the wave (LDS banks)
  auto ctile = [&](int ct) -> int { return (ct + wave) & 3; };
  f32x4 bacc = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  // transposed-read lane coordinates (see v3); row parts are added per pair
  const int g4 = lane >> 4, li = lane & 15, lq = li >> 2, lp = li & 3;
  const int prow = g4 >> 1, pcol = 8 * (g4 & 1) + lq;
  const uint32_t hoff = (lp & 1) * 8;
  uint32_t acol[NCA][2], bcol[NT][2];
  int bky[NT];
#pragma unroll
  for (int ct = 0; ct < NCA; ++ct)
#pragma unroll
    for (int h = 0; h < 2; ++h) acol[ct][h] = swz128t(pcol + 4 * h, 2 * ctile(ct) + (lp >> 1)) + hoff;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = J0 + t, tap = j >> 2, it = j & 3, kx = tap % 3;
    bky[t] = tap / 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) bcol[t][h] = DY_RING + swz128t(pcol + kx + 4 * h, 2 * it + (lp >> 1)) + hoff;
  }

  // slot offsets: dY row r -> slot r & (RD-1); input row r -> slot (r + 1) % RX.
  // Per pair the lane's A row is 2j + prow, its B rows 2j + prow + ky (ky of tap t).
  int boffr[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) boffr[t] = prow + bky[t];  // 0..3
  auto slots = [&](int j, uint32_t& ra, uint32_t (&rb)[NT]) __attribute__((always_inline)) {
    ra = (uint32_t)(((2 * j + prow) & (RD - 1)) * DSLOT);
    int sb = (2 * j) % RX;  // uniform
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      int sl = sb + boffr[t];
      sl = sl >= RX ? sl - RX : sl;
      rb[t] = (uint32_t)(sl * XSLOT);
    }
  };
  auto load_a = [&](uint32_t ra, int kc, bf16x8 (&a)[NCA]) __attribute__((always_inline)) {
#pragma unroll
    for (int ct = 0; ct < NCA; ++ct)
      a[ct] = cat_tr(lds_tr(smem, ra + acol[ct][0] + kc * 2048), lds_tr(smem, ra + acol[ct][1] + kc * 2048));
  };
  auto load_b = [&](const uint32_t (&rb)[NT], int kc, bf16x8 (&b)[NT]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
      b[t] = cat_tr(lds_tr(smem, rb[t] + bcol[t][0] + kc * 2048), lds_tr(smem, rb[t] + bcol[t][1] + kc * 2048));
  };
  auto load_step = [&](uint32_t ra, const uint32_t (&rb)[NT], int kc, bf16x8 (&a)[NCA], bf16x8 (&b)[NT])
      __attribute__((always_inline)) {
#pragma unroll
    for (int ct = 0; ct < NCA; ++ct)
      a[ct] = cat_tr(lds_tr(smem, ra + acol[ct][0] + kc * 2048), lds_tr(smem, ra + acol[ct][1] + kc * 2048));
#pragma unroll
    for (int t = 0; t < NT; ++t)
      b[t] = cat_tr(lds_tr(smem, rb[t] + bcol[t][0] + kc * 2048), lds_tr(smem, rb[t] + bcol[t][1] + kc * 2048));
  };
  // vmcnt helper: this wave owns 7 (waves 0,1) or 6 (waves 2,3) groups of a pair
  auto wait_groups = [&](int full_pairs, int extra) __attribute__((always_inline)) {
    const int n = full_pairs * (wave_s < 2 ? 7 : 6) + extra;
    if (n >= 14) wait_vm<14>();
    else if (n == 13) wait_vm<13>();
    else if (n == 12) wait_vm<12>();
    else if (n == 11) wait_vm<11>();
    else if (n == 10) wait_vm<10>();
    else if (n == 9) wait_vm<9>();
    else if (n == 7) wait_vm<7>();
    else if (n == 6) wait_vm<6>();
    else if (n == 5) wait_vm<5>();
    else wait_vm<0>();
  };

  // (gx_s: dy is the gradient stream g) du = bf16(g s + dm / HW) formed in place on this
  // wave's own dY groups of a pair once they landed, before the barrier that publishes
  // them (as the dgrad's input ring, conv64_body_defer); s and dm / HW of the image in an
  // LDS table past the rings.  A lane's 16 B of group g are channels 8 c .. 8 c + 7, c =
  // cl0 (g even) / cl1 (g odd)
  const bool gx = DUG && p.gx.rec != nullptr;  // (uniform)
  float* const gxt = reinterpret_cast<float*>(smem + LDS);  // [s 64][dmh 64]
  auto gx_pair = [&](int P) __attribute__((always_inline)) {
    // (a wave's three dY groups of a pair are g = k % 6 of one parity: one channel chunk c)
    static_assert(GD % 2 == 0, "g = k - rr GD keeps the parity of k = wave + 4 m");
    const int c = (wave_s & 1) ? cl1 : cl0;
    float sv[8], mv[8];
    const float4 s0 = *reinterpret_cast<const float4*>(gxt + c * 8);
    const float4 s1 = *reinterpret_cast<const float4*>(gxt + c * 8 + 4);
    const float4 m0 = *reinterpret_cast<const float4*>(gxt + 64 + c * 8);
    const float4 m1 = *reinterpret_cast<const float4*>(gxt + 64 + c * 8 + 4);
    sv[0] = s0.x; sv[1] = s0.y; sv[2] = s0.z; sv[3] = s0.w; sv[4] = s1.x; sv[5] = s1.y; sv[6] = s1.z; sv[7] = s1.w;
    mv[0] = m0.x; mv[1] = m0.y; mv[2] = m0.z; mv[3] = m0.w; mv[4] = m1.x; mv[5] = m1.y; mv[6] = m1.z; mv[7] = m1.w;
    uint4* q[3];
    uint4 v[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int k = wave_s + 4 * m, rr = k / GD, g = k - rr * GD;
      q[m] = reinterpret_cast<uint4*>(smem + ((2 * P + rr) & (RD - 1)) * DSLOT + g * 1024 + lane * 16);
      v[m] = *q[m];
    }
#pragma unroll
    for (int m = 0; m < 3; ++m) *q[m] = du_from_g8(v[m], sv, mv);
  };
  // the image's CALayer backward MLP (ca_bwd.hpp) by waves 4-7 (8 waves), which issue no
  // DMA: the compiler's wait for its operands then drains no DMA group of the prologue
  const int mt = NW == 8 ? tid - 256 : tid;  // MLP thread
  CaBwdPre cbq;
  if (gx && mt >= 0) {
    if (p.gx.mlp) {
      ca_bwd_load(p.gx, n, mt, cbq);
    } else if (mt < 128) {  // (s and dm read: an MLP launch ran)
      gxt[mt] = mt < 64 ? p.gx.rec[(size_t)n * (128 + p.gx.CR) + 64 + p.gx.CR + mt]
                        : p.gx.brec[(size_t)p.gx.N * (128 + p.gx.CR) + (size_t)n * 64 + mt - 64] * p.gx.inv_hw;
    }
  }

  // prologue: input rows -1, 0 and pairs 0 .. PF-1; wait for the rows and pair 0
  if constexpr (kMain) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (wave_s + 4 * m < 2 * GX) dma(0, wave_s + 4 * m, true);
    for (int P = 0; P < PF && P < np; ++P) dma_pair_part(P, 0, 7);
  }
  if (gx) {
    if (p.gx.mlp) {
      float* sm = reinterpret_cast<float*>(smem + LDS + 512);
      ca_bwd_mlp(p.gx, n, mt, cbq, sm, false);
      if (mt >= 0 && mt < 128) gxt[mt] = mt < 64 ? sm[kCaBwdS + mt] : sm[kCaBwdDm + mt - 64] * p.gx.inv_hw;
    }
    __syncthreads();  // (the table)
  }
  wait_groups(min(PF, np) - 1, 0);
  if constexpr (kMain) {
    if (gx) gx_pair(0);
  }
  __syncthreads();
  WSTAMP(1);

  // fragments double-buffered across K-steps; a pair has 3 K-steps, so the pair loop
  // is unrolled by two (np is even) to keep the buffer parity compile-time.  8 waves
  // (256 registers a wave): B single-buffered, each tile reloaded right behind its
  // MFMAs (the partner wave on the SIMD covers the read latency).
  constexpr int NB = NW == 8 ? 1 : 2;
  bf16x8 A[2][NCA], B[NB][NT];
  uint32_t ra, rb[NT];
  slots(0, ra, rb);
  load_step(ra, rb, 0, A[0], B[0]);

#pragma unroll 1
  for (int j0 = 0; j0 < np; j0 += 2) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j = j0 + q;
      WSTAMP(2 + min(j, 59));
      const bool pf = j + PF < np;
      const bool more = j + 1 < np;
      uint32_t ran, rbn[NT];
      slots(j + 1, ran, rbn);
#pragma unroll
      for (int kc = 0; kc < 3; ++kc) {
        const int cur = (3 * q + kc) & 1, nxt = cur ^ 1;
        if (kMain && pf)
          dma_pair_part(j + PF, kc == 0 ? 0 : (kc == 1 ? 3 : 5), kc == 0 ? 3 : (kc == 1 ? 5 : 7));
        __builtin_amdgcn_sched_barrier(0);
        const bool ld = kc < 2 || more;
        if constexpr (NB == 2) {
          if (kc < 2) load_step(ra, rb, kc + 1, A[nxt], B[nxt]);
          else if (more) load_step(ran, rbn, 0, A[nxt], B[nxt]);  // next pair's first K-step
        } else {
          if (kc < 2) load_a(ra, kc + 1, A[nxt]);
          else if (more) load_a(ran, 0, A[nxt]);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int ct = 0; ct < NCA; ++ct) acc[ct][t] = mfma16(A[cur][ct], B[cur % NB][t], acc[ct][t]);
        if constexpr (kBias) bacc = mfma16(A[cur][0], ones, bacc);  // slot 0 = this wave's own co tile
        if constexpr (NB == 1) {
          if (kc < 2) load_b(rb, kc + 1, B[0]);
          else if (more) load_b(rbn, 0, B[0]);
        }
        // the next K-step's transposed reads issued behind the MFMAs, one per MFMA
        constexpr int NRD = 2 * (NCA + NT), NMF = NCA * NT + (kBias ? 1 : 0);
        constexpr int NPAIR = NRD < NMF ? NRD : NMF;
        if (ld) {
#pragma unroll
          for (int i = 0; i < NPAIR; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          }
          if constexpr (NMF > NPAIR) __builtin_amdgcn_sched_group_barrier(0x008, NMF - NPAIR, 0);
          if constexpr (NRD > NPAIR) __builtin_amdgcn_sched_group_barrier(0x100, NRD - NPAIR, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kMain) {
          // (gx) du of pair j+1 behind K-step 0's MFMAs: in flight may stay pair j+2 and the
          // 3 groups of pair j+PF issued above; the barrier of K-step 1 publishes it
          if (SRMI_GX_INLOOP != 0 && kc == 0 && gx && more) {
            if (j + 2 < np) wait_groups(1, pf ? 3 : 0);
            else wait_groups(0, 0);
            gx_pair(j + 1);
          }
        }
        if (kc == 1) {
          // pair j+1 must have landed before K-step 2 reads its first fragments.  In
          // flight may stay: pair j+2 (whole) and the 5 groups of pair j+PF issued above.
          if (j + 2 < np) wait_groups(1, pf ? 5 : 0);
          else wait_groups(0, 0);
          if constexpr (kMain && !SRMI_GX_INLOOP) {
            if (gx && more) gx_pair(j + 1);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
      }
      ra = ran;
#pragma unroll
      for (int t = 0; t < NT; ++t) rb[t] = rbn[t];
    }
  }

  // partial slab in the MFMA-native order (slab layout 1): every store instruction
  // writes 1 KiB contiguous; wgrad_reduce_kernel maps it back to (co, ci, tap).
  // Write-through: in the step (two engines, the reduction one or two launches
  // later) +1.1 % over plain stores, whose 9.4 MB of dirty lines per fused launch
  // left in the flush at its end (a standalone wgrad + reduce pair measured the
  // other way round in round 2: the launch 0.9 us shorter, the reduce 1.9 us longer)
  // (N tile J, slot ct of rotation `wave`) -> the 4-wave position (wave J / 9, tile
  // J % 9, the slot of the same output-channel tile under that wave's rotation)
  const size_t soff = (size_t)chunk * Cout * 576 + (size_t)cb * (64 * 576);
  // (write-through: the slab leaves the XCD's L2 while the other waves still
  //  compute, instead of in the dirty-line flush at the end of the launch)
  // (slab16: the same order in bf16, 512 contiguous bytes per store instruction)
  const uint32_t esz = p.slab16 ? 2u : 4u;
  [[maybe_unused]] const auto rsl = wt_rsrc(p.slab, (uint32_t)((size_t)(chunk + 1) * Cout * 576 * esz));
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ct = 0; ct < NCA; ++ct) {
      const int J = J0 + t, w4 = J / 9, t4 = J % 9, s4 = (ctile(ct) - w4) & 3;
      const size_t o = soff + (size_t)w4 * (9 * 4 * 256) + ((t4 * 4 + s4) * 64 + lane) * 4;
      if (p.slab16)  // (uniform)
        st_wt8(rsl, p.slab, (uint32_t)(o * 2),
               make_uint2(pack2(acc[ct][t][0], acc[ct][t][1]), pack2(acc[ct][t][2], acc[ct][t][3])));
      else
        st_wt16(rsl, p.slab, (uint32_t)(o * 4),
                make_float4(acc[ct][t][0], acc[ct][t][1], acc[ct][t][2], acc[ct][t][3]));
    }
  if (kBias && (lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      p.bslab[(size_t)chunk * Cout + cb * 64 + ctile(0) * 16 + 4 * (lane >> 4) + r] = bacc[r];
  }
  WSTAMP(63);
}

template <int NW = 4, bool DUG = false>
__device__ __forceinline__ void wgrad48_dispatch(const WgradParams& p, char* smem, int chunk, int cb) {
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: wgrad48_body<0, NW, DUG>(p, smem, chunk, cb); break;
    case 1: wgrad48_body<1, NW, DUG>(p, smem, chunk, cb); break;
    case 2: wgrad48_body<2, NW, DUG>(p, smem, chunk, cb); break;
    case 3: wgrad48_body<3, NW, DUG>(p, smem, chunk, cb); break;
    default:
      if constexpr (NW == 8) {
        switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
          case 4: wgrad48_body<4, NW, DUG>(p, smem, chunk, cb); break;
          case 5: wgrad48_body<5, NW, DUG>(p, smem, chunk, cb); break;
          case 6: wgrad48_body<6, NW, DUG>(p, smem, chunk, cb); break;
          default: wgrad48_body<7, NW, DUG>(p, smem, chunk, cb); break;
        }
      }
      break;
  }
}

constexpr int kWgradNW = 8;  // waves per workgroup of the standalone filter gradient (two per SIMD)
__global__ void __launch_bounds__(kWgradNW * 64, 1) wgrad48_kernel(WgradParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  wgrad48_dispatch<kWgradNW>(p, smem, blockIdx.x, blockIdx.y);
}

// ---------------------------------------------------------------------------
// Horizontally fused RCAB backward launch: a data-gradient conv (conv64 body:
// dgrad of conv2 with the ReLU mask, or dgrad of conv1 accumulating into the
// gradient stream) and the filter gradient of the SAME conv (wgrad48 body) read
// the same upstream gradient and are independent, so one launch runs both: the
// conv's runs and the wgrad's row chunks are dealt over the grid evenly
// (Bresenham interleave), each sized for its share of the CU budget, one
// workgroup per CU.  This replaces the two-stream overlap of round 1 (a side
// stream per engine with cross-stream event waits) by co-scheduling inside one
// launch on one stream: no events, one launch instead of two.
//
// Block -> role map.  `paired` (the conv's runs and the wgrad's row chunks cover
// the same image rows one to one: conv run k <-> chunk k): blocks are dealt in
// groups of 16, eight conv runs then the eight chunks of the same rows, so run k
// and chunk k sit 8 blocks apart -- the same XCD under round-robin dispatch -- and
// the second reader of dY and of the shared operand finds its rows in that XCD's
// L2 instead of fetching them again.  Otherwise a Bresenham interleave.
//
// tail > 0 (paired map only): the filter-gradient half finishes earlier than the
// dgrad half (F1: 24.7 vs 36.9 us at C2), so the last `tail` strips of dgrad run k
// move to the workgroup of chunk k, which runs them before its chunk (same rows, same
// XCD), with its own filter prologue (SRMI_FUSE_TAIL_FIRST; after it: 0).
template <int EPI, int NW>
__global__ void __launch_bounds__(NW * 64, 1) rcab_bwd_kernel(ConvParams cp, int run_len, int nconv, WgradParams wp,
                                                              int nwg, int paired, int tail) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, tot = nconv + nwg;
  int conv = -1, w;
  if (paired) {
    const int base = (b >> 4) << 3, i = b & 15, m = min(8, nconv - base);
    if (i < m) conv = base + i;
    else w = base + i - m;
  } else {
    const int c0 = (int)(((long long)b * nconv) / tot), c1 = (int)(((long long)(b + 1) * nconv) / tot);
    if (c1 > c0) conv = c0;
    else w = b - c0;
  }
  if (conv >= 0) {
    conv64_body<48, EPI, NW>(cp, run_len, conv, smem, tail, false);
    return;
  }
  const int nch = wp.N * wp.row_splits;
#if SRMI_FUSE_TAIL_FIRST
  if (tail > 0) {
    conv64_body<48, EPI, NW>(cp, run_len, w, smem, tail, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is past its last LDS access of the strips
  }
  wgrad48_dispatch<NW, EPI == EPI_DG_RELUMASK>(wp, smem, w % nch, w / nch);
#else
  wgrad48_dispatch<NW, EPI == EPI_DG_RELUMASK>(wp, smem, w % nch, w / nch);
  if (tail > 0) {
    __syncthreads();  // every wave is past its last LDS read of the chunk
    conv64_body<48, EPI, NW>(cp, run_len, w, smem, tail, true);
  }
#endif
}

bool rcab_bwd_du_from_g() { return conv64_defers<EPI_DG_RELUMASK>(); }

int rcab_bwd_fusable(const ConvParams& cp, const WgradParams& wp) {
  return !cp.f32 && !wp.f32 && cp.Cin == 64 && cp.Cout == 64 && cp.in_mode == IN_PLAIN && cp.W == 48 &&
         cp.H % 4 == 0 && wp.W == 48 && wp.Cout == 64 && wp.dy_mode == IN_PLAIN && wp.row_splits > 0 &&
         wp.H % wp.row_splits == 0 && (wp.H / wp.row_splits) % 4 == 0;
}

// waves per workgroup of the fused launch (8: two per SIMD in both roles)
constexpr int kFuseNW = 8;

// the partial slabs are stored through a buffer resource with a 32-bit byte range
static bool slab_range_ok(const WgradParams& p, int nslabs) {
  return (size_t)nslabs * p.Cout * 576 * 4 < ((size_t)1 << 32);
}

int rcab_bwd_launch(const ConvParams& cp, int epi, int conv_cus, const WgradParams& wp, hipStream_t st) {
  if (!rcab_bwd_fusable(cp, wp)) return SRMI_ERR_SHAPE;
  // du formed from the gradient stream g (gx_*): both roles together, in the deferred
  // ReLU-mask dgrad (conv64_body_defer) beside a 64-channel filter gradient
  if ((cp.gx.rec != nullptr) != (wp.gx.rec != nullptr) ||
      (cp.gx.rec && std::memcmp(&cp.gx, &wp.gx, sizeof(CaBwdIn)) != 0))
    return SRMI_ERR_ARG;
  if (cp.gx.rec && (epi != EPI_DG_RELUMASK || !conv64_defers<EPI_DG_RELUMASK>() || cp.x != wp.dy ||
                    !cp.gx.part || !cp.gx.w1 || !cp.gx.w2 || !cp.gx.brec || cp.gx.CR < 4 || cp.gx.CR > 32 ||
                    cp.gx.CR % 4 || cp.Cin != 64))
    return SRMI_ERR_ARG;
  if (!slab_range_ok(wp, wp.N * wp.row_splits)) return SRMI_ERR_SHAPE;
  const int run_len = conv64_run_len(cp, 48, conv_cus);
  const int nconv = conv64_blocks(cp, 48, run_len);
  const int nwg = wp.N * wp.row_splits * (wp.Cout / 64);
  // (+ the CA backward MLP's scratch of the dgrad runs past their body's LDS, ca_bwd.hpp;
  //  the filter gradient's du table and MLP scratch sit past its rings)
  const int lds = (Conv2Smem<48>::TOTAL > v4::LDS ? Conv2Smem<48>::TOTAL : v4::LDS) + (cp.gx.rec ? kCaBwdScratch * 4 : 0);
  static_assert(Conv2Smem<48>::TOTAL >= v4::LDS + 512 + kCaBwdScratch * 4, "the filter gradient's du table and MLP scratch");
  ConvParams c = cp;
  c.stamps = conv3x3_stamps_for(epi);  // (null in production; the dgrad runs' phase stamps in diagnostic builds)
  WgradParams w = wp;
  const dim3 grid(nconv + nwg);
  // (diagnostic: the filter-gradient body's stamps in a second [grid][64] region)
  w.stamps = c.stamps ? c.stamps + (size_t)grid.x * 64 : nullptr;
  // conv run k and wgrad chunk k cover the same rows of the same image
  const int runs_per_col = (cp.H / kTH + run_len - 1) / run_len;
  const int paired =
      nconv == nwg && cp.N == wp.N && runs_per_col == wp.row_splits && run_len * kTH == wp.H / wp.row_splits;
  // dgrad strips per run handed to the paired filter-gradient workgroup (see the kernel)
  // (one strip in F1; none in F2, whose ReLU-mask strip is cheaper than the extra
  //  filter prologue, nor in F1 with its epilogue deferred: SRMI_F1_DEFER_TAIL)
  const bool f1_defer = epi == EPI_DG_ACC_CA16 && conv64_defers<EPI_DG_ACC_CA16>();
  const int tail = !paired ? 0 : std::min(run_len - 1, epi == EPI_DG_RELUMASK ? 0 : (f1_defer ? SRMI_F1_DEFER_TAIL : 1));
  switch (epi) {
    case EPI_DG_RELUMASK:
      if (!c.aux) return SRMI_ERR_ARG;
      hipLaunchKernelGGL((rcab_bwd_kernel<EPI_DG_RELUMASK, kFuseNW>), grid, dim3(kFuseNW * 64), lds, st, c, run_len,
                         nconv, w, nwg, paired, tail);
      break;
    case EPI_DG_ACC_CA:
      if (!c.r1 || !c.aux || !c.part || c.yb || c.r2 || c.r3 || !c.yf || c.r1b) return SRMI_ERR_ARG;
      hipLaunchKernelGGL((rcab_bwd_kernel<EPI_DG_ACC_CA, kFuseNW>), grid, dim3(kFuseNW * 64), lds, st, c, run_len,
                         nconv, w, nwg, paired, tail);
      break;
    case EPI_DG_ACC_CA16:
      if (!c.r1b || !c.aux || !c.part || !c.yb || c.r1 || c.r2 || c.r3 || c.yf) return SRMI_ERR_ARG;
      hipLaunchKernelGGL((rcab_bwd_kernel<EPI_DG_ACC_CA16, kFuseNW>), grid, dim3(kFuseNW * 64), lds, st, c, run_len,
                         nconv, w, nwg, paired, tail);
      break;
    case EPI_DG_ACC_G1:
      if (!c.r1b || !c.r2 || !c.yf || !c.yb || c.r1 || c.aux || c.part) return SRMI_ERR_ARG;
      hipLaunchKernelGGL((rcab_bwd_kernel<EPI_DG_ACC_G1, kFuseNW>), grid, dim3(kFuseNW * 64), lds, st, c, run_len,
                         nconv, w, nwg, paired, tail);
      break;
    case EPI_DG_CA16:
      if (!c.aux || !c.part || !c.yb || c.r1 || c.r1b || c.r2 || c.r3 || c.yf) return SRMI_ERR_ARG;
      hipLaunchKernelGGL((rcab_bwd_kernel<EPI_DG_CA16, kFuseNW>), grid, dim3(kFuseNW * 64), lds, st, c, run_len,
                         nconv, w, nwg, paired, tail);
      break;
    case EPI_DG_ACC:
      if ((!c.yf && !c.yb) || (c.part && !c.aux) || (c.r1 && c.r1b)) return SRMI_ERR_ARG;
      hipLaunchKernelGGL((rcab_bwd_kernel<EPI_DG_ACC, kFuseNW>), grid, dim3(kFuseNW * 64), lds, st, c, run_len, nconv, w, nwg, paired, tail);
      break;
    default:
      return SRMI_ERR_ARG;
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}


static bool use_wgrad48(const WgradParams& p) {
  // v4 (row-pair rings, per-wave specialised) for W a multiple of 48: one chunk per
  // (image, row band, 48-column block)
  return !p.f32 && p.W % 48 == 0 && p.row_splits > 0 && (p.H / p.row_splits) % 2 == 0;
}

int wgrad3x3_nslabs(const WgradParams& p) { return p.N * p.row_splits * (use_wgrad48(p) ? p.W / 48 : 1); }

int wgrad3x3_slab_layout(const WgradParams& p) { return use_wgrad48(p) ? 1 : 0; }

int wgrad3x3_launch(const WgradParams& p, hipStream_t st) {
  if (p.gx.rec) return SRMI_ERR_ARG;  // (du formed from g: the fused backward launch only)
  if (p.f32) return wgrad_f32_launch(p, st);
  if (p.Cout % 64 || p.H % p.row_splits || (p.H / p.row_splits) % 4) return SRMI_ERR_SHAPE;
  if (p.dy_mode == IN_UNSHUF && p.Cout != 256) return SRMI_ERR_SHAPE;
  if (!slab_range_ok(p, wgrad3x3_nslabs(p))) return SRMI_ERR_SHAPE;
  dim3 grid(wgrad3x3_nslabs(p), p.Cout / 64);
  WgradParams q = p;
  q.stamps = g_wg_stamps;
  if (use_wgrad48(p)) {
    hipLaunchKernelGGL(wgrad48_kernel, grid, dim3(kWgradNW * 64), v4::LDS, st, q);
  } else if (p.W % 48 == 0) {
    hipLaunchKernelGGL(wgrad3x3_kernel<48>, grid, dim3(256), Wg3<48>::TOTAL, st, q);
  } else if (p.W % 32 == 0) {
    hipLaunchKernelGGL(wgrad3x3_kernel<32>, grid, dim3(256), Wg3<32>::TOTAL, st, q);
  } else {
    return SRMI_ERR_SHAPE;
  }
  SRMI_CHECK_LAUNCH();
  return 0;
}

__global__ void __launch_bounds__(kRedQ * kRedPh) wgrad_reduce_kernel(ReduceSet r) {
  wgrad_reduce_body<kRedPh>(r, blockIdx.x);
}

// two independent reductions in one launch (blockIdx.y selects the set): the two
// filter gradients of an RCAB on the side stream share one launch and one boundary
__global__ void __launch_bounds__(kRedQ * kRedPh) wgrad_reduce2_kernel(ReduceSet r0, ReduceSet r1) {
  const ReduceSet& r = blockIdx.y ? r1 : r0;
  wgrad_reduce_body<kRedPh>(r, blockIdx.x);
}

int wgrad_reduce_launch(const float* slab, const float* bslab, int nslab, int Cout, int ps, int layout, float alpha,
                        float* gw, float* gb, hipStream_t st, int slab16) {
  if (Cout % 64 || (slab16 && layout != 1)) return SRMI_ERR_SHAPE;
  const int blocks = wgrad_reduce_blocks(Cout);
  const ReduceSet r{slab, bslab, nslab, Cout, ps, layout, alpha, gw, gb, slab16};
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(kRedQ * kRedPh), 0, st, r);
  SRMI_CHECK_LAUNCH();
  return 0;
}

// up to kRedSets reductions of one launch, passed by value (kernel arguments, no upload)
constexpr int kRedSets = 42;
struct ReduceSets {
  ReduceSet s[kRedSets];
};
// (64 quads x 8 phases: a thread sums 8 of a launch's 64 slabs with 4 loads in flight, a
//  block 256 outputs -- a quarter of the blocks of the 16 x 32 form, each latency-bound)
constexpr int kSetQ = 64, kSetPh = 8;
__global__ void __launch_bounds__(kSetQ * kSetPh) wgrad_reduce_sets_kernel(ReduceSets r) {
  wgrad_reduce_body<kSetPh, kSetQ>(r.s[blockIdx.y], blockIdx.x);
}

int wgrad_reduce_sets_launch(const ReduceSet* sets, int n, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += kRedSets) {
    const int m = std::min(kRedSets, n - i0);
    ReduceSets r{};
    for (int i = 0; i < m; ++i) {
      if (sets[i0 + i].Cout != sets[i0].Cout || sets[i0].Cout % 64) return SRMI_ERR_SHAPE;
      r.s[i] = sets[i0 + i];
    }
    hipLaunchKernelGGL(wgrad_reduce_sets_kernel, dim3(wgrad_reduce_blocks(sets[i0].Cout, kSetQ), m),
                       dim3(kSetQ * kSetPh), 0, st, r);
    SRMI_CHECK_LAUNCH();
  }
  return 0;
}

int wgrad_reduce2_launch(const ReduceSet& r0, const ReduceSet& r1, hipStream_t st) {
  if (r0.Cout % 64 || r1.Cout != r0.Cout) return SRMI_ERR_SHAPE;
  const int blocks = wgrad_reduce_blocks(r0.Cout);
  hipLaunchKernelGGL(wgrad_reduce2_kernel, dim3(blocks, 2), dim3(kRedQ * kRedPh), 0, st, r0, r1);
  SRMI_CHECK_LAUNCH();
  return 0;
}

}  // namespace srmi
