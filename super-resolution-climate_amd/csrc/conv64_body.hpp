// The persistent-run 3x3 conv body (Cin == 64, IN_PLAIN) of conv3x3.hip, shared
// with the horizontally fused backward launch of wgrad3x3.hip.  Included by those
// two translation units only (its zero page and stamp buffer are per-TU statics).
#pragma once
#include <type_traits>

#include "ca_bwd.hpp"
#include "ca_scale.hpp"

#include "common.hpp"
#include "srmi_internal.hpp"

namespace srmi {

static __device__ uint4 kZeros[64];  // 1 KiB zero page (padding source, absent bias)

#ifdef SRMI_STAMPS
#define STAMP(i)                                                                                   \
  do {                                                                                             \
    if (p.stamps && tid == 0) {                                                                    \
      p.stamps[blockIdx.x * 64 + (i)] = __builtin_amdgcn_s_memtime();                              \
      if ((i) == 0 || (i) == 61) p.stamps[blockIdx.x * 64 + 62 + ((i) == 61)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                              \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

constexpr int kTH = 4;
constexpr int kThreads = 256;

// ============================================================================
// v2 (Cin == 64): persistent runs.  A workgroup owns a vertical run of strips of
// one image column and one 64-wide output-channel block.  All 9 filter slices
// ([9][64 co][64 ci] bf16, 72 KiB) stay resident in LDS for the whole run; the
// input rows live in a ring of 3 groups of 4 rows (group g = rows 4g-3..4g), so
// strip k reads groups k and k+1 while group k+2 is prefetched into registers
// (issued before the MFMAs, written to LDS after them: hipcc counts these loads
// itself).  Halo rows are therefore fetched once per run (1.17x input traffic at
// 12-row runs instead of 1.5x), with one barrier per strip instead of one per tap.
template <int TW>
struct Conv2Smem {
  static constexpr int ROWB = (TW + 2) * 128;      // one halo row (TW+2 px x 64 ch bf16)
  static constexpr int GROUPB = 4 * ROWB;
  static constexpr int WB = 9 * 64 * 128;          // resident filters
  static constexpr int RING = 3 * GROUPB;
  static constexpr int RED = 2 * 4 * 128 * 4;      // cross-wave channel sums (two buffers: deferred form)
  static constexpr int TOTAL = WB + RING + RED;
  static constexpr int GCH = GROUPB / 16;          // 16-B chunks per group
  static constexpr int GPT = (GCH + kThreads - 1) / kThreads;
};

// Epilogue operands that live in global memory are prefetched into registers
// before the MFMA phase.  NCT = output-channel tiles (16 wide) per wave: 4 when a
// wave owns the whole 64-channel block of its row, 2 in the 8-wave form (a wave
// per row and channel half), whose tiles start at ct0.
template <int NPT, int EPI, int NCT = 4>
struct EpiPre {
  float4 r1[NPT][NCT];     // (DG_ACC_CA, DG_ACC: the gradient streams' 16-byte chunks of the
  uint2 aux[NPT][NCT];     //  wave's 1 KiB store runs, and u's 8 bytes beside them -- see
  float4 r2[NPT][NCT];     //  conv_epilogue2)
  uint2 gb[NPT][NCT];      // (DG_ACC_CA16: the bf16 gradient stream's 8 bytes of the run)
};

// the gradient-stream epilogues (DG_ACC_CA, DG_ACC) add their fp32 operands to the
// staged dgrad in the 1 KiB run layout of the stores instead of the MFMA layout
// h' = h + s u into the residual pair: the inference RCAB's conv2 (u never stored) and
// the training one's (u stored for backward, and rounded to bf16 before the product)
template <int EPI>
constexpr bool epi_cr() {
  return EPI == EPI_CA_RESID || EPI == EPI_CA_RESID_U;
}
// conv2's h' = h + s u with u rounded to bf16 first (staged once as bf16): the training
// conv2 always (it stores that u for backward), the inference one per SRMI_INFER_BF16U
template <int EPI>
constexpr bool epi_cr_bf16() {
  return EPI == EPI_CA_RESID_U || (EPI == EPI_CA_RESID && SRMI_INFER_BF16U);
}
// the bf16 in-group gradient stream's epilogues (with / without the stream's input r1b)
template <int EPI>
constexpr bool epi_g16() {
  return EPI == EPI_DG_ACC_CA16 || EPI == EPI_DG_CA16;
}
template <int EPI>
constexpr bool epi_run() {
  return EPI == EPI_DG_ACC_CA || epi_g16<EPI>() || EPI == EPI_DG_ACC || EPI == EPI_DG_ACC_G1 || epi_cr<EPI>();
}
__device__ __forceinline__ float4 unpack_bf16x4(uint32_t a, uint32_t b) {
  return make_float4(bf2f(a & 0xFFFFu), bf2f(a >> 16), bf2f(b & 0xFFFFu), bf2f(b >> 16));
}

// one (pt, c) element (idx = pt * NCT + c), issued one or two per K-step
template <int NPT, int EPI, int NCT>
__device__ __forceinline__ void epi_prefetch_one(const ConvParams& p, EpiPre<NPT, EPI, NCT>& e, int n, int cb, int y,
                                                 int x0, int fr, int fk, int ct0, int idx) {
  if constexpr (EPI == EPI_RESID || EPI == EPI_DG_ACC || EPI == EPI_DG_RELUMASK || EPI == EPI_DG_ACC_CA ||
                epi_g16<EPI>() || EPI == EPI_DG_ACC_G1 || epi_cr<EPI>()) {
    const int pt = idx / NCT, c = idx % NCT;
    const size_t HW = (size_t)p.H * p.W;
    const size_t pix = (size_t)n * HW + (size_t)y * p.W + x0 + pt * 16 + fr;
    const size_t o = pix * p.Cout + cb * 64 + (ct0 + c) * 16 + fk * 4;
    if constexpr (EPI == EPI_RESID) e.r1[pt][c] = *reinterpret_cast<const float4*>(p.r1 + o);
    if constexpr (EPI == EPI_DG_ACC && !epi_run<EPI>()) {
      e.r1[pt][c] = p.r1 ? *reinterpret_cast<const float4*>(p.r1 + o) : make_float4(0.f, 0.f, 0.f, 0.f);
      e.aux[pt][c] = p.part ? *reinterpret_cast<const uint2*>(p.aux + o) : make_uint2(0, 0);
    }
    if constexpr (EPI == EPI_DG_RELUMASK) e.aux[pt][c] = *reinterpret_cast<const uint2*>(p.aux + o);
    if constexpr (epi_run<EPI>()) {
      // load q of the wave = 16-byte chunk `lane` of its q-th 1 KiB output run (the
      // layout of the fp32 store loop of conv_epilogue2): full 128-byte lines, half
      // the requests of the MFMA layout's 64-byte pieces (and a quarter for u)
      constexpr bool kSh = NCT < 4;
      constexpr int HALF = NPT * 8, JW = kSh ? NPT : 2 * NPT;  // runs per half-row per wave
      const int h = idx / JW, j = idx % JW, lane = fk * 16 + fr;
      const int i = kSh ? 2 * j + (ct0 >> 1) : j;
      const int lin = i * 1024 + lane * 16, lpx = lin >> 8, ch = (lin >> 4) & 15;
      const size_t oc = ((size_t)n * HW + (size_t)y * p.W + x0 + h * HALF + lpx) * p.Cout + cb * 64 + ch * 4;
      if constexpr (epi_cr<EPI>()) {  // h: the pair's raw bits (decoded in the store loop) or fp32
        if (p.r1h) {
          const uint2 hh = *reinterpret_cast<const uint2*>(p.r1h + oc);
          const uint32_t ll = *reinterpret_cast<const uint32_t*>(p.r1l + oc);
          e.r1[pt][c] = make_float4(__uint_as_float(hh.x), __uint_as_float(hh.y), __uint_as_float(ll), 0.f);
        } else {
          e.r1[pt][c] = *reinterpret_cast<const float4*>(p.r1 + oc);
        }
      } else if constexpr (EPI == EPI_DG_ACC_CA) {
        e.r1[pt][c] = *reinterpret_cast<const float4*>(p.r1 + oc);  // (load q = idx at [q / NCT][q % NCT])
        e.aux[pt][c] = *reinterpret_cast<const uint2*>(p.aux + oc);
      } else if constexpr (EPI == EPI_DG_ACC_G1) {
        e.gb[pt][c] = *reinterpret_cast<const uint2*>(p.r1b + oc);
        e.r2[pt][c] = *reinterpret_cast<const float4*>(p.r2 + oc);
      } else if constexpr (epi_g16<EPI>()) {
        if constexpr (EPI == EPI_DG_ACC_CA16)
          e.gb[pt][c] = *reinterpret_cast<const uint2*>(p.r1b + oc);  // 512 contiguous bytes per wave
        e.aux[pt][c] = *reinterpret_cast<const uint2*>(p.aux + oc);
      } else {  // DG_ACC: every operand optional (uniform branches)
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.r1b) {  // the bf16 stream's raw bits in .x / .y, decoded in the store loop
          const uint2 gq = *reinterpret_cast<const uint2*>(p.r1b + oc);
          e.r1[pt][c] = make_float4(__uint_as_float(gq.x), __uint_as_float(gq.y), 0.f, 0.f);
        } else {
          e.r1[pt][c] = p.r1 ? *reinterpret_cast<const float4*>(p.r1 + oc) : z;
        }
        e.r2[pt][c] = p.r2 ? *reinterpret_cast<const float4*>(p.r2 + oc) : z;
        e.aux[pt][c] = p.part ? *reinterpret_cast<const uint2*>(p.aux + oc) : make_uint2(0, 0);
      }
      (void)o;
    }
  }
}

__device__ __forceinline__ float relu_mask(uint32_t bits16, float v) {
  return (bits16 & 0x7FFFu) && !(bits16 & 0x8000u) ? v : 0.f;
}

// Orders one wave's LDS accesses across lanes: the hardware executes a wave's DS
// instructions in order, but the compiler reasons per lane and would move a
// lane's read of another lane's staged data above that lane's write.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// conv1's share of its image's CA mean (EPI_RELU_POOL with cas_on, training,
// SRMI_CA_MPART): what the run's epilogues gather for ca_matvec at the run's end
struct CaPart {
  float colA[4][4], colB[4][4];  // [c][r]: the lane's sums of column 0 / column W-1 of t
  float tacc;                    // tid < 64: T over the run's strips, channel tid
  float* scr;                    // the LDS scratch (ca_scale.hpp layout: bs, cn zeroed)
};

// Fused epilogue of the v2 kernel (same semantics as conv_epilogue).  A wave holds
// row `row` of the strip, channel tiles ct0 .. ct0+NCT-1.  NCT < 4: two waves (the
// channel halves) share the row's LDS staging, so their writes and the full-line
// stores that read them are separated by workgroup barriers and each wave stores
// every other 1 KiB run.
template <int NPT, int EPI, int NCT = 4>
__device__ __forceinline__ void conv_epilogue2(const ConvParams& p, f32x4 (&acc)[NPT][NCT],
                                               const EpiPre<NPT, EPI, NCT>& e, const float4 (&bias)[NCT], int n,
                                               int cb, int y, int x0, int strip, int nstrips, float* red, int fr,
                                               int fk, int row, int ct0, int tid, char* stage,
                                               const float4& fs = float4{0.f, 0.f, 0.f, 0.f},
                                               CaPart* cp = nullptr, bool cpon = false) {
  constexpr bool kShared = NCT < 4;
  const int half_id = ct0 >> 1;  // shared form: which of the two waves of the row
  auto stage_sync = [&]() __attribute__((always_inline)) {
    if constexpr (kShared) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      lds_order();
    }
  };
  const size_t HW = (size_t)p.H * p.W;
  [[maybe_unused]] const auto rfa = wt_rsrc(p.yf, (uint32_t)((size_t)p.N * HW * p.Cout * 4));
  constexpr bool kPart1 = (EPI == EPI_POOL_BF16 || EPI == EPI_RELU_POOL);
  constexpr bool kPart2 = (EPI == EPI_DG_ACC || EPI == EPI_DG_ACC_CA || epi_g16<EPI>());
  float ps0[NCT][4], ps1[NCT][4];
  // fp32 output staged through LDS (DG_ACC, whose epilogue also reads r2/r3 from
  // global memory, measured faster with direct stores)
  constexpr bool kRun = epi_run<EPI>();  // g added in the run layout
  constexpr bool kF = (EPI == EPI_RESID || kRun);
  float4 fv[NPT][NCT];  // fp32 outputs, written back through LDS after the loop
  uint2 bv[NPT][NCT];   // bf16 outputs, likewise
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
      const int col = (ct0 + c) * 16 + fk * 4;
      const int co = cb * 64 + col;
      const size_t o = pix * p.Cout + co;
      f32x4 v = acc[pt][c];
      if constexpr (EPI == EPI_RELU_BF16 || EPI == EPI_POOL_BF16 || EPI == EPI_RESID || EPI == EPI_PS_BF16 ||
                    EPI == EPI_PLAIN_BF16 || EPI == EPI_RELU_POOL || epi_cr<EPI>()) {
        v[0] += bias[c].x; v[1] += bias[c].y; v[2] += bias[c].z; v[3] += bias[c].w;
      }
      if constexpr (EPI == EPI_RELU_BF16 || EPI == EPI_RELU_POOL) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if constexpr (EPI == EPI_RESID) {
        const float4 rr = e.r1[pt][c];
        v[0] = p.alpha * v[0] + rr.x; v[1] = p.alpha * v[1] + rr.y;
        v[2] = p.alpha * v[2] + rr.z; v[3] = p.alpha * v[3] + rr.w;
        fv[pt][c] = make_float4(v[0], v[1], v[2], v[3]);
      }
      if constexpr (EPI == EPI_DG_RELUMASK) {
        const uint2 tt = e.aux[pt][c];
        v[0] = p.alpha * relu_mask(tt.x & 0xFFFFu, v[0]);
        v[1] = p.alpha * relu_mask(tt.x >> 16, v[1]);
        v[2] = p.alpha * relu_mask(tt.y & 0xFFFFu, v[2]);
        v[3] = p.alpha * relu_mask(tt.y >> 16, v[3]);
      }
      if constexpr (EPI == EPI_DG_ACC && !kRun) {
        const float4 rr = e.r1[pt][c];
        v[0] += rr.x; v[1] += rr.y; v[2] += rr.z; v[3] += rr.w;
        if (p.r2) {
          const float4 q = *reinterpret_cast<const float4*>(p.r2 + o);
          v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
        }
        if (p.r3) {
          const float4 q = *reinterpret_cast<const float4*>(p.r3 + o);
          v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
        }
        st_wt16(rfa, p.yf, (uint32_t)(o * 4), make_float4(v[0], v[1], v[2], v[3]));
        if (p.part) {
          const uint2 uu = e.aux[pt][c];
          ps0[c][0] += v[0]; ps0[c][1] += v[1]; ps0[c][2] += v[2]; ps0[c][3] += v[3];
          ps1[c][0] += v[0] * bf2f(uu.x & 0xFFFFu);
          ps1[c][1] += v[1] * bf2f(uu.x >> 16);
          ps1[c][2] += v[2] * bf2f(uu.y & 0xFFFFu);
          ps1[c][3] += v[3] * bf2f(uu.y >> 16);
        }
      }
      if constexpr (epi_cr_bf16<EPI>()) {  // u in bf16: the product's operand (and stored for backward)
        bv[pt][c] = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        continue;
      }
      if constexpr (kRun) {
        fv[pt][c] = make_float4(v[0], v[1], v[2], v[3]);  // dx; g is added in the store loop
        continue;  // no bf16 copy
      }
      if constexpr (EPI == EPI_POOL_BF16) {  // the pooled mean of the fp32 conv output
        ps0[c][0] += v[0]; ps0[c][1] += v[1]; ps0[c][2] += v[2]; ps0[c][3] += v[3];
      }
      bv[pt][c] = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      if constexpr (EPI == EPI_RELU_POOL) {  // sums of the bf16 t conv2 reads (ca_scale.hpp)
        const uint2 b = bv[pt][c];
        const float t4[4] = {bf2f(b.x & 0xFFFFu), bf2f(b.x >> 16), bf2f(b.y & 0xFFFFu), bf2f(b.y >> 16)};
#pragma unroll
        for (int r = 0; r < 4; ++r) ps0[c][r] += t4[r];
      }
    }
  }
  if constexpr (EPI == EPI_RELU_POOL) {
    if (cpon) {  // (uniform) the image's border columns and corners in this wave's row, from
                 // the first and last pixel tiles' bf16 t (outside the loop above: inside it
                 // the corner stores cost 0.4 K cycles per strip)
      const bool c0 = fr == 0 && x0 == 0, cw = fr == 15 && x0 + NPT * 16 == p.W;
      const bool yc = y == 0 || y == p.H - 1;
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        const uint2 a = bv[0][c], b = bv[NPT - 1][c];
        const float ta[4] = {bf2f(a.x & 0xFFFFu), bf2f(a.x >> 16), bf2f(a.y & 0xFFFFu), bf2f(a.y >> 16)};
        const float tb[4] = {bf2f(b.x & 0xFFFFu), bf2f(b.x >> 16), bf2f(b.y & 0xFFFFu), bf2f(b.y >> 16)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          cp->colA[c][r] += c0 ? ta[r] : 0.f;
          cp->colB[c][r] += cw ? tb[r] : 0.f;
        }
        if (yc) {
          float* cn = cp->scr + 512 + (ct0 + c) * 16 + fk * 4;  // (0,0) (0,W-1) (H-1,0) (H-1,W-1)
#pragma unroll
          for (int e = 0; e < 2; ++e) {  // e = 0: row 0, 1: row H-1 (both for a one-row image)
            if (e == 0 ? y != 0 : y != p.H - 1) continue;
            if (c0) *reinterpret_cast<float4*>(cn + (2 * e) * 64) = make_float4(ta[0], ta[1], ta[2], ta[3]);
            if (cw) *reinterpret_cast<float4*>(cn + (2 * e + 1) * 64) = make_float4(tb[0], tb[1], tb[2], tb[3]);
          }
        }
      }
    }
  }
  const int lane = tid & 63;
  // conv2 with u rounded to bf16 before anything reads it (epi_cr_bf16): the row is
  // staged once as bf16 (128 B per pixel, chunk-swizzled: one barrier, not the fp32
  // path's two halves and four) and read back in the pair's run layout
  if constexpr (epi_cr_bf16<EPI>()) {
    constexpr int HALF = NPT * 8, RUNS = HALF / 4;
    static_assert(kShared, "the 8-wave body");
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        const int px = pt * 16 + fr, c16 = (ct0 + c) * 2 + (fk >> 1);
        *reinterpret_cast<uint2*>(stage + px * 128 + ((c16 ^ (px & 7)) << 4) + (fk & 1) * 8) = bv[pt][c];
      }
    stage_sync();
    [[maybe_unused]] const auto rbb = wt_rsrc(p.yb, (uint32_t)((size_t)p.N * HW * p.Cout * 2));
    const auto rph = wt_rsrc(p.yph, (uint32_t)((size_t)p.N * HW * p.Cout * 2));
    const auto rpl = wt_rsrc(p.ypl, (uint32_t)((size_t)p.N * HW * p.Cout));
    const size_t pix0 = (size_t)n * HW + (size_t)y * p.W + x0;
    // every run's u first (the stage's last reads), then the strip-end barrier here (the
    // body skips its own for these epilogues), then the arithmetic and the stores: the
    // stores' issue no longer holds every wave at that barrier
    uint2 ubs[RUNS];
#pragma unroll
    for (int q = 0; q < RUNS; ++q) {
      const int h = q / (RUNS / 2), i = 2 * (q % (RUNS / 2)) + half_id;
      const int lin = i * 1024 + lane * 16, px = h * HALF + (lin >> 8), c = (lin >> 4) & 15;
      ubs[q] = *reinterpret_cast<const uint2*>(stage + px * 128 + (((c >> 1) ^ (px & 7)) << 4) + (c & 1) * 8);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < RUNS / 2; ++j) {
        // run i of the half: pixels 4 (i & ..) -- lane = channels 4c..4c+3 of pixel px
        const int i = 2 * j + half_id;
        const int lin = i * 1024 + lane * 16, px = h * HALF + (lin >> 8), c = (lin >> 4) & 15;
        const int q = h * (RUNS / 2) + j;
        const uint2 ub = ubs[q];
        float4 hh = e.r1[q / NCT][q % NCT];
        if (p.r1h) hh = pair_decode4(make_uint2(__float_as_uint(hh.x), __float_as_uint(hh.y)), __float_as_uint(hh.z));
        const uint32_t oe = (uint32_t)((pix0 + px) * p.Cout + cb * 64 + c * 4);  // element
        if constexpr (EPI == EPI_CA_RESID_U) st_wt8(rbb, p.yb, oe * 2, ub);  // u for backward
        const float o0 = fmaf(bf2f(ub.x & 0xFFFFu), fs.x, hh.x), o1 = fmaf(bf2f(ub.x >> 16), fs.y, hh.y);
        const float o2 = fmaf(bf2f(ub.y & 0xFFFFu), fs.z, hh.z), o3 = fmaf(bf2f(ub.y >> 16), fs.w, hh.w);
        uint2 hi;
        const uint32_t lo = pair_encode4(o0, o1, o2, o3, hi);
        st_wt8(rph, p.yph, oe * 2, hi);
        st_wt4(rpl, p.ypl, oe, lo);
      }
    return;
  }
  // fp32 output: staged in LDS in two halves of the row (256 B per pixel,
  // chunk-swizzled) and written back as 1 KiB contiguous runs (full lines)
  if constexpr (kF) {
    if (kRun || p.yf) {
      constexpr int HALF = NPT * 8;  // pixels per half
      constexpr int RUNS = HALF / 4;  // 1 KiB runs per half
      const auto rf = wt_rsrc(p.yf, (uint32_t)((size_t)p.N * HW * p.Cout * 4));
      [[maybe_unused]] const auto rbb = wt_rsrc(p.yb, (uint32_t)((size_t)p.N * HW * p.Cout * 2));
      [[maybe_unused]] const auto rph = wt_rsrc(p.yph, (uint32_t)((size_t)p.N * HW * p.Cout * 2));
      [[maybe_unused]] const auto rpl = wt_rsrc(p.ypl, (uint32_t)((size_t)p.N * HW * p.Cout));
      const size_t pix0 = (size_t)n * HW + (size_t)y * p.W + x0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
          for (int c = 0; c < NCT; ++c) {
            const int px = pt * 16 + fr;
            if ((px >= HALF) == (h == 1)) {
              const int lpx = px - h * HALF, c16 = (ct0 + c) * 4 + fk;
              *reinterpret_cast<float4*>(stage + lpx * 256 + ((c16 ^ (lpx & 15)) << 4)) = fv[pt][c];
            }
          }
        stage_sync();
#pragma unroll
        for (int j = 0; j < (kShared ? RUNS / 2 : RUNS); ++j) {
          const int i = kShared ? 2 * j + half_id : j;
          const int lin = i * 1024 + lane * 16, lpx = lin >> 8, c = (lin >> 4) & 15;
          float4 val = *reinterpret_cast<const float4*>(stage + lpx * 256 + ((c ^ (lpx & 15)) << 4));
          if constexpr (epi_cr<EPI>()) {  // (EPI_CA_RESID with SRMI_INFER_BF16U = 0: fp32 u)
            // h' = h + s u in the run layout (the lane's channels 4c..4c+3: s in fs), out as the pair
            const int q = h * (kShared ? RUNS / 2 : RUNS) + j;
            float4 hh = e.r1[q / NCT][q % NCT];
            if (p.r1h)
              hh = pair_decode4(make_uint2(__float_as_uint(hh.x), __float_as_uint(hh.y)), __float_as_uint(hh.z));
            const uint32_t oe = (uint32_t)((pix0 + h * HALF + lpx) * p.Cout + cb * 64 + c * 4);  // element
            const float o0 = fmaf(val.x, fs.x, hh.x), o1 = fmaf(val.y, fs.y, hh.y);
            const float o2 = fmaf(val.z, fs.z, hh.z), o3 = fmaf(val.w, fs.w, hh.w);
            uint2 hi;
            const uint32_t lo = pair_encode4(o0, o1, o2, o3, hi);
            st_wt8(rph, p.yph, oe * 2, hi);
            st_wt4(rpl, p.ypl, oe, lo);
            continue;
          }
          if constexpr (kRun) {
            // g += dx in the run layout; the lane's channels 4c..4c+3 (c = lane & 15)
            // are the same in every run, so its sums accumulate in registers
            const int q = h * (kShared ? RUNS / 2 : RUNS) + j;
            float4 gg;
            if constexpr (EPI == EPI_DG_ACC_CA16) {
              const uint2 gq = e.gb[q / NCT][q % NCT];
              gg = unpack_bf16x4(gq.x, gq.y);
            } else if constexpr (EPI == EPI_DG_CA16) {
              gg = make_float4(0.f, 0.f, 0.f, 0.f);
            } else if constexpr (EPI == EPI_DG_ACC_G1) {
              const uint2 gq = e.gb[q / NCT][q % NCT];
              gg = unpack_bf16x4(gq.x, gq.y);
            } else {
              gg = e.r1[q / NCT][q % NCT];
              if constexpr (EPI == EPI_DG_ACC) {
                if (p.r1b) gg = unpack_bf16x4(__float_as_uint(gg.x), __float_as_uint(gg.y));
              }
            }
            const uint2 uu = e.aux[q / NCT][q % NCT];
            val.x += gg.x; val.y += gg.y; val.z += gg.z; val.w += gg.w;
            if constexpr (EPI == EPI_DG_ACC || EPI == EPI_DG_ACC_G1) {
              const float4 g2 = e.r2[q / NCT][q % NCT];
              val.x += g2.x; val.y += g2.y; val.z += g2.z; val.w += g2.w;
              if (p.r3) {
                const float4 g3 = *reinterpret_cast<const float4*>(
                    p.r3 + (pix0 + h * HALF + lpx) * p.Cout + cb * 64 + c * 4);
                val.x += g3.x; val.y += g3.y; val.z += g3.z; val.w += g3.w;
              }
            }
            // the bf16 gradient stream (DG_ACC_CA16, or DG_ACC without an fp32 output): g is
            // rounded once, and the CA sums and the store take that stored value
            if (epi_g16<EPI>() || (EPI == EPI_DG_ACC && !p.yf)) {  // (uniform)
              const uint32_t a = pack2(val.x, val.y), b = pack2(val.z, val.w);
              val = unpack_bf16x4(a, b);
            }
            if constexpr (EPI != EPI_DG_ACC_G1) {  // (the CA sums of the RCAB below)
              ps0[0][0] += val.x; ps0[0][1] += val.y; ps0[0][2] += val.z; ps0[0][3] += val.w;
              ps1[0][0] += val.x * bf2f(uu.x & 0xFFFFu);
              ps1[0][1] += val.y * bf2f(uu.x >> 16);
              ps1[0][2] += val.z * bf2f(uu.y & 0xFFFFu);
              ps1[0][3] += val.w * bf2f(uu.y >> 16);
            }
          }
          const uint32_t oel = (uint32_t)((pix0 + h * HALF + lpx) * p.Cout + cb * 64 + c * 4);  // element
          if constexpr (epi_g16<EPI>()) {  // 512 contiguous bytes per instruction
            st_wt8(rbb, p.yb, oel * 2, make_uint2(pack2(val.x, val.y), pack2(val.z, val.w)));
            continue;
          }
          if (EPI != EPI_DG_ACC || p.yf) st_wt16(rf, p.yf, oel * 4, val);
          if constexpr (EPI == EPI_DG_ACC_G1) {  // the group input gradient's bf16 copy
            st_wt8(rbb, p.yb, oel * 2, make_uint2(pack2(val.x, val.y), pack2(val.z, val.w)));
          }
          if constexpr (EPI == EPI_DG_ACC) {
            if (p.yb)  // its bf16 copy (or, yf null, the stream itself): 512 contiguous bytes per instruction
              st_wt8(rbb, p.yb, oel * 2, make_uint2(pack2(val.x, val.y), pack2(val.z, val.w)));
          }
        }
        stage_sync();
      }
    }
  }
  // bf16 output staged in LDS (the row, 128 B per pixel, chunk-swizzled)
  if constexpr (!kRun) {
    if (p.yb) {
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
        for (int c = 0; c < NCT; ++c) {
          const int px = pt * 16 + fr, c16 = (ct0 + c) * 2 + (fk >> 1);
          *reinterpret_cast<uint2*>(stage + px * 128 + ((c16 ^ (px & 7)) << 4) + (fk & 1) * 8) = bv[pt][c];
        }
    }
  }
  if constexpr (!kRun) stage_sync();  // (kRun: the staging loop above ended with one)
  // ... and written back as full 128-byte lines: one 1 KiB contiguous run per
  // instruction (the per-lane 8-byte stores of the MFMA layout touched 32-byte
  // pieces of 16 lines each and stalled the store path for ~2 K cycles per strip).
  // The wave's own LDS writes precede its reads (in-order LDS per wave).
  if (!kRun && p.yb) {
    const auto rb = wt_rsrc(p.yb, (uint32_t)((size_t)p.N * HW * p.Cout * 2));
#pragma unroll
    for (int j = 0; j < (kShared ? NPT : NPT * 2); ++j) {
      const int i = kShared ? 2 * j + half_id : j;
      const int lin = i * 1024 + lane * 16, px = lin >> 7, c = (lin >> 4) & 7;
      const uint4 val = *reinterpret_cast<const uint4*>(stage + px * 128 + ((c ^ (px & 7)) << 4));
      size_t line;
      if constexpr (EPI == EPI_PS_BF16) {
        line = (((size_t)n * (2 * p.H) + 2 * y + (cb >> 1)) * (size_t)(2 * p.W) + 2 * (x0 + px) + (cb & 1)) * 64;
      } else {
        line = ((size_t)n * HW + (size_t)y * p.W + x0 + px) * p.Cout + cb * 64;
      }
      st_wt16(rb, p.yb, (uint32_t)((line + c * 8) * 2), val);
    }
  }
  if constexpr (kRun) {
   if (EPI != EPI_DG_ACC_G1 && (EPI == EPI_DG_ACC_CA || epi_g16<EPI>() || p.part)) {  // (uniform)
    // lanes l, l ^ 16, l ^ 32, l ^ 48 hold the same 4 channels: fixed-order xor
    // sums, then one 64-channel partial per wave in red[wave][2][64], summed over
    // the waves in wave order
    const int wave = tid >> 6;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = ps0[0][r], b = ps1[0][r];
      a += __shfl_xor(a, 16, 64);
      b += __shfl_xor(b, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 32, 64);
      if (lane < 16) {
        red[(wave * 2 + 0) * 64 + lane * 4 + r] = a;
        red[(wave * 2 + 1) * 64 + lane * 4 + r] = b;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    constexpr int NWV = kShared ? 8 : 4;
    if (tid < 128) {
      const int s = tid >> 6, c = tid & 63;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) sum += red[(w * 2 + s) * 64 + c];
      p.part[((size_t)n * nstrips + strip) * p.part_stride + s * 64 + c] = sum;
    }
   }
  } else if constexpr (kPart1 || kPart2) {
    const bool on = EPI != EPI_DG_ACC || p.part;
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // red[] writes visible; global stores may stay in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (on) {
      if (tid < 64) {
        const float sum = red[tid] + red[128 + tid] + red[256 + tid] + red[384 + tid];
        p.part[((size_t)n * nstrips + strip) * p.part_stride + cb * 64 + tid] = sum;
        if constexpr (EPI == EPI_RELU_POOL) {
          if (cpon) {  // T over the run, and the per-row sums (red) of the image's first / last row
            cp->tacc += sum;
            const int y0 = y - row;
            if (y0 == 0) cp->scr[256 + tid] = red[tid];
            if (y0 + kTH - 1 == p.H - 1) cp->scr[256 + 64 + tid] = red[(kTH - 1) * 128 + tid];
          }
        }
      } else if (kPart2 && tid < 128) {
        const int c = tid - 64;
        const float sum = red[64 + c] + red[192 + c] + red[320 + c] + red[448 + c];
        p.part[((size_t)n * nstrips + strip) * p.part_stride + 64 + c] = sum;
      }
    }
  }
}

constexpr int kFragBuf = 2;  // register buffers of A/B fragments (K-steps)

template <int EPI>
constexpr bool conv64_defers() {
  return ((SRMI_DEFER & 1) && EPI == EPI_RELU_BF16) || ((SRMI_DEFER & 2) && EPI == EPI_POOL_BF16) ||
         ((SRMI_DEFER & 4) && EPI == EPI_DG_RELUMASK) || ((SRMI_DEFER & 8) && EPI == EPI_DG_ACC_CA) ||
         ((SRMI_DEFER & 16) && EPI == EPI_RELU_POOL) || ((SRMI_DEFER & 32) && EPI == EPI_CA_RESID) ||
         ((SRMI_DEFER & (64 | 128)) && EPI == EPI_DG_ACC_CA16);
  // (EPI_CA_RESID_U: the non-deferred body only)
}
template <int TW, int EPI>
__device__ __forceinline__ void conv64_body_defer(const ConvParams& p, int run_len, int bid, char* smem, int tail,
                                                  bool tail_part);

// The kernel body as a device function of a virtual block index `bid` and the
// workgroup's LDS (>= Conv2Smem<TW>::TOTAL bytes), so that a horizontally fused
// launch (wgrad3x3.hip, rcab_bwd_kernel) can run it beside other work.
// tail > 0 splits each run: the workgroup of run `bid` does its strips except the
// last `tail` ones (tail_part = false), or only those (tail_part = true; the fused
// backward hands them to the filter-gradient workgroup of the same rows)
//
// NW = waves per workgroup: 4 (one per output row of the strip, all 64 output
// channels) or 8 (a wave per row and channel half: two waves per SIMD, so one wave's
// LDS / memory waits overlap the other's MFMAs; same LDS footprint)
// WRES: the filter image is already resident in LDS (the caller loaded it): no filter DMA
template <int TW, int EPI, int NW = 4, bool WRES = false>
__device__ __forceinline__ void conv64_body(const ConvParams& p, int run_len, int bid, char* smem, int tail = 0,
                                            bool tail_part = false) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  if constexpr (NW == 8 && conv64_defers<EPI>()) {
    conv64_body_defer<TW, EPI>(p, run_len, bid, smem, tail, tail_part);
    return;
  }
  constexpr int NCT = NW == 8 ? 2 : 4;  // 16-wide output-channel tiles per wave
  using S = Conv2Smem<TW>;
  constexpr int NPT = TW / 16;
  char* wl = smem;
  char* ring = smem + S::WB;
  float* red = reinterpret_cast<float*>(smem + S::WB + S::RING);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = wave & 3, ct0 = NCT * (wave >> 2);  // strip row, first channel tile
  const int fr = lane & 15, fk = lane >> 4;
  const int nsx = p.W / TW, nsy = p.H / kTH;
  const int runs_per_col = (nsy + run_len - 1) / run_len;
  int r = bid;
  const int ry = r % runs_per_col;
  r /= runs_per_col;
  const int sx = r % nsx;
  r /= nsx;
  const int n = r % p.N;
  const int cb = r / p.N;
  int k0 = ry * run_len, k1 = min(nsy, k0 + run_len);
  if (tail > 0) {
    if (tail_part) k0 = max(k0, k1 - tail);
    else k1 = max(k0, k1 - tail);
  }
  if (k0 >= k1) return;
  const int x0 = sx * TW;
  STAMP(0);

  const bf16_t* xn = p.x + (size_t)n * p.H * p.W * 64;
  // conv2 with its CA scale (cas_on: the training EPI_CA_RESID_U, the inference RCAB's
  // EPI_CA_RESID): its image's CA scale, computed after
  // the first strip's MFMAs (only that strip's epilogue needs it): its global operands
  // (t's border lines from other workgroups' conv1 output) are issued after the
  // prologue's wait and land under those MFMAs
  [[maybe_unused]] CaScalePre cq;
  constexpr bool kCas = epi_cr<EPI>() && NW == 8;  // (the scale needs 512 threads)
  // conv1 with cas_on (training, SRMI_CA_MPART): its share of the image's CA mean
  constexpr bool kMp = EPI == EPI_RELU_POOL && NW == 8;
  // conv2 reading those (the training EPI_CA_RESID_U under SRMI_CA_MPART; the launch
  // refuses cas_on without mpart there) or computing the scale from t (the inference one)
  constexpr bool kFromMp = EPI == EPI_CA_RESID_U && SRMI_CA_MPART;
  [[maybe_unused]] CaPart cpart;
  [[maybe_unused]] uint2 w2v[2][9];  // the lane's slices of conv2's filter image (run end)
  [[maybe_unused]] const bool cpon = kMp && p.cas_on;
  if constexpr (kMp) {
    cpart.scr = reinterpret_cast<float*>(smem + S::TOTAL);
    cpart.tacc = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) cpart.colA[c][r] = cpart.colB[c][r] = 0.f;
    if (cpon) cpart.scr[256 + threadIdx.x] = 0.f;  // bs and cn (published by the prologue barrier)
  }

  // LDS-DMA of one 4-row input group into its ring slot: one wave instruction per
  // 8 pixels (1 KiB), swizzle applied on the source side, halo lanes read the zero
  // page.  No registers hold in-flight data, so no compiler-inserted vmcnt waits.
  const int wv_s = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t rbase = lds_u32(ring);
  const void* const zpage = uniform_ptr(kZeros);
  constexpr int NGRP = S::GROUPB / 1024;         // 1 KiB DMA pieces per group
  constexpr int NGW = (NGRP + NW - 1) / NW;      // pieces per wave (upper bound)
  // Per-lane parts of the DMA source, computed once: piece i = wv_s + 4m covers ring
  // pixels q = 8i + lane/8, i.e. row rr and halo column hx of the group; the chunk
  // swizzle (q & 7) is the same in all three ring slots (4 (TW + 2) px apart).
  int loff[NGW], lrr[NGW];
  uint32_t okx = 0;
#pragma unroll
  for (int m = 0; m < NGW; ++m) {
    const int i = wv_s + NW * m;
    const int q = 8 * i + (lane >> 3);
    const int c = (lane & 7) ^ (q & 7);
    const int rr = q / (TW + 2), hx = q - rr * (TW + 2);
    const int xx = x0 - 1 + hx;
    okx |= (i < NGRP && xx >= 0 && xx < p.W) ? (1u << m) : 0u;
    loff[m] = ((rr * p.W + hx - 1) * 64 + c * 8) * (int)sizeof(bf16_t);
    lrr[m] = rr;
  }
  auto group_dma_one = [&](int gidx, int m) __attribute__((always_inline)) {
    const int slot = gidx % 3, y0 = 4 * gidx - 3;
    const char* base = reinterpret_cast<const char*>(xn + ((ptrdiff_t)y0 * p.W + x0) * 64);
    const int o = loff[m];  // ring slots are 4 (TW + 2) px apart, a multiple of 8: same swizzle
    const bool ok = ((okx >> m) & 1u) && y0 + lrr[m] >= 0 && y0 + lrr[m] < p.H;
    const void* src = ok ? (const void*)(base + o) : zpage;
    glds16(src, rbase + (uint32_t)(slot * 4 * (TW + 2)) * 128u + (uint32_t)(wv_s + NW * m) * 1024u);
  };
  auto group_dma = [&](int gidx) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < NGW; ++m)
      if (wv_s + NW * m < NGRP) group_dma_one(gidx, m);
  };

  // bias first (read only by the epilogue): its latency hides under the prologue wait
  // instead of following it (~650 cycles per workgroup)
  float4 bias[NCT];
  {
    const float* bp = p.bias ? p.bias : reinterpret_cast<const float*>(kZeros);  // pointer select, no branch
#pragma unroll
    for (int c = 0; c < NCT; ++c) bias[c] = *reinterpret_cast<const float4*>(bp + cb * 64 + (ct0 + c) * 16 + fk * 4);
  }
  // prologue: filters (all 9 taps, 72 KiB) and input groups k0, k0+1, all by LDS-DMA
  // (swizzle on the source side), everything in flight before the one wait.  (Waiting
  // only for the groups and the first taps, the rest landing under the first strip's
  // K-steps, measured slower: the prologue is latency-, not byte-bound, -300 cycles,
  // while the first strip's MFMA phase grew by 500.)
  {
    const uint32_t wbase = lds_u32(wl);
    if constexpr (!WRES) {
      for (int i = wv_s; i < 72; i += NW) {
        const int tap = i >> 3, row = 8 * (i & 7) + (lane >> 3), c = (lane & 7) ^ (row & 7);
        glds16(p.w + ((size_t)(tap * p.Cout + cb * 64 + row)) * 64 + c * 8, wbase + (uint32_t)i * 1024u);
      }
    }
    group_dma(k0);  // strip k reads input groups k and k + 1
    group_dma(k0 + 1);
    wait_vm<0>();
  }
  STAMP(1);
  // lane-constant A-fragment byte offsets (tap adds 8192)
  uint32_t aoff[2][NCT];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int c = 0; c < NCT; ++c) aoff[kk][c] = swz128((ct0 + c) * 16 + fr, kk * 4 + fk);
  // CA_RESID(_U): s for the lane's 4 run-layout channels (conv_epilogue2)
  float4 fs = float4{0.f, 0.f, 0.f, 0.f};
  if constexpr (epi_cr<EPI>()) {
    if (!kCas || !p.cas_on) fs = *reinterpret_cast<const float4*>(p.escale + (size_t)n * p.escale_stride + 4 * (lane & 15));
  }
  __syncthreads();
  if constexpr (kCas) {
    if constexpr (kFromMp) {
      // (the MLP weights too: conv2 has the registers here, and the finish's first
      //  barrier would otherwise wait for them)
      if (p.cas_on) {
        ca_mpart_load(p.cas, n, cq);
        ca_scale_load_params(p.cas, cq);
      }
    } else {
      if (p.cas_on) ca_scale_load_t(p.cas, n, p.H, p.W, cq);
    }
#ifdef SRMI_TLAT  // diagnostic: the latency of the scale's t operands alone (scale stamps 8, 9)
    if (p.cas.stamps && tid == 0) p.cas.stamps[blockIdx.x * 64 + 8] = __builtin_amdgcn_s_memtime();
    wait_vm<0>();
    if (p.cas.stamps && tid == 0) p.cas.stamps[blockIdx.x * 64 + 9] = __builtin_amdgcn_s_memtime();
#endif
  }

#pragma unroll 1
  for (int k = k0; k < k1; ++k) {
    const int y = 4 * k + row;
    const bool pf = (k + 1 < k1);
    // group k+2 -> ring slot (k+2)%3, which held group k-1 (last read by strip k-1,
    // released by the barrier that ended it)
    EpiPre<NPT, EPI, NCT> ep;
    [[maybe_unused]] const int sj = 2 + 5 * min(k - k0, 11);
    STAMP(sj);

    // B-fragment byte offsets per (ky, kx, kk); +2048 per 16-pixel tile
    uint32_t boff[3][3][2];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int rr = y + ky - 1 + 3;  // >= 2
      const int slot = ((rr >> 2) % 3) * 4 + (rr & 3);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) boff[ky][kx][kk] = swz128(slot * (TW + 2) + fr + kx, kk * 4 + fk);
    }

    f32x4 acc[NPT][NCT];
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // 18 K-steps (9 taps x 2 halves of 32 ci), fragments triple-buffered in
    // registers: steps s+1 and s+2's ds_reads are in flight while step s's MFMAs run.
    bf16x8 A[kFragBuf][NCT], B[kFragBuf][NPT];
    auto load_step = [&](int s, bf16x8 (&a)[NCT], bf16x8 (&b)[NPT]) __attribute__((always_inline)) {
      const int tap = s >> 1, kk = s & 1, ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int c = 0; c < NCT; ++c) a[c] = lds_frag(wl, tap * 8192 + aoff[kk][c]);
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) b[pt] = lds_frag(ring, boff[ky][kx][kk] + pt * 2048);
    };
    constexpr int LA = kFragBuf - 1;  // K-steps of LDS reads in flight ahead of the MFMAs
#pragma unroll
    for (int s = 0; s < LA; ++s) load_step(s, A[s], B[s]);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      // group k+2's DMA pieces and the epilogue operands are issued one or two per
      // K-step, so a full memory queue stalls the wave between MFMA groups only
      if (s < NGW && pf && wv_s + NW * s < NGRP) group_dma_one(k + 2, s);
      // the epilogue operands, two per K-step from the first one: a whole strip of
      // MFMAs to land (spread over K-steps 2..13, the heavy fp32 epilogue of
      // DG_ACC_CA waited on its last ones at the end of the K-loop: +1.3 % step)
      if (2 * s < NPT * NCT) epi_prefetch_one<NPT, EPI, NCT>(p, ep, n, cb, y, x0, fr, fk, ct0, 2 * s);
      if (2 * s + 1 < NPT * NCT) epi_prefetch_one<NPT, EPI, NCT>(p, ep, n, cb, y, x0, fr, fk, ct0, 2 * s + 1);
      __builtin_amdgcn_sched_barrier(0);
      const bool ld = s + LA < 18;
      if (ld) load_step(s + LA, A[(s + LA) % kFragBuf], B[(s + LA) % kFragBuf]);
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
        for (int c = 0; c < NCT; ++c)
          acc[pt][c] = mfma16(A[s % kFragBuf][c], B[s % kFragBuf][pt], acc[pt][c]);
      // one fragment read issued behind each MFMA: the reads' issue time hides under
      // the MFMA pipe instead of stalling it between K-steps
      if (ld) {
#pragma unroll
        for (int j = 0; j < NCT + NPT; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        }
        if constexpr (NCT * NPT > NCT + NPT) __builtin_amdgcn_sched_group_barrier(0x008, NCT * NPT - (NCT + NPT), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // group k+2's DMA, the epilogue operands and the previous strip's stores had the
    // whole MFMA phase to land: drain them here, before the epilogue (the barrier at
    // the end of the strip then publishes group k+2 to every wave)
    wait_vm<0>();
    STAMP(sj + 1);
    if constexpr (kCas) {
      if (p.cas_on && k == k0) {  // the image's scale (every wave: uniform), before the first epilogue
        // scratch beyond the body's LDS (the launch adds kCaScaleFloats floats); the first
        // workgroup of the image writes its record m | z1 | s for backward
        if constexpr (!kFromMp) ca_scale_load_params(p.cas, cq);  // (L2-resident; used after two barriers)
        float* sm = reinterpret_cast<float*>(smem + S::TOTAL);
        if constexpr (kFromMp)  // from conv1's partial means
          ca_scale_from_mpart(p.cas, cq, n, p.H * p.W, sm, ry == 0 && sx == 0 && cb == 0 && !tail_part);
        else
          ca_scale_finish<false>(p.cas, cq, n, p.H, p.W, sm, wl, ry == 0 && sx == 0 && cb == 0 && !tail_part);
        fs = *reinterpret_cast<const float4*>(sm + kCaScaleS + 4 * (lane & 15));
      }
    }
    STAMP(sj + 2);
    // every wave is past its last read of input group k: its ring slot stages the
    // strip's bf16 output rows (slot k%3 is next written by group k+3's DMA,
    // issued after the barrier that ends this strip)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (kMp) {  // conv2's filter slices for the run-end matvec, under the last epilogue
      if (cpon && k == k1 - 1) ca_matvec_load_w(p.cas.wimg, tid, w2v);
    }
    conv_epilogue2<NPT, EPI, NCT>(p, acc, ep, bias, n, cb, y, x0, k * nsx + sx,
                                                               nsy * nsx, red, fr, fk, row, ct0,
                                  tid, ring + (k % 3) * S::GROUPB + row * TW * 128, fs, &cpart, kMp && cpon);
    STAMP(sj + 3);
    // LDS-only barrier: this strip's global stores stay in flight into the next strip
    // (the bf16-staged conv2 epilogues run it themselves, after their last stage reads)
    if constexpr (!epi_cr_bf16<EPI>()) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    STAMP(sj + 4);
  }
  if constexpr (kMp) {
    if (cpon) {  // the run's share of the image's CA mean: border columns over the 4 rows,
                 // then ca_matvec on conv2's filter image -> mpart[n][run]
      float* scr = cpart.scr;
      float* colacc = scr + 768;  // [4 rows][2][64]
      if (fr == 0 || fr == 15) {  // (one branch: lanes of column 0 write colA, of W-1 colB)
        const int l = fr == 0 ? 0 : 1;
#pragma unroll
        for (int c = 0; c < NCT; ++c)
          *reinterpret_cast<float4*>(colacc + (row * 2 + l) * 64 + (ct0 + c) * 16 + fk * 4) =
              l == 0 ? make_float4(cpart.colA[c][0], cpart.colA[c][1], cpart.colA[c][2], cpart.colA[c][3])
                     : make_float4(cpart.colB[c][0], cpart.colB[c][1], cpart.colB[c][2], cpart.colB[c][3]);
      }
      if (tid < 64) scr[tid] = cpart.tacc;  // T in the first of ca_matvec's four partial rows
      else if (tid < 256) scr[tid] = 0.f;
      STAMP(57);
      __syncthreads();
      STAMP(58);
      if (tid < 128) {
        const int l = tid >> 6, ch = tid & 63;
        scr[256 + (2 + l) * 64 + ch] = ((colacc[(0 * 2 + l) * 64 + ch] + colacc[(1 * 2 + l) * 64 + ch]) +
                                        colacc[(2 * 2 + l) * 64 + ch]) + colacc[(3 * 2 + l) * 64 + ch];
      }
      __syncthreads();
      STAMP(59);
      const float a = ca_matvec(scr, scr + 256, scr + 512, w2v, tid);
      const int runs_per_col = (nsy + run_len - 1) / run_len;
      if ((tid & 7) == 0) p.cas.mpart[((size_t)n * p.cas.nruns + sx * runs_per_col + ry) * 64 + (tid >> 3)] = a;
      STAMP(60);
    }
  }
  STAMP(61);
}

// ============================================================================
// Deferred-epilogue form of the 8-wave body (the four hot epilogues: conv1 RELU and
// conv2 POOL forward, the ReLU-mask dgrad of conv2 and the gradient-stream dgrad of
// conv1).  In the form above every strip ends with its epilogue behind a barrier:
// the MFMA pipe idles for ~2.6 K cycles per strip (bias / mask, packing, LDS
// staging, two more barriers, the stores) against ~3.5 K cycles of MFMA
// (profiles/r02_conv_stamps_8wave.txt).  Here the epilogue of strip k-1 runs
// inside strip k's K-loop, one pixel tile per K-step behind that step's MFMAs, from
// the previous strip's accumulators held in registers; its operands (ReLU output t,
// gradient stream g, CA input u) are loaded at the first K-steps of strip k; strip
// k ends with ONE barrier (ring-slot release + group k+2's DMA published).  Only
// the last strip of a run keeps an exposed epilogue.
//
// No LDS staging: each wave stores its own results straight from registers.  For
// the bf16 outputs the filter rows are read permuted -- accumulator row 4fk + r of
// tile c is output channel ct0*16 + 8fk + 4c + r -- so a lane holds 8 contiguous
// channels of its pixel and one 16-byte store per pixel tile writes, per pixel, the
// wave's whole 64-byte channel half (16 such runs per instruction).  The fp32
// gradient stream keeps the natural rows: a lane's 4 channels of a tile are 16
// contiguous bytes, 64 contiguous bytes per pixel per store.  Channel sums (POOL,
// DG_ACC_CA) go through two LDS buffers: strip k-1's per-row sums are written
// during strip k, summed over the 4 rows and stored during strip k+1.  Results are
// bit-identical to the form above (same MFMA order per output element, same sum
// order).

// opaque to the IR passes (a value "redefined" here cannot be computed with earlier)
__device__ __forceinline__ void pin(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(uint32_t& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin4(f32x4& v) {
  float a = v[0], b = v[1], c = v[2], d = v[3];
  pin(a); pin(b); pin(c); pin(d);
  v = f32x4{a, b, c, d};
}
__device__ __forceinline__ void pin4f(float4& v) { pin(v.x); pin(v.y); pin(v.z); pin(v.w); }
__device__ __forceinline__ void pin4u(uint4& v) { pin(v.x); pin(v.y); pin(v.z); pin(v.w); }

// deferred epilogue stores: write-through (sc1) like the others (SRMI_WT)
template <typename V>
__device__ __forceinline__ void st_defer(__amdgpu_buffer_rsrc_t r, void* base, uint32_t off, const V& v) {
  st_wt16(r, base, off, v);
}

template <int NPT>
struct DeferOps {
  uint4 t[NPT];      // DG_RELUMASK: the ReLU output t, 8 bf16 (permuted rows)
  float4 g[NPT][2];  // DG_ACC_CA: gradient stream in (natural rows)
  uint2 u[NPT][2];   // DG_ACC_CA: the CA input u
  uint4 uq[NPT];     // DG_ACC_CA16: the CA input u, 8 bf16 (permuted rows; the stream g in t)
};

template <int TW, int EPI>
__device__ __forceinline__ void conv64_body_defer(const ConvParams& p, int run_len, int bid, char* smem, int tail,
                                                  bool tail_part) {
  constexpr int NW = 8, NCT = 2;
  using S = Conv2Smem<TW>;
  constexpr int NPT = TW / 16;
  constexpr bool kPerm = EPI != EPI_DG_ACC_CA;  // bf16 output: permuted filter rows
  constexpr bool kG16 = EPI == EPI_DG_ACC_CA16;  // the bf16 gradient stream: g in / out as 8 bf16 per lane
  constexpr bool kPart = EPI == EPI_POOL_BF16 || EPI == EPI_DG_ACC_CA || EPI == EPI_RELU_POOL || kG16;
  constexpr bool kCA = EPI == EPI_DG_ACC_CA;
  constexpr bool kS1 = kCA || kG16;  // the second channel sum (g * u)
  // DG_ACC_CA16 with SRMI_DEFER bit 128: this body's register-direct epilogue, run right
  // after its own strip's K-loop (operands loaded at the strip's first K-steps) instead of
  // inside the next strip's: no LDS staging, one barrier per strip
  constexpr bool kImm = kG16 && (SRMI_DEFER & 128);
  constexpr bool kCR = EPI == EPI_CA_RESID;  // h' = h + s u: 8 contiguous channels per lane (permuted rows)
  constexpr int ES = 10;  // K-step of the first deferred epilogue tile
  char* wl = smem;
  char* ring = smem + S::WB;
  float* red = reinterpret_cast<float*>(smem + S::WB + S::RING);  // [2 buffers][4 rows][2][64]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = wave & 3, ct0 = NCT * (wave >> 2);
  const int fr = lane & 15, fk = lane >> 4;
  const int nsx = p.W / TW, nsy = p.H / kTH;
  const int runs_per_col = (nsy + run_len - 1) / run_len;
  int r = bid;
  const int ry = r % runs_per_col;
  r /= runs_per_col;
  const int sx = r % nsx;
  r /= nsx;
  const int n = r % p.N;
  const int cb = r / p.N;
  int k0 = ry * run_len, k1 = min(nsy, k0 + run_len);
  if (tail > 0) {
    if (tail_part) k0 = max(k0, k1 - tail);
    else k1 = max(k0, k1 - tail);
  }
  if (k0 >= k1) return;
  const int x0 = sx * TW;
  STAMP(0);
  const bf16_t* xn = p.x + (size_t)n * p.H * p.W * 64;
  const size_t HW = (size_t)p.H * p.W;

  // input-group DMA (as conv64_body)
  const int wv_s = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t rbase = lds_u32(ring);
  const void* const zpage = uniform_ptr(kZeros);
  constexpr int NGRP = S::GROUPB / 1024;
  constexpr int NGW = (NGRP + NW - 1) / NW;
  int loff[NGW], lrr[NGW];
  uint32_t okx = 0;
#pragma unroll
  for (int m = 0; m < NGW; ++m) {
    const int i = wv_s + NW * m;
    const int q = 8 * i + (lane >> 3);
    const int c = (lane & 7) ^ (q & 7);
    const int rr = q / (TW + 2), hx = q - rr * (TW + 2);
    const int xx = x0 - 1 + hx;
    okx |= (i < NGRP && xx >= 0 && xx < p.W) ? (1u << m) : 0u;
    loff[m] = ((rr * p.W + hx - 1) * 64 + c * 8) * (int)sizeof(bf16_t);
    lrr[m] = rr;
  }
  auto group_dma_one = [&](int gidx, int m) __attribute__((always_inline)) {
    const int slot = gidx % 3, y0 = 4 * gidx - 3;
    const char* base = reinterpret_cast<const char*>(xn + ((ptrdiff_t)y0 * p.W + x0) * 64);
    const bool ok = ((okx >> m) & 1u) && y0 + lrr[m] >= 0 && y0 + lrr[m] < p.H;
    const void* src = ok ? (const void*)(base + loff[m]) : zpage;
    glds16(src, rbase + (uint32_t)(slot * 4 * (TW + 2)) * 128u + (uint32_t)(wv_s + NW * m) * 1024u);
  };
  auto group_dma = [&](int gidx) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < NGW; ++m)
      if (wv_s + NW * m < NGRP) group_dma_one(gidx, m);
  };
  // (DG_RELUMASK with p.gx: x is the gradient stream g) the image's CALayer backward MLP in
  // the prologue (ca_bwd.hpp; its operands issued behind the DMA, the first run of the image
  // writes the record) or its s and dm read, then du = bf16(g s + dm / HW) formed in place on
  // the wave's own DMA pieces of a group once they landed, before the barrier that publishes
  // them; the padding (zero page) stays zero.  A lane's 16 B are the channels 8 cc .. 8 cc + 7
  // of its pixel in every piece (the swizzle (lane & 7) ^ (q & 7), q = 8 i + lane / 8)
  [[maybe_unused]] const bool gx = EPI == EPI_DG_RELUMASK && p.gx.rec != nullptr;  // (uniform)
  [[maybe_unused]] float gxs[8], gxm[8];
  [[maybe_unused]] CaBwdPre cbq;
  auto gx_ok = [&](int gidx, int m) __attribute__((always_inline)) -> bool {
    const int y0 = 4 * gidx - 3;
    return wv_s + NW * m < NGRP && ((okx >> m) & 1u) && y0 + lrr[m] >= 0 && y0 + lrr[m] < p.H;
  };
  auto gx_ptr = [&](int gidx, int m) __attribute__((always_inline)) -> uint4* {
    return reinterpret_cast<uint4*>(ring + ((gidx % 3) * 4 * (TW + 2)) * 128 + (wv_s + NW * m) * 1024 + lane * 16);
  };
  // a group's pieces: every read first, then the arithmetic and the writes
  auto gx_group = [&](int gidx) __attribute__((always_inline)) {
    uint4 v[NGW];
#pragma unroll
    for (int m = 0; m < NGW; ++m)
      if (gx_ok(gidx, m)) v[m] = *gx_ptr(gidx, m);
#pragma unroll
    for (int m = 0; m < NGW; ++m)
      if (gx_ok(gidx, m)) *gx_ptr(gidx, m) = du_from_g8(v[m], gxs, gxm);
  };

  // channel of accumulator row (c, r) of this lane, and the lane's channel bases
  auto chan = [&](int c, int rr) -> int { return kPerm ? ct0 * 16 + 8 * fk + 4 * c + rr : (ct0 + c) * 16 + 4 * fk + rr; };
  float4 bias[NCT];
  {
    const float* bp = p.bias ? p.bias : reinterpret_cast<const float*>(kZeros);
#pragma unroll
    for (int c = 0; c < NCT; ++c) bias[c] = *reinterpret_cast<const float4*>(bp + cb * 64 + chan(c, 0));
  }
  {
    const uint32_t wbase = lds_u32(wl);
    // the filter image uses the swz128t chunk swizzle (c ^ (bit1, bit3 of the row)):
    // conflict-free for the permuted A rows (8 (fr >> 2) + 4c + (fr & 3)) as well as
    // the natural ones, where swz128 would collide 2-way on the permuted rows and make
    // the K-loop LDS-bound (20 -> 28 LDS cycles per wave and K-step against 24 of MFMA)
    for (int i = wv_s; i < 72; i += NW) {
      const int tap = i >> 3, rw = 8 * (i & 7) + (lane >> 3);
      const int c = (lane & 7) ^ ((((rw >> 1) & 1) << 1) | (((rw >> 3) & 1) << 2));
      glds16(p.w + ((size_t)(tap * p.Cout + cb * 64 + rw)) * 64 + c * 8, wbase + (uint32_t)i * 1024u);
    }
    group_dma(k0);
    group_dma(k0 + 1);
    [[maybe_unused]] const int cc = (lane & 7) ^ (lane >> 3);
    if constexpr (EPI == EPI_DG_RELUMASK) {
      if (gx) {
        if (p.gx.mlp) {
          if (tid < 256) ca_bwd_load(p.gx, n, tid, cbq);
        } else {
          const float* sp = p.gx.rec + (size_t)n * (128 + p.gx.CR) + 64 + p.gx.CR + cc * 8;
          const float* mp = p.gx.brec + (size_t)p.gx.N * (128 + p.gx.CR) + (size_t)n * 64 + cc * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            gxs[i] = sp[i];
            gxm[i] = mp[i] * p.gx.inv_hw;
          }
        }
      }
    }
    wait_vm<0>();
    if constexpr (EPI == EPI_DG_RELUMASK) {
      if (gx) {
        STAMP(32);
        if (p.gx.mlp) {
          float* sm = reinterpret_cast<float*>(smem + S::TOTAL);
          ca_bwd_mlp(p.gx, n, tid < 256 ? tid : -1, cbq, sm, ry == 0 && sx == 0 && cb == 0 && !tail_part);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            gxs[i] = sm[kCaBwdS + cc * 8 + i];
            gxm[i] = sm[kCaBwdDm + cc * 8 + i] * p.gx.inv_hw;
          }
        }
        STAMP(33);
        gx_group(k0);
        gx_group(k0 + 1);
        STAMP(34);
      }
    }
  }
  STAMP(1);
  // A-fragment rows: lane fr of tile c reads the filter row of the channel its
  // accumulator row fr will hold (permuted for bf16 outputs)
  uint32_t aoff[2][NCT];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int c = 0; c < NCT; ++c) {
      const int arow = kPerm ? ct0 * 16 + 8 * (fr >> 2) + 4 * c + (fr & 3) : (ct0 + c) * 16 + fr;
      aoff[kk][c] = swz128t(arow, kk * 4 + fk);
    }
  __syncthreads();

  const auto rout = kPerm ? wt_rsrc(p.yb, (uint32_t)((size_t)p.N * HW * p.Cout * 2))
                          : wt_rsrc(p.yf, (uint32_t)((size_t)p.N * HW * p.Cout * 4));
  [[maybe_unused]] const auto rph = wt_rsrc(p.yph, (uint32_t)((size_t)p.N * HW * p.Cout * 2));
  [[maybe_unused]] const auto rpl = wt_rsrc(p.ypl, (uint32_t)((size_t)p.N * HW * p.Cout));
  [[maybe_unused]] float sv[8];  // CA_RESID: s of the lane's 8 channels
  if constexpr (kCR) {
    const float* sp = p.escale + (size_t)n * p.escale_stride + ct0 * 16 + 8 * fk;
    const float4 a = *reinterpret_cast<const float4*>(sp), b = *reinterpret_cast<const float4*>(sp + 4);
    sv[0] = a.x; sv[1] = a.y; sv[2] = a.z; sv[3] = a.w; sv[4] = b.x; sv[5] = b.y; sv[6] = b.z; sv[7] = b.w;
  }
  const int nstrips_all = nsy * nsx;
  f32x4 accp[NPT][NCT];  // the previous strip's accumulators
  DeferOps<NPT> ops;     // operands of the pending epilogue

  // operand loads of the epilogue of strip kp (pixel row 4 kp + row), load slot i
  constexpr int NLD = (EPI == EPI_DG_RELUMASK || kCR) ? NPT : ((kCA || kG16) ? NPT * 2 : 0);
  auto op_load = [&](int kp, int i) __attribute__((always_inline)) {
    const int yy = 4 * kp + row;
    if constexpr (EPI == EPI_DG_RELUMASK) {
      const size_t pix = (size_t)n * HW + (size_t)yy * p.W + x0 + i * 16 + fr;
      ops.t[i] = *reinterpret_cast<const uint4*>(p.aux + pix * p.Cout + cb * 64 + chan(0, 0));
    } else if constexpr (kG16) {  // load i: tile i / 2, g (even) or u (odd), 16 B each
      const int pt = i >> 1;
      const size_t pix = (size_t)n * HW + (size_t)yy * p.W + x0 + pt * 16 + fr;
      const size_t o = pix * p.Cout + cb * 64 + chan(0, 0);
      if (i & 1) ops.uq[pt] = *reinterpret_cast<const uint4*>(p.aux + o);
      else ops.t[pt] = *reinterpret_cast<const uint4*>(p.r1b + o);
    } else if constexpr (kCA) {
      const int pt = i / NCT, c = i % NCT;
      const size_t pix = (size_t)n * HW + (size_t)yy * p.W + x0 + pt * 16 + fr;
      const size_t o = pix * p.Cout + cb * 64 + chan(c, 0);
      ops.g[pt][c] = *reinterpret_cast<const float4*>(p.r1 + o);
      ops.u[pt][c] = *reinterpret_cast<const uint2*>(p.aux + o);
    } else if constexpr (kCR) {  // h: the pair (hi 16 B + lo 8 B) or fp32 (32 B), 8 channels
      const size_t pix = (size_t)n * HW + (size_t)yy * p.W + x0 + i * 16 + fr;
      const size_t o = pix * p.Cout + cb * 64 + chan(0, 0);
      if (p.r1h) {
        ops.t[i] = *reinterpret_cast<const uint4*>(p.r1h + o);
        ops.u[i][0] = *reinterpret_cast<const uint2*>(p.r1l + o);
      } else {
        ops.g[i][0] = *reinterpret_cast<const float4*>(p.r1 + o);
        ops.g[i][1] = *reinterpret_cast<const float4*>(p.r1 + o + 4);
      }
    }
  };
  // epilogue of pixel tile pt of strip kp from accp
  float ps0[NCT][4], ps1[NCT][4];
  auto epi_tile = [&](int kp, int pt) __attribute__((always_inline)) {
    // pin the tile's work to this K-step: without these the IR passes hoist the
    // arithmetic (and the operand waits with it) up to the loads at K-step 0
#pragma unroll
    for (int c = 0; c < NCT; ++c) pin4(accp[pt][c]);
    if constexpr (EPI == EPI_DG_RELUMASK) pin4u(ops.t[pt]);
    if constexpr (kG16) {
      pin4u(ops.t[pt]);
      pin4u(ops.uq[pt]);
    }
    if constexpr (kCR) {
      if (p.r1h) {
        pin4u(ops.t[pt]);
        pin(ops.u[pt][0].x);
        pin(ops.u[pt][0].y);
      } else {
        pin4f(ops.g[pt][0]);
        pin4f(ops.g[pt][1]);
      }
    }
    if constexpr (kCA) {
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        pin4f(ops.g[pt][c]);
        pin(ops.u[pt][c].x);
        pin(ops.u[pt][c].y);
      }
    }
    const int yy = 4 * kp + row;
    const size_t pix = (size_t)n * HW + (size_t)yy * p.W + x0 + pt * 16 + fr;
    if constexpr (kCR) {
      float hv[8];
      if (p.r1h) {
        const uint4 th = ops.t[pt];
        const uint2 tl = ops.u[pt][0];
        const float4 a = pair_decode4(make_uint2(th.x, th.y), tl.x), b = pair_decode4(make_uint2(th.z, th.w), tl.y);
        hv[0] = a.x; hv[1] = a.y; hv[2] = a.z; hv[3] = a.w; hv[4] = b.x; hv[5] = b.y; hv[6] = b.z; hv[7] = b.w;
      } else {
        const float4 a = ops.g[pt][0], b = ops.g[pt][1];
        hv[0] = a.x; hv[1] = a.y; hv[2] = a.z; hv[3] = a.w; hv[4] = b.x; hv[5] = b.y; hv[6] = b.z; hv[7] = b.w;
      }
      float o[8];
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        const f32x4 v = accp[pt][c];
        const float b[4] = {bias[c].x, bias[c].y, bias[c].z, bias[c].w};
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) o[4 * c + rr] = fmaf(v[rr] + b[rr], sv[4 * c + rr], hv[4 * c + rr]);
      }
      uint2 h0, h1;
      const uint32_t l0 = pair_encode4(o[0], o[1], o[2], o[3], h0);
      const uint32_t l1 = pair_encode4(o[4], o[5], o[6], o[7], h1);
      const uint32_t oe = (uint32_t)(pix * p.Cout + cb * 64 + chan(0, 0));
      st_wt16(rph, p.yph, oe * 2, make_uint4(h0.x, h0.y, h1.x, h1.y));
      st_wt8(rpl, p.ypl, oe, make_uint2(l0, l1));
    } else if constexpr (kG16) {
      // g = bf16(acc + g_in): the CA sums take the rounded (stored) value, as conv_epilogue2
      const uint32_t gw[4] = {ops.t[pt].x, ops.t[pt].y, ops.t[pt].z, ops.t[pt].w};
      const uint32_t uw[4] = {ops.uq[pt].x, ops.uq[pt].y, ops.uq[pt].z, ops.uq[pt].w};
      uint32_t ow[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = accp[pt][q >> 1];
        const float a = v[2 * (q & 1)] + bf2f(gw[q] & 0xFFFFu), b = v[2 * (q & 1) + 1] + bf2f(gw[q] >> 16);
        ow[q] = pack2(a, b);
        const float ra = bf2f(ow[q] & 0xFFFFu), rb = bf2f(ow[q] >> 16);
        const int c = q >> 1, r0 = 2 * (q & 1);
        ps0[c][r0] += ra;
        ps0[c][r0 + 1] += rb;
        ps1[c][r0] += ra * bf2f(uw[q] & 0xFFFFu);
        ps1[c][r0 + 1] += rb * bf2f(uw[q] >> 16);
      }
      st_defer(rout, p.yb, (uint32_t)((pix * p.Cout + cb * 64 + chan(0, 0)) * 2), make_uint4(ow[0], ow[1], ow[2], ow[3]));
    } else if constexpr (kPerm) {
      float o[8];
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        const f32x4 v = accp[pt][c];
        const float b[4] = {bias[c].x, bias[c].y, bias[c].z, bias[c].w};
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          float x = v[rr];
          if constexpr (EPI == EPI_RELU_BF16) x = fmaxf(x + b[rr], 0.f);
          if constexpr (EPI == EPI_RELU_POOL) x = fmaxf(x + b[rr], 0.f);  // (summed as bf16 below)
          if constexpr (EPI == EPI_POOL_BF16) {
            x += b[rr];
            ps0[c][rr] += x;
          }
          if constexpr (EPI == EPI_DG_RELUMASK) {
            const uint32_t w = (c ? (rr < 2 ? ops.t[pt].z : ops.t[pt].w) : (rr < 2 ? ops.t[pt].x : ops.t[pt].y));
            x = p.alpha * relu_mask((rr & 1) ? (w >> 16) : (w & 0xFFFFu), x);
          }
          o[4 * c + rr] = x;
        }
      }
      const uint4 val = make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
      if constexpr (EPI == EPI_RELU_POOL) {  // sums of the bf16 t conv2 reads (ca_scale.hpp)
        const uint32_t w[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) ps0[i >> 2][i & 3] += bf2f((i & 1) ? (w[i >> 1] >> 16) : (w[i >> 1] & 0xFFFFu));
      }
      st_defer(rout, p.yb, (uint32_t)((pix * p.Cout + cb * 64 + chan(0, 0)) * 2), val);
    } else {
#pragma unroll
      for (int c = 0; c < NCT; ++c) {
        const f32x4 a = accp[pt][c];
        const float4 gg = ops.g[pt][c];
        const uint2 uu = ops.u[pt][c];
        const float v[4] = {a[0] + gg.x, a[1] + gg.y, a[2] + gg.z, a[3] + gg.w};
        st_defer(rout, p.yf, (uint32_t)((pix * p.Cout + cb * 64 + chan(c, 0)) * 4), make_float4(v[0], v[1], v[2], v[3]));
        ps0[c][0] += v[0]; ps0[c][1] += v[1]; ps0[c][2] += v[2]; ps0[c][3] += v[3];
        ps1[c][0] += v[0] * bf2f(uu.x & 0xFFFFu);
        ps1[c][1] += v[1] * bf2f(uu.x >> 16);
        ps1[c][2] += v[2] * bf2f(uu.y & 0xFFFFu);
        ps1[c][3] += v[3] * bf2f(uu.y >> 16);
      }
    }
  };
  // this wave's row sums of strip kp -> red buffer kp & 1
  auto part_rows = [&](int kp) __attribute__((always_inline)) {
    float* rb = red + (kp & 1) * 512;
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float s0 = sum16(ps0[c][rr]);
        float s1 = 0.f;
        if constexpr (kS1) s1 = sum16(ps1[c][rr]);
        if (fr == 0) {
          rb[(row * 2 + 0) * 64 + chan(c, rr)] = s0;
          if constexpr (kS1) rb[(row * 2 + 1) * 64 + chan(c, rr)] = s1;
        }
      }
  };
  // the 4 rows' sums of strip kp -> the per-strip partial record (published by a barrier)
  auto part_store = [&](int kp) __attribute__((always_inline)) {
    const float* rb = red + (kp & 1) * 512;
    const size_t rec = ((size_t)n * nstrips_all + kp * nsx + sx) * p.part_stride;
    if (tid < 64) {
      p.part[rec + cb * 64 + tid] = rb[tid] + rb[128 + tid] + rb[256 + tid] + rb[384 + tid];
    } else if (kS1 && tid < 128) {
      const int c = tid - 64;
      p.part[rec + 64 + c] = rb[64 + c] + rb[192 + c] + rb[320 + c] + rb[448 + c];
    }
  };
  auto zero_ps = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < NCT; ++c)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) ps0[c][rr] = ps1[c][rr] = 0.f;
  };

  // one strip; PREV: run strip k-1's epilogue inside it; LAST: prefetch strip k's
  // own epilogue operands at its end (the exposed epilogue after the loop reads them)
  auto strip = [&](int k, auto prev_tag, auto last_tag) __attribute__((always_inline)) {
    constexpr bool PREV = decltype(prev_tag)::value;
    constexpr bool LAST = decltype(last_tag)::value;
    const int y = 4 * k + row;
    const bool pf = (k + 1 < k1);
    const bool red_store = kPart && (k - (kImm ? 1 : 2) >= k0) && tid < (kS1 ? 128 : 64);
    [[maybe_unused]] const int sj = 2 + 5 * min(k - k0, 11);
    STAMP(sj);
    uint32_t boff[3][3][2];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int rr = y + ky - 1 + 3;
      const int slot = ((rr >> 2) % 3) * 4 + (rr & 3);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) boff[ky][kx][kk] = swz128(slot * (TW + 2) + fr + kx, kk * 4 + fk);
    }
    f32x4 acc[NPT][NCT];
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PREV) zero_ps();
    bf16x8 A[kFragBuf][NCT], B[kFragBuf][NPT];
    [[maybe_unused]] uint4 gxv[NGW];  // (gx) group k+2's pieces, read one K-step ahead
    auto load_step = [&](int st, bf16x8 (&a)[NCT], bf16x8 (&b)[NPT]) __attribute__((always_inline)) {
      const int tap = st >> 1, kk = st & 1, ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int c = 0; c < NCT; ++c) a[c] = lds_frag(wl, tap * 8192 + aoff[kk][c]);
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) b[pt] = lds_frag(ring, boff[ky][kx][kk] + pt * 2048);
    };
    constexpr int LA = kFragBuf - 1;
#pragma unroll
    for (int st = 0; st < LA; ++st) load_step(st, A[st], B[st]);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      // VMEM issue order in a strip: the deferred epilogue's operand loads (K-steps
      // 0-2), group k+2's DMA (0-3), the deferred stores (K-steps ES..), the
      // previous-but-one strip's partial record (17): the DMA is waited for at the
      // end with a count of the stores behind it
      if constexpr ((PREV || kImm) && NLD > 0) {
        constexpr int PER = (NLD + 2) / 3;
#pragma unroll
        for (int i = 0; i < PER; ++i)
          if (st < 3 && st * PER + i < NLD) op_load(kImm ? k : k - 1, st * PER + i);
      }
      if (st < NGW && pf && wv_s + NW * st < NGRP) group_dma_one(k + 2, st);
      __builtin_amdgcn_sched_barrier(0);
      const bool ld = st + LA < 18;
      if (ld) load_step(st + LA, A[(st + LA) % kFragBuf], B[(st + LA) % kFragBuf]);
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
        for (int c = 0; c < NCT; ++c) acc[pt][c] = mfma16(A[st % kFragBuf][c], B[st % kFragBuf][pt], acc[pt][c]);
      if (ld) {
#pragma unroll
        for (int j = 0; j < NCT + NPT; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (NCT * NPT > NCT + NPT) __builtin_amdgcn_sched_group_barrier(0x008, NCT * NPT - (NCT + NPT), 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PREV) {
        if (st >= ES && st < ES + NPT) epi_tile(k - 1, st - ES);
        if constexpr (kPart)
          if (st == ES + NPT) part_rows(k - 1);
      }
      if constexpr (kPart)
        if (st == 17 && red_store) part_store(kImm ? k - 1 : k - 2);
      if constexpr (EPI == EPI_DG_RELUMASK) {
        // du of group k+2 (gx), one DMA piece per K-step behind that step's MFMAs over the
        // strip's last K-steps, each piece read one K-step ahead: the pieces (issued at
        // K-steps 0-3) have landed once only the deferred stores of K-steps ES.. may still
        // be in flight behind them
        constexpr int GXS = 18 - NGW;
        if (SRMI_GX_INLOOP == 2 && gx && pf && st >= 17 - 2 * NGW) {
          // (variant: a piece every other K-step from K-step 18 - 2 NGW, each read the step
          //  before; the wait at 17 - 2 NGW also takes the deferred epilogue's operands)
          constexpr int G0 = 17 - 2 * NGW;
          const int m = (st - G0) >> 1;
          if (st == G0) wait_vm<0>();
          if (((st - G0) & 1) == 0) {
            if (gx_ok(k + 2, m)) gxv[m < NGW ? m : 0] = *gx_ptr(k + 2, m);
          } else if (gx_ok(k + 2, m)) {
            *gx_ptr(k + 2, m) = du_from_g8(gxv[m < NGW ? m : 0], gxs, gxm);
          }
        }
        if (SRMI_GX_INLOOP == 1 && gx && pf && st >= GXS - 1) {
          if (st == GXS - 1) {
            if constexpr (PREV) wait_vm<NPT>();
            else wait_vm<0>();
            if (gx_ok(k + 2, 0)) gxv[0] = *gx_ptr(k + 2, 0);
          } else {
            const int m = st - GXS;
            if (m + 1 < NGW && gx_ok(k + 2, m + 1)) gxv[m + 1 < NGW ? m + 1 : 0] = *gx_ptr(k + 2, m + 1);
            if (gx_ok(k + 2, m)) *gx_ptr(k + 2, m) = du_from_g8(gxv[m], gxs, gxm);
          }
        }
      }
      if constexpr (LAST && NLD > 0) {
        // the exposed epilogue's operands, behind this strip's last MFMAs
        constexpr int PER = (NLD + 1) / 2;
#pragma unroll
        for (int i = 0; i < PER; ++i)
          if (st >= 16 && (st - 16) * PER + i < NLD) op_load(k, (st - 16) * PER + i);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    STAMP(sj + 1);
    // group k+2 has landed once only this strip's deferred stores (and the partial
    // record) may still be in flight behind it
    constexpr int NST = PREV ? (kCR ? 2 * NPT : (kPerm ? NPT : NPT * NCT)) : 0;
    if constexpr (kImm) {
      // the strip's own epilogue: its operands, group k+2 and the partial record landed
      wait_vm<0>();
#pragma unroll
      for (int i = 0; i < NPT; ++i)
#pragma unroll
        for (int j = 0; j < NCT; ++j) accp[i][j] = acc[i][j];
      zero_ps();
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) epi_tile(k, pt);
      part_rows(k);
    } else if (!pf) {
      // no DMA in this strip: nothing to wait for (the loads of the exposed
      // epilogue are waited for where they are used)
    } else if (red_store) {
      wait_vm<NST + 1>();
    } else {
      wait_vm<NST>();
    }
    if constexpr (EPI == EPI_DG_RELUMASK && !SRMI_GX_INLOOP) {
      if (gx && pf) gx_group(k + 2);  // (its pieces landed: the wait above)
    }
    STAMP(sj + 2);
#ifdef SRMI_STAMPS
    // diagnostic: every wave's arrival at the strip barrier (slots 40 + 8 j + wave, j < 3)
    if (p.stamps && lane == 0 && k - k0 < 3) p.stamps[blockIdx.x * 64 + 40 + 8 * (k - k0) + wave] = __builtin_amdgcn_s_memtime();
#endif
    // every wave is past its reads of group k (ring slot released) and its red[]
    // writes; group k+2 is published
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    STAMP(sj + 3);
    STAMP(sj + 4);
#pragma unroll
    for (int i = 0; i < NPT; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j) accp[i][j] = acc[i][j];
  };
  using T = std::true_type;
  using F = std::false_type;
  if constexpr (kImm) {
#pragma unroll 1
    for (int k = k0; k < k1; ++k) strip(k, F{}, F{});
    part_store(k1 - 1);  // (its rows' sums published by the last strip's barrier)
    STAMP(61);
    return;
  }
  if (k1 - k0 == 1) {
    strip(k0, F{}, T{});
  } else {
    strip(k0, F{}, F{});
#pragma unroll 1
    for (int k = k0 + 1; k < k1 - 1; ++k) strip(k, T{}, F{});
    strip(k1 - 1, T{}, T{});
  }
  // the last strip's epilogue, exposed
  if constexpr (kPart)
    if (k1 - 2 >= k0) part_store(k1 - 2);
  zero_ps();
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) epi_tile(k1 - 1, pt);
  if constexpr (kPart) {
    part_rows(k1 - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    part_store(k1 - 1);
  }
  STAMP(61);
}

template <int TW, int EPI, int NW>
__global__ void __launch_bounds__(NW * 64, 1) conv64_kernel(ConvParams p, int run_len) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv64_body<TW, EPI, NW>(p, run_len, blockIdx.x, smem);
}

// runs of the v2 kernel for a CU budget: ~one workgroup per CU of the budget
inline int conv64_run_len(const ConvParams& p, int TW, int cus) {
  const int nsy = p.H / kTH;
  const int units = (p.Cout / 64) * p.N * (p.W / TW);
  int R = (cus + units / 2) / units;
  R = R < 1 ? 1 : (R > nsy ? nsy : R);
  return (nsy + R - 1) / R;
}
inline int conv64_blocks(const ConvParams& p, int TW, int run_len) {
  const int nsy = p.H / kTH;
  return (p.Cout / 64) * p.N * (p.W / TW) * ((nsy + run_len - 1) / run_len);
}


}  // namespace srmi
