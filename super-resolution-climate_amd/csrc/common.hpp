// Shared device helpers for the srmi CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tuning.hpp"

namespace srmi {

typedef uint16_t bf16_t;                                        // raw bf16 bits
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;      // MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;        // 16x16 accumulator
typedef __attribute__((ext_vector_type(4))) short s16x4;        // ds_read_b64_tr_b16 result

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// round-to-nearest-even f32 -> bf16 (v_cvt_pk_bf16_f32 on gfx950; NaN stays NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// storage-type conversions of the two engine modes (bf16 operands / exact fp32)
template <typename T>
__device__ __forceinline__ T from_f32(float v);
template <>
__device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) { return f2bf(v); }
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_t v) { return bf2f(v); }
__device__ __forceinline__ float to_f32(float v) { return v; }

// two floats -> one dword of 2 bf16 (a low): ONE v_cvt_pk_bf16_f32 (the scalar
// form above made the compiler emit 2 converts + 4 shifts/ors per dword)
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// du = bf16(g s + dmh) of 8 bf16 channels (the CALayer backward's du, ca_bwd_du_kernel;
// dmh = dm / HW): one fma per channel, so every producer of du rounds the same value
// (two channels per packed fma: v_pk_fma_f32, the same fma per element)
__device__ __forceinline__ uint4 du_from_g8(uint4 gq, const float (&s)[8], const float (&m)[8]) {
  const uint32_t w[4] = {gq.x, gq.y, gq.z, gq.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 x = {__uint_as_float(w[q] << 16), __uint_as_float(w[q] & 0xFFFF0000u)};
    const f32x2 sv = {s[2 * q], s[2 * q + 1]}, mv = {m[2 * q], m[2 * q + 1]};
    const f32x2 r = __builtin_elementwise_fma(x, sv, mv);
    o[q] = pack2(r.x, r.y);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// The pair: a value as hi = bf16(h) plus an 8-bit remainder lo -- 16 significant bits
// in 3 bytes (the bf16 engine's residual stream inside a residual group).  In the fp32
// bit pattern A = (T << 16) + L of h (bit patterns of one sign are monotonic integers):
//   hi = (A + 0x8000) >> 16      bf16 of h rounded half away from zero (= T + [L >= 2^15])
//   lo = (A >> 8) & 0xFF         byte 1 of A
//   A' = ((hi << 16) | 0x80) + (sext8(lo) << 8)  =  A - (L & 0xFF) + 128
// so the decoded value is h moved by at most 128 fp32 steps of its binade (2^-16
// relative), centred, across binade boundaries too, and bf16_rne(A') == hi exactly (the
// decoded low half is never a tie): the next conv1's operand is the stored hi.  Encode
// and decode are byte permutes, shifts and adds -- no exponent arithmetic (the former
// ldexp form of the same precision cost 2.4 % in C5: DESIGN.md section 3).
__device__ __forceinline__ float4 pair_decode4(uint2 hi, uint32_t lo) {
  const int q0 = (int)(int8_t)(lo & 0xFFu), q1 = (int)(int8_t)((lo >> 8) & 0xFFu);
  const int q2 = (int)(int8_t)((lo >> 16) & 0xFFu), q3 = (int)(int8_t)(lo >> 24);
  return make_float4(__uint_as_float(((hi.x << 16) | 0x80u) + (uint32_t)(q0 << 8)),
                     __uint_as_float(((hi.x & 0xFFFF0000u) | 0x80u) + (uint32_t)(q1 << 8)),
                     __uint_as_float(((hi.y << 16) | 0x80u) + (uint32_t)(q2 << 8)),
                     __uint_as_float(((hi.y & 0xFFFF0000u) | 0x80u) + (uint32_t)(q3 << 8)));
}
__device__ __forceinline__ uint32_t pair_encode4(float a, float b, float c, float d, uint2& hi) {
  const uint32_t A = __float_as_uint(a), B = __float_as_uint(b), C = __float_as_uint(c), D = __float_as_uint(d);
  hi = make_uint2(__builtin_amdgcn_perm(B + 0x8000u, A + 0x8000u, 0x07060302u),
                  __builtin_amdgcn_perm(D + 0x8000u, C + 0x8000u, 0x07060302u));
  // byte 1 of each: [A.1, B.1] and [C.1, D.1] in the low halves, then the two halves
  const uint32_t ab = __builtin_amdgcn_perm(B, A, 0x0C0C0501u), cd = __builtin_amdgcn_perm(D, C, 0x0C0C0501u);
  return ab | (cd << 16);
}

// Write-through (sc1) 16-byte stores.  A kernel's end-of-launch release writes
// back every dirty L2 line before the next dependent kernel starts (MI355X
// kernel boundary: ~1.8 us + dirty bytes / 6 TB/s); stores that write through
// reach memory while the kernel still computes, so the boundary finds nothing
// to flush.  Used for the large outputs (activations, gradient streams, slabs).
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
template <typename T>
__device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t r, void* base, uint32_t byte_off, const T& v) {
  static_assert(sizeof(T) == 16, "16-byte store");
#if SRMI_WT
  (void)base;
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byte_off, 0, 16);
#else
  (void)r;
  *reinterpret_cast<T*>(static_cast<char*>(base) + byte_off) = v;
#endif
}

template <typename T>
__device__ __forceinline__ void st_wt8(__amdgpu_buffer_rsrc_t r, void* base, uint32_t byte_off, const T& v) {
  static_assert(sizeof(T) == 8, "8-byte store");
#if SRMI_WT
  (void)base;
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, byte_off, 0, 16);
#else
  (void)r;
  *reinterpret_cast<T*>(static_cast<char*>(base) + byte_off) = v;
#endif
}

__device__ __forceinline__ void st_wt4(__amdgpu_buffer_rsrc_t r, void* base, uint32_t byte_off, uint32_t v) {
#if SRMI_WT
  (void)base;
  __builtin_amdgcn_raw_buffer_store_b32(v, r, byte_off, 0, 16);
#else
  (void)r;
  *reinterpret_cast<uint32_t*>(static_cast<char*>(base) + byte_off) = v;
#endif
}

// 16-byte chunk swizzle for an LDS image of 128-byte rows (64 bf16 channels per
// pixel/row).  Chunk c of row q lives at slot c ^ (q & 7).  The MFMA operand read is
// a ds_read_b128 of rows q0 + (lane & 15) at chunk c0 + (lane >> 4), served in the
// 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...: with this swizzle every
// group covers 16 distinct 16-B slots of the 256-B bank row for ANY q0 (the 3x3 taps
// shift q0 by one pixel); the earlier c ^ ((q >> 1) & 7) collided 2-way at most
// shifts (25 % of the conv's LDS cycles), see DESIGN.md §3.
__device__ __forceinline__ uint32_t swz128(uint32_t q, uint32_t c) {
  return q * 128u + ((c ^ (q & 7u)) << 4);
}
// swizzle used by the transposed-read (ds_read_b64_tr_b16) images of the wgrad
// kernel: rows q..q+3 and q+8..q+11 of one 32-lane half hit distinct banks.
__device__ __forceinline__ uint32_t swz128t(uint32_t q, uint32_t c) {
  return q * 128u + ((c ^ ((((q >> 1) & 1u) << 1) | (((q >> 3) & 1u) << 2))) << 4);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 lds_frag(const char* lds, uint32_t byte_off) {
  uint4 v = *reinterpret_cast<const uint4*>(lds + byte_off);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ s16x4 lds_tr(const char* lds, uint32_t byte_off) {
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  v4i16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (v4i16 __attribute__((address_space(3)))*)(lds + byte_off));
  return __builtin_bit_cast(s16x4, r);
}

__device__ __forceinline__ bf16x8 cat_tr(s16x4 lo, s16x4 hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// sum over the 16 lanes of a DPP row (lanes sharing lane >> 4), all in VALU:
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror.  Every
// lane ends with the row sum (fixed association order -> deterministic).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float sum16(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// LDS-DMA of 16 bytes per lane: LDS[lds_base + 16*lane] <- *src (wave-uniform
// lds_base).  Issued through inline asm so that hipcc does not treat the in-flight
// DMA as aliasing every later ds_read (it would drain everything with vmcnt(0));
// completion is ordered by the caller's own s_waitcnt vmcnt + barrier
// (cdna_hip_programming.md §5.7: M0 saved/restored inside the statement).
// A pointer (e.g. the address of a __device__ zero page) pinned in SGPRs once.
// Without this the compiler re-loads a global's address from the GOT (s_load)
// after every asm volatile with a "memory" clobber (glds16), and the
// s_waitcnt lgkmcnt(0) for that scalar load also drains every LDS read in flight.
__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

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

__device__ __forceinline__ void glds16_nt(const void* src, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
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

}  // namespace srmi

#define SRMI_CHECK_LAUNCH()                                  \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return -(int)_e;                   \
  } while (0)
