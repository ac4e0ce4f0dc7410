// MFMA / cross-lane helpers shared by the gfx950 MLP kernels (policy_kernels.hip,
// update_kernels.hip): lane-group reductions on permlane16/32 swaps, the exact three-way
// bf16 split of fp32 operands and its MFMA products, mask loads/stores, counted vmcnt waits.
#pragma once
#include "common.h"

namespace d2d {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Exchanges between the four 16-lane groups with the gfx950 lane-swap instructions (VALU; no LDS
// round trip).  permlane16_swap(v, v) returns {rows 0,0,2,2 ; rows 1,1,3,3} of v, permlane32_swap
// {lower half twice ; upper half twice}: the sum / max / or of the pair is the xor-16 / xor-32
// reduction in every lane (same association as v + shfl_xor(v, 16) then + shfl_xor(., 32)), and
// the element on the other side of lane bit 4 / 5 is the partner value.
__device__ __forceinline__ uint32_t fu(float v) { return __float_as_uint(v); }
__device__ __forceinline__ float uf(uint32_t u) { return __uint_as_float(u); }
// HALF: reduce over the two groups of each 32-lane half only (paired epilogue, below)
template <bool HALF, class Op>
__device__ __forceinline__ uint32_t group_reduce(uint32_t v, Op op) {
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const uint32_t s = op(p[0], p[1]);
  if constexpr (HALF) return s;
  const auto q = __builtin_amdgcn_permlane32_swap(s, s, false, false);
  return op(q[0], q[1]);
}
template <bool HALF = false>
__device__ __forceinline__ float group_sum(float v) {
  return uf(group_reduce<HALF>(fu(v), [](uint32_t a, uint32_t b) { return fu(uf(a) + uf(b)); }));
}
// max of two floats as one v_max_f32: fmaxf under the IEEE mode first quiets each operand with a canonicalizing
// v_max_f32 x, x, x (the compiler cannot prove an MFMA result or a lane swap canonical) -- three VALU instead of one.
// The same value for every non-NaN input; a NaN in stays a NaN out.
__device__ __forceinline__ float fmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <bool HALF = false>
__device__ __forceinline__ float group_max(float v) {
  return uf(group_reduce<HALF>(fu(v), [](uint32_t a, uint32_t b) { return fu(fmax_raw(uf(a), uf(b))); }));
}
template <bool HALF = false>
__device__ __forceinline__ uint32_t group_or(uint32_t v) {
  return group_reduce<HALF>(v, [](uint32_t a, uint32_t b) { return a | b; });
}
template <bool HALF = false>
__device__ __forceinline__ int group_min(int v) {
  return (int)group_reduce<HALF>((uint32_t)v, [](uint32_t a, uint32_t b) { return (uint32_t)min((int)a, (int)b); });
}
// value of the lane whose group index differs in bit 0 (xor 16) / bit 1 (xor 32)
__device__ __forceinline__ uint32_t partner16(uint32_t v, int g) {
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return (g & 1) ? p[0] : p[1];
}
__device__ __forceinline__ uint32_t partner32(uint32_t v, int g) {
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (g & 2) ? p[0] : p[1];
}

// XCD-aware block mapping.  MI355X dispatches workgroups round-robin over its 8 XCDs, each with
// its own L2, so in an agent-fast grid (x = agent) the agents of one env chunk -- whose obs rows
// ([env][agent][F] floats) share cache lines -- land on eight different L2s and every line is
// fetched by about two of them.  The remap gives XCD j the j-th contiguous eighth of the
// x-fast block order (a bijection on the first 8 * floor(total / 8) blocks, identity on the
// rest), so an env chunk's agents run on one XCD.  bx, by are wave-uniform.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
  const uint32_t nx = gridDim.x, total = nx * gridDim.y, per = total / 8;
  uint32_t b = blockIdx.x + nx * blockIdx.y;
  if (b < per * 8) b = (b % 8) * per + b / 8;
  bx = (int)(b % nx);
  by = (int)(b / nx);
}

constexpr float kLn2 = 0.693147180559945309f;

// log2 on the hardware instruction (v_log_f32, ~1 ulp in log2).  Every caller passes a clamped
// probability >= eps = 2^-23, far above the denormal range, so the library logf's denormal
// rescaling and extended-precision ln 2 product (12 VALU per call; 8 calls per sample in the PPO
// epilogue, ~90 VALU per 32-sample actor tile) buy nothing: callers sum log2 terms and scale by
// ln 2 once (or multiply each result, where a single log is taken).
__device__ __forceinline__ float hw_log2(float x) { return __builtin_amdgcn_logf(x); }

// relu as one v_max_i32 on the bit pattern (negative floats are negative ints, -0 -> +0);
// fmaxf(x, 0) costs a NaN-quieting canonicalize plus the max under the IEEE mode
__device__ __forceinline__ float relu(float x) { return __int_as_float(max(__float_as_int(x), 0)); }

// channel masks of 1 / 2 / 4 bytes (d2d_mask_bytes): one typed access, no byte loop
__device__ __forceinline__ uint32_t load_mask(const void* base, size_t cell, int mask_bytes) {
  if (mask_bytes == 1) return reinterpret_cast<const uint8_t*>(base)[cell];
  if (mask_bytes == 2) return reinterpret_cast<const uint16_t*>(base)[cell];
  return reinterpret_cast<const uint32_t*>(base)[cell];
}
__device__ __forceinline__ void store_mask(void* base, size_t cell, int mask_bytes, uint32_t v) {
  if (mask_bytes == 1) reinterpret_cast<uint8_t*>(base)[cell] = (uint8_t)v;
  else if (mask_bytes == 2) reinterpret_cast<uint16_t*>(base)[cell] = (uint16_t)v;
  else reinterpret_cast<uint32_t*>(base)[cell] = v;
}

// Compact obs record (D2D_OBS_U8, env kernel's obs_record): byte j (compile-time) of record word w
// as a network input.  m = 0x80 in the bytes that are int8 (the ack columns), 0 in the uint8 ones:
// int8 b = (b ^ 0x80) - 128, so every byte is one v_cvt_f32_ubyte of w ^ m minus a per-lane
// constant (0 or 128, loop-invariant) -- no per-element select.  The record's byte obs_dim holds
// the constant 1 of the layer-1 bias input and the bytes past it are 0, so no column masking either.
__device__ __forceinline__ float rec_byte(uint32_t w, int j, uint32_t m) {
  return (float)(((w ^ m) >> (8 * j)) & 0xFFu) - (float)((m >> (8 * j)) & 0xFFu);
}
// 0x80-per-byte masks of 4 int8 flags (bit r of `bits` -> byte r)
__device__ __forceinline__ uint32_t sign_bytes(uint32_t bits) {
  return ((bits & 1u) << 7) | ((bits & 2u) << 14) | ((bits & 4u) << 21) | ((bits & 8u) << 28);
}

// Exact bf16 split.  Every fp32 operand v is written EXACTLY as v = vh + vm + vl with
// three bf16 parts (8 + 8 + 8 significand bits, truncation split: vh = v with the low 16 bits
// cleared, vm likewise of v - vh, vl = v - vh - vm).  A product w.x is then the sum of the nine
// part products; the six with combined weight >= 2^-16 (hh, hm, mh, hl, mm, lh) are kept, so each
// term is accurate to ~2^-24 relative, i.e. fp32 level, while each v_mfma_f32_16x16x32_bf16
// (16 cycles/SIMD) does the K=32 work of eight v_mfma_f32_16x16x4_f32 (32 cycles each).
// Observations are usually bf16-exact (integer buffer counts, channel / ACK bits): a tile whose
// values all have zero low halves (one ballot) needs only the three weight parts against xh.
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

struct Parts {
  bf16x8 h, m, l;
};

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float ffrom(uint32_t u) { return __uint_as_float(u); }
// bf16 truncations (high halves) of a (low 16 bits of the result) and b (high 16 bits)
__device__ __forceinline__ uint32_t pack_hi(float a, float b) {
  return __builtin_amdgcn_perm(fbits(b), fbits(a), 0x07060302u);
}
__device__ __forceinline__ bf16x8 as_frag(const uint32_t (&u)[4]) {
  u32x4v v = {u[0], u[1], u[2], u[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// exact three-way split of 8 floats into bf16 fragments
__device__ __forceinline__ Parts split3(const float (&v)[8]) {
  uint32_t H[4], M[4], L[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = v[2 * p], b = v[2 * p + 1];
    const float ar = a - ffrom(fbits(a) & 0xFFFF0000u), br = b - ffrom(fbits(b) & 0xFFFF0000u);
    const float al = ar - ffrom(fbits(ar) & 0xFFFF0000u), bl = br - ffrom(fbits(br) & 0xFFFF0000u);
    H[p] = pack_hi(a, b);
    M[p] = pack_hi(ar, br);
    L[p] = pack_hi(al, bl);
  }
  return {as_frag(H), as_frag(M), as_frag(L)};
}

__device__ __forceinline__ f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// acc += W.X for split W and X: the six terms of weight >= 2^-16, smallest first.  X exact in
// bf16 (xm = xl = 0) skips the three terms that would multiply zeros.
__device__ __forceinline__ f32x4 mfma_split(const Parts& w, const Parts& x, bool x_exact, f32x4 acc) {
  if (!x_exact) {
    acc = mfma_bf16(w.h, x.l, acc);
    acc = mfma_bf16(w.m, x.m, acc);
    acc = mfma_bf16(w.h, x.m, acc);
  }
  acc = mfma_bf16(w.l, x.h, acc);
  acc = mfma_bf16(w.m, x.h, acc);
  acc = mfma_bf16(w.h, x.h, acc);
  return acc;
}

// Sum over the 16 lanes of a row (lanes with equal g), result in every lane of the row.
__device__ __forceinline__ float row_sum16(float v) {
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}

// order a wave's LDS writes before its following LDS reads of other lanes' data
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int N_OUTSTANDING>
__device__ __forceinline__ void wait_vmem() {
  static_assert(N_OUTSTANDING < 64, "vmcnt field is 6 bits");
  // vmcnt = N (bits 3:0 and 15:14), expcnt / lgkmcnt at their maxima = no wait on them
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N_OUTSTANDING & 15) | ((N_OUTSTANDING >> 4) << 14));
}

}  // namespace d2d
