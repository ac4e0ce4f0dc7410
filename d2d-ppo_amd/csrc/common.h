// Shared device/host helpers for the gfx950 kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "d2d_hip.h"

namespace d2d {

constexpr int kWave = 64;  // CDNA wavefront: every ballot below is 64-bit

enum : uint32_t { kStreamFlip = 0, kStreamArrival = 1, kStreamAction = 2, kPerEnv = 0xFFFFFFFFu };

struct u32x4 {
  uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11); identical to oracle/philox.py and
// oracle/c/d2d_oracle.c, pinned to the Random123 known-answer vectors.
__device__ __forceinline__ u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    // one 32x32->64 multiply per product (v_mad_u64_u32) gives both halves
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
#ifndef D2D_PHILOX_XOR3
#define D2D_PHILOX_XOR3 1
#endif
#if D2D_PHILOX_XOR3
    // three-input xor in one v_bitop3_b32 (the compiler emits two v_xor_b32; the key words are
    // kernel-argument uniform, hence SGPR operands): comb step 65.4 -> 62.7 us at 64 x 8 x 65,536
    uint32_t n0, n2;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"((uint32_t)(p1 >> 32)), "v"(c1), "s"(k0));
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"((uint32_t)(p0 >> 32)), "v"(c3), "s"(k1));
#else
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
#endif
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
  }
  return {c0, c1, c2, c3};
}

__device__ __forceinline__ uint32_t pick(const u32x4& r, int i) {
  return i == 0 ? r.x : (i == 1 ? r.y : (i == 2 ? r.z : r.w));
}

// Poisson(lam) draw of word r: the sequential CDF inversion "x = 0, p = F = exp(-lam); while
// u >= F and x < 255: x += 1, p = p * lam / x, F += p" of u = r * 2^-32 (capped at 255, the uint8
// buffer cells), evaluated as a search of the agent's precomputed thresholds
// t[x] = ceil(F_x * 2^32) - 1 (d2d_env_desc.poisson_cdf, built on the host in the same IEEE double
// order): u >= F_x <=> r > t[x], t is nondecreasing and t[255] = 2^32 - 1, so the result is the
// count of leading entries below r -- bitwise the division loop, at four compares per 16-byte load
// instead of a double division per step.
__device__ __forceinline__ uint32_t poisson_lookup(uint32_t r, const uint32_t* __restrict__ t) {
  uint32_t x = 0;
  for (;;) {
    const uint4 q = *reinterpret_cast<const uint4*>(t + x);
    const uint32_t n = (uint32_t)(r > q.x) + (uint32_t)(r > q.y) + (uint32_t)(r > q.z) + (uint32_t)(r > q.w);
    x += n;
    if (n < 4u) return x;
  }
}

}  // namespace d2d

// thread-local last-error string for the C ABI
void d2d_set_error(const char* fmt, ...);

#define D2D_CHECK_HIP(expr)                                                    \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      d2d_set_error("%s: %s", #expr, hipGetErrorString(_e));                   \
      return D2D_EHIP;                                                         \
    }                                                                          \
  } while (0)

// obs_format of a d2d_mlp_desc / d2d_gru_desc: the obs argument as fp32 rows (f32) or as the
// env kernel's compact record (rec, with the int8-column masks sgn); exactly one is set
inline int obs_format_args(int32_t format, const uint32_t* sgn_in, int32_t obs_dim, const void* obs, const float*& f32,
                           const uint8_t*& rec, const uint32_t*& sgn) {
  f32 = nullptr; rec = nullptr; sgn = nullptr;
  if (format == D2D_OBS_F32) { f32 = static_cast<const float*>(obs); return D2D_OK; }
  if (format != D2D_OBS_U8) { d2d_set_error("unknown obs_format %d", format); return D2D_EINVAL; }
  if (!sgn_in) { d2d_set_error("obs_format D2D_OBS_U8 needs obs_signed"); return D2D_EINVAL; }
  if (reinterpret_cast<uintptr_t>(obs) & 15) { d2d_set_error("the obs record must be 16-byte aligned"); return D2D_EINVAL; }
  (void)obs_dim;
  rec = static_cast<const uint8_t*>(obs); sgn = sgn_in;
  return D2D_OK;
}
