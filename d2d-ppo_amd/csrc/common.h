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
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
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

// Poisson(lam) by sequential CDF inversion of u = r * 2^-32, capped at 255
// (uint8 buffer cells).  Same IEEE double op order as the oracles; built with
// -ffp-contract=off so no FMA changes the rounding.
__device__ __forceinline__ uint32_t poisson_inv(uint32_t r, double lam, double p0) {
  const double u = (double)r * (1.0 / 4294967296.0);
  double p = p0, F = p;
  uint32_t x = 0;
  while (u >= F && x < 255u) {
    x += 1u;
    p = (p * lam) / (double)x;
    F = F + p;
  }
  return x;
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
