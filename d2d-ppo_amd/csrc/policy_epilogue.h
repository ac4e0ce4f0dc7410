// Behaviour-policy epilogue shared by the MLP policy kernel (policy_kernels.hip) and the GRU
// policy kernel (gru_kernels.hip): probabilities -> sampled / deterministic / forced actions,
// log-prob and the stores of one env tile (algorithms/ippo.py:154-176, d2d_ppo.py:159-181).
#pragma once
#include <cmath>

#include "mlp_common.h"

namespace d2d {

struct MlpArgs {
  int E, N, F, H, A, kind, deterministic, envs_per_wave;
  float inv_A;
  uint32_t rng_step;
  const uint32_t* rng_off;  // optional device word added to rng_step (graph replays)
  uint64_t seed, env_base;
  const float *w1, *b1, *w2, *b2, *v1, *c1, *v2, *c2;
  const float* obs;      // [E][N][F]
  const uint8_t* rec;    // D2D_OBS_U8: compact record [E][N][32 KC] instead of obs
  const uint32_t* sgn;   // D2D_OBS_U8: [N][KC] int8-column masks
  const void* forced;   // NULL or comb mask [E][N] / chsel uint8 [E][N]
  void* act_out;         // comb mask [E][N] / chsel uint8 [E][N]
  float* logp_out;       // [N][E]
  float* value_out;      // [N][E] or NULL
  int mask_bytes;
};

constexpr uint32_t kStreamPolicy = 3;
// kModeValue: the split kernel's value-only instantiation (the iPPO critic as its own launch beside the actor:
// policy_kernels.hip, D2D_POLICY_CRITIC_SPLIT)
enum { kModeSample = 0, kModeDeterministic = 1, kModeForced = 2, kModeValue = 3, kModeRuntime = -1 };
// The epilogue takes logits pre-multiplied by log2(e) (folded into W2, b2 by the split kernel) so
// the softmax exponentials are bare v_exp_f32 (exp2, 1 ulp); the relative rounding of the scaled
// logits is ~2^-24, i.e. a log-prob error ~|logit| * 1e-7.
constexpr float kLog2e = 1.4426950408889634f;


// torch.distributions.Bernoulli(probs).log_prob(t) = -BCEWithLogits(logit(clamp(p)), t) with p
// clamped to [eps, 1-eps]: mathematically log(pc) for t = 1 and log(1 - pc) for t = 0.  One
// hardware log (hw_log2: v_log_f32, ~1 ulp in log2, times ln 2) of the selected argument: 1 - pc is exact for
// pc >= 1/2 and within 2^-24 relative below, so the absolute error of the result is ~1e-7 (the
// library logf/log1pf pair costs ~190 instructions per call; parity tolerance is 1e-5 absolute).
__device__ __forceinline__ float bernoulli_logp(float p, bool t) {
  const float eps = 1.1920928955078125e-07f;
  const float pc = fminf(fmaxf(p, eps), 1.f - eps);
  return hw_log2(t ? pc : 1.f - pc) * kLn2;
}

// Input index carried by lane group g at MFMA k-step s.  The k order is permuted so that a
// lane's KS inputs are KS/4 contiguous 4-float chunks of its obs row: [16q + 4g, 16q + 4g + 4).
__device__ __forceinline__ int kidx(int s, int g) { return 16 * (s >> 2) + 4 * g + (s & 3); }

// B operand of the obs tile: lane (g, i) <- X[env][kidx(s, g)], 0 past F / past E.
// Branch-free: every load stays inside the row (indices clamped to F-1 / F-2), the
// out-of-row values are zeroed by a select; even F uses 8-byte loads.
template <int KS>
__device__ __forceinline__ void load_obs_tile(float (&xf)[KS], const float* __restrict__ obs, int env, bool env_ok,
                                              int N, int k, int F, int g) {
  const float* row = obs + ((size_t)(env_ok ? env : 0) * N + k) * F;
  if ((F & 1) == 0) {
#pragma unroll
    for (int q = 0; q < KS / 4; ++q) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int c = 16 * q + 4 * g + 2 * m;
        const float2 v = *reinterpret_cast<const float2*>(row + min(c, F - 2));
        xf[4 * q + 2 * m] = (env_ok && c < F) ? v.x : 0.f;
        xf[4 * q + 2 * m + 1] = (env_ok && c + 1 < F) ? v.y : 0.f;
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int c = kidx(s, g);
      const float v = row[min(c, F - 1)];
      xf[s] = (env_ok && c < F) ? v : 0.f;
    }
  }
}


// The Philox block policy_epilogue draws in sample mode for (env, agent k, action group ga) -- KIND 1 draws
// group 0's block in every lane
template <int KIND>
__device__ __forceinline__ u32x4 policy_rng_block(const MlpArgs& a, int env, bool env_ok, int k, int ga, uint32_t rng) {
  const uint32_t genv = (uint32_t)(a.env_base + (uint64_t)(env_ok ? env : 0));
  return philox(genv, (uint32_t)k, rng, (kStreamPolicy << 24) | (KIND == 0 ? (uint32_t)ga : 0u), a.seed);
}

// Softmax over the A action logits of env i (action group ga holds actions 4ga..4ga+3 in lg),
// sampling / forced / deterministic actions, log-prob and the stores (ippo.py:154-176).
// HALF (A <= 8): each 32-lane half is its own env tile -- lanes 0-31 one tile, lanes 32-63 the
// next -- with action group ga = g & 1, so one pass serves two tiles; the Philox counter is
// (env, agent, step, stream 3 | ga) either way, so the random stream does not depend on it.
// MODE: kModeSample / kModeDeterministic / kModeForced as a compile-time constant (the split
// kernel: no forced-mask load exists in the sampling kernel, so nothing in it can drain the obs
// prefetch), or kModeRuntime (tested per launch from a.forced / a.deterministic).
// PRE (forced mode): the forced mask / id was loaded ahead by the caller and arrives in `fpre`
// (the split kernel's paired epilogue); otherwise the epilogue loads it itself.
// RNG (sample mode): the lane's Philox block drawn ahead by the caller and passed in `rpre` -- the split
// kernel draws it before its tile MFMAs so that the ten dependent rounds (20 v_mad_u64_u32) fill the MFMA issue
// gaps instead of running as a serial chain after them; the same counter and key, so the same words.
// AF != 0: the action count as a compile-time constant (a.A == AF; the split kernel's A = 8 instantiation, the
// combinatorial envs' 8 channels): no per-action range selects
template <int KIND, bool CRITIC, bool HALF = false, int MODE = kModeRuntime, bool PRE = false, bool SIGMOID = false,
          bool RNG = false, int AF = 0>
__device__ __forceinline__ void policy_epilogue(const MlpArgs& a, f32x4 lg, float value, int env, bool env_ok,
                                                int k, int g, uint32_t rng, uint32_t fpre = 0, u32x4 rpre = {}) {
  const int N = a.N, A = AF ? AF : a.A;
  constexpr bool critic = CRITIC;
  const int ga = HALF ? (g & 1) : g;
  const bool forced = MODE == kModeRuntime ? a.forced != nullptr : MODE == kModeForced;
  const bool deterministic = MODE == kModeRuntime ? a.deterministic != 0 : MODE == kModeDeterministic;
  float p[4];
  if constexpr (SIGMOID) {
    // independent sigmoid per output (the GRU policy's combinatorial head, ippo.py:49-50):
    // p = 1 / (1 + 2^-lg) with lg = logit * log2(e)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      p[r] = (4 * ga + r < A) ? __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-lg[r])) : 0.f;
  } else {
    // ---- softmax over the A actions of env i (lane group g holds actions 4g..4g+3)
    float mx = 4 * ga < A ? lg[0] : -INFINITY;
#pragma unroll
    for (int r = 1; r < 4; ++r)
      if (4 * ga + r < A) mx = fmax_raw(mx, lg[r]);
    mx = group_max<HALF>(mx);
    float ex[4], sum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ex[r] = (4 * ga + r < A) ? __builtin_amdgcn_exp2f(lg[r] - mx) : 0.f;  // v_exp_f32, 1 ulp
      sum += ex[r];
    }
    sum = group_sum<HALF>(sum);
    const float inv = __builtin_amdgcn_rcpf(sum);  // 1 ulp
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = ex[r] * inv;
  }

  const size_t cell = (size_t)env * N + k;
  const uint32_t genv = (uint32_t)(a.env_base + (uint64_t)(env_ok ? env : 0));
  float lp;
  uint32_t out_bits = 0;
  int out_id = 0;
  if constexpr (KIND == 0) {
    // ---- Bernoulli per channel (combinatorial): u < p, one Philox block per lane group
    // bit r of `taken` = action 4g + r.  An in-epilogue forced-mask load (PRE false) is waited for
    // with vmcnt(0), which also drains any obs prefetch in flight; the split kernel's paired
    // epilogue therefore takes the mask preloaded (PRE).
    uint32_t taken = 0;
    if (forced) {
      taken = ((PRE ? fpre : load_mask(a.forced, env_ok ? cell : 0, a.mask_bytes)) >> (4 * ga)) & 0xFu;
    } else if (deterministic) {
#pragma unroll
      for (int r = 0; r < 4; ++r) taken |= (uint32_t)(p[r] > 0.5f) << r;  // dist.probs > 0.5 (ippo.py:166)
    } else {
      const u32x4 rr = RNG ? rpre : philox(genv, (uint32_t)k, rng, (kStreamPolicy << 24) | (uint32_t)ga, a.seed);
#pragma unroll
      for (int r = 0; r < 4; ++r) taken |= (uint32_t)((float)(pick(rr, r) >> 8) * (1.f / 16777216.f) < p[r]) << r;
    }
    float lsum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int act = 4 * ga + r;
      const bool bit = act < A && ((taken >> r) & 1u);
      out_bits |= (uint32_t)bit << act;
      const float l = bernoulli_logp(p[r], bit);
      lsum += act < A ? l : 0.f;
    }
    lsum = group_sum<HALF>(lsum);
    lp = lsum * (AF ? 1.f / (float)AF : a.inv_A);  // log_prob(action).mean(-1)
    out_bits = group_or<HALF>(out_bits);
  } else {
    // ---- Categorical over A ids (channel selection): Categorical(probs) renormalises, log of
    // the clamped probability; sampling by inverse CDF of one Philox uniform; argmax when deterministic
    const float eps = 1.1920928955078125e-07f;
    float psum = p[0] + p[1] + p[2] + p[3];
    float tot = psum;
    tot = group_sum<HALF>(tot);
    int chosen = 0;
    if (forced) {
      chosen = PRE ? (int)fpre : env_ok ? reinterpret_cast<const unsigned char*>(a.forced)[cell] : 0;
    } else if (deterministic) {
      // first index of the maximum (torch.argmax)
      float bv = -INFINITY;
      int bi = A;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * ga + r < A && p[r] > bv) { bv = p[r]; bi = 4 * ga + r; }
#pragma unroll
      for (int m = 16; m <= (HALF ? 16 : 32); m <<= 1) {
        const float ov = uf(m == 16 ? partner16(fu(bv), g) : partner32(fu(bv), g));
        const int oi = (int)(m == 16 ? partner16((uint32_t)bi, g) : partner32((uint32_t)bi, g));
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      chosen = bi;
    } else {
      // prefix over lane groups: exclusive sum of psum for groups < g
      const u32x4 rr = RNG ? rpre : philox(genv, (uint32_t)k, rng, (kStreamPolicy << 24), a.seed);
      const float u = (float)(rr.x >> 8) * (1.f / 16777216.f) * tot;
      const float s16 = uf(partner16(fu(psum), g));  // partner in pair (g ^ 1)
      const float pair = psum + s16;
      float before = 0.f;
      if constexpr (!HALF) {
        const float s32 = uf(partner32(fu(pair), g));
        if (g & 2) before += s32;
      }
      if (g & 1) before += s16;
      int pick_id = A;  // A = "not in my group"
      float c = before;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (4 * ga + r < A && pick_id == A) {
          c += p[r];
          if (u < c) pick_id = 4 * ga + r;
        }
      }
      int best = pick_id;
      best = group_min<HALF>(best);
      chosen = best < A ? best : A - 1;  // rounding at the very top of the CDF
    }
    float lpv = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * ga + r == chosen) lpv = hw_log2(fminf(fmaxf(p[r] * __builtin_amdgcn_rcpf(tot), eps), 1.f - eps)) * kLn2;
    lpv = group_sum<HALF>(lpv);
    lp = lpv;
    out_id = chosen;
  }
  if (env_ok && ga == 0) {
    // forced mode with act_out NULL: the actions are the caller's input, nothing to store
    if (!forced || a.act_out) {
      if constexpr (KIND == 0) {
        store_mask(a.act_out, cell, a.mask_bytes, out_bits);
      } else {
        reinterpret_cast<unsigned char*>(a.act_out)[cell] = (unsigned char)out_id;
      }
    }
    a.logp_out[(size_t)k * a.E + env] = lp;
    if (critic && a.value_out) a.value_out[(size_t)k * a.E + env] = value;
  }
}

}  // namespace d2d
