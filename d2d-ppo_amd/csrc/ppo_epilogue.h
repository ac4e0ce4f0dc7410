// PPO loss-gradient epilogue shared by the MLP update kernels (update_kernels.hip) and the GRU
// update kernel (gru_kernels.hip): log-prob, entropy, clipped surrogate and dL/dlogits per sample
// (algorithms/ippo.py:178-217, d2d_ppo.py:183-216).
#pragma once
#include <cmath>

#include "mlp_common.h"

namespace d2d {

constexpr float kEps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps (probs_to_logits clamp)

// dL/dz for one epilogue pass.  Lane (g, i): sample i of its half, actions 4 ga + r (HALF: the
// two 32-lane halves are independent tiles, ga = g & 1; else ga = g).
// Bernoulli (KIND 0, ippo.py:157-160 + 185-189, quirk Q6: softmax probs as Bernoulli probs):
//   logp = mean_c log_prob(a_c) with torch's clamp(p, eps, 1-eps); entropy = mean_c
//   BCEWithLogits(logit(pc), p) = -p log pc - (1-p) log(1-pc).
// Categorical (KIND 1): Categorical(probs) renormalises q = p / sum p; logp = log clamp(q_a);
//   entropy = -sum q log clamp(q).
// Surrogate -min(r W, clamp(r) W) with torch.min's tie rule (each side gets half the gradient,
// so inside [1-eps, 1+eps] the slope is r W) and clamp passing the gradient inclusively.
// SIGMOID (KIND 0 only): the GRU policy's head, p_c = sigmoid(z_c) independently per channel
// (ippo.py:49-50); dL/dz_c = p_c (1 - p_c) dL/dp_c.
// Args: any struct with A, inv_A, clip_lo, clip_hi, beta, scale (UpdArgs, GruArgs).
// AFIX > 0: the action count is known at compile time (the headline A = 8: every lane's four actions
// are real, so the per-action validity selects fold away).
template <int KIND, bool HALF, bool SIGMOID = false, int AFIX = 0, class Args>
__device__ __forceinline__ f32x4 ppo_dz(const Args& a, f32x4 z, uint32_t act, float lo, float W, bool ok, int ga,
                                        float& surr_acc, float& ent_acc) {
  const int A = AFIX > 0 ? AFIX : a.A;
  bool valid[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) valid[r] = 4 * ga + r < A;
  float p[4];
  if constexpr (SIGMOID) {
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = valid[r] ? __builtin_amdgcn_rcpf(1.f + __expf(-z[r])) : 0.f;
  } else {
    float mx = valid[0] ? z[0] : -INFINITY;
#pragma unroll
    for (int r = 1; r < 4; ++r)
      if (valid[r]) mx = fmax_raw(mx, z[r]);  // one v_max_f32 each (mlp_common.h)
    mx = group_max<HALF>(mx);
    float ex[4], sum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ex[r] = valid[r] ? __expf(z[r] - mx) : 0.f;
      sum += ex[r];
    }
    sum = group_sum<HALF>(sum);
    const float inv = __builtin_amdgcn_rcpf(sum);  // v_rcp_f32, 1 ulp (IEEE division: ~10 VALU + branches)
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = ex[r] * inv;
  }
  float gr[4], dsur[4];
  float logp, ent;
  if constexpr (KIND == 0) {
    const uint32_t bits = act >> (4 * ga);
    // log terms in log2 units (hw_log2); ln 2 is folded into the per-sample scales below
    float lsum = 0.f, esum = 0.f, logit[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pc = fminf(fmaxf(p[r], kEps), 1.f - kEps);
      const bool inside = pc == p[r];  // == (p >= eps && p <= 1 - eps): the clamp passes p through
      const float l1 = hw_log2(pc), l0 = hw_log2(1.f - pc);
      const bool bit = (bits >> r) & 1u;
      lsum += valid[r] ? (bit ? l1 : l0) : 0.f;
      esum += valid[r] ? -(p[r] * l1 + (1.f - p[r]) * l0) : 0.f;
      logit[r] = l1 - l0;
      // d log_prob / dp: 1/pc or -1/(1-pc) -- one reciprocal of the selected (signed) denominator
      dsur[r] = (valid[r] && inside) ? __builtin_amdgcn_rcpf(bit ? pc : -(1.f - pc)) : 0.f;
    }
    const float lA = kLn2 * a.inv_A;  // wave-uniform
    logp = group_sum<HALF>(lsum) * lA;
    ent = group_sum<HALF>(esum) * lA;
    const float ratio = __expf(logp - lo);
    const float cr = __builtin_amdgcn_fmed3f(ratio, a.clip_lo, a.clip_hi);  // clamp: one v_med3_f32
    const float s1 = ratio * W, s2 = cr * W;
    const bool gate = (ratio >= a.clip_lo && ratio <= a.clip_hi) || s1 < s2;
    const float coef = gate ? -a.scale * ratio * W * a.inv_A : 0.f;
    const float eb = a.beta * a.scale * lA;  // d(-beta*mean ent)/dp_c = +beta * logit_c / A / B (logit in log2 units)
#pragma unroll
    for (int r = 0; r < 4; ++r) gr[r] = valid[r] ? coef * dsur[r] + eb * logit[r] : 0.f;
    surr_acc += (ok && ga == 0) ? fminf(s1, s2) : 0.f;
    ent_acc += (ok && ga == 0) ? ent : 0.f;
    f32x4 dz;
    if constexpr (SIGMOID) {
#pragma unroll
      for (int r = 0; r < 4; ++r) dz[r] = (ok && valid[r]) ? p[r] * (1.f - p[r]) * gr[r] : 0.f;
      return dz;
    }
    float dot = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) dot += p[r] * gr[r];
    dot = group_sum<HALF>(dot);
#pragma unroll
    for (int r = 0; r < 4; ++r) dz[r] = (ok && valid[r]) ? p[r] * (gr[r] - dot) : 0.f;
    return dz;
  } else {
    const int aid = (int)act;
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) psum += p[r];
    psum = group_sum<HALF>(psum);
    const float ipsum = __builtin_amdgcn_rcpf(psum);
    float q[4], lsel = 0.f, esum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      q[r] = p[r] * ipsum;
      const float qc = fminf(fmaxf(q[r], kEps), 1.f - kEps);
      const bool inside = qc == q[r];  // the clamp passes q through
      const float lq = hw_log2(qc) * kLn2;
      const bool chosen = valid[r] && 4 * ga + r == aid;
      lsel += chosen ? lq : 0.f;
      esum += valid[r] ? q[r] * lq : 0.f;
      const float iqc = __builtin_amdgcn_rcpf(qc);
      dsur[r] = (chosen && inside) ? iqc : 0.f;
      // d(-beta * ent)/dq = beta * (log qc + q * [inside] / qc)
      gr[r] = valid[r] ? (lq + (inside ? q[r] * iqc : 0.f)) : 0.f;
    }
    logp = group_sum<HALF>(lsel);
    ent = -group_sum<HALF>(esum);
    const float ratio = __expf(logp - lo);
    const float cr = __builtin_amdgcn_fmed3f(ratio, a.clip_lo, a.clip_hi);  // clamp: one v_med3_f32
    const float s1 = ratio * W, s2 = cr * W;
    const bool gate = (ratio >= a.clip_lo && ratio <= a.clip_hi) || s1 < s2;
    const float coef = gate ? -a.scale * ratio * W : 0.f;
    const float eb = a.beta * a.scale;
    float gq = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      gr[r] = coef * dsur[r] + eb * gr[r];  // dL/dq
      gq += gr[r] * q[r];
    }
    gq = group_sum<HALF>(gq);
    float dp[4], dot = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dp[r] = valid[r] ? (gr[r] - gq) * ipsum : 0.f;  // through q = p / sum p
      dot += p[r] * dp[r];
    }
    dot = group_sum<HALF>(dot);
    surr_acc += (ok && ga == 0) ? fminf(s1, s2) : 0.f;
    ent_acc += (ok && ga == 0) ? ent : 0.f;
    f32x4 dz;
#pragma unroll
    for (int r = 0; r < 4; ++r) dz[r] = (ok && valid[r]) ? p[r] * (dp[r] - dot) : 0.f;
    return dz;
  }
}

}  // namespace d2d
