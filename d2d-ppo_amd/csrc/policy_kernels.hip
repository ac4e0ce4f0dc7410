// Fused behaviour-policy slot for the MLP learners on gfx950 (fp32 MFMA).
//
// Replaces, for every agent of every env in one launch, the reference's
// per-agent batch-1 calls in create_rollouts / test
//   Policy.forward + Value.forward   /root/reference/algorithms/ippo.py:54-90
//   PPO.select_action                ippo.py:154-176 (d2d_ppo.py:159-181)
// i.e. relu(W1 x + b1) -> W2 h + b2 -> softmax -> Bernoulli per channel
// (combinatorial; softmax-as-Bernoulli quirk Q6) or Categorical (channel
// selection) -> log-prob (mean over channels for Bernoulli) -> action
// mask / id, plus the iPPO critic relu(V1 x + c1) -> V2 h + c2.
//
// Mapping: workgroup = one agent k x a chunk of envs; each wave owns 16-env
// tiles.  Layer 1 is computed TRANSPOSED, H^T[hidden][env] = W1 . X^T, with
// v_mfma_f32_16x16x4_f32 (A = W1 fragment, register-resident for the whole
// workgroup; B = the obs tile).  Its accumulator has the env on the lane and
// 4 hidden rows per lane in registers, which is exactly a B operand of the
// next MFMA when the k order is permuted (step (t, r) <-> hidden 16t+4g+r):
// actor layer 2 is 16 more MFMAs with no data movement; the critic's 64->1
// layer is a per-lane dot product + 2 cross-group shuffles.  fp32 MFMA is an
// exact k-ordered fmaf chain, so results match the torch fp32 reference to
// ~1e-6 (parity tests use 1e-5).
#include <cmath>

#include "common.h"

namespace d2d {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct MlpArgs {
  int E, N, F, H, A, kind, deterministic, envs_per_wave;
  uint32_t rng_step;
  uint64_t seed, env_base;
  const float *w1, *b1, *w2, *b2, *v1, *c1, *v2, *c2;
  const float* obs;      // [E][N][F]
  const void* forced;    // NULL or comb mask [E][N] / chsel uint8 [E][N]
  void* act_out;         // comb mask [E][N] / chsel uint8 [E][N]
  float* logp_out;       // [N][E]
  float* value_out;      // [N][E] or NULL
  int mask_bytes;
};

constexpr uint32_t kStreamPolicy = 3;

__device__ __forceinline__ float shfl_xor_f(float v, int m) { return __shfl_xor(v, m, 64); }

// torch.distributions.Bernoulli(probs).log_prob(t) = -BCEWithLogits(logit(clamp(p)), t) with p
// clamped to [eps, 1-eps]: mathematically log(pc) for t = 1 and log1p(-pc) for t = 0, which is
// what is evaluated here (one transcendental instead of four; agrees to ~1e-7 relative).
__device__ __forceinline__ float bernoulli_logp(float p, bool t) {
  const float eps = 1.1920928955078125e-07f;
  const float pc = fminf(fmaxf(p, eps), 1.f - eps);
  return t ? logf(pc) : log1pf(-pc);
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

// KS = input k-steps of 4 (F <= 4*KS), HT = hidden tiles of 16 (H <= 16*HT),
// KIND 0 Bernoulli / 1 Categorical, CRITIC: iPPO per-agent critic present
template <int KS, int HT, int KIND, bool CRITIC>
__global__ __launch_bounds__(256) void policy_mlp_kernel(MlpArgs a) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;   // lane group: k-slot of A/B operands, row group of C/D
  const int i = lane & 15;   // row of A / column of B, C/D (the env of the tile)
  const int k = blockIdx.x;  // agent (fast grid axis: all agents of an env chunk run together)
  const int wave = threadIdx.x >> 6;
  const int N = a.N, F = a.F, H = a.H, A = a.A;
  constexpr bool critic = CRITIC;

  // ---- register-resident weight fragments of agent k
  float w1f[HT][KS], v1f[HT][KS], w2f[HT][4], v2f[HT][4];
  f32x4 b1i[HT], c1i[HT];
  const float* W1 = a.w1 + (size_t)k * H * F;
  const float* V1 = critic ? a.v1 + (size_t)k * H * F : nullptr;
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    const int hrow = 16 * t + i;  // A row = hidden unit
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int kk = kidx(s, g);
      const bool ok = hrow < H && kk < F;
      w1f[t][s] = ok ? W1[(size_t)hrow * F + kk] : 0.f;
      v1f[t][s] = (ok && critic) ? V1[(size_t)hrow * F + kk] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hid = 16 * t + 4 * g + r;  // hidden unit held in accumulator register r
      const bool hok = hid < H;
      b1i[t][r] = hok ? a.b1[(size_t)k * H + hid] : 0.f;
      c1i[t][r] = (hok && critic) ? a.c1[(size_t)k * H + hid] : 0.f;
      // actor layer 2 A operand: row = action i, k-slot g <-> hidden 16t+4g+r (step (t, r))
      w2f[t][r] = (hok && i < A) ? a.w2[((size_t)k * A + i) * H + hid] : 0.f;
      v2f[t][r] = (hok && critic) ? a.v2[(size_t)k * H + hid] : 0.f;
    }
  }
  f32x4 b2i;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int act = 4 * g + r;
    b2i[r] = act < A ? a.b2[(size_t)k * A + act] : 0.f;
  }
  const float c2 = critic ? a.c2[k] : 0.f;

  const int tiles = a.envs_per_wave / 16;
  const int wave_env0 = (blockIdx.y * (blockDim.x >> 6) + wave) * a.envs_per_wave;
  float xnext[KS];
  load_obs_tile<KS>(xnext, a.obs, wave_env0 + i, wave_env0 + i < a.E, N, k, F, g);
  for (int tt = 0; tt < tiles; ++tt) {
    const int e0 = wave_env0 + tt * 16;
    if (e0 >= a.E) break;  // wave-uniform
    const int env = e0 + i;
    const bool env_ok = env < a.E;
    float xf[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) xf[s] = xnext[s];
    // prefetch the next tile's obs while this one computes
    if (tt + 1 < tiles) load_obs_tile<KS>(xnext, a.obs, env + 16, env + 16 < a.E, N, k, F, g);
    // ---- layer 1 (actor, critic): H^T = W1 . X^T, bias as the initial accumulator
    f32x4 ha[HT], hv[HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      ha[t] = b1i[t];
      hv[t] = c1i[t];
#pragma unroll
      for (int s = 0; s < KS; ++s) ha[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1f[t][s], xf[s], ha[t], 0, 0, 0);
      if (critic) {
#pragma unroll
        for (int s = 0; s < KS; ++s) hv[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(v1f[t][s], xf[s], hv[t], 0, 0, 0);
      }
    }
    // ---- actor layer 2: logits^T = W2 . relu(H^T), accumulator registers used as B directly
    f32x4 lg = b2i;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        lg = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[t][r], fmaxf(ha[t][r], 0.f), lg, 0, 0, 0);
    }
    // ---- critic layer 2 on VALU: per-lane partial dot + reduction over the 4 lane groups
    float value = 0.f;
    if (critic) {
      float pv = 0.f;
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) pv += fmaxf(hv[t][r], 0.f) * v2f[t][r];
      pv += shfl_xor_f(pv, 16);
      pv += shfl_xor_f(pv, 32);
      value = pv + c2;
    }
    // ---- softmax over the A actions of env i (lane group g holds actions 4g..4g+3)
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * g + r < A) mx = fmaxf(mx, lg[r]);
    mx = fmaxf(mx, shfl_xor_f(mx, 16));
    mx = fmaxf(mx, shfl_xor_f(mx, 32));
    float ex[4], sum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ex[r] = (4 * g + r < A) ? expf(lg[r] - mx) : 0.f;
      sum += ex[r];
    }
    sum += shfl_xor_f(sum, 16);
    sum += shfl_xor_f(sum, 32);
    float p[4];
    const float inv = 1.f / sum;
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = ex[r] * inv;

    const size_t cell = (size_t)env * N + k;
    const uint32_t genv = (uint32_t)(a.env_base + (uint64_t)(env_ok ? env : 0));
    float lp;
    uint32_t out_bits = 0;
    int out_id = 0;
    if constexpr (KIND == 0) {
      // ---- Bernoulli per channel (combinatorial): u < p, one Philox block per lane group
      uint32_t forced_bits = 0;
      if (a.forced && env_ok) {
        const unsigned char* fb = reinterpret_cast<const unsigned char*>(a.forced) + cell * a.mask_bytes;
        for (int b = 0; b < a.mask_bytes; ++b) forced_bits |= (uint32_t)fb[b] << (8 * b);
      }
      u32x4 rr = {0, 0, 0, 0};
      if (!a.forced && !a.deterministic)
        rr = philox(genv, (uint32_t)k, a.rng_step, (kStreamPolicy << 24) | (uint32_t)g, a.seed);
      float lsum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int act = 4 * g + r;
        if (act < A) {
          bool bit;
          if (a.forced) bit = (forced_bits >> act) & 1u;
          else if (a.deterministic) bit = p[r] > 0.5f;  // dist.probs > 0.5 (ippo.py:166)
          else bit = (float)(pick(rr, r) >> 8) * (1.f / 16777216.f) < p[r];
          out_bits |= (uint32_t)bit << act;
          lsum += bernoulli_logp(p[r], bit);
        }
      }
      lsum += shfl_xor_f(lsum, 16);
      lsum += shfl_xor_f(lsum, 32);
      lp = lsum / (float)A;  // log_prob(action).mean(-1)
      out_bits |= (uint32_t)__shfl_xor((int)out_bits, 16, 64);
      out_bits |= (uint32_t)__shfl_xor((int)out_bits, 32, 64);
    } else {
      // ---- Categorical over A ids (channel selection): Categorical(probs) renormalises, log of
      // the clamped probability; sampling by inverse CDF of one Philox uniform; argmax when deterministic
      const float eps = 1.1920928955078125e-07f;
      float psum = p[0] + p[1] + p[2] + p[3];
      float tot = psum;
      tot += shfl_xor_f(tot, 16);
      tot += shfl_xor_f(tot, 32);
      int chosen = 0;
      if (a.forced) {
        chosen = env_ok ? reinterpret_cast<const unsigned char*>(a.forced)[cell] : 0;
      } else if (a.deterministic) {
        // first index of the maximum (torch.argmax)
        float bv = -INFINITY;
        int bi = A;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * g + r < A && p[r] > bv) { bv = p[r]; bi = 4 * g + r; }
#pragma unroll
        for (int m = 16; m <= 32; m <<= 1) {
          const float ov = shfl_xor_f(bv, m);
          const int oi = __shfl_xor(bi, m, 64);
          if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        chosen = bi;
      } else {
        // prefix over lane groups: exclusive sum of psum for groups < g
        const u32x4 rr = philox(genv, (uint32_t)k, a.rng_step, (kStreamPolicy << 24), a.seed);
        const float u = (float)(rr.x >> 8) * (1.f / 16777216.f) * tot;
        const float s16 = __shfl_xor(psum, 16, 64);  // partner in pair (g ^ 1)
        const float pair = psum + s16;
        const float s32 = __shfl_xor(pair, 32, 64);
        float before = 0.f;
        if (g & 2) before += s32;
        if (g & 1) before += s16;
        int pick_id = A;  // A = "not in my group"
        float c = before;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (4 * g + r < A && pick_id == A) {
            c += p[r];
            if (u < c) pick_id = 4 * g + r;
          }
        }
        int best = pick_id;
        best = min(best, __shfl_xor(best, 16, 64));
        best = min(best, __shfl_xor(best, 32, 64));
        chosen = best < A ? best : A - 1;  // rounding at the very top of the CDF
      }
      float lpv = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r == chosen) lpv = logf(fminf(fmaxf(p[r] / tot, eps), 1.f - eps));
      lpv += shfl_xor_f(lpv, 16);
      lpv += shfl_xor_f(lpv, 32);
      lp = lpv;
      out_id = chosen;
    }
    if (env_ok && g == 0) {
      if constexpr (KIND == 0) {
        unsigned char* ob = reinterpret_cast<unsigned char*>(a.act_out) + cell * a.mask_bytes;
        for (int b = 0; b < a.mask_bytes; ++b) ob[b] = (unsigned char)(out_bits >> (8 * b));
      } else {
        reinterpret_cast<unsigned char*>(a.act_out)[cell] = (unsigned char)out_id;
      }
      a.logp_out[(size_t)k * a.E + env] = lp;
      if (critic && a.value_out) a.value_out[(size_t)k * a.E + env] = value;
    }
  }
}

}  // namespace d2d

using namespace d2d;

template <int KS, int HT>
static int launch_policy(const MlpArgs& a, hipStream_t s) {
  const int waves = 4;
  const int envs_per_block = waves * a.envs_per_wave;
  dim3 grid(a.N, (a.E + envs_per_block - 1) / envs_per_block);
  const bool critic = a.v1 != nullptr;
  if (a.kind == 0 && critic) hipLaunchKernelGGL((policy_mlp_kernel<KS, HT, 0, true>), grid, dim3(64 * waves), 0, s, a);
  else if (a.kind == 0) hipLaunchKernelGGL((policy_mlp_kernel<KS, HT, 0, false>), grid, dim3(64 * waves), 0, s, a);
  else if (critic) hipLaunchKernelGGL((policy_mlp_kernel<KS, HT, 1, true>), grid, dim3(64 * waves), 0, s, a);
  else hipLaunchKernelGGL((policy_mlp_kernel<KS, HT, 1, false>), grid, dim3(64 * waves), 0, s, a);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_policy_mlp_step(const d2d_mlp_desc* d, const float* obs, const void* forced, uint32_t rng_step,
                                   int32_t deterministic, void* actions, float* logp, float* value, void* stream) {
  if (!d || !obs || !actions || !logp || !d->w1 || !d->b1 || !d->w2 || !d->b2) {
    d2d_set_error("d2d_policy_mlp_step: NULL argument");
    return D2D_EINVAL;
  }
  if (d->kind != 0 && d->kind != 1) { d2d_set_error("kind must be 0 (Bernoulli) or 1 (Categorical)"); return D2D_EINVAL; }
  if (d->n_out < 1 || d->n_out > 16) { d2d_set_error("n_out=%d outside [1,16]", d->n_out); return D2D_EUNSUPPORTED; }
  if (d->hidden < 1 || d->hidden > 64) { d2d_set_error("hidden=%d outside [1,64]", d->hidden); return D2D_EUNSUPPORTED; }
  if (d->obs_dim < 1 || d->obs_dim > 64) { d2d_set_error("obs_dim=%d outside [1,64]", d->obs_dim); return D2D_EUNSUPPORTED; }
  if (d->kind == 0 && d->n_out > 32) { d2d_set_error("too many channels"); return D2D_EUNSUPPORTED; }
  if (d->v1 && (!d->c1 || !d->v2 || !d->c2)) { d2d_set_error("critic needs v1, c1, v2, c2"); return D2D_EINVAL; }
  MlpArgs a;
  a.E = d->n_envs; a.N = d->n_agents; a.F = d->obs_dim; a.H = d->hidden; a.A = d->n_out; a.kind = d->kind;
  a.deterministic = deterministic ? 1 : 0;
  a.envs_per_wave = 256;
  a.rng_step = rng_step; a.seed = d->seed; a.env_base = d->env_base;
  a.w1 = d->w1; a.b1 = d->b1; a.w2 = d->w2; a.b2 = d->b2; a.v1 = d->v1; a.c1 = d->c1; a.v2 = d->v2; a.c2 = d->c2;
  a.obs = obs; a.forced = forced; a.act_out = actions; a.logp_out = logp; a.value_out = value;
  a.mask_bytes = d->n_out <= 8 ? 1 : d->n_out <= 16 ? 2 : 4;
  if (a.E == 0 || a.N == 0) return D2D_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ks = (a.F + 3) / 4;
  const int ht = (a.H + 15) / 16;
  if (ks <= 8) {
    if (ht <= 2) return launch_policy<8, 2>(a, s);
    return launch_policy<8, 4>(a, s);
  }
  if (ht <= 2) return launch_policy<16, 2>(a, s);
  return launch_policy<16, 4>(a, s);
}
