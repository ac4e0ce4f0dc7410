// Fused PPO update (gradients) for the MLP learners on gfx950.
//
// Replaces, for all N agents at once, the backward passes of
//   iPPO  PPO.train_step        /root/reference/algorithms/ippo.py:194-217
//         (clipped surrogate + 0.01 entropy bonus -> policy Adam; MSE -> value Adam)
//   D2D   PPO.train_step        /root/reference/algorithms/d2d_ppo.py:198-216
//         (the same surrogate with the per-sample multiplier M and beta_entropy)
// i.e. evaluate() (ippo.py:178-191) + loss + loss.backward() for the per-agent networks
//   Policy  Linear(F,H) -> ReLU -> Linear(H,A) -> softmax   (ippo.py:54-75)
//   Value   Linear(F,H) -> ReLU -> Linear(H,1)             (ippo.py:78-90)
// over every rollout sample.  Output: the gradient of each agent's loss w.r.t. its
// parameters (the values torch autograd leaves in .grad) plus the loss sums; the optimizer
// step (Adam, grad clipping, the cross-rank all-reduce) stays with the caller.
//
// Sample tile = 32 consecutive envs of one rollout slot t for one agent k (obs read straight
// from the rollout buffer [T][E][N][F]).  Two 16-sample halves s = 0, 1 of a tile.  Operand
// conventions of v_mfma_f32_16x16x32_bf16 (lane = (g, i), g = lane >> 4, i = lane & 15): A and B
// fragments hold row / column i and k-slots 8g .. 8g+7; the accumulator holds column i and rows
// 4g .. 4g+3.  A GEMM whose contracted index is the rows of the previous accumulator can
// consume it directly; the forward contracts hidden units, the weight gradients contract
// samples, so the hidden layer is computed in both orientations (the layer-1 fragments of W1
// and X serve as A or B unchanged; that costs 3 MFMAs per 16x16 tile on bf16-exact obs):
//   HT = W1 . X^T   (hidden on rows, sample on i)   -> logits  Z^T = W2 . relu(HT)
//   HN = X . W1^T   (sample on rows, hidden on i)   -> relu mask, h^T operand of dW2
// dZ (sample on i, action on rows) is both the A operand of dH = dZ . W2 and, transposed
// through LDS, the B operand of dW2^T = h^T . dZ.  dW1 = dH^T . X takes dH straight from its
// accumulator (hidden on i, samples on rows) against X loaded sample-on-k.  Layer-1 bias = input
// column F (x = 1), so db1 is column F of dW1.  All products use the exact three-way bf16 split
// (mlp_common.h): fp32-accurate, parity with torch fp32 autograd at 1e-5-relative.
//
// Partial sums: every wave accumulates its tiles in registers; the four waves of a workgroup
// are summed in fixed order through LDS and written as one partial per (workgroup, agent);
// update_reduce_kernel sums the partials in fixed order.  No atomics: bitwise reproducible.
#include <algorithm>
#include <cmath>

#include "mlp_common.h"

namespace d2d {

struct UpdArgs {
  int T, E, N, F, H, A, kind, mask_bytes;
  int tiles_per_t, n_tiles, G, P;
  float inv_A, clip_lo, clip_hi, beta, scale;
  const float *w1, *b1, *w2, *b2;  // actor (Policy) or critic (Value: A = 1)
  const float* obs;                 // [T][E][N][F]
  const void* actions;              // [T][E][N] masks (kind 0) / ids (kind 1)
  const float* logp_old;            // actor: element (t, e, k) at t*st[0] + e*st[1] + k*st[2]
  const float* weight;              // actor: advantage / M; critic: return target
  int64_t lo_st[3], w_st[3];
  float* partial;                   // [G][N][P]
};

constexpr float kEps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps (probs_to_logits clamp)

// three bf16 parts of 4 floats as 2 + 2 + 2 dwords
struct Parts4 {
  uint32_t h[2], m[2], l[2];
};
__device__ __forceinline__ Parts4 split3_4(const float (&v)[4]) {
  Parts4 o;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float a = v[2 * p], b = v[2 * p + 1];
    const float ar = a - ffrom(fbits(a) & 0xFFFF0000u), br = b - ffrom(fbits(b) & 0xFFFF0000u);
    const float al = ar - ffrom(fbits(ar) & 0xFFFF0000u), bl = br - ffrom(fbits(br) & 0xFFFF0000u);
    o.h[p] = pack_hi(a, b);
    o.m[p] = pack_hi(ar, br);
    o.l[p] = pack_hi(al, bl);
  }
  return o;
}
__device__ __forceinline__ bf16x8 cat(const uint32_t (&a)[2], const uint32_t (&b)[2]) {
  u32x4v v = {a[0], a[1], b[0], b[1]};
  return __builtin_bit_cast(bf16x8, v);
}
// high parts only (bf16-exact values)
__device__ __forceinline__ bf16x8 hi_frag(const float (&v)[8]) {
  uint32_t u[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) u[q] = pack_hi(v[2 * q], v[2 * q + 1]);
  return as_frag(u);
}

// Sum over the 16 lanes of a row (lanes with equal g), result in every lane of the row.
__device__ __forceinline__ float row_sum16(float v) {
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v += uf((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fu(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return v;
}

__device__ __forceinline__ float ld_st(const float* base, const int64_t (&st)[3], int t, int e, int k) {
  return base[(int64_t)t * st[0] + (int64_t)e * st[1] + (int64_t)k * st[2]];
}

// Layer-1 operand of one 16-sample half: lane (g, i) <- x[sample e][32c + 8g + j], bias 1 at
// column F, 0 past it and for samples past E.
template <int KC>
__device__ __forceinline__ void load_x_rows(float (&x)[KC][8], const UpdArgs& a, int t, int e, bool ok, int k, int g) {
  const float* row = a.obs + ((size_t)((size_t)t * a.E + (ok ? e : 0)) * a.N + k) * a.F;
  const int F = a.F;
#pragma unroll
  for (int c = 0; c < KC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 32 * c + 8 * g + j;
      const float v = row[min(col, F - 1)];
      x[c][j] = !ok ? 0.f : col < F ? v : col == F ? 1.f : 0.f;
    }
}

// Sample-on-k operand of dW1 = dH^T . X for input tile q (inputs 16q .. 16q+15): lane (g, i)
// slot j <- x[sample 16(j >> 2) + 4g + (j & 3)][16q + i] (the row order of the dH accumulator).
__device__ __forceinline__ void load_x_cols(float (&x)[8], const UpdArgs& a, int t, int e0, int k, int g, int i, int q) {
  const int F = a.F, col = 16 * q + i;
  const int cc = min(col, F - 1);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int e = e0 + 16 * (j >> 2) + 4 * g + (j & 3);
    const bool ok = e < a.E;
    const float v = a.obs[((size_t)((size_t)t * a.E + (ok ? e : 0)) * a.N + k) * F + cc];
    x[j] = !ok ? 0.f : col < F ? v : col == F ? 1.f : 0.f;
  }
}

// dL/dz for one 16-sample half (lane (g, i): sample e, actions 4g + r), plus loss sums.
// Bernoulli (KIND 0, ippo.py:157-160 + 185-189, quirk Q6: softmax probs as Bernoulli probs):
//   logp = mean_c log_prob(a_c) with torch's clamp(p, eps, 1-eps); entropy = mean_c
//   BCEWithLogits(logit(pc), p) = -p log pc - (1-p) log(1-pc).
// Categorical (KIND 1): Categorical(probs) renormalises q = p / sum p; logp = log clamp(q_a);
//   entropy = -sum q log clamp(q).
// Surrogate -min(r W, clamp(r) W) with torch.min's tie rule (each side gets half the gradient,
// so inside [1-eps, 1+eps] the slope is r W) and clamp passing the gradient inclusively.
template <int KIND>
__device__ __forceinline__ f32x4 ppo_dz(const UpdArgs& a, f32x4 z, int t, int e, bool ok, int k, int g,
                                        float& surr_acc, float& ent_acc) {
  const int A = a.A;
  bool valid[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) valid[r] = 4 * g + r < A;
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (valid[r]) mx = fmaxf(mx, z[r]);
  mx = group_max(mx);
  float ex[4], sum = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ex[r] = valid[r] ? __expf(z[r] - mx) : 0.f;
    sum += ex[r];
  }
  sum = group_sum(sum);
  const float inv = 1.f / sum;
  float p[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) p[r] = ex[r] * inv;

  const size_t cell = ((size_t)t * a.E + (ok ? e : 0)) * a.N + k;
  const float lo = ok ? ld_st(a.logp_old, a.lo_st, t, e, k) : 0.f;
  const float W = ok ? ld_st(a.weight, a.w_st, t, e, k) : 0.f;
  float gr[4];
  float logp, ent;
  // per-action pieces that scale with the surrogate coefficient (known after logp)
  float dsur[4];
  if constexpr (KIND == 0) {
    const uint32_t bits = ok ? (load_mask(a.actions, cell, a.mask_bytes) >> (4 * g)) : 0u;
    float lsum = 0.f, esum = 0.f;
    float logit[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pc = fminf(fmaxf(p[r], kEps), 1.f - kEps);
      const bool inside = p[r] >= kEps && p[r] <= 1.f - kEps;
      const float l1 = __logf(pc), l0 = __logf(1.f - pc);
      const bool bit = (bits >> r) & 1u;
      lsum += valid[r] ? (bit ? l1 : l0) : 0.f;
      esum += valid[r] ? -(p[r] * l1 + (1.f - p[r]) * l0) : 0.f;
      logit[r] = l1 - l0;
      dsur[r] = (valid[r] && inside) ? (bit ? 1.f / pc : -1.f / (1.f - pc)) : 0.f;
    }
    logp = group_sum(lsum) * a.inv_A;
    ent = group_sum(esum) * a.inv_A;
    const float ratio = __expf(logp - lo);
    const float cr = fminf(fmaxf(ratio, a.clip_lo), a.clip_hi);
    const float s1 = ratio * W, s2 = cr * W;
    const bool gate = (ratio >= a.clip_lo && ratio <= a.clip_hi) || s1 < s2;
    const float coef = gate ? -a.scale * ratio * W * a.inv_A : 0.f;
    const float eb = a.beta * a.scale * a.inv_A;  // d(-beta*mean ent)/dp_c = +beta * logit_c / A / B
#pragma unroll
    for (int r = 0; r < 4; ++r) gr[r] = valid[r] ? coef * dsur[r] + eb * logit[r] : 0.f;
    if (ok && g == 0) {
      surr_acc += fminf(s1, s2);
      ent_acc += ent;
    }
    float dot = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) dot += p[r] * gr[r];
    dot = group_sum(dot);
    f32x4 dz;
#pragma unroll
    for (int r = 0; r < 4; ++r) dz[r] = (ok && valid[r]) ? p[r] * (gr[r] - dot) : 0.f;
    return dz;
  } else {
    const int aid = ok ? (int)reinterpret_cast<const unsigned char*>(a.actions)[cell] : -1;
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) psum += p[r];
    psum = group_sum(psum);
    const float ipsum = 1.f / psum;
    float q[4], lq[4], lsel = 0.f, esum = 0.f;
    bool inside[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      q[r] = p[r] * ipsum;
      const float qc = fminf(fmaxf(q[r], kEps), 1.f - kEps);
      inside[r] = q[r] >= kEps && q[r] <= 1.f - kEps;
      lq[r] = __logf(qc);
      lsel += (valid[r] && 4 * g + r == aid) ? lq[r] : 0.f;
      esum += valid[r] ? q[r] * lq[r] : 0.f;
      dsur[r] = (valid[r] && inside[r] && 4 * g + r == aid) ? 1.f / qc : 0.f;
      // d(-beta * ent)/dq = beta * (log qc + q * [inside] / qc)
      gr[r] = valid[r] ? (lq[r] + (inside[r] ? q[r] / qc : 0.f)) : 0.f;
    }
    logp = group_sum(lsel);
    ent = -group_sum(esum);
    const float ratio = __expf(logp - lo);
    const float cr = fminf(fmaxf(ratio, a.clip_lo), a.clip_hi);
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
    gq = group_sum(gq);
    float dp[4], dot = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dp[r] = valid[r] ? (gr[r] - gq) * ipsum : 0.f;  // through q = p / sum p
      dot += p[r] * dp[r];
    }
    dot = group_sum(dot);
    if (ok && g == 0) {
      surr_acc += fminf(s1, s2);
      ent_acc += ent;
    }
    f32x4 dz;
#pragma unroll
    for (int r = 0; r < 4; ++r) dz[r] = (ok && valid[r]) ? p[r] * (dp[r] - dot) : 0.f;
    return dz;
  }
}

// Deterministic cross-wave sum of NV per-lane accumulators into wave 0's registers.
template <int NV>
__device__ __forceinline__ void reduce_waves(float (&acc)[NV], float* red, int wave, int lane) {
#pragma unroll 1
  for (int w = 1; w < 4; ++w) {
    __syncthreads();
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < NV; ++q) red[q * 64 + lane] = acc[q];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int q = 0; q < NV; ++q) acc[q] += red[q * 64 + lane];
    }
  }
}

// ------------------------------------------------------------------------- actor gradients
// KC = input chunks of 32 (F + 1 <= 32 KC), HT = hidden tiles of 16 (H <= 16 HT, even), A <= 16.
template <int KC, int HT, int KIND>
__global__ __launch_bounds__(256) void ppo_actor_grad_kernel(UpdArgs a) {
  static_assert(HT % 2 == 0, "layer 2 consumes hidden tiles in pairs");
  constexpr int QT = 2 * KC;  // input tiles of 16 in dW1
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  const int k = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, A = a.A, F = a.F;

  // ---- weights of agent k
  Parts w1p[HT][KC], w2p[HT / 2];
  Parts4 w2b[HT];
  f32x4 b2i;
  {
    const float* W1 = a.w1 + (size_t)k * H * F;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      const int hrow = 16 * t + i;
      const bool hok = hrow < H;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        float wv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = 32 * c + 8 * g + j;
          wv[j] = !hok ? 0.f : col < F ? W1[(size_t)hrow * F + col] : col == F ? a.b1[(size_t)k * H + hrow] : 0.f;
        }
        w1p[t][c] = split3(wv);
      }
      // B operand of dH = dZ . W2: k-slot (g, j < 4) <-> action 4g + j, column = hidden 16t + i
      float wb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int act = 4 * g + j;
        wb[j] = (hok && act < A) ? a.w2[((size_t)k * A + act) * H + hrow] : 0.f;
      }
      w2b[t] = split3_4(wb);
    }
#pragma unroll
    for (int c2 = 0; c2 < HT / 2; ++c2) {
      float wv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int hid = 16 * (2 * c2 + (j >> 2)) + 4 * g + (j & 3);
        wv[j] = (i < A && hid < H) ? a.w2[((size_t)k * A + i) * H + hid] : 0.f;
      }
      w2p[c2] = split3(wv);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) b2i[r] = 4 * g + r < A ? a.b2[(size_t)k * A + 4 * g + r] : 0.f;
  }

  f32x4 dw1[HT][QT], dw2[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    dw2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < QT; ++q) dw1[t][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 db2 = {0.f, 0.f, 0.f, 0.f};
  float surr_acc = 0.f, ent_acc = 0.f;

  __shared__ __attribute__((aligned(16))) float dzt[4][2][16][20];  // per-wave dZ transpose (row stride 20: conflict-light)
  __shared__ float red[(HT * QT * 4 + HT * 4 + 4 + 2) * 64];

  const int stride = a.G * 4;
  for (int tile = blockIdx.y * 4 + wave; tile < a.n_tiles; tile += stride) {
    const int t = tile / a.tiles_per_t;  // wave-uniform
    const int e0 = (tile - t * a.tiles_per_t) * 32;

    // ---- inputs, sample-on-i (layer 1 A/B operand)
    bf16x8 xh[2][KC];
    Parts xp[2][KC];
    uint32_t low = 0;
    float xr[2][KC][8];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int e = e0 + 16 * s + i;
      load_x_rows<KC>(xr[s], a, t, e, e < a.E, k, g);
#pragma unroll
      for (int c = 0; c < KC; ++c) {
#pragma unroll
        for (int j = 0; j < 8; ++j) low |= fbits(xr[s][c][j]) & 0xFFFFu;
        xh[s][c] = hi_frag(xr[s][c]);
      }
    }
    const bool x_exact = __builtin_amdgcn_ballot_w64(low != 0) == 0;  // wave-uniform
    if (!x_exact) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int c = 0; c < KC; ++c) xp[s][c] = split3(xr[s][c]);
    }

    // ---- forward (transposed): HT = W1 . X^T, Z^T = W2 . relu(HT) + b2; epilogue -> dZ
    f32x4 dz[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      f32x4 ht[HT];
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) {
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          const f32x4 z0 = c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : ht[t2];
          ht[t2] = mfma_bf16(w1p[t2][c].l, xh[s][c], z0);
          ht[t2] = mfma_bf16(w1p[t2][c].m, xh[s][c], ht[t2]);
          ht[t2] = mfma_bf16(w1p[t2][c].h, xh[s][c], ht[t2]);
        }
        if (!x_exact) {
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            ht[t2] = mfma_bf16(w1p[t2][c].h, xp[s][c].l, ht[t2]);
            ht[t2] = mfma_bf16(w1p[t2][c].m, xp[s][c].m, ht[t2]);
            ht[t2] = mfma_bf16(w1p[t2][c].h, xp[s][c].m, ht[t2]);
          }
        }
      }
      f32x4 zt = b2i;
#pragma unroll
      for (int c2 = 0; c2 < HT / 2; ++c2) {
        float hv[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          hv[r] = relu(ht[2 * c2][r]);
          hv[4 + r] = relu(ht[2 * c2 + 1][r]);
        }
        zt = mfma_split(w2p[c2], split3(hv), false, zt);
      }
      const int e = e0 + 16 * s + i;
      dz[s] = ppo_dz<KIND>(a, zt, t, e, e < a.E, k, g, surr_acc, ent_acc);
      db2 += dz[s];
    }

    // ---- hidden layer again, sample-on-rows: HN = X . W1^T
    f32x4 hn[2][HT];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) {
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          const f32x4 z0 = c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : hn[s][t2];
          hn[s][t2] = mfma_bf16(xh[s][c], w1p[t2][c].l, z0);
          hn[s][t2] = mfma_bf16(xh[s][c], w1p[t2][c].m, hn[s][t2]);
          hn[s][t2] = mfma_bf16(xh[s][c], w1p[t2][c].h, hn[s][t2]);
        }
        if (!x_exact) {
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            hn[s][t2] = mfma_bf16(xp[s][c].l, w1p[t2][c].h, hn[s][t2]);
            hn[s][t2] = mfma_bf16(xp[s][c].m, w1p[t2][c].m, hn[s][t2]);
            hn[s][t2] = mfma_bf16(xp[s][c].m, w1p[t2][c].h, hn[s][t2]);
          }
        }
      }

    // ---- dH = (dZ . W2) * [HN > 0]; the 4 live k-slots of each fragment half carry a second
    // split part, so the six split terms take three MFMAs
    f32x4 dh[2][HT];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float dv[4] = {dz[s][0], dz[s][1], dz[s][2], dz[s][3]};
      const Parts4 zp = split3_4(dv);
      const bf16x8 a_hm = cat(zp.h, zp.m), a_hl = cat(zp.h, zp.l);
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) {
        f32x4 acc = mfma_bf16(a_hl, cat(w2b[t2].l, w2b[t2].h), f32x4{0.f, 0.f, 0.f, 0.f});
        acc = mfma_bf16(a_hm, cat(w2b[t2].m, w2b[t2].h), acc);
        acc = mfma_bf16(a_hm, cat(w2b[t2].h, w2b[t2].m), acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = hn[s][t2][r] > 0.f ? acc[r] : 0.f;
        dh[s][t2] = acc;
      }
    }

    // ---- dZ transposed through LDS: lane (g, i) <- dZ[action i][sample 16(j>>2) + 4g + (j&3)]
    float dzn[8];
    {
      float(*buf)[16][20] = dzt[wave];
#pragma unroll
      for (int s = 0; s < 2; ++s)
        *reinterpret_cast<f32x4*>(&buf[s][i][4 * g]) = dz[s];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
      for (int j = 0; j < 8; ++j) dzn[j] = buf[j >> 2][4 * g + (j & 3)][i];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    const Parts dznp = split3(dzn);

    // ---- dW2^T += relu(HN)^T . dZ   (hidden on i / rows, samples on k)
#pragma unroll
    for (int t2 = 0; t2 < HT; ++t2) {
      float hv[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hv[r] = relu(hn[0][t2][r]);
        hv[4 + r] = relu(hn[1][t2][r]);
      }
      dw2[t2] = mfma_split(split3(hv), dznp, false, dw2[t2]);
    }

    // ---- dW1 += dH^T . X  (X loaded sample-on-k)
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      float xc[8];
      load_x_cols(xc, a, t, e0, k, g, i, q);
      const Parts xq = x_exact ? Parts{hi_frag(xc), {}, {}} : split3(xc);
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) {
        float hv[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          hv[r] = dh[0][t2][r];
          hv[4 + r] = dh[1][t2][r];
        }
        dw1[t2][q] = mfma_split(split3(hv), xq, x_exact, dw1[t2][q]);
      }
    }
  }

  // ---- workgroup partial
  constexpr int NV = HT * QT * 4 + HT * 4 + 4 + 2;
  float acc[NV];
  {
    int n = 0;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int q = 0; q < QT; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[n++] = dw1[t][q][r];
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[n++] = dw2[t][r];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[n++] = db2[r];
    acc[n++] = surr_acc;
    acc[n++] = ent_acc;
  }
  reduce_waves<NV>(acc, red, wave, lane);
  if (wave != 0) return;
  float* out = a.partial + ((size_t)blockIdx.y * a.N + k) * a.P;
  const int OB1 = H * F, OW2 = OB1 + H, OB2 = OW2 + A * H, OST = OB2 + A;
  int n = 0;
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int q = 0; q < QT; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = 16 * t + 4 * g + r, col = 16 * q + i;
        const float v = acc[n++];
        if (hid < H) {
          if (col < F) out[hid * F + col] = v;
          else if (col == F) out[OB1 + hid] = v;
        }
      }
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hid = 16 * t + 4 * g + r;
      const float v = acc[n++];
      if (hid < H && i < A) out[OW2 + i * H + hid] = v;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float v = row_sum16(acc[n++]);
    if (i == 0 && 4 * g + r < A) out[OB2 + 4 * g + r] = v;
  }
  const float ss = group_sum(row_sum16(acc[n++]));
  const float es = group_sum(row_sum16(acc[n++]));
  if (lane == 0) {
    out[OST] = ss;
    out[OST + 1] = es;
  }
}

// ------------------------------------------------------------------------ critic gradients
// Value(x) = V2 relu(V1 x + c1) + c2, loss = mean (v - R)^2 (ippo.py:210-216).  Hidden layer in
// the sample-on-rows orientation only: the 64 -> 1 layer is a per-lane product + a 16-lane row
// sum, dV1 = dHv^T . X as in the actor.  a.w2 = V2 [N][1][H], a.b2 = c2 [N][1], a.weight = R.
template <int KC, int HT>
__global__ __launch_bounds__(256) void ppo_critic_grad_kernel(UpdArgs a) {
  constexpr int QT = 2 * KC;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  const int k = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, F = a.F;

  Parts v1p[HT][KC];
  float v2f[HT];
  {
    const float* V1 = a.w1 + (size_t)k * H * F;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      const int hrow = 16 * t + i;
      const bool hok = hrow < H;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        float wv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = 32 * c + 8 * g + j;
          wv[j] = !hok ? 0.f : col < F ? V1[(size_t)hrow * F + col] : col == F ? a.b1[(size_t)k * H + hrow] : 0.f;
        }
        v1p[t][c] = split3(wv);
      }
      v2f[t] = hok ? a.w2[(size_t)k * H + hrow] : 0.f;
    }
  }
  const float c2 = a.b2[k];

  f32x4 dv1[HT][QT];
  float dv2[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    dv2[t] = 0.f;
#pragma unroll
    for (int q = 0; q < QT; ++q) dv1[t][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float dc2 = 0.f, loss_acc = 0.f;
  __shared__ float red[(HT * QT * 4 + HT + 2) * 64];

  const int stride = a.G * 4;
  for (int tile = blockIdx.y * 4 + wave; tile < a.n_tiles; tile += stride) {
    const int t = tile / a.tiles_per_t;
    const int e0 = (tile - t * a.tiles_per_t) * 32;
    bf16x8 xh[2][KC];
    Parts xp[2][KC];
    uint32_t low = 0;
    float xr[2][KC][8];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int e = e0 + 16 * s + i;
      load_x_rows<KC>(xr[s], a, t, e, e < a.E, k, g);
#pragma unroll
      for (int c = 0; c < KC; ++c) {
#pragma unroll
        for (int j = 0; j < 8; ++j) low |= fbits(xr[s][c][j]) & 0xFFFFu;
        xh[s][c] = hi_frag(xr[s][c]);
      }
    }
    const bool x_exact = __builtin_amdgcn_ballot_w64(low != 0) == 0;
    if (!x_exact) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int c = 0; c < KC; ++c) xp[s][c] = split3(xr[s][c]);
    }
    // HV = X . V1^T (sample 16s + 4g + r on rows, hidden 16t + i on lanes)
    f32x4 hv[2][HT];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) {
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          const f32x4 z0 = c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : hv[s][t2];
          hv[s][t2] = mfma_bf16(xh[s][c], v1p[t2][c].l, z0);
          hv[s][t2] = mfma_bf16(xh[s][c], v1p[t2][c].m, hv[s][t2]);
          hv[s][t2] = mfma_bf16(xh[s][c], v1p[t2][c].h, hv[s][t2]);
        }
        if (!x_exact) {
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            hv[s][t2] = mfma_bf16(xp[s][c].l, v1p[t2][c].h, hv[s][t2]);
            hv[s][t2] = mfma_bf16(xp[s][c].m, v1p[t2][c].m, hv[s][t2]);
            hv[s][t2] = mfma_bf16(xp[s][c].m, v1p[t2][c].h, hv[s][t2]);
          }
        }
      }
    // value, dL/dv = 2 (v - R) / B
    float dvs[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pv = 0.f;
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) pv = fmaf(relu(hv[s][t2][r]), v2f[t2], pv);
        const float v = row_sum16(pv) + c2;
        const int e = e0 + 16 * s + 4 * g + r;
        const bool ok = e < a.E;
        const float R = ok ? ld_st(a.weight, a.w_st, t, e, k) : 0.f;
        const float d = v - R;
        dvs[s][r] = ok ? 2.f * a.scale * d : 0.f;
        if (ok && i == 0) loss_acc += d * d;
      }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dc2 += i == 0 ? dvs[s][r] : 0.f;
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) dv2[t2] = fmaf(dvs[s][r], relu(hv[s][t2][r]), dv2[t2]);
      }
    // dV1 += dHv^T . X
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      float xc[8];
      load_x_cols(xc, a, t, e0, k, g, i, q);
      const Parts xq = x_exact ? Parts{hi_frag(xc), {}, {}} : split3(xc);
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) {
        float dv[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dv[r] = hv[0][t2][r] > 0.f ? dvs[0][r] * v2f[t2] : 0.f;
          dv[4 + r] = hv[1][t2][r] > 0.f ? dvs[1][r] * v2f[t2] : 0.f;
        }
        dv1[t2][q] = mfma_split(split3(dv), xq, x_exact, dv1[t2][q]);
      }
    }
  }

  constexpr int NV = HT * QT * 4 + HT + 2;
  float acc[NV];
  {
    int n = 0;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int q = 0; q < QT; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[n++] = dv1[t][q][r];
#pragma unroll
    for (int t = 0; t < HT; ++t) acc[n++] = dv2[t];
    acc[n++] = dc2;
    acc[n++] = loss_acc;
  }
  reduce_waves<NV>(acc, red, wave, lane);
  if (wave != 0) return;
  float* out = a.partial + ((size_t)blockIdx.y * a.N + k) * a.P;
  const int OB1 = H * F, OW2 = OB1 + H, OB2 = OW2 + H, OST = OB2 + 1;
  int n = 0;
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int q = 0; q < QT; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = 16 * t + 4 * g + r, col = 16 * q + i;
        const float v = acc[n++];
        if (hid < H) {
          if (col < F) out[hid * F + col] = v;
          else if (col == F) out[OB1 + hid] = v;
        }
      }
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    // lane (g, i) holds hidden 16t + i summed over its samples: add the four row groups
    const float v = group_sum(acc[n++]);
    if (g == 0 && 16 * t + i < H) out[OW2 + 16 * t + i] = v;
  }
  const float dcs = group_sum(row_sum16(acc[n++]));
  const float ls = group_sum(row_sum16(acc[n++]));
  if (lane == 0) {
    out[OB2] = dcs;
    out[OST] = ls;
    out[OST + 1] = 0.f;
  }
}

// Fixed-order sum of the G workgroup partials of every (agent, parameter) -> gradient tensors.
__global__ void update_reduce_kernel(const float* __restrict__ partial, int G, int N, int P, int H, int F, int A,
                                     float* gw1, float* gb1, float* gw2, float* gb2, float* stats) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * P) return;
  const int k = (int)(idx / P), p = (int)(idx - (int64_t)k * P);
  float s = 0.f;
  for (int b = 0; b < G; ++b) s += partial[((size_t)b * N + k) * P + p];
  const int OB1 = H * F, OW2 = OB1 + H, OB2 = OW2 + A * H, OST = OB2 + A;
  if (p < OB1) gw1[(size_t)k * H * F + p] = s;
  else if (p < OW2) gb1[(size_t)k * H + (p - OB1)] = s;
  else if (p < OB2) gw2[(size_t)k * A * H + (p - OW2)] = s;
  else if (p < OST) gb2[(size_t)k * A + (p - OB2)] = s;
  else if (stats) stats[(size_t)k * 2 + (p - OST)] = s;
}

}  // namespace d2d

using namespace d2d;

static int update_blocks(int N, int64_t n_tiles) {
  // about 4 workgroups per CU over the whole grid, at least one tile per wave
  int G = (int)std::max<int64_t>(1, std::min<int64_t>((1024 + N - 1) / N, (n_tiles + 3) / 4));
  return G;
}

extern "C" int64_t d2d_ppo_workspace(int32_t n_agents, int32_t T, int32_t n_envs, int32_t obs_dim, int32_t hidden,
                                     int32_t n_out) {
  if (n_agents <= 0 || T <= 0 || n_envs <= 0) return 0;
  const int64_t tiles = (int64_t)T * ((n_envs + 31) / 32);
  const int G = update_blocks(n_agents, tiles);
  const int64_t P = (int64_t)hidden * obs_dim + hidden + (int64_t)n_out * hidden + n_out + 2;
  return (int64_t)G * n_agents * P;
}

static int check_update(const d2d_mlp_desc* d, int T, const float* obs, const void* grads_w1, float* workspace,
                        int64_t ws, int critic) {
  if (!d || !obs || !d->w1 || !d->b1 || !d->w2 || !d->b2 || !grads_w1 || !workspace) {
    d2d_set_error("NULL argument");
    return D2D_EINVAL;
  }
  if (T < 0 || d->n_envs < 0 || d->n_agents < 0) { d2d_set_error("negative size"); return D2D_EINVAL; }
  if (d->hidden < 1 || d->hidden > 64) { d2d_set_error("hidden=%d outside [1,64]", d->hidden); return D2D_EUNSUPPORTED; }
  if (d->obs_dim < 1 || d->obs_dim + 1 > 64) { d2d_set_error("obs_dim=%d outside [1,63]", d->obs_dim); return D2D_EUNSUPPORTED; }
  if (!critic && (d->n_out < 1 || d->n_out > 16)) { d2d_set_error("n_out=%d outside [1,16]", d->n_out); return D2D_EUNSUPPORTED; }
  if (!critic && d->kind != 0 && d->kind != 1) { d2d_set_error("kind must be 0 or 1"); return D2D_EINVAL; }
  const int64_t need = d2d_ppo_workspace(d->n_agents, T, d->n_envs, d->obs_dim, d->hidden, critic ? 1 : d->n_out);
  if (ws < need) { d2d_set_error("workspace %lld < %lld floats", (long long)ws, (long long)need); return D2D_EINVAL; }
  return D2D_OK;
}

static UpdArgs make_args(const d2d_mlp_desc* d, int T, const float* obs, float* workspace, int critic) {
  UpdArgs a{};
  a.T = T; a.E = d->n_envs; a.N = d->n_agents; a.F = d->obs_dim; a.H = d->hidden;
  a.A = critic ? 1 : d->n_out; a.kind = d->kind;
  a.mask_bytes = a.A <= 8 ? 1 : a.A <= 16 ? 2 : 4;
  a.tiles_per_t = (a.E + 31) / 32;
  a.n_tiles = T * a.tiles_per_t;
  a.G = update_blocks(a.N, a.n_tiles);
  a.P = a.H * a.F + a.H + a.A * a.H + a.A + 2;
  a.inv_A = 1.f / (float)a.A;
  a.w1 = d->w1; a.b1 = d->b1; a.w2 = d->w2; a.b2 = d->b2;
  a.obs = obs;
  a.partial = workspace;
  return a;
}

static int launch_reduce(const UpdArgs& a, float* gw1, float* gb1, float* gw2, float* gb2, float* stats, hipStream_t s) {
  const int64_t n = (int64_t)a.N * a.P;
  const int threads = 256;
  hipLaunchKernelGGL(update_reduce_kernel, dim3((unsigned)((n + threads - 1) / threads)), dim3(threads), 0, s,
                     a.partial, a.G, a.N, a.P, a.H, a.F, a.A, gw1, gb1, gw2, gb2, stats);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

template <int KC, int HT>
static void launch_actor(const UpdArgs& a, hipStream_t s) {
  dim3 grid(a.N, a.G);
  if (a.kind == 0) hipLaunchKernelGGL((ppo_actor_grad_kernel<KC, HT, 0>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((ppo_actor_grad_kernel<KC, HT, 1>), grid, dim3(256), 0, s, a);
}

extern "C" int d2d_ppo_actor_grad(const d2d_mlp_desc* d, int32_t T, const float* obs, const void* actions,
                                  const float* logp_old, const int64_t* logp_strides, const float* weight,
                                  const int64_t* weight_strides, float clip, float beta, float scale, float* gw1,
                                  float* gb1, float* gw2, float* gb2, float* stats, float* workspace,
                                  int64_t workspace_floats, void* stream) {
  int rc = check_update(d, T, obs, gw1, workspace, workspace_floats, 0);
  if (rc) return rc;
  if (!actions || !logp_old || !logp_strides || !weight || !weight_strides || !gb1 || !gw2 || !gb2) {
    d2d_set_error("d2d_ppo_actor_grad: NULL argument");
    return D2D_EINVAL;
  }
  UpdArgs a = make_args(d, T, obs, workspace, 0);
  a.actions = actions;
  a.logp_old = logp_old;
  a.weight = weight;
  for (int q = 0; q < 3; ++q) { a.lo_st[q] = logp_strides[q]; a.w_st[q] = weight_strides[q]; }
  a.clip_lo = 1.f - clip; a.clip_hi = 1.f + clip; a.beta = beta; a.scale = scale;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a.N == 0) return D2D_OK;
  if (a.n_tiles == 0) {
    D2D_CHECK_HIP(hipMemsetAsync(workspace, 0, sizeof(float) * (size_t)a.N * a.P, s));
    a.G = 1;
    return launch_reduce(a, gw1, gb1, gw2, gb2, stats, s);
  }
  const int ht = (a.H + 15) / 16;
  if (a.F + 1 <= 32) {
    if (ht <= 2) launch_actor<1, 2>(a, s); else launch_actor<1, 4>(a, s);
  } else {
    if (ht <= 2) launch_actor<2, 2>(a, s); else launch_actor<2, 4>(a, s);
  }
  D2D_CHECK_HIP(hipGetLastError());
  return launch_reduce(a, gw1, gb1, gw2, gb2, stats, s);
}

extern "C" int d2d_ppo_critic_grad(const d2d_mlp_desc* d, int32_t T, const float* obs, const float* returns,
                                   const int64_t* return_strides, float scale, float* gw1, float* gb1, float* gw2,
                                   float* gb2, float* stats, float* workspace, int64_t workspace_floats,
                                   void* stream) {
  int rc = check_update(d, T, obs, gw1, workspace, workspace_floats, 1);
  if (rc) return rc;
  if (!returns || !return_strides || !gb1 || !gw2 || !gb2) {
    d2d_set_error("d2d_ppo_critic_grad: NULL argument");
    return D2D_EINVAL;
  }
  UpdArgs a = make_args(d, T, obs, workspace, 1);
  a.weight = returns;
  for (int q = 0; q < 3; ++q) a.w_st[q] = return_strides[q];
  a.scale = scale;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a.N == 0) return D2D_OK;
  if (a.n_tiles == 0) {
    D2D_CHECK_HIP(hipMemsetAsync(workspace, 0, sizeof(float) * (size_t)a.N * a.P, s));
    a.G = 1;
    return launch_reduce(a, gw1, gb1, gw2, gb2, stats, s);
  }
  const int ht = (a.H + 15) / 16;
  dim3 grid(a.N, a.G);
  if (a.F + 1 <= 32) {
    if (ht <= 2) hipLaunchKernelGGL((ppo_critic_grad_kernel<1, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ppo_critic_grad_kernel<1, 4>), grid, dim3(256), 0, s, a);
  } else {
    if (ht <= 2) hipLaunchKernelGGL((ppo_critic_grad_kernel<2, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ppo_critic_grad_kernel<2, 4>), grid, dim3(256), 0, s, a);
  }
  D2D_CHECK_HIP(hipGetLastError());
  return launch_reduce(a, gw1, gb1, gw2, gb2, stats, s);
}
