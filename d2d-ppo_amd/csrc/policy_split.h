// The split-bf16 MLP behaviour policy of one agent on one 16-env tile (ippo.py:54-90, 154-176), shared by the
// policy slot kernel (policy_kernels.hip: policy_split_kernel, obs through a per-wave LDS DMA ring) and the
// fused env + policy slot (env_kernels.hip: comb_policy_fused_kernel, the records of its env slice in LDS):
// the agent's weight fragments split once per wave (SplitNet::load), the input staging of a tile, and layers
// 1-2 of a tile (SplitNet::tile) on v_mfma_f32_16x16x32_bf16 over the exact three-way bf16 split of every fp32
// operand (mlp_common.h).  Layer-1 bias rides in the input column F (x = 1), so KC = ceil((F + 1) / 32) chunks.
#pragma once
#include "policy_epilogue.h"

#ifndef D2D_POLICY_L2_F32
// 1 (A/B): actor layer 2 on v_mfma_f32_16x16x4_f32 straight from relu(H^T) (an exact fmaf chain, 16 MFMAs
// of 32 cycles per tile) instead of the three-way split of relu(H^T) (88 VALU per tile) and 6 bf16 MFMAs
#define D2D_POLICY_L2_F32 0
#endif

namespace d2d {

// x[c][j] <- slot, then input F := 1.0 (layer-1 bias input) and inputs past F := 0
template <int KC>
__device__ __forceinline__ void stage_inputs(float (&x)[KC][8], const float* slot, int lane, int F, int g) {
#pragma unroll
  for (int c = 0; c < KC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // (v & keep) | bias: one v_and_or_b32 -- a select of the loaded value would be turned
      // into a branch around the LDS read
      const int col = 32 * c + 8 * g + j;
      const uint32_t keep = col < F ? 0xFFFFFFFFu : 0u, bias = col == F ? 0x3F800000u : 0u;
      x[c][j] = uf((fu(slot[(c * 8 + j) * 64 + lane]) & keep) | bias);
    }
}

// The same from compact-record words: chunk c's two words d[c][0..1] of this lane (record bytes 32c + 8g ..
// 32c + 8g + 7 of its env row).  The record row already holds the bias input 1 at column F and zeros past it
// (the env kernel writes them); sm[c][h] = this lane's int8 byte masks of words h = 0, 1 (rec_byte)
template <int KC>
__device__ __forceinline__ void stage_record_words(float (&x)[KC][8], const uint32_t (&d)[KC][2],
                                                   const uint32_t (&sm)[KC][2]) {
#pragma unroll
  for (int c = 0; c < KC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) x[c][j] = rec_byte(d[c][j >> 2], j & 3, sm[c][j >> 2]);
}

// int8 byte masks of this lane's record words (agent k, columns 32c + 8g + 4h + r)
template <int KC>
__device__ __forceinline__ void record_sign_masks(uint32_t (&sm)[KC][2], const uint32_t* sgn, int k, int g) {
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const uint32_t sg = (sgn[(size_t)k * KC + c] >> (8 * g)) & 0xFFu;
    sm[c][0] = sign_bytes(sg & 0xFu);
    sm[c][1] = sign_bytes(sg >> 4);
  }
}

// KC = input chunks of 32 (F + 1 <= 32*KC), HT = hidden tiles of 16 (H <= 16*HT, even)
template <int KC, int HT, bool ACTOR, bool CRITIC>
struct SplitNet {
  Parts w1p[ACTOR ? HT : 1][KC], v1p[CRITIC ? HT : 1][KC];
#if D2D_POLICY_L2_F32
  float w2f[HT][4];  // A operand of step (t, r): row = action i, k-slot g <-> hidden 16t + 4g + r
#else
  Parts w2p[HT / 2];
#endif
  float v2f[HT][4];
  f32x4 b2i;
  float c2;

  // weight fragments of agent k, split once (kModeValue: the critic's only); lane (g, i)
  __device__ __forceinline__ void load(const MlpArgs& a, int k, int g, int i) {
    const int F = a.F, H = a.H, A = a.A;
    const float* W1 = a.w1 + (size_t)k * H * F;
    const float* V1 = CRITIC ? a.v1 + (size_t)k * H * F : nullptr;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      const int hrow = 16 * t + i;
      const bool hok = hrow < H;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        float wv[8], vv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = 32 * c + 8 * g + j;
          wv[j] = !hok ? 0.f : col < F ? W1[(size_t)hrow * F + col] : col == F ? a.b1[(size_t)k * H + hrow] : 0.f;
          if constexpr (CRITIC)
            vv[j] = !hok ? 0.f : col < F ? V1[(size_t)hrow * F + col] : col == F ? a.c1[(size_t)k * H + hrow] : 0.f;
        }
        if constexpr (ACTOR) w1p[t][c] = split3(wv);
        if constexpr (CRITIC) v1p[t][c] = split3(vv);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = 16 * t + 4 * g + r;
        v2f[t][r] = (CRITIC && hid < H) ? a.v2[(size_t)k * H + hid] : 0.f;
      }
    }
#if D2D_POLICY_L2_F32
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = 16 * t + 4 * g + r;
        w2f[t][r] = (i < A && hid < H) ? a.w2[((size_t)k * A + i) * H + hid] * kLog2e : 0.f;
      }
#else
#pragma unroll
    for (int c2i = 0; c2i < (ACTOR ? HT / 2 : 0); ++c2i) {
      // element j of lane group g <-> hidden 16 * (2 c2i + (j >> 2)) + 4 g + (j & 3): the
      // accumulator registers of layer-1 tiles 2 c2i and 2 c2i + 1
      float wv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int hid = 16 * (2 * c2i + (j >> 2)) + 4 * g + (j & 3);
        wv[j] = (i < A && hid < H) ? a.w2[((size_t)k * A + i) * H + hid] * kLog2e : 0.f;
      }
      w2p[c2i] = split3(wv);
    }
#endif
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int act = 4 * g + r;
      b2i[r] = act < A ? a.b2[(size_t)k * A + act] * kLog2e : 0.f;
    }
    c2 = CRITIC ? a.c2[k] : 0.f;
  }

  // layers 1-2 of one tile from its staged inputs -> (pre-scaled) logits lg and critic value
  template <bool U8>
  __device__ __forceinline__ void tile(const float (&xc)[KC][8], f32x4& lg, float& value) const {
    // bf16 high parts of the inputs; the residual parts only when some input of the tile is
    // not bf16-exact (wave-uniform branch, rare for env observations; never for the record,
    // whose integers in [-128, 255] are bf16-exact)
    bf16x8 xh[KC];
    uint32_t low = 0;
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      uint32_t u[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        low |= (fbits(xc[c][2 * q]) | fbits(xc[c][2 * q + 1])) & 0xFFFFu;
        u[q] = pack_hi(xc[c][2 * q], xc[c][2 * q + 1]);
      }
      xh[c] = as_frag(u);
    }
    const bool x_exact = U8 || __builtin_amdgcn_ballot_w64(low != 0) == 0;  // wave-uniform

    // ---- layer 1 (actor, critic), transposed: H^T = W1' . [X | 1]^T; the three weight parts
    // against the high parts of X, then (rarely) the residual terms of X
    f32x4 ha[HT], hv[HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) {
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        if constexpr (ACTOR) {
          const f32x4 za = c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : ha[t];
          ha[t] = mfma_bf16(w1p[t][c].l, xh[c], za);
          ha[t] = mfma_bf16(w1p[t][c].m, xh[c], ha[t]);
          ha[t] = mfma_bf16(w1p[t][c].h, xh[c], ha[t]);
        }
        if constexpr (CRITIC) {
          const f32x4 zv = c == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : hv[t];
          hv[t] = mfma_bf16(v1p[t][c].l, xh[c], zv);
          hv[t] = mfma_bf16(v1p[t][c].m, xh[c], hv[t]);
          hv[t] = mfma_bf16(v1p[t][c].h, xh[c], hv[t]);
        }
      }
    }
    if (!x_exact) {
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        const Parts xp = split3(xc[c]);
#pragma unroll
        for (int t = 0; t < HT; ++t) {
          if constexpr (ACTOR) {
            ha[t] = mfma_bf16(w1p[t][c].h, xp.l, ha[t]);
            ha[t] = mfma_bf16(w1p[t][c].m, xp.m, ha[t]);
            ha[t] = mfma_bf16(w1p[t][c].h, xp.m, ha[t]);
          }
          if constexpr (CRITIC) {
            hv[t] = mfma_bf16(v1p[t][c].h, xp.l, hv[t]);
            hv[t] = mfma_bf16(v1p[t][c].m, xp.m, hv[t]);
            hv[t] = mfma_bf16(v1p[t][c].h, xp.m, hv[t]);
          }
        }
      }
    }

    // ---- actor layer 2 on the accumulators of tile pairs (split, full six terms)
    lg = b2i;
#if D2D_POLICY_L2_F32 == 1
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) lg = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[t][r], relu(ha[t][r]), lg, 0, 0, 0);
#elif D2D_POLICY_L2_F32 == 2
    {  // two independent accumulation chains (hidden tiles [0, HT/2) and [HT/2, HT)), summed once
      f32x4 lh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < HT / 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          lg = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[t][r], relu(ha[t][r]), lg, 0, 0, 0);
          lh = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[HT / 2 + t][r], relu(ha[HT / 2 + t][r]), lh, 0, 0, 0);
        }
      lg += lh;
    }
#else
#pragma unroll
    for (int c2i = 0; c2i < (ACTOR ? HT / 2 : 0); ++c2i) {
      float hvals[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hvals[r] = relu(ha[2 * c2i][r]);
        hvals[4 + r] = relu(ha[2 * c2i + 1][r]);
      }
      lg = mfma_split(w2p[c2i], split3(hvals), false, lg);
    }
#endif
    // ---- critic layer 2 (64 -> 1) on VALU
    value = 0.f;
    if constexpr (CRITIC) {
      float pv = 0.f;
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) pv = fmaf(relu(hv[t][r]), v2f[t][r], pv);
      pv = group_sum(pv);
      value = pv + c2;
    }
  }
};

// d2d_policy_mlp_step's argument checks and kernel arguments (policy_kernels.hip; D2D_OK or an error code with
// d2d_last_error set)
int policy_mlp_args(const d2d_mlp_desc* d, const void* obs, const void* forced, uint32_t rng_step, int32_t deterministic,
                    void* actions, float* logp, float* value, MlpArgs& a);

}  // namespace d2d
