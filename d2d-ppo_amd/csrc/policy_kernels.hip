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
#include <atomic>
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "policy_split.h"

namespace d2d {


// KS = input k-steps of 4 (F <= 4*KS), HT = hidden tiles of 16 (H <= 16*HT),
// KIND 0 Bernoulli / 1 Categorical, CRITIC: iPPO per-agent critic present
template <int KS, int HT, int KIND, bool CRITIC>
__global__ __launch_bounds__(256) void policy_mlp_kernel(MlpArgs a) {
  // Philox step of the launch, read once (the optional device offset of graph replays)
  const uint32_t rng = a.rng_off ? a.rng_step + *a.rng_off : a.rng_step;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;   // lane group: k-slot of A/B operands, row group of C/D
  const int i = lane & 15;   // row of A / column of B, C/D (the env of the tile)
  const int k = blockIdx.x;  // agent (fast grid axis: all agents of an env chunk run together)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
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
        for (int r = 0; r < 4; ++r) pv = fmaf(relu(hv[t][r]), v2f[t][r], pv);
      pv = group_sum(pv);
      value = pv + c2;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) lg[r] *= kLog2e;
    policy_epilogue<KIND, CRITIC>(a, lg, value, env, env_ok, k, g, rng);
  }
}


// ---------------------------------------------------------------------------------------------
// Split-bf16 kernel (default): v_mfma_f32_16x16x32_bf16 on the exact three-way split of every
// fp32 operand (mlp_common.h).  Layer-1 bias rides in the input column F (x = 1), so
// KC = ceil((F + 1) / 32) chunks.

// Obs staging: a per-wave ring of RING tile slots in LDS, filled by buffer->LDS DMA
// (buffer_load_dword ... lds, no VGPR destination) RING - 2 tiles ahead of use.  Slot layout
// [c][j][lane] (lane-linear, as the DMA writes it): DMA instruction (c, j) brings lane (g, i) the
// input 32c + 8g + j of its env row, which is exactly element j of its MFMA B fragment.  The
// buffer descriptor's range check returns 0 past the obs buffer, so the row is read unclamped:
// the columns past F hold the next agent's inputs and are zeroed by stage_inputs().
// hipcc does not order the DMA's LDS write before the ds_read of the slot, so the waits are
// explicit, counted s_waitcnt vmcnt (see the loop).
// ring depth: 6 tiles at KC = 1; 4 at KC = 2 (the counted wait must stay below vmcnt's 63);
// the compact record (U8) brings a row chunk in 2 DMAs instead of 8: 8 / 6 tiles
template <int KC, bool U8>
constexpr int ring_tiles() { return U8 ? (KC == 1 ? 8 : 6) : (KC == 1 ? 6 : 4); }
// dwords of one lane's row chunk (8 inputs): 8 floats or 8 record bytes
template <bool U8>
constexpr int chunk_dwords() { return U8 ? 2 : 8; }


// The same from a ring slot of compact-record words [c][2][lane]: the record row already holds the
// bias input 1 at column F and zeros past it (the env kernel writes them); sm[c][h] = this lane's
// int8 byte masks of words h = 0, 1 (rec_byte)
template <int KC>
__device__ __forceinline__ void stage_record(float (&x)[KC][8], const uint32_t* slot, int lane,
                                             const uint32_t (&sm)[KC][2]) {
  uint32_t d[KC][2];
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    d[c][0] = slot[(c * 2) * 64 + lane];
    d[c][1] = slot[(c * 2 + 1) * 64 + lane];
  }
  stage_record_words<KC>(x, d, sm);
}

#ifndef D2D_POLICY_RNG_EARLY
// 1 (A/B): draw the paired epilogue's Philox block before the tile MFMAs instead of in the epilogue.  The
// scheduler then issues the ten dependent rounds as one chain ahead of the MFMAs rather than in their gaps,
// and the partner wave already hides the chain: 233.7 / 229.6 vs 232.7 / 227.5 us per 65,536-env slot
// (r04i, two boxes' runs each) -- no gain, off
#define D2D_POLICY_RNG_EARLY 0
#endif
#ifndef D2D_POLICY_ABLATE_NOREAD
// != 0 only in tools/gpu/build_fusion_bound.sh's timing variant: every obs DMA aimed outside the buffer (zeros, no
// memory traffic) -- the policy kernel without its read of the slot's record, i.e. what fusing the env step into
// it could save at most (tools/gpu/fusion_bound.py)
#define D2D_POLICY_ABLATE_NOREAD 0
#endif
#ifndef D2D_POLICY_ABLATE_FORCED_DMA
// != 0 only in timing variants (tools/gpu/run_r06o.sh): forced mode without the forced-word DMA (every forced mask
// reads as 0) -- what the forced words' DMA and extraction cost
#define D2D_POLICY_ABLATE_FORCED_DMA 0
#endif
#ifndef D2D_POLICY_FORCED_PAIR
// 1: one forced-word DMA per tile PAIR (lanes of group 0 bring tile t's words, group 1 tile t + 1's) instead of one per
// tile (group 0 only)
#define D2D_POLICY_FORCED_PAIR 1
#endif
#ifndef D2D_POLICY_ACTOR_WAVES
// waves per SIMD of the actor-only record instantiation (137 VGPRs at 3; 4 needs <= 128)
#define D2D_POLICY_ACTOR_WAVES 3
#endif
#ifndef D2D_POLICY_AF8_WAVES
// the same for the A = 8 instantiations (AF = 8: 124-133 VGPRs at 3, 128 with no spills at 4 -- the forced mode
// 128.2 / 129.9 -> 124.0 / 124.8 us per 65,536-env slot, sampled and deterministic unchanged; profiles/r06/policy_waves_ab.json)
#define D2D_POLICY_AF8_WAVES 4
#endif
// KC = input chunks of 32 (F + 1 <= 32*KC), HT = hidden tiles of 16 (H <= 16*HT, even);
// U8: the inputs are the env kernel's compact obs record (D2D_OBS_U8)
// AF: the action count as a compile-time constant (0: a.A at run time; 8: the combinatorial envs' 8 channels)
template <int KC, int HT, int KIND, bool CRITIC, int MODE, bool U8, int AF = 0>
// (H <= 64, F + 1 <= 32: 2 waves / SIMD with the iPPO critic or on fp32 rows (their DMA ring is 48 KB), 3 for the
// actor alone on the record (137 VGPRs: test(), D2D-PPO,
// and iPPO training rollouts whose values come from the first epoch's critic pass); H in (64, 128] -- the
// learners' default hidden_size 128 -- or F + 1 > 32: one wave / SIMD with the doubled weight fragments)
__global__ __launch_bounds__(256, (KC == 1 && HT <= 4) ? ((CRITIC || !U8) ? 2 : AF == 8 ? D2D_POLICY_AF8_WAVES : D2D_POLICY_ACTOR_WAVES) : 1) void policy_split_kernel(MlpArgs a) {
  static_assert(HT % 2 == 0, "layer 2 consumes hidden tiles in pairs");
  // Philox step of the launch, read once before the obs pipeline starts (the optional device
  // offset of graph replays; a load inside the epilogue would add a wait to every tile pair)
  const uint32_t rng = (MODE == kModeSample && a.rng_off) ? a.rng_step + *a.rng_off : a.rng_step;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int i = lane & 15;
  int k, by;
  xcd_block(k, by);  // k = agent, by = env chunk
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int N = a.N, F = a.F, A = AF ? AF : a.A;
  const int tiles = a.envs_per_wave / 16;
  const int wave_env0 = (by * (blockDim.x >> 6) + wave) * a.envs_per_wave;

  // ---- weight fragments of agent k, split once per workgroup (kModeValue: the critic's only)
  constexpr bool ACTOR = MODE != kModeValue;
  static_assert(ACTOR || CRITIC, "the value-only instantiation needs the critic");
  SplitNet<KC, HT, ACTOR, CRITIC> net;
  net.load(a, k, g, i);

  // Two obs register sets alternate (loop unrolled by two), so each tile's loads are issued two
  // tiles ahead of their use without a register copy that would wait on them early.
  constexpr int RING = ring_tiles<KC, U8>();
  constexpr int DPC = chunk_dwords<U8>();
  __shared__ float ring[4][RING][KC][DPC][64];
  // forced mode: the forced-action words of each tile travel through the same DMA ring (one more
  // buffer_load_dword ... lds per tile: lane i of group 0 brings the dword holding env i's byte), so no
  // register load inside the tile loop drains the ring with vmcnt(0) and a wave can run any number of
  // tiles (one resident round).  Paired epilogue (A <= 8, one byte per cell) only; otherwise the DMA is
  // aimed outside the buffer (no traffic) and the epilogue loads its masks itself.
  constexpr int FD = (MODE == kModeForced && !D2D_POLICY_ABLATE_FORCED_DMA) ? 1 : 0;
  constexpr bool FP = D2D_POLICY_FORCED_PAIR != 0;           // one forced DMA per tile pair
  constexpr int FSLOTS = FD ? (FP ? RING / 2 : RING) : 1;     // forced-word ring slots
  __shared__ uint32_t fring[4][FSLOTS][64];
  const int64_t fbytes = MODE == kModeForced ? ((int64_t)a.E * N * a.mask_bytes + 3) / 4 * 4 : 0;
  const __amdgpu_buffer_rsrc_t frsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(MODE == kModeForced ? a.forced : (const void*)a.act_out), 0,
      fbytes > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)fbytes, 0x00020000);
  // row bytes: F floats, or the record's 32 KC bytes
  const int RB = U8 ? 32 * KC : 4 * F;
  const uint8_t* wbase = (U8 ? a.rec : reinterpret_cast<const uint8_t*>(a.obs)) + ((size_t)wave_env0 * N + k) * RB;
  const int64_t total = (int64_t)a.E * N * RB, done = ((int64_t)wave_env0 * N + k) * RB;
  const int64_t rest = total - done;
  const uint32_t nbytes = rest <= 0 ? 0u : rest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)rest;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(wbase), 0, nbytes, 0x00020000);
  // int8 byte masks of this lane's record words (agent k, columns 32c + 8g + 4h + r)
  uint32_t sm[KC][2] = {};
  if constexpr (U8) record_sign_masks<KC>(sm, a.sgn, k, g);
  auto issue = [&](int t, bool even) {
    // look-ahead tiles past this wave's last are still issued (the counted waits need a fixed
    // DMA count) but aimed outside the descriptor's range: no memory traffic, zeros
    const uint32_t vo = (t < tiles && !D2D_POLICY_ABLATE_NOREAD) ? (uint32_t)((t * 16 + i) * N * RB) + (U8 ? 8 : 32) * g
                                                                   : 0x80000000u;
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
      for (int j = 0; j < DPC; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsrc, (__attribute__((address_space(3))) void*)&ring[wave][t % RING][c][j][0], 4,
            vo + (U8 ? 32 * c + 4 * j : 4 * (32 * c + j)), 0, 0, 0);
    if constexpr (FD) {
      // 32-bit cell offsets: policy_mlp_args caps the forced buffer at 2 GiB.  FP: issued with the even tile of a pair
      // (wave-uniform branch), lane group 0 bringing tile t's words and group 1 tile t + 1's
      if (!FP || even) {
        const int tf = FP ? t + (g & 1) : t;
        const int env = wave_env0 + tf * 16 + i;
        const uint32_t fo = (tf < tiles && (FP ? g < 2 : g == 0) && A <= 8 && env < a.E)
                                ? ((uint32_t)env * (uint32_t)N + (uint32_t)k) & ~3u
                                : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            frsrc, (__attribute__((address_space(3))) void*)&fring[wave][(FP ? t >> 1 : t) % FSLOTS][0], 4, fo, 0, 0, 0);
      }
    }
  };
  // layers 1-2 of one tile -> (pre-scaled) logits lg and critic value
  auto tile = [&](int tt, f32x4& lg, float& value) {
    float xc[KC][8];
    if constexpr (U8)
      stage_record<KC>(xc, reinterpret_cast<const uint32_t*>(&ring[wave][tt % RING][0][0][0]), lane, sm);
    else
      stage_inputs<KC>(xc, &ring[wave][tt % RING][0][0][0], lane, F, g);
    net.template tile<U8>(xc, lg, value);
  };
  // every wave runs the same even number of tiles (tiles past E read zeros and store nothing), so
  // the DMA count between a tile's issue and its wait is fixed: RING - 2 tiles of KC * DPC DMAs
  // (anything else issued in between -- the stores -- only makes the counted wait stricter)
  static_assert(RING >= 4 && RING % 2 == 0, "two tiles per iteration");
  for (int t = 0; t < RING - 2; ++t) issue(t, (t & 1) == 0);
  for (int tt = 0; tt < tiles; tt += 2) {
    issue(tt + RING - 2, true);
    issue(tt + RING - 1, false);
    wait_vmem<(RING - 2) * KC * DPC + (FP ? (RING - 2) / 2 : RING - 2) * FD>();  // tiles tt, tt + 1 have landed
    __builtin_amdgcn_sched_barrier(0);        // no LDS read of the slots moves above the wait
    const int env0 = wave_env0 + tt * 16 + i, env1 = env0 + 16;
    // forced byte of this lane's paired-epilogue cell (env0 for groups 0-1, env1 for 2-3), read before the
    // slots are released
    uint32_t fpre = 0;
    if constexpr (FD) {
      const int envc = g < 2 ? env0 : env1;
      const uint32_t w = FP ? fring[wave][(tt >> 1) % FSLOTS][(g < 2 ? 0 : 16) + i]
                            : fring[wave][(g < 2 ? tt : tt + 1) % FSLOTS][i];
      fpre = (w >> (8 * (((uint32_t)(envc < a.E ? envc : 0) * (uint32_t)N + (uint32_t)k) & 3u))) & 0xFFu;
    }
    // the paired epilogue's Philox block, drawn here: inside the scheduling region of the tiles' MFMAs (the
    // barrier below would otherwise keep it behind them as a serial chain of ten dependent rounds)
    u32x4 rpre = {};
    if constexpr (MODE == kModeSample && D2D_POLICY_RNG_EARLY) {
      if (A <= 8) {
        const int envc = g < 2 ? env0 : env1;
        rpre = policy_rng_block<KIND>(a, envc, envc < a.E, k, g & 1, rng);
      }
    }
    f32x4 lg0, lg1;
    float v0, v1;
    tile(tt, lg0, v0);
    tile(tt + 1, lg1, v1);
    __builtin_amdgcn_sched_barrier(0);        // the slots are read before the next DMA reuses them
    if constexpr (!ACTOR) {
      // value only: lane group 0 stores tile tt's values, group 1 tile tt + 1's (every lane of a row
      // holds its env's value after the group sum)
      const int envv = g == 0 ? env0 : env1;
      if (g < 2 && envv < a.E) a.value_out[(size_t)k * a.E + envv] = g == 0 ? v0 : v1;
      continue;
    }
    if (A <= 8) {
      // one epilogue for both tiles: lanes 0-31 keep tile tt (action groups 0, 1), lanes 32-63
      // take tile tt + 1's lanes 0-31 (permlane32_swap: vdst upper half <- src lower half)
      f32x4 lgc;
#pragma unroll
      for (int r = 0; r < 4; ++r) lgc[r] = uf(__builtin_amdgcn_permlane32_swap(fu(lg0[r]), fu(lg1[r]), false, false)[0]);
      const int envc = g < 2 ? env0 : env1;
      policy_epilogue<KIND, CRITIC, true, MODE, MODE == kModeForced, false, MODE == kModeSample && D2D_POLICY_RNG_EARLY, AF>(
          a, lgc, g < 2 ? v0 : v1, envc, envc < a.E, k, g, rng, fpre, rpre);
    } else {
      policy_epilogue<KIND, CRITIC, false, MODE>(a, lg0, v0, env0, env0 < a.E, k, g, rng);
      policy_epilogue<KIND, CRITIC, false, MODE>(a, lg1, v1, env1, env1 < a.E, k, g, rng);
    }
  }
  wait_vmem<0>();  // no LDS-DMA may land after the wave (and its LDS allocation) is gone
}

}  // namespace d2d

using namespace d2d;

// option words set by d2d_set_option from any host thread: relaxed atomics, read once per call
std::atomic<int> g_policy_f32_mfma{0};  // d2d_set_option(D2D_OPT_POLICY_F32_MFMA, 1): fp32-MFMA kernel
#ifndef D2D_POLICY_CRITIC_SPLIT
// the iPPO critic's weight fragments (48 + 16 registers at H = 64) hold the fused actor + critic kernel at two
// waves per SIMD (224 VGPRs; the actor alone: 137); 1 = the value as a separate value-only launch
#define D2D_POLICY_CRITIC_SPLIT 0
#endif
std::atomic<int> g_policy_critic_split{D2D_POLICY_CRITIC_SPLIT};  // d2d_set_option(D2D_OPT_POLICY_CRITIC_SPLIT, v)

template <int KS, int HT>
static int launch_policy_f32(const MlpArgs& a, hipStream_t s) {
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


// Workgroups of kernel K resident on the device at once (its occupancy x the CU count), queried once
template <auto K>
static int resident_blocks() {
  static const int n = [] {  // (a function-local static: initialised once, thread-safe)
    int per = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, K, 256, 0) != hipSuccess) per = 2;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return std::max(1, per * cus);
  }();
  return n;
}
// (A/B) D2D_POLICY_SIZING=r: r resident rounds (0: the 256-envs-per-wave rule only); read once per process
static int policy_sizing() {
  static const int r = [] {
    const char* e = getenv("D2D_POLICY_SIZING");
    return e ? atoi(e) : 1;
  }();
  return r;
}

// envs per wave for one resident round of K (every wave's per-agent weight split amortised over all of its
// tiles, no partial last round)
template <auto K>
static MlpArgs one_round(MlpArgs x) {
  const int rounds = policy_sizing();
  if (rounds <= 0) return x;
  const int64_t per_agent = std::max<int64_t>(1, (int64_t)resident_blocks<K>() * rounds / x.N);
  int64_t epw = ((int64_t)x.E + 4 * per_agent - 1) / (4 * per_agent);
  epw = (epw + 31) / 32 * 32;
  // a wave's row offsets are 32-bit buffer offsets from its first row: epw * N row bytes stay below 2 GiB
  const int64_t rb = x.rec ? 32 * ((x.F + 1 + 31) / 32) : 4 * (int64_t)x.F;
  const int64_t cap = std::max<int64_t>(32, ((int64_t)0x7FF00000 / ((int64_t)x.N * rb)) / 32 * 32);
  x.envs_per_wave = (int)std::max<int64_t>(x.envs_per_wave, std::min(epw, cap));
  return x;
}
template <auto K>
static void launch_one(const MlpArgs& a, hipStream_t s) {
  const MlpArgs x = one_round<K>(a);
  const dim3 grid(x.N, (x.E + 4 * x.envs_per_wave - 1) / (4 * x.envs_per_wave));
  hipLaunchKernelGGL(K, grid, dim3(256), 0, s, x);
}

template <int KC, int HT, int KIND, bool CRITIC, bool U8, int AF>
static void launch_split_af(const MlpArgs& a, hipStream_t s) {
  if (a.forced) launch_one<policy_split_kernel<KC, HT, KIND, CRITIC, kModeForced, U8, AF>>(a, s);
  else if (a.deterministic) launch_one<policy_split_kernel<KC, HT, KIND, CRITIC, kModeDeterministic, U8, AF>>(a, s);
  else launch_one<policy_split_kernel<KC, HT, KIND, CRITIC, kModeSample, U8, AF>>(a, s);
}
#ifndef D2D_POLICY_AFIX
// 1: the record kernels of the combinatorial actor at A = 8 (the benched 8 channels) with the action count compile-time
#define D2D_POLICY_AFIX 1
#endif
template <int KC, int HT, int KIND, bool CRITIC, bool U8>
static void launch_split_fmt(const MlpArgs& a, hipStream_t s) {
  if constexpr (KIND == 0 && U8 && D2D_POLICY_AFIX) {
    if (a.A == 8) return launch_split_af<KC, HT, KIND, CRITIC, U8, 8>(a, s);
  }
  launch_split_af<KC, HT, KIND, CRITIC, U8, 0>(a, s);
}

template <int KC, int HT, int KIND, bool CRITIC, bool U8>
static void launch_split_mode(const MlpArgs& a, hipStream_t s, bool critic_split) {
  if (CRITIC && critic_split) {
    // the actor (actions, log-probs) and the critic value as two launches of the same arithmetic, each at its
    // own occupancy (actor 137 VGPRs, value-only 119, fused 224 at H = 64)
    MlpArgs av = a;
    av.v1 = av.c1 = av.v2 = av.c2 = nullptr;
    launch_split_fmt<KC, HT, KIND, false, U8>(av, s);
    // the value-only launch stores nothing but the value: skipped when the caller passes value = NULL
    // (the fused kernel guards the same store with a.value_out)
    if (a.value_out) launch_one<policy_split_kernel<KC, HT, KIND, true, kModeValue, U8>>(a, s);
    return;
  }
  launch_split_fmt<KC, HT, KIND, CRITIC, U8>(a, s);
}

template <int KC, int HT, int KIND, bool CRITIC>
static void launch_split_kind(const MlpArgs& a, hipStream_t s, bool critic_split) {
  if (a.rec) launch_split_mode<KC, HT, KIND, CRITIC, true>(a, s, critic_split);
  else launch_split_mode<KC, HT, KIND, CRITIC, false>(a, s, critic_split);
}

template <int KC, int HT>
static int launch_policy_split(const MlpArgs& a, hipStream_t s) {
  const bool critic = a.v1 != nullptr;
  const bool cs = g_policy_critic_split.load(std::memory_order_relaxed) != 0;  // one snapshot per call
  if (a.kind == 0 && critic) launch_split_kind<KC, HT, 0, true>(a, s, cs);
  else if (a.kind == 0) launch_split_kind<KC, HT, 0, false>(a, s, cs);
  else if (critic) launch_split_kind<KC, HT, 1, true>(a, s, cs);
  else launch_split_kind<KC, HT, 1, false>(a, s, cs);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

// d2d_policy_mlp_step's argument checks and kernel arguments (also the fused env + policy slot's,
// env_kernels.hip d2d_comb_policy_fused_step)
int d2d::policy_mlp_args(const d2d_mlp_desc* d, const void* obs, const void* forced, uint32_t rng_step,
                         int32_t deterministic, void* actions, float* logp, float* value, MlpArgs& a) {
  // actions may be NULL in forced mode only (the log-probs of given actions: nothing else to write)
  if (!d || !obs || (!actions && !forced) || !logp || !d->w1 || !d->b1 || !d->w2 || !d->b2) {
    d2d_set_error("d2d_policy_mlp_step: NULL argument");
    return D2D_EINVAL;
  }
  if (d->kind != 0 && d->kind != 1) { d2d_set_error("kind must be 0 (Bernoulli) or 1 (Categorical)"); return D2D_EINVAL; }
  if (d->n_out < 1 || d->n_out > 16) { d2d_set_error("n_out=%d outside [1,16]", d->n_out); return D2D_EUNSUPPORTED; }
  if (d->obs_dim < 1 || d->obs_dim > 64) { d2d_set_error("obs_dim=%d outside [1,64]", d->obs_dim); return D2D_EUNSUPPORTED; }
  // hidden <= 128 with one input chunk (F + 1 <= 32), else <= 64
  const int hmax = d->obs_dim + 1 <= 32 ? 128 : 64;
  if (d->hidden < 1 || d->hidden > hmax) {
    d2d_set_error("hidden=%d outside [1,%d] (obs_dim %d)", d->hidden, hmax, d->obs_dim);
    return D2D_EUNSUPPORTED;
  }
  if (d->kind == 0 && d->n_out > 32) { d2d_set_error("too many channels"); return D2D_EUNSUPPORTED; }
  if (d->v1 && (!d->c1 || !d->v2 || !d->c2)) { d2d_set_error("critic needs v1, c1, v2, c2"); return D2D_EINVAL; }
  a = MlpArgs{};
  a.E = d->n_envs; a.N = d->n_agents; a.F = d->obs_dim; a.H = d->hidden; a.A = d->n_out; a.kind = d->kind;
  a.deterministic = deterministic ? 1 : 0;
  a.inv_A = 1.f / (float)a.A;
  // 256 envs (16 tiles) per wave amortise the per-wave weight split; a small batch takes fewer,
  // down to 32 (the tile loop runs tiles in pairs), so that >= 2048 waves (2 per SIMD) fill the chip
  a.envs_per_wave = 256;
  while (a.envs_per_wave > 32 && (int64_t)d->n_envs * d->n_agents / a.envs_per_wave < 2048) a.envs_per_wave >>= 1;
  a.rng_step = rng_step; a.rng_off = d->rng_offset; a.seed = d->seed; a.env_base = d->env_base;
  a.w1 = d->w1; a.b1 = d->b1; a.w2 = d->w2; a.b2 = d->b2; a.v1 = d->v1; a.c1 = d->c1; a.v2 = d->v2; a.c2 = d->c2;
  const int rc = obs_format_args(d->obs_format, d->obs_signed, d->obs_dim, obs, a.obs, a.rec, a.sgn);
  if (rc) return rc;
  a.forced = forced; a.act_out = actions; a.logp_out = logp; a.value_out = value;
  a.mask_bytes = d->n_out <= 8 ? 1 : d->n_out <= 16 ? 2 : 4;
  if (forced && (int64_t)d->n_envs * d->n_agents * a.mask_bytes > 0x7FFFFFFF) {
    // the forced words travel through a buffer descriptor with 32-bit offsets (the DMA ring)
    d2d_set_error("d2d_policy_mlp_step: forced buffer of %lld bytes exceeds 2 GiB",
                  (long long)d->n_envs * d->n_agents * a.mask_bytes);
    return D2D_EUNSUPPORTED;
  }
  return D2D_OK;
}

extern "C" int d2d_policy_mlp_step(const d2d_mlp_desc* d, const void* obs, const void* forced, uint32_t rng_step,
                                   int32_t deterministic, void* actions, float* logp, float* value, void* stream) {
  MlpArgs a;
  if (const int rc = policy_mlp_args(d, obs, forced, rng_step, deterministic, actions, logp, value, a)) return rc;
  if (a.E == 0 || a.N == 0) return D2D_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ht = (a.H + 15) / 16;
  if (g_policy_f32_mfma.load(std::memory_order_relaxed) || a.F + 1 > 64) {
    if (a.rec) { d2d_set_error("the fp32-MFMA policy kernel reads fp32 obs only"); return D2D_EUNSUPPORTED; }
    const int ks = (a.F + 3) / 4;
    if (ks <= 8) return ht <= 2 ? launch_policy_f32<8, 2>(a, s) : ht <= 4 ? launch_policy_f32<8, 4>(a, s)
                                                                      : launch_policy_f32<8, 8>(a, s);
    return ht <= 2 ? launch_policy_f32<16, 2>(a, s) : launch_policy_f32<16, 4>(a, s);
  }
  if (a.F + 1 <= 32)
    return ht <= 2 ? launch_policy_split<1, 2>(a, s) : ht <= 4 ? launch_policy_split<1, 4>(a, s)
                                                               : launch_policy_split<1, 8>(a, s);
  return ht <= 2 ? launch_policy_split<2, 2>(a, s) : launch_policy_split<2, 4>(a, s);
}
