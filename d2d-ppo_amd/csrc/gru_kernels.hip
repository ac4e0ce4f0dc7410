// GRU window policies on gfx950 (gru_common.h has the cell and the layout).
//
// 1. gru_policy_kernel -- the behaviour policy / value of the RNN learners, replacing per agent and
//    per step the reference's batch-1 calls
//      RNN.forward over the history window          /root/reference/algorithms/ippo.py:14-51
//      PPO.select_action / evaluate                 ippo.py:154-191 (d2d_ppo.py:159-196)
//    for every (slot, env, agent) tile of a launch.  Windows are rebuilt in-kernel from the rollout
//    buffer obs[T][E][N][F]: for slot s with episode position p = s % ep_len the window is the last
//    S = min(p + 1, L) obs of the episode, either unpadded (rollout / test: create_rollouts
//    ippo.py:302-304, test ippo.py:362-364) or front-zero-padded to L steps (training:
//    preprocess_input_for_rnn ippo.py:390-403; quirk Q5).  h0 = 0 for every window.
// 2. gru_grad_kernel -- evaluate + clipped-surrogate / MSE loss + backward of PPO.train_step
//    (ippo.py:194-217, d2d_ppo.py:198-216) for GRU policies and the iPPO GRU critic: per 16-sample
//    tile the padded window's forward (hidden states kept in a per-wave global scratch), the head
//    and the loss gradient, then backpropagation through time over the window.  Weight gradients:
//    each BPTT step's gradient / h_{j-1} rows go to a per-wave global history, and per tile two
//    GEMM passes over it (K = window steps x 16 samples) add dW_hh / dW_ih into per-wave sums; the
//    head's gradients are per-wave sums too; one partial per (workgroup, agent), summed in fixed
//    order by gru_reduce_kernel (no atomics).
#include <atomic>
#include <algorithm>
#include <cmath>

#include "gru_common.h"
#include "policy_epilogue.h"
#include "ppo_epilogue.h"

#ifndef D2D_GRU_ABLATE
// != 0 only in tools/gpu/build_ablate_gru.sh's timing builds (wrong gradients by design):
// 1 no weight-gradient GEMMs, 2 no dh MFMAs, 3 no history staging, 4 no BPTT gate recompute
#define D2D_GRU_ABLATE 0
#endif

#ifndef D2D_GRU_DW_BF16
// 1 (default since round 3): the update kernel's weight-gradient GEMMs dW_hh = sum dgh h^T, dW_ih = sum
// dgi x^T on v_mfma_f32_16x16x32_bf16 over two-way RNE splits of the history operands (~2^-17 relative
// per product term, as the MLP update kernels' dW1 / dW2; x is bf16-exact): 60 bf16 MFMAs of 16 cycles
// per step and pass instead of 144 fp32 MFMAs of 32 (298 -> 278 ms per 3.3 M agent-samples,
// profiles/r03).  Round 2 kept it off because one D2D categorical GRU reference trace missed a flat
// 1e-4 final-weight bar (1.5e-4 on one of 768 elements, an element whose gradient is ~0, where Adam's
// normalised step is decided by rounding); the learner parity test now bounds every final weight by
// Adam's own sensitivity to the gradient error the kernels are held to (tests/test_learner_gpu.py
// adam bound), and every GRU gradient / learner / driver test passes on it.  0: v_mfma_f32_16x16x4_f32
// with exact products (fp32 numerics).
#define D2D_GRU_DW_BF16 1
#endif

#ifndef D2D_GRU_DH_BF16
// 1: the BPTT's dh_{j-1} = W_hh^T dg on v_mfma_f32_16x16x32_bf16: the transposed W_hh image holds a
// two-way RNE bf16 split [W_h(4 rows) | W_m(4 rows)] per (unit, gate tile, lane group) -- 16 bytes, the
// same LDS as the fp32 image -- and dg is split two ways per step, so one A fragment serves two MFMAs
// (B = [g_h | g_h] and [g_m | g_m]: W_h g_h + W_m g_h + W_h g_m + W_m g_m, ~2^-16 relative per product).
// 96 bf16 MFMAs of 16 cycles per step instead of 192 fp32 v_mfma_f32_16x16x4_f32 of 32.
// 0: the fp32 MFMAs on the fp32 transposed image (exact products).
#define D2D_GRU_DH_BF16 1
#endif

namespace d2d {

// RNE bf16 pair (lo = a, hi = b) and the residual pair, as two dwords each (the dh GEMM's B operands)
__device__ __forceinline__ uint32_t rne_pair(float a, float b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const bf2 v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ void split2_pairs(const float (&v)[4], uint32_t (&h)[2], uint32_t (&m)[2]) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    h[p] = rne_pair(v[2 * p], v[2 * p + 1]);
    // h << 16 on v_perm_b32: written as a shift, the compiler re-derives it from a second conversion
    m[p] = rne_pair(v[2 * p] - __uint_as_float(__builtin_amdgcn_perm(h[p], h[p], 0x01000c0cu)),
                    v[2 * p + 1] - __uint_as_float(h[p] & 0xFFFF0000u));
  }
}

// Two-way RNE bf16 split of 4 fp32 values as one dword per value, (RNE(v), RNE(v - RNE(v))): the A
// fragment [h0 m0 h1 m1 h2 m2 h3 m3] of k-slots (value q, part p) = 2q + p
__device__ __forceinline__ u32x4v split_pairs(const f32x4 v) {
  u32x4v o;
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    // one conversion rounds both values; their bf16 parts back as fp32 bits on v_perm_b32 / v_and
    const uint32_t h = rne_pair(v[2 * p], v[2 * p + 1]);
    const float r0 = v[2 * p] - ffrom(__builtin_amdgcn_perm(h, h, 0x01000c0cu));
    const float r1 = v[2 * p + 1] - ffrom(h & 0xFFFF0000u);
    const bf2 hm0 = {(__bf16)v[2 * p], (__bf16)r0}, hm1 = {(__bf16)v[2 * p + 1], (__bf16)r1};
    o[2 * p] = __builtin_bit_cast(uint32_t, hm0);
    o[2 * p + 1] = __builtin_bit_cast(uint32_t, hm1);
  }
  return o;
}

struct GruArgs {
  int T, E, N, F, H, A, L, ep_len, kind;
  int slot0, n_slots, padded, env_tiles;  // tiles: slots [slot0, slot0 + n_slots) x ceil(E / 16)
  GruW w;
  ObsView ov;                             // the rollout buffer [T][E][N]: fp32 rows or compact record
  // ---- policy kernel
  MlpArgs ep;                             // epilogue view: ep.E = n_slots * E (slot-major samples)
  float* value_out;                       // kind 2: [N][n_slots * E]
  float* ptab_g;                          // padded windows longer than the LDS table: [G][N][L - 1][HW] (or NULL)
  float* hcarry;                          // one-slot unpadded launches: h after the window, [N][env_tiles][4 HT][64]
  int carry_in;                           // 1: hcarry holds h after slot - 1's window (a prefix of this one)
  // ---- grad kernel
  float clip_lo, clip_hi, beta, scale, inv_A;
  int mask_bytes;
  const void* actions;                    // [T][E][N] masks / ids
  const float* logp_old;                  // element (t, e, k) at t*st[0] + e*st[1] + k*st[2]
  const float* weight;                    // advantage / M (actor) or return target (critic)
  int64_t lo_st[3], w_st[3];
  float* partial;                         // [G][N][P]
  float* hist;                            // [G * N * 4 waves][2 L (COOP + PADC: 3 L)][64 lanes][4 HT] per-wave h scratch
  float* wimg;                            // [N][3 * 16 HT][16 IT] input images (gru_wih_image_kernel)
  float* hacc;                            // [G * N * 4 waves][GruHeadAcc::NV][64] head-gradient sums
  float* himg;                            // [N][HeadImg::SIZE] padded head images (gru_images_kernel)
  float* ghist;                           // [G * N * 4 waves][L][5 HW][16] per-step dgi / dgh_n / h_{j-1} rows
  float* gpart;                           // [G * N * 4 waves][(3 HT (HT + IT)) * 4][64] dW_hh / dW_ih sums
  int G, P;
};

enum { kGruBernoulli = 0, kGruCategorical = 1, kGruValue = 2 };
constexpr int kGruPadTab = 63;  // padding-table steps of the policy kernel (history_len <= 64)
constexpr int kFlushSteps = 64;  // BPTT steps per weight-gradient MFMA accumulation chain (coop_flush)


// ------------------------------------------------------------------------------ policy kernel
// Workgroup = agent k x a strided set of tiles; 8 waves (2 per SIMD), one 16-env tile per wave at a
// time.  LDS: the agent's input and recurrent images (fp32, swizzled; 72 KB at H = 64, F < 32).
// SPLIT: the step on v_mfma_f32_16x16x32_bf16 over exact three-way splits (gru_preact_split; LDS:
// the split images, 108 KB at H = 64, F < 32), else on v_mfma_f32_16x16x4_f32 (gru_preact).  Plus the
// head image and the 16 KB padding table of padded windows: 147.5 KB at H = 64.
template <int HT, int IT, int KIND, int MODE, bool SPLIT>
__global__ __launch_bounds__(512, 1) void gru_policy_kernel(GruArgs a) {
  constexpr int HW = 16 * HT, IW = 16 * IT, R3 = 3 * HW;
  using SP = GruSplit<HT, IT>;
  constexpr int IMG_BYTES = SPLIT ? 16 * (SP::WIH + SP::WHH) : 4 * (R3 * IW + R3 * HW);
  __shared__ __attribute__((aligned(16))) unsigned char img_raw[IMG_BYTES];
  float* wih_s = reinterpret_cast<float*>(img_raw);
  float* whh_s = wih_s + R3 * IW;
  bf16x8* wih_b = reinterpret_cast<bf16x8*>(img_raw);
  bf16x8* whh_b = wih_b + SP::WIH;
  __shared__ float head_s[HeadImg<HT>::SIZE];
  const int k = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, F = a.F, N = a.N, E = a.E;
  if constexpr (SPLIT) load_gru_split_images<HT, IT>(wih_b, whh_b, a.w, k, H, F, tid, blockDim.x);
  else load_gru_images<HT, IT>(wih_s, whh_s, a.w, k, H, F, tid, blockDim.x);
  for (int idx = tid; idx < HeadImg<HT>::SIZE; idx += blockDim.x)
    head_s[idx] = head_img_elem<HT>(a.w, k, H, KIND == kGruValue ? 1 : a.A, idx);
  f32x4 bhn[HT];
  load_bhn<HT>(bhn, a.w, k, H, g);
  const uint32_t rng = (MODE == kModeSample && a.ep.rng_off) ? a.ep.rng_step + *a.ep.rng_off : a.ep.rng_step;
  const SwzOff<IW> oi(g, i);
  const SwzOff<HW> oh(g, i);
  const XSigns<IT> xsg(a.ov, k);
  // Padded (training) windows: the front-padding steps (x = the bias input only, h0 = 0) give the same
  // h_j for every sample, so wave 0 runs them once into an LDS table -- the very instructions and data
  // of any tile's padding steps, so bitwise the same h -- and tiles start their window at step pad.
  __shared__ float ptab_s[kGruPadTab * HW];  // [step j][unit]: h after j + 1 padding steps
  const bool use_tab = a.padded && a.L - 1 <= kGruPadTab;
  // longer windows (xp_n_agents: history_len = N up to 256) keep the table in global memory, one per workgroup
  // (a tile reads one row of it: h after its pad steps); without it every tile ran its pad steps itself
  const bool use_gtab = a.padded && !use_tab && a.ptab_g;
  float* gtab = use_gtab ? a.ptab_g + ((size_t)blockIdx.y * gridDim.x + k) * (size_t)(a.L - 1) * HW : nullptr;
  if ((use_tab || use_gtab) && wave == 0) {
    float h[HT][4];
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) h[t][r] = 0.f;
    for (int j = 0; j + 1 < a.L; ++j) {
      XRaw<IT> xr;
      load_x_raw<IT>(xr, a.ov, 0, g, i, false, true);  // a padding step: nothing is read
      float x[IT][4];
      decode_x<IT>(x, xr, a.ov, xsg, g);
      f32x4 rz[2 * HT], ni[HT], nh[HT];
      const int z = opaque_zero();
      if constexpr (SPLIT)
        gru_preact_split<HT, IT>(wih_b + z, whh_b + z, lane, x, x_exact_step<IT>(a.ov, x), h, bhn, rz, ni, nh, j == 0);
      else
        gru_preact<HT, IT, true>(wih_s + z, whh_s + z, oi, oh, x, h, bhn, rz, ni, nh, g, i, j == 0);
      gru_gates<HT>(rz, ni, nh, h);
      if (i == 0) {  // every sample lane holds the same h: lanes (g, 0) write units 16t + 4g + r
#pragma unroll
        for (int t = 0; t < HT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) (use_tab ? ptab_s : gtab)[(size_t)j * HW + 16 * t + 4 * g + r] = h[t][r];
      }
    }
  }
  __syncthreads();

  const int n_tiles = a.n_slots * a.env_tiles;
  const int nw = gridDim.y * (blockDim.x >> 6);
  for (int tile = blockIdx.y * (blockDim.x >> 6) + wave; tile < n_tiles; tile += nw) {  // wave-uniform
    const int sl = tile / a.env_tiles;
    const int slot = a.slot0 + sl;
    const int e0 = (tile - sl * a.env_tiles) * 16;
    const int env = e0 + i;
    const bool ok = env < E;
    const int pos = slot % a.ep_len;
    const int S = min(pos + 1, a.L);
    const int lo = slot - S + 1;
    const int pad = a.padded ? a.L - S : 0;
    const int j0 = use_tab || use_gtab ? pad : 0;  // the first step computed here (steps j < j0: the padding table)
    float h[HT][4];
    const float* hrow = use_tab ? ptab_s : gtab;
    // carried state (rollout / test windows, one slot per launch): while pos < L the window of slot s is the window
    // of slot s - 1 plus obs_s, so h after slot s - 1's window (hcarry, written by the previous launch) enters the
    // window's last step -- the same h the recompute reaches, hence bitwise the same step and head
    float* hc = a.hcarry ? a.hcarry + ((size_t)k * a.env_tiles + (size_t)(e0 >> 4)) * (4 * HT * 64) + lane : nullptr;
    const bool cin = hc && a.carry_in;
    const int j1 = cin ? S - 1 : j0;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        h[t][r] = cin ? hc[(4 * t + r) * 64] : j0 > 0 ? hrow[(size_t)(j0 - 1) * HW + 16 * t + 4 * g + r] : 0.f;
    // the window step's x tile is loaded one step ahead (its latency hides behind a step's MFMAs)
    float x[IT][4];
    XRaw<IT> xn;
    auto load_step = [&](int j) {
      const bool zero = j < pad;
      const int row_slot = zero ? lo : lo + (j - pad);
      load_x_raw<IT>(xn, a.ov, ((size_t)row_slot * E + e0) * N + k, g, i, ok, zero);
    };
    load_step(j1);
    for (int j = j1; j < pad + S; ++j) {
      decode_x<IT>(x, xn, a.ov, xsg, g);
      if (j + 1 < pad + S) load_step(j + 1);
      f32x4 rz[2 * HT], ni[HT], nh[HT];
      const int z = opaque_zero();
      if constexpr (SPLIT) {
        // every input bf16-exact (record bytes, integer fp32 rows): three weight-part products only
        gru_preact_split<HT, IT>(wih_b + z, whh_b + z, lane, x, x_exact_step<IT>(a.ov, x), h, bhn, rz, ni, nh, j == 0);
      } else {
        gru_preact<HT, IT, true>(wih_s + z, whh_s + z, oi, oh, x, h, bhn, rz, ni, nh, g, i, j == 0);
      }
      gru_gates<HT>(rz, ni, nh, h);
    }
    if (hc && pos + 1 < a.L) {  // the next slot's window extends this one: carry h (coalesced, one dword per lane)
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) hc[(4 * t + r) * 64] = h[t][r];
    }
    f32x4 pre1[HT], lg;
    float y[HT][4];
    gru_head<HT>(head_s + opaque_zero(), h, pre1, y, lg, g, i);
    const int samp = sl * E + env;  // slot-major sample index of the launch
    if constexpr (KIND == kGruValue) {
      if (ok && g == 0) a.value_out[(size_t)k * a.ep.E + samp] = lg[0];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) lg[r] *= kLog2e;
      // HALF = false: every lane group holds 4 outputs of the same sample
      policy_epilogue<KIND == kGruBernoulli ? 0 : 1, false, false, MODE, false, KIND == kGruBernoulli>(
          a.ep, lg, 0.f, samp, ok, k, g, rng);
    }
  }
}


// -------------------------------------------------------------------------------- grad kernel
// Per-wave LDS scratch: accumulator-layout columns (one sample per lane i) written so that the MFMA
// k axis runs over samples: row-major [rows][16], sample e at column pcol(e) = 4 (e & 3) + (e >> 2),
// so the ds_read_b128 of lane (g, i) at columns [4g, 4g + 4) yields samples 4s + g for k-steps
// s = 0..3 (the A fragment of row `row`, or the B fragment of column `row`).
__device__ __forceinline__ int pcol(int e) { return ((e & 3) << 2) | (e >> 2); }
__device__ __forceinline__ f32x4 sc_frag(const float* sc, int row, int g) {
  return *reinterpret_cast<const f32x4*>(sc + row * 16 + 4 * g);
}

// Per-sample epilogue inputs of a tile (every lane group holds its sample's values).
struct GruIn {
  uint32_t act;
  float lo, w;
};

template <int KIND>
__device__ __forceinline__ GruIn load_gru_in(const GruArgs& a, int t, int env, int k, bool ok) {
  GruIn in{0u, 0.f, 0.f};
  const int e = ok ? env : 0;
  in.w = a.weight[(int64_t)t * a.w_st[0] + (int64_t)e * a.w_st[1] + (int64_t)k * a.w_st[2]];
  if constexpr (KIND != kGruValue) {
    const size_t cell = ((size_t)t * a.E + e) * a.N + k;
    in.act = KIND == kGruCategorical ? reinterpret_cast<const unsigned char*>(a.actions)[cell]
                                     : load_mask(a.actions, cell, a.mask_bytes);
    in.lo = a.logp_old[(int64_t)t * a.lo_st[0] + (int64_t)e * a.lo_st[1] + (int64_t)k * a.lo_st[2]];
  }
  return in;
}

// Register partial sums of one wave, flattened for the cross-wave reduction.  The head's gradients
// (layers.0 / layers.2, once per window) are accumulated in a per-wave global block instead
// (GruHeadAcc, read-modify-write per tile), which keeps the BPTT loop within the register file.
template <int HT, int IT>
struct GruAcc {
  f32x4 wih[3 * HT][IT];   // dW_ih (+ bias column F): D[gate row 16T + 4g + r][input 16U + i]
  float bhn[HT][4];        // per-sample-lane partial sums of dL/db_hn (unit 16t + 4g + r)
  float st[2];             // loss sums
  static constexpr int NV = 3 * HT * IT * 4 + HT * 4 + 2;
  template <class Fn>
  __device__ __forceinline__ void each(Fn fn) {
    int v = 0;
#pragma unroll
    for (int T = 0; T < 3 * HT; ++T)
#pragma unroll
      for (int U = 0; U < IT; ++U)
#pragma unroll
        for (int r = 0; r < 4; ++r) { float x = wih[T][U][r]; fn(v++, x); wih[T][U][r] = x; }
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) fn(v++, bhn[t][r]);
    fn(v++, st[0]);
    fn(v++, st[1]);
  }
};

// Register partial sums that stay in the BPTT loop: dL/db_hn lanes and the loss sums (dW_ih, dW_hh
// are per-tile GEMMs over the step history, GruWAcc).
template <int HT>
struct GruSAcc {
  float bhn[HT][4];
  float st[2];
  static constexpr int NV = HT * 4 + 2;
  template <class Fn>
  __device__ __forceinline__ void each(Fn fn) {
    int v = 0;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) fn(v++, bhn[t][r]);
    fn(v++, st[0]);
    fn(v++, st[1]);
  }
};
// Per-wave global sums of the recurrent / input weight gradients, [v][64 lanes]: dW_hh tiles
// D[gate row 16T + 4g + r][unit 16U + i] at v = (T HT + U) 4 + r, then dW_ih tiles D[gate row][input
// 16U + i] at WI + (T IT + U) 4 + r (the bias column F included).
template <int HT, int IT>
struct GruWAcc {
  static constexpr int WI = 3 * HT * HT * 4, NV = WI + 3 * HT * IT * 4;
};

// Head gradients of one wave in global memory, [v][64 lanes] (coalesced): dW1 tiles
// D[unit 16t + 4g + r][unit 16U + i], dW2 tiles D[output 4g + r][unit 16U + i], and per-sample-lane
// partial sums of db1 (unit 16t + 4g + r) and db2 (output 4g + r).
template <int HT>
struct GruHeadAcc {
  static constexpr int W1 = 0, W2 = HT * HT * 4, B1 = W2 + HT * 4, B2 = B1 + HT * 4, NV = B2 + 4;
};

// base[(v0 + v) * 64 + lane] += d[v] for a block of per-lane sums: every old value is loaded before
// any is written back (one memory wait for the block)
template <int NV>
__device__ __forceinline__ void rmw_block(float* base, int lane, int v0, const float (&d)[NV]) {
  float old[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) old[v] = base[(v0 + v) * 64 + lane];
#pragma unroll
  for (int v = 0; v < NV; ++v) base[(v0 + v) * 64 + lane] = old[v] + d[v];
}

// Partial layout per (workgroup, agent): the gradient of every torch tensor of the RNN module
// (StackedNets "rnn": w_ih, w_hh, b_ih, b_hh, layers.0 w/b, layers.2 w/b), then the 2 loss sums.
struct GruOff {
  int wih, whh, bih, bhh, w1, b1, w2, b2, st, P;
  __device__ __host__ GruOff(int H, int F, int A) {
    wih = 0; whh = 3 * H * F; bih = whh + 3 * H * H; bhh = bih + 3 * H; w1 = bhh + 3 * H; b1 = w1 + H * H;
    w2 = b1 + H; b2 = w2 + A * H; st = b2 + A; P = st + 2;
  }
};

// COOP (H in (32, 64], compact-record inputs, F + 1 <= 48): the weight gradients without
// the global row history.  The four waves run their tiles' BPTT steps in lockstep; every step each wave
// in turn writes its 16 samples' rows -- the r, z, n_in and n_h pre-activation gradients and h_{j-1} as
// RNE two-way bf16 split planes, x (bf16-exact) as one -- into ONE shared LDS region, and all four waves
// accumulate their share of the dW_hh / dW_ih output tiles from it (wave w: hidden tile w of the r, z,
// n gates, every column tile; 12 + 3 IT accumulator tiles held for the whole kernel).  The history's
// 2.6 MB of HBM traffic per tile and the per-tile read-modify-writes of the wave sums are gone; the
// products are the bf16 path's (a_h b_h + a_m b_h + a_h b_m, x exact), summed in a fixed order.
// Region layout (bf16 elements): planes p = 0..9 (r h/m, z h/m, n_in h/m, n_h h/m, h_{j-1} h/m) of
// [16 samples][64 rows], then x [16 samples][16 IT]; 4-element quads XOR-swizzled by sample so that
// both the writers (ds_write_b64: 4 rows of one sample) and the transposing readers
// (ds_read_b64_tr_b16: 4 samples of one row per lane) touch every bank pair at most twice per wave.
template <int IT>
struct CoopRegion {
  static constexpr int PLANE = 16 * 64, X = 10 * PLANE, ELEMS = X + 16 * 16 * IT, BYTES = 2 * ELEMS;
};
__device__ __forceinline__ int coop_off(int plane, int s, int c) {
  return plane * 1024 + s * 64 + (c ^ (((s >> 1) & 3) << 4));
}
template <int IT>
__device__ __forceinline__ int coop_xoff(int s, int c) {  // (the swizzle needs a power-of-two row of >= 32)
  return CoopRegion<IT>::X + s * 16 * IT + (IT == 2 || IT == 4 ? (c ^ (((s >> 2) & 1) << 4)) : c);
}
typedef short v4i16_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16_t* lds_v4i16_t;
// 4 samples (4g .. 4g + 3) of row `col` (16-column block base + i) of a plane: two dwords
__device__ __forceinline__ uint2 coop_tr(const uint16_t* reg, int off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t)(reg + off)));
}
__device__ __forceinline__ bf16x8 cat2(uint2 a, uint2 b) {
  const u32x4v v = {a.x, a.y, b.x, b.y};
  return __builtin_bit_cast(bf16x8, v);
}
// The A operand of dh = W_hh^T dg for unit tile t and gate tile T, [W_h x4 | W_m x4] of lane (g, i) =
// W_hh[gate row 16T + 4g + r][unit 16t + i], r = 0..3 -- two transposing reads of the FORWARD split
// image (split3_rne: its h, m parts are the RNE two-way split).  The forward fragment (T, c = t / 2)
// holds W_hh[16T + i_f][unit 16 (2c + j / 4) + 4 g_f + j % 4] at slot 16 g_f + i_f, element j; output
// element r of lane (g, i) comes from the chunk (8-byte half t % 2, element i & 3) addressed by lane
// (g, 4r + (i >> 2)), so lane (g, L) addresses slot 16 (L & 3) + 4g + (L >> 2) (swizzled, whh_slot).
template <int HT>
__device__ __forceinline__ bf16x8 whh_dh_frag(const bf16x8* whh_b, int T, int t, int g, int i) {
  constexpr int CH = (HT + 1) / 2;
  const int slot = whh_slot(16 * (i & 3) + 4 * g + (i >> 2));
  const uint16_t* base = reinterpret_cast<const uint16_t*>(whh_b + ((T * CH + (t >> 1)) * 3) * 64 + slot) + 4 * (t & 1);
  return cat2(coop_tr(base, 0), coop_tr(base, 64 * 8));  // part h, then part m (64 words on)
}

// Workgroup = agent k x a strided set of 16-sample tiles; 4 waves (one per SIMD).
// LDS (H = 64, !SPLIT): W_hh image 48 KB (forward A fragments) + its transpose 49 KB (the A fragments
// of dh = W_hh^T dg, one ds_read_b128 per 4 MFMAs) + 4 x 12 KB wave scratch = 145 KB (SPLIT: below).
// The weight gradients dW_hh = sum_j dgh_j h_{j-1}^T and dW_ih = sum_j dgi_j x_j^T are not summed
// step by step (that took one LDS atomic per element per step, ~40 % of the LDS issue): every step
// writes its dgi / dgh_n / h_{j-1} rows (sample-on-k layout, through the wave's LDS scratch) to a
// per-wave global history, and after the window one GEMM per tile with K = L x 16 accumulates them
// in registers and adds them into the wave's global sums -- deterministic (no atomics anywhere).
// SPLIT (default): the forward and the BPTT recompute on the policy kernel's split step
// (gru_preact_split: the 74 KB split W_hh image in LDS, the split W_ih image from L2); the scratch is
// then 2 HW rows per wave (the step's gradient rows leave it in three passes), 155 KB in all.
// LONGW (COOP): windows longer than kFlushSteps steps, the cooperative accumulators flushed every kFlushSteps
//
// PADC (COOP, D2D_GRU_PAD_COLLAPSE): the BPTT of the front-padding region once per wave instead of once per
// tile.  A padding step j < pad has the same h_{j-1} (the padding table), the same x (the bias input) and
// hence the same gates for every sample, so the backward through the padding region is one LINEAR map of
// dh_{pad-1}, the same for every sample, and so are the weight-gradient rows it produces (dg (x) h_{j-1},
// dg (x) x, dgh_n).  A tile's BPTT therefore stops at jlo (the smallest pad of the workgroup's four tiles
// of the round: they step in lockstep), adds its dh_{jlo-1} into the wave's entry sums ent[jlo-1], and one
// extra all-padding pass after the last round runs j = L-2 .. 0 once with dh += ent[j] at each step.
// Exact in real arithmetic; in fp32 only the summation order of the padding rows' contributions changes.
// Saves the padding steps' share of the BPTT: ~16 % at L = 64 (ep_len 200), ~60 % at L = 256.
#ifndef D2D_GRU_PAD_COLLAPSE
#define D2D_GRU_PAD_COLLAPSE 1
#endif
template <int HT, int IT, int KIND, bool SPLIT, bool COOP = false, bool LONGW = false>
__global__ __launch_bounds__(256, 1) void gru_grad_kernel(GruArgs a) {
  constexpr int HW = 16 * HT, R3 = 3 * HW, RT = R3 + 4, SROWS = 2 * HW;
  constexpr bool PADC = COOP && D2D_GRU_PAD_COLLAPSE != 0;
  static_assert(!COOP || (HT == 4 && SPLIT && D2D_GRU_DH_BF16), "COOP: H in (32, 64], the split step, bf16 dh");
  static_assert(COOP || !LONGW, "LONGW: the cooperative path");
  using SP = GruSplit<HT, IT>;
  using CR = CoopRegion<IT>;
  __shared__ __attribute__((aligned(16))) unsigned char whh_raw[SPLIT ? 16 * SP::WHH : 4 * R3 * HW];
  float* whh_s = reinterpret_cast<float*>(whh_raw);
  bf16x8* whh_b = reinterpret_cast<bf16x8*>(whh_raw);
  // [unit u][gate row R], row stride R3 + 4 (COOP: none, the dh operands come from whh_b, whh_dh_frag)
  __shared__ __attribute__((aligned(16))) float whhT_s[COOP ? 4 : HW * RT];
  // COOP: one staging region per wave (also its head-phase scratch; region 0 the final reduction
  // buffer) instead of the per-wave scratch blocks
  __shared__ __attribute__((aligned(16))) float scr[COOP ? 1 : 4][COOP ? 4 : SROWS * 16];
  __shared__ __attribute__((aligned(16))) unsigned char creg_raw[COOP ? 4 * CR::BYTES : 16];
  static_assert(!COOP || CR::BYTES >= SROWS * 16 * 4, "COOP region holds the head scratch");
  const int k = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, F = a.F, N = a.N, E = a.E, A = KIND == kGruValue ? 1 : a.A, L = a.L;
  uint16_t* creg = reinterpret_cast<uint16_t*>(creg_raw);
  float* sc = COOP ? reinterpret_cast<float*>(creg_raw + wave * CR::BYTES) : scr[COOP ? 0 : wave];
  // DH_BF16: the transposed image as 16-byte entries [unit u][gate tile T * 4 + lane group][W_h x4 | W_m x4],
  // TE entries per unit row (one of padding: the 16 lanes' A-fragment reads hit distinct banks)
  constexpr int TE = 3 * HT * 4 + 1;
  static_assert(HW * TE * 16 <= HW * RT * 4, "bf16 transposed image exceeds the fp32 one");
  {
    const float* Whh = a.w.w_hh + (size_t)k * 3 * H * H;
    for (int idx = tid; idx < R3 * HW; idx += blockDim.x) {
      const int R = idx / HW, c = idx - R * HW, G = R / HW, u = R - G * HW;
      const float v = (u < H && c < H) ? Whh[(size_t)(G * H + u) * H + c] : 0.f;
      if constexpr (!SPLIT) whh_s[swz<HW>(R, c)] = v;
      if (!D2D_GRU_DH_BF16) whhT_s[c * RT + R] = v;
    }
#if D2D_GRU_DH_BF16
    bf16x8* whhTb = reinterpret_cast<bf16x8*>(whhT_s);
    for (int idx = tid; idx < (COOP ? 0 : HW * 3 * HT * 4); idx += blockDim.x) {
      const int c = idx / (3 * HT * 4), rem = idx - c * (3 * HT * 4), T = rem >> 2, gg = rem & 3;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = 16 * T + 4 * gg + r, G = R / HW, u = R - G * HW;
        v[r] = (u < H && c < H) ? Whh[(size_t)(G * H + u) * H + c] : 0.f;
      }
      uint32_t hw[2], mw[2];
      split2_pairs(v, hw, mw);
      const u32x4v e = {hw[0], hw[1], mw[0], mw[1]};
      whhTb[c * TE + T * 4 + gg] = __builtin_bit_cast(bf16x8, e);
    }
#endif
    if constexpr (SPLIT) load_gru_split_images<HT, IT, COOP>(nullptr, whh_b, a.w, k, H, F, tid, blockDim.x);
  }
  f32x4 bhn[HT];
  load_bhn<HT>(bhn, a.w, k, H, g);
  GruSAcc<HT> acc;
  acc.each([](int, float& x) { x = 0.f; });
  using HI = HeadImg<HT>;
  const float* himg = a.himg + (size_t)k * HI::SIZE;  // padded head image (gru_images_kernel)
  // the input image of gru_common.h (bias column F) written by gru_wih_image_kernel: A fragments
  // straight from L2 every step (registers are the update kernel's scarce resource)
  const float* wimg = a.wimg + (size_t)k * 3 * HW * (16 * IT);
  const bf16x8* wih_g = reinterpret_cast<const bf16x8*>(a.wimg) + (size_t)k * SP::WIH;  // SPLIT: split image
  const SwzOff<16 * IT> oi(g, i);  // (unused: W_ih comes from the global image)
  const SwzOff<HW> oh(g, i);
  const XSigns<IT> xsg(a.ov, k);
  const size_t wave_id = (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave;
  // per wave: [0, L) the tile's h_j, [L, 2L) the front-padding table: h after j + 1 all-padding steps,
  // (PADC) [2L, 3L) the padding-region entry sums: ent[j] = sum of dh_j over the tiles whose BPTT stopped at j + 1
  float* hist = a.hist + wave_id * (size_t)(PADC ? 3 : 2) * L * 64 * 4 * HT;
  float* ptab = hist + (size_t)L * 64 * 4 * HT;
  float* ent = ptab + (size_t)L * 64 * 4 * HT;
  if constexpr (PADC)
    for (int j = 0; j < L; ++j)
#pragma unroll
      for (int t = 0; t < HT; ++t) reinterpret_cast<f32x4*>(ent + ((size_t)j * 64 + lane) * 4 * HT)[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* hacc = a.hacc + wave_id * (size_t)GruHeadAcc<HT>::NV * 64;
  for (int v = 0; v < GruHeadAcc<HT>::NV; ++v) hacc[v * 64 + lane] = 0.f;
  using WA = GruWAcc<HT, IT>;
  float* ghist = a.ghist + wave_id * (size_t)L * 5 * HW * 16;
  // per-wave weight-gradient sums in global memory: the row-history GEMMs' (!COOP), or (COOP) the
  // running sums the cooperative accumulators are flushed into after every tile
  constexpr int NVC = (3 * HT + 3 * IT) * 4;  // COOP: this wave's 3 HT + 3 IT output tiles, 4 values per lane
  float* gpart = a.gpart + wave_id * (size_t)(COOP ? NVC : WA::NV) * 64;
  for (int v = 0; v < (COOP ? NVC : WA::NV); ++v) gpart[v * 64 + lane] = 0.f;
  // COOP: this wave's output tiles, all tiles of the kernel: dW_hh [gate g3][column tile U] and dW_ih
  // [g3][input tile U] of gate rows 16 (4 g3 + wave) + 4g + r
  f32x4 cwh[COOP ? 3 : 1][COOP ? HT : 1], cwi[COOP ? 3 : 1][COOP ? IT : 1];
  if constexpr (COOP) {
#pragma unroll
    for (int g3 = 0; g3 < 3; ++g3) {
#pragma unroll
      for (int U = 0; U < HT; ++U) cwh[g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int U = 0; U < IT; ++U) cwi[g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  // COOP: add the accumulators into the wave's running sums and restart them.  After every tile, and inside
  // a window every kFlushSteps BPTT steps: one MFMA chain over a whole L = 256 window (64 L terms) measured
  // 100x torch fp32's error against float64 at 256 agents (tests/test_gru_gpu.py::test_gru_grads_long_window);
  // windows of <= kFlushSteps steps (xp_load's 64) flush exactly as before
  auto coop_flush = [&]() {
    if constexpr (COOP) {
      float d[NVC];
      int v = 0;
#pragma unroll
      for (int g3 = 0; g3 < 3; ++g3) {
#pragma unroll
        for (int U = 0; U < HT; ++U)
#pragma unroll
          for (int r = 0; r < 4; ++r) d[v++] = cwh[g3][U][r];
#pragma unroll
        for (int U = 0; U < IT; ++U)
#pragma unroll
          for (int r = 0; r < 4; ++r) d[v++] = cwi[g3][U][r];
      }
      rmw_block(gpart, lane, 0, d);
#pragma unroll
      for (int g3 = 0; g3 < 3; ++g3) {
#pragma unroll
        for (int U = 0; U < HT; ++U) cwh[g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int U = 0; U < IT; ++U) cwi[g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  __syncthreads();

  // The front-padding steps of a training window (x = the bias input only, h0 = 0) give the same h_j
  // for every sample: the wave runs them once here -- the very instructions and data of any tile's
  // padding steps, so bitwise the same h -- and its tiles start their forward at step pad.
  for (int j = 0; j + 1 < L; ++j) {
    float h[HT][4];
    if (j == 0) {
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) h[t][r] = 0.f;
    } else {
      const f32x4* src = reinterpret_cast<const f32x4*>(ptab + ((size_t)(j - 1) * 64 + lane) * 4 * HT);
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        const f32x4 v = src[t];
#pragma unroll
        for (int r = 0; r < 4; ++r) h[t][r] = v[r];
      }
    }
    XRaw<IT> xr;
    load_x_raw<IT>(xr, a.ov, 0, g, i, false, true);  // a padding step: nothing is read
    float x[IT][4];
    decode_x<IT>(x, xr, a.ov, xsg, g);
    f32x4 rz[2 * HT], ni[HT], nh[HT];
    const int z = opaque_zero();
    if constexpr (SPLIT)
      gru_preact_split<HT, IT, COOP>(wih_g + z, whh_b + z, lane, x, x_exact_step<IT>(a.ov, x), h, bhn, rz, ni, nh, j == 0);
    else
      gru_preact<HT, IT, false>(wimg + z, whh_s + z, oi, oh, x, h, bhn, rz, ni, nh, g, i, j == 0);
    gru_gates<HT>(rz, ni, nh, h);
    f32x4* dst = reinterpret_cast<f32x4*>(ptab + ((size_t)j * 64 + lane) * 4 * HT);
#pragma unroll
    for (int t = 0; t < HT; ++t) dst[t] = f32x4{h[t][0], h[t][1], h[t][2], h[t][3]};
  }

  const int n_tiles = a.T * a.env_tiles;
  // COOP: block-uniform rounds (the waves' BPTT steps meet at barriers); a wave without a tile in the
  // last round runs an all-invalid tile (every sample masked: zero gradient rows) through the barriers
  const int rounds = (n_tiles + 4 * (int)gridDim.y - 1) / (4 * (int)gridDim.y);
  // PADC: round `rounds` is the padding-region pass (block-uniform, every wave)
  auto pad_of = [&](int tl) { return L - min((tl < n_tiles ? tl / a.env_tiles : 0) % a.ep_len + 1, L); };
  for (int rnd = 0; COOP ? rnd < rounds + (PADC ? 1 : 0) : true; ++rnd) {
    const bool ppass = PADC && rnd == rounds;
    const int tbase = (rnd * (int)gridDim.y + (int)blockIdx.y) * 4;
    const int tile = tbase + wave;  // wave-uniform
    if (!COOP && tile >= n_tiles) break;
    const bool active = !ppass && tile < n_tiles;
    const int slot = active ? tile / a.env_tiles : 0;
    const int e0 = active ? (tile - slot * a.env_tiles) * 16 : 0;
    const int env = e0 + i;
    const bool ok = active && env < E;
    const int pos = slot % a.ep_len;
    const int S = min(pos + 1, L);
    const int lo = slot - S + 1;
    // training windows: front-zero-padded to L (preprocess_input_for_rnn); the padding pass: all padding
    const int pad = ppass ? L : L - S;
    // PADC: this round's BPTT stops at jlo, the smallest pad of the workgroup's four tiles (inactive tiles: any)
    const int jlo = PADC && !ppass ? min(min(pad_of(tbase), pad_of(tbase + 1)), min(pad_of(tbase + 2), pad_of(tbase + 3)))
                                   : 0;
    const GruIn in = active ? load_gru_in<KIND>(a, slot, env, k, ok) : GruIn{0u, 0.f, 0.f};
    auto row_of = [&](int j) { return ((size_t)(j < pad ? lo : lo + j - pad) * E + e0) * N + k; };

    float gcur[HT][4];
    if (ppass) {
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) gcur[t][r] = 0.f;
    } else {
    // ---- forward over the window; h_j (j < L - 1) to the wave's scratch
    // (steps j < pad: the padding table)
    float h[HT][4];
    if (pad == 0) {
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) h[t][r] = 0.f;
    } else {
      const f32x4* src = reinterpret_cast<const f32x4*>(ptab + ((size_t)(pad - 1) * 64 + lane) * 4 * HT);
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        const f32x4 v = src[t];
#pragma unroll
        for (int r = 0; r < 4; ++r) h[t][r] = v[r];
      }
    }
    XRaw<IT> xn;  // the next step's x tile, loaded one step ahead
    load_x_raw<IT>(xn, a.ov, row_of(pad), g, i, ok, false);
    for (int j = pad; j < L; ++j) {
      float x[IT][4];
      decode_x<IT>(x, xn, a.ov, xsg, g);
      if (j + 1 < L) load_x_raw<IT>(xn, a.ov, row_of(j + 1), g, i, ok, j + 1 < pad);
      f32x4 rz[2 * HT], ni[HT], nh[HT];
      const int z = opaque_zero();
      if constexpr (SPLIT)
        gru_preact_split<HT, IT, COOP>(wih_g + z, whh_b + z, lane, x, x_exact_step<IT>(a.ov, x), h, bhn, rz, ni, nh, j == 0);
      else
        gru_preact<HT, IT, false>(wimg + z, whh_s + z, oi, oh, x, h, bhn, rz, ni, nh, g, i, j == 0);
      gru_gates<HT>(rz, ni, nh, h);
      if (j + 1 < L) {
        f32x4* dst = reinterpret_cast<f32x4*>(hist + ((size_t)j * 64 + lane) * 4 * HT);
#pragma unroll
        for (int t = 0; t < HT; ++t) dst[t] = f32x4{h[t][0], h[t][1], h[t][2], h[t][3]};
      }
    }

    // ---- head forward + loss gradient w.r.t. the head outputs (COOP: the scratch is the wave's region)
    auto head_phase = [&]() {
    f32x4 pre1[HT], lg;
    float y[HT][4];
    const float* hi_ = himg + opaque_zero();
    gru_head<HT>(hi_, h, pre1, y, lg, g, i);
    f32x4 dlg;
    if constexpr (KIND == kGruValue) {
      const float d = lg[0] - in.w;  // V - R
      acc.st[0] += (ok && g == 0) ? d * d : 0.f;
      dlg = f32x4{(ok && g == 0) ? 2.f * a.scale * d : 0.f, 0.f, 0.f, 0.f};
    } else {
      dlg = ppo_dz<KIND == kGruBernoulli ? 0 : 1, false, KIND == kGruBernoulli>(a, lg, in.act, in.lo, in.w, ok, g,
                                                                                  acc.st[0], acc.st[1]);
    }

    // ---- head backward.  dW2 += dlg y^T, db2, dy = W2^T dlg, dpre1 = dy [pre1 > 0]; dW1 += dpre1 h_L^T,
    // db1; dh_L = W1^T dpre1.  The head's gradient sums are read-modified-written in the wave's global block.
    // (the per-tile sums are batched: a block's old values are all loaded before any is written back,
    // one memory wait per block instead of one per value)
    using HA = GruHeadAcc<HT>;
    static_assert(HA::B1 == HA::W2 + 4 * HT && HA::B2 == HA::B1 + 4 * HT, "head sums: W2 | b1 | b2 contiguous");
    float hd[8 * HT + 4];  // this tile's dW2 (4U + r), db1 (4HT + 4t + r), db2 (8HT + r)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[(4 * g + r) * 16 + pcol(i)] = dlg[r];
      hd[8 * HT + r] = dlg[r];
#pragma unroll
      for (int t = 0; t < HT; ++t) sc[(16 + 16 * t + 4 * g + r) * 16 + pcol(i)] = y[t][r];
    }
    lds_order();
    {
      const f32x4 af = sc_frag(sc, i, g);
#pragma unroll
      for (int U = 0; U < HT; ++U) {
        const f32x4 bf = sc_frag(sc, 16 + 16 * U + i, g);
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) d = mfma4(af[s4], bf[s4], d);
#pragma unroll
        for (int r = 0; r < 4; ++r) hd[4 * U + r] = d[r];
      }
    }
    float dpre1[HT][4];
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      f32x4 dy = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) dy = mfma4(hi_[HI::W2 + (4 * g + s4) * HW + 16 * t + i], dlg[s4], dy);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dpre1[t][r] = pre1[t][r] > 0.f ? dy[r] : 0.f;
        hd[4 * HT + 4 * t + r] = dpre1[t][r];
      }
    }
    rmw_block(hacc, lane, HA::W2, hd);
    lds_order();
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sc[(16 * t + 4 * g + r) * 16 + pcol(i)] = dpre1[t][r];
        sc[(HW + 16 * t + 4 * g + r) * 16 + pcol(i)] = h[t][r];
      }
    lds_order();
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      const f32x4 af = sc_frag(sc, 16 * t + i, g);
      float dw1[4 * HT];
#pragma unroll
      for (int U = 0; U < HT; ++U) {
        const f32x4 bf = sc_frag(sc, HW + 16 * U + i, g);
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) d = mfma4(af[s4], bf[s4], d);
#pragma unroll
        for (int r = 0; r < 4; ++r) dw1[4 * U + r] = d[r];
      }
      rmw_block(hacc, lane, HA::W1 + t * HT * 4, dw1);
    }
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      f32x4 dh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < HT; ++q)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          dh = mfma4(hi_[HI::W1 + (16 * q + 4 * g + s4) * HW + 16 * t + i], dpre1[q][s4], dh);
#pragma unroll
      for (int r = 0; r < 4; ++r) gcur[t][r] = dh[r];
    }
    lds_order();
    };
    head_phase();
    }  // !ppass

    // ---- backpropagation through time, j = L-1 .. 0 (gates recomputed from h_{j-1}); the step's
    // h_{j-1} and x tile are loaded one step ahead
    f32x4 hpn[HT];
    XRaw<IT> xb;
    auto load_bstep = [&](int j) {
      if (j == 0) {
#pragma unroll
        for (int t = 0; t < HT; ++t) hpn[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        const f32x4* src = reinterpret_cast<const f32x4*>((j - 1 < pad ? ptab : hist) + ((size_t)(j - 1) * 64 + lane) * 4 * HT);
#pragma unroll
        for (int t = 0; t < HT; ++t) hpn[t] = src[t];
      }
      load_x_raw<IT>(xb, a.ov, row_of(j), g, i, ok, j < pad);
    };
    // (PADC: down to jlo; the padding pass from L - 2, adding the entry sums, prefetched with the step.  One loop
    // for both: a second instance of the step loop for the padding pass cost the tiles' loop spill reloads, so
    // every step adds an entry row -- in the tiles' rounds always row L - 1, which is zeroed at the start and never
    // written (entries go to rows <= L - 2): a cache-hot zero)
    const int jtop = ppass ? L - 2 : L - 1;
    const float* entp = ppass ? ent : ent + (size_t)(L - 1) * 64 * 4 * HT;
    const size_t est = ppass ? (size_t)64 * 4 * HT : 0;
    f32x4 entn[PADC ? HT : 1];
    auto load_ent = [&](int j) {
#pragma unroll
      for (int t = 0; t < HT; ++t) entn[t] = reinterpret_cast<const f32x4*>(entp + (size_t)j * est + (size_t)lane * 4 * HT)[t];
    };
    if (jtop >= 0) {
      load_bstep(jtop);
      if constexpr (PADC) load_ent(jtop);
    }
    for (int j = jtop; j >= jlo; --j) {
      if constexpr (PADC) {
#pragma unroll
        for (int t = 0; t < HT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) gcur[t][r] += entn[t][r];
      }
      float hp[HT][4];
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) hp[t][r] = hpn[t][r];
      float x[IT][4];
      decode_x<IT>(x, xb, a.ov, xsg, g);
      if (j > jlo) {
        load_bstep(j - 1);
        if constexpr (PADC) load_ent(j - 1);
      }
      f32x4 rz[2 * HT], ni[HT], nh[HT];
      const int z = opaque_zero();
#if D2D_GRU_ABLATE == 4
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        rz[t] = rz[HT + t] = f32x4{hp[t][0], hp[t][1], hp[t][2], hp[t][3]};
        ni[t] = nh[t] = f32x4{x[0][0], x[0][1], x[0][2], x[0][3]};
      }
#else
      if constexpr (SPLIT)
        gru_preact_split<HT, IT, COOP>(wih_g + z, whh_b + z, lane, x, x_exact_step<IT>(a.ov, x), hp, bhn, rz, ni, nh, j == 0);
      else
        gru_preact<HT, IT, false>(wimg + z, whh_s + z, oi, oh, x, hp, bhn, rz, ni, nh, g, i, j == 0);
#endif
      __builtin_amdgcn_sched_barrier(0);
      float drp[HT][4], dzp[HT][4], dnp[HT][4], dghn[HT][4], gz[HT][4];
#pragma unroll
      for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float rr = sigmoidf_(rz[t][r]), zz = sigmoidf_(rz[HT + t][r]);
          const float nn = gru_n(ni[t][r], rr, nh[t][r]);
          const float gv = gcur[t][r];
          const float dn = gv * (1.f - zz), dz = gv * (hp[t][r] - nn);
          dnp[t][r] = dn * fmaf(-nn, nn, 1.f);
          dghn[t][r] = dnp[t][r] * rr;
          drp[t][r] = dnp[t][r] * nh[t][r] * rr * (1.f - rr);
          dzp[t][r] = dz * zz * (1.f - zz);
          gz[t][r] = gv * zz;
          acc.bhn[t][r] += dghn[t][r];
        }
      // this step's rows of the weight-gradient GEMMs, through the wave's scratch (sample-on-k layout)
      // to the global history, two row blocks per pass: dgi (r, z, n_in rows), dgh_n (= dn_pre * r),
      // h_{j-1} -- rows [0, 5 HW) of the step's history block
      float* hrow = ghist + (size_t)j * 5 * HW * 16;
      auto stage_rows = [&](const float (&b0)[HT][4], const float (*b1)[4], int row0) {
#pragma unroll
        for (int t = 0; t < HT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int u = 16 * t + 4 * g + r, c = pcol(i);
            sc[u * 16 + c] = b0[t][r];
            if (b1) sc[(HW + u) * 16 + c] = b1[t][r];
          }
        lds_order();
        const int nv = (b1 ? 2 : 1) * HW * 4 / 64;
#pragma unroll
        for (int v = 0; v < 2 * HW * 4 / 64; ++v)
          if (v < nv)
            reinterpret_cast<f32x4*>(hrow + row0 * 16)[v * 64 + lane] = reinterpret_cast<const f32x4*>(sc)[v * 64 + lane];
        lds_order();
      };
#if D2D_GRU_ABLATE != 3
      if constexpr (!COOP) {
        stage_rows(drp, dzp, 0);
        stage_rows(dnp, dghn, 2 * HW);
        stage_rows(hp, nullptr, 4 * HW);
      }
#endif
      __builtin_amdgcn_sched_barrier(0);
      // dh_{j-1} = g z + W_hh^T dgh: A fragments from the transposed image
      const float* wt = whhT_s + z;
#if D2D_GRU_DH_BF16 && D2D_GRU_ABLATE != 2
      // dg split two ways once per step: B1 = [g_h | g_h], B2 = [g_m | g_m] per gate tile (rows 16T + 4g + r)
      bf16x8 gb1[3 * HT], gb2[3 * HT];
#pragma unroll
      for (int T = 0; T < 3 * HT; ++T) {
        float v[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) v[s4] = T < HT ? drp[T][s4] : T < 2 * HT ? dzp[T - HT][s4] : dghn[T - 2 * HT][s4];
        uint32_t hw[2], mw[2];
        split2_pairs(v, hw, mw);
        const u32x4v b1 = {hw[0], hw[1], hw[0], hw[1]}, b2 = {mw[0], mw[1], mw[0], mw[1]};
        gb1[T] = __builtin_bit_cast(bf16x8, b1);
        gb2[T] = __builtin_bit_cast(bf16x8, b2);
      }
      const bf16x8* wtb = reinterpret_cast<const bf16x8*>(wt);
#endif
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        f32x4 dh = {gz[t][0], gz[t][1], gz[t][2], gz[t][3]};
#if D2D_GRU_ABLATE == 2
        dh += f32x4{drp[t][0], dzp[t][1], dghn[t][2], wt[lane]};
#elif D2D_GRU_DH_BF16
#pragma unroll
        for (int T = 0; T < 3 * HT; ++T) {
          const bf16x8 af = COOP ? whh_dh_frag<HT>(whh_b, T, t, g, i) : wtb[(16 * t + i) * TE + T * 4 + g];
          dh = mfma_bf16(af, gb1[T], dh);
          dh = mfma_bf16(af, gb2[T], dh);
        }
#else
#pragma unroll
        for (int T = 0; T < 3 * HT; ++T) {
          const f32x4 wv = *reinterpret_cast<const f32x4*>(wt + (16 * t + i) * RT + 16 * T + 4 * g);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            const float bv = T < HT ? drp[T][s4] : T < 2 * HT ? dzp[T - HT][s4] : dghn[T - 2 * HT][s4];
            dh = mfma4(wv[s4], bv, dh);
          }
        }
#endif
#pragma unroll
        for (int r = 0; r < 4; ++r) gcur[t][r] = dh[r];
      }
#if D2D_GRU_DH_BF16 && D2D_GRU_ABLATE != 2
      if constexpr (COOP) {
        // this step's rows as split pairs (r, z, n_h: the dh operands' splits; n_in and h_{j-1} here)
        uint32_t nih[HT][2], nim[HT][2], hph[HT][2], hpm[HT][2], xw[IT][2];
#pragma unroll
        for (int t = 0; t < HT; ++t) {
          split2_pairs(dnp[t], nih[t], nim[t]);
          split2_pairs(hp[t], hph[t], hpm[t]);
        }
#pragma unroll
        for (int q = 0; q < IT; ++q) {  // the record's inputs are bf16-exact: their high halves
          xw[q][0] = pack_hi(x[q][0], x[q][1]);
          xw[q][1] = pack_hi(x[q][2], x[q][3]);
        }
        uint16_t* own = creg + wave * CR::ELEMS;
        auto put = [&](int plane, int t, uint32_t w0, uint32_t w1) {
          *reinterpret_cast<uint2*>(own + coop_off(plane, i, 16 * t + 4 * g)) = make_uint2(w0, w1);
        };
        const int sA = 4 * g + (i >> 2), cq = 4 * (i & 3);  // this lane's transposing-read row / column
        if (D2D_GRU_ABLATE != 6) {  // (ablation 6: no exchange)
          __syncthreads();  // every wave has consumed the previous step's regions
          {
#pragma unroll
            for (int t = 0; t < HT; ++t) {
              const u32x4v rh = __builtin_bit_cast(u32x4v, gb1[t]), rm = __builtin_bit_cast(u32x4v, gb2[t]);
              const u32x4v zh = __builtin_bit_cast(u32x4v, gb1[HT + t]), zm = __builtin_bit_cast(u32x4v, gb2[HT + t]);
              const u32x4v nh_ = __builtin_bit_cast(u32x4v, gb1[2 * HT + t]), nm = __builtin_bit_cast(u32x4v, gb2[2 * HT + t]);
              put(0, t, rh[0], rh[1]);
              put(1, t, rm[0], rm[1]);
              put(2, t, zh[0], zh[1]);
              put(3, t, zm[0], zm[1]);
              put(4, t, nih[t][0], nih[t][1]);
              put(5, t, nim[t][0], nim[t][1]);
              put(6, t, nh_[0], nh_[1]);
              put(7, t, nm[0], nm[1]);
              put(8, t, hph[t][0], hph[t][1]);
              put(9, t, hpm[t][0], hpm[t][1]);
            }
#pragma unroll
            for (int q = 0; q < IT; ++q)
              *reinterpret_cast<uint2*>(own + coop_xoff<IT>(i, 16 * q + 4 * g)) = make_uint2(xw[q][0], xw[q][1]);
          }
          __syncthreads();
        }
#pragma unroll 1
        for (int src = 0; src < (D2D_GRU_ABLATE == 5 || D2D_GRU_ABLATE == 6 ? 0 : 4); ++src) {  // (ablation 5: barriers and writes only)
          const uint16_t* reg = creg + src * CR::ELEMS;
          // every wave: its output tiles += the writer's 16 samples (k = sample 4g + q x split part).
          // All 18 fragment reads are issued before the first MFMA (one LDS wait per sub-phase).
          uint2 th[HT], tm[HT], tx[IT], ta[4][2];
#pragma unroll
          for (int U = 0; U < HT; ++U) {
            th[U] = coop_tr(reg, coop_off(8, sA, 16 * U + cq));
            tm[U] = coop_tr(reg, coop_off(9, sA, 16 * U + cq));
          }
#pragma unroll
          for (int U = 0; U < IT; ++U) tx[U] = coop_tr(reg, coop_xoff<IT>(sA, 16 * U + cq));
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // planes r, z, n_h (dW_hh rows; r, z also dW_ih rows), n_in
            const int ph = q == 0 ? 0 : q == 1 ? 2 : q == 2 ? 6 : 4;
            ta[q][0] = coop_tr(reg, coop_off(ph, sA, 16 * wave + cq));
            ta[q][1] = coop_tr(reg, coop_off(ph + 1, sA, 16 * wave + cq));
          }
#pragma unroll
          for (int g3 = 0; g3 < 3; ++g3) {
            const bf16x8 ah = cat2(ta[g3][0], ta[g3][1]);
#pragma unroll
            for (int U = 0; U < HT; ++U) {
              cwh[g3][U] = mfma_bf16(ah, cat2(th[U], th[U]), cwh[g3][U]);
              cwh[g3][U] = mfma_bf16(ah, cat2(tm[U], make_uint2(0u, 0u)), cwh[g3][U]);
            }
            const bf16x8 ai = g3 < 2 ? ah : cat2(ta[3][0], ta[3][1]);
#pragma unroll
            for (int U = 0; U < IT; ++U) cwi[g3][U] = mfma_bf16(ai, cat2(tx[U], tx[U]), cwi[g3][U]);
          }
        }
        // windows longer than kFlushSteps (LONGW instantiations only: the conditional flush inside the step
        // loop cost the xp_load update, L = 64, ~8 % -- 1,097 vs 1,187 ms per 5-epoch GRU D2D-PPO iteration,
        // profiles/r04/gru_flush_ab.log -- as a nest of 64-step chunks it broke the row-history instantiation's
        // code generation, so the loop stays one loop)
        if constexpr (LONGW)
          if (((L - 1 - j) % kFlushSteps) == kFlushSteps - 1 && j > 0) coop_flush();  // wave-uniform
      }
#endif
    }
    if constexpr (PADC) {
      if (!ppass && jlo > 0) {  // dh_{jlo-1} of this tile's samples (lane columns) into the entry sums
        f32x4* e = reinterpret_cast<f32x4*>(ent + ((size_t)(jlo - 1) * 64 + lane) * 4 * HT);
        f32x4 ev[HT];
#pragma unroll
        for (int t = 0; t < HT; ++t) ev[t] = e[t];
#pragma unroll
        for (int t = 0; t < HT; ++t) e[t] = ev[t] + f32x4{gcur[t][0], gcur[t][1], gcur[t][2], gcur[t][3]};
      }
    }
    if constexpr (COOP) {
      __syncthreads();  // the regions' last readers are done before the next head phase
      // flush the tile's sums into the wave's running sums (one fp32 add per tile): MFMA accumulation of
      // every tile of the kernel into the same registers measured 2x the float64 band at 64 envs
      coop_flush();
    }

    // ---- the tile's weight-gradient GEMMs over the history, K = L steps x 16 samples, TBP hidden
    // tiles tb (their r, z, n gate tiles) per pass over the history: dW_hh += dgh h_{j-1}^T,
    // dW_ih += dgi x^T.  A step's fragments are loaded one step ahead (the history is HBM-resident:
    // 1.3 MB per wave and window), so their latency hides behind the previous step's MFMAs; two
    // passes instead of one per hidden tile read the h_{j-1} rows twice instead of HT times.  Every
    // accumulator still sums j = 0 .. L-1, then s4 = 0 .. 3 in order (bitwise the one-tile passes).
    constexpr int TBP = HT >= 2 ? 2 : 1;
    struct WFr {
      f32x4 ai[TBP][3], an[TBP], bh[HT];
      uint32_t xr[IT][4];  // raw x^T words (record: one byte each), decoded where they are used
      bool zero;
    };
    auto load_fr = [&](WFr& f, int j, int tb0) {
      const float* hrow = ghist + (size_t)j * 5 * HW * 16;
#pragma unroll
      for (int p = 0; p < TBP; ++p) {
#pragma unroll
        for (int g3 = 0; g3 < 3; ++g3) f.ai[p][g3] = sc_frag(hrow, 16 * (g3 * HT + tb0 + p) + i, g);
        f.an[p] = sc_frag(hrow, R3 + 16 * (tb0 + p) + i, g);
      }
#pragma unroll
      for (int U = 0; U < HT; ++U) f.bh[U] = sc_frag(hrow, R3 + HW + 16 * U + i, g);
      // x^T operand sample-on-k from the rollout buffer (sample 4 s4 + g, input 16U + i): raw loads only
      // (a decode right after its load would make the wave wait for it there)
      f.zero = j < pad;
      const __amdgpu_buffer_rsrc_t rsrc = rows_rsrc(a.ov, row_of(j), f.zero);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int ee = 4 * s4 + g;
        const bool eok = e0 + ee < E;
        const uint32_t vb = eok ? (uint32_t)(ee * N * a.ov.RB) : 0x80000000u;
#pragma unroll
        for (int U = 0; U < IT; ++U) {
          // record: the aligned dword holding byte col (rows are whole dwords); fp32 rows: word col
          const uint32_t col = 16 * U + i;
          f.xr[U][s4] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, a.ov.u8 ? (vb + col) & ~3u : vb + 4u * col, 0, 0);
        }
      }
    };
    // this lane's x^T columns 16U + i: record int8 masks (rec_byte) and the fp32-row column class
    uint32_t xtm[IT];  // (record) the int8 mask of column 16U + i at its byte i & 3 of the loaded dword
#pragma unroll
    for (int U = 0; U < IT; ++U) xtm[U] = (xsg.bit(16 * U + i) << 7) << (8 * (i & 3));
    auto decode_xt = [&](float (&xt)[IT][4], const WFr& f) {
#pragma unroll
      for (int U = 0; U < IT; ++U) {
        const int col = 16 * U + i;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const float v = a.ov.u8 ? rec_byte(f.xr[U][s4], i & 3, xtm[U]) : (col < F ? uf(f.xr[U][s4]) : 0.f);
          xt[U][s4] = col == F && (f.zero || !a.ov.u8) ? 1.f : v;  // the bias column
        }
      }
    };
#pragma unroll 1
    for (int tb0 = 0; tb0 < (COOP || D2D_GRU_ABLATE == 1 ? 0 : HT); tb0 += TBP) {
      f32x4 dwh[TBP][3][HT], dwi[TBP][3][IT];
#pragma unroll
      for (int p = 0; p < TBP; ++p)
#pragma unroll
        for (int g3 = 0; g3 < 3; ++g3) {
#pragma unroll
          for (int U = 0; U < HT; ++U) dwh[p][g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int U = 0; U < IT; ++U) dwi[p][g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      // the passes' sums into the wave's global sums, accumulators restarted: at the end of the window and,
      // for windows longer than kFlushSteps steps, every kFlushSteps steps (see coop_flush)
      auto hist_flush = [&]() {
#pragma unroll
        for (int p = 0; p < TBP; ++p) {
          if (tb0 + p >= HT) break;
#pragma unroll
          for (int g3 = 0; g3 < 3; ++g3) {
            const int T = g3 * HT + tb0 + p;
            float dh_[4 * HT], di_[4 * IT];
#pragma unroll
            for (int U = 0; U < HT; ++U)
#pragma unroll
              for (int r = 0; r < 4; ++r) dh_[4 * U + r] = dwh[p][g3][U][r];
#pragma unroll
            for (int U = 0; U < IT; ++U)
#pragma unroll
              for (int r = 0; r < 4; ++r) di_[4 * U + r] = dwi[p][g3][U][r];
            rmw_block(gpart, lane, T * HT * 4, dh_);
            rmw_block(gpart, lane, WA::WI + T * IT * 4, di_);
#pragma unroll
            for (int U = 0; U < HT; ++U) dwh[p][g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int U = 0; U < IT; ++U) dwi[p][g3][U] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
      };
      WFr cur, nxt;
      load_fr(nxt, 0, tb0);
#pragma unroll 1
      for (int j = 0; j < L; ++j) {
        cur = nxt;
        if (j + 1 < L) load_fr(nxt, j + 1, tb0);
        float xt[IT][4];
        decode_xt(xt, cur);
#if D2D_GRU_DW_BF16
        // B operands with the A fragments' k-slots (sample 4 s4 + g, part): h_{j-1} as [h h] and [m 0]
        // (the two MFMAs give a_h b_h + a_m b_h and a_h b_m), x (bf16-exact) as [x x]
        bf16x8 bh1[HT], bh2[HT], bx[IT];
#pragma unroll
        for (int U = 0; U < HT; ++U) {
          const u32x4v w = split_pairs(cur.bh[U]);
          u32x4v d1, d2;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            d1[q] = __builtin_amdgcn_perm(w[q], w[q], 0x01000100u);
            d2[q] = w[q] >> 16;
          }
          bh1[U] = __builtin_bit_cast(bf16x8, d1);
          bh2[U] = __builtin_bit_cast(bf16x8, d2);
        }
#pragma unroll
        for (int U = 0; U < IT; ++U) {
          u32x4v d;
#pragma unroll
          for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_perm(fbits(xt[U][q]), fbits(xt[U][q]), 0x03020302u);
          bx[U] = __builtin_bit_cast(bf16x8, d);
        }
        // fp32-row inputs that are not bf16-exact (the chsel env's 1/n ACK fractions): x is the exact sum of
        // three truncation parts x_h + x_m + x_l; [x_h x_h] above leaves a_h x_m + a_m x_m ([x_m x_m]) and
        // a_h x_l ([x_l 0]) to two more MFMAs (wave-uniform: the record's integers never take this branch).
        // Without them dW_ih carried x's 2^-8 truncation coherently over every sample of a fractional
        // ACK value: 1.5e-4 - 5.6e-4 of max|g| on the categorical GRU learner traces (tools/gpu/gru_learner_diag.py)
        bool xfrac = false;
        bf16x8 bxm[IT], bxl[IT];
        if (!a.ov.u8) {
          uint32_t low = 0;
#pragma unroll
          for (int U = 0; U < IT; ++U)
#pragma unroll
            for (int q = 0; q < 4; ++q) low |= fbits(xt[U][q]) & 0xFFFFu;
          xfrac = __builtin_amdgcn_ballot_w64(low != 0) != 0;
          if (xfrac) {
#pragma unroll
            for (int U = 0; U < IT; ++U) {
              u32x4v dm, dl;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float rm = xt[U][q] - ffrom(fbits(xt[U][q]) & 0xFFFF0000u);  // x - x_h, exact
                const uint32_t rb = fbits(rm) & 0xFFFF0000u;                       // x_m
                const float rl = rm - ffrom(rb);                                  // x_l, exact in bf16
                dm[q] = __builtin_amdgcn_perm(rb, rb, 0x03020302u);
                dl[q] = fbits(rl) >> 16;
              }
              bxm[U] = __builtin_bit_cast(bf16x8, dm);
              bxl[U] = __builtin_bit_cast(bf16x8, dl);
            }
          }
        }
#pragma unroll
        for (int p = 0; p < TBP; ++p) {
          if (tb0 + p >= HT) break;
          bf16x8 ag[3], an2;
#pragma unroll
          for (int g3 = 0; g3 < 3; ++g3) ag[g3] = __builtin_bit_cast(bf16x8, split_pairs(cur.ai[p][g3]));
          an2 = __builtin_bit_cast(bf16x8, split_pairs(cur.an[p]));
#pragma unroll
          for (int U = 0; U < HT; ++U)
#pragma unroll
            for (int g3 = 0; g3 < 3; ++g3) {
              const bf16x8 af = g3 < 2 ? ag[g3] : an2;
              dwh[p][g3][U] = mfma_bf16(af, bh1[U], dwh[p][g3][U]);
              dwh[p][g3][U] = mfma_bf16(af, bh2[U], dwh[p][g3][U]);
            }
#pragma unroll
          for (int g3 = 0; g3 < 3; ++g3)
#pragma unroll
            for (int U = 0; U < IT; ++U) dwi[p][g3][U] = mfma_bf16(ag[g3], bx[U], dwi[p][g3][U]);
          if (xfrac) {
#pragma unroll
            for (int g3 = 0; g3 < 3; ++g3)
#pragma unroll
              for (int U = 0; U < IT; ++U) {
                dwi[p][g3][U] = mfma_bf16(ag[g3], bxl[U], dwi[p][g3][U]);
                dwi[p][g3][U] = mfma_bf16(ag[g3], bxm[U], dwi[p][g3][U]);
              }
          }
        }
#else
#pragma unroll
        for (int p = 0; p < TBP; ++p) {
          if (tb0 + p >= HT) break;  // (odd HT: the last pass has one tile)
#pragma unroll
          for (int U = 0; U < HT; ++U)
#pragma unroll
            for (int g3 = 0; g3 < 3; ++g3) {
              const f32x4 af = g3 < 2 ? cur.ai[p][g3] : cur.an[p];
#pragma unroll
              for (int s4 = 0; s4 < 4; ++s4) dwh[p][g3][U] = mfma4(af[s4], cur.bh[U][s4], dwh[p][g3][U]);
            }
#pragma unroll
          for (int g3 = 0; g3 < 3; ++g3)
#pragma unroll
            for (int U = 0; U < IT; ++U)
#pragma unroll
              for (int s4 = 0; s4 < 4; ++s4) dwi[p][g3][U] = mfma4(cur.ai[p][g3][s4], xt[U][s4], dwi[p][g3][U]);
        }
#endif
        if ((j % kFlushSteps) == kFlushSteps - 1 && j + 1 < L) hist_flush();  // wave-uniform
      }
      hist_flush();
    }
  }

  // ---- cross-wave sum of the register partials (fixed order, through the scratch), then the
  // workgroup's partial: registers of wave 0 + the four waves' global weight-gradient sums
  constexpr int NV = GruSAcc<HT>::NV;
  float* red = COOP ? reinterpret_cast<float*>(creg_raw) : &scr[0][0];
  static_assert(NV * 64 <= (COOP ? CR::BYTES / 4 : 4 * SROWS * 16), "reduction buffer");
#pragma unroll 1
  for (int w = 1; w < 4; ++w) {
    __syncthreads();
    if (wave == w) acc.each([&](int v, float& x) { red[v * 64 + lane] = x; });
    __syncthreads();
    if (wave == 0) acc.each([&](int v, float& x) { x += red[v * 64 + lane]; });
  }
  __syncthreads();
  const GruOff o(H, F, A);
  float* part = a.partial + ((size_t)blockIdx.y * N + k) * a.P;
  if constexpr (COOP) {  // every wave writes its own dW_hh / dW_ih tiles (disjoint rows) from its sums
#pragma unroll
    for (int g3 = 0; g3 < 3; ++g3)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int u = 16 * wave + 4 * g + r;
        if (u >= H) continue;
        const int v0 = g3 * (HT + IT) * 4;
#pragma unroll
        for (int U = 0; U < HT; ++U) {
          const int c = 16 * U + i;
          if (c < H) part[o.whh + (g3 * H + u) * H + c] = gpart[(v0 + 4 * U + r) * 64 + lane];
        }
#pragma unroll
        for (int U = 0; U < IT; ++U) {
          const int c = 16 * U + i;
          const float v = gpart[(v0 + 4 * (HT + U) + r) * 64 + lane];
          if (c < F) part[o.wih + (g3 * H + u) * F + c] = v;
          else if (c == F) {
            part[o.bih + g3 * H + u] = v;
            if (g3 < 2) part[o.bhh + g3 * H + u] = v;  // b_hr / b_hz enter exactly like b_ir / b_iz
          }
        }
      }
  }
  if (wave == 0) {
    const float* wb = a.gpart + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 * WA::NV * 64;
    auto wsum = [&](int v) {
      return ((wb[v * 64 + lane] + wb[(WA::NV + v) * 64 + lane]) + wb[(2 * WA::NV + v) * 64 + lane]) +
             wb[(3 * WA::NV + v) * 64 + lane];
    };
#pragma unroll 1
    for (int T = 0; T < (COOP ? 0 : 3 * HT); ++T)
#pragma unroll
      for (int U = 0; U < HT; ++U)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 16 * T + 4 * g + r, G = R / HW, u = R - G * HW, c = 16 * U + i;
          const float v = wsum((T * HT + U) * 4 + r);
          if (u < H && c < H) part[o.whh + (G * H + u) * H + c] = v;
        }
#pragma unroll 1
    for (int T = 0; T < (COOP ? 0 : 3 * HT); ++T)
#pragma unroll
      for (int U = 0; U < IT; ++U)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 16 * T + 4 * g + r, G = R / HW, u = R - G * HW, c = 16 * U + i;
          const float v = wsum(WA::WI + (T * IT + U) * 4 + r);
          if (u >= H) continue;
          if (c < F) part[o.wih + (G * H + u) * F + c] = v;
          else if (c == F) {
            part[o.bih + G * H + u] = v;
            if (G < 2) part[o.bhh + G * H + u] = v;  // b_hr / b_hz enter exactly like b_ir / b_iz
          }
        }
    // the head's sums: the workgroup's four wave blocks in fixed order
    using HA = GruHeadAcc<HT>;
    const float* hb = a.hacc + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 4 * HA::NV * 64;
    auto hsum = [&](int v) {
      return ((hb[v * 64 + lane] + hb[(HA::NV + v) * 64 + lane]) + hb[(2 * HA::NV + v) * 64 + lane]) +
             hb[(3 * HA::NV + v) * 64 + lane];
    };
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int U = 0; U < HT; ++U)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * t + 4 * g + r, col = 16 * U + i;
          const float v = hsum(HA::W1 + (t * HT + U) * 4 + r);
          if (row < H && col < H) part[o.w1 + row * H + col] = v;
        }
#pragma unroll
    for (int U = 0; U < HT; ++U)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * g + r, col = 16 * U + i;
        const float v = hsum(HA::W2 + 4 * U + r);
        if (row < A && col < H) part[o.w2 + row * H + col] = v;
      }
    // bias sums: the 16 sample lanes of each row group
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int u = 16 * t + 4 * g + r;
        const float sb1 = row_sum16(hsum(HA::B1 + 4 * t + r)), sbn = row_sum16(acc.bhn[t][r]);
        if (i == 0 && u < H) {
          part[o.b1 + u] = sb1;
          part[o.bhh + 2 * H + u] = sbn;
        }
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float sb2 = row_sum16(hsum(HA::B2 + r));
      if (i == 0 && 4 * g + r < A) part[o.b2 + 4 * g + r] = sb2;
    }
    float s0 = acc.st[0], s1 = acc.st[1];
    s0 = group_sum(row_sum16(s0));
    s1 = group_sum(row_sum16(s1));
    if (lane == 0) {
      part[o.st] = s0;
      part[o.st + 1] = s1;
    }
  }
}

// The input images of all agents, unswizzled: img[k][R][c] (gate row R of the padded layout, input
// column c; column F = the biases of gru_common.h), zero outside the real rows / columns.
template <int HT>
__global__ void gru_head_image_kernel(GruW w, int N, int H, int A, float* img) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int SZ = HeadImg<HT>::SIZE;
  if (idx >= (int64_t)N * SZ) return;
  const int k = (int)(idx / SZ);
  img[idx] = head_img_elem<HT>(w, k, H, A, (int)(idx - (int64_t)k * SZ));
}

__global__ void gru_wih_image_kernel(GruW w, int N, int H, int F, int HW, int IW, float* img) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * 3 * HW * IW) return;
  const int k = (int)(idx / (3 * HW * IW)), rem = (int)(idx - (int64_t)k * 3 * HW * IW);
  const int R = rem / IW, c = rem - R * IW, G = R / HW, u = R - G * HW, src = G * H + u;
  float v = 0.f;
  if (u < H) {
    if (c < F) v = w.w_ih[((size_t)k * 3 * H + src) * F + c];
    else if (c == F) v = G < 2 ? w.b_ih[(size_t)k * 3 * H + src] + w.b_hh[(size_t)k * 3 * H + src]
                               : w.b_ih[(size_t)k * 3 * H + src];
  }
  img[idx] = v;
}

// Fixed-order sum of the G workgroup partials -> the gradient tensors (+ loss sums).
__global__ void gru_reduce_kernel(const float* __restrict__ partial, int G, int N, int P, int H, int F, int A,
                                  float* gwih, float* gwhh, float* gbih, float* gbhh, float* gw1, float* gb1,
                                  float* gw2, float* gb2, float* stats) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * P) return;
  const int k = (int)(idx / P), p = (int)(idx - (int64_t)k * P);
  float s = 0.f;
  for (int b = 0; b < G; ++b) s += partial[((size_t)b * N + k) * P + p];
  const GruOff o(H, F, A);
  if (p < o.whh) gwih[(size_t)k * 3 * H * F + p] = s;
  else if (p < o.bih) gwhh[(size_t)k * 3 * H * H + (p - o.whh)] = s;
  else if (p < o.bhh) gbih[(size_t)k * 3 * H + (p - o.bih)] = s;
  else if (p < o.w1) gbhh[(size_t)k * 3 * H + (p - o.bhh)] = s;
  else if (p < o.b1) gw1[(size_t)k * H * H + (p - o.w1)] = s;
  else if (p < o.w2) gb1[(size_t)k * H + (p - o.b1)] = s;
  else if (p < o.b2) gw2[(size_t)k * A * H + (p - o.w2)] = s;
  else if (p < o.st) gb2[(size_t)k * A + (p - o.b2)] = s;
  else if (stats) stats[(size_t)k * 2 + (p - o.st)] = s;
}

}  // namespace d2d

using namespace d2d;

extern std::atomic<int> g_policy_f32_mfma;  // policy_kernels.hip (D2D_OPT_POLICY_F32_MFMA)

template <int HT, int IT, int KIND, bool SPLIT>
static void launch_policy_split(const GruArgs& a, dim3 grid, int threads, hipStream_t s) {
  if (KIND == kGruValue || a.ep.forced == nullptr) {
    if (KIND != kGruValue && a.ep.deterministic)
      hipLaunchKernelGGL((gru_policy_kernel<HT, IT, KIND, kModeDeterministic, SPLIT>), grid, dim3(threads), 0, s, a);
    else
      hipLaunchKernelGGL((gru_policy_kernel<HT, IT, KIND, kModeSample, SPLIT>), grid, dim3(threads), 0, s, a);
  } else {
    hipLaunchKernelGGL((gru_policy_kernel<HT, IT, KIND, kModeForced, SPLIT>), grid, dim3(threads), 0, s, a);
  }
}

// the split kernel where its images fit LDS (IT <= 2: F < 32); the fp32-MFMA kernel otherwise or
// when D2D_OPT_POLICY_F32_MFMA asks for it (A/B timing and tests)
template <int HT, int IT, int KIND>
static void launch_policy_mode(const GruArgs& a, dim3 grid, int threads, hipStream_t s) {
  if constexpr (IT <= 2) {
    if (!g_policy_f32_mfma.load(std::memory_order_relaxed)) {
      launch_policy_split<HT, IT, KIND, true>(a, grid, threads, s);
      return;
    }
  }
  launch_policy_split<HT, IT, KIND, false>(a, grid, threads, s);
}

template <int HT, int IT>
static void launch_policy_kind(const GruArgs& a, dim3 grid, int threads, hipStream_t s) {
  if (a.kind == kGruBernoulli) launch_policy_mode<HT, IT, kGruBernoulli>(a, grid, threads, s);
  else if (a.kind == kGruCategorical) launch_policy_mode<HT, IT, kGruCategorical>(a, grid, threads, s);
  else launch_policy_mode<HT, IT, kGruValue>(a, grid, threads, s);
}

template <int HT>
static void launch_policy_it(const GruArgs& a, dim3 grid, int threads, hipStream_t s) {
  if (a.F + 1 <= 16) launch_policy_kind<HT, 1>(a, grid, threads, s);
  else if (a.F + 1 <= 32) launch_policy_kind<HT, 2>(a, grid, threads, s);
  else launch_policy_kind<HT, 4>(a, grid, threads, s);  // (the swizzled fp32 images need 16 / 32 / 64 columns)
}

static int check_gru_desc(const d2d_gru_desc* d, const void* obs) {
  if (!d || !d->w_ih || !d->w_hh || !d->b_ih || !d->b_hh || !d->w1 || !d->b1 || !d->w2 || !d->b2) {
    d2d_set_error("d2d_gru: NULL weight");
    return D2D_EINVAL;
  }
  if (d->n_agents < 0 || d->n_envs < 0) { d2d_set_error("negative size"); return D2D_EINVAL; }
  if (d->hidden < 1 || d->hidden > 64) { d2d_set_error("hidden=%d outside [1,64]", d->hidden); return D2D_EUNSUPPORTED; }
  if (d->obs_dim < 1 || d->obs_dim + 1 > 64) { d2d_set_error("obs_dim=%d outside [1,63]", d->obs_dim); return D2D_EUNSUPPORTED; }
  if (d->kind < 0 || d->kind > 2) { d2d_set_error("kind=%d outside [0,2]", d->kind); return D2D_EINVAL; }
  if (d->kind != 2 && (d->n_out < 1 || d->n_out > 16)) { d2d_set_error("n_out=%d outside [1,16]", d->n_out); return D2D_EUNSUPPORTED; }
  if (d->history_len < 1 || d->episode_length < 1) { d2d_set_error("history_len / episode_length < 1"); return D2D_EINVAL; }
  const float* f32;
  const uint8_t* rec;
  const uint32_t* sgn;
  return obs_format_args(d->obs_format, d->obs_signed, d->obs_dim, obs, f32, rec, sgn);
}

static GruArgs make_gru_args(const d2d_gru_desc* d, int T, const void* obs) {
  GruArgs a{};
  a.T = T; a.E = d->n_envs; a.N = d->n_agents; a.F = d->obs_dim; a.H = d->hidden;
  a.A = d->kind == 2 ? 1 : d->n_out; a.kind = d->kind;
  a.L = d->history_len; a.ep_len = d->episode_length;
  a.env_tiles = (a.E + 15) / 16;
  a.w = {d->w_ih, d->w_hh, d->b_ih, d->b_hh, d->w1, d->b1, d->w2, d->b2};
  const float* f32;
  const uint8_t* rec;
  const uint32_t* sgn;
  obs_format_args(d->obs_format, d->obs_signed, d->obs_dim, obs, f32, rec, sgn);  // checked by check_gru_desc
  a.ov.base = rec ? rec : reinterpret_cast<const uint8_t*>(f32);
  a.ov.rows = (int64_t)T * a.E * a.N;
  a.ov.RB = rec ? D2D_RECORD_BYTES(a.F) : 4 * a.F;
  a.ov.N = a.N; a.ov.F = a.F; a.ov.u8 = rec ? 1 : 0; a.ov.sgn = sgn;
  a.inv_A = 1.f / (float)a.A;
  a.mask_bytes = a.A <= 8 ? 1 : a.A <= 16 ? 2 : 4;
  return a;
}

static int policy_gru(const d2d_gru_desc* d, int32_t T, const void* obs, int32_t slot0, int32_t n_slots,
                      int32_t padded, const void* forced, uint32_t rng_step, int32_t deterministic, void* actions,
                      float* out, float* hcarry, int32_t carry_in, void* stream);

extern "C" int64_t d2d_gru_carry_floats(const d2d_gru_desc* d) {
  if (!d || d->n_agents < 0 || d->n_envs < 0 || d->hidden < 1 || d->hidden > 64) return -1;
  const int64_t ht = (d->hidden + 15) / 16;
  return (int64_t)d->n_agents * ((d->n_envs + 15) / 16) * 4 * (ht <= 1 ? 1 : ht <= 2 ? 2 : 4) * 64;
}

extern "C" int d2d_policy_gru(const d2d_gru_desc* d, int32_t T, const void* obs, int32_t slot0, int32_t n_slots,
                              int32_t padded, const void* forced, uint32_t rng_step, int32_t deterministic,
                              void* actions, float* out, void* stream) {
  return policy_gru(d, T, obs, slot0, n_slots, padded, forced, rng_step, deterministic, actions, out, nullptr, 0,
                    stream);
}

extern "C" int d2d_policy_gru_carry(const d2d_gru_desc* d, int32_t T, const void* obs, int32_t slot,
                                    const void* forced, uint32_t rng_step, int32_t deterministic, void* actions,
                                    float* out, float* hcarry, int32_t carry_in, void* stream) {
  if (!hcarry) { d2d_set_error("d2d_policy_gru_carry: NULL hcarry"); return D2D_EINVAL; }
  if (d && d->episode_length > 0 && slot >= 0) {
    const int pos = slot % d->episode_length;
    if (carry_in && (pos < 1 || pos >= d->history_len)) {
      d2d_set_error("d2d_policy_gru_carry: slot %d (episode position %d) does not extend the previous slot's window "
                    "(history_len %d)", slot, pos, d->history_len);
      return D2D_EINVAL;
    }
  }
  return policy_gru(d, T, obs, slot, 1, 0, forced, rng_step, deterministic, actions, out, hcarry, carry_in ? 1 : 0,
                    stream);
}

static int policy_gru(const d2d_gru_desc* d, int32_t T, const void* obs, int32_t slot0, int32_t n_slots,
                      int32_t padded, const void* forced, uint32_t rng_step, int32_t deterministic, void* actions,
                      float* out, float* hcarry, int32_t carry_in, void* stream) {
  int rc = check_gru_desc(d, obs);
  if (rc) return rc;
  // actions may be NULL in forced mode (the log-probs of given actions: nothing else to write)
  if (!obs || !out || (d->kind != 2 && !actions && !forced)) { d2d_set_error("d2d_policy_gru: NULL buffer"); return D2D_EINVAL; }
  if (T < 1 || slot0 < 0 || n_slots < 0 || slot0 + n_slots > T) {
    d2d_set_error("d2d_policy_gru: slots [%d, %d) outside the %d-slot buffer", slot0, slot0 + n_slots, T);
    return D2D_EINVAL;
  }
  if (T % d->episode_length != 0 && slot0 + n_slots > T - T % d->episode_length + d->episode_length) {
    d2d_set_error("d2d_policy_gru: buffer is not whole episodes");
    return D2D_EINVAL;
  }
  GruArgs a = make_gru_args(d, T, obs);
  a.slot0 = slot0; a.n_slots = n_slots; a.padded = padded ? 1 : 0;
  a.hcarry = hcarry; a.carry_in = carry_in;
  MlpArgs& ep = a.ep;
  ep.E = n_slots * a.E; ep.N = a.N; ep.F = a.F; ep.H = a.H; ep.A = a.A; ep.kind = d->kind == 0 ? 0 : 1;
  ep.deterministic = deterministic ? 1 : 0; ep.inv_A = a.inv_A; ep.rng_step = rng_step; ep.rng_off = d->rng_offset;
  ep.seed = d->seed; ep.env_base = d->env_base; ep.forced = forced; ep.act_out = actions; ep.logp_out = out;
  ep.value_out = nullptr; ep.mask_bytes = a.mask_bytes;
  a.value_out = out;
  if (a.N == 0 || a.E == 0 || n_slots == 0) return D2D_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t tiles = (int64_t)n_slots * a.env_tiles;
  // about 2 workgroups of 8 waves per CU over the whole grid, at least one tile per wave.  A batch too small
  // to give every CU a workgroup (the xp_load rollout: 64 agents x 16 tiles) takes 4-wave workgroups instead
  // (the LDS images allow one workgroup per CU either way): one wave per SIMD on twice as many CUs, so each
  // window step's MFMAs no longer share a SIMD's pipe with a second wave's
  int threads = 512;
  int gy = (int)std::max<int64_t>(1, std::min<int64_t>((512 + a.N - 1) / a.N, (tiles + 7) / 8));
  if ((int64_t)a.N * gy < 256 && tiles > 4) {
    threads = 256;
    gy = (int)std::max<int64_t>(1, std::min<int64_t>((256 + a.N - 1) / a.N, (tiles + 3) / 4));
  }
  dim3 grid(a.N, gy);
  const int ht = (a.H + 15) / 16;
  // padded windows beyond the LDS padding table: a stream-ordered scratch table per workgroup (not while the
  // stream is being captured: those launches run the pad steps per tile, the same arithmetic)
  void* gtab = nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (a.padded && a.L - 1 > kGruPadTab) {
    if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone) {
      const size_t bytes = sizeof(float) * (size_t)gy * a.N * (size_t)(a.L - 1) * 16 * (ht <= 1 ? 1 : ht <= 2 ? 2 : 4);
      if (hipMallocAsync(&gtab, bytes, s) != hipSuccess) gtab = nullptr;
    }
    // a failed query or allocation leaves HIP's sticky last error set: clear it, so the status checked after
    // the launch is the launch's own (the fallback -- pad steps per tile -- is a valid launch)
    if (!gtab) (void)hipGetLastError();
  }
  a.ptab_g = reinterpret_cast<float*>(gtab);
  if (ht <= 1) launch_policy_it<1>(a, grid, threads, s);
  else if (ht <= 2) launch_policy_it<2>(a, grid, threads, s);
  else launch_policy_it<4>(a, grid, threads, s);
  const hipError_t le = hipGetLastError();
  if (gtab) D2D_CHECK_HIP(hipFreeAsync(gtab, s));  // stream-ordered: released after the kernel
  D2D_CHECK_HIP(le);
  return D2D_OK;
}

// ------------------------------------------------------------------------------------ grad ABI
static int gru_grad_blocks(int N, int64_t n_tiles) {
  // about one workgroup (4 waves, 160 KB LDS) per CU over the grid, at least one tile per wave
  return (int)std::max<int64_t>(1, std::min<int64_t>((256 + N - 1) / N, (n_tiles + 3) / 4));
}

// Float offsets of the grad kernel's workspace pieces (each rounded to 64 floats: 16-byte vector
// accesses stay aligned): partials, h history, input images, head sums, head images, the per-step
// gradient-row history, the weight-gradient sums.
#ifndef D2D_GRU_GRAD_SPLIT
#define D2D_GRU_GRAD_SPLIT 1  // 0: the fp32-MFMA step in the update kernel (ablation builds)
#endif
constexpr bool kGradSplit = D2D_GRU_GRAD_SPLIT != 0;

struct GruWs {
  int64_t partial, hist, wimg, hacc, himg, ghist, gpart, total;
};
// d2d_set_option(D2D_OPT_GRU_GRAD_HISTORY, 1).  Atomic, and read ONCE per workspace query / launch: the
// option selects the workspace layout, so it must be set before the query that sizes the caller's
// buffer; d2d_gru_grad re-derives the size from its own snapshot and refuses (EINVAL) a buffer sized
// for the other layout instead of overrunning it.
std::atomic<int> g_gru_grad_history{0};
// the cooperative weight-gradient path of gru_grad_kernel (COOP): hidden tiles 4 (H in (32, 64]),
// input tiles <= 3 (F + 1 <= 48: four staging regions + the W_hh image fit the 160 KB of LDS), the
// compact record (bf16-exact inputs), the split step; `history` = the option's snapshot
static bool gru_coop(int htp, int itp, bool u8, bool history) {
  return !history && htp == 4 && itp <= 3 && u8 && D2D_GRU_GRAD_SPLIT && D2D_GRU_DH_BF16 &&
         (D2D_GRU_ABLATE == 0 || D2D_GRU_ABLATE >= 5);
}
static GruWs gru_ws_layout(int64_t G, int64_t N, int64_t P, int64_t L, int htp, int itp, bool coop) {
  auto up = [](int64_t v) { return (v + 63) / 64 * 64; };
  const int64_t waves = G * N * 4, HW = 16 * htp;
  GruWs w;
  w.partial = 0;
  w.hist = up(G * N * P);
  // per wave: the tile's h history + the padding table (+ COOP: the padding-region entry sums, PADC)
  w.wimg = w.hist + up(waves * (coop && D2D_GRU_PAD_COLLAPSE ? 3 : 2) * L * 64 * 4 * htp);
  // fp32 input images [N][3 HW][16 itp] or the split ones [N][3 htp][CI][3 parts][64] 16-byte words
  const int64_t ci = (itp + 1) / 2;
  w.hacc = w.wimg + up(N * std::max<int64_t>(3 * HW * 16 * itp, 3 * htp * ci * 3 * 64 * 4));
  w.himg = w.hacc + up(waves * 64 * (htp * htp * 4 + htp * 8 + 4));
  w.ghist = w.himg + up(N * (HW * HW + 16 * HW + HW + 16));
  w.gpart = w.ghist + (coop ? 0 : up(waves * L * 5 * HW * 16));  // COOP: no row history
  // wave sums: all dW tiles per wave (history), or (COOP) the wave's own 3 (HT + IT) tiles
  w.total = w.gpart + up(waves * 64 * (coop ? 3 * (htp + itp) * 4 : 3 * htp * (htp + itp) * 4));
  return w;
}

// 16-column input tiles of the x operand (the inputs and the bias column F): F + 1 <= 64
static int gru_input_tiles(int F) { return F + 1 <= 16 ? 1 : F + 1 <= 32 ? 2 : F + 1 <= 48 ? 3 : 4; }

static int64_t gru_grad_workspace(const d2d_gru_desc* d, int32_t T, bool history) {
  if (!d || d->n_agents <= 0 || T <= 0 || d->n_envs <= 0 || d->hidden < 1 || d->history_len < 1) return 0;
  const int A = d->kind == 2 ? 1 : d->n_out, H = d->hidden, ht = H <= 16 ? 1 : H <= 32 ? 2 : 4;
  const int64_t tiles = (int64_t)T * ((d->n_envs + 15) / 16);
  const int G = gru_grad_blocks(d->n_agents, tiles);
  const GruOff o(H, d->obs_dim, A);
  return gru_ws_layout(G, d->n_agents, o.P, d->history_len, ht, gru_input_tiles(d->obs_dim),
                       gru_coop(ht, gru_input_tiles(d->obs_dim), d->obs_format == D2D_OBS_U8, history)).total;
}

extern "C" int64_t d2d_gru_grad_workspace(const d2d_gru_desc* d, int32_t T) {
  return gru_grad_workspace(d, T, g_gru_grad_history.load(std::memory_order_relaxed) != 0);
}


template <int HT, int IT>
static void launch_grad_kind(const GruArgs& a, dim3 grid, hipStream_t s, bool coop) {
  if constexpr (HT == 4 && IT <= 3 && kGradSplit && D2D_GRU_DH_BF16) {
    if (coop && a.L > kFlushSteps) {
      if (a.kind == kGruBernoulli)
        hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruBernoulli, true, true, true>), grid, dim3(256), 0, s, a);
      else if (a.kind == kGruCategorical)
        hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruCategorical, true, true, true>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruValue, true, true, true>), grid, dim3(256), 0, s, a);
      return;
    }
    if (coop) {
      if (a.kind == kGruBernoulli)
        hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruBernoulli, true, true>), grid, dim3(256), 0, s, a);
      else if (a.kind == kGruCategorical)
        hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruCategorical, true, true>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruValue, true, true>), grid, dim3(256), 0, s, a);
      return;
    }
  }
  if (a.kind == kGruBernoulli)
    hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruBernoulli, kGradSplit>), grid, dim3(256), 0, s, a);
  else if (a.kind == kGruCategorical)
    hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruCategorical, kGradSplit>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((gru_grad_kernel<HT, IT, kGruValue, kGradSplit>), grid, dim3(256), 0, s, a);
}

// the split W_ih images of all agents in the update workspace ([N][GruSplit::WIH] 16-byte words)
template <int HT, int IT>
__global__ void gru_wih_split_image_kernel(GruW w, int N, int H, int F, bf16x8* img) {
  using S = GruSplit<HT, IT>;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int PER = S::NT * S::CI * 64;
  if (idx >= (int64_t)N * PER) return;
  const int k = (int)(idx / PER), rel = (int)(idx - (int64_t)k * PER);
  store_parts(img + (size_t)k * S::WIH + split_word(rel), split_frag<HT, IT>(w, k, H, F, true, rel));
}
template <int HT, int IT>
static void launch_wih_split_it(const GruArgs& a, hipStream_t s) {
  using S = GruSplit<HT, IT>;
  const int64_t n = (int64_t)a.N * S::NT * S::CI * 64;
  bf16x8* img = reinterpret_cast<bf16x8*>(a.wimg);
  hipLaunchKernelGGL((gru_wih_split_image_kernel<HT, IT>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.w, a.N,
                     a.H, a.F, img);
}
template <int HT>
static void launch_wih_split(const GruArgs& a, int itp, hipStream_t s) {
  if (itp == 1) launch_wih_split_it<HT, 1>(a, s);
  else if (itp == 2) launch_wih_split_it<HT, 2>(a, s);
  else if (itp == 3) launch_wih_split_it<HT, 3>(a, s);
  else launch_wih_split_it<HT, 4>(a, s);
}

template <int HT>
static void launch_grad_it(const GruArgs& a, int itp, dim3 grid, hipStream_t s, bool coop) {
  if (itp == 1) launch_grad_kind<HT, 1>(a, grid, s, coop);
  else if (itp == 2) launch_grad_kind<HT, 2>(a, grid, s, coop);
  else if (itp == 3) launch_grad_kind<HT, 3>(a, grid, s, coop);
  else launch_grad_kind<HT, 4>(a, grid, s, coop);
}

extern "C" int d2d_gru_grad(const d2d_gru_desc* d, int32_t T, const void* obs, const void* actions,
                            const float* logp_old, const int64_t* logp_strides, const float* weight,
                            const int64_t* weight_strides, float clip, float beta, float scale, float* g_w_ih,
                            float* g_w_hh, float* g_b_ih, float* g_b_hh, float* g_w1, float* g_b1, float* g_w2,
                            float* g_b2, float* stats, float* workspace, int64_t workspace_floats, void* stream) {
  int rc = check_gru_desc(d, obs);
  if (rc) return rc;
  if (!obs || !weight || !weight_strides || !g_w_ih || !g_w_hh || !g_b_ih || !g_b_hh || !g_w1 || !g_b1 || !g_w2 ||
      !g_b2 || !workspace || (d->kind != 2 && (!actions || !logp_old || !logp_strides))) {
    d2d_set_error("d2d_gru_grad: NULL argument");
    return D2D_EINVAL;
  }
  if (T < 0 || (T > 0 && T % d->episode_length != 0)) {
    d2d_set_error("d2d_gru_grad: T=%d is not a whole number of %d-slot episodes", T, d->episode_length);
    return D2D_EINVAL;
  }
  const bool history = g_gru_grad_history.load(std::memory_order_relaxed) != 0;  // one snapshot per launch
  const int64_t need = gru_grad_workspace(d, T, history);
  if (workspace_floats < need) {
    d2d_set_error("workspace %lld < %lld floats (D2D_OPT_GRU_GRAD_HISTORY=%d: set the option before the "
                  "d2d_gru_grad_workspace query)", (long long)workspace_floats, (long long)need, (int)history);
    return D2D_EINVAL;
  }
  GruArgs a = make_gru_args(d, T, obs);
  a.actions = actions; a.logp_old = logp_old; a.weight = weight;
  for (int q = 0; q < 3; ++q) {
    a.lo_st[q] = logp_strides ? logp_strides[q] : 0;
    a.w_st[q] = weight_strides[q];
  }
  a.clip_lo = 1.f - clip; a.clip_hi = 1.f + clip; a.beta = beta; a.scale = scale;
  const int64_t tiles = (int64_t)T * a.env_tiles;
  a.G = gru_grad_blocks(a.N, tiles);
  const GruOff o(a.H, a.F, a.A);
  a.P = o.P;
  const int ht = (a.H + 15) / 16, htp = ht <= 1 ? 1 : ht <= 2 ? 2 : 4, itp = gru_input_tiles(a.F);
  const bool coop = gru_coop(htp, itp, a.ov.u8 != 0, history);
  const GruWs ws = gru_ws_layout(a.G, a.N, a.P, a.L, htp, itp, coop);
  a.partial = workspace + ws.partial;
  a.hist = workspace + ws.hist;
  a.wimg = workspace + ws.wimg;
  a.hacc = workspace + ws.hacc;
  a.himg = workspace + ws.himg;
  a.ghist = workspace + ws.ghist;
  a.gpart = workspace + ws.gpart;
  if (a.N == 0) return D2D_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  {
    if (kGradSplit) {
      if (htp == 1) launch_wih_split<1>(a, itp, s);
      else if (htp == 2) launch_wih_split<2>(a, itp, s);
      else launch_wih_split<4>(a, itp, s);
    } else {
      const int64_t n = (int64_t)a.N * 3 * 16 * htp * 16 * itp;
      hipLaunchKernelGGL(gru_wih_image_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.w, a.N, a.H, a.F,
                         16 * htp, 16 * itp, a.wimg);
    }
    const int64_t nh = (int64_t)a.N * (16 * htp * 16 * htp + 16 * 16 * htp + 16 * htp + 16);
    const dim3 gh((unsigned)((nh + 255) / 256));
    if (htp == 1) hipLaunchKernelGGL(gru_head_image_kernel<1>, gh, dim3(256), 0, s, a.w, a.N, a.H, a.A, a.himg);
    else if (htp == 2) hipLaunchKernelGGL(gru_head_image_kernel<2>, gh, dim3(256), 0, s, a.w, a.N, a.H, a.A, a.himg);
    else hipLaunchKernelGGL(gru_head_image_kernel<4>, gh, dim3(256), 0, s, a.w, a.N, a.H, a.A, a.himg);
  }
  if (tiles == 0) {
    D2D_CHECK_HIP(hipMemsetAsync(workspace, 0, sizeof(float) * (size_t)a.N * a.P, s));
    a.G = 1;
  } else {
    dim3 grid(a.N, a.G);
    if (ht <= 1) launch_grad_it<1>(a, itp, grid, s, false);
    else if (ht <= 2) launch_grad_it<2>(a, itp, grid, s, false);
    else launch_grad_it<4>(a, itp, grid, s, coop);
    D2D_CHECK_HIP(hipGetLastError());
  }
  const int64_t n = (int64_t)a.N * a.P;
  hipLaunchKernelGGL(gru_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a.partial, a.G, a.N, a.P,
                     a.H, a.F, a.A, g_w_ih, g_w_hh, g_b_ih, g_b_hh, g_w1, g_b1, g_w2, g_b2, stats);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}
