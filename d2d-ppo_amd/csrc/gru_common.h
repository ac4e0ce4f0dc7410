// GRU window policies (the reference's RNN module, /root/reference/algorithms/ippo.py:14-51 ==
// d2d_ppo.py:24-59) on gfx950: shared pieces of the behaviour-policy kernel and the BPTT update
// kernel (gru_kernels.hip).
//
//   r = sigmoid(W_ir x + b_ir + W_hr h + b_hr)          torch.nn.GRU, gate order (r, z, n)
//   z = sigmoid(W_iz x + b_iz + W_hz h + b_hz)
//   n = tanh   (W_in x + b_in + r * (W_hn h + b_hn))
//   h' = (1 - z) * n + z * h                             h0 = 0 for every window
//   head: relu(W1 h_L + b1) -> W2 . + b2 -> sigmoid (combinatorial) / softmax / none (value)
//
// Layout (v_mfma_f32_16x16x4_f32, lane = (g, i), g = lane >> 4, i = lane & 15): one 16-sample
// tile per wave, the sample (env) on i.  Gate pre-activations are computed transposed,
// G^T[gate row][sample] = W . [x | h]^T, so an accumulator tile holds gate rows 16T + 4g + r of
// sample i -- and the r, z and n rows of hidden unit u = 16t + 4g + r sit in the SAME lane and
// register (tiles t, HT + t, 2HT + t): the gate math is lane-local, and the new h lands exactly
// where the next step's MFMA wants its B operand with the k order permuted to
// kidx(s, g) = 16 (s >> 2) + 4 g + (s & 3) (k-step s, lane group g).  No data movement
// between steps.  fp32 MFMA: every product exact, fp32 accumulation -- the torch fp32 numerics to
// ~1e-7 relative per step.
//
// Gate-row index R in [0, 3 HW), HW = 16 HT: gate G = R / HW, unit u = R % HW (rows with u >= H are
// zero and keep their h at 0).  Input column F of the input image carries the biases (x_F = 1):
// b_ir + b_hr, b_iz + b_hz, b_in; b_hn is added to the recurrent n part separately.
#pragma once
#include "mlp_common.h"

namespace d2d {

struct GruW {  // agent-stacked torch tensors (StackedNets kind "rnn")
  const float *w_ih, *w_hh, *b_ih, *b_hh;  // [N][3H][F], [N][3H][H], [N][3H], [N][3H]
  const float *w1, *b1, *w2, *b2;          // layers.0 [N][H][H], [N][H]; layers.2 [N][A][H], [N][A]
};

// A zero the compiler cannot see through (an SGPR through an empty volatile asm).  Weight-image
// addresses offset by it inside a loop are loop-variant, so the fragment loads of every window step /
// tile are not hoisted out of the loop into hundreds of registers (LDS and the images are never
// written inside those loops, which would otherwise make the loads invariant).
__device__ __forceinline__ int opaque_zero() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// LDS weight images, fp32, row-major with an XOR swizzle of the 4-float groups (row-dependent)
// so that the 16 rows of a ds_read_b128 A fragment hit distinct banks.  W = 16, 32 or 64.
template <int W>
__device__ __forceinline__ int swz(int row, int col) {
  return row * W + (col ^ ((row & (W / 4 - 1)) << 2));
}
template <int W>
__device__ __forceinline__ f32x4 lds4(const float* img, int row, int col4) {
  return *reinterpret_cast<const f32x4*>(img + swz<W>(row, col4));
}
// Per-lane offsets of the A-fragment reads of a W-wide image: row 16T + i, columns [16q + 4g, +4)
// (forward), and row 16T + 4g + s, column 16t + i (transposed), both = 16 T W + a per-lane offset
// independent of T (the swizzle only reads row bits below 4), so every tile T is an immediate
// offset from a handful of registers instead of one computed address per (T, q) / (T, s, t).
template <int W>
struct SwzOff {
  int fwd[W / 16];
  int tr[W / 16][4];
  __device__ __forceinline__ SwzOff(int g, int i) {
#pragma unroll
    for (int q = 0; q < W / 16; ++q) {
      fwd[q] = swz<W>(i, 16 * q + 4 * g);
#pragma unroll
      for (int s = 0; s < 4; ++s) tr[q][s] = swz<W>(4 * g + s, 16 * q + i);
    }
  }
};

// 1 + e^(kS v) to ~1 ulp on the hardware exp2 (the sigmoid / tanh denominators): kS v log2(e) is
// carried as th + tl (FMA residual plus the low part of log2 e), 2^tl ~ 1 + tl ln 2, and the 1 + is
// one more FMA.  (__expf rounds v * log2 e first: ~|v| ulp of error, which the recurrence accumulates
// over the window.)  kS = 1 or 2 scales log2 e's split exactly.  The file is built with
// -ffp-contract=off (the env kernels' oracle-exact arithmetic), so every multiply-add of the gate math
// is an explicit fmaf: one VALU and one rounding instead of two of each (gate math 36 -> 25 VALU per
// element).
template <int kS = 1>
__device__ __forceinline__ float one_plus_exp_acc(float v) {
  const float kL = 1.44269502162933349609375f * kS, kLlo = 1.925963033500e-08f * kS;
  const float th = v * kL;
  const float tl = fmaf(v, kLlo, fmaf(v, kL, -th));
  return fmaf(__builtin_amdgcn_exp2f(th), fmaf(tl, 0.693147180559945f, 1.f), 1.f);
}
__device__ __forceinline__ float sigmoidf_(float v) { return __builtin_amdgcn_rcpf(one_plus_exp_acc(-v)); }
// tanh(v) = 1 - 2 / (e^{2v} + 1): absolute error ~1e-7, saturates cleanly at +-1
__device__ __forceinline__ float tanhf_(float v) { return fmaf(-2.f, __builtin_amdgcn_rcpf(one_plus_exp_acc<2>(v)), 1.f); }
// the candidate gate n = tanh(W_in x + b_in + r (W_hn h + b_hn)) from its two pre-activation parts
__device__ __forceinline__ float gru_n(float ni, float rr, float nh) { return tanhf_(fmaf(rr, nh, ni)); }

// Fill the input / recurrent images of agent k (all threads of the workgroup).
template <int HT, int IT>
__device__ void load_gru_images(float* wih_s, float* whh_s, const GruW& w, int k, int H, int F, int tid, int nthr) {
  constexpr int HW = 16 * HT, IW = 16 * IT, R3 = 3 * HW;
  const float* Wih = w.w_ih + (size_t)k * 3 * H * F;
  const float* Whh = w.w_hh + (size_t)k * 3 * H * H;
  const float* bih = w.b_ih + (size_t)k * 3 * H;
  const float* bhh = w.b_hh + (size_t)k * 3 * H;
  for (int idx = tid; idx < R3 * IW; idx += nthr) {
    const int R = idx / IW, c = idx - R * IW, G = R / HW, u = R - G * HW;
    float v = 0.f;
    if (u < H) {
      const int src = G * H + u;
      if (c < F) v = Wih[(size_t)src * F + c];
      else if (c == F) v = G < 2 ? bih[src] + bhh[src] : bih[src];
    }
    wih_s[swz<IW>(R, c)] = v;
  }
  for (int idx = tid; idx < R3 * HW; idx += nthr) {
    const int R = idx / HW, c = idx - R * HW, G = R / HW, u = R - G * HW;
    whh_s[swz<HW>(R, c)] = (u < H && c < H) ? Whh[(size_t)(G * H + u) * H + c] : 0.f;
  }
}

// The rollout buffer as the GRU kernels read it: fp32 rows [..][N][F] or (u8) the env kernel's
// compact record [..][N][RB] (D2D_OBS_U8: one byte per input, int8 on the columns sgn marks).
struct ObsView {
  const uint8_t* base;
  int64_t rows;          // T * E * N
  int RB, N, F, u8;      // row bytes (4 F or D2D_RECORD_BYTES(F))
  const uint32_t* sgn;   // u8: [N][RB / 32] int8-column masks
};

// agent k's int8-column masks of the record (wave-uniform: scalar registers, not VGPRs the update
// kernel cannot spare); bit of column col = bit col & 31 of word col >> 5
template <int IT>
struct XSigns {
  uint32_t w[(IT + 1) / 2];
  __device__ __forceinline__ XSigns(const ObsView& ov, int k) {
#pragma unroll
    for (int c = 0; c < (IT + 1) / 2; ++c) w[c] = ov.u8 ? ov.sgn[(size_t)k * (ov.RB >> 5) + c] : 0u;
  }
  __device__ __forceinline__ uint32_t bit(int col) const { return (w[col >> 5] >> (col & 31)) & 1u; }
  // flags of columns col .. col + 3 (col % 4 == 0)
  __device__ __forceinline__ uint32_t bits4(int col) const { return (w[col >> 5] >> (col & 31)) & 0xFu; }
};

// x tile of one window step: lane (g, i) <- x[env i][16q + 4g + r] (q < IT, r < 4), the bias
// column F = 1, columns past F = 0.  `row0` = row index (slot, e0, agent k) of env e0; consecutive
// envs are N rows apart; rows of envs >= E read 0 through the range-checked buffer descriptor
// (zero: the x of a front-padding step, bias column only).
// A range-checked buffer descriptor from WAVE-UNIFORM values, read through readfirstlane: the
// compiler cannot always prove a base / extent uniform (they derive from the tile and window step),
// and a descriptor it takes for divergent costs a waterfall loop (readfirstlane, compare, exec
// masking, one load per pass) around every buffer load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint32_t nbytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
}

// descriptor of the rows from row0 on (row0 and zero wave-uniform; zero: none -- reads return 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const ObsView& ov, size_t row0, bool zero) {
  const int64_t rest = (ov.rows - (int64_t)row0) * ov.RB;
  const uint32_t nbytes = zero || rest <= 0 ? 0u : rest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)rest;
  return uniform_rsrc(ov.base + row0 * ov.RB, nbytes);
}

template <int IT>
struct XRaw {     // the raw words of one x tile (issued ahead of use: decode_x waits for them)
  uint32_t w[IT][4];  // fp32 rows: inputs 16q + 4g + r; record: w[q][0] = bytes 16q + 4g .. + 3
  bool zero;
};
template <int IT>
__device__ __forceinline__ void load_x_raw(XRaw<IT>& xr, const ObsView& ov, size_t row0, int g, int i, bool env_ok,
                                           bool zero) {
  const __amdgpu_buffer_rsrc_t rsrc = rows_rsrc(ov, row0, zero);
  const uint32_t vbase = env_ok ? (uint32_t)(i * ov.N * ov.RB) : 0x80000000u;
  xr.zero = zero;
#pragma unroll
  for (int q = 0; q < IT; ++q) {
    if (ov.u8) {  // wave-uniform
      xr.w[q][0] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vbase + (uint32_t)(16 * q + 4 * g), 0, 0);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        xr.w[q][r] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vbase + 4u * (uint32_t)(16 * q + 4 * g + r), 0, 0);
    }
  }
}
template <int IT>
__device__ __forceinline__ void decode_x(float (&x)[IT][4], const XRaw<IT>& xr, const ObsView& ov,
                                         const XSigns<IT>& sg, int g) {
  const int F = ov.F;
#pragma unroll
  for (int q = 0; q < IT; ++q) {
    if (ov.u8) {  // the record row holds the bias input 1 at column F, zeros past it (a padding step
                  // reads nothing: its bias input is set here)
      const uint32_t m = sign_bytes(sg.bits4(16 * q + 4 * g));
#pragma unroll
      for (int r = 0; r < 4; ++r) x[q][r] = (xr.zero && 16 * q + 4 * g + r == F) ? 1.f : rec_byte(xr.w[q][0], r, m);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = 16 * q + 4 * g + r;
        x[q][r] = col < F ? uf(xr.w[q][r]) : col == F ? 1.f : 0.f;
      }
    }
  }
}
// x tile of one window step: lane (g, i) <- x[env i][16q + 4g + r] (q < IT, r < 4), the bias
// column F = 1, columns past F = 0.  `row0` = row index (slot, e0, agent k) of env e0; consecutive
// envs are N rows apart; rows of envs >= E read 0 through the range-checked buffer descriptor
// (zero: the x of a front-padding step, bias column only).
template <int IT>
__device__ __forceinline__ void load_x(float (&x)[IT][4], const ObsView& ov, size_t row0, const XSigns<IT>& sg, int g,
                                       int i, bool env_ok, bool zero) {
  XRaw<IT> xr;
  load_x_raw<IT>(xr, ov, row0, g, i, env_ok, zero);
  decode_x<IT>(x, xr, ov, sg, g);
}

// Pre-activations of one step: rz[T] (T < 2 HT: input + recurrent + both biases of r / z rows),
// ni[t] (input part of n incl. b_in), nh[t] (recurrent part of n incl. b_hn).  h_zero: h = 0 (the
// recurrent products vanish).  W_ih from the swizzled LDS image (WIH_LDS) or from the same image
// unswizzled in global memory (L2-resident; the update kernel).
template <int HT, int IT, bool WIH_LDS>
__device__ __forceinline__ void gru_preact(const float* wih, const float* whh_s, const SwzOff<16 * IT>& oi,
                                           const SwzOff<16 * HT>& oh, const float (&x)[IT][4],
                                           const float (&h)[HT][4], const f32x4 (&bhn)[HT], f32x4 (&rz)[2 * HT],
                                           f32x4 (&ni)[HT], f32x4 (&nh)[HT], int g, int i, bool h_zero) {
  constexpr int HW = 16 * HT, IW = 16 * IT;
#pragma unroll
  for (int T = 0; T < 3 * HT; ++T) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < IT; ++q) {
      f32x4 wv;
      if constexpr (WIH_LDS) wv = *reinterpret_cast<const f32x4*>(wih + 16 * T * IW + oi.fwd[q]);
      else wv = *reinterpret_cast<const f32x4*>(wih + (size_t)(16 * T + i) * IW + 16 * q + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = mfma4(wv[r], x[q][r], acc);
    }
    if (T < 2 * HT) rz[T] = acc;
    else ni[T - 2 * HT] = acc;
  }
#pragma unroll
  for (int t = 0; t < HT; ++t) nh[t] = bhn[t];
  if (h_zero) return;
#pragma unroll
  for (int T = 0; T < 3 * HT; ++T) {
    f32x4 acc = T < 2 * HT ? rz[T] : nh[T - 2 * HT];
#pragma unroll
    for (int q = 0; q < HT; ++q) {
      const f32x4 wv = *reinterpret_cast<const f32x4*>(whh_s + 16 * T * HW + oh.fwd[q]);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = mfma4(wv[r], h[q][r], acc);
    }
    if (T < 2 * HT) rz[T] = acc;
    else nh[T - 2 * HT] = acc;
  }
}

// Gate math in place: h <- (1 - z) n + z h.  Optionally returns r, z, n (the backward recomputes).
template <int HT>
__device__ __forceinline__ void gru_gates(const f32x4 (&rz)[2 * HT], const f32x4 (&ni)[HT], const f32x4 (&nh)[HT],
                                          float (&h)[HT][4]) {
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float rr = sigmoidf_(rz[t][r]), zz = sigmoidf_(rz[HT + t][r]);
      const float nn = gru_n(ni[t][r], rr, nh[t][r]);
      h[t][r] = fmaf(zz, h[t][r] - nn, nn);  // (1 - z) n + z h
    }
}

// ---- exact-split bf16 variant of the step (the behaviour-policy kernel): v_mfma_f32_16x16x32_bf16
// on three-way bf16 splits of the weights and of h (mlp_common.h split3 / mfma_split: the six part
// products of weight >= 2^-16, fp32-accurate), 3.2x fewer MFMA cycles per step than the fp32
// 16x16x4 products; policy slot 95 -> 50 ms at 65,536 envs x 64 agents x 64-step windows.
//
// K chunk c of a 16-row tile covers two accumulator tiles: lane (g, i) holds x[q][r] / h[t][r] for
// q, t in {2c, 2c + 1}, so its B fragment takes k-slot 8g + j <-> input / unit 16 (2c + (j >> 2)) +
// 4g + (j & 3) -- the h of one step is the next step's B operand without any data movement -- and
// the weight images store each A fragment with the same permuted columns: fragment (T, c, part) of
// lane (g, i) = the 8 k-slots of row 16T + i, as one 16-byte word ([T][c][part][lane], conflict-free
// ds_read_b128).  Odd tile counts leave the upper half of the last chunk zero on both sides.
#ifndef D2D_GRU_ABLATE_X
#define D2D_GRU_ABLATE_X 0  // != 0 only in tools/gpu/build_ablate_gru.sh's variant 7 (timing only)
#endif
// bf16 high parts of 8 floats (their exact value when the inputs are bf16-exact)
__device__ __forceinline__ bf16x8 hi_frag_(const float (&v)[8]) {
  uint32_t u[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) u[q] = pack_hi(v[2 * q], v[2 * q + 1]);
  return as_frag(u);
}
__device__ __forceinline__ int chunk_col(int c, int g, int j) { return 16 * (2 * c + (j >> 2)) + 4 * g + (j & 3); }

template <int HT, int IT>
struct GruSplit {
  static constexpr int HW = 16 * HT, NT = 3 * HT, CH = (HT + 1) / 2, CI = (IT + 1) / 2;
  static constexpr int WIH = NT * CI * 3 * 64, WHH = NT * CH * 3 * 64;  // bf16x8 words
};

// Exact three-way split by rounding to nearest even: h = RNE(v), m = RNE(v - h), l = v - h - m (exact in
// bf16: v's 24 significant bits span three 8-bit parts).  The update kernel's cooperative path splits
// its W_hh image so, and its (h, m) parts ARE the RNE two-way split of W_hh: the dh = W_hh^T dg operands
// come from the same image (whh_dh_frag) instead of a second, transposed copy.  The forward products
// keep the six terms of mfma_split (|m| <= 2^-9 |v|, |l| <= 2^-18 |v|: the dropped ones are below 2^-26).
__device__ __forceinline__ Parts split3_rne(const float (&v)[8]) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  uint32_t H[4], M[4], L[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = v[2 * p], b = v[2 * p + 1];
    const bf2 hv = {(__bf16)a, (__bf16)b};
    H[p] = __builtin_bit_cast(uint32_t, hv);
    const float ar = a - ffrom(__builtin_amdgcn_perm(H[p], H[p], 0x01000c0cu)), br = b - ffrom(H[p] & 0xFFFF0000u);
    const bf2 mv = {(__bf16)ar, (__bf16)br};
    M[p] = __builtin_bit_cast(uint32_t, mv);
    const float al = ar - ffrom(__builtin_amdgcn_perm(M[p], M[p], 0x01000c0cu)), bl = br - ffrom(M[p] & 0xFFFF0000u);
    const bf2 lv = {(__bf16)al, (__bf16)bl};
    L[p] = __builtin_bit_cast(uint32_t, lv);
  }
  return {as_frag(H), as_frag(M), as_frag(L)};
}

// Fragment `rel` of agent k's input (inp) or recurrent split image: rel = (T * NC + c) * 64 + lane,
// its three parts stored 64 words apart ([T][c][part][lane]).  The input image carries the summed
// r / z biases and b_in at column F (x_F = 1), as load_gru_images does for the fp32 image.
template <int HT, int IT, bool RNE_HH = false>
__device__ __forceinline__ Parts split_frag(const GruW& w, int k, int H, int F, bool inp, int rel) {
  using S = GruSplit<HT, IT>;
  const int NC = inp ? S::CI : S::CH;
  const int T = rel / (NC * 64), c = (rel / 64) % NC, lane = rel & 63, g = lane >> 4, i = lane & 15;
  const int R = 16 * T + i, G = R / S::HW, u = R - G * S::HW, src = G * H + u;
  const float* Wih = w.w_ih + (size_t)k * 3 * H * F;
  const float* Whh = w.w_hh + (size_t)k * 3 * H * H;
  const float* bih = w.b_ih + (size_t)k * 3 * H;
  const float* bhh = w.b_hh + (size_t)k * 3 * H;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = chunk_col(c, g, j);
    v[j] = 0.f;
    if (u < H) {
      if (inp) {
        if (col < F) v[j] = Wih[(size_t)src * F + col];
        else if (col == F) v[j] = G < 2 ? bih[src] + bhh[src] : bih[src];
      } else if (col < H) {
        v[j] = Whh[(size_t)src * H + col];
      }
    }
    if (2 * c + (j >> 2) >= (inp ? IT : HT)) v[j] = 0.f;
  }
  return inp || !RNE_HH ? split3(v) : split3_rne(v);
}
__device__ __forceinline__ void store_parts(bf16x8* dst, const Parts& p) {
  dst[0] = p.h;
  dst[64] = p.m;
  dst[128] = p.l;
}
__device__ __forceinline__ int split_word(int rel) { return (rel >> 6) * 3 * 64 + (rel & 63); }
// Slot of lane l's A fragment in the W_hh split image (an involution inside each 16-slot group):
// 16 g + 4 ((i >> 2) ^ g) + (i & 3) for l = 16 g + i.  The forward reads (one 16-byte slot per lane)
// stay conflict-free, and the update kernel's transposing reads of the same image (the dh operands,
// whh_dh_frag) touch 16 distinct 16-byte bank groups per 16 lanes instead of 4.
__device__ __forceinline__ int whh_slot(int l) { return (l & 0x30) | ((((l >> 2) ^ (l >> 4)) & 3) << 2) | (l & 3); }

// Fill agent k's split images in LDS (all threads of the workgroup); either may be NULL.
// RNE_HH: the W_hh image split by rounding (split3_rne; the update kernel's cooperative path reads its
// dh operands from it), else by truncation like every other split image.
template <int HT, int IT, bool RNE_HH = false>
__device__ void load_gru_split_images(bf16x8* wih_b, bf16x8* whh_b, const GruW& w, int k, int H, int F, int tid,
                                      int nthr) {
  using S = GruSplit<HT, IT>;
  if (wih_b)
    for (int rel = tid; rel < S::NT * S::CI * 64; rel += nthr)
      store_parts(wih_b + split_word(rel), split_frag<HT, IT>(w, k, H, F, true, rel));
  if (whh_b)
    for (int rel = tid; rel < S::NT * S::CH * 64; rel += nthr)
      store_parts(whh_b + (split_word(rel) & ~63) + whh_slot(rel & 63),
                  split_frag<HT, IT, RNE_HH>(w, k, H, F, false, rel));
}

// Whether every input of a window step is bf16-exact (wave-uniform): always for the compact record,
// one ballot over the low halves for fp32 rows.
template <int IT>
__device__ __forceinline__ bool x_exact_step(const ObsView& ov, const float (&x)[IT][4]) {
  if (ov.u8) return true;
  uint32_t low = 0;
#pragma unroll
  for (int q = 0; q < IT; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) low |= fbits(x[q][r]) & 0xFFFFu;
  return __builtin_amdgcn_ballot_w64(low != 0) == 0;
}

// chunk c of a lane's two accumulator-layout tiles as 8 k-slot values
template <int NTL>
__device__ __forceinline__ void chunk_vals(float (&v)[8], const float (&t)[NTL][4], int c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 2 * c + (j >> 2) < NTL ? t[2 * c + (j >> 2)][j & 3] : 0.f;
}

// acc += W.X with all split products of weight >= 2^-24 (mfma_split's six plus m.l and l.m; only
// l.l dropped): ~2^-32 relative per product.  Ablation D2D_GRU_SPLIT8: measured 12 % slower per
// policy slot than the default six terms (2^-23 per product, the MLP kernels' choice) with the same
// worst-case log-prob error in tests/test_gru_gpu.py (tools/gpu/gru_diag.py: the window's fp32 gate
// math and the fp32 Bernoulli probabilities dominate, not the product split).
__device__ __forceinline__ f32x4 mfma_split8(const Parts& w, const Parts& x, f32x4 acc) {
  acc = mfma_bf16(w.m, x.l, acc);
  acc = mfma_bf16(w.l, x.m, acc);
  acc = mfma_bf16(w.h, x.l, acc);
  acc = mfma_bf16(w.m, x.m, acc);
  acc = mfma_bf16(w.l, x.h, acc);
  acc = mfma_bf16(w.h, x.m, acc);
  acc = mfma_bf16(w.m, x.h, acc);
  acc = mfma_bf16(w.h, x.h, acc);
  return acc;
}

// gru_preact on the split images.  x_exact (wave-uniform): every input of the step is bf16-exact
// (always for the compact record), so the input products need only the three weight parts.
// XEXACT: the inputs are bf16-exact by construction (the compact record) -- no per-tile branch on
// x_exact, so the input products of all gate tiles are one basic block and their W_ih fragment loads
// (from L2 in the update kernel) are issued together instead of one latency per gate tile.
template <int HT, int IT, bool XEXACT = false>
__device__ __forceinline__ void gru_preact_split(const bf16x8* wih_b, const bf16x8* whh_b, int lane,
                                                 const float (&x)[IT][4], bool x_exact, const float (&h)[HT][4],
                                                 const f32x4 (&bhn)[HT], f32x4 (&rz)[2 * HT], f32x4 (&ni)[HT],
                                                 f32x4 (&nh)[HT], bool h_zero) {
  using S = GruSplit<HT, IT>;
  if constexpr (XEXACT) {
    // exact inputs (the update kernel's cooperative path, W_ih fragments from L2): every W_ih fragment
    // load is issued first, the recurrent products (LDS-fed) run while they are in flight, and the
    // input products come last -- the L2 latency is paid once per step behind 144 MFMAs instead of at
    // the head of the step.  The input terms are summed in their own accumulator (smallest part first,
    // as mfma_split does) and added to the recurrent sum with one fp32 add: accumulating them into the
    // already large recurrent sum measured 50x the torch-fp32 band on the xp_load value-critic dW_ih.
    bf16x8 wi[S::NT][S::CI][3];
#pragma unroll
    for (int T = 0; T < S::NT; ++T)
#pragma unroll
      for (int c = 0; c < S::CI; ++c)
#pragma unroll
        for (int q = 0; q < 3; ++q) wi[T][c][q] = wih_b[((T * S::CI + c) * 3) * 64 + lane + 64 * q];
    bf16x8 xh[S::CI];
#pragma unroll
    for (int c = 0; c < S::CI; ++c) {
      float v[8];
      chunk_vals<IT>(v, x, c);
      xh[c] = hi_frag_(v);
    }
    f32x4 acc[S::NT];
#pragma unroll
    for (int T = 0; T < S::NT; ++T) acc[T] = T < 2 * HT ? f32x4{0.f, 0.f, 0.f, 0.f} : bhn[T - 2 * HT];
    if (!h_zero) {
      const int hl = whh_slot(lane);
      Parts hp[S::CH];
#pragma unroll
      for (int c = 0; c < S::CH; ++c) {
        float v[8];
        chunk_vals<HT>(v, h, c);
        hp[c] = split3(v);
      }
#pragma unroll
      for (int T = 0; T < S::NT; ++T)
#pragma unroll
        for (int c = 0; c < S::CH; ++c) {
          const bf16x8* wf = whh_b + ((T * S::CH + c) * 3) * 64 + hl;
          acc[T] = mfma_split(Parts{wf[0], wf[64], wf[128]}, hp[c], false, acc[T]);
        }
    }
#pragma unroll
    for (int T = 0; T < S::NT; ++T) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < (D2D_GRU_ABLATE_X ? 0 : S::CI); ++c) {
        a = mfma_bf16(wi[T][c][2], xh[c], a);
        a = mfma_bf16(wi[T][c][1], xh[c], a);
        a = mfma_bf16(wi[T][c][0], xh[c], a);
      }
      if (T < 2 * HT) {
        rz[T] = a + acc[T];
      } else {
        ni[T - 2 * HT] = a;
        nh[T - 2 * HT] = acc[T];
      }
    }
    return;
  }
  Parts xp[S::CI];
#pragma unroll
  for (int c = 0; c < S::CI; ++c) {
    float v[8];
    chunk_vals<IT>(v, x, c);
    if (x_exact) {
      xp[c].h = hi_frag_(v);
      xp[c].m = xp[c].l = bf16x8{};
    } else {
      xp[c] = split3(v);
    }
  }
#pragma unroll
  for (int T = 0; T < S::NT; ++T) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < (D2D_GRU_ABLATE_X ? 0 : S::CI); ++c) {  // (timing ablation: no input products)
      const bf16x8* wf = wih_b + ((T * S::CI + c) * 3) * 64 + lane;
      acc = mfma_split(Parts{wf[0], wf[64], wf[128]}, xp[c], x_exact, acc);
    }
    if (T < 2 * HT) rz[T] = acc;
    else ni[T - 2 * HT] = acc;
  }
#pragma unroll
  for (int t = 0; t < HT; ++t) nh[t] = bhn[t];
  if (h_zero) return;
  const int hl = whh_slot(lane);
  Parts hp[S::CH];
#pragma unroll
  for (int c = 0; c < S::CH; ++c) {
    float v[8];
    chunk_vals<HT>(v, h, c);
    hp[c] = split3(v);
  }
#pragma unroll
  for (int T = 0; T < S::NT; ++T) {
    f32x4 acc = T < 2 * HT ? rz[T] : nh[T - 2 * HT];
#pragma unroll
    for (int c = 0; c < S::CH; ++c) {
      const bf16x8* wf = whh_b + ((T * S::CH + c) * 3) * 64 + hl;
#if D2D_GRU_SPLIT8  // ablation: eight terms
      acc = mfma_split8(Parts{wf[0], wf[64], wf[128]}, hp[c], acc);
#else
      acc = mfma_split(Parts{wf[0], wf[64], wf[128]}, hp[c], false, acc);
#endif
    }
    if (T < 2 * HT) rz[T] = acc;
    else nh[T - 2 * HT] = acc;
  }
}

// b_hn of agent k in accumulator layout (unit 16t + 4g + r)
template <int HT>
__device__ __forceinline__ void load_bhn(f32x4 (&bhn)[HT], const GruW& w, int k, int H, int g) {
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int u = 16 * t + 4 * g + r;
      bhn[t][r] = u < H ? w.b_hh[(size_t)k * 3 * H + 2 * H + u] : 0.f;
    }
}

// Zero-padded head image of one agent: W1p [HW][HW], W2p [16][HW], b1p [HW], b2p [16] (HW = 16 HT):
// no masks in the fragment loads, every address an immediate offset from a per-lane base.
template <int HT>
struct HeadImg {
  static constexpr int HW = 16 * HT, W1 = 0, W2 = HW * HW, B1 = W2 + 16 * HW, B2 = B1 + HW, SIZE = B2 + 16;
};

// idx-th element of agent k's head image (threads of a workgroup or a grid fill it cooperatively)
template <int HT>
__device__ __forceinline__ float head_img_elem(const GruW& w, int k, int H, int A, int idx) {
  using HI = HeadImg<HT>;
  constexpr int HW = HI::HW;
  if (idx < HI::W2) {
    const int r = idx / HW, c = idx - r * HW;
    return (r < H && c < H) ? w.w1[((size_t)k * H + r) * H + c] : 0.f;
  }
  if (idx < HI::B1) {
    const int r = (idx - HI::W2) / HW, c = (idx - HI::W2) - r * HW;
    return (r < A && c < H) ? w.w2[((size_t)k * A + r) * H + c] : 0.f;
  }
  if (idx < HI::B2) {
    const int u = idx - HI::B1;
    return u < H ? w.b1[(size_t)k * H + u] : 0.f;
  }
  const int o = idx - HI::B2;
  return o < A ? w.b2[(size_t)k * A + o] : 0.f;
}

// Head forward: pre1 = W1 h + b1 (accumulator layout, unit 16t + 4g + r), y = relu(pre1),
// lg = W2 y + b2 (rows = output 4g + r, sample i), from the padded head image.
template <int HT>
__device__ __forceinline__ void gru_head(const float* img, const float (&h)[HT][4], f32x4 (&pre1)[HT],
                                         float (&y)[HT][4], f32x4& lg, int g, int i) {
  using HI = HeadImg<HT>;
  constexpr int HW = HI::HW;
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    f32x4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = img[HI::B1 + 16 * t + 4 * g + r];
#pragma unroll
    for (int q = 0; q < HT; ++q) {
      const f32x4 wv = *reinterpret_cast<const f32x4*>(img + HI::W1 + (16 * t + i) * HW + 16 * q + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = mfma4(wv[r], h[q][r], acc);
    }
    pre1[t] = acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) y[t][r] = relu(acc[r]);
  }
  f32x4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = img[HI::B2 + 4 * g + r];
#pragma unroll
  for (int q = 0; q < HT; ++q) {
    const f32x4 wv = *reinterpret_cast<const f32x4*>(img + HI::W2 + i * HW + 16 * q + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc = mfma4(wv[r], y[q][r], acc);
  }
  lg = acc;
}

}  // namespace d2d
