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
// column F (x = 1), so db1 is column F of dW1.  Precision: the forward (both layer-1
// orientations, dH) on the exact three-way bf16 split (mlp_common.h), the logits and dW2 on fp32
// MFMA -- fp32-accurate; the weight-gradient GEMMs dW1 = dH^T X and dW2 = h^T dZ on two-way RNE
// splits of their per-tile operands (<= 2^-17 relative per term).
// Parity with torch autograd: tests/test_update_gpu.py (2e-5 of max|grad| vs float64).
//
// Partial sums: every wave accumulates its tiles in registers; the four waves of a workgroup
// are summed in fixed order through LDS and written as one partial per (workgroup, agent);
// update_reduce_kernel sums the partials in fixed order.  No atomics: bitwise reproducible.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "ppo_epilogue.h"

#ifndef D2D_UPD_ABLATE
#define D2D_UPD_ABLATE 0  // != 0 only in tools/gpu/ablate_update.py's timing builds
#endif
#ifndef D2D_ACTOR_TR
// actor on the compact record: the sample-on-rows layer 1 (HN = X . W1^T: 3 MFMAs per hidden tile
// per half, its relu, the relu mask and the two-way split of relu(HN) for dW2) is not recomputed --
// relu(HT)'s split parts, already made for the logits, are transposed through LDS with
// ds_read_b64_tr_b16 into the dW2 operand layout, and their high part is the relu mask
#define D2D_ACTOR_TR 1
#endif
#ifndef D2D_CRITIC_MASK
// critic dV1 = sum_s dHv_s x_s^T with dHv = relu'(HV) * dv * v2 factored as
//   dV1[h][:] = v2[h] * sum_s M[s][h] (dv_s x_s),   M = relu'(HV) in {0, 1}
// M is exact in bf16 (no split); dv_s x_s is split two ways once per tile (16 values per lane)
// instead of dHv (32), the relu' select and the dv * v2 products go, and v2 scales the sums once
#define D2D_CRITIC_MASK 1
#endif
#ifndef D2D_LOGITS_SPLIT3
#define D2D_LOGITS_SPLIT3 1  // 0 (timing A/B only): relu(HT) on the two-way split in the logits
#endif
#ifndef D2D_SPLIT_DOT2
// split residuals v - (bf16 half): 2 (default since round 4) a v_perm / v_and plus one scalar v_sub_f32;
// 1: one v_dot2c_f32_bf16 (round 3; fewer VALU but each one issues at a higher price beside the MFMAs:
// actor 1.85 -> 1.83 ms, critic 0.776 -> 0.747 ms per 26 M agent-samples with 2, profiles/r04/upd_ab_sub2.json);
// 0 (A/B only): the subtraction left to the compiler, which pairs it into v_pk_add_f32.  All three are exact
// (v - h is representable), so the gradients are bitwise the same
#define D2D_SPLIT_DOT2 2
#endif
#ifndef D2D_DW2_PAIRED
// 1 (A/B only): record-path actor dW2^T = relu(H)^T . dZ over both 16-sample halves at once, k-slots =
// 4 samples of half 0 | the same 4 of half 1: (h_h, h_m) x (dz_h, dz_m) in 3 MFMAs per hidden tile instead
// of 2 x 2 with the duplicated [dz_h | dz_h] and zero-padded [dz_m | 0] operands.  ~1.5 % faster, but its
// summation order differs from the fp32-row instantiation's, whose gradients the record path reproduces
// bit for bit (tests/test_record_gpu.py); off
#define D2D_DW2_PAIRED 0
#endif
#ifndef D2D_ACTOR_DZ_ONCE
// record-path actor, paired epilogue (A <= 8): dZ split three ways ONCE in the epilogue's paired layout (both
// halves at once) and the parts moved to each half's dH A operand by permlane32 swaps -- was a split per half of
// the swapped values; dW2's dZ operand (two-way RNE = the first two parts) reaches the sample-on-k layout as bf16
// through LDS with ds_read_b64_tr_b16 instead of an fp32 transpose and a second split; dH's relu mask applied to
// the split parts with packed u16 ops.  Bitwise the same operands (and so gradients) as before
#define D2D_ACTOR_DZ_ONCE 1
#endif
#ifndef D2D_UPD_WAVES
#define D2D_UPD_WAVES 2  // waves per SIMD the update kernels are register-budgeted for (KC = 1)
#endif
#ifndef D2D_LOGITS_BF16
// logits Z^T = W2 . relu(HT) on bf16 MFMAs: W2's three-way split against a three-way RNE split of
// relu(HT) (every product term down to 2^-24), 3 x 16 instead of 4 x 32 MFMA cycles per hidden tile
// (actor kernel 2.55 -> 2.44 ms per 26 M agent-samples); 0 = v_mfma_f32_16x16x4_f32 (exact fmaf chain)
#define D2D_LOGITS_BF16 1
#endif

namespace d2d {

struct UpdArgs {
  int T, E, N, F, H, A, kind, mask_bytes;
  int tiles_per_t, n_tiles, G, P;
  float inv_A, clip_lo, clip_hi, beta, scale;
  const float *w1, *b1, *w2, *b2;  // actor (Policy) or critic (Value: A = 1)
  const float* obs;                 // [T][E][N][F] (D2D_OBS_F32)
  const uint8_t* rec;               // [T][E][N][32 KC] compact record (D2D_OBS_U8)
  const uint32_t* sgn;              // [N][KC] int8-column masks of the record
  const void* actions;              // [T][E][N] masks (kind 0) / ids (kind 1)
  const float* logp_old;            // actor: element (t, e, k) at t*st[0] + e*st[1] + k*st[2]
  const float* weight;              // actor: advantage / M; critic: return target
  int64_t lo_st[3], w_st[3];
  int64_t lo_ext, w_ext;            // 1 + the largest element offset of logp_old / weight (floats)
  float* partial;                   // [G][N][P]
  float* vout;                      // critic: NULL, or the value of sample (t, e, k) at t*v_st[0] + e*v_st[1] + k*v_st[2]
  int64_t v_st[3];
};


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
// Two-way round-to-nearest bf16 split of 4 floats: v = h + m + e, |e| <= 2^-17 |v| (the dW1 / dV1
// operand dH: a per-tile value used against 2 x-tiles only, where the 3-way split's VALU cost
// outweighs its MFMAs; the weight gradients then carry ~2^-17 relative error per product term,
// below the fp32 accumulation error of their 10^5-10^6-sample sums)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t rne2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32
  return __builtin_bit_cast(uint32_t, v);
}
// the low bf16 of a packed pair as fp32 bits (h << 16) on v_perm_b32: written as a shift, the
// compiler re-derives it from the pair's first operand (a second v_cvt_pk_bf16_f32 plus the shift)
__device__ __forceinline__ uint32_t bf16_lo_as_f32bits(uint32_t h) { return __builtin_amdgcn_perm(h, h, 0x01000c0cu); }
struct Parts2x4 {
  uint32_t h[2], m[2];
};
// v minus the low / high bf16 of a packed pair on one v_dot2c_f32_bf16 (h.lo * -1 + h.hi * 0 + v):
// the split residuals, exact (v - h is representable: h is v rounded to 8 bits); replaces the pair's
// unpacking (v_perm + v_and) and subtraction.  The (-1, 0) / (0, -1) bf16 pairs are held in SGPRs: the
// compiler encodes 0x0000BF80 as the inline constant -1.0, which the hardware does not read as that
// pair (tools/gpu/probe/dot2_probe.hip: 65,487 of 65,536 residuals wrong; register and 32-bit literal
// forms exact on all).  Contract: both values of the pair are finite.  The partner enters as h.x * 0, so
// an inf / NaN partner makes the finite value's residual NaN (the per-value subtraction kept them apart);
// the operands split here (relu(HT), dH, dZ, dv x) are finite for finite weights and inputs, and a
// non-finite one already makes its gradient tensor non-finite through h itself, as in torch autograd.
// Denormal values (|v| < 2^-126) may lose their residual (the probe prints what the hardware does):
// an absolute error below 1.2e-38 per operand, far under any gradient's fp32 resolution.
__device__ __forceinline__ uint32_t bf16_pair_neg1_lo() {
  uint32_t c;
  asm("s_mov_b32 %0, 0x0000bf80" : "=s"(c));
  return c;
}
__device__ __forceinline__ uint32_t bf16_pair_neg1_hi() {
  uint32_t c;
  asm("s_mov_b32 %0, 0xbf800000" : "=s"(c));
  return c;
}
// D2D_SPLIT_DOT2 == 2 (A/B): the residual as one v_perm / v_and plus one scalar v_sub_f32 (asm, so the
// compiler cannot pair the subtractions into v_pk_add_f32)
__device__ __forceinline__ float sub_f32_asm(float a, float b) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float sub_bf16_lo(float v, uint32_t h) {
#if D2D_SPLIT_DOT2 == 2
  return sub_f32_asm(v, ffrom(bf16_lo_as_f32bits(h)));
#elif !D2D_SPLIT_DOT2
  return v - ffrom(bf16_lo_as_f32bits(h));
#endif
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, h), __builtin_bit_cast(bf16x2_t, bf16_pair_neg1_lo()), v, false);
}
__device__ __forceinline__ float sub_bf16_hi(float v, uint32_t h) {
#if D2D_SPLIT_DOT2 == 2
  return sub_f32_asm(v, ffrom(h & 0xFFFF0000u));
#elif !D2D_SPLIT_DOT2
  return v - ffrom(h & 0xFFFF0000u);
#endif
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, h), __builtin_bit_cast(bf16x2_t, bf16_pair_neg1_hi()), v, false);
}
__device__ __forceinline__ Parts2x4 split2_4(const float (&v)[4]) {
  Parts2x4 o;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t h = rne2(v[2 * p], v[2 * p + 1]);
    o.h[p] = h;
    o.m[p] = rne2(sub_bf16_lo(v[2 * p], h), sub_bf16_hi(v[2 * p + 1], h));
  }
  return o;
}
// Three-way round-to-nearest split of 4 floats (v = h + m + l + e, |e| <= 2^-26 |v|): the two-way
// split plus the remainder's part
__device__ __forceinline__ Parts4 split3rne_4(const float (&v)[4]) {
  Parts4 o;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t h = rne2(v[2 * p], v[2 * p + 1]);
    const float r0 = sub_bf16_lo(v[2 * p], h), r1 = sub_bf16_hi(v[2 * p + 1], h);
    const uint32_t m = rne2(r0, r1);
    o.h[p] = h;
    o.m[p] = m;
    o.l[p] = rne2(sub_bf16_lo(r0, m), sub_bf16_hi(r1, m));
  }
  return o;
}
// two transposing LDS reads (four bf16 each, element 0 in the low half) as one MFMA operand
__device__ __forceinline__ bf16x8 cat_tr(v4i16 a, v4i16 b) {
  const uint2 x = __builtin_bit_cast(uint2, a), y = __builtin_bit_cast(uint2, b);
  const u32x4v v = {x.x, x.y, y.x, y.y};
  return __builtin_bit_cast(bf16x8, v);
}
// Compensated (Kahan) running sum of per-tile sums: the scalar gradient and loss accumulators of
// one lane add one tile sum per tile, 10^3-10^4 of them at the headline batch, where a plain fp32
// running sum drifts by ~n ulps (measured: the critic's db2 at 65,536 envs, 20x torch fp32's error)
struct KahanSum {
  float s = 0.f, c = 0.f;
  __device__ __forceinline__ void add(float x) {
    const float y = x - c;
    const float t = s + y;
    c = (t - s) - y;
    s = t;
  }
  __device__ __forceinline__ float value() const { return s; }
};

// bf16 1.0 / 0.0 for h > 0 (the relu derivative, torch's convention at 0) of two values, packed; from
// relu(h) (relu() above: the bit pattern is > 0 exactly when h > 0), one v_min_u32 each
// (asm: the compiler turns a plain min into a float compare + select, two instructions)
// Packed form: the two high halves side by side (v_perm_b32), min(., 1) per half (v_pk_min_u16) and
// x 0x3F80 per half (v_pk_mul_lo_u16): 3 VALU per pair instead of 4.  The high half of relu(h) is
// nonzero exactly when relu(h) >= 2^-133 (the actor's relu mask has the same bf16-underflow edge).
// (asm: the compiler turns the packed min and multiply into a compare + select per half)
__device__ __forceinline__ uint32_t relu_mask_pair(float r0, float r1) {
  const uint32_t hi = __builtin_amdgcn_perm(fbits(r1), fbits(r0), 0x07060302u);
  uint32_t m, o;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(hi), "s"(0x00010001u));
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(o) : "v"(m), "s"(0x3F803F80u));
  return o;
}

// v_pk_min_u16 / v_pk_mul_lo_u16 (asm: the compiler turns the packed forms into per-half compares + selects)
__device__ __forceinline__ uint32_t pk_min1_u16(uint32_t x) {
  uint32_t m;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(x), "s"(0x00010001u));
  return m;
}
__device__ __forceinline__ uint32_t pk_mul_lo_u16(uint32_t a, uint32_t b) {
  uint32_t o;
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b));
  return o;
}

// high parts only (bf16-exact values)
__device__ __forceinline__ bf16x8 hi_frag(const float (&v)[8]) {
  uint32_t u[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) u[q] = pack_hi(v[2 * q], v[2 * q + 1]);
  return as_frag(u);
}

// Per-sample scalars of one tile (slot t, envs e0 .., agent k) through a range-checked buffer
// descriptor based at the tile's first element: the 64-bit offset math is scalar (once per tile),
// each load is one buffer_load with a loop-invariant lane offset d * st[1] (d = the lane's sample
// within the tile).  Samples past the tensor read 0; those past E are masked by the callers.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sample_rsrc(const float* base, const int64_t (&st)[3], int64_t ext,
                                                              int t, int e0, int k) {
  const int64_t off = (int64_t)t * st[0] + (int64_t)e0 * st[1] + (int64_t)k * st[2];
  const int64_t rest = (ext - off) * 4;
  const uint32_t n = rest <= 0 ? 0u : rest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)rest;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + off), 0, n, 0x00020000);
}
__device__ __forceinline__ float ld_sample(const __amdgpu_buffer_rsrc_t& r, const int64_t (&st)[3], int d) {
  return uf(__builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)(d * (int)st[1]) * 4u, 0, 0));
}

// (slot t, first env e0) of a sample tile; a wave's tiles advance by a fixed stride, so the cursor
// moves without the per-tile scalar division tile / tiles_per_t (a ~20-instruction sequence, twice
// per tile: the look-ahead load and the staging)
struct TileCur {
  int tile, t, e0;
};
__device__ __forceinline__ TileCur tile_at(const UpdArgs& a, int tile) {
  const int t = tile / a.tiles_per_t;
  return TileCur{tile, t, (tile - t * a.tiles_per_t) * 32};
}
struct TileStride {
  int tiles, dt, de, row;  // stride in tiles = dt * tiles_per_t + de / 32; row = 32 * tiles_per_t
  __device__ __forceinline__ TileStride(const UpdArgs& a, int stride) {
    tiles = stride;
    dt = stride / a.tiles_per_t;
    de = (stride - dt * a.tiles_per_t) * 32;
    row = 32 * a.tiles_per_t;
  }
  __device__ __forceinline__ TileCur next(TileCur c) const {
    c.tile += tiles;
    c.t += dt;
    c.e0 += de;
    if (c.e0 >= row) {
      c.e0 -= row;
      c.t += 1;
    }
    return c;
  }
};

// Per-tile inputs of the actor kernel, loaded one tile ahead (registers): the obs rows of the
// 32 samples (lane (g, i) of half s: x[sample 16s + i][32c + 8g + j], raw -- columns past F and
// samples past E are fixed up by stage_tile) and the per-sample action / logp_old / weight of
// the epilogue lanes (PAIR: lane (g, i) serves sample 16 (g >> 1) + i; else sample 16s + i).
// Raw input rows of one tile, lane (g, i) of half s: inputs 32c + 8g .. 32c + 8g + 7 of sample
// 16s + i as 8 fp32 words, or (U8) as the 8 bytes of the compact record (2 words, a quarter of
// the registers held across the look-ahead)
template <int KC, bool U8>
struct XRows {
  uint32_t v[2][KC][U8 ? 2 : 8];
  // input j of chunk c of half s (U8: sm[c][h] = this lane's int8 byte masks of word h, rec_byte)
  __device__ __forceinline__ float at(int s, int c, int j, const uint32_t (&sm)[KC][2]) const {
    if constexpr (U8) return rec_byte(v[s][c][j >> 2], j & 3, sm[c][j >> 2]);
    else return uf(v[s][c][j]);
  }
};

template <int KC, bool PAIR, bool U8>
struct ActorIn {
  XRows<KC, U8> x;
  uint32_t act[PAIR ? 1 : 2];
  float lo[PAIR ? 1 : 2], w[PAIR ? 1 : 2];
};

// obs rows of one tile through a range-checked buffer descriptor based at the tile's first row
// (rows of samples past E, or past the buffer, read as 0)
template <int KC, bool U8>
__device__ __forceinline__ void load_rows(XRows<KC, U8>& x, const UpdArgs& a, int t, int e0, int k, int g, int i) {
  const int RB = U8 ? 32 * KC : 4 * a.F;  // row bytes
  const size_t row0 = ((size_t)t * a.E + e0) * a.N + k;
  const int64_t rest = ((int64_t)a.T * a.E * a.N - (int64_t)row0) * RB;
  const uint32_t nbytes = rest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)rest;
  const uint8_t* base = (U8 ? a.rec : reinterpret_cast<const uint8_t*>(a.obs)) + row0 * RB;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, nbytes, 0x00020000);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int e = e0 + 16 * s + i;
    const uint32_t vo = e < a.E ? (uint32_t)((16 * s + i) * a.N * RB) + (U8 ? 8 : 32) * g : 0x80000000u;
#pragma unroll
    for (int c = 0; c < KC; ++c)
#pragma unroll
      for (int j = 0; j < (U8 ? 2 : 8); ++j)
        x.v[s][c][j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vo + (U8 ? 32 * c + 4 * j : 4 * (32 * c + j)), 0, 0);
  }
}

// this lane's int8 byte masks of agent k's record words (columns 32c + 8g + 4h + r, rec_byte)
template <int KC, bool U8>
__device__ __forceinline__ void record_signs(uint32_t (&sm)[KC][2], const UpdArgs& a, int k, int g) {
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const uint32_t sg = U8 ? (a.sgn[(size_t)k * KC + c] >> (8 * g)) & 0xFFu : 0u;
    sm[c][0] = sign_bytes(sg & 0xFu);
    sm[c][1] = sign_bytes(sg >> 4);
  }
}

template <int KC, bool PAIR, bool U8>
__device__ __forceinline__ void load_actor_in(ActorIn<KC, PAIR, U8>& in, const UpdArgs& a, TileCur c, int k, int g,
                                              int i) {
  const int t = c.t, e0 = c.e0;
  load_rows<KC, U8>(in.x, a, t, e0, k, g, i);
  const __amdgpu_buffer_rsrc_t rl = sample_rsrc(a.logp_old, a.lo_st, a.lo_ext, t, e0, k);
  const __amdgpu_buffer_rsrc_t rw = sample_rsrc(a.weight, a.w_st, a.w_ext, t, e0, k);
  // actions [T][E][N] (ids: 1 byte, masks: mask_bytes): byte offset of the tile's first cell
  const int mb = a.kind == 1 ? 1 : a.mask_bytes;
  const int64_t cell0 = ((int64_t)t * a.E + e0) * a.N + k;
  const int64_t arest = ((int64_t)a.T * a.E * a.N - cell0) * mb;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(reinterpret_cast<const uint8_t*>(a.actions) + cell0 * mb), 0,
      arest <= 0 ? 0u : arest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)arest, 0x00020000);
#pragma unroll
  for (int s = 0; s < (PAIR ? 1 : 2); ++s) {
    const int d = 16 * (PAIR ? (g >> 1) : s) + i;  // the lane's sample in the tile
    const uint32_t ao = (uint32_t)(d * a.N * mb);
    in.act[s] = mb == 1 ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(ra, ao, 0, 0)
              : mb == 2 ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(ra, ao, 0, 0)
                        : __builtin_amdgcn_raw_buffer_load_b32(ra, ao, 0, 0);
    in.lo[s] = ld_sample(rl, a.lo_st, d);
    in.w[s] = ld_sample(rw, a.w_st, d);
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

template <int XS>
__device__ __forceinline__ void lds_row(float (&v)[8], const float (*xw)[XS], int row, int col) {
  const f32x4 p = *reinterpret_cast<const f32x4*>(&xw[row][col]), q = *reinterpret_cast<const f32x4*>(&xw[row][col + 4]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = p[j];
    v[4 + j] = q[j];
  }
}


// ------------------------------------------------------------------------- actor gradients
// KC = input chunks of 32 (F + 1 <= 32 KC), HT = hidden tiles of 16 (H <= 16 HT), A <= 16;
// PAIR (A <= 8): one epilogue pass serves both halves (lanes 0-31 half 0, 32-63 half 1).
// Products: layer 1 (both orientations) and dH on the exact bf16 split (the weight splits are
// made once; x is bf16-exact on env observations, so 3 MFMAs per 16x16x32); the logits on
// v_mfma_f32_16x16x4_f32 (an exact fmaf chain) straight from the accumulator registers; the
// weight gradients dW1, dW2 on two-way RNE splits of their per-tile operands.
template <int KC, int HT, int KIND, bool PAIR, bool U8, int AFIX = 0>
__global__ __launch_bounds__(256, (KC == 1 && HT <= 4) ? D2D_UPD_WAVES : 1) void ppo_actor_grad_kernel(UpdArgs a) {
  constexpr int QT = 2 * KC;  // input tiles of 16 in dW1
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  int k, by;
  xcd_block(k, by);  // k = agent, by = sample-chunk group
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, A = AFIX > 0 ? AFIX : a.A, F = a.F;
  // the transposed-relu(HT) path (D2D_ACTOR_TR): record inputs only (always bf16-exact, so the
  // fractional-input body never runs) and the bf16 logits, whose split parts it transposes
  constexpr bool TR = U8 && D2D_LOGITS_BF16 && D2D_ACTOR_TR;

  // ---- weights of agent k: the W1 split in registers; the two W2 operand sets (used once per
  // half per hidden tile) in LDS, shared by the workgroup's four waves
  Parts w1p[HT][KC];
  f32x4 b2i;
  // dH's three B operands [h|l], [m|h], [h|m], stored whole so one ds_read_b128 lands each in
  // the four consecutive registers the MFMA reads (no operand assembly moves)
  __shared__ __attribute__((aligned(16))) bf16x8 w2b_s[HT][3][64];
#if D2D_LOGITS_BF16
  __shared__ __attribute__((aligned(16))) bf16x8 w2z_s[HT][3][64];       // Z^T's bf16 A operands [h|h], [m|m], [l|h]
#else
  __shared__ __attribute__((aligned(16))) float w2f_s[HT][64][4];        // Z^T's fp32 A operand
#endif
  {
    const float* W1 = a.w1 + (size_t)k * H * F;
    const float* W2 = a.w2 + (size_t)k * A * H;
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
    }
    for (int t = wave; t < HT; t += 4) {
      const int hrow = 16 * t + i;
      const bool hok = hrow < H;
      // B operand of dH = dZ . W2: k-slot (g, j < 4) <-> action 4g + j, column = hidden 16t + i
      float wb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) wb[j] = (hok && 4 * g + j < A) ? W2[(size_t)(4 * g + j) * H + hrow] : 0.f;
      const Parts4 p4 = split3_4(wb);
      w2b_s[t][0][lane] = cat(p4.h, p4.l);
      w2b_s[t][1][lane] = cat(p4.m, p4.h);
      w2b_s[t][2][lane] = cat(p4.h, p4.m);
      // A operand of Z^T = W2 . relu(HT): row = action i, k = hidden 16t + 4g + r
      float wz[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = 16 * t + 4 * g + r;
        wz[r] = (i < A && hid < H) ? W2[(size_t)i * H + hid] : 0.f;
      }
#if !D2D_LOGITS_BF16
#pragma unroll
      for (int r = 0; r < 4; ++r) w2f_s[t][lane][r] = wz[r];
#else
      {
        const Parts4 pz = split3_4(wz);
        w2z_s[t][0][lane] = cat(pz.h, pz.h);
        w2z_s[t][1][lane] = cat(pz.m, pz.m);
#if D2D_LOGITS_SPLIT3
        w2z_s[t][2][lane] = cat(pz.l, pz.h);
#else
        w2z_s[t][2][lane] = cat(pz.l, pz.l);
#endif
      }
#endif
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) b2i[r] = 4 * g + r < A ? a.b2[(size_t)k * A + 4 * g + r] : 0.f;
    __syncthreads();
  }

  f32x4 dw1[HT][QT], dw2[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    dw2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < QT; ++q) dw1[t][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  KahanSum db2[4];
  float surr_acc = 0.f, ent_acc = 0.f;

  // per-wave LDS: the obs tile row-major (fp32; TR: its bf16 high parts, exact for the record) and
  // the dZ transpose (row stride 20)
  constexpr int XS = 32 * KC + 4;    // fp32 row stride = 4 mod 16 floats: sample-on-k reads hit 64 banks
  constexpr int XS16 = 32 * KC + 4;  // bf16 rows of 8-byte multiples, 8 banks apart per 4 rows
  __shared__ __attribute__((aligned(16))) unsigned char xs_raw[TR ? 4 * 32 * XS16 * 2 : 4 * 32 * XS * 4];
  __shared__ __attribute__((aligned(16))) float dzt[4][2][16][20];
  // DZ1 (D2D_ACTOR_DZ_ONCE): dZ's bf16 parts [half][part h / m][sample][16 actions] in the dzt space
  constexpr bool DZ1 = TR && PAIR && D2D_ACTOR_DZ_ONCE;
  static_assert(2 * 2 * 16 * 16 * 2 <= 2 * 16 * 20 * 4, "the dZ part image fits the wave's dzt slice");
  constexpr int NV = HT * QT * 4 + HT * 4 + 4 + 2;
  // TR: relu(HT)'s split parts [wave][half][hidden tile][part][16 samples][16 hidden] bf16; the
  // cross-wave reduction buffer (used only after the tile loop) shares the space
  constexpr int TRU16 = TR ? 4 * 2 * HT * 2 * 16 * 16 : 0;
  constexpr int RAWB = TRU16 * 2 > NV * 64 * 4 ? TRU16 * 2 : NV * 64 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char tr_raw[RAWB];
  float* red = reinterpret_cast<float*>(tr_raw);
  uint16_t* trimg = reinterpret_cast<uint16_t*>(tr_raw);
  float(*xw)[XS] = reinterpret_cast<float(*)[XS]>(xs_raw + (TR ? 0 : wave * 32 * XS * 4));
  uint16_t(*xw16)[XS16] = reinterpret_cast<uint16_t(*)[XS16]>(xs_raw + (TR ? wave * 32 * XS16 * 2 : 0));
  float(*zb)[16][20] = dzt[wave];
  uint16_t* zim = reinterpret_cast<uint16_t*>(&dzt[wave][0][0][0]);  // DZ1: [s][part][16][16]

  const int stride = a.G * 4;
  const int tile0 = by * 4 + wave;
  int e0 = 0;
  ActorIn<KC, PAIR, U8> cur;  // per-sample scalars of the tile being computed
  bf16x8 xh[2][KC];
  uint32_t sm[KC][2];
  record_signs<KC, U8>(sm, a, k, g);
  // ---- inputs: bias column, zeros past it; bf16 high parts; the tile to LDS for dW1.
  // Returns whether every input of the tile is bf16-exact (wave-uniform).
  auto stage = [&](const ActorIn<KC, PAIR, U8>& src, TileCur c) -> bool {
    e0 = c.e0;
#pragma unroll
    for (int s = 0; s < (PAIR ? 1 : 2); ++s) {
      cur.act[s] = src.act[s];
      cur.lo[s] = src.lo[s];
      cur.w[s] = src.w[s];
    }
    uint32_t low = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        float xr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = 32 * c + 8 * g + j;
          // the record carries the bias input at column F and zeros past it
          xr[j] = U8 ? src.x.at(s, c, j, sm) : col < F ? src.x.at(s, c, j, sm) : col == F ? 1.f : 0.f;
          low |= fbits(xr[j]) & 0xFFFFu;
        }
        xh[s][c] = hi_frag(xr);
        if constexpr (TR) {  // the bf16 high parts (exact) as two 8-byte stores
          const u32x4v hv = __builtin_bit_cast(u32x4v, xh[s][c]);
          *reinterpret_cast<uint2*>(&xw16[16 * s + i][32 * c + 8 * g]) = make_uint2(hv[0], hv[1]);
          *reinterpret_cast<uint2*>(&xw16[16 * s + i][32 * c + 8 * g + 4]) = make_uint2(hv[2], hv[3]);
        } else {
          *reinterpret_cast<f32x4*>(&xw[16 * s + i][32 * c + 8 * g]) = f32x4{xr[0], xr[1], xr[2], xr[3]};
          *reinterpret_cast<f32x4*>(&xw[16 * s + i][32 * c + 8 * g + 4]) = f32x4{xr[4], xr[5], xr[6], xr[7]};
        }
      }
    // the record's integers in [-128, 255] are bf16-exact
    return U8 || __builtin_amdgcn_ballot_w64(low != 0) == 0;
  };

  {
    // the tile body, XE: every input bf16-exact (env observations: one MFMA per split part of
    // W1), else the residual parts of x too
    auto body = [&](auto xe) {
      constexpr bool XE = decltype(xe)::value;
      // ---- forward (transposed): HT = W1 . X^T (bf16 split), Z^T = W2 . relu(HT) + b2 (fp32)
      f32x4 zt[2];
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
        }
        if constexpr (!XE) {  // rare (fractional observations): residual parts, x re-read from LDS
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            float xv[8];
            lds_row(xv, xw, 16 * s + i, 32 * c + 8 * g);
            const Parts xp = split3(xv);
#pragma unroll
            for (int t2 = 0; t2 < HT; ++t2) {
              ht[t2] = mfma_bf16(w1p[t2][c].h, xp.l, ht[t2]);
              ht[t2] = mfma_bf16(w1p[t2][c].m, xp.m, ht[t2]);
              ht[t2] = mfma_bf16(w1p[t2][c].h, xp.m, ht[t2]);
            }
          }
        }
        f32x4 z = b2i;
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
#if !D2D_LOGITS_BF16
          const f32x4 w2f = *reinterpret_cast<const f32x4*>(&w2f_s[t2][lane][0]);
#pragma unroll
          for (int r = 0; r < 4; ++r)
#if D2D_UPD_ABLATE == 2  // timing ablation: logits without the fp32 MFMAs
            z[r] += w2f[r] * relu(ht[t2][r]);
#else
            z = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[r], relu(ht[t2][r]), z, 0, 0, 0);
#endif
#else
          {  // relu(HT) on a three-way RNE split: k-slots [h_m | h_h] against W2's [h|h], [m|m] parts and
             // [h_h | h_l] against [l|h] -- every product down to 2^-24 in 3 MFMAs (the two-way split
             // alone leaves ~2^-18 per logit, which the PPO gradient's cancellation over 10^5-10^7
             // samples amplified to ~2e-5 of max|g| at the headline batch)
            float hv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) hv[r] = relu(ht[t2][r]);
#if D2D_LOGITS_SPLIT3
            const Parts4 hp = split3rne_4(hv);
            // (part order m, h, l: the two operands can share h's registers)
            const bf16x8 bh = cat(hp.m, hp.h), bl = cat(hp.h, hp.l);
#else
            const Parts2x4 hp = split2_4(hv);
            const uint32_t z2[2] = {0u, 0u};
            const bf16x8 bh = cat(hp.m, hp.h), bl = cat(hp.h, z2);
#endif
            z = mfma_bf16(w2z_s[t2][2][lane], bl, z);
            z = mfma_bf16(w2z_s[t2][1][lane], bh, z);
            z = mfma_bf16(w2z_s[t2][0][lane], bh, z);
            if constexpr (TR) {
              // the split parts to this half's image [part][sample i][hidden 4g .. 4g + 3]
              uint16_t* im = trimg + (((wave * 2 + s) * HT + t2) * 2) * 256 + i * 16 + 4 * g;
              *reinterpret_cast<uint2*>(im) = make_uint2(hp.h[0], hp.h[1]);
              *reinterpret_cast<uint2*>(im + 256) = make_uint2(hp.m[0], hp.m[1]);
            }
          }
#endif
        }
        zt[s] = z;
      }

      // ---- epilogue -> dZ (lane (g, i): sample 16s + i, actions 4g + r), written transposed to LDS
      f32x4 dz[2];
      bf16x8 za_hm[2], za_hl[2];  // DZ1: dH's A operands of each half
      if constexpr (DZ1) {
        f32x4 zc;
#pragma unroll
        for (int r = 0; r < 4; ++r) zc[r] = uf(__builtin_amdgcn_permlane32_swap(fu(zt[0][r]), fu(zt[1][r]), false, false)[0]);
        const int e = e0 + 16 * (g >> 1) + i;
#if D2D_UPD_ABLATE == 1  // timing ablation: no epilogue (dz = z)
        const f32x4 dzc = zc;
#else
        const f32x4 dzc = ppo_dz<KIND, true, false, AFIX>(a, zc, cur.act[0], cur.lo[0], cur.w[0], e < a.E, g & 1, surr_acc, ent_acc);
#endif
#pragma unroll
        for (int r = 0; r < 4; ++r) db2[r].add(dzc[r]);
        // three RNE parts of this lane's 4 actions (half g >> 1, sample i, actions 4 (g & 1) .. + 3)
        const float dv[4] = {dzc[0], dzc[1], dzc[2], dzc[3]};
        const Parts4 zp = split3rne_4(dv);
        // dW2's operand: the h and m parts (= the two-way RNE split) as bf16 rows [half][part][sample][action]
        uint16_t* zw = zim + ((g >> 1) * 2) * 256 + i * 16 + 4 * (g & 1);
        *reinterpret_cast<uint2*>(zw) = make_uint2(zp.h[0], zp.h[1]);
        *reinterpret_cast<uint2*>(zw + 256) = make_uint2(zp.m[0], zp.m[1]);
        // each half's parts into lanes 0-31 (lanes 32-63: 0, against W2's zero k-slots of actions 8-15)
        uint32_t ph[2][2], pm[2][2], pl[2][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const auto sh = __builtin_amdgcn_permlane32_swap(zp.h[q], 0u, false, false);
          const auto sm_ = __builtin_amdgcn_permlane32_swap(zp.m[q], 0u, false, false);
          const auto sl = __builtin_amdgcn_permlane32_swap(zp.l[q], 0u, false, false);
          ph[0][q] = sh[0]; ph[1][q] = sh[1];
          pm[0][q] = sm_[0]; pm[1][q] = sm_[1];
          pl[0][q] = sl[0]; pl[1][q] = sl[1];
        }
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          // (part order l, h, m: the two operands share h's registers, as cat(zp.h, zp.m) / cat(zp.l, zp.h))
          za_hm[h2] = cat(ph[h2], pm[h2]);
          za_hl[h2] = cat(pl[h2], ph[h2]);
        }
      } else if constexpr (PAIR) {
        f32x4 zc;
#pragma unroll
        for (int r = 0; r < 4; ++r) zc[r] = uf(__builtin_amdgcn_permlane32_swap(fu(zt[0][r]), fu(zt[1][r]), false, false)[0]);
        const int e = e0 + 16 * (g >> 1) + i;
#if D2D_UPD_ABLATE == 1  // timing ablation: no epilogue (dz = z)
        const f32x4 dzc = zc;
#else
        const f32x4 dzc = ppo_dz<KIND, true, false, AFIX>(a, zc, cur.act[0], cur.lo[0], cur.w[0], e < a.E, g & 1, surr_acc, ent_acc);
#endif
#pragma unroll
        for (int r = 0; r < 4; ++r) db2[r].add(dzc[r]);
        *reinterpret_cast<f32x4*>(&zb[g >> 1][i][4 * (g & 1)]) = dzc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane32_swap(fu(dzc[r]), 0u, false, false);
          dz[0][r] = uf(sw[0]);  // lanes 0-31: half 0's dZ, lanes 32-63: 0
          dz[1][r] = uf(sw[1]);  // lanes 0-31: half 1's dZ, lanes 32-63: 0
        }
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int e = e0 + 16 * s + i;
          dz[s] = ppo_dz<KIND, false>(a, zt[s], cur.act[s], cur.lo[s], cur.w[s], e < a.E, g, surr_acc, ent_acc);
#pragma unroll
          for (int r = 0; r < 4; ++r) db2[r].add(dz[s][r]);
          *reinterpret_cast<f32x4*>(&zb[s][i][4 * g]) = dz[s];
        }
      }
      lds_order();

      // ---- per half s: HN = X . W1^T (sample on rows), dH = (dZ . W2) * [HN > 0],
      //      dW2^T += relu(HN)^T . dZ  (fp32, k = sample 16s + 4g + r of step r),
      //      dW1 += dH^T . X (k-slots: dH's 4 samples x its two RNE split parts; X sample-on-k
      //      from LDS, bf16-exact on env observations, else split too)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 bz1, bz2;
        const uint32_t zz[2] = {0u, 0u};
        if constexpr (DZ1) {
          // dZ's h / m parts of samples 4g .. 4g + 3 (this half), action i, transposed from the bf16 rows
          typedef __attribute__((address_space(3))) v4i16* lds_v4i16;
          const uint16_t* zr = zim + (s * 2) * 256 + (4 * g + (i >> 2)) * 16 + 4 * (i & 3);
          const uint2 zh = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(zr)));
          const uint2 zm = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(zr + 256)));
          const uint32_t zh2[2] = {zh.x, zh.y}, zm2[2] = {zm.x, zm.y};
          bz1 = cat(zh2, zh2);
          bz2 = cat(zm2, zz);
        } else {
          float dzn[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) dzn[r] = zb[s][4 * g + r][i];
          // dW2^T operand B: dZ (k = sample 4g + j of this half, column = action i), two-way split
          // (v_mfma_f32_16x16x4_f32 on the unsplit operands -- four chains of 4 per hidden tile -- removes
          // 120 VALU per tile but measured 13 % slower: the fp32 MFMAs' issue cost outweighs the VALU)
          const Parts2x4 zn = split2_4(dzn);
          bz1 = cat(zn.h, zn.h);
          bz2 = cat(zn.m, zz);
        }
        bf16x8 bx1[QT], bx2[QT];
#pragma unroll
        for (int q = 0; q < QT; ++q) {
          if constexpr (TR) {
            // the bf16 image holds the (exact) inputs already as operand halves: samples 4g .. 4g + 3 of
            // input column 16q + i in one transposing read (lane 4q' + p of each 16-lane group
            // addresses row 16s + 4g + q', columns 16q + 4p .. 16q + 4p + 3)
            typedef __attribute__((address_space(3))) v4i16* lds_v4i16;
            const v4i16 xt = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_v4i16)(&xw16[16 * s + 4 * g + (i >> 2)][16 * q + 4 * (i & 3)]));
            const uint2 xu = __builtin_bit_cast(uint2, xt);
            const uint32_t xh2[2] = {xu.x, xu.y};
            bx1[q] = cat(xh2, xh2);
            continue;
          }
          float xc[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) xc[r] = xw[16 * s + 4 * g + r][16 * q + i];
          if constexpr (XE) {
            const uint32_t xh2[2] = {pack_hi(xc[0], xc[1]), pack_hi(xc[2], xc[3])};
            bx1[q] = cat(xh2, xh2);  // (dH_h + dH_m) x
          } else {
            const Parts2x4 xq = split2_4(xc);
            const uint32_t z2[2] = {0u, 0u};
            bx1[q] = cat(xq.h, xq.h);  // (dH_h + dH_m) x_h
            bx2[q] = cat(xq.m, z2);    // dH_h x_m
          }
        }
        bf16x8 a_hm, a_hl;
        if constexpr (DZ1) {
          a_hm = za_hm[s];
          a_hl = za_hl[s];
        } else {
          const float dv[4] = {dz[s][0], dz[s][1], dz[s][2], dz[s][3]};
          const Parts4 zp = split3rne_4(dv);
          // (part order l, h, m: the two operands can share h's registers)
          a_hm = cat(zp.h, zp.m);
          a_hl = cat(zp.l, zp.h);
        }
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
          if constexpr (TR) {
            // relu(HT)'s split parts of hidden tile t2, transposed: lane (g, i) <- samples 4g .. 4g + 3
            // (element r) of hidden unit 16 t2 + i; lane 4q + p of each 16-lane group addresses
            // row (sample) 4g + q, columns 4p .. 4p + 3 of the [sample][hidden] image
            uint16_t* im = trimg + (((wave * 2 + s) * HT + t2) * 2) * 256 + (4 * g + (i >> 2)) * 16 + 4 * (i & 3);
            typedef __attribute__((address_space(3))) v4i16* lds_v4i16;
            const v4i16 th = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(im));
            f32x4 acc = mfma_bf16(a_hl, w2b_s[t2][0][lane], f32x4{0.f, 0.f, 0.f, 0.f});
            acc = mfma_bf16(a_hm, w2b_s[t2][1][lane], acc);
            acc = mfma_bf16(a_hm, w2b_s[t2][2][lane], acc);
            // relu' from the high part: nonzero exactly when relu(h) is (down to bf16's underflow at
            // ~1e-40, far below any pre-activation of normal-magnitude weights and inputs)
#if !D2D_DW2_PAIRED
            const v4i16 tm = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(im + 256));
            const bf16x8 h_hm = cat_tr(th, tm);
            dw2[t2] = mfma_bf16(h_hm, bz2, dw2[t2]);
            dw2[t2] = mfma_bf16(h_hm, bz1, dw2[t2]);
#endif
            bf16x8 d_hm;
            if constexpr (DZ1) {
              // split, then the mask on the packed parts: min(h-part bits, 1) is 0 / 1 per sample, and
              // x 0 / 1 keeps or zeroes a part (split2(0) = (0, 0): the same operand as masking first)
              const float av[4] = {acc[0], acc[1], acc[2], acc[3]};
              const Parts2x4 dp = split2_4(av);
              const uint2 tw = __builtin_bit_cast(uint2, th);
              const uint32_t m0 = pk_min1_u16(tw.x), m1 = pk_min1_u16(tw.y);
              const uint32_t dh2[2] = {pk_mul_lo_u16(m0, dp.h[0]), pk_mul_lo_u16(m1, dp.h[1])};
              const uint32_t dm2[2] = {pk_mul_lo_u16(m0, dp.m[0]), pk_mul_lo_u16(m1, dp.m[1])};
              d_hm = cat(dh2, dm2);
            } else {
              float dh[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) dh[r] = th[r] != 0 ? acc[r] : 0.f;
              const Parts2x4 dp = split2_4(dh);
              d_hm = cat(dp.h, dp.m);
            }
#pragma unroll
            for (int q = 0; q < QT; ++q) dw1[t2][q] = mfma_bf16(d_hm, bx1[q], dw1[t2][q]);
            continue;
          }
          f32x4 hn = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            hn = mfma_bf16(xh[s][c], w1p[t2][c].l, hn);
            hn = mfma_bf16(xh[s][c], w1p[t2][c].m, hn);
            hn = mfma_bf16(xh[s][c], w1p[t2][c].h, hn);
          }
          if constexpr (!XE) {
#pragma unroll
            for (int c = 0; c < KC; ++c) {
              float xv[8];
              lds_row(xv, xw, 16 * s + i, 32 * c + 8 * g);
              const Parts xp = split3(xv);
              hn = mfma_bf16(xp.l, w1p[t2][c].h, hn);
              hn = mfma_bf16(xp.m, w1p[t2][c].m, hn);
              hn = mfma_bf16(xp.m, w1p[t2][c].h, hn);
            }
          }
          // the 4 live k-slots of each fragment half carry a second split part: 6 terms, 3 MFMAs
          f32x4 acc = mfma_bf16(a_hl, w2b_s[t2][0][lane], f32x4{0.f, 0.f, 0.f, 0.f});
          acc = mfma_bf16(a_hm, w2b_s[t2][1][lane], acc);
          acc = mfma_bf16(a_hm, w2b_s[t2][2][lane], acc);
          float dh[4], hr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dh[r] = hn[r] > 0.f ? acc[r] : 0.f;
            hr[r] = relu(hn[r]);
          }
          // dW2^T += relu(HN)^T . dZ: (h_h + h_m) dz_h + h_h dz_m, k-slots = 4 samples x 2 parts
          const Parts2x4 hp = split2_4(hr);
          const bf16x8 h_hm = cat(hp.h, hp.m);
          dw2[t2] = mfma_bf16(h_hm, bz2, dw2[t2]);
          dw2[t2] = mfma_bf16(h_hm, bz1, dw2[t2]);
          const Parts2x4 dp = split2_4(dh);
          const bf16x8 d_hm = cat(dp.h, dp.m);
#pragma unroll
          for (int q = 0; q < QT; ++q) {
            if constexpr (!XE) dw1[t2][q] = mfma_bf16(d_hm, bx2[q], dw1[t2][q]);
#if D2D_UPD_ABLATE != 3  // timing ablation 3: no dW1 products
            dw1[t2][q] = mfma_bf16(d_hm, bx1[q], dw1[t2][q]);
#endif
          }
        }
      }
#if D2D_DW2_PAIRED
      if constexpr (TR) {
        // dW2^T += relu(H)^T . dZ for both halves: lane (g, i) k-slots = samples 4g .. 4g + 3 of half 0,
        // then the same of half 1 (relu(HT)'s parts from the transposed image, dZ from its LDS transpose)
        float d0[4], d1[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          d0[r] = zb[0][4 * g + r][i];
          d1[r] = zb[1][4 * g + r][i];
        }
        const Parts2x4 z0 = split2_4(d0), z1 = split2_4(d1);
        const bf16x8 bzh = cat(z0.h, z1.h), bzm = cat(z0.m, z1.m);
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
          typedef __attribute__((address_space(3))) v4i16* lds_v4i16;
          uint16_t* im0 = trimg + (((wave * 2 + 0) * HT + t2) * 2) * 256 + (4 * g + (i >> 2)) * 16 + 4 * (i & 3);
          uint16_t* im1 = trimg + (((wave * 2 + 1) * HT + t2) * 2) * 256 + (4 * g + (i >> 2)) * 16 + 4 * (i & 3);
          const bf16x8 ah = cat_tr(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(im0)),
                                   __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(im1)));
          const bf16x8 am = cat_tr(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(im0 + 256)),
                                   __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(im1 + 256)));
          dw2[t2] = mfma_bf16(ah, bzm, dw2[t2]);  // h_h dz_m
          dw2[t2] = mfma_bf16(am, bzh, dw2[t2]);  // h_m dz_h
          dw2[t2] = mfma_bf16(ah, bzh, dw2[t2]);  // h_h dz_h
        }
      }
#endif
    };
    // Exact tiles run the branch-free XE body as they stream by (one tile of look-ahead: the
    // next tile's loads are issued as soon as this tile is staged); a tile with fractional inputs
    // is deferred to a second pass over the wave's tiles with the general body, so neither body
    // carries the other's live ranges or branches.
    ActorIn<KC, PAIR, U8> in;
    bool deferred = false;
    const TileStride ts(a, stride);
    TileCur cur_t = tile_at(a, tile0);
    if (tile0 < a.n_tiles) load_actor_in<KC, PAIR, U8>(in, a, cur_t, k, g, i);
    while (cur_t.tile < a.n_tiles) {
      const bool x_exact = stage(in, cur_t);
      const TileCur nxt = ts.next(cur_t);
      if (nxt.tile < a.n_tiles) load_actor_in<KC, PAIR, U8>(in, a, nxt, k, g, i);
      if (x_exact)
        body(std::true_type{});
      else
        deferred = true;
      lds_order();
      cur_t = nxt;
    }
    if (deferred) {
      for (TileCur c = tile_at(a, tile0); c.tile < a.n_tiles; c = ts.next(c)) {
        load_actor_in<KC, PAIR, U8>(in, a, c, k, g, i);
        if (!stage(in, c)) body(std::false_type{});
        lds_order();
      }
    }
  }

  // ---- workgroup partial
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
    for (int r = 0; r < 4; ++r) acc[n++] = db2[r].value();
    acc[n++] = surr_acc;
    acc[n++] = ent_acc;
  }
  reduce_waves<NV>(acc, red, wave, lane);
  if (wave != 0) return;
  float* out = a.partial + ((size_t)by * a.N + k) * a.P;
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
  // db2: lane (g, i) holds action 4 ga + r summed over its samples; PAIR: ga = g & 1 and the two
  // 32-lane halves hold different samples of the same actions
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = row_sum16(acc[n++]);
    if constexpr (PAIR) v += uf(partner32(fu(v), g));
    const int act = 4 * (PAIR ? (g & 1) : g) + r;
    if (i == 0 && (!PAIR || g < 2) && act < A) out[OB2 + act] = v;
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
template <int KC, bool U8>
struct CriticIn {
  XRows<KC, U8> x;
  float R[2][4];  // returns of samples 16s + 4g + r
};

template <int KC, bool U8>
__device__ __forceinline__ void load_critic_in(CriticIn<KC, U8>& in, const UpdArgs& a, TileCur c, int k, int g, int i) {
  const int t = c.t, e0 = c.e0;
  load_rows<KC, U8>(in.x, a, t, e0, k, g, i);
  const __amdgpu_buffer_rsrc_t rw = sample_rsrc(a.weight, a.w_st, a.w_ext, t, e0, k);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int r = 0; r < 4; ++r) in.R[s][r] = ld_sample(rw, a.w_st, 16 * s + 4 * g + r);
}

template <int KC, int HT, bool U8>
__global__ __launch_bounds__(256, (KC == 1 && HT <= 4) ? D2D_UPD_WAVES : 1) void ppo_critic_grad_kernel(UpdArgs a) {
  constexpr int QT = 2 * KC;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  int k, by;
  xcd_block(k, by);  // k = agent, by = sample-chunk group
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
  KahanSum dv2[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) {
#pragma unroll
    for (int q = 0; q < QT; ++q) dv1[t][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  KahanSum dc2, loss_acc;
  constexpr int XS = 32 * KC + 4;  // row stride = 4 mod 16 floats: sample-on-k reads hit 64 banks
  __shared__ __attribute__((aligned(16))) float xs[4][32][XS];
  constexpr int NV = HT * QT * 4 + HT + 2;
  __shared__ float red[NV * 64];
  float(*xw)[XS] = xs[wave];

  const int stride = a.G * 4;
  const int tile0 = by * 4 + wave;
  int e0 = 0, tslot = 0;
  float R[2][4];
  bf16x8 xh[2][KC];
  uint32_t sm[KC][2];
  record_signs<KC, U8>(sm, a, k, g);
  auto stage = [&](const CriticIn<KC, U8>& src, TileCur c) -> bool {
    e0 = c.e0;
    tslot = c.t;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) R[s][r] = src.R[s][r];
    uint32_t low = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        float xr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = 32 * c + 8 * g + j;
          // the record carries the bias input at column F and zeros past it
          xr[j] = U8 ? src.x.at(s, c, j, sm) : col < F ? src.x.at(s, c, j, sm) : col == F ? 1.f : 0.f;
          low |= fbits(xr[j]) & 0xFFFFu;
        }
        xh[s][c] = hi_frag(xr);
        *reinterpret_cast<f32x4*>(&xw[16 * s + i][32 * c + 8 * g]) = f32x4{xr[0], xr[1], xr[2], xr[3]};
        *reinterpret_cast<f32x4*>(&xw[16 * s + i][32 * c + 8 * g + 4]) = f32x4{xr[4], xr[5], xr[6], xr[7]};
      }
    // the record's integers in [-128, 255] are bf16-exact
    return U8 || __builtin_amdgcn_ballot_w64(low != 0) == 0;
  };
  {
    // the tile body (XE: bf16-exact inputs), deferred tiles as in the actor kernel
    auto body = [&](auto xe) {
      constexpr bool XE = decltype(xe)::value;
#if D2D_CRITIC_MASK
      uint32_t mk[HT][2][2];  // relu' of HV as bf16 pairs [t2][half][r pair]
      float dvh[2][4];        // dL/dv of samples 16s + 4g + r
#endif
      // this tile's sums of dL/db2, the loss and dL/dv2, added to the running sums once per tile
      float tdc = 0.f, tls = 0.f, tv2[HT];
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) tv2[t2] = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // HV = X . V1^T (sample 16s + 4g + r on rows, hidden 16t + i on lanes)
        f32x4 hv[HT];
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            acc = mfma_bf16(xh[s][c], v1p[t2][c].l, acc);
            acc = mfma_bf16(xh[s][c], v1p[t2][c].m, acc);
            acc = mfma_bf16(xh[s][c], v1p[t2][c].h, acc);
          }
          if constexpr (!XE) {
#pragma unroll
            for (int c = 0; c < KC; ++c) {
              float xv[8];
              lds_row(xv, xw, 16 * s + i, 32 * c + 8 * g);
              const Parts xp = split3(xv);
              acc = mfma_bf16(xp.l, v1p[t2][c].h, acc);
              acc = mfma_bf16(xp.m, v1p[t2][c].m, acc);
              acc = mfma_bf16(xp.m, v1p[t2][c].h, acc);
            }
          }
          hv[t2] = acc;
        }
        // value and dL/dv = 2 (v - R) / B of samples 16s + 4g + r
        float dvs[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pv = 0.f;
#pragma unroll
          for (int t2 = 0; t2 < HT; ++t2) pv = fmaf(relu(hv[t2][r]), v2f[t2], pv);
#if D2D_UPD_ABLATE == 4  // timing ablation: no cross-lane value reduction
          const float v = pv + c2;
#else
          const float v = row_sum16(pv) + c2;
#endif
          const bool ok = e0 + 16 * s + 4 * g + r < a.E;
          if (a.vout && i == 0 && ok)  // the value of every sample (d2d_ppo_critic_grad_values)
            a.vout[(int64_t)tslot * a.v_st[0] + (int64_t)(e0 + 16 * s + 4 * g + r) * a.v_st[1] + (int64_t)k * a.v_st[2]] = v;
          // every lane of the row holds the same sample's v and R: all of them accumulate (no
          // per-lane selects) and the partial keeps lane i = 0's sums (the same values and order)
          const float d = ok ? v - R[s][r] : 0.f;
          dvs[r] = 2.f * a.scale * d;
          tls = fmaf(d, d, tls);
          tdc += dvs[r];
        }
#if D2D_CRITIC_MASK
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
          float hr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            hr[r] = relu(hv[t2][r]);
            tv2[t2] = fmaf(dvs[r], hr[r], tv2[t2]);
          }
#pragma unroll
          for (int p = 0; p < 2; ++p) mk[t2][s][p] = relu_mask_pair(hr[2 * p], hr[2 * p + 1]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) dvh[s][r] = dvs[r];
      }
      // dV1 / v2 += M^T . (dv x): k-slots of lane group g = (half s, r) <-> sample 16s + 4g + r
#pragma unroll
      for (int q = 0; q < QT; ++q) {
        float bv[8];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[4 * s + r] = dvh[s][r] * xw[16 * s + 4 * g + r][16 * q + i];
        const float b0[4] = {bv[0], bv[1], bv[2], bv[3]}, b1[4] = {bv[4], bv[5], bv[6], bv[7]};
        const Parts2x4 p0 = split2_4(b0), p1 = split2_4(b1);
        const bf16x8 bh = cat(p0.h, p1.h), bm = cat(p0.m, p1.m);
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
          const uint32_t m01[2] = {mk[t2][0][0], mk[t2][0][1]}, m23[2] = {mk[t2][1][0], mk[t2][1][1]};
          const bf16x8 am = cat(m01, m23);
          dv1[t2][q] = mfma_bf16(am, bm, dv1[t2][q]);
#if D2D_UPD_ABLATE != 5  // timing ablation 5: no dV1 products
          dv1[t2][q] = mfma_bf16(am, bh, dv1[t2][q]);
#endif
        }
      }
      (void)XE;
#else
        // X sample-on-k for this half: B fragments with the split parts paired to dHv's
        bf16x8 bx1[QT], bx2[QT];
#pragma unroll
        for (int q = 0; q < QT; ++q) {
          float xc[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) xc[r] = xw[16 * s + 4 * g + r][16 * q + i];
          if constexpr (XE) {
            const uint32_t xh2[2] = {pack_hi(xc[0], xc[1]), pack_hi(xc[2], xc[3])};
            bx1[q] = cat(xh2, xh2);
          } else {
            const Parts2x4 xq = split2_4(xc);
            const uint32_t z2[2] = {0u, 0u};
            bx1[q] = cat(xq.h, xq.h);
            bx2[q] = cat(xq.m, z2);
          }
        }
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
          float dh[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            tv2[t2] = fmaf(dvs[r], relu(hv[t2][r]), tv2[t2]);
            dh[r] = hv[t2][r] > 0.f ? dvs[r] * v2f[t2] : 0.f;
          }
          const Parts2x4 dp = split2_4(dh);
          const bf16x8 d_hm = cat(dp.h, dp.m);
#pragma unroll
          for (int q = 0; q < QT; ++q) {
            if constexpr (!XE) dv1[t2][q] = mfma_bf16(d_hm, bx2[q], dv1[t2][q]);
#if D2D_UPD_ABLATE != 5  // timing ablation 5: no dV1 products
            dv1[t2][q] = mfma_bf16(d_hm, bx1[q], dv1[t2][q]);
#endif
          }
        }
      }
#endif
      dc2.add(tdc);
      loss_acc.add(tls);
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) dv2[t2].add(tv2[t2]);
    };
    CriticIn<KC, U8> in;
    bool deferred = false;
    const TileStride ts(a, stride);
    TileCur cur_t = tile_at(a, tile0);
    if (tile0 < a.n_tiles) load_critic_in<KC, U8>(in, a, cur_t, k, g, i);
    while (cur_t.tile < a.n_tiles) {
      const bool x_exact = stage(in, cur_t);
      const TileCur nxt = ts.next(cur_t);
      if (nxt.tile < a.n_tiles) load_critic_in<KC, U8>(in, a, nxt, k, g, i);
      lds_order();
      if (x_exact)
        body(std::true_type{});
      else
        deferred = true;
      lds_order();
      cur_t = nxt;
    }
    if (deferred) {
      for (TileCur c = tile_at(a, tile0); c.tile < a.n_tiles; c = ts.next(c)) {
        load_critic_in<KC, U8>(in, a, c, k, g, i);
        const bool x_exact = stage(in, c);
        lds_order();
        if (!x_exact) body(std::false_type{});
        lds_order();
      }
    }
  }

  float acc[NV];
  {
    int n = 0;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int q = 0; q < QT; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#if D2D_CRITIC_MASK
          const int hid = 16 * t + 4 * g + r;  // accumulator row: the factored-out v2[hid]
          acc[n++] = dv1[t][q][r] * (hid < H ? a.w2[(size_t)k * H + hid] : 0.f);
#else
          acc[n++] = dv1[t][q][r];
#endif
        }
#pragma unroll
    for (int t = 0; t < HT; ++t) acc[n++] = dv2[t].value();
    acc[n++] = dc2.value();
    acc[n++] = loss_acc.value();
  }
  reduce_waves<NV>(acc, red, wave, lane);
  if (wave != 0) return;
  float* out = a.partial + ((size_t)by * a.N + k) * a.P;
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
  const float dcs = group_sum(row_sum16(i == 0 ? acc[n] : 0.f));
  const float ls = group_sum(row_sum16(i == 0 ? acc[n + 1] : 0.f));
  if (lane == 0) {
    out[OB2] = dcs;
    out[OST] = ls;
    out[OST + 1] = 0.f;
  }
}


// -------------------------------------------------- critic gradients, hidden on rows (round 5, default)
// The same Value(x) = V2 relu(V1 x + c1) + c2 and loss as ppo_critic_grad_kernel above, arranged so that the
// per-(sample, hidden) work is one relu, one fma and a u16 mask per element (the sample-on-rows kernel above:
// 11 VALU per MFMA, VALU-issue bound, profiles/pmc_mfma.json):
//   * HVT = V1 . X^T (lane (g, i): hidden 16 t + 4 g + r of sample i -- the actor's forward orientation); the
//     64 -> 1 head is a per-lane fma over the lane's 4 HT hidden units and a sum over the four lane groups (two
//     permlane swaps) instead of 16-lane row sums of every (sample, tile);
//   * dV1[h][j] = v2[h] G[h][j],  G[h][j] = sum_s M[s][h] dv_s x_s[j],  M = relu'(hv) in {0, 1}: the A operand
//     (row = hidden, k = samples) is M times the bf16 parts (dv_h, dv_m) of dv's two-way RNE split -- M . dv_h
//     is dv_h or 0, exact -- built with one v_pk_min_u16 per sample pair and one v_pk_mul_lo_u16 per part; the B
//     operand (k = samples, column = input) is x itself, bf16-exact (the record; exact fp32 tiles), read
//     sample-on-k from the tile's bf16 LDS image with ds_read_b64_tr_b16 (no product, no split per (sample,
//     input));
//   * M reaches the A layout (hidden on lanes) through LDS: relu(HVT)'s bf16 high halves (nonzero exactly when
//     relu(h) >= 2^-133, the actor's relu-mask edge) written [sample][hidden] and read back transposed;
//   * dv2[h] = sum_s dv_s relu(h_s) = sum_j V1ext[h][j] G[h][j] (relu(h_s) = M[s][h] (V1ext x_s)[h], V1ext = [V1 | c1]
//     against x_s's bias column): from the workgroup's G partial once, no per-sample work (D2D_CRITIC_DV2_G; 0
//     keeps per-sample fmas and Kahan sums for A/B).
// Precision: forward as above (exact three-way V1 split, exact x); dv on a two-way RNE split (2^-17 relative per
// term, as the sample-on-rows kernel's (dv x) split); x exact.  Fractional inputs (fp32 rows that are not
// bf16-exact: the chsel env's 1/n ACKs) take the deferred body: x's residual parts in the forward, and
// (dv_h + dv_m) x_h + dv_h x_m on x's two-way RNE split in dV1.
#ifndef D2D_CRITIC_DV2_G
#define D2D_CRITIC_DV2_G 1
#endif
template <int KC, bool U8>
struct CriticInT {
  XRows<KC, U8> x;
  float R[2];  // returns of samples i and 16 + i
};

template <int KC, bool U8>
__device__ __forceinline__ void load_critic_in_t(CriticInT<KC, U8>& in, const UpdArgs& a, TileCur c, int k, int g,
                                                 int i) {
  load_rows<KC, U8>(in.x, a, c.t, c.e0, k, g, i);
  const __amdgpu_buffer_rsrc_t rw = sample_rsrc(a.weight, a.w_st, a.w_ext, c.t, c.e0, k);
#pragma unroll
  for (int s = 0; s < 2; ++s) in.R[s] = ld_sample(rw, a.w_st, 16 * s + i);
}


#ifndef D2D_CRITIC_T_WAVES
// waves per SIMD the hidden-on-rows critic is register-budgeted for (KC = 1, H <= 64, the record).  3 (168 VGPRs)
// spills 18 registers, two scratch accesses per tile; on real rollouts 2 is faster: 0.708 / 0.712 -> 0.660 / 0.663 ms
// per 26.2 M agent-samples, alternating A/B on one box (profiles/r05/critic_waves); random inputs had favoured 3
#define D2D_CRITIC_T_WAVES 2
#endif
template <int KC, int HT, bool U8>
__global__ __launch_bounds__(256, (KC == 1 && HT <= 4) ? (U8 ? D2D_CRITIC_T_WAVES : D2D_UPD_WAVES) : 1) void ppo_critic_grad_t_kernel(UpdArgs a) {
  constexpr int QT = 2 * KC;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15;
  int k, by;
  xcd_block(k, by);  // k = agent, by = sample-chunk group
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, F = a.F;
  typedef __attribute__((address_space(3))) v4i16* lds_v4i16;

  Parts v1p[HT][KC];
  float v2r[HT][4];  // V2 of hidden 16 t + 4 g + r: the rows of this lane's HVT accumulators
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
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = 16 * t + 4 * g + r;
        v2r[t][r] = hid < H ? a.w2[(size_t)k * H + hid] : 0.f;
      }
    }
  }
  const float c2 = a.b2[k];

  f32x4 dv1[HT][QT];
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int q = 0; q < QT; ++q) dv1[t][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  KahanSum dc2, loss_acc;
#if !D2D_CRITIC_DV2_G
  KahanSum dv2k[HT][4];
#endif

  // per-wave LDS: the tile's inputs as bf16 high parts (exact on the tiles the main body runs) and, for the
  // deferred fractional tiles of fp32 rows, as fp32; relu(HVT)'s high halves [half][t2][sample][hidden]; dv's
  // two bf16 parts [part][half][sample].  The cross-wave reduction buffer (after the tile loop) aliases the
  // relu image.
  constexpr int XS = 32 * KC + 4;    // fp32 row stride = 4 mod 16 floats: sample-on-k reads hit 64 banks
  constexpr int XS16 = 32 * KC + 4;  // bf16 rows of 8-byte multiples, 8 banks apart per 4 rows
  __shared__ __attribute__((aligned(16))) uint16_t xs16[4][32][XS16];
  constexpr int X32B = U8 ? 16 : 4 * 32 * XS * 4;
  __shared__ __attribute__((aligned(16))) unsigned char xs32_raw[X32B];
  constexpr int NV = HT * QT * 4 + 2 + (D2D_CRITIC_DV2_G ? 0 : HT * 4);
  constexpr int MIMGB = 4 * 2 * HT * 256 * 2;
  constexpr int RAWB = MIMGB > NV * 64 * 4 ? MIMGB : NV * 64 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char raw[RAWB];
  __shared__ __attribute__((aligned(16))) uint16_t dvimg[4][64];
  float* red = reinterpret_cast<float*>(raw);
  uint16_t* mimg = reinterpret_cast<uint16_t*>(raw) + wave * 2 * HT * 256;
  uint16_t(*xw16)[XS16] = xs16[wave];
  float(*xw)[XS] = reinterpret_cast<float(*)[XS]>(xs32_raw + (U8 ? 0 : wave * 32 * XS * 4));
  uint16_t* dvw = dvimg[wave];

  const int stride = a.G * 4;
  const int tile0 = by * 4 + wave;
  int e0 = 0;
  float R[2];
  bf16x8 xh[2][KC];
  uint32_t sm[KC][2];
  record_signs<KC, U8>(sm, a, k, g);
  // inputs: bias column, zeros past it; bf16 high parts to registers (forward B operand) and LDS (dV1 B
  // operand); F32: the fp32 image too (the deferred pass).  Returns whether every input is bf16-exact.
  int tslot = 0;
  auto stage = [&](const CriticInT<KC, U8>& src, TileCur c, auto f32img) -> bool {
    constexpr bool F32 = decltype(f32img)::value;
    e0 = c.e0;
    tslot = c.t;
    R[0] = src.R[0];
    R[1] = src.R[1];
    uint32_t low = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int cc = 0; cc < KC; ++cc) {
        float xr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = 32 * cc + 8 * g + j;
          // the record carries the bias input at column F and zeros past it
          xr[j] = U8 ? src.x.at(s, cc, j, sm) : col < F ? src.x.at(s, cc, j, sm) : col == F ? 1.f : 0.f;
          low |= fbits(xr[j]) & 0xFFFFu;
        }
        xh[s][cc] = hi_frag(xr);
        const u32x4v hv = __builtin_bit_cast(u32x4v, xh[s][cc]);
        *reinterpret_cast<uint2*>(&xw16[16 * s + i][32 * cc + 8 * g]) = make_uint2(hv[0], hv[1]);
        *reinterpret_cast<uint2*>(&xw16[16 * s + i][32 * cc + 8 * g + 4]) = make_uint2(hv[2], hv[3]);
        if constexpr (F32 && !U8) {
          *reinterpret_cast<f32x4*>(&xw[16 * s + i][32 * cc + 8 * g]) = f32x4{xr[0], xr[1], xr[2], xr[3]};
          *reinterpret_cast<f32x4*>(&xw[16 * s + i][32 * cc + 8 * g + 4]) = f32x4{xr[4], xr[5], xr[6], xr[7]};
        }
      }
    // the record's integers in [-128, 255] are bf16-exact
    return U8 || __builtin_amdgcn_ballot_w64(low != 0) == 0;
  };
  {
    auto body = [&](auto xe) {
      constexpr bool XE = decltype(xe)::value;
      float dvv[2];  // dL/dv of samples i and 16 + i
      float tdc = 0.f, tls = 0.f;
#if !D2D_CRITIC_DV2_G
      float tv2[HT][4];
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2)
#pragma unroll
        for (int r = 0; r < 4; ++r) tv2[t2][r] = 0.f;
#endif
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // HVT = V1 . X^T (hidden 16 t2 + 4 g + r on rows, sample 16 s + i on lanes)
        // (part-outer, tile-inner: HT independent accumulation chains interleave)
        f32x4 hv[HT];
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) hv[t2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < KC; ++c) {
#pragma unroll
          for (int t2 = 0; t2 < HT; ++t2) hv[t2] = mfma_bf16(v1p[t2][c].l, xh[s][c], hv[t2]);
#pragma unroll
          for (int t2 = 0; t2 < HT; ++t2) hv[t2] = mfma_bf16(v1p[t2][c].m, xh[s][c], hv[t2]);
#pragma unroll
          for (int t2 = 0; t2 < HT; ++t2) hv[t2] = mfma_bf16(v1p[t2][c].h, xh[s][c], hv[t2]);
        }
        if constexpr (!XE) {
#pragma unroll
          for (int c = 0; c < KC; ++c) {
            float xv[8];
            lds_row(xv, xw, 16 * s + i, 32 * c + 8 * g);
            const Parts xp = split3(xv);
#pragma unroll
            for (int t2 = 0; t2 < HT; ++t2) {
              hv[t2] = mfma_bf16(v1p[t2][c].h, xp.l, hv[t2]);
              hv[t2] = mfma_bf16(v1p[t2][c].m, xp.m, hv[t2]);
              hv[t2] = mfma_bf16(v1p[t2][c].h, xp.m, hv[t2]);
            }
          }
        }
        // value of sample 16 s + i: the lane's 4 HT hidden units, then the four lane groups; relu(HVT)'s high
        // halves to the image [half s][t2][sample i][hidden 4 g .. 4 g + 3]
        // (four partial sums: the fma chain's dependent latency, not its issue, bounded the one-sum form)
        float pv4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2) {
          float hr[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            hr[r] = relu(hv[t2][r]);
            pv4[r] = fmaf(hr[r], v2r[t2][r], pv4[r]);
          }
          *reinterpret_cast<uint2*>(mimg + (s * HT + t2) * 256 + i * 16 + 4 * g) =
              make_uint2(pack_hi(hr[0], hr[1]), pack_hi(hr[2], hr[3]));
#if !D2D_CRITIC_DV2_G
#pragma unroll
          for (int r = 0; r < 4; ++r) hv[t2][r] = hr[r];
#endif
        }
        const float pv = (pv4[0] + pv4[1]) + (pv4[2] + pv4[3]);
#if D2D_UPD_ABLATE == 4  // timing ablation: no cross-lane value reduction
        const float v = pv + c2;
#else
        const float v = group_sum(pv) + c2;
#endif
        const bool ok = e0 + 16 * s + i < a.E;
        // the critic's value of every sample (iPPO's deferred rollout values, d2d_ppo_critic_grad_values)
        if (a.vout && g == 0 && ok)
          a.vout[(int64_t)tslot * a.v_st[0] + (int64_t)(e0 + 16 * s + i) * a.v_st[1] + (int64_t)k * a.v_st[2]] = v;
        // the four lane groups hold the same sample: all accumulate, the partial keeps group 0's sums
        const float d = ok ? v - R[s] : 0.f;
        dvv[s] = 2.f * a.scale * d;
        tls = fmaf(d, d, tls);
        tdc += dvv[s];
#if !D2D_CRITIC_DV2_G
#pragma unroll
        for (int t2 = 0; t2 < HT; ++t2)
#pragma unroll
          for (int r = 0; r < 4; ++r) tv2[t2][r] = fmaf(dvv[s], hv[t2][r], tv2[t2][r]);
#endif
      }
      // dv's two-way RNE split, shared through LDS: [part][half][sample] (every lane group writes the same value)
      {
        const uint32_t dh = rne2(dvv[0], dvv[1]);
        const uint32_t dm = rne2(sub_bf16_lo(dvv[0], dh), sub_bf16_hi(dvv[1], dh));
        dvw[i] = (uint16_t)dh;
        dvw[16 + i] = (uint16_t)(dh >> 16);
        dvw[32 + i] = (uint16_t)dm;
        dvw[48 + i] = (uint16_t)(dm >> 16);
      }
      lds_order();
      // A operand k-slots of lane group g: samples 4 g .. 4 g + 3 of half 0, then of half 1
      const uint2 h0 = *reinterpret_cast<const uint2*>(dvw + 4 * g), h1 = *reinterpret_cast<const uint2*>(dvw + 16 + 4 * g);
      const uint2 m0 = *reinterpret_cast<const uint2*>(dvw + 32 + 4 * g), m1 = *reinterpret_cast<const uint2*>(dvw + 48 + 4 * g);
      const uint32_t DH[4] = {h0.x, h0.y, h1.x, h1.y}, DM[4] = {m0.x, m0.y, m1.x, m1.y};
      // B operands: x sample-on-k (column 16 q + i), the same k-slot order
      bf16x8 bx[QT], bxm[QT];
#pragma unroll
      for (int q = 0; q < QT; ++q) {
        if constexpr (XE) {
          const v4i16 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(&xw16[4 * g + (i >> 2)][16 * q + 4 * (i & 3)]));
          const v4i16 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(&xw16[16 + 4 * g + (i >> 2)][16 * q + 4 * (i & 3)]));
          bx[q] = cat_tr(x0, x1);
          bxm[q] = bx[q];
        } else {
          float x0[4], x1[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            x0[r] = xw[4 * g + r][16 * q + i];
            x1[r] = xw[16 + 4 * g + r][16 * q + i];
          }
          const Parts2x4 p0 = split2_4(x0), p1 = split2_4(x1);
          bx[q] = cat(p0.h, p1.h);
          bxm[q] = cat(p0.m, p1.m);
        }
      }
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2) {
        // relu(HVT)'s high halves of hidden 16 t2 + i, samples 4 g .. 4 g + 3 of each half (lane 4 q' + p of a
        // 16-lane group addresses row 4 g + q', columns 4 p .. 4 p + 3 of the [sample][hidden] image)
        const v4i16 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(mimg + (0 * HT + t2) * 256 + (4 * g + (i >> 2)) * 16 + 4 * (i & 3)));
        const v4i16 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(mimg + (1 * HT + t2) * 256 + (4 * g + (i >> 2)) * 16 + 4 * (i & 3)));
        const uint2 w0 = __builtin_bit_cast(uint2, t0), w1 = __builtin_bit_cast(uint2, t1);
        const uint32_t W[4] = {w0.x, w0.y, w1.x, w1.y};
        uint32_t ah[4], am[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const uint32_t m01 = pk_min1_u16(W[p]);  // relu'(h) of the two samples, 0 / 1 per half
          ah[p] = pk_mul_lo_u16(m01, DH[p]);
          am[p] = pk_mul_lo_u16(m01, DM[p]);
        }
        const bf16x8 Ah = as_frag(ah), Am = as_frag(am);
        // (part-outer: the QT accumulators' chains interleave)
        if constexpr (!XE) {
#pragma unroll
          for (int q = 0; q < QT; ++q) dv1[t2][q] = mfma_bf16(Ah, bxm[q], dv1[t2][q]);  // dv_h x_m
        }
#pragma unroll
        for (int q = 0; q < QT; ++q) dv1[t2][q] = mfma_bf16(Am, bx[q], dv1[t2][q]);     // dv_m x_h
#if D2D_UPD_ABLATE != 5  // timing ablation 5: no dV1 products
#pragma unroll
        for (int q = 0; q < QT; ++q) dv1[t2][q] = mfma_bf16(Ah, bx[q], dv1[t2][q]);     // dv_h x_h
#endif
      }
      dc2.add(tdc);
      loss_acc.add(tls);
#if !D2D_CRITIC_DV2_G
#pragma unroll
      for (int t2 = 0; t2 < HT; ++t2)
#pragma unroll
        for (int r = 0; r < 4; ++r) dv2k[t2][r].add(tv2[t2][r]);
#endif
    };
    CriticInT<KC, U8> in;
    bool deferred = false;
    const TileStride ts(a, stride);
    TileCur cur_t = tile_at(a, tile0);
    if (tile0 < a.n_tiles) load_critic_in_t<KC, U8>(in, a, cur_t, k, g, i);
    while (cur_t.tile < a.n_tiles) {
      const bool x_exact = stage(in, cur_t, std::false_type{});
      const TileCur nxt = ts.next(cur_t);
      if (nxt.tile < a.n_tiles) load_critic_in_t<KC, U8>(in, a, nxt, k, g, i);
      lds_order();
      if (x_exact)
        body(std::true_type{});
      else
        deferred = true;
      lds_order();
      cur_t = nxt;
    }
    if constexpr (!U8) {
      if (deferred) {
        for (TileCur c = tile_at(a, tile0); c.tile < a.n_tiles; c = ts.next(c)) {
          load_critic_in_t<KC, U8>(in, a, c, k, g, i);
          const bool x_exact = stage(in, c, std::true_type{});
          lds_order();
          if (!x_exact) body(std::false_type{});
          lds_order();
        }
      }
    }
    (void)deferred;
  }

  float acc[NV];
  {
    int n = 0;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int q = 0; q < QT; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[n++] = dv1[t][q][r];
    acc[n++] = dc2.value();
    acc[n++] = loss_acc.value();
#if !D2D_CRITIC_DV2_G
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[n++] = dv2k[t][r].value();
#endif
  }
  __syncthreads();  // every wave is past its last read of the relu image the reduction buffer aliases
  reduce_waves<NV>(acc, red, wave, lane);
  if (wave != 0) return;
  float* out = a.partial + ((size_t)by * a.N + k) * a.P;
  const int OB1 = H * F, OW2 = OB1 + H, OB2 = OW2 + H, OST = OB2 + 1;
  const float* V1 = a.w1 + (size_t)k * H * F;
  float dv2p[HT][4];
  int n = 0;
#pragma unroll
  for (int t = 0; t < HT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) dv2p[t][r] = 0.f;
#pragma unroll
    for (int q = 0; q < QT; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = 16 * t + 4 * g + r, col = 16 * q + i;
        const float G = acc[n++];
        if (hid < H) {
          if (col < F) out[hid * F + col] = G * v2r[t][r];
          else if (col == F) out[OB1 + hid] = G * v2r[t][r];
#if D2D_CRITIC_DV2_G
          const float w = col < F ? V1[(size_t)hid * F + col] : col == F ? a.b1[(size_t)k * H + hid] : 0.f;
          dv2p[t][r] = fmaf(w, G, dv2p[t][r]);
#endif
        }
      }
  }
  const float dcs = row_sum16(acc[n]);
  const float ls = row_sum16(acc[n + 1]);
#if !D2D_CRITIC_DV2_G
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dv2p[t][r] = acc[n + 2 + 4 * t + r];
#endif
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = row_sum16(dv2p[t][r]);
      const int hid = 16 * t + 4 * g + r;
      if (i == 0 && hid < H) out[OW2 + hid] = v;
    }
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

// 1 + the largest element offset of a [T][E][N] view with these strides (-1: a negative stride)
static int64_t tensor_extent(const int64_t (&st)[3], int T, int E, int N) {
  if (st[0] < 0 || st[1] < 0 || st[2] < 0) return -1;
  if (T <= 0 || E <= 0 || N <= 0) return 0;
  return 1 + (int64_t)(T - 1) * st[0] + (int64_t)(E - 1) * st[1] + (int64_t)(N - 1) * st[2];
}

// Workgroups per agent: whole rounds of the kernel's resident workgroups (its occupancy x the CU count: a
// partial last round leaves CUs idle -- the hidden-on-rows critic at 3 workgroups per CU over a 4-per-CU grid ran
// a second round one third full), at least one tile per wave, and at most kMaxWaveTiles tiles per wave.  A wave
// sums its tiles' weight gradients in MFMA accumulators, an fp32 chain whose rounding error grows with its
// length: at the 65,536-env batch 16 workgroups per agent left 6,400 tiles per wave and dW2 at 4x torch fp32's
// error against float64 (tools/gpu/ppo_grads_full_batch.py); the G partials are summed by update_reduce_kernel
// (G x N x P floats, 0.26 GB at that batch).
#ifndef D2D_UPD_MAX_WAVE_TILES
#define D2D_UPD_MAX_WAVE_TILES 256
#endif
constexpr int64_t kMaxWaveTiles = D2D_UPD_MAX_WAVE_TILES;
#ifndef D2D_UPD_MIN_ROUNDS
// at least this many resident rounds of workgroups per launch (a small batch's waves then run fewer tiles each and the
// last round's stragglers cost less); D2D_UPD_MIN_ROUNDS in the environment overrides it (A/B, read once per process)
#define D2D_UPD_MIN_ROUNDS 1
#endif
static int upd_min_rounds() {
  static const int r = [] {
    const char* e = getenv("D2D_UPD_MIN_ROUNDS");
    const int v = e ? atoi(e) : D2D_UPD_MIN_ROUNDS;
    return v < 1 ? 1 : v > 8 ? 8 : v;
  }();
  return r;
}
static int update_blocks(int N, int64_t n_tiles, int resident) {
  const int64_t need = (int64_t)N * ((n_tiles + 4 * kMaxWaveTiles - 1) / (4 * kMaxWaveTiles));
  const int64_t rounds = std::max<int64_t>(upd_min_rounds(), (need + resident - 1) / resident);
  const int64_t G = (rounds * resident + N - 1) / N;
  // (grid.y <= 65535: past that, more tiles per wave)
  return (int)std::max<int64_t>(1, std::min<int64_t>({G, (n_tiles + 3) / 4, 65535}));
}
static int cu_count() {
  static const int n = [] {  // (a function-local static: initialised once, thread-safe)
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return std::max(1, cus);
  }();
  return n;
}
// resident 256-thread workgroups of update kernel K on the device, queried once per instantiation
template <auto K>
static int upd_resident() {
  static const int n = [] {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, K, 256, 0) != hipSuccess || per < 1) per = 2;
    return per * cu_count();
  }();
  return n;
}
// the workspace bound for any kernel's G: rounds x resident < need + resident <= need + 8 workgroups per CU
static int update_blocks_bound(int N, int64_t n_tiles) {
  const int64_t need = (int64_t)N * ((n_tiles + 4 * kMaxWaveTiles - 1) / (4 * kMaxWaveTiles));
  const int64_t G = (std::max<int64_t>(need + 8 * (int64_t)cu_count(), (int64_t)upd_min_rounds() * 8 * cu_count()) + N - 1) / N;
  return (int)std::max<int64_t>(1, std::min<int64_t>({G, (n_tiles + 3) / 4, 65535}));
}

extern "C" int64_t d2d_ppo_workspace(int32_t n_agents, int32_t T, int32_t n_envs, int32_t obs_dim, int32_t hidden,
                                     int32_t n_out) {
  if (n_agents <= 0 || T <= 0 || n_envs <= 0) return 0;
  const int64_t tiles = (int64_t)T * ((n_envs + 31) / 32);
  const int G = update_blocks_bound(n_agents, tiles);
  const int64_t P = (int64_t)hidden * obs_dim + hidden + (int64_t)n_out * hidden + n_out + 2;
  return (int64_t)G * n_agents * P;
}

static int check_update(const d2d_mlp_desc* d, int T, const void* obs, const void* grads_w1, float* workspace,
                        int64_t ws, int critic) {
  if (!d || !obs || !d->w1 || !d->b1 || !d->w2 || !d->b2 || !grads_w1 || !workspace) {
    d2d_set_error("NULL argument");
    return D2D_EINVAL;
  }
  if (T < 0 || d->n_envs < 0 || d->n_agents < 0) { d2d_set_error("negative size"); return D2D_EINVAL; }
  // hidden <= 128 with one input chunk (F + 1 <= 32: the learners' default hidden_size 128), else <= 64
  const int hmax = d->obs_dim + 1 <= 32 ? 128 : 64;
  if (d->hidden < 1 || d->hidden > hmax) {
    d2d_set_error("hidden=%d outside [1,%d] (obs_dim %d)", d->hidden, hmax, d->obs_dim);
    return D2D_EUNSUPPORTED;
  }
  if (d->obs_dim < 1 || d->obs_dim + 1 > 64) { d2d_set_error("obs_dim=%d outside [1,63]", d->obs_dim); return D2D_EUNSUPPORTED; }
  if (!critic && (d->n_out < 1 || d->n_out > 16)) { d2d_set_error("n_out=%d outside [1,16]", d->n_out); return D2D_EUNSUPPORTED; }
  if (!critic && d->kind != 0 && d->kind != 1) { d2d_set_error("kind must be 0 or 1"); return D2D_EINVAL; }
  const float* f32;
  const uint8_t* rec;
  const uint32_t* sgn;
  const int rc = obs_format_args(d->obs_format, d->obs_signed, d->obs_dim, obs, f32, rec, sgn);
  if (rc) return rc;
  const int64_t need = d2d_ppo_workspace(d->n_agents, T, d->n_envs, d->obs_dim, d->hidden, critic ? 1 : d->n_out);
  if (ws < need) { d2d_set_error("workspace %lld < %lld floats", (long long)ws, (long long)need); return D2D_EINVAL; }
  return D2D_OK;
}

static UpdArgs make_args(const d2d_mlp_desc* d, int T, const void* obs, float* workspace, int critic) {
  UpdArgs a{};
  a.T = T; a.E = d->n_envs; a.N = d->n_agents; a.F = d->obs_dim; a.H = d->hidden;
  a.A = critic ? 1 : d->n_out; a.kind = d->kind;
  a.mask_bytes = a.A <= 8 ? 1 : a.A <= 16 ? 2 : 4;
  a.tiles_per_t = (a.E + 31) / 32;
  a.n_tiles = T * a.tiles_per_t;
  a.G = 0;  // set by the launch (update_blocks with the launched kernel's residency)
  a.P = a.H * a.F + a.H + a.A * a.H + a.A + 2;
  a.inv_A = 1.f / (float)a.A;
  a.w1 = d->w1; a.b1 = d->b1; a.w2 = d->w2; a.b2 = d->b2;
  obs_format_args(d->obs_format, d->obs_signed, d->obs_dim, obs, a.obs, a.rec, a.sgn);  // checked by check_update
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

// KRES: the instantiation whose residency sizes the grid -- the record (U8) one for both input formats, so that
// fp32 rows and the record split the tiles into the same workgroup partials and sum them in the same order (their
// gradients are bitwise equal on bf16-exact inputs, tests/test_record_gpu.py)
template <auto K, auto KRES = K>
static void launch_upd(UpdArgs& a, hipStream_t s) {
  a.G = update_blocks(a.N, a.n_tiles, upd_resident<KRES>());
  hipLaunchKernelGGL(K, dim3(a.N, a.G), dim3(256), 0, s, a);
}
template <int KC, int HT, bool U8>
static void launch_actor_fmt(UpdArgs& a, hipStream_t s) {
  const bool pair = a.A <= 8;
  // the headline action count (8 channels / 8 ids) on the record: A at compile time
  // (grids sized by the record instantiation of the same kind and pairing, launch_upd)
  if (U8 && a.kind == 0 && a.A == 8) launch_upd<ppo_actor_grad_kernel<KC, HT, 0, true, U8, 8>>(a, s);
  else if (U8 && a.kind == 1 && a.A == 8) launch_upd<ppo_actor_grad_kernel<KC, HT, 1, true, U8, 8>>(a, s);
  else if (a.kind == 0 && a.A == 8)
    launch_upd<ppo_actor_grad_kernel<KC, HT, 0, true, U8>, ppo_actor_grad_kernel<KC, HT, 0, true, true, 8>>(a, s);
  else if (a.kind == 1 && a.A == 8)
    launch_upd<ppo_actor_grad_kernel<KC, HT, 1, true, U8>, ppo_actor_grad_kernel<KC, HT, 1, true, true, 8>>(a, s);
  else if (a.kind == 0 && pair) launch_upd<ppo_actor_grad_kernel<KC, HT, 0, true, U8>, ppo_actor_grad_kernel<KC, HT, 0, true, true>>(a, s);
  else if (a.kind == 0) launch_upd<ppo_actor_grad_kernel<KC, HT, 0, false, U8>, ppo_actor_grad_kernel<KC, HT, 0, false, true>>(a, s);
  else if (pair) launch_upd<ppo_actor_grad_kernel<KC, HT, 1, true, U8>, ppo_actor_grad_kernel<KC, HT, 1, true, true>>(a, s);
  else launch_upd<ppo_actor_grad_kernel<KC, HT, 1, false, U8>, ppo_actor_grad_kernel<KC, HT, 1, false, true>>(a, s);
}
template <int KC, int HT>
static void launch_actor(UpdArgs& a, hipStream_t s) {
  if (a.rec) launch_actor_fmt<KC, HT, true>(a, s);
  else launch_actor_fmt<KC, HT, false>(a, s);
}
// d2d_set_option(D2D_OPT_CRITIC_GRAD_ROWS, 1): the sample-on-rows critic kernel of rounds 2-4 (A/B)
std::atomic<int> g_critic_grad_rows{0};
template <int KC, int HT>
static void launch_critic(UpdArgs& a, hipStream_t s) {
  // H in (64, 128]: the hidden-on-rows kernel holds 340 VGPRs at one wave per SIMD and measured slower there
  // (1.69 vs 1.54 ms per 26 M agent-samples, tools/gpu/upd_ab.py); the sample-on-rows kernel keeps that shape
  if (HT > 4 || g_critic_grad_rows.load(std::memory_order_relaxed)) {
    if (a.rec) launch_upd<ppo_critic_grad_kernel<KC, HT, true>>(a, s);
    else launch_upd<ppo_critic_grad_kernel<KC, HT, false>, ppo_critic_grad_kernel<KC, HT, true>>(a, s);
    return;
  }
  if (a.rec) launch_upd<ppo_critic_grad_t_kernel<KC, HT, true>>(a, s);
  else launch_upd<ppo_critic_grad_t_kernel<KC, HT, false>, ppo_critic_grad_t_kernel<KC, HT, true>>(a, s);
}

extern "C" int d2d_ppo_actor_grad(const d2d_mlp_desc* d, int32_t T, const void* obs, const void* actions,
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
  a.lo_ext = tensor_extent(a.lo_st, a.T, a.E, a.N);
  a.w_ext = tensor_extent(a.w_st, a.T, a.E, a.N);
  if (a.lo_ext < 0 || a.w_ext < 0) { d2d_set_error("negative logp / weight strides"); return D2D_EINVAL; }
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
    if (ht <= 2) launch_actor<1, 2>(a, s); else if (ht <= 4) launch_actor<1, 4>(a, s); else launch_actor<1, 8>(a, s);
  } else {
    if (ht <= 2) launch_actor<2, 2>(a, s); else launch_actor<2, 4>(a, s);
  }
  D2D_CHECK_HIP(hipGetLastError());
  return launch_reduce(a, gw1, gb1, gw2, gb2, stats, s);
}

extern "C" int d2d_ppo_critic_grad_values(const d2d_mlp_desc* d, int32_t T, const void* obs, const float* returns,
                                          const int64_t* return_strides, float scale, float* gw1, float* gb1,
                                          float* gw2, float* gb2, float* stats, float* workspace,
                                          int64_t workspace_floats, float* values, const int64_t* values_strides,
                                          void* stream);
extern "C" int d2d_ppo_critic_grad(const d2d_mlp_desc* d, int32_t T, const void* obs, const float* returns,
                                   const int64_t* return_strides, float scale, float* gw1, float* gb1, float* gw2,
                                   float* gb2, float* stats, float* workspace, int64_t workspace_floats,
                                   void* stream) {
  return d2d_ppo_critic_grad_values(d, T, obs, returns, return_strides, scale, gw1, gb1, gw2, gb2, stats, workspace,
                                    workspace_floats, nullptr, nullptr, stream);
}

extern "C" int d2d_ppo_critic_grad_values(const d2d_mlp_desc* d, int32_t T, const void* obs, const float* returns,
                                          const int64_t* return_strides, float scale, float* gw1, float* gb1,
                                          float* gw2, float* gb2, float* stats, float* workspace,
                                          int64_t workspace_floats, float* values, const int64_t* values_strides,
                                          void* stream) {
  int rc = check_update(d, T, obs, gw1, workspace, workspace_floats, 1);
  if (rc) return rc;
  if (!returns || !return_strides || !gb1 || !gw2 || !gb2) {
    d2d_set_error("d2d_ppo_critic_grad: NULL argument");
    return D2D_EINVAL;
  }
  if (values && !values_strides) { d2d_set_error("d2d_ppo_critic_grad_values: values without strides"); return D2D_EINVAL; }
  UpdArgs a = make_args(d, T, obs, workspace, 1);
  a.weight = returns;
  for (int q = 0; q < 3; ++q) a.w_st[q] = return_strides[q];
  a.w_ext = tensor_extent(a.w_st, a.T, a.E, a.N);
  if (a.w_ext < 0) { d2d_set_error("negative return strides"); return D2D_EINVAL; }
  a.vout = values;
  if (values) {
    for (int q = 0; q < 3; ++q) a.v_st[q] = values_strides[q];
    if (tensor_extent(a.v_st, a.T, a.E, a.N) < 0) { d2d_set_error("negative value strides"); return D2D_EINVAL; }
  }
  a.scale = scale;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a.N == 0) return D2D_OK;
  if (a.n_tiles == 0) {
    D2D_CHECK_HIP(hipMemsetAsync(workspace, 0, sizeof(float) * (size_t)a.N * a.P, s));
    a.G = 1;
    return launch_reduce(a, gw1, gb1, gw2, gb2, stats, s);
  }
  const int ht = (a.H + 15) / 16;
  if (a.F + 1 <= 32) {
    if (ht <= 2) launch_critic<1, 2>(a, s); else if (ht <= 4) launch_critic<1, 4>(a, s); else launch_critic<1, 8>(a, s);
  } else {
    if (ht <= 2) launch_critic<2, 2>(a, s); else launch_critic<2, 4>(a, s);
  }
  D2D_CHECK_HIP(hipGetLastError());
  return launch_reduce(a, gw1, gb1, gw2, gb2, stats, s);
}
