// D2D-PPO's central critic on gfx950: the forward over the bf16 state operand fused with the per-sample part of
// the backward.
//
// Replaces, for every sample b of an epoch (d2d_ppo.py:62-98 Value, 208-216 the critic's MSE update):
//   pre_b = W1 x_b + b1,  v_b = w2 . relu(pre_b) + b2                  (Value.forward on state x_b)
//   d_b = v_b - R_b,  dv_b = 2 d_b / B                                    (F.mse_loss(values, returns.mean(1)))
//   dpre_b = [pre_b > 0] w2 dv_b                                           (linear2 / relu backward)
// and the sums db1 = sum_b dpre_b, dW2 = sum_b relu(pre_b) dv_b, db2 = sum_b dv_b, sum_b d_b^2.  dW1 = sum_b
// dpre_b x_b^T stays a split-K GEMM over the operand (d2d_ppo.py _dw1_gemm): dpre is written as its three-way RNE
// bf16 split, sample-major [B][3H] (the d2d_critic_dpre_split3 parts, ~2^-24 relative per product term).
//
// Before (round 4): one hipBLASLt GEMM [3H x S] . [S x B] -> fp32 [3H][B] partial products of W1's three parts, a
// sum, relu, the 64 -> 1 GEMM, then the dpre split kernel over pre: ~1.6 GB of fp32 intermediates per epoch at 256
// agents x 4,096 envs beside the 6.3 GB operand (critic_fwd 3.5 ms per epoch, profiles/r04).  Here the operand
// is read once, the intermediates stay in registers, and the kernel writes v [B] and dpre's parts [B][3H] (bf16).
//
// Mapping: a 256-thread workgroup owns 64 ST samples (each wave 16 ST: ST sample tiles of 16) and all H <= 16 HT
// hidden units.  K loop over the state in chunks of 32 features: lane (g, i) of sample tile st holds sample
// 16 st + i, features 32c + 8g .. + 7 as its B fragment (one 16-byte load, prefetched one chunk ahead); W1's exact
// three-way split (truncation parts, mlp_common.h split3: the products are exact, x is an integer) arrives as a
// per-chunk image of A fragments [t][part][lane] (built once per epoch by critic_w1_image_kernel), staged through
// a double-buffered LDS slice shared by the workgroup's four waves (one barrier per KCH chunks).  The accumulator
// (hidden 16t + 4g + r on rows, sample on lanes) is the actor kernels' forward orientation: the 64 -> 1 head is a
// per-lane fma over the lane's hidden units plus a sum over the four lane groups.
#include <algorithm>

#include "mlp_common.h"

namespace d2d {

struct CriticArgs {
  int H, S, nchunk;
  int64_t B, ldx;
  const uint16_t* xb;   // [B][ldx] bf16 (exact integer states; columns [S, ldx) zero)
  const bf16x8* w1img;  // [nchunk][HT][3][64] A fragments
  const float *b1, *w2, *b2, *ret;
  float two_over_B;
  float* values;        // [B]
  uint16_t* dhm;        // [B][3H] bf16: dpre's RNE parts h | m | l
  float* partial;       // [G][2H + 2]: db1 | dW2 | db2 | sum d^2
};

// the chunk image: chunk c, hidden tile t, part p (0 h, 1 m, 2 l), lane (g, i) <- W1[16t + i][32c + 8g .. + 7]
template <int HT>
__global__ __launch_bounds__(256) void critic_w1_image_kernel(int H, int S, int nchunk, const float* __restrict__ w1,
                                                              bf16x8* __restrict__ img) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)nchunk * HT * 64) return;
  const int lane = (int)(idx & 63), t = (int)((idx >> 6) % HT), c = (int)((idx >> 6) / HT);
  const int g = lane >> 4, i = lane & 15, hrow = 16 * t + i;
  float wv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = 32 * c + 8 * g + j;
    wv[j] = (hrow < H && col < S) ? w1[(size_t)hrow * S + col] : 0.f;
  }
  const Parts p = split3(wv);
  bf16x8* o = img + ((size_t)(c * HT + t) * 3) * 64 + lane;
  o[0] = p.h;
  o[64] = p.m;
  o[128] = p.l;
}

// RNE bf16 of a (low half) and b (high half)
__device__ __forceinline__ uint32_t rne_pk(float a, float b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const bf2 v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float bf_lo(uint32_t p) { return __uint_as_float(p << 16); }
typedef short v4i16 __attribute__((ext_vector_type(4)));
// two transposing LDS reads (four bf16 each) as one MFMA operand
__device__ __forceinline__ bf16x8 cat_tr16(v4i16 a, v4i16 b) {
  const uint2 x = __builtin_bit_cast(uint2, a), y = __builtin_bit_cast(uint2, b);
  const u32x4v v = {x.x, x.y, y.x, y.y};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ float bf_hi(uint32_t p) { return __uint_as_float(p & 0xFFFF0000u); }

#ifndef D2D_CRITIC_WAVES
// waves per workgroup (2 per SIMD either way): 8 halves the W1 image slices each sample's workgroup reads from L2
// and writes to LDS
#define D2D_CRITIC_WAVES 4
#endif
#ifndef D2D_CRITIC_XLDS
// 1: the operand through LDS in full 128-byte lines (KCH = 2, ST = 4): each load instruction brings 8 sample rows x 128 B
// (the iteration's two chunks) instead of 16 rows x 64 B, the rows are written to a per-wave XOR-swizzled image and the
// MFMA B fragments read back by ds_read_b128 (MI355X_MICROARCH / cdna_hip_programming: fragment-shaped loads cost the
// texture path twice the work of full-line ones)
#define D2D_CRITIC_XLDS 1
#endif
#ifndef D2D_CRITIC_WPD
// XL path: W1's image slices loaded 1 iteration ahead, or (2) two ahead in two register sets -- measured 4 % SLOWER
// (1.82-1.84 vs 1.75-1.76 ms per epoch at 256 agents, profiles/r05/critic_wpd: +46 VGPRs, and the slice is L2-resident)
#define D2D_CRITIC_WPD 1
#endif
#ifndef D2D_CRITIC_PD
// operand prefetch distance in iterations + 1: 3 = three register sets in rotation (two iterations in flight), 2 =
// two sets, the next iteration's chunks only (round 5 first version)
#define D2D_CRITIC_PD 3
#endif
// KCH chunks of 32 features per iteration (one barrier per iteration; the operand loads of the next iteration in
// flight behind this one's 48 KCH MFMAs per wave: at KCH = 1 the kernel read the 6.3 GB operand at ~3 TB/s)
template <int HT, int ST, int KCH>
__global__ __launch_bounds__(64 * D2D_CRITIC_WAVES, 8 / D2D_CRITIC_WAVES) void critic_fwd_kernel(CriticArgs a) {
  constexpr int WV = D2D_CRITIC_WAVES, NT = 64 * WV;  // waves / threads per workgroup
  constexpr int NI = HT * 3 * 64;  // 16-byte image entries per chunk
  // XL: the operand through the per-wave LDS image (D2D_CRITIC_XLDS): 64 rows x 8 16-byte slots per wave, slot s of row r
  // at r * 8 + (s ^ ((r >> 1) & 7)) -- conflict-free for the 8-lane row writes and the 16-lane groups of the fragment
  // reads; the workgroup's sums reuse wave 0's image after the loop (80 KB per workgroup: two per CU)
  constexpr bool XL = D2D_CRITIC_XLDS && KCH == 2 && ST == 4;
  constexpr int NRED = WV * (2 * 16 * HT + 2);
  __shared__ __attribute__((aligned(16))) bf16x8 wl[2][KCH * NI];
  __shared__ __attribute__((aligned(16))) uint4 xim[XL ? WV : 1][XL ? 64 * 8 : 1];
  __shared__ float red_s[XL ? 1 : NRED];
  static_assert(!XL || NRED * 4 <= 64 * 8 * 16, "the sums fit wave 0's image");
  float (*red)[2 * 16 * HT + 2] = reinterpret_cast<float (*)[2 * 16 * HT + 2]>(XL ? reinterpret_cast<float*>(&xim[0][0]) : red_s);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H;
  const int64_t s0 = (int64_t)blockIdx.x * (16 * ST * WV) + (int64_t)wave * (16 * ST);  // this wave's first sample
  // the wave's rows through a range-checked descriptor: rows past B read 0
  const int64_t rest = (a.B - s0) * a.ldx * 2;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.xb + (rest > 0 ? s0 * a.ldx : 0)), 0,
      rest <= 0 ? 0u : rest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)rest, 0x00020000);
  uint32_t vo[ST];
#pragma unroll
  for (int st = 0; st < ST; ++st) vo[st] = (uint32_t)(((int64_t)(16 * st + i) * a.ldx + 8 * g) * 2);
  auto load_x = [&](bf16x8 (&x)[KCH][ST], int it) {
#pragma unroll
    for (int q = 0; q < KCH; ++q)
#pragma unroll
      for (int st = 0; st < ST; ++st)
        x[q][st] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xr, vo[st] + 64u * (uint32_t)(KCH * it + q), 0, 0));
  };
  constexpr int NE = KCH * NI, NW = (NE + NT - 1) / NT;  // image entries per iteration, per thread
  bf16x8 wr[NW];
  auto load_w = [&](int it) {
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int e = tid + NT * q;
      if (NE % NT == 0 || e < NE) wr[q] = a.w1img[(size_t)it * NE + e];
    }
  };
  f32x4 acc[ST][HT];
#pragma unroll
  for (int st = 0; st < ST; ++st)
#pragma unroll
    for (int t = 0; t < HT; ++t) acc[st][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int iters = a.nchunk / KCH;  // (nchunk is padded to a multiple of KCH; the image is zero there)
  // one iteration: W1's image slice of iteration it to LDS, the next slice's and (PD) the operand chunks of iteration
  // it + PD - 1 into flight, one barrier, the MFMAs on xc
  auto body = [&](int it, const bf16x8 (&xc)[KCH][ST], bf16x8 (&xl)[KCH][ST]) {
    // buffer it & 1 was last read in iteration it - 2: every wave passed iteration it - 1's barrier since
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int e = tid + NT * q;
      if (NE % NT == 0 || e < NE) wl[it & 1][e] = wr[q];
    }
    if (it + 1 < iters) load_w(it + 1);
    if (it + D2D_CRITIC_PD - 1 < iters) load_x(xl, it + D2D_CRITIC_PD - 1);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KCH; ++q)
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        const bf16x8* w = &wl[it & 1][q * NI + (t * 3) * 64 + lane];
        const bf16x8 ah = w[0], am = w[64], al = w[128];
#pragma unroll
        for (int st = 0; st < ST; ++st) {
          acc[st][t] = mfma_bf16(al, xc[q][st], acc[st][t]);
          acc[st][t] = mfma_bf16(am, xc[q][st], acc[st][t]);
          acc[st][t] = mfma_bf16(ah, xc[q][st], acc[st][t]);
        }
      }
  };
  load_w(0);
  if constexpr (XL) {
    // lane l brings row 8j + (l >> 3), 16-byte slot l & 7 of the iteration's 128-byte segment, for j = 0..7
    uint32_t lo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) lo[j] = (uint32_t)(((int64_t)(8 * j + (lane >> 3)) * a.ldx) * 2 + 16 * (lane & 7));
    uint4 xv[8];
    auto load_xl = [&](int it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(xr, lo[j] + 128u * (uint32_t)it, 0, 0);
        xv[j] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    };
    uint4* own = &xim[XL ? wave : 0][0];
    // W1's image slices two iterations ahead in two register sets (the loop unrolled by two: no set is copied),
    // the operand one iteration ahead
    bf16x8 wr2[NW];
    auto load_w2 = [&](bf16x8 (&w)[NW], int it) {
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int e = tid + NT * q;
        if (NE % NT == 0 || e < NE) w[q] = a.w1img[(size_t)it * NE + e];
      }
    };
    auto xbody = [&](int it, bf16x8 (&wc)[NW]) {
      // buffer it & 1 was last read in iteration it - 2: every wave passed iteration it - 1's barrier since
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int e = tid + NT * q;
        if (NE % NT == 0 || e < NE) wl[it & 1][e] = wc[q];
      }
      // the wave's rows of iteration it (its own reads of the image in iteration it - 1 were issued before these
      // writes, and one wave's LDS operations complete in order)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = 8 * j + (lane >> 3);
        own[r * 8 + ((lane & 7) ^ ((r >> 1) & 7))] = xv[j];
      }
      if (it + 1 < iters) load_xl(it + 1);
      if (it + D2D_CRITIC_WPD < iters) load_w2(wc, it + D2D_CRITIC_WPD);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < KCH; ++q) {
        bf16x8 xf[ST];
#pragma unroll
        for (int st = 0; st < ST; ++st) {
          const int r = 16 * st + i;
          xf[st] = __builtin_bit_cast(bf16x8, own[r * 8 + ((4 * q + g) ^ ((r >> 1) & 7))]);
        }
#pragma unroll
        for (int t = 0; t < HT; ++t) {
          const bf16x8* w = &wl[it & 1][q * NI + (t * 3) * 64 + lane];
          const bf16x8 ah = w[0], am = w[64], al = w[128];
#pragma unroll
          for (int st = 0; st < ST; ++st) {
            acc[st][t] = mfma_bf16(al, xf[st], acc[st][t]);
            acc[st][t] = mfma_bf16(am, xf[st], acc[st][t]);
            acc[st][t] = mfma_bf16(ah, xf[st], acc[st][t]);
          }
        }
      }
    };
    load_xl(0);
#if D2D_CRITIC_WPD == 2
    if (iters > 1) load_w2(wr2, 1);
    for (int it = 0; it < iters; it += 2) {
      xbody(it, wr);
      if (it + 1 < iters) xbody(it + 1, wr2);
    }
#else
    for (int it = 0; it < iters; ++it) xbody(it, wr);
#endif
    __syncthreads();  // wave 0's image becomes the workgroup's sums below
  } else {
#if D2D_CRITIC_PD == 3
  // three operand register sets in rotation (the loop unrolled by three, so no set is copied: a copy would wait on
  // its load at the end of the iteration that issued it): each chunk's loads are in flight for two iterations
  bf16x8 x0[KCH][ST], x1[KCH][ST], x2[KCH][ST];
  load_x(x0, 0);
  if (iters > 1) load_x(x1, 1);
  for (int it = 0; it < iters; it += 3) {
    body(it, x0, x2);
    if (it + 1 < iters) body(it + 1, x1, x0);
    if (it + 2 < iters) body(it + 2, x2, x1);
  }
#else
  bf16x8 xc[KCH][ST], xn[KCH][ST];
  load_x(xc, 0);
  for (int it = 0; it < iters; ++it) {
    body(it, xc, xn);
#pragma unroll
    for (int q = 0; q < KCH; ++q)
#pragma unroll
      for (int st = 0; st < ST; ++st) xc[q][st] = xn[q][st];
  }
#endif
  }

  // ---- epilogue: bias, relu, value, dv, dpre's split; the lane's sums over its samples
  float b1r[HT][4], w2r[HT][4];
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 16 * t + 4 * g + r;
      b1r[t][r] = h < H ? a.b1[h] : 0.f;
      w2r[t][r] = h < H ? a.w2[h] : 0.f;
    }
  const float b2 = a.b2[0];
  float pdb1[HT][4], pdw2[HT][4], pdc2 = 0.f, ploss = 0.f;
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) pdb1[t][r] = pdw2[t][r] = 0.f;
  const int H3 = 3 * H;
#pragma unroll
  for (int st = 0; st < ST; ++st) {
    const int64_t b = s0 + 16 * st + i;
    const bool ok = b < a.B;
    float pre[HT][4], hr[HT][4], pv4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pre[t][r] = acc[st][t][r] + b1r[t][r];
        hr[t][r] = relu(pre[t][r]);
        pv4[r] = fmaf(hr[t][r], w2r[t][r], pv4[r]);
      }
    const float v = group_sum((pv4[0] + pv4[1]) + (pv4[2] + pv4[3])) + b2;
    const float R = ok ? a.ret[b] : 0.f;
    const float d = ok ? v - R : 0.f;
    const float dv = d * a.two_over_B;
    if (ok && g == 0) a.values[b] = v;
    pdc2 += g == 0 ? dv : 0.f;
    ploss = fmaf(g == 0 ? d : 0.f, d, ploss);
    uint16_t* row = a.dhm + (ok ? b : 0) * H3;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      float dp[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dp[r] = pre[t][r] > 0.f ? w2r[t][r] * dv : 0.f;
        pdb1[t][r] += dp[r];
        pdw2[t][r] = fmaf(hr[t][r], dv, pdw2[t][r]);
      }
      // three RNE parts (d2d_critic_dpre_split3): h = RNE(dp), m = RNE(dp - h), l = RNE(dp - h - m)
      uint32_t ph[2], pm[2], pl[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float x0 = dp[2 * q], x1 = dp[2 * q + 1];
        ph[q] = rne_pk(x0, x1);
        const float r0 = x0 - bf_lo(ph[q]), r1 = x1 - bf_hi(ph[q]);
        pm[q] = rne_pk(r0, r1);
        pl[q] = rne_pk(r0 - bf_lo(pm[q]), r1 - bf_hi(pm[q]));
      }
      const int h0 = 16 * t + 4 * g;
      if (ok && h0 < H) {  // (H is a multiple of 4 on this path: the four units of a lane are all real or none)
        *reinterpret_cast<uint2*>(row + h0) = make_uint2(ph[0], ph[1]);
        *reinterpret_cast<uint2*>(row + H + h0) = make_uint2(pm[0], pm[1]);
        *reinterpret_cast<uint2*>(row + 2 * H + h0) = make_uint2(pl[0], pl[1]);
      }
    }
  }
  // ---- the workgroup's sums: over the 16 samples of a row (lanes i), then the four waves in order
  float* rw = red[wave];
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s1 = row_sum16(pdb1[t][r]), s2 = row_sum16(pdw2[t][r]);
      if (i == 0) {
        rw[16 * t + 4 * g + r] = s1;
        rw[16 * HT + 16 * t + 4 * g + r] = s2;
      }
    }
  const float sc = group_sum(row_sum16(pdc2)), sl = group_sum(row_sum16(ploss));
  if (lane == 0) {
    rw[32 * HT] = sc;
    rw[32 * HT + 1] = sl;
  }
  __syncthreads();
  float* out = a.partial + (size_t)blockIdx.x * (2 * H + 2);
  for (int q = tid; q < 2 * H + 2; q += NT) {
    const int src = q < H ? q : q < 2 * H ? 16 * HT + (q - H) : 32 * HT + (q - 2 * H);
    float v = red[0][src];
#pragma unroll
    for (int w = 1; w < WV; ++w) v += red[w][src];
    out[q] = v;
  }
}

// ---------------------------------------------------------------------------------------------------------------
// dW1 = sum_b dpre_b x_b^T (d2d_ppo.py:440-446, value_loss.backward() into linear1.weight) on v_mfma_f32_16x16x32_bf16:
// A = dpre's three RNE parts [B][3H] (the forward's dhm, sample-major), B = the bf16 state operand xb [B][ldx]; the
// three parts accumulate into ONE accumulator (the part index is a further k-slot), so the kernel emits dW1 itself
// rather than [3H][S] partial products summed afterwards (the hipBLASLt split-K bmm of rounds 4-5).
// Both operands are sample-major and the contraction runs over samples, so every K step of 32 samples goes through
// LDS: the rows of xb's column block and of dhm are copied in (16-byte / 8-byte coalesced loads, prefetched into
// registers one step ahead, double-buffered images) and read back with ds_read_b64_tr_b16, which delivers 4 samples
// of one column per lane -- the A fragment of a hidden unit and the B fragment of a state feature.  k-slot order of
// lane group g: samples 4g .. 4g + 3, then 16 + 4g .. 16 + 4g + 3 (the same for both operands).  Image rows are
// padded by 32 bytes so that the two 16-lane groups of a 32-lane half read 8 distinct 8-bank slots (conflict-free).
// Mapping: a workgroup (4 waves) owns a column block of 64 NF features (wave w: feature tiles w NF .. w NF + NF - 1,
// every hidden tile) and a contiguous range of K steps; its fp32 partial [H][S] goes to the workspace and
// critic_dw1_reduce_kernel sums the KS partials in fixed order (deterministic, no atomics).  XCD-aware order: the
// column blocks of one K range are consecutive on one XCD, so they share its dhm rows in that XCD's L2.
constexpr int kDw1Ws = 512;  // workgroups per launch (2 per CU), a multiple of the 8 XCDs

template <int HT, int NF>
struct Dw1Cfg {
  static constexpr int WC = 4 * NF * 16;          // columns per workgroup
  static constexpr int XS = WC + 16;              // x image row stride (bf16): +32 bytes
  static constexpr int DS = 3 * 16 * HT + 16;     // dhm image row stride (bf16)
  static constexpr int XCH = 32 * WC / 8 / 256;   // 16-byte x chunks per thread per K step
};

struct Dw1Args {
  int H, S, CB, KS, steps_per;
  int64_t B, ldx;
  const uint16_t* xb;
  const uint16_t* dhm;
  float* partial;  // [KS][H][S]
};

template <int HT, int NF>
__global__ __launch_bounds__(256, 2) void critic_dw1_kernel(Dw1Args a) {
  using C = Dw1Cfg<HT, NF>;
  typedef __attribute__((address_space(3))) v4i16* lds_v4i16;
  __shared__ __attribute__((aligned(16))) uint16_t xim[2][32 * C::XS];
  __shared__ __attribute__((aligned(16))) uint16_t dim_[2][32 * C::DS];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware: workgroup id -> (xcd, local); a K range's CB column blocks run consecutively on one XCD
  const int id = blockIdx.x, per = (int)gridDim.x / 8;
  const int xcd = id % 8, local = id / 8;
  const int cb = local % a.CB, kc = xcd * (per / a.CB) + local / a.CB;
  const int H = a.H, H3 = 3 * H;
  const int64_t steps_total = (a.B + 31) / 32;
  const int64_t st0 = (int64_t)kc * a.steps_per;
  const int64_t st1 = std::min<int64_t>(st0 + a.steps_per, steps_total);
  const int nsteps = (int)std::max<int64_t>(0, st1 - st0);
  const int64_t kb = st0 * 32;  // first sample
  const int col0 = cb * C::WC;
  // range-checked descriptors from the workgroup's first sample (rows past B read 0)
  const int64_t xrest = (a.B - kb) * a.ldx * 2 - 2 * (int64_t)col0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.xb + (xrest > 0 ? kb * a.ldx + col0 : 0)), 0,
      xrest <= 0 ? 0u : xrest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)xrest, 0x00020000);
  const int64_t drest = (a.B - kb) * H3 * 2;
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.dhm + (drest > 0 ? kb * H3 : 0)), 0,
      drest <= 0 ? 0u : drest > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)drest, 0x00020000);
  // dhm's pad columns (units H .. 16 HT - 1 of each part) are never written by the copies: zero them once
  for (int e = tid; e < 2 * 32 * C::DS; e += 256) (&dim_[0][0])[e] = 0;
  // per-thread copy plan, offsets computed once: x chunk j = row rx, 16-byte column chunk cx of the block; dhm 8-byte
  // chunk q of the 32 x (3H / 4) grid of a step (part p = 4c / H, unit h), placed in its part's 16 HT-unit slot
  constexpr int CPR = C::WC / 8;       // 16-byte chunks per x row
  constexpr int NDM = 3 * HT / 2;      // 8-byte dhm chunks per thread at most (H = 16 HT)
  uint32_t xg[C::XCH], xl[C::XCH], dg[NDM], dl[NDM];
#pragma unroll
  for (int j = 0; j < C::XCH; ++j) {
    const int c = tid + 256 * j, rx = c / CPR, cx = c % CPR;
    xg[j] = (uint32_t)(((int64_t)rx * a.ldx + 8 * cx) * 2);
    xl[j] = (uint32_t)(rx * C::XS + 8 * cx);
  }
  const int DQ = H3 / 4;               // 8-byte dhm chunks per row
  const int nq = 32 * DQ;
#pragma unroll
  for (int j = 0; j < NDM; ++j) {
    const int q = min(tid + 256 * j, nq - 1);  // (threads past the grid repeat its last chunk: same value, same place)
    const int r = q / DQ, c = q - r * DQ;
    const int p = (4 * c) / H, h = 4 * c - p * H;
    dg[j] = (uint32_t)((r * H3 + 4 * c) * 2);
    dl[j] = (uint32_t)(r * C::DS + p * 16 * HT + h);
  }
  const uint32_t xstep = (uint32_t)(32 * a.ldx * 2), dstep = (uint32_t)(32 * H3 * 2);
  u32x4v xv[C::XCH];
  uint2 dv[NDM];
  auto load = [&](int step) {
    const uint32_t xb0 = (uint32_t)step * xstep, db0 = (uint32_t)step * dstep;
#pragma unroll
    for (int j = 0; j < C::XCH; ++j) xv[j] = __builtin_amdgcn_raw_buffer_load_b128(xr, xb0 + xg[j], 0, 0);
#pragma unroll
    for (int j = 0; j < NDM; ++j) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(dr, db0 + dg[j], 0, 0);
      dv[j] = make_uint2(v[0], v[1]);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < C::XCH; ++j) *reinterpret_cast<u32x4v*>(&xim[buf][xl[j]]) = xv[j];
#pragma unroll
    for (int j = 0; j < NDM; ++j) *reinterpret_cast<uint2*>(&dim_[buf][dl[j]]) = dv[j];
  };
  f32x4 acc[HT][NF];
#pragma unroll
  for (int t = 0; t < HT; ++t)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[t][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // the zeroed pads before any copy lands
  if (nsteps > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  const int ra = 4 * g + (i >> 2), ca = 4 * (i & 3);  // this lane's row / column offset of a transposing read
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) load(s + 1);
    const uint16_t* X = xim[buf];
    const uint16_t* D = dim_[buf];
    bf16x8 bx[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int col = (wave * NF + f) * 16 + ca;
      bx[f] = cat_tr16(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(&X[ra * C::XS + col])),
                       __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(&X[(16 + ra) * C::XS + col])));
    }
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int p = 2; p >= 0; --p) {  // smallest part first
        const int col = p * 16 * HT + 16 * t + ca;
        const bf16x8 ad = cat_tr16(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(&D[ra * C::DS + col])),
                                   __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16)(&D[(16 + ra) * C::DS + col])));
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[t][f] = mfma_bf16(ad, bx[f], acc[t][f]);
      }
    if (s + 1 < nsteps) store(buf ^ 1);  // buffer buf ^ 1 was last read in step s - 1, before the last barrier
    __syncthreads();
  }
  // the partial: lane (g, i) of tile (t, f) holds hidden 16 t + 4 g + r, feature col0 + (wave NF + f) 16 + i
  float* out = a.partial + (size_t)kc * H * a.S;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int sc = col0 + (wave * NF + f) * 16 + i;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = 16 * t + 4 * g + r;
        if (h < H && sc < a.S) out[(size_t)h * a.S + sc] = acc[t][f][r];
      }
  }
}

// dW1[h][s] = sum over the KS partials, in index order
__global__ __launch_bounds__(256) void critic_dw1_reduce_kernel(int64_t n, int KS, const float* __restrict__ partial,
                                                                float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  // four interleaved chains (k mod 4), combined in a fixed order: independent loads in flight, deterministic
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  int k = 0;
  for (; k + 4 <= KS; k += 4) {
    v0 += partial[(size_t)k * n + e];
    v1 += partial[(size_t)(k + 1) * n + e];
    v2 += partial[(size_t)(k + 2) * n + e];
    v3 += partial[(size_t)(k + 3) * n + e];
  }
  for (; k < KS; ++k) v0 += partial[(size_t)k * n + e];
  out[e] = (v0 + v1) + (v2 + v3);
}

}  // namespace d2d

using namespace d2d;

static int critic_ht(int H) { return H <= 32 ? 2 : H <= 64 ? 4 : H <= 128 ? 8 : 0; }
#ifndef D2D_CRITIC_ST4
// sample tiles per wave / chunks per iteration at HT = 3..4 (A/B builds; the XL path needs 4 / 2)
#define D2D_CRITIC_ST4 4
#define D2D_CRITIC_KCH4 2
#endif
static int critic_st(int ht) { return ht <= 2 ? 4 : ht <= 4 ? D2D_CRITIC_ST4 : 2; }
static int critic_kch(int ht) { return ht <= 2 ? 2 : ht <= 4 ? D2D_CRITIC_KCH4 : 1; }  // chunks per iteration (LDS: 2 x KCH x 12 HT/4 KB)
static int critic_chunks(int ht, int S) { const int k = critic_kch(ht); return ((S + 31) / 32 + k - 1) / k * k; }

extern "C" int32_t d2d_central_critic_blocks(int32_t H, int64_t B) {
  const int ht = critic_ht(H);
  if (ht == 0 || B <= 0) return 0;
  const int64_t per = 16 * D2D_CRITIC_WAVES * critic_st(ht);
  return (int32_t)((B + per - 1) / per);
}

extern "C" int64_t d2d_central_critic_image_bytes(int32_t H, int32_t S) {
  const int ht = critic_ht(H);
  if (ht == 0 || S < 1) return 0;
  return (int64_t)critic_chunks(ht, S) * ht * 3 * 64 * 16;
}

extern "C" int d2d_central_critic_fwd(int32_t H, int64_t B, int32_t S, int64_t ldx, const uint16_t* xb, const float* w1,
                                      const float* b1, const float* w2, const float* b2, const float* ret,
                                      void* w1img, float* values, uint16_t* dhm, float* partial, int32_t G,
                                      void* stream) {
  const int ht = critic_ht(H);
  if (ht == 0 || H % 4) { d2d_set_error("d2d_central_critic_fwd: hidden=%d (a multiple of 4 in [4, 128])", H); return D2D_EUNSUPPORTED; }
  if (B < 0 || S < 1 || ldx < S || (ldx & 7) || !w1 || !b1 || !w2 || !b2 || !w1img || G != d2d_central_critic_blocks(H, B) ||
      (B > 0 && (!xb || !ret || !values || !dhm || !partial)) || (reinterpret_cast<uintptr_t>(xb) & 15) ||
      (reinterpret_cast<uintptr_t>(w1img) & 15) || (reinterpret_cast<uintptr_t>(dhm) & 7)) {
    d2d_set_error("d2d_central_critic_fwd: bad arguments (ldx a multiple of 8 >= S, 16-byte aligned operand and "
                  "image, G = d2d_central_critic_blocks)");
    return D2D_EINVAL;
  }
  if (B == 0) return D2D_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  CriticArgs a{};
  a.H = H; a.S = S; a.nchunk = critic_chunks(ht, S); a.B = B; a.ldx = ldx; a.xb = xb;
  a.w1img = reinterpret_cast<const bf16x8*>(w1img);
  a.b1 = b1; a.w2 = w2; a.b2 = b2; a.ret = ret; a.two_over_B = 2.f / (float)B;
  a.values = values; a.dhm = dhm; a.partial = partial;
  const int64_t img_n = (int64_t)a.nchunk * ht * 64;
  const unsigned ig = (unsigned)((img_n + 255) / 256);
  bf16x8* img = reinterpret_cast<bf16x8*>(w1img);
  if (ht == 2) {
    hipLaunchKernelGGL(critic_w1_image_kernel<2>, dim3(ig), dim3(256), 0, s, H, S, a.nchunk, w1, img);
    hipLaunchKernelGGL((critic_fwd_kernel<2, 4, 2>), dim3(G), dim3(64 * D2D_CRITIC_WAVES), 0, s, a);
  } else if (ht == 4) {
    hipLaunchKernelGGL(critic_w1_image_kernel<4>, dim3(ig), dim3(256), 0, s, H, S, a.nchunk, w1, img);
    hipLaunchKernelGGL((critic_fwd_kernel<4, D2D_CRITIC_ST4, D2D_CRITIC_KCH4>), dim3(G), dim3(64 * D2D_CRITIC_WAVES), 0, s, a);
  } else {
    hipLaunchKernelGGL(critic_w1_image_kernel<8>, dim3(ig), dim3(256), 0, s, H, S, a.nchunk, w1, img);
    hipLaunchKernelGGL((critic_fwd_kernel<8, 2, 1>), dim3(G), dim3(64 * D2D_CRITIC_WAVES), 0, s, a);
  }
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

// ---- dW1 (ABI 14)
// feature tiles per wave: 4 (256 columns per workgroup) unless the state is narrower than 160 columns (configs[1]'s
// S = 117, the sweep's 8 agents: 128) or the hidden tiles are 8 (register budget)
static int dw1_nf(int ht, int S) { return ht <= 4 && S > 160 ? 4 : 2; }
// K ranges: a multiple of 8 (the XCD-aware mapping), kDw1Ws workgroups in all where the column blocks allow, and a
// workgroup's rows within the buffer descriptors' 2 GB offset range
static void dw1_plan(int H, int64_t B, int S, int64_t ldx, int& CB, int& KS, int& steps_per) {
  const int ht = critic_ht(H);
  const int wc = 64 * dw1_nf(ht, S);
  CB = (S + wc - 1) / wc;
  KS = std::max(8, (kDw1Ws / std::max(CB, 1)) / 8 * 8);
  const int64_t steps = (B + 31) / 32;
  for (;;) {
    steps_per = (int)std::max<int64_t>(1, (steps + KS - 1) / KS);
    if ((int64_t)steps_per * 32 * std::max<int64_t>(ldx, 3 * H) * 2 < 0x7FFFFFFF || KS >= (1 << 20)) break;
    KS *= 2;
  }
}

extern "C" int64_t d2d_central_critic_dw1_workspace(int32_t H, int64_t B, int32_t S, int64_t ldx) {
  if (critic_ht(H) == 0 || H % 4 || B < 0 || S < 1 || ldx < S) return -1;
  int CB, KS, sp;
  dw1_plan(H, B, S, ldx, CB, KS, sp);
  return (int64_t)KS * H * S;
}

extern "C" int d2d_central_critic_dw1(int32_t H, int64_t B, int32_t S, int64_t ldx, const uint16_t* xb,
                                      const uint16_t* dhm, float* workspace, int64_t workspace_floats, float* dw1,
                                      void* stream) {
  const int ht = critic_ht(H);
  if (ht == 0 || H % 4) { d2d_set_error("d2d_central_critic_dw1: hidden=%d (a multiple of 4 in [4, 128])", H); return D2D_EUNSUPPORTED; }
  if (B < 0 || S < 1 || ldx < S || (ldx & 7) || !dw1 || (B > 0 && (!xb || !dhm || !workspace)) ||
      (reinterpret_cast<uintptr_t>(xb) & 15) || (reinterpret_cast<uintptr_t>(dhm) & 7) ||
      workspace_floats < d2d_central_critic_dw1_workspace(H, B, S, ldx)) {
    d2d_set_error("d2d_central_critic_dw1: bad arguments (ldx a multiple of 8 >= S, 16-byte aligned operand, 8-byte "
                  "aligned dhm, workspace of d2d_central_critic_dw1_workspace floats)");
    return D2D_EINVAL;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (B == 0) {
    D2D_CHECK_HIP(hipMemsetAsync(dw1, 0, sizeof(float) * (size_t)H * S, s));
    return D2D_OK;
  }
  Dw1Args a{};
  dw1_plan(H, B, S, ldx, a.CB, a.KS, a.steps_per);
  a.H = H; a.S = S; a.B = B; a.ldx = ldx; a.xb = xb; a.dhm = dhm; a.partial = workspace;
  const dim3 grid((unsigned)(a.CB * a.KS));
  const int nf = dw1_nf(ht, S);
  if (ht == 2) {
    if (nf == 4) hipLaunchKernelGGL((critic_dw1_kernel<2, 4>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((critic_dw1_kernel<2, 2>), grid, dim3(256), 0, s, a);
  } else if (ht == 4) {
    if (nf == 4) hipLaunchKernelGGL((critic_dw1_kernel<4, 4>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((critic_dw1_kernel<4, 2>), grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((critic_dw1_kernel<8, 2>), grid, dim3(256), 0, s, a);
  }
  const int64_t n = (int64_t)H * S;
  hipLaunchKernelGGL(critic_dw1_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, a.KS, workspace, dw1);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}
