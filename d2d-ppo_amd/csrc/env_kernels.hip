// Env reset/step kernels for gfx950 (MI355X, CDNA4, wave64).
//
// Replaces the per-slot Python body of
//   CombinatorialEnv.reset/step    /root/reference/envs/combinatorial_env.py:61-114, 116-124, 127-242
//   ChannelSelectionEnv.reset/step /root/reference/envs/channel_selection_env.py:49-98, 104-113, 116-214
// for a batch of E independent envs.  One lane = one agent of one env:
//   * N <= 64 : an env is a power-of-two lane segment of one wavefront (64/seg
//               envs per wave); per-channel attempt counts are 64-bit wave
//               ballots masked to the segment + popcount (no LDS, no barrier).
//   * N  > 64 : one env per workgroup of ceil(N/64) waves; each wave ballots,
//               the per-channel counts are combined through LDS.
// A lane keeps its agent's whole buffer row (DW x uint32 = DW*4 slots, byte j =
// packets with j slots left) in registers: packet removal, expiry and the
// shift are byte ops (ctz, funnel shift), arrivals are one byte insert.
// obs/state rows are staged in LDS and written back as contiguous float4
// streams, so every HBM write is a full-line coalesced store.
// Randomness: recorded draws (replay, parity) or Philox4x32-10 (production).
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "policy_split.h"

namespace d2d {

constexpr int kBlock = 256;
// comb_kernel register budget and the lane count of a record-only step (no LDS staging): 7 waves
// per SIMD (<= 72 VGPRs, no spills; unhinted the allocator takes 91 and runs 5) in 256-lane blocks
// (512-lane blocks would fit only 3 per SIMD pair of waves): record step 68.5 -> 64.9 us at
// 64 x 8 x 65,536; 8 waves spill (76 us).  Ablation builds override both
// (tools/gpu/build_ablate_env.sh).
#ifndef D2D_COMB_WAVES_PER_EU
#define D2D_COMB_WAVES_PER_EU 7
#endif
#ifndef D2D_COMB_REC_BLOCK
#define D2D_COMB_REC_BLOCK 256
#endif
constexpr int kMaxAgents = 1024;

struct EnvArgs {
  int E, N, C, D, F, S, state_stride, seg, reset, cnt_words;
  uint32_t flags;  // bit 0: non-temporal (streaming) stores for the obs/state flush
  uint32_t rng_step;
  uint64_t env_base, seed;
  const d2d_agent_entry* agents;
  const uint64_t* flip_thr;
  const uint32_t* pois_cdf;  // [N][256] inverse-CDF thresholds of the Poisson arrival draw
  uint32_t* buf;
  void* chan;
  uint32_t* recv;
  uint32_t* disc;
  uint32_t* selq;
  uint32_t* seln;
  const void* actions;
  const void* flips;
  const uint8_t* arrivals;
  float* obs;
  uint8_t* rec;   // comb: compact obs record [E][N][rec_bytes] (D2D_RECORD_BYTES(F))
  int rec_bytes;
  float* state;
  uint16_t* state_b;       // comb: bf16 state rows (d2d_env_out.state_bf16), row e at state_b + e * state_b_ld
  int64_t state_b_ld;
  int32_t* reward;
  void* ack;
  uint8_t* success;
  const int32_t* gather;  // single: [N*F + S] obs/state gather codes
  const uint32_t* rng_off;  // optional device word added to rng_step (graph replays)
  uint64_t draw[kMaxAgents / 64];
};

// ------------------------------------------------------------ buffer row ops
template <int DW>
struct Row {
  uint32_t w[DW];
};

template <int DW>
__device__ __forceinline__ void load_row(Row<DW>& r, const uint32_t* p) {
  if constexpr (DW == 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
  } else if constexpr (DW == 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    r.w[0] = v.x; r.w[1] = v.y;
  } else if constexpr (DW == 8) {
    const uint4 v0 = reinterpret_cast<const uint4*>(p)[0];
    const uint4 v1 = reinterpret_cast<const uint4*>(p)[1];
    r.w[0] = v0.x; r.w[1] = v0.y; r.w[2] = v0.z; r.w[3] = v0.w;
    r.w[4] = v1.x; r.w[5] = v1.y; r.w[6] = v1.z; r.w[7] = v1.w;
  } else {
#pragma unroll
    for (int i = 0; i < DW; ++i) r.w[i] = p[i];
  }
}

template <int DW>
__device__ __forceinline__ void store_row(const Row<DW>& r, uint32_t* p) {
  if constexpr (DW == 4) {
    *reinterpret_cast<uint4*>(p) = make_uint4(r.w[0], r.w[1], r.w[2], r.w[3]);
  } else if constexpr (DW == 2) {
    *reinterpret_cast<uint2*>(p) = make_uint2(r.w[0], r.w[1]);
  } else if constexpr (DW == 8) {
    reinterpret_cast<uint4*>(p)[0] = make_uint4(r.w[0], r.w[1], r.w[2], r.w[3]);
    reinterpret_cast<uint4*>(p)[1] = make_uint4(r.w[4], r.w[5], r.w[6], r.w[7]);
  } else {
#pragma unroll
    for (int i = 0; i < DW; ++i) p[i] = r.w[i];
  }
}

template <int DW>
__device__ __forceinline__ bool row_any(const Row<DW>& r) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < DW; ++i) o |= r.w[i];
  return o != 0;
}

// next_buffers[u, col.min()] -= 1   (combinatorial_env.py:169-170)
template <int DW>
__device__ __forceinline__ void row_remove_first(Row<DW>& r) {
  bool done = false;
#pragma unroll
  for (int i = 0; i < DW; ++i) {
    const uint32_t v = r.w[i];
    if (!done && v) {
      const uint32_t sh = (uint32_t)__builtin_ctz(v) & ~7u;
      r.w[i] = v - (1u << sh);
      done = true;
    }
  }
}

// evolve_buffer: expired = B[:,0]; B = shift_left(B)  (combinatorial_env.py:120-124)
template <int DW>
__device__ __forceinline__ uint32_t row_expire_shift(Row<DW>& r) {
  const uint32_t expired = r.w[0] & 0xFFu;
#pragma unroll
  for (int i = 0; i < DW; ++i) {
    const uint32_t hi = (i + 1 < DW) ? r.w[i + 1] : 0u;
    r.w[i] = __builtin_amdgcn_alignbyte(hi, r.w[i], 1);
  }
  return expired;
}

// next_buffers[i, d_i - 1] = arrival  (the cell is 0 after the shift)
template <int DW>
__device__ __forceinline__ void row_set(Row<DW>& r, int col, uint32_t v) {
  // branch-free select per word: an `if` here gets sunk into a dynamically
  // indexed store, which spills the row to scratch
  const uint32_t ins = (v & 0xFFu) << ((col & 3) * 8);
  const int wi = col >> 2;
#pragma unroll
  for (int i = 0; i < DW; ++i) r.w[i] |= (wi == i) ? ins : 0u;
}

template <int DW>
__device__ __forceinline__ float row_byte(const Row<DW>& r, int j) {
  return (float)((r.w[j >> 2] >> ((j & 3) * 8)) & 0xFFu);
}

// Philox step of this launch: the call's rng_step plus the optional device offset (one scalar load)
__device__ __forceinline__ uint32_t rng_of(const EnvArgs& a) { return a.rng_step + (a.rng_off ? *a.rng_off : 0u); }

// ------------------------------------------------------------------ draws
__device__ __forceinline__ bool draws_now(const EnvArgs& a, int k) {
  return (a.draw[k >> 6] >> (k & 63)) & 1ull;
}

__device__ __forceinline__ uint32_t arrival_value(const EnvArgs& a, const d2d_agent_entry& ag, size_t row, int k,
                                                  uint64_t genv) {
  if (a.arrivals) return a.arrivals[row];
  const u32x4 r = philox((uint32_t)genv, (uint32_t)k, rng_of(a), kStreamArrival << 24, a.seed);
  if (ag.arrival_kind == D2D_ARRIVAL_POISSON) return poisson_lookup(r.x, a.pois_cdf + (size_t)k * 256);
  return (uint64_t)r.x < ag.arrival_thr ? 1u : 0u;
}

// one 16-byte record word, streaming (non-temporal) when nt (D2D_OPT_NT_STORES): the record is written once
// and read by the next slot's consumers only, so it need not displace the env state from L2 / MALL
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_rec(uint4* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d, bool nt) {
  const v4u32 v = {a, b, c, d};
  if (nt)
    __builtin_nontemporal_store(v, reinterpret_cast<v4u32*>(p));
  else
    *reinterpret_cast<v4u32*>(p) = v;
}

// ------------------------------------------------------ LDS -> HBM flushing
// Copy `count` floats from LDS to a contiguous global range with float4 stores
// when both ends allow it (every obs/state row group of a block is contiguous).
template <typename T>
__device__ __forceinline__ void st_stream(T* p, const T& v, bool nt) {
  if (nt)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

__device__ __forceinline__ void flush_contig(float* __restrict__ dst, const float* src, int count, bool nt) {
  const bool vec = ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) && ((count & 3) == 0);
  if (vec) {
    float4* d4 = reinterpret_cast<float4*>(dst);
    const float4* s4 = reinterpret_cast<const float4*>(src);
    for (int i = threadIdx.x; i < (count >> 2); i += blockDim.x) {
      const float4 v = s4[i];
      if (nt) {
        __builtin_nontemporal_store(v.x, &d4[i].x);
        __builtin_nontemporal_store(v.y, &d4[i].y);
        __builtin_nontemporal_store(v.z, &d4[i].z);
        __builtin_nontemporal_store(v.w, &d4[i].w);
      } else {
        d4[i] = v;
      }
    }
  } else {
    for (int i = threadIdx.x; i < count; i += blockDim.x) st_stream(dst + i, src[i], nt);
  }
}

__device__ __forceinline__ void flush_rows(float* __restrict__ dst, int stride, const float* src, int rows, int S,
                                           bool nt) {
  if ((S & 3) == 0 && (stride & 3) == 0 && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
    const int q = S >> 2;
    for (int i = threadIdx.x; i < rows * q; i += blockDim.x) {
      const int r = i / q, j = i - r * q;
      float4* d4 = reinterpret_cast<float4*>(dst + (size_t)r * stride) + j;
      const float4 v = reinterpret_cast<const float4*>(src + r * S)[j];
      if (nt) {
        __builtin_nontemporal_store(v.x, &d4->x);
        __builtin_nontemporal_store(v.y, &d4->y);
        __builtin_nontemporal_store(v.z, &d4->z);
        __builtin_nontemporal_store(v.w, &d4->w);
      } else {
        *d4 = v;
      }
    }
  } else {
    for (int i = threadIdx.x; i < rows * S; i += blockDim.x) {
      const int r = i / S, j = i - r * S;
      st_stream(dst + (size_t)r * stride + j, src[r * S + j], nt);
    }
  }
}

// ---------------------------------------------------- geometry of a lane
struct Lane {
  int env, k, local_env, envs_per_block, lane;
  bool active;
  uint64_t segmask;
};

template <bool LARGE>
__device__ __forceinline__ Lane lane_geometry(const EnvArgs& a, int bidx = blockIdx.x) {
  Lane L;
  L.lane = threadIdx.x & (kWave - 1);
  if (LARGE) {
    L.env = bidx;
    L.k = threadIdx.x;
    L.local_env = 0;
    L.envs_per_block = 1;
    L.segmask = ~0ull;
  } else {
    L.local_env = threadIdx.x / a.seg;
    L.k = threadIdx.x - L.local_env * a.seg;
    L.envs_per_block = blockDim.x / a.seg;
    L.env = bidx * L.envs_per_block + L.local_env;
    const int seg_base = L.lane & ~(a.seg - 1);
    L.segmask = (a.seg == kWave) ? ~0ull : (((1ull << a.seg) - 1ull) << seg_base);
  }
  L.active = (L.k < a.N) && (L.env < a.E);
  return L;
}

// Sum of `v` over the lanes of this lane's env (segment ballot or LDS).
template <bool LARGE>
__device__ __forceinline__ int env_count(bool v, const Lane& L, int* lds_acc) {
  const int part = __popcll(__ballot(v) & L.segmask);
  if (!LARGE) return part;
  if (L.lane == 0) atomicAdd(lds_acc, part);
  __syncthreads();
  const int tot = *lds_acc;
  return tot;
}

// Wave-local LDS hand-off: every lane's LDS writes are complete (lgkmcnt(0)) before
// any lane of the same wave reads them; no workgroup barrier needed.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Copy `count` floats of this wave's LDS slot to a contiguous global range.
__device__ __forceinline__ void wave_flush(float* __restrict__ dst, const float* src, int count, bool nt) {
  const int lane = threadIdx.x & (kWave - 1);
  if (((reinterpret_cast<uintptr_t>(dst) & 15) == 0) && ((reinterpret_cast<uintptr_t>(src) & 15) == 0) &&
      ((count & 3) == 0)) {
    float4* d4 = reinterpret_cast<float4*>(dst);
    const float4* s4 = reinterpret_cast<const float4*>(src);
    for (int i = lane; i < (count >> 2); i += kWave) {
      const float4 v = s4[i];
      if (nt) {
        __builtin_nontemporal_store(v.x, &d4[i].x);
        __builtin_nontemporal_store(v.y, &d4[i].y);
        __builtin_nontemporal_store(v.z, &d4[i].z);
        __builtin_nontemporal_store(v.w, &d4[i].w);
      } else {
        d4[i] = v;
      }
    }
  } else {
    for (int i = lane; i < count; i += kWave) st_stream(dst + i, src[i], nt);
  }
}

// The same rows as bf16 (state values are integers in [-1, 255]: the fp32 -> bf16 truncation is exact), S8 =
// S rounded up to 8 columns, the pad zero: one 16-byte store per 8 columns.  lanes / stride: the lanes that
// share the row (a wave, or the whole block for one LARGE env)
__device__ __forceinline__ void flush_bf16(uint16_t* __restrict__ dst, const float* src, int S, int first, int stride,
                                           bool nt) {
  const int q8 = (S + 7) >> 3;
  for (int q = first; q < q8; q += stride) {
    uint32_t w[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int j = 8 * q + 2 * p;
      const uint32_t lo = j < S ? __float_as_uint(src[j]) >> 16 : 0u;
      const uint32_t hi = j + 1 < S ? __float_as_uint(src[j + 1]) & 0xFFFF0000u : 0u;
      w[p] = lo | hi;
    }
    st_rec(reinterpret_cast<uint4*>(dst) + q, w[0], w[1], w[2], w[3], nt);
  }
}

// =====================================================================
// Combinatorial env: action = binary N x C matrix, per-(agent, channel)
// Markov channel, ACK vector in {-1, 0, 1}.
//   CT    : compile-time channel count (0 = runtime a.C)
//   RESET : reset instead of step (combinatorial_env.py:61-114)
// LDS: [cnt_words][per-wave obs slots: 64*F floats each][state]
//   N <= 64 : state staged per wave (the wave's envs), flushed by the wave;
//   N  > 64 : state of the block's single env staged per block.
// =====================================================================
// The step of the envs of one (virtual) workgroup index bidx: comb_kernel runs it once per workgroup
// (bidx = blockIdx.x); the fused env + policy slot (comb_policy_fused_kernel) runs it for the consecutive
// env groups of its slice and passes lrec, an LDS image of the slice's records (agent k's row of env e at
// lrec[k * lstride + 2 (e - lenv0)], two 16-byte words) that the slot's policy then reads instead of HBM.
template <typename MaskT, int DW, bool LARGE, int CT, bool RESET>
__device__ __forceinline__ void comb_step(const EnvArgs a, float* lds, int bidx, uint4* lrec, int lstride, int lenv0) {
  const Lane L = lane_geometry<LARGE>(a, bidx);
  const int N = a.N, F = a.F;
  const int C = CT ? CT : a.C;
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  int* cnt = reinterpret_cast<int*>(lds);  // LARGE: n[32], g[32]; reward at [64]
  const int slot = (kWave * F + 3) & ~3;
  float* lds_obs = lds + a.cnt_words + wave * slot;
  const int epw = LARGE ? 1 : kWave / a.seg;  // envs per wave
  float* lds_state = LARGE ? lds + a.cnt_words + nwaves * slot
                           : lds + a.cnt_words + nwaves * slot + wave * ((epw * a.S + 3) & ~3);
  const size_t row = (size_t)L.env * N + L.k;
  const uint64_t genv = a.env_base + (uint64_t)L.env;
  const uint32_t cmask = (C >= 32) ? 0xFFFFFFFFu : ((1u << C) - 1u);

  Row<DW> b;
#pragma unroll
  for (int i = 0; i < DW; ++i) b.w[i] = 0;
  uint32_t h_pre = cmask, act = 0, rc = 0, dc = 0;
  d2d_agent_entry ag{};
  if (L.active) {
    ag = a.agents[L.k];
    if (!RESET) {
      load_row<DW>(b, a.buf + row * DW);
      h_pre = (uint32_t)reinterpret_cast<const MaskT*>(a.chan)[row] & cmask;
      act = (uint32_t)reinterpret_cast<const MaskT*>(a.actions)[row] & cmask;
      rc = a.recv[row];
      dc = a.disc[row];
    }
  }
  if (LARGE) {
    if (threadIdx.x < 80) cnt[threadIdx.x] = 0;
    __syncthreads();
  }

  uint32_t ack_one = cmask, ack_zero = 0, h_new = h_pre;
  bool succ = false;
  int nsucc = 0;
  if (!RESET) {
    ack_one = 0;
    // attempts = actions * has_a_packet; attempts_good_channels = attempts * channel_state (135-138)
    const uint32_t att = row_any<DW>(b) ? act : 0u;
    const uint32_t good = att & h_pre;
    // n_users_per_channel, good-attempt count, acknack (148, 155-157): two ballots per channel
    auto count_channel = [&](int c) {
      const uint64_t m = __ballot((att >> c) & 1u) & L.segmask;
      const uint64_t g = __ballot((good >> c) & 1u) & L.segmask;
      if (!LARGE) {
        const int n = __popcll(m);
        ack_zero |= (uint32_t)(n == 0) << c;
        ack_one |= (uint32_t)(n == 1 && g != 0) << c;
      } else if (L.lane == 0) {
        atomicAdd(&cnt[c], __popcll(m));
        atomicAdd(&cnt[32 + c], __popcll(g));
      }
    };
    if constexpr (CT != 0) {
#pragma unroll
      for (int c = 0; c < CT; ++c) count_channel(c);
    } else {
      for (int c = 0; c < C; ++c) count_channel(c);
    }
    if (LARGE) {
      __syncthreads();
      for (int c = 0; c < C; ++c) {
        const int n = cnt[c];
        ack_zero |= (uint32_t)(n == 0) << c;
        ack_one |= (uint32_t)(n == 1 && cnt[32 + c] == 1) << c;
      }
    }
    // successful_attempts = (acknack * attempts_good) == 1; one packet per user (160-170)
    succ = L.active && ((good & ack_one) != 0);
    nsucc = env_count<LARGE>(succ, L, cnt + 64);
    if (succ) row_remove_first<DW>(b);
    dc += row_expire_shift<DW>(b);  // discarded_packets += expired (173-174)
    // evolve_channel: channel_state = |channel_state - Bernoulli(channel_switch)| (116-118, 175)
    uint32_t f = 0;
    if (L.active) {
      if (a.flips) {
        f = (uint32_t)reinterpret_cast<const MaskT*>(a.flips)[row];
      } else {
        const uint64_t* thr = a.flip_thr + (size_t)L.k * C;
        auto flip_block = [&](int blk) {
          const u32x4 r = philox((uint32_t)genv, (uint32_t)L.k, rng_of(a), (kStreamFlip << 24) | (uint32_t)blk, a.seed);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = blk * 4 + i;
            if (c < C) f |= (uint32_t)((uint64_t)pick(r, i) < thr[c]) << c;
          }
        };
        if constexpr (CT != 0) {
#pragma unroll
          for (int blk = 0; blk < (CT + 3) / 4; ++blk) flip_block(blk);
        } else {
          for (int blk = 0; blk * 4 < C; ++blk) flip_block(blk);
        }
      }
    }
    h_new = (h_pre ^ f) & cmask;
  }
  // arrivals (reset 66-85, step 178-196); N <= 64 keeps the draw mask in one word
  const bool drew = L.active && (LARGE ? draws_now(a, L.k) : ((a.draw[0] >> L.k) & 1ull));
  if (drew) {
    const uint32_t x = arrival_value(a, ag, row, L.k, genv);
    row_set<DW>(b, (int)ag.deadline - 1, x);
    rc = (RESET ? 0u : rc) + x;
  } else if (RESET) {
    rc = 0;
  }
  if (RESET) dc = 0;
  // ---- state update
  if (L.active) {
    store_row<DW>(b, a.buf + row * DW);
    reinterpret_cast<MaskT*>(a.chan)[row] = (MaskT)h_new;
    a.recv[row] = rc;
    a.disc[row] = dc;
    if (!RESET) {
      if (a.success) a.success[row] = succ ? 1 : 0;
      if (L.k == 0) {
        if (a.reward) a.reward[L.env] = nsucc;  // rewards = len(successful_users) (211)
        if (a.ack) {
          int8_t* ak = reinterpret_cast<int8_t*>(a.ack) + (size_t)L.env * C;
          for (int c = 0; c < C; ++c) ak[c] = ((ack_one >> c) & 1) ? 1 : (((ack_zero >> c) & 1) ? 0 : -1);
        }
      }
    }
  }
  // reset obs/state carry ones(C) in the channel and feedback slots (108-112)
  // ---- obs_k = [B'[k,:w_k], channel_obs[k] (pre-evolve), acknack] (199-206)
  const int wave_env0 = LARGE ? bidx : (bidx * L.envs_per_block + wave * epw);
  const int wave_nenv = LARGE ? 1 : max(0, min(epw, a.E - wave_env0));
  if (a.obs) {
    if (L.active) {
      const int lrow = LARGE ? (L.k - wave * kWave) : ((L.local_env - wave * epw) * N + L.k);
      float* o = lds_obs + lrow * F;
      const int w = ag.obs_width;
#pragma unroll
      for (int j = 0; j < DW * 4; ++j)
        if (j < w) o[j] = row_byte<DW>(b, j);
      auto obs_channel = [&](int c) {
        o[w + c] = (float)((h_pre >> c) & 1u);
        o[w + C + c] = ((ack_one >> c) & 1u) ? 1.f : (((ack_zero >> c) & 1u) ? 0.f : -1.f);
      };
      if constexpr (CT != 0) {
#pragma unroll
        for (int c = 0; c < CT; ++c) obs_channel(c);
      } else {
        for (int c = 0; c < C; ++c) obs_channel(c);
      }
      for (int j = w + 2 * C; j < F; ++j) o[j] = 0.f;
    }
    wave_lds_sync();
    if (LARGE) {
      const int k0 = wave * kWave;
      const int nrows = max(0, min(kWave, N - k0));
      if (nrows > 0) wave_flush(a.obs + ((size_t)bidx * N + k0) * F, lds_obs, nrows * F, a.flags & 1u);
    } else if (wave_nenv > 0) {
      wave_flush(a.obs + (size_t)wave_env0 * N * F, lds_obs, wave_nenv * N * F, a.flags & 1u);
    }
  }
  // ---- the same row as the compact record: one byte per obs column (packet counts and channel
  // bits unsigned, acks int8), zero-padded to rec_bytes.  Built in registers (the column of a byte
  // is fixed by the unrolled position; w_k, C are wave-uniform) and stored by each lane as whole
  // 16-byte words: the rows of a wave's agents are contiguous, so the stores coalesce fully.
  if (a.rec && L.active) {
    const int w = ag.obs_width;
    const uint32_t ack_neg = ~(ack_one | ack_zero) & cmask;
    // byte value of obs column p >= w (channel bits, acks, padding; column F: the constant 1 the
    // network kernels take as their layer-1 bias input)
    auto tail_byte = [&](int p) -> uint32_t {
      const int m = p - w;
      if (m < C) return (h_pre >> m) & 1u;
      const int c = m - C;
      if (c < C) return ((ack_one >> c) & 1u) | (((ack_neg >> c) & 1u) * 0xFFu);
      return p == F ? 1u : 0u;
    };
    uint4* dst = reinterpret_cast<uint4*>(a.rec + row * (size_t)a.rec_bytes);
    uint32_t v[8];
    bool built = false;
    if constexpr (CT != 0 && 2 * CT <= 16 && 4 * DW <= 16) {
      if (a.rec_bytes == 32) {  // wave-uniform: the whole row (F <= 31) in one 32-byte record
        // word-level build: the buffer words as they are (their bytes >= w_k are zero), the channel
        // bits and ack codes expanded 4 bits -> 4 bytes by one multiply (bit k of a nibble lands on
        // bit 8k of n * 0x204081, the other copies are masked off), the 2C-byte block funnel-shifted
        // to byte w_k, and the bias byte at column F
        constexpr int NB = CT / 2;  // block words: CT/4 channel words, CT/4 ack words
        auto expand4 = [](uint32_t n) { return (n * 0x204081u) & 0x01010101u; };
        uint32_t blk[NB];
#pragma unroll
        for (int u = 0; u < CT / 4; ++u) {
          blk[u] = expand4((h_pre >> (4 * u)) & 0xFu);
          blk[CT / 4 + u] = expand4((ack_one >> (4 * u)) & 0xFu) | expand4((ack_neg >> (4 * u)) & 0xFu) * 0xFFu;
        }
        const int ws = w >> 2, bs = w & 3;
        uint32_t sh[NB + 1];  // the block shifted up by bs bytes
#pragma unroll
        for (int j = 0; j <= NB; ++j) {
          const uint32_t hi = j < NB ? blk[j] : 0u, lo = j > 0 ? blk[j - 1] : 0u;
          sh[j] = bs == 0 ? hi : __builtin_amdgcn_alignbyte(hi, lo, 4 - bs);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          uint32_t word = q < DW ? b.w[q < DW ? q : 0] : 0u;
#pragma unroll
          for (int c = 0; c <= 16 / 4; ++c)  // w_k <= 4 DW <= 16: word shift 0 .. 4
            if (q - c >= 0 && q - c <= NB) word |= ws == c ? sh[q - c] : 0u;
          word |= (q == (F >> 2)) ? (1u << (8 * (F & 3))) : 0u;
          v[q] = word;
        }
        const bool nt = a.flags & 1u;
        st_rec(dst, v[0], v[1], v[2], v[3], nt);
        st_rec(dst + 1, v[4], v[5], v[6], v[7], nt);
        if (lrec) {
          uint4* l = lrec + (size_t)L.k * lstride + 2 * (L.env - lenv0);
          l[0] = make_uint4(v[0], v[1], v[2], v[3]);
          l[1] = make_uint4(v[4], v[5], v[6], v[7]);
        }
        built = true;
      }
    }
    if (!built) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = 4 * q + j;
        const uint32_t bb = p < 4 * DW ? (b.w[(p < 4 * DW ? p : 0) >> 2] >> (8 * (p & 3))) & 0xFFu : 0u;
        word |= (p < w ? bb : tail_byte(p)) << (8 * j);
      }
      v[q] = word;
    }
    dst[0] = make_uint4(v[0], v[1], v[2], v[3]);
    dst[1] = make_uint4(v[4], v[5], v[6], v[7]);
    if (lrec) {  // (the fused slot takes 32-byte records only)
      uint4* l = lrec + (size_t)L.k * lstride + 2 * (L.env - lenv0);
      l[0] = make_uint4(v[0], v[1], v[2], v[3]);
      l[1] = make_uint4(v[4], v[5], v[6], v[7]);
    }
    for (int q32 = 1; q32 < a.rec_bytes / 32; ++q32) {  // columns >= 32: channel bits and acks only
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) word |= tail_byte(32 * q32 + 4 * q + j) << (8 * j);
        v[q] = word;
      }
      dst[2 * q32] = make_uint4(v[0], v[1], v[2], v[3]);
      dst[2 * q32 + 1] = make_uint4(v[4], v[5], v[6], v[7]);
    }
    }
  }
  // state = [concat_k B'[k,:d_k], channel_state (post-evolve).flatten(), acknack] (207-209)
  if (a.state || a.state_b) {
    if (L.active) {
      float* st = lds_state + (LARGE ? 0 : (L.local_env - wave * epw) * a.S);
      const int off = ag.state_offset, d = ag.deadline;
#pragma unroll
      for (int j = 0; j < DW * 4; ++j)
        if (j < d) st[off + j] = row_byte<DW>(b, j);
      const int sb = a.S - C * (N + 1);
      for (int c = 0; c < C; ++c) st[sb + L.k * C + c] = (float)((h_new >> c) & 1u);
      if (L.k == 0)
        for (int c = 0; c < C; ++c)
          st[sb + N * C + c] = ((ack_one >> c) & 1u) ? 1.f : (((ack_zero >> c) & 1u) ? 0.f : -1.f);
    }
    if (LARGE) {
      __syncthreads();
      if (a.state) flush_rows(a.state + (size_t)bidx * a.state_stride, a.state_stride, lds_state, 1, a.S, a.flags & 1u);
      if (a.state_b) flush_bf16(a.state_b + (size_t)bidx * a.state_b_ld, lds_state, a.S, threadIdx.x, blockDim.x, a.flags & 1u);
    } else {
      wave_lds_sync();
      for (int r = 0; r < wave_nenv; ++r) {
        if (a.state)
          wave_flush(a.state + (size_t)(wave_env0 + r) * a.state_stride, lds_state + r * a.S, a.S, a.flags & 1u);
        if (a.state_b)
          flush_bf16(a.state_b + (size_t)(wave_env0 + r) * a.state_b_ld, lds_state + r * a.S, a.S, L.lane, kWave,
                     a.flags & 1u);
      }
    }
  }
}

template <typename MaskT, int DW, bool LARGE, int CT, bool RESET>
__global__ __launch_bounds__(kMaxAgents) __attribute__((amdgpu_waves_per_eu(D2D_COMB_WAVES_PER_EU))) void comb_kernel(EnvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  comb_step<MaskT, DW, LARGE, CT, RESET>(a, lds, blockIdx.x, nullptr, 0, 0);
}

// =====================================================================
// Fused env + policy slot (ippo.py:293-330): one launch runs the env step of slot t
// (comb_step, actions_t -> record_{t+1}, env state, rewards) and the behaviour policy of slot t + 1
// (SplitNet, record_{t+1} -> actions_{t+1}, log-probs) for a slice of SE envs.  The record is still written to
// HBM (it is the rollout buffer the update reads) but the policy reads the slice's copy in LDS, and the launch
// boundary between the two kernels is gone.  The policy's weight split, amortised over 256 envs per wave in
// policy_split_kernel, is here paid once per (slice, agent): the price of an env-major slice.
// Prototype for the benched shape: 64 agents (one wave per env), 8 channels, the 32-byte record, the actor
// alone (no critic value), the Bernoulli head with A <= 8 (paired epilogue).
//   LDS: the slice's records [agent][SE envs x 32 B + 16 B] (the pad makes the 64 agents' 16-byte writes of one
//   env conflict-free); a tile read is 64 lanes x 8 contiguous bytes of one agent row.
// =====================================================================
template <int DW, int HT, int SE, int MODE>
__global__ __launch_bounds__(256, SE <= 32 ? 2 : 1) void comb_policy_fused_kernel(EnvArgs e, MlpArgs p) {
  static_assert(SE % 32 == 0, "the policy runs 16-env tiles in pairs");
  constexpr int LSTR = 2 * SE + 1;  // uint4 words per agent row
  __shared__ uint4 lrec[64 * LSTR];
  const int env0 = blockIdx.x * SE;
  // ---- env step of slot t: SE / 4 groups of four envs (one per wave, lane = agent)
  for (int q = 0; q < SE / 4; ++q)
    comb_step<uint8_t, DW, false, 8, false>(e, nullptr, blockIdx.x * (SE / 4) + q, lrec, LSTR, env0);
  __syncthreads();
  // ---- policy of slot t + 1 on the slice: wave w takes agents w, w + 4, ...
  const uint32_t rng = (MODE == kModeSample && p.rng_off) ? p.rng_step + *p.rng_off : p.rng_step;
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int k = wave; k < p.N; k += 4) {
    SplitNet<1, HT, true, false> net;
    net.load(p, k, g, i);
    uint32_t sm[1][2];
    record_sign_masks<1>(sm, p.sgn, k, g);
    const uint4* row = lrec + k * LSTR;
    auto tile = [&](int t, f32x4& lg) {
      // bytes 8g .. 8g + 7 of env 16t + i's record
      const uint2 w = reinterpret_cast<const uint2*>(row + 2 * (16 * t + i))[g];
      const uint32_t d[1][2] = {{w.x, w.y}};
      float xc[1][8];
      stage_record_words<1>(xc, d, sm);
      float v;
      net.template tile<true>(xc, lg, v);
    };
    for (int tt = 0; tt < SE / 16; tt += 2) {
      f32x4 lg0, lg1;
      tile(tt, lg0);
      tile(tt + 1, lg1);
      // paired epilogue (policy_split_kernel): lanes 0-31 keep tile tt, lanes 32-63 take tile tt + 1
      f32x4 lgc;
#pragma unroll
      for (int r = 0; r < 4; ++r) lgc[r] = uf(__builtin_amdgcn_permlane32_swap(fu(lg0[r]), fu(lg1[r]), false, false)[0]);
      const int envc = env0 + tt * 16 + i + (g < 2 ? 0 : 16);
      policy_epilogue<0, false, true, MODE>(p, lgc, 0.f, envc, envc < p.E, k, g, rng);
    }
  }
}

// =====================================================================
// Channel-selection env: action = channel id 0..C, one Markov state per
// channel shared by all agents, ACK = 1/n on good attempted channels.
// =====================================================================
template <int DW, bool LARGE>
__global__ __launch_bounds__(kMaxAgents) void chsel_kernel(EnvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Lane L = lane_geometry<LARGE>(a);
  const int N = a.N, C = a.C, F = a.F;
  // LDS carve: [per-env counts: 33 ints + reward][obs rows][state rows]
  int* cnt_all = reinterpret_cast<int*>(lds);
  int* cnt = cnt_all + L.local_env * 34;
  float* lds_obs = lds + a.cnt_words;
  float* lds_state = lds_obs + ((L.envs_per_block * N * F + 3) & ~3);
  const size_t row = (size_t)L.env * N + L.k;
  const uint64_t genv = a.env_base + (uint64_t)L.env;
  const uint32_t hmask = (C + 1 >= 32) ? 0xFFFFFFFFu : ((1u << (C + 1)) - 1u);
  uint32_t* chan = reinterpret_cast<uint32_t*>(a.chan);
  const bool env_ok = L.env < a.E;

  Row<DW> b;
#pragma unroll
  for (int i = 0; i < DW; ++i) b.w[i] = 0;
  uint32_t H = hmask, act = 0, rc = 0, dc = 0;
  d2d_agent_entry ag{};
  if (L.active) {
    ag = a.agents[L.k];
    if (!a.reset) {
      load_row<DW>(b, a.buf + row * DW);
      act = reinterpret_cast<const uint8_t*>(a.actions)[row];
      rc = a.recv[row];
      dc = a.disc[row];
    }
  }
  if (env_ok && !a.reset) H = chan[L.env] & hmask;
  for (int i = threadIdx.x; i < L.envs_per_block * 34; i += blockDim.x) cnt_all[i] = 0;
  __syncthreads();

  bool succ = false;
  int nsucc = 0;
  uint32_t H_new = H, attempted = 0;
  if (!a.reset) {
    // attempts = actions * has_a_packet (124-125); unique ids + counts (127-128)
    const uint32_t att = (L.active && row_any<DW>(b) && act <= (uint32_t)C) ? act : 0u;
    for (int j = 1; j <= C; ++j) {
      const int n = __popcll(__ballot(att == (uint32_t)j) & L.segmask);
      if (!LARGE) {
        if (L.k == 0) cnt[j] = n;
      } else if (L.lane == 0) {
        atomicAdd(&cnt[j], n);
      }
    }
    __syncthreads();
    for (int j = 1; j <= C; ++j) attempted |= (uint32_t)(cnt[j] > 0) << j;
    // successful users: their channel has exactly one attempt and is good (140-142)
    succ = att != 0 && cnt[att] == 1 && ((H >> att) & 1u);
    nsucc = env_count<LARGE>(succ, L, cnt + 33);
    if (succ) row_remove_first<DW>(b);
    dc += row_expire_shift<DW>(b);  // (154-155)
    // evolve_channel: C+1 scalar Bernoulli flips, channel 0 included (104-107, 156)
    uint32_t f = 0;
    if (env_ok) {
      if (a.flips) {
        f = reinterpret_cast<const uint32_t*>(a.flips)[L.env];
      } else {
        for (int blk = 0; blk * 4 < C + 1; ++blk) {
          const u32x4 r = philox((uint32_t)genv, kPerEnv, rng_of(a), (kStreamFlip << 24) | (uint32_t)blk, a.seed);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int j = blk * 4 + i;
            if (j <= C) f |= (uint32_t)((uint64_t)pick(r, i) < a.flip_thr[j]) << j;
          }
        }
      }
    }
    H_new = (H ^ f) & hmask;
  }
  // arrivals (reset 54-71, step 159-177)
  const bool drew = L.active && draws_now(a, L.k);
  if (drew) {
    const uint32_t x = arrival_value(a, ag, row, L.k, genv);
    row_set<DW>(b, (int)ag.deadline - 1, x);
    rc = (a.reset ? 0u : rc) + x;
  }
  if (a.reset) {
    rc = drew ? rc : 0u;
    dc = 0;
  }
  if (L.active) {
    store_row<DW>(b, a.buf + row * DW);
    a.recv[row] = rc;
    a.disc[row] = dc;
    if (a.success) a.success[row] = succ ? 1 : 0;
  }
  if (env_ok && L.k == 0) {
    chan[L.env] = H_new;
    if (!a.reset) {
      if (a.reward) a.reward[L.env] = nsucc;    // (188)
      a.selq[L.env] += __popc(attempted & H);  // (acknack > 0).sum()  (132)
      a.seln[L.env] += __popc(attempted);      // (acknack != 0).sum() (133)
      if (a.ack) {
        double* ak = reinterpret_cast<double*>(a.ack) + (size_t)L.env * (C + 1);
        ak[0] = 0.0;
        for (int j = 1; j <= C; ++j) {
          const int n = cnt[j];
          ak[j] = n == 0 ? 0.0 : (((H >> j) & 1u) ? 1.0 / (double)n : -1.0);
        }
      }
    } else {
      a.selq[L.env] = 0;
      a.seln[L.env] = 0;
    }
  }
  // obs_k = [B'[k,:d_k], acknack] (180-184); acknack[idx] = 2H-1, good -> 1/count
  // (129-137), rounded to float once from the double value like the reference's cast
  const int env0 = LARGE ? blockIdx.x : blockIdx.x * L.envs_per_block;
  const int nenv = min(L.envs_per_block, a.E - env0);
  if (a.obs && L.active) {
    float* o = lds_obs + (L.local_env * N + L.k) * F;
    const int w = ag.obs_width;
#pragma unroll
    for (int j = 0; j < DW * 4; ++j)
      if (j < w) o[j] = row_byte<DW>(b, j);
    o[w] = 0.f;
    for (int j = 1; j <= C; ++j) {
      const int n = a.reset ? 0 : cnt[j];
      o[w + j] = n == 0 ? 0.f : (((H >> j) & 1u) ? (float)(1.0 / (double)n) : -1.f);
    }
    for (int j = w + C + 1; j < F; ++j) o[j] = 0.f;
  }
  // state = [concat_k B'[k,:d_k], channel_state (post-evolve)] (185-186)
  if (a.state && L.active) {
    float* s = lds_state + L.local_env * a.S;
    const int off = ag.state_offset, d = ag.deadline;
#pragma unroll
    for (int j = 0; j < DW * 4; ++j)
      if (j < d) s[off + j] = row_byte<DW>(b, j);
    const int sb = a.S - (C + 1);
    if (L.k == 0)
      for (int j = 0; j <= C; ++j) s[sb + j] = (float)((H_new >> j) & 1u);
  }
  if (a.obs || a.state) {
    __syncthreads();
    if (a.obs && nenv > 0) flush_contig(a.obs + (size_t)env0 * N * F, lds_obs, nenv * N * F, a.flags & 1u);
    if (a.state && nenv > 0) flush_rows(a.state + (size_t)env0 * a.state_stride, a.state_stride, lds_state, nenv, a.S, a.flags & 1u);
  }
}


// =====================================================================
// D2DEnv: one shared channel, Discrete(2) actions, neighbourhood observations
// (/root/reference/envs/env.py: reset 51-99, decode_signal 101-103,
// evolve_channel 105-107, evolve_buffer 109-113, step 116-213).
// One lane = one agent; an env is a lane segment (N <= 64) or a workgroup.
//   n_attempts = #(action != 0 and has a packet).  Exactly one attempt is
//   decoded with probability channel_state[idx], and that state only ever
//   flips between 0 and 1 (reset ones, env.py:78; 1 - state, 105-107), so the
//   decode is the attempter's channel bit.  ack = 1 decoded / 0 channel error
//   or silence / -1 collision; every agent's reward is ack (207).
// obs_k = [B'[j,:d_j] for j in nbr(k)] + [H'[j] for j in nbr(k)] + [ack]
//   (post-evolve channel, 198-202) gathered from the env's rows staged in LDS
//   and written straight to HBM (full neighbourhoods make rows long:
//   F = sum d + N + 1); state = [concat_k B'[k,:d_k], H', ack] (204-205).
// Counters: sel_quality = channel_errors, sel_count = n_collisions.
// =====================================================================
template <int DW, bool LARGE>
__global__ __launch_bounds__(kMaxAgents) void single_kernel(EnvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const Lane L = lane_geometry<LARGE>(a);
  const int N = a.N, F = a.F;
  int* cnt = reinterpret_cast<int*>(lds) + L.local_env * 4;
  uint32_t* rows = reinterpret_cast<uint32_t*>(lds) + a.cnt_words + (size_t)L.local_env * N * (DW + 1);
  const size_t row = (size_t)L.env * N + L.k;
  const uint64_t genv = a.env_base + (uint64_t)L.env;
  const bool env_ok = L.env < a.E;
  // compact record (ABI 14): the agents' gather codes staged in LDS, one row of rec_bytes + 4 codes per agent (the pad
  // keeps the 16-byte reads of 8 consecutive agents on distinct banks): columns < F the obs codes, column F the
  // layer-1 bias input (-3: the byte 1), past it -2 (0)
  const int CS = a.rec_bytes + 4;
  int* codes_s = reinterpret_cast<int*>(lds) + a.cnt_words + (size_t)L.envs_per_block * N * (DW + 1);
  if (a.rec) {
    // pre-decoded: a row byte as (LDS word of the block's row image) | (bit shift << 16), else -1 ack / -2 zero / -3 one
    for (int idx = threadIdx.x; idx < N * CS; idx += blockDim.x) {
      const int j = idx / CS, c = idx - j * CS;
      int code = c < F ? a.gather[(size_t)j * F + c] : c == F ? -3 : -2;
      if (code >= 0) {
        const int jj = code >> 6, q = code & 63;
        code = (jj * (DW + 1) + (q == 32 ? DW : (q >> 2))) | ((q == 32 ? 0 : (q & 3) * 8) << 16);
      }
      codes_s[idx] = code;
    }
  }

  Row<DW> b;
#pragma unroll
  for (int i = 0; i < DW; ++i) b.w[i] = 0;
  uint32_t h = 1, act = 0, rc = 0, dc = 0;
  d2d_agent_entry ag{};
  if (L.active) {
    ag = a.agents[L.k];
    if (!a.reset) {
      load_row<DW>(b, a.buf + row * DW);
      h = reinterpret_cast<const uint8_t*>(a.chan)[row] & 1u;
      act = reinterpret_cast<const uint8_t*>(a.actions)[row];
      rc = a.recv[row];
      dc = a.disc[row];
    }
  }
  if (LARGE) {
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
  }
  int ackv = 0, n = 0, ng = 0;
  bool succ = false;
  uint32_t h_new = 1;  // reset: channel_state = ones (78)
  if (!a.reset) {
    const bool att = L.active && act != 0 && row_any<DW>(b);   // attempts = actions * has_a_packet (124-125)
    n = env_count<LARGE>(att, L, cnt);                          // n_attempts (126)
    ng = env_count<LARGE>(att && h != 0, L, cnt + 1);
    const bool decoded = n == 1 && ng == 1;                     // decode_signal (101-103, 133)
    ackv = n == 1 ? (decoded ? 1 : 0) : (n > 1 ? -1 : 0);       // 134-152
    succ = att && decoded;
    if (succ) row_remove_first<DW>(b);                          // 141-142
    dc += row_expire_shift<DW>(b);                              // 155-156
    uint32_t f = 0;                                             // evolve_channel (157, 105-107)
    if (L.active) {
      if (a.flips) {
        f = reinterpret_cast<const uint8_t*>(a.flips)[row] & 1u;
      } else {
        const u32x4 r = philox((uint32_t)genv, (uint32_t)L.k, rng_of(a), kStreamFlip << 24, a.seed);
        f = (uint64_t)r.x < a.flip_thr[L.k] ? 1u : 0u;
      }
    }
    h_new = h ^ f;
  }
  // arrivals (reset 56-76, step 160-181)
  const bool drew = L.active && draws_now(a, L.k);
  if (drew) {
    const uint32_t x = arrival_value(a, ag, row, L.k, genv);
    row_set<DW>(b, (int)ag.deadline - 1, x);
    rc = (a.reset ? 0u : rc) + x;
  }
  if (a.reset) {
    rc = drew ? rc : 0u;
    dc = 0;
  }
  if (L.active) {
    store_row<DW>(b, a.buf + row * DW);
    reinterpret_cast<uint8_t*>(a.chan)[row] = (uint8_t)h_new;
    a.recv[row] = rc;
    a.disc[row] = dc;
    if (a.success && !a.reset) a.success[row] = succ ? 1 : 0;
  }
  if (env_ok && L.k == 0) {
    if (!a.reset) {
      if (a.reward) a.reward[L.env] = ackv;                          // rewards = ack (207)
      if (a.ack) reinterpret_cast<int8_t*>(a.ack)[L.env] = (int8_t)ackv;
      a.selq[L.env] += (n == 1 && ng != 1) ? 1 : 0;                   // channel_errors (144-145)
      a.seln[L.env] += n > 1 ? 1 : 0;                                 // n_collisions (147-148)
    } else {
      a.selq[L.env] = 0;
      a.seln[L.env] = 0;
    }
  }
  // The env's rows + channel bits go to LDS; the block then writes its envs'
  // contiguous obs range [epb][N][F] (and state rows) cooperatively, one float
  // per lane per store (coalesced), each element resolved through the gather
  // table: j*64+q = byte q of agent j's row, j*64+32 = agent j's channel, -1 ack.
  if (L.active) {
#pragma unroll
    for (int i = 0; i < DW; ++i) rows[L.k * (DW + 1) + i] = b.w[i];
    rows[L.k * (DW + 1) + DW] = h_new;
  }
  if (L.k == 0) cnt[2] = ackv;
  __syncthreads();
  const int epb = L.envs_per_block;
  const int env0 = LARGE ? blockIdx.x : blockIdx.x * epb;
  const int nenv = min(epb, a.E - env0);
  const bool nt = a.flags & 1u;
  const uint32_t* rows0 = reinterpret_cast<const uint32_t*>(lds) + a.cnt_words;
  const int* cnt0 = reinterpret_cast<const int*>(lds);
  // one gather code per output column, decoded once and applied to every env of the block
  // (column-outer loop: no per-element division, each code load amortised over epb envs)
  const int NW = N * (DW + 1);
  auto decode = [&](int code, int& word, int& shift) {
    word = code;
    shift = 0;
    if (code >= 0) {
      const int j = code >> 6, q = code & 63;
      word = j * (DW + 1) + (q == 32 ? DW : (q >> 2));
      shift = q == 32 ? 0 : (q & 3) * 8;
    }
  };
  auto value = [&](int le, int word, int shift) -> float {
    if (word >= 0) return (float)((rows0[le * NW + word] >> shift) & 0xFFu);
    return word == -1 ? (float)cnt0[le * 4 + 2] : 0.f;
  };
  auto emit = [&](float* base, size_t env_stride, const int* codes, int cols) {
    const bool vec = (cols & 3) == 0 && (env_stride & 3) == 0 && (reinterpret_cast<uintptr_t>(base) & 15) == 0;
    if (vec) {  // 16-byte stores: four columns per lane
      for (int r4 = threadIdx.x; r4 < (cols >> 2); r4 += blockDim.x) {
        const int4 c = reinterpret_cast<const int4*>(codes)[r4];
        int w0, w1, w2, w3, s0, s1, s2, s3;
        decode(c.x, w0, s0);
        decode(c.y, w1, s1);
        decode(c.z, w2, s2);
        decode(c.w, w3, s3);
        float4* o = reinterpret_cast<float4*>(base) + r4;
        for (int le = 0; le < nenv; ++le) {
          const float4 v = make_float4(value(le, w0, s0), value(le, w1, s1), value(le, w2, s2), value(le, w3, s3));
          float4* d = o + (size_t)le * (env_stride >> 2);
          if (nt) {
            __builtin_nontemporal_store(v.x, &d->x);
            __builtin_nontemporal_store(v.y, &d->y);
            __builtin_nontemporal_store(v.z, &d->z);
            __builtin_nontemporal_store(v.w, &d->w);
          } else {
            *d = v;
          }
        }
      }
      return;
    }
    for (int r = threadIdx.x; r < cols; r += blockDim.x) {
      int word, shift;
      decode(codes[r], word, shift);
      float* o = base + r;
      for (int le = 0; le < nenv; ++le) st_stream(o + (size_t)le * env_stride, value(le, word, shift), nt);
    }
  };
  if (a.obs && nenv > 0) emit(a.obs + (size_t)env0 * N * F, (size_t)N * F, a.gather, N * F);
  if (a.state && nenv > 0)
    emit(a.state + (size_t)env0 * a.state_stride, (size_t)a.state_stride, a.gather + (size_t)N * F, a.S);
  if (a.rec && L.active) {
    // the lane's own record row [env][agent][rec_bytes]: byte c = obs column c (uint8 buffer counts and channel
    // bits, the int8 ack), byte F = 1, zeros past it -- 32 bytes per agent-step instead of 4 F of fp32 rows
    const int le = L.local_env;
    const int* cj = codes_s + L.k * CS;
    const uint32_t ackb = (uint32_t)cnt0[le * 4 + 2] & 0xFFu;
    const uint32_t* rle = rows0 + le * NW;
    auto byte_at = [&](int code) -> uint32_t {
      if (code >= 0) return (rle[code & 0xFFFF] >> (code >> 16)) & 0xFFu;
      return code == -1 ? ackb : code == -3 ? 1u : 0u;
    };
    uint4* dst = reinterpret_cast<uint4*>(a.rec + row * (size_t)a.rec_bytes);
    for (int p16 = 0; p16 < (a.rec_bytes >> 4); ++p16) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int4 c4 = *reinterpret_cast<const int4*>(cj + 16 * p16 + 4 * q);
        w[q] = byte_at(c4.x) | (byte_at(c4.y) << 8) | (byte_at(c4.z) << 16) | (byte_at(c4.w) << 24);
      }
      st_rec(dst + p16, w[0], w[1], w[2], w[3], nt);
    }
  }
}

// =====================================================================
// synthetic actions (env-only benchmark / baseline policies)
// =====================================================================
template <typename MaskT>
__global__ __launch_bounds__(256) void sample_actions_kernel(int E, int N, int C, int chsel, uint64_t env_base,
                                                             uint64_t seed, uint32_t rng_step, uint64_t thr,
                                                             void* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)E * N) return;
  const int env = (int)(i / N), k = (int)(i - (int64_t)env * N);
  const uint32_t genv = (uint32_t)(env_base + (uint64_t)env);
  if (chsel == 1) {
    const u32x4 r = philox(genv, (uint32_t)k, rng_step, kStreamAction << 24, seed);
    reinterpret_cast<uint8_t*>(out)[i] = (uint8_t)(((uint64_t)r.x * (uint64_t)(C + 1)) >> 32);
    return;
  }
  if (chsel == 2) {  // single channel: transmit with probability thr / 2^32 (GFAccess.act, baselines.py:121-125)
    const u32x4 r = philox(genv, (uint32_t)k, rng_step, kStreamAction << 24, seed);
    reinterpret_cast<uint8_t*>(out)[i] = (uint8_t)((uint64_t)r.x < thr ? 1 : 0);
    return;
  }
  uint32_t m = 0;
  for (int blk = 0; blk * 4 < C; ++blk) {
    const u32x4 r = philox(genv, (uint32_t)k, rng_step, (kStreamAction << 24) | (uint32_t)blk, seed);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = blk * 4 + j;
      if (c < C) m |= (uint32_t)((uint64_t)pick(r, j) < thr) << c;
    }
  }
  reinterpret_cast<MaskT*>(out)[i] = (MaskT)m;
}

}  // namespace d2d

// =====================================================================
// C ABI launchers
// =====================================================================
using namespace d2d;

namespace {

// streaming (non-temporal) stores for the obs/state flush: d2d_set_option(D2D_OPT_NT_STORES, v),
// initial value from the environment variable D2D_NT_STORES
// (a relaxed atomic: d2d_set_option may run on another host thread; -1 = not yet read from the environment)
std::atomic<int> g_nt_stores{-1};
uint32_t store_flags() {
  int v = g_nt_stores.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("D2D_NT_STORES");
    int expect = -1;
    g_nt_stores.compare_exchange_strong(expect, (e && e[0] == '1') ? 1 : 0, std::memory_order_relaxed);
    v = g_nt_stores.load(std::memory_order_relaxed);
  }
  return (uint32_t)v;
}

int buffer_words(int D) { return D <= 4 ? 1 : D <= 8 ? 2 : D <= 12 ? 3 : D <= 16 ? 4 : 8; }

int check_desc(const d2d_env_desc* d) {
  if (!d) { d2d_set_error("desc is NULL"); return D2D_EINVAL; }
  const bool comb = d->env_kind == D2D_ENV_COMBINATORIAL;
  const bool single = d->env_kind == D2D_ENV_SINGLE;
  if (!comb && !single && d->env_kind != D2D_ENV_CHANNEL_SELECTION) { d2d_set_error("unknown env_kind %d", d->env_kind); return D2D_EINVAL; }
  if (single) {
    if (d->n_agents < 1 || d->n_agents > kMaxAgents) { d2d_set_error("n_agents=%d outside [1,%d]", d->n_agents, kMaxAgents); return D2D_EUNSUPPORTED; }
    if (d->n_channels != 1) { d2d_set_error("the single-channel env needs n_channels == 1"); return D2D_EINVAL; }
    if (d->max_deadline < 1 || d->max_deadline > 32) { d2d_set_error("max_deadline=%d outside [1,32]", d->max_deadline); return D2D_EUNSUPPORTED; }
    if (d->n_envs < 0) { d2d_set_error("n_envs < 0"); return D2D_EINVAL; }
    if (d->obs_dim < 2 || d->state_dim != 0 && d->state_stride < d->state_dim) { d2d_set_error("bad obs/state dims"); return D2D_EINVAL; }
    if (!d->agents || !d->flip_thr || !d->arrival_kind_host || !d->period_host || !d->offset_host || !d->gather ||
        !d->poisson_cdf) {
      d2d_set_error("desc tables (incl. the gather map and poisson_cdf) must be non-NULL"); return D2D_EINVAL;
    }
    return D2D_OK;
  }
  if (d->n_agents < 1 || d->n_agents > kMaxAgents) { d2d_set_error("n_agents=%d outside [1,%d]", d->n_agents, kMaxAgents); return D2D_EUNSUPPORTED; }
  if (d->n_channels < 1 || d->n_channels > (comb ? 32 : 31)) { d2d_set_error("n_channels=%d unsupported", d->n_channels); return D2D_EUNSUPPORTED; }
  if (d->max_deadline < 1 || d->max_deadline > 32) { d2d_set_error("max_deadline=%d outside [1,32]", d->max_deadline); return D2D_EUNSUPPORTED; }
  if (d->n_envs < 0) { d2d_set_error("n_envs < 0"); return D2D_EINVAL; }
  const int F = comb ? d->max_deadline + 2 * d->n_channels : d->max_deadline + d->n_channels + 1;
  if (d->obs_dim != F) { d2d_set_error("obs_dim=%d, expected %d", d->obs_dim, F); return D2D_EINVAL; }
  if (d->state_stride < d->state_dim) { d2d_set_error("state_stride < state_dim"); return D2D_EINVAL; }
  if (!d->agents || !d->flip_thr || !d->arrival_kind_host || !d->period_host || !d->offset_host || !d->poisson_cdf) {
    d2d_set_error("desc tables (incl. poisson_cdf) must be non-NULL"); return D2D_EINVAL;
  }
  return D2D_OK;
}

// which agents draw an arrival at timestep t: numpy float semantics of
// `timestep % period == offsets` (combinatorial_env.py:183,194), t = 0 at reset
void draw_mask(const d2d_env_desc* d, int t, uint64_t* mask) {
  memset(mask, 0, sizeof(uint64_t) * (kMaxAgents / 64));
  for (int k = 0; k < d->n_agents; ++k) {
    const int kind = d->arrival_kind_host[k];
    bool dr = kind == D2D_ARRIVAL_POISSON;
    if (kind == D2D_ARRIVAL_SCHEDULED_BERNOULLI) dr = std::fmod((double)t, d->period_host[k]) == d->offset_host[k];
    if (dr) mask[k >> 6] |= 1ull << (k & 63);
  }
}

template <typename K>
int set_lds(K kernel, size_t bytes) {
  if (bytes > 163840) { d2d_set_error("LDS requirement %zu B exceeds 160 KiB (N*obs_dim too large)", bytes); return D2D_EUNSUPPORTED; }
  if (bytes > 65536)
    D2D_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  return D2D_OK;
}

// dynamic LDS of one workgroup (must match the carve in the kernels)
size_t lds_need(const EnvArgs& a, int block, int kind) {
  const bool large = a.N > kWave;
  const bool stage = a.obs || a.state || a.state_b;
  const bool comb = kind == D2D_ENV_COMBINATORIAL;
  if (kind == D2D_ENV_SINGLE) {
    const int epb = large ? 1 : block / a.seg;
    return sizeof(float) * ((size_t)a.cnt_words + (size_t)epb * a.N * (a.D <= 4 ? 2 : a.D <= 8 ? 3 : a.D <= 12 ? 4 : a.D <= 16 ? 5 : 9) +
                            (a.rec ? (size_t)a.N * (a.rec_bytes + 4) : 0));
  }
  if (comb) {
    const int nwaves = block / kWave;
    const int epw = large ? 1 : kWave / a.seg;
    const size_t slot = (size_t)((kWave * a.F + 3) & ~3);
    size_t w = (size_t)a.cnt_words + (stage ? nwaves * slot : 0);
    if (a.state || a.state_b) w += large ? (size_t)a.S : (size_t)nwaves * ((epw * a.S + 3) & ~3);
    return sizeof(float) * w;
  }
  const int epb = large ? 1 : block / a.seg;
  return sizeof(float) * ((size_t)a.cnt_words + (size_t)(stage ? ((epb * a.N * a.F + 3) & ~3) : 0) +
                          (a.state ? (size_t)epb * a.S : 0));
}

template <typename K>
int launch(K kernel, const EnvArgs& a, int block, hipStream_t s, int kind) {
  const bool large = a.N > kWave;
  const int epb = large ? 1 : block / a.seg;
  const int grid = (a.E + epb - 1) / epb;
  if (grid == 0) return D2D_OK;
  const size_t lds = lds_need(a, block, kind);
  int rc = set_lds(kernel, lds);
  if (rc) return rc;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), lds, s, a);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

template <typename MaskT, int DW, int CT, bool RESET>
int dispatch_comb_ct(const EnvArgs& a, int block, hipStream_t s) {
  if (a.N > kWave) return launch(comb_kernel<MaskT, DW, true, CT, RESET>, a, block, s, D2D_ENV_COMBINATORIAL);
  return launch(comb_kernel<MaskT, DW, false, CT, RESET>, a, block, s, D2D_ENV_COMBINATORIAL);
}

template <int DW>
int dispatch_comb(const EnvArgs& a, int block, hipStream_t s) {
  const int C = a.C;
  if (a.reset) {
    if (C <= 8) return dispatch_comb_ct<uint8_t, DW, 0, true>(a, block, s);
    if (C <= 16) return dispatch_comb_ct<uint16_t, DW, 0, true>(a, block, s);
    return dispatch_comb_ct<uint32_t, DW, 0, true>(a, block, s);
  }
  if (C == 8) return dispatch_comb_ct<uint8_t, DW, 8, false>(a, block, s);
  if (C == 4) return dispatch_comb_ct<uint8_t, DW, 4, false>(a, block, s);
  if (C == 16) return dispatch_comb_ct<uint16_t, DW, 16, false>(a, block, s);
  if (C <= 8) return dispatch_comb_ct<uint8_t, DW, 0, false>(a, block, s);
  if (C <= 16) return dispatch_comb_ct<uint16_t, DW, 0, false>(a, block, s);
  return dispatch_comb_ct<uint32_t, DW, 0, false>(a, block, s);
}

template <int DW>
int dispatch_dw(const EnvArgs& a, int block, int kind, hipStream_t s) {
  if (kind == D2D_ENV_SINGLE) {
    if (a.N > kWave) return launch(single_kernel<DW, true>, a, block, s, kind);
    return launch(single_kernel<DW, false>, a, block, s, kind);
  }
  if (kind == D2D_ENV_CHANNEL_SELECTION) {
    if (a.N > kWave) return launch(chsel_kernel<DW, true>, a, block, s, kind);
    return launch(chsel_kernel<DW, false>, a, block, s, kind);
  }
  return dispatch_comb<DW>(a, block, s);
}

// the kernel arguments of one reset / step (everything but the launch geometry)
int env_args(const d2d_env_desc* d, const d2d_env_state* st, const void* actions, const d2d_env_replay* rp,
             const d2d_env_out* out, int reset, int t, uint32_t rng_step, EnvArgs& a) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!st || !st->buffers || !st->channels || !st->received || !st->discarded) {
    d2d_set_error("state buffers must be non-NULL"); return D2D_EINVAL;
  }
  const bool comb = d->env_kind == D2D_ENV_COMBINATORIAL;
  if (!comb && (!st->sel_quality || !st->sel_count)) {
    d2d_set_error("chsel / single need sel_quality / sel_count"); return D2D_EINVAL;
  }
  if (!reset && !actions) { d2d_set_error("actions is NULL"); return D2D_EINVAL; }
  memset(&a, 0, sizeof(a));
  a.E = d->n_envs; a.N = d->n_agents; a.C = d->n_channels; a.D = d->max_deadline; a.F = d->obs_dim;
  a.S = d->state_dim; a.state_stride = d->state_stride; a.reset = reset; a.rng_step = rng_step;
  a.env_base = d->env_base; a.seed = d->seed; a.agents = d->agents; a.flip_thr = d->flip_thr;
  a.pois_cdf = d->poisson_cdf;
  a.buf = st->buffers; a.chan = st->channels; a.recv = st->received; a.disc = st->discarded;
  a.selq = st->sel_quality; a.seln = st->sel_count; a.actions = actions;
  if (rp) { a.flips = rp->flips; a.arrivals = rp->arrivals; }
  a.gather = d->gather;
  a.rng_off = d->rng_offset;
  if (out) {
    a.obs = out->obs; a.state = out->state; a.reward = out->reward; a.ack = out->ack; a.success = out->success;
    a.rec = out->obs_record;
    a.state_b = out->state_bf16;
    a.state_b_ld = out->state_bf16_ld;
  }
  if (a.state_b) {
    if (!comb) { d2d_set_error("state_bf16 is implemented for the combinatorial env only"); return D2D_EUNSUPPORTED; }
    if ((reinterpret_cast<uintptr_t>(a.state_b) & 15) || (a.state_b_ld & 7) || a.state_b_ld < ((int64_t)a.S + 7) / 8 * 8) {
      d2d_set_error("state_bf16: 16-byte aligned rows of state_bf16_ld >= state_dim rounded up to 8 (a multiple of 8)");
      return D2D_EINVAL;
    }
  }
  a.rec_bytes = D2D_RECORD_BYTES(a.F);
  if (a.rec && !comb && d->env_kind != D2D_ENV_SINGLE) {
    d2d_set_error("obs_record is implemented for the combinatorial env and the D2DEnv only"); return D2D_EUNSUPPORTED;
  }
  if (a.rec && (reinterpret_cast<uintptr_t>(a.rec) & 15)) { d2d_set_error("obs_record must be 16-byte aligned"); return D2D_EINVAL; }
  draw_mask(d, reset ? 0 : t, a.draw);
  a.flags = store_flags();
  return D2D_OK;
}

int run_env(const d2d_env_desc* d, const d2d_env_state* st, const void* actions, const d2d_env_replay* rp,
            const d2d_env_out* out, int reset, int t, uint32_t rng_step, void* stream) {
  EnvArgs a;
  if (const int rc = env_args(d, st, actions, rp, out, reset, t, rng_step, a)) return rc;
  const int kind = d->env_kind;
  const bool comb = kind == D2D_ENV_COMBINATORIAL;
  const bool large = a.N > kWave;
  int seg = 1;
  while (seg < a.N) seg <<= 1;
  a.seg = large ? ((a.N + kWave - 1) / kWave) * kWave : seg;
  // block: 256 lanes (4 waves) unless the LDS staging of that many envs would
  // exceed 64 KiB (keep >= 2 workgroups per CU); LARGE: one env per block
  auto cnt_words = [&](int epb) {
    return kind == D2D_ENV_SINGLE ? epb * 4 : comb ? (large ? 80 : 0) : (((epb * 34) + 3) & ~3);
  };
  // single: 512-lane blocks amortise each gather-code load over more envs (measured 256: 130 us,
  // 512: 125 us, 1024: 134 us per 65,536 x 64-agent step)
  // 512-lane blocks (8 envs of 64 agents): comb 64 x 8 x 65,536 141 -> 137 us against 256-lane
  // blocks; single: 8 envs per gather-table read (256: 130 us, 512: 125 us, 1024: 134 us)
  int block = large ? a.seg : (comb && !a.obs && !a.state && !a.state_b) ? D2D_COMB_REC_BLOCK : 512;
  a.cnt_words = cnt_words(large ? 1 : block / a.seg);
  while (!large && block > kWave && block > a.seg && lds_need(a, block, kind) > 65536) {
    block >>= 1;
    a.cnt_words = cnt_words(block / a.seg);
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (buffer_words(a.D)) {
    case 1: return dispatch_dw<1>(a, block, kind, s);
    case 2: return dispatch_dw<2>(a, block, kind, s);
    case 3: return dispatch_dw<3>(a, block, kind, s);
    case 4: return dispatch_dw<4>(a, block, kind, s);
    default: return dispatch_dw<8>(a, block, kind, s);
  }
}

// envs per workgroup of the fused slot: 32 (default) or 64 (d2d_set_option(D2D_OPT_FUSED_SLICE, 64))
std::atomic<int> g_fused_slice{32};

template <int DW, int HT, int MODE>
int launch_fused_se(const EnvArgs& e, const MlpArgs& p, hipStream_t s) {
  const int se = g_fused_slice.load(std::memory_order_relaxed);
  const dim3 grid((e.E + se - 1) / se);
  if (se == 64) hipLaunchKernelGGL((comb_policy_fused_kernel<DW, HT, 64, MODE>), grid, dim3(256), 0, s, e, p);
  else hipLaunchKernelGGL((comb_policy_fused_kernel<DW, HT, 32, MODE>), grid, dim3(256), 0, s, e, p);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

template <int DW>
int launch_fused(const EnvArgs& e, const MlpArgs& p, hipStream_t s) {
  const bool det = p.deterministic != 0;
  if (p.H <= 32) return det ? launch_fused_se<DW, 2, kModeDeterministic>(e, p, s) : launch_fused_se<DW, 2, kModeSample>(e, p, s);
  return det ? launch_fused_se<DW, 4, kModeDeterministic>(e, p, s) : launch_fused_se<DW, 4, kModeSample>(e, p, s);
}

}  // namespace

extern std::atomic<int> g_policy_f32_mfma;  // policy_kernels.hip
extern std::atomic<int> g_policy_critic_split;  // policy_kernels.hip
extern std::atomic<int> g_gru_grad_history;  // gru_kernels.hip
extern std::atomic<int> g_critic_grad_rows;  // update_kernels.hip

extern "C" int d2d_set_option(int32_t option, int32_t value) {
  if (option == D2D_OPT_GRU_GRAD_HISTORY) {
    g_gru_grad_history.store(value ? 1 : 0, std::memory_order_relaxed);
    return D2D_OK;
  }
  if (option == D2D_OPT_NT_STORES) {
    g_nt_stores.store(value ? 1 : 0, std::memory_order_relaxed);
    return D2D_OK;
  }
  if (option == D2D_OPT_FUSED_SLICE) {
    if (value != 0 && value != 32 && value != 64) { d2d_set_error("D2D_OPT_FUSED_SLICE: 0, 32 or 64"); return D2D_EINVAL; }
    g_fused_slice.store(value == 64 ? 64 : 32, std::memory_order_relaxed);
    return D2D_OK;
  }
  if (option == D2D_OPT_CRITIC_GRAD_ROWS) {
    g_critic_grad_rows.store(value ? 1 : 0, std::memory_order_relaxed);
    return D2D_OK;
  }
  if (option == D2D_OPT_POLICY_F32_MFMA) {
    g_policy_f32_mfma.store(value ? 1 : 0, std::memory_order_relaxed);
    return D2D_OK;
  }
  if (option == D2D_OPT_POLICY_CRITIC_SPLIT) {
    g_policy_critic_split.store(value ? 1 : 0, std::memory_order_relaxed);
    return D2D_OK;
  }
  d2d_set_error("unknown option %d", option);
  return D2D_EINVAL;
}

extern "C" int d2d_buffer_words(int32_t max_deadline) { return buffer_words(max_deadline); }

extern "C" int d2d_env_single_gather_map(int32_t n_agents, const int32_t* deadlines, const int32_t* nbr_ptr,
                                          const int32_t* nbr_idx, int32_t obs_dim, int32_t* out, int64_t out_len) {
  const int N = n_agents;
  if (N < 1 || N > d2d::kMaxAgents || !deadlines || !nbr_ptr || !nbr_idx || !out) {
    d2d_set_error("gather map: bad arguments"); return D2D_EINVAL;
  }
  int64_t S = N + 1;
  for (int k = 0; k < N; ++k) {
    if (deadlines[k] < 1 || deadlines[k] > 32) { d2d_set_error("gather map: deadline[%d]=%d", k, deadlines[k]); return D2D_EINVAL; }
    S += deadlines[k];
  }
  const int64_t need = (int64_t)N * obs_dim + S;
  if (obs_dim < 1 || out_len < need) { d2d_set_error("gather map: out_len %lld < %lld", (long long)out_len, (long long)need); return D2D_EINVAL; }
  if (nbr_ptr[0] != 0) { d2d_set_error("gather map: nbr_ptr[0] != 0"); return D2D_EINVAL; }
  for (int k = 0; k < N; ++k) {
    int32_t* o = out + (int64_t)k * obs_dim;
    const int p0 = nbr_ptr[k], p1 = nbr_ptr[k + 1];
    if (p1 < p0) { d2d_set_error("gather map: nbr_ptr not monotone"); return D2D_EINVAL; }
    int64_t len = 1;
    for (int p = p0; p < p1; ++p) {
      if (nbr_idx[p] < 0 || nbr_idx[p] >= N) { d2d_set_error("gather map: neighbour %d out of range", nbr_idx[p]); return D2D_EINVAL; }
      len += deadlines[nbr_idx[p]] + 1;
    }
    if (len > obs_dim) { d2d_set_error("gather map: agent %d needs obs_dim >= %lld", k, (long long)len); return D2D_EINVAL; }
    int off = 0;
    for (int p = p0; p < p1; ++p) {                 // buffers of the neighbours (env.py:91-92)
      const int j = nbr_idx[p];
      for (int q = 0; q < deadlines[j]; ++q) o[off++] = j * 64 + q;
    }
    for (int p = p0; p < p1; ++p) o[off++] = nbr_idx[p] * 64 + 32;   // their channel states (93)
    o[off++] = -1;                                                     // last feedback (94)
    while (off < obs_dim) o[off++] = -2;
  }
  int32_t* st = out + (int64_t)N * obs_dim;        // state (env.py:97-98)
  int off = 0;
  for (int k = 0; k < N; ++k)
    for (int q = 0; q < deadlines[k]; ++q) st[off++] = k * 64 + q;
  for (int k = 0; k < N; ++k) st[off++] = k * 64 + 32;
  st[off++] = -1;
  return (int)need;
}

extern "C" int d2d_mask_bytes(int32_t n_channels) { return n_channels <= 8 ? 1 : n_channels <= 16 ? 2 : 4; }

extern "C" int d2d_env_reset(const d2d_env_desc* desc, const d2d_env_state* st, const d2d_env_replay* replay,
                             const d2d_env_out* out, uint32_t rng_step, void* stream) {
  return run_env(desc, st, nullptr, replay, out, 1, 0, rng_step, stream);
}

extern "C" int d2d_env_step(const d2d_env_desc* desc, const d2d_env_state* st, const void* actions,
                            const d2d_env_replay* replay, const d2d_env_out* out, int32_t timestep, uint32_t rng_step,
                            void* stream) {
  return run_env(desc, st, actions, replay, out, 0, timestep, rng_step, stream);
}

extern "C" int d2d_comb_policy_fused_step(const d2d_env_desc* desc, const d2d_env_state* st, const void* actions,
                                          const d2d_env_out* out, int32_t timestep, uint32_t env_rng_step,
                                          const d2d_mlp_desc* policy, uint32_t policy_rng_step, int32_t deterministic,
                                          void* actions_out, float* logp_out, void* stream) {
  EnvArgs e;
  if (const int rc = env_args(desc, st, actions, nullptr, out, 0, timestep, env_rng_step, e)) return rc;
  if (desc->env_kind != D2D_ENV_COMBINATORIAL || e.N != 64 || e.C != 8 || e.rec_bytes != 32) {
    d2d_set_error("the combinatorial env with 64 agents, 8 channels and a 32-byte record only");
    return D2D_EUNSUPPORTED;
  }
  if (!e.rec || e.obs || e.state || e.state_b) {
    d2d_set_error("out must carry obs_record and no obs / state rows");
    return D2D_EINVAL;
  }
  e.seg = 64;  // run_env's geometry for N = 64: one env per wave, no LDS staging
  e.cnt_words = 0;
  if (!policy) { d2d_set_error("policy is NULL"); return D2D_EINVAL; }
  MlpArgs p;
  if (const int rc = policy_mlp_args(policy, e.rec, nullptr, policy_rng_step, deterministic, actions_out, logp_out,
                                     nullptr, p))
    return rc;
  if (!p.rec || p.N != e.N || p.E != e.E || p.F != e.F || policy->env_base != desc->env_base) {
    d2d_set_error("the policy must read this env's record (D2D_OBS_U8, same agents, envs, obs_dim and env_base)");
    return D2D_EINVAL;
  }
  if (p.kind != 0 || p.A > 8 || p.H > 64 || p.F + 1 > 32 || p.v1) {
    d2d_set_error("the Bernoulli actor with n_out <= 8, hidden <= 64, obs_dim < 32 and no critic only");
    return D2D_EUNSUPPORTED;
  }
  if (e.E == 0) return D2D_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (buffer_words(e.D)) {
    case 1: return launch_fused<1>(e, p, s);
    case 2: return launch_fused<2>(e, p, s);
    case 3: return launch_fused<3>(e, p, s);
    case 4: return launch_fused<4>(e, p, s);
    default: return launch_fused<8>(e, p, s);
  }
}

extern "C" int d2d_sample_actions(const d2d_env_desc* d, void* actions, uint64_t threshold, uint32_t rng_step,
                                  void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!actions) { d2d_set_error("actions is NULL"); return D2D_EINVAL; }
  const int64_t n = (int64_t)d->n_envs * d->n_agents;
  if (n == 0) return D2D_OK;
  const int grid = (int)((n + 255) / 256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int chsel = d->env_kind == D2D_ENV_CHANNEL_SELECTION ? 1 : d->env_kind == D2D_ENV_SINGLE ? 2 : 0;
  const int C = d->n_channels;
  if (chsel || C <= 8)
    hipLaunchKernelGGL(sample_actions_kernel<uint8_t>, dim3(grid), dim3(256), 0, s, d->n_envs, d->n_agents, C, chsel,
                       d->env_base, d->seed, rng_step, threshold, actions);
  else if (C <= 16)
    hipLaunchKernelGGL(sample_actions_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, d->n_envs, d->n_agents, C, 0,
                       d->env_base, d->seed, rng_step, threshold, actions);
  else
    hipLaunchKernelGGL(sample_actions_kernel<uint32_t>, dim3(grid), dim3(256), 0, s, d->n_envs, d->n_agents, C, 0,
                       d->env_base, d->seed, rng_step, threshold, actions);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}
