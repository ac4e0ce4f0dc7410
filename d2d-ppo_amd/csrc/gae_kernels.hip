// GAE / discounted-return scan and column normalisation for gfx950.
//
// Replaces compute_gae + discount_rewards (/root/reference/algorithms/ippo.py:92-116,
// identical to algorithms/d2d_ppo.py:100-124).  The reference builds the
// sequence with list.insert(0, .) (O(T^2)) in float64 and normalises per
// column (adv: numpy std ddof=0, returns: torch std ddof=1; each gated on ALL
// columns having std > 0, quirk Q2).
//
// Layout [T][E][cols] or [T][cols][E] (`_tce` entry points: the policy kernel's
// value layout, and the update kernels' preferred per-sample layout): for a fixed
// t, the (env, column) pairs are contiguous, so one thread per (env, column)
// walking t backwards reads and writes fully coalesced rows; the recursion state
// (gae, R) lives in f64 registers.
// Normalisation = deterministic two-level column sums (block partials in a
// fixed order), so results do not depend on atomics ordering and the stats can
// be all-reduced across ranks between the passes.
#include <cmath>

#include "common.h"

namespace d2d {

__global__ __launch_bounds__(256) void gae_scan_kernel(int T, int E, int cols, int rcols, const float* __restrict__ rew,
                                                       const float* __restrict__ val, const uint8_t* __restrict__ done,
                                                       double gamma, double lam, int last_shard, float* __restrict__ adv,
                                                       float* __restrict__ ret, int tce) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t width = (int64_t)E * cols;
  if (i >= width) return;
  // [T][E][cols]: i = e * cols + c; [T][cols][E] (tce): i = c * E + e -- coalesced either way
  const int e = tce ? (int)(i % E) : (int)(i / cols);
  const bool global_last = last_shard && (e == E - 1);
  double gae = 0.0, R = 0.0, v_next = 0.0;
  // step t's inputs are loaded one step ahead (t + 1's recursion hides their latency)
  auto r_at = [&](int t) { return rew[rcols == 1 ? (int64_t)t * E + e : (int64_t)t * width + i]; };
  float rn = T > 0 ? r_at(T - 1) : 0.f, vn = T > 0 ? val[(int64_t)(T - 1) * width + i] : 0.f;
  uint8_t dn = T > 0 ? done[T - 1] : 0;
  for (int t = T - 1; t >= 0; --t) {
    const int64_t o = (int64_t)t * width + i;
    const double r = (double)rn;
    const double v = (double)vn;
    const double nd = dn ? 0.0 : 1.0;
    if (t > 0) {
      rn = r_at(t - 1);
      vn = val[o - width];
      dn = done[t - 1];
    }
    // discount_rewards: R = r + R * gamma * (1 - done)   (ippo.py:107-109)
    R = r + R * gamma * nd;
    double a;
    if (t == T - 1 && global_last) {
      a = r - v;  // adv = [rewards[-1] - values[-1]]  (ippo.py:94)
      gae = 0.0;  // the reference's running gae starts at 0 for step T-2 (ippo.py:93)
    } else {
      // delta = r + gamma V' (1-done) - V ; gae = delta + gamma lam (1-done) gae ; adv = gae + V (96-98)
      const double delta = r + gamma * v_next * nd - v;
      gae = delta + gamma * lam * nd * gae;
      a = gae + v;
    }
    adv[o] = (float)a;
    ret[o] = (float)R;
    v_next = v;
  }
}

// ---------------------------------------------------------------- scan + normalisation moments
// The scan of gae_scan_kernel with the column statistics of both outputs fused into it: every
// thread owns one (env, column) sequence of T elements, so while it writes adv / ret it also
// accumulates their (shifted) sums in double; the block combines its threads' moments per column
// with Chan's pairwise formula in a fixed tree order and writes one partial per (column, block);
// gae_moments_reduce_kernel combines the partials of a column in a fixed order.  Result per column:
// n, sum and M2 = sum of squared deviations from the column mean -- what two_pass_column_stats
// (d2dhip/gae.py) needs, without a second or third pass over adv / ret.
//
// Block = EPB envs x CT column lanes (EPB * CT = 256), lane tid = el * CT + cl:
//   layout 1 ([T][cols][E]): CT = 1, block (bx, by) = envs [256 bx, 256 bx + 256) of column by;
//   layout 0 ([T][E][cols]): CT = min(pow2(cols), 256), block (bx, by) = envs [EPB bx, ...) x columns
//   [CT by, CT by + CT).  Consecutive lanes read consecutive addresses in both layouts.
struct Mom {
  double n, mean, m2;
};

__device__ __forceinline__ Mom mom_combine(Mom a, Mom b) {  // Chan et al., pairwise update
  if (b.n == 0.0) return a;
  if (a.n == 0.0) return b;
  const double n = a.n + b.n;
  const double d = b.mean - a.mean;
  Mom r;
  r.n = n;
  r.mean = a.mean + d * (b.n / n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / n);
  return r;
}

// per-thread moments of one sequence: sums shifted by its first element (exact 0 for a constant column)
struct SeqMom {
  double k, s1, s2;
  __device__ __forceinline__ void add(double x, bool first) {
    if (first) k = x;
    const double d = x - k;
    s1 += d;
    s2 += d * d;
  }
  __device__ __forceinline__ Mom get(int n) const {
    Mom m;
    m.n = (double)n;
    m.mean = n ? k + s1 / (double)n : 0.0;
    m.m2 = n ? s2 - s1 * (s1 / (double)n) : 0.0;
    if (m.m2 < 0.0) m.m2 = 0.0;
    return m;
  }
};

//
// MODE (ABI 9): 0 = write adv / ret and accumulate the moments; 1 = moments only (no writes: the first
// of two scans when the outputs are normalised); 2 = write the NORMALISED outputs, no moments (the
// second scan, after the statistics of the first have been finalised and, across ranks, all-reduced).
// Recomputing the recursion costs a few f64 FMAs per element; it saves the separate normalisation
// pass (8 B read + 8 B written per element) and the first pass's 8 B of writes: 16 B per element over
// the two scans instead of 28 B for scan + normalise.  The recursion, the fp32 roundings and the
// normalisation expression (nrm) are those of the scan and of normalize_pair_kernel, so every output
// is bitwise the same as scan + normalise.
struct NormArgs {
  const double *mean0, *scale0, *mean1, *scale1;  // adv (0) and ret (1); NULL mean = written raw
  const int32_t *gate0, *gate1;
};
__device__ __forceinline__ float nrm(float v, double m, double sc) { return (float)(((double)v - m) * sc); }

template <int TCE, int MODE>
__global__ __launch_bounds__(256) void gae_scan_moments_kernel(int T, int E, int cols, int rcols, int ct,
                                                               const float* __restrict__ rew,
                                                               const float* __restrict__ val,
                                                               const uint8_t* __restrict__ done, double gamma,
                                                               double lam, int last_shard, float* __restrict__ adv,
                                                               float* __restrict__ ret, double* __restrict__ partial,
                                                               NormArgs na) {
  __shared__ Mom red[MODE == 2 ? 1 : 2][MODE == 2 ? 1 : 256];
  const int tid = threadIdx.x;
  const int epb = 256 / ct;
  const int el = tid / ct, cl = tid - (tid / ct) * ct;
  const int e = (int)blockIdx.x * epb + el;
  const int c = TCE ? (int)blockIdx.y : (int)blockIdx.y * ct + cl;
  const bool active = e < E && c < cols;
  const int64_t width = (int64_t)E * cols;
  const int64_t i = TCE ? (int64_t)c * E + e : (int64_t)e * cols + c;
  SeqMom ma{0.0, 0.0, 0.0}, mr{0.0, 0.0, 0.0};
  // MODE 2: this thread's column statistics (gate off or no statistics = identity)
  double m0 = 0.0, s0 = 1.0, m1 = 0.0, s1 = 1.0;
  bool n0 = false, n1 = false;
  if (MODE == 2 && active) {
    n0 = na.mean0 && *na.gate0;
    n1 = na.mean1 && *na.gate1;
    if (n0) { m0 = na.mean0[c]; s0 = na.scale0[c]; }
    if (n1) { m1 = na.mean1[c]; s1 = na.scale1[c]; }
  }
  if (active) {
    const bool global_last = last_shard && (e == E - 1);
    // per-column rewards share the values' layout; broadcast rewards are [T][E]
    const int64_t r_off = rcols == 1 ? (int64_t)e : i;
    const int64_t r_stride = rcols == 1 ? (int64_t)E : width;
    // inputs of the next U steps are loaded while the current U are computed (U loads in flight)
    constexpr int U = 4;
    float rb[U], vb[U];
    uint8_t db[U];
    auto load = [&](int t0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = t0 - u;
        if (t >= 0) {
          rb[u] = rew[(int64_t)t * r_stride + r_off];
          vb[u] = val[(int64_t)t * width + i];
          db[u] = done[t];
        }
      }
    };
    double gae = 0.0, R = 0.0, v_next = 0.0;
    load(T - 1);
    for (int t0 = T - 1; t0 >= 0; t0 -= U) {
      float rc[U], vc[U];
      uint8_t dc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        rc[u] = rb[u];
        vc[u] = vb[u];
        dc[u] = db[u];
      }
      if (t0 - U >= 0) load(t0 - U);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = t0 - u;
        if (t < 0) break;
        const double r = (double)rc[u], v = (double)vc[u];
        const double nd = dc[u] ? 0.0 : 1.0;
        R = r + R * gamma * nd;  // discount_rewards (ippo.py:107-109)
        double a;
        if (t == T - 1 && global_last) {
          a = r - v;  // adv = [rewards[-1] - values[-1]]  (ippo.py:94)
          gae = 0.0;
        } else {
          const double delta = r + gamma * v_next * nd - v;  // (ippo.py:96-98)
          gae = delta + gamma * lam * nd * gae;
          a = gae + v;
        }
        v_next = v;
        const float af = (float)a, rf = (float)R;
        const int64_t o = (int64_t)t * width + i;
        if constexpr (MODE == 0) {
          adv[o] = af;
          ret[o] = rf;
        } else if constexpr (MODE == 2) {
          adv[o] = n0 ? nrm(af, m0, s0) : af;
          ret[o] = n1 ? nrm(rf, m1, s1) : rf;
        }
        if constexpr (MODE != 2) {
          // the statistics are those of the stored fp32 values, as a separate pass over adv / ret sees them
          ma.add((double)af, t == T - 1);
          mr.add((double)rf, t == T - 1);
        }
      }
    }
  }
  if constexpr (MODE == 2) return;
  red[0][tid] = ma.get(active ? T : 0);
  red[1][tid] = mr.get(active ? T : 0);
  __syncthreads();
  for (int s = epb >> 1; s >= 1; s >>= 1) {  // fixed-order tree over the block's envs, per column lane
    if (el < s) {
      red[0][tid] = mom_combine(red[0][tid], red[0][tid + s * ct]);
      red[1][tid] = mom_combine(red[1][tid], red[1][tid + s * ct]);
    }
    __syncthreads();
  }
  if (el == 0 && c < cols) {
    // partial [cols][nbx][2][3]
    double* p = partial + ((int64_t)c * gridDim.x + blockIdx.x) * 6;
    p[0] = red[0][tid].n;
    p[1] = red[0][tid].mean;
    p[2] = red[0][tid].m2;
    p[3] = red[1][tid].n;
    p[4] = red[1][tid].mean;
    p[5] = red[1][tid].m2;
  }
}

// one block per column: combine its nb partials in a fixed order -> moments [2][3][cols] (n, sum, M2)
__global__ __launch_bounds__(256) void gae_moments_reduce_kernel(int nb, int cols, const double* __restrict__ partial,
                                                                 double* __restrict__ moments) {
  __shared__ Mom red[2][256];
  const int c = blockIdx.x, tid = threadIdx.x;
  Mom a{0.0, 0.0, 0.0}, r{0.0, 0.0, 0.0};
  for (int b = tid; b < nb; b += 256) {
    const double* p = partial + ((int64_t)c * nb + b) * 6;
    a = mom_combine(a, Mom{p[0], p[1], p[2]});
    r = mom_combine(r, Mom{p[3], p[4], p[5]});
  }
  red[0][tid] = a;
  red[1][tid] = r;
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if (tid < s) {
      red[0][tid] = mom_combine(red[0][tid], red[0][tid + s]);
      red[1][tid] = mom_combine(red[1][tid], red[1][tid + s]);
    }
    __syncthreads();
  }
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const Mom m = red[k][0];
      moments[(3 * k + 0) * cols + c] = m.n;
      moments[(3 * k + 1) * cols + c] = m.n * m.mean;
      moments[(3 * k + 2) * cols + c] = m.m2;
    }
  }
}

// x_k = gate_k ? (x_k - mean_k) * scale_k : x_k for both outputs in one pass (x1 may be null).
// No integer division per element (a 64-bit divide is a ~100-instruction software sequence):
//   [T][cols][E] (TCE): block (bx, row = t * cols + c) streams float4s of one row -- the column and its
//                       mean / scale are wave-uniform scalars, loaded once per block;
//   [T][E][cols]:       flat float4 stream, column of element j = j mod cols in 32-bit arithmetic.
template <bool TCE>
__global__ __launch_bounds__(256) void normalize_pair_kernel(int64_t n, int rows, int E, int cols,
                                                             float* __restrict__ x0, const double* __restrict__ mean0,
                                                             const double* __restrict__ scale0,
                                                             const int32_t* __restrict__ gate0, float* __restrict__ x1,
                                                             const double* __restrict__ mean1,
                                                             const double* __restrict__ scale1,
                                                             const int32_t* __restrict__ gate1) {
  const bool g0 = x0 && *gate0, g1 = x1 && *gate1;
  if (!g0 && !g1) return;
  if constexpr (TCE) {
    for (int row = blockIdx.y; row < rows; row += gridDim.y) {
      const int c = row % cols;
      const double m0 = g0 ? mean0[c] : 0.0, s0 = g0 ? scale0[c] : 1.0;
      const double m1 = g1 ? mean1[c] : 0.0, s1 = g1 ? scale1[c] : 1.0;
      const int64_t base = (int64_t)row * E;
      if ((E & 3) == 0) {  // rows of whole float4s (16-byte aligned: x 16-byte aligned, E % 4 == 0)
        const int E4 = E >> 2;
        for (int q = blockIdx.x * 256 + threadIdx.x; q < E4; q += gridDim.x * 256) {
          if (g0) {
            float4* p = reinterpret_cast<float4*>(x0 + base) + q;
            float4 v = *p;
            v = make_float4(nrm(v.x, m0, s0), nrm(v.y, m0, s0), nrm(v.z, m0, s0), nrm(v.w, m0, s0));
            *p = v;
          }
          if (g1) {
            float4* p = reinterpret_cast<float4*>(x1 + base) + q;
            float4 v = *p;
            v = make_float4(nrm(v.x, m1, s1), nrm(v.y, m1, s1), nrm(v.z, m1, s1), nrm(v.w, m1, s1));
            *p = v;
          }
        }
      } else {
        for (int e = blockIdx.x * 256 + threadIdx.x; e < E; e += gridDim.x * 256) {
          if (g0) x0[base + e] = nrm(x0[base + e], m0, s0);
          if (g1) x1[base + e] = nrm(x1[base + e], m1, s1);
        }
      }
    }
  } else {
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const bool small = n < ((int64_t)1 << 31);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
      const int64_t j = q << 2;
      const int c0 = cols == 1 ? 0 : small ? (int)((uint32_t)j % (uint32_t)cols) : (int)(j % cols);
      int cc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int cu = c0 + u;
        cc[u] = cols == 1 ? 0 : cu < cols ? cu : cu % cols;
      }
      if (g0) {
        float4* p = reinterpret_cast<float4*>(x0) + q;
        float4 v = *p;
        v = make_float4(nrm(v.x, mean0[cc[0]], scale0[cc[0]]), nrm(v.y, mean0[cc[1]], scale0[cc[1]]),
                        nrm(v.z, mean0[cc[2]], scale0[cc[2]]), nrm(v.w, mean0[cc[3]], scale0[cc[3]]));
        *p = v;
      }
      if (g1) {
        float4* p = reinterpret_cast<float4*>(x1) + q;
        float4 v = *p;
        v = make_float4(nrm(v.x, mean1[cc[0]], scale1[cc[0]]), nrm(v.y, mean1[cc[1]], scale1[cc[1]]),
                        nrm(v.z, mean1[cc[2]], scale1[cc[2]]), nrm(v.w, mean1[cc[3]], scale1[cc[3]]));
        *p = v;
      }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {  // tail
      const int64_t j = (n4 << 2) + threadIdx.x;
      const int c = (int)(j % cols);
      if (g0) x0[j] = nrm(x0[j], mean0[c], scale0[c]);
      if (g1) x1[j] = nrm(x1[j], mean1[c], scale1[c]);
    }
  }
}

constexpr int kStatRowBlocks = 1024;

// partial[y][c] = sum over this block's rows of (x - center)^p
__global__ __launch_bounds__(256) void colstats_partial_kernel(int64_t rows, int cols, int ct, const float* __restrict__ x,
                                                               const double* __restrict__ center,
                                                               double* __restrict__ partial) {
  __shared__ double acc[256];
  const int cl = threadIdx.x % ct, rl = threadIdx.x / ct, rlanes = blockDim.x / ct;
  const int c = blockIdx.x * ct + cl;
  double s = 0.0;
  if (c < cols) {
    const double m = center ? center[c] : 0.0;
    for (int64_t r = (int64_t)blockIdx.y * rlanes + rl; r < rows; r += (int64_t)gridDim.y * rlanes) {
      const double v = (double)x[r * cols + c] - m;
      s += center ? v * v : v;
    }
  }
  acc[threadIdx.x] = s;
  __syncthreads();
  if (rl == 0 && c < cols) {
    double t = 0.0;
    for (int j = 0; j < rlanes; ++j) t += acc[j * ct + cl];
    partial[(int64_t)blockIdx.y * cols + c] = t;
  }
}

// [T][cols][E] layout: block (c, b) sums column c over slots t = b, b + nb, ... (fixed order)
__global__ __launch_bounds__(256) void colstats_tce_partial_kernel(int T, int cols, int E, const float* __restrict__ x,
                                                                   const double* __restrict__ center,
                                                                   double* __restrict__ partial) {
  __shared__ double acc[256];
  const int c = blockIdx.x, b = blockIdx.y, nb = gridDim.y;
  const double m = center ? center[c] : 0.0;
  double s = 0.0;
  for (int t = b; t < T; t += nb) {
    const float* row = x + ((int64_t)t * cols + c) * E;
    for (int e = threadIdx.x; e < E; e += blockDim.x) {
      const double v = (double)row[e] - m;
      s += center ? v * v : v;
    }
  }
  acc[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int j = 0; j < (int)blockDim.x; ++j) tot += acc[j];
    partial[(int64_t)b * cols + c] = tot;
  }
}

__global__ void colstats_reduce_kernel(int nb, int cols, const double* __restrict__ partial, double* __restrict__ out) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < cols; c += gridDim.x * blockDim.x) {
    double t = 0.0;
    for (int y = 0; y < nb; ++y) t += partial[(int64_t)y * cols + c];
    out[c] = t;
  }
}

__global__ __launch_bounds__(256) void colstats_finalize_kernel(int cols, const double* sum, const double* m2, double n,
                                                                int ddof, double* mean, double* scale, int32_t* gate) {
  int ok = 1;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) {
    mean[c] = sum[c] / n;
    if (m2) {
      const double sd = sqrt(m2[c] / (n - (double)ddof));
      ok &= sd > 0.0;
      scale[c] = 1.0 / sd;
    }
  }
  if (m2) {
    ok = __syncthreads_and(ok);
    if (threadIdx.x == 0) *gate = ok;
  }
}

__global__ __launch_bounds__(256) void normalize_kernel(int64_t n, int cols, float* __restrict__ x,
                                                        const double* __restrict__ mean,
                                                        const double* __restrict__ scale, const int32_t* __restrict__ gate,
                                                        int inner) {
  if (!*gate) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = inner > 0 ? (int)((i / inner) % cols) : (int)(i % cols);
    x[i] = (float)(((double)x[i] - mean[c]) * scale[c]);
  }
}

}  // namespace d2d

using namespace d2d;

static int gae_scan(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards, const float* values,
                    const uint8_t* dones, double gamma, double lam, int32_t last_shard, float* adv, float* ret, void* stream,
                    int tce) {
  if (T < 0 || E < 0 || cols < 1 || (reward_cols != 1 && reward_cols != cols) || !rewards || !values || !dones || !adv || !ret) {
    d2d_set_error("d2d_gae_scan: bad arguments");
    return D2D_EINVAL;
  }
  const int64_t width = (int64_t)E * cols;
  if (T == 0 || width == 0) return D2D_OK;
  hipLaunchKernelGGL(gae_scan_kernel, dim3((unsigned)((width + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), T, E, cols, reward_cols, rewards, values, dones, gamma, lam, last_shard,
                     adv, ret, tce);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

// ---------------------------------------------------------------- D2D-PPO agent chain
// M[sigma_j][b] = adv[b] * r_sigma_0[b] * ... * r_sigma_{j-1}[b], multiplied left to right in fp32
// like the reference's sequential loop over the permuted agents (d2d_ppo.py:405-433), with
// r_k[b] = exp(logp_new[k][b] - logp_old[k][b]) of the epoch-start policy.  One thread per sample
// b = t*E + e; logp_old is read in the rollout's [T][N][E] layout (no agent-major copy).
__global__ __launch_bounds__(256) void happo_chain_kernel(int N, int T, int E, const float* __restrict__ adv,
                                                          const float* __restrict__ logp_new,
                                                          const float* __restrict__ logp_old,
                                                          const int32_t* __restrict__ perm, float* __restrict__ M) {
  const int64_t B = (int64_t)T * E;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int t = (int)(b / E), e = (int)(b - (int64_t)t * E);
  float cur = adv[b];
  for (int j = 0; j < N; ++j) {
    const int k = perm[j];
    M[(int64_t)k * B + b] = cur;
    if (j + 1 < N) cur = expf(logp_new[(int64_t)k * B + b] - logp_old[((int64_t)t * N + k) * E + e]) * cur;
  }
}

extern "C" int d2d_happo_chain(int32_t n_agents, int32_t T, int32_t E, const float* adv, const float* logp_new,
                               const float* logp_old, const int32_t* perm, float* M, void* stream) {
  if (n_agents < 1 || T < 0 || E < 0 || !adv || !logp_new || !logp_old || !perm || !M) {
    d2d_set_error("d2d_happo_chain: bad arguments");
    return D2D_EINVAL;
  }
  const int64_t B = (int64_t)T * E;
  if (B == 0) return D2D_OK;
  hipLaunchKernelGGL(happo_chain_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), n_agents, T, E, adv, logp_new, logp_old, perm, M);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_gae_scan(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards, const float* values,
                            const uint8_t* dones, double gamma, double lam, int32_t last_shard, float* adv, float* ret,
                            void* stream) {
  return gae_scan(T, E, cols, reward_cols, rewards, values, dones, gamma, lam, last_shard, adv, ret, stream, 0);
}

extern "C" int d2d_gae_scan_tce(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards,
                                const float* values, const uint8_t* dones, double gamma, double lam, int32_t last_shard,
                                float* adv, float* ret, void* stream) {
  return gae_scan(T, E, cols, reward_cols, rewards, values, dones, gamma, lam, last_shard, adv, ret, stream, 1);
}

static void moments_grid(int32_t E, int32_t cols, int32_t layout, int* ct, dim3* grid) {
  int c = 1;
  if (!layout)
    while (c < cols && c < 256) c <<= 1;
  const int epb = 256 / c;
  *ct = c;
  *grid = dim3((unsigned)((E + epb - 1) / epb), (unsigned)(layout ? cols : (cols + c - 1) / c));
}

extern "C" int64_t d2d_gae_moments_workspace(int32_t E, int32_t cols, int32_t layout) {
  if (E < 1 || cols < 1) return 6;
  int ct;
  dim3 g;
  moments_grid(E, cols, layout, &ct, &g);
  return (int64_t)cols * g.x * 6;
}

template <int MODE>
static void launch_scan(int32_t layout, dim3 grid, hipStream_t s, int T, int E, int cols, int rcols, int ct,
                        const float* rew, const float* val, const uint8_t* done, double gamma, double lam,
                        int last_shard, float* adv, float* ret, double* partial, NormArgs na) {
  if (layout)
    hipLaunchKernelGGL((gae_scan_moments_kernel<1, MODE>), grid, dim3(256), 0, s, T, E, cols, rcols, ct, rew, val, done,
                       gamma, lam, last_shard, adv, ret, partial, na);
  else
    hipLaunchKernelGGL((gae_scan_moments_kernel<0, MODE>), grid, dim3(256), 0, s, T, E, cols, rcols, ct, rew, val, done,
                       gamma, lam, last_shard, adv, ret, partial, na);
}

extern "C" int d2d_gae_scan_moments(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards,
                                    const float* values, const uint8_t* dones, double gamma, double lam,
                                    int32_t last_shard, int32_t layout, float* adv, float* ret, double* moments,
                                    double* workspace, int64_t workspace_len, void* stream) {
  // adv == ret == NULL: moments only (ABI 9)
  if (T < 0 || E < 0 || cols < 1 || (reward_cols != 1 && reward_cols != cols) || (layout != 0 && layout != 1) ||
      !rewards || !values || !dones || (!adv != !ret) || !moments || !workspace ||
      workspace_len < d2d_gae_moments_workspace(E, cols, layout)) {
    d2d_set_error("d2d_gae_scan_moments: bad arguments");
    return D2D_EINVAL;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (T == 0 || E == 0) {
    D2D_CHECK_HIP(hipMemsetAsync(moments, 0, sizeof(double) * 6 * cols, s));
    return D2D_OK;
  }
  int ct;
  dim3 grid;
  moments_grid(E, cols, layout, &ct, &grid);
  const NormArgs na{};
  if (adv)
    launch_scan<0>(layout, grid, s, T, E, cols, reward_cols, ct, rewards, values, dones, gamma, lam, last_shard, adv, ret,
                   workspace, na);
  else
    launch_scan<1>(layout, grid, s, T, E, cols, reward_cols, ct, rewards, values, dones, gamma, lam, last_shard, adv, ret,
                   workspace, na);
  D2D_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(gae_moments_reduce_kernel, dim3((unsigned)cols), dim3(256), 0, s, (int)grid.x, cols, workspace,
                     moments);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_gae_scan_normalized(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards,
                                       const float* values, const uint8_t* dones, double gamma, double lam,
                                       int32_t last_shard, int32_t layout, float* adv, const double* mean0,
                                       const double* scale0, const int32_t* gate0, float* ret, const double* mean1,
                                       const double* scale1, const int32_t* gate1, void* stream) {
  if (T < 0 || E < 0 || cols < 1 || (reward_cols != 1 && reward_cols != cols) || (layout != 0 && layout != 1) ||
      !rewards || !values || !dones || !adv || !ret || (mean0 && (!scale0 || !gate0)) ||
      (mean1 && (!scale1 || !gate1))) {
    d2d_set_error("d2d_gae_scan_normalized: bad arguments");
    return D2D_EINVAL;
  }
  if (T == 0 || E == 0) return D2D_OK;
  int ct;
  dim3 grid;
  moments_grid(E, cols, layout, &ct, &grid);
  const NormArgs na{mean0, scale0, mean1, scale1, gate0, gate1};
  launch_scan<2>(layout, grid, reinterpret_cast<hipStream_t>(stream), T, E, cols, reward_cols, ct, rewards, values, dones,
                 gamma, lam, last_shard, adv, ret, nullptr, na);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_normalize_pair(int32_t T, int32_t E, int32_t cols, int32_t layout, float* x0, const double* mean0,
                                  const double* scale0, const int32_t* gate0, float* x1, const double* mean1,
                                  const double* scale1, const int32_t* gate1, void* stream) {
  if (T < 0 || E < 0 || cols < 1 || (layout != 0 && layout != 1) || (!x0 && !x1) ||
      (x0 && (!mean0 || !scale0 || !gate0)) || (x1 && (!mean1 || !scale1 || !gate1)) ||
      (reinterpret_cast<uintptr_t>(x0) & 15) || (reinterpret_cast<uintptr_t>(x1) & 15)) {
    d2d_set_error("d2d_normalize_pair: bad arguments (x0 / x1 16-byte aligned)");
    return D2D_EINVAL;
  }
  const int64_t n = (int64_t)T * E * cols;
  if (n == 0) return D2D_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (layout) {
    // a block streams 4 float4s per lane of one row; rows beyond gridDim.y loop
    const int64_t rows = (int64_t)T * cols;
    if (rows > 0x7FFFFFFF) { d2d_set_error("d2d_normalize_pair: T * cols too large"); return D2D_EINVAL; }
    const int per = (E & 3) == 0 ? 4 * 256 * 4 : 256 * 4;
    const unsigned gx = (unsigned)((E + per - 1) / per);
    const unsigned gy = (unsigned)(rows < 65535 ? rows : 65535);
    hipLaunchKernelGGL(normalize_pair_kernel<true>, dim3(gx, gy), dim3(256), 0, s, n, (int)rows, E, cols, x0, mean0,
                       scale0, gate0, x1, mean1, scale1, gate1);
  } else {
    int64_t grid = ((n >> 2) + 255) / 256;
    grid = grid < 1 ? 1 : grid > 16384 ? 16384 : grid;
    hipLaunchKernelGGL(normalize_pair_kernel<false>, dim3((unsigned)grid), dim3(256), 0, s, n, 0, E, cols, x0, mean0,
                       scale0, gate0, x1, mean1, scale1, gate1);
  }
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int64_t d2d_colstats_workspace(int64_t rows, int32_t cols) {
  (void)rows;
  return (int64_t)kStatRowBlocks * cols;
}

extern "C" int d2d_colstats(int64_t rows, int32_t cols, const float* x, const double* center, double* partial,
                            double* out, void* stream) {
  if (rows < 0 || cols < 1 || !x || !partial || !out) {
    d2d_set_error("d2d_colstats: bad arguments");
    return D2D_EINVAL;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int ct = 1;
  while (ct < cols && ct < 64) ct <<= 1;
  const int rlanes = 256 / ct;
  int64_t nb = (rows + (int64_t)rlanes * 16 - 1) / ((int64_t)rlanes * 16);
  nb = nb < 1 ? 1 : (nb > kStatRowBlocks ? kStatRowBlocks : nb);
  hipLaunchKernelGGL(colstats_partial_kernel, dim3((cols + ct - 1) / ct, (unsigned)nb), dim3(256), 0, s, rows, cols, ct,
                     x, center, partial);
  D2D_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(colstats_reduce_kernel, dim3((cols + 255) / 256), dim3(256), 0, s, (int)nb, cols, partial, out);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_colstats_tce(int32_t T, int32_t cols, int32_t E, const float* x, const double* center, double* partial,
                                double* out, void* stream) {
  if (T < 0 || E < 0 || cols < 1 || !x || !partial || !out) {
    d2d_set_error("d2d_colstats_tce: bad arguments");
    return D2D_EINVAL;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = T < 1 ? 1 : (T > kStatRowBlocks ? kStatRowBlocks : T);
  hipLaunchKernelGGL(colstats_tce_partial_kernel, dim3(cols, nb), dim3(256), 0, s, T, cols, E, x, center, partial);
  D2D_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(colstats_reduce_kernel, dim3((cols + 255) / 256), dim3(256), 0, s, nb, cols, partial, out);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_colstats_finalize(int32_t cols, const double* sum, const double* m2, double n, int32_t ddof,
                                     double* mean, double* scale, int32_t* gate, void* stream) {
  if (cols < 1 || !sum || !mean || (m2 && (!scale || !gate))) {
    d2d_set_error("d2d_colstats_finalize: bad arguments");
    return D2D_EINVAL;
  }
  hipLaunchKernelGGL(colstats_finalize_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), cols, sum,
                     m2, n, ddof, mean, scale, gate);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

static int normalize(int64_t n, int32_t cols, int32_t inner, float* x, const double* mean, const double* scale,
                     const int32_t* gate, void* stream) {
  if (n == 0) return D2D_OK;
  int64_t grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(normalize_kernel, dim3((unsigned)grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), n, cols,
                     x, mean, scale, gate, inner);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_normalize_columns(int64_t rows, int32_t cols, float* x, const double* mean, const double* scale,
                                     const int32_t* gate, void* stream) {
  if (rows < 0 || cols < 1 || !x || !mean || !scale || !gate) {
    d2d_set_error("d2d_normalize_columns: bad arguments");
    return D2D_EINVAL;
  }
  return normalize(rows * cols, cols, 0, x, mean, scale, gate, stream);
}

extern "C" int d2d_normalize_columns_tce(int32_t T, int32_t cols, int32_t E, float* x, const double* mean,
                                         const double* scale, const int32_t* gate, void* stream) {
  if (T < 0 || E < 0 || cols < 1 || !x || !mean || !scale || !gate) {
    d2d_set_error("d2d_normalize_columns_tce: bad arguments");
    return D2D_EINVAL;
  }
  return normalize((int64_t)T * cols * E, cols, E, x, mean, scale, gate, stream);
}

// ---------------------------------------------------------------------------------------------
// fp32 -> bf16 with an exactness check, one pass (the D2D central critic's bf16 GEMM operand,
// algorithms/d2d_ppo.py _critic_split_forward): out = the high 16 bits of every x; *inexact = 1 if
// any x has nonzero low bits (then the caller keeps the fp32 path).  One read of x and one write of
// out instead of torch's conversion + a chunked compare / all() over a second fp32 copy.  The flag
// is a plain (benign-race) store of 1 by the lanes that found one: no atomics.
__global__ __launch_bounds__(256) void bf16_exact_kernel(int64_t n, const float* __restrict__ x,
                                                         uint16_t* __restrict__ out, int32_t* __restrict__ inexact) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint32_t low = 0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += stride) {
    const uint4 v = reinterpret_cast<const uint4*>(x)[q];
    low |= (v.x | v.y | v.z | v.w) & 0xFFFFu;
    reinterpret_cast<uint2*>(out)[q] = make_uint2((v.x >> 16) | (v.y & 0xFFFF0000u), (v.z >> 16) | (v.w & 0xFFFF0000u));
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {  // tail
    const uint32_t v = __float_as_uint(x[(n4 << 2) + threadIdx.x]);
    low |= v & 0xFFFFu;
    out[(n4 << 2) + threadIdx.x] = (uint16_t)(v >> 16);
  }
  if (low) inexact[0] = 1;
}

// The same conversion + check straight from the rollout's slot-major state buffer x [T][E][ld] into the
// env-major operand out [E*T][S] (out row e*T + t <- x row t*E + e, its first S floats): the central
// critic no longer needs an fp32 env-major copy of the states first.  One workgroup per output row.
// out rows are out_ld wide: columns [S, out_ld) are written as zeros (a GEMM-aligned operand for state
// widths such as configs[1]'s 117)
template <bool VEC>
__global__ __launch_bounds__(256) void states_bf16_kernel(int T, int E, int S, int64_t ld, const float* __restrict__ x,
                                                          uint16_t* __restrict__ out, int64_t out_ld,
                                                          int32_t* __restrict__ inexact) {
  const int64_t rows = (int64_t)T * E;
  uint32_t low = 0;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const int64_t e = r / T, t = r - e * T;
    const float* xr = x + (t * E + e) * ld;
    uint16_t* orow = out + r * out_ld;
    if constexpr (VEC) {  // S % 4 == 0, ld % 4 == 0, out_ld % 4 == 0, 16-byte aligned x
      for (int q = threadIdx.x; q < (S >> 2); q += blockDim.x) {
        const uint4 v = reinterpret_cast<const uint4*>(xr)[q];
        low |= (v.x | v.y | v.z | v.w) & 0xFFFFu;
        reinterpret_cast<uint2*>(orow)[q] = make_uint2((v.x >> 16) | (v.y & 0xFFFF0000u), (v.z >> 16) | (v.w & 0xFFFF0000u));
      }
    } else {
      for (int q = threadIdx.x; q < S; q += blockDim.x) {
        const uint32_t v = __float_as_uint(xr[q]);
        low |= v & 0xFFFFu;
        orow[q] = (uint16_t)(v >> 16);
      }
    }
    for (int64_t q = S + threadIdx.x; q < out_ld; q += blockDim.x) orow[q] = 0;
  }
  if (low) inexact[0] = 1;
}

extern "C" int d2d_states_to_bf16_padded(int32_t T, int32_t E, int32_t S, int64_t ld, const float* x, uint16_t* out,
                                         int64_t out_ld, int32_t* inexact, void* stream) {
  if (T < 0 || E < 0 || S < 1 || ld < S || out_ld < S || !inexact || ((int64_t)T * E > 0 && (!x || !out))) {
    d2d_set_error("d2d_states_to_bf16: bad arguments");
    return D2D_EINVAL;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  D2D_CHECK_HIP(hipMemsetAsync(inexact, 0, sizeof(int32_t), s));
  const int64_t rows = (int64_t)T * E;
  if (rows == 0) return D2D_OK;
  const unsigned grid = (unsigned)(rows < 16384 ? rows : 16384);
  const bool vec = (S % 4 == 0) && (ld % 4 == 0) && (out_ld % 4 == 0) && !(reinterpret_cast<uintptr_t>(x) & 15) &&
                   !(reinterpret_cast<uintptr_t>(out) & 7);
  if (vec)
    hipLaunchKernelGGL(states_bf16_kernel<true>, dim3(grid), dim3(256), 0, s, T, E, S, ld, x, out, out_ld, inexact);
  else
    hipLaunchKernelGGL(states_bf16_kernel<false>, dim3(grid), dim3(256), 0, s, T, E, S, ld, x, out, out_ld, inexact);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_states_to_bf16_exact(int32_t T, int32_t E, int32_t S, int64_t ld, const float* x, uint16_t* out,
                                        int32_t* inexact, void* stream) {
  return d2d_states_to_bf16_padded(T, E, S, ld, x, out, S, inexact, stream);
}

extern "C" int d2d_f32_to_bf16_exact(int64_t n, const float* x, uint16_t* out, int32_t* inexact, void* stream) {
  if (n < 0 || (n > 0 && (!x || !out)) || !inexact) {
    d2d_set_error("d2d_f32_to_bf16_exact: bad arguments");
    return D2D_EINVAL;
  }
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(out) & 7)) {
    d2d_set_error("d2d_f32_to_bf16_exact: x must be 16-byte and out 8-byte aligned");
    return D2D_EINVAL;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  D2D_CHECK_HIP(hipMemsetAsync(inexact, 0, sizeof(int32_t), s));
  if (n == 0) return D2D_OK;
  int64_t grid = ((n >> 2) + 255) / 256;
  grid = grid < 1 ? 1 : grid > 16384 ? 16384 : grid;
  hipLaunchKernelGGL(bf16_exact_kernel, dim3((unsigned)grid), dim3(256), 0, s, n, x, out, inexact);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

// ---------------------------------------------------------------------------------------------
// D2D central critic, backward glue (algorithms/d2d_ppo.py _critic_split_backward; the reference's
// value_loss.backward() through Value = linear2(relu(linear1(state))), d2d_ppo.py:95-98, 208-216):
//   dpre[h][b] = pre[h][b] > 0 ? w2[h] * dv[b] : 0                 (torch.where(pre > 0, w2^T dv, 0))
//   dhm[h][b] = RNE_bf16(dpre), dhm[H + h][b] = RNE_bf16(dpre - dhm[h][b])   (the dW1 GEMM's A operand)
//   partial[g][h] = sum_b dpre (db1),  partial[g][H + h] = sum_b relu(pre) dv (dW2)   over block g's samples
// One pass over pre instead of ~8 torch elementwise kernels over [H][B].  Block g owns samples
// [g chunk, (g + 1) chunk); its sums are reduced in a fixed order (wave shuffles, then the 4 waves
// in order): deterministic, no atomics.
// PARTS = 2 (ABI v7) or 3 (ABI v10: dhm [3H][B], rows 2H + h = RNE(dpre - hb - mb): dW1 = sum of the three
// parts' GEMMs is then accurate to ~2^-24 per product term, torch fp32's level, where the two-way split's
// 2^-17 let near-zero dW1 elements take the other sign and Adam's first step move them by 2 lr)
template <int PARTS>
__global__ __launch_bounds__(256) void critic_dpre_kernel(int H, int64_t B, int64_t chunk, const float* __restrict__ pre,
                                                          const float* __restrict__ w2, const float* __restrict__ dv,
                                                          uint16_t* __restrict__ dhm, float* __restrict__ partial) {
  __shared__ float red[2][4];
  const int64_t b0 = (int64_t)blockIdx.x * chunk;
  const int64_t b1 = b0 + chunk < B ? b0 + chunk : B;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int h = 0; h < H; ++h) {
    const float m = w2[h];
    float s_db = 0.f, s_gw = 0.f;
    for (int64_t b = b0 + threadIdx.x; b < b1; b += 256) {
      const float p = pre[(int64_t)h * B + b], d = dv[b];
      const float dp = p > 0.f ? m * d : 0.f;
      const __bf16 hb = (__bf16)dp;  // v_cvt_pk_bf16_f32: round to nearest even, like torch's .to(bfloat16)
      const float r1 = dp - (float)hb;  // exact
      const __bf16 mb = (__bf16)r1;
      dhm[(int64_t)h * B + b] = __builtin_bit_cast(uint16_t, hb);
      dhm[(int64_t)(H + h) * B + b] = __builtin_bit_cast(uint16_t, mb);
      if constexpr (PARTS == 3) dhm[(int64_t)(2 * H + h) * B + b] = __builtin_bit_cast(uint16_t, (__bf16)(r1 - (float)mb));
      s_db += dp;
      s_gw += fmaxf(p, 0.f) * d;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s_db += __shfl_xor(s_db, o);
      s_gw += __shfl_xor(s_gw, o);
    }
    if (lane == 0) {
      red[0][wave] = s_db;
      red[1][wave] = s_gw;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float* out = partial + (int64_t)blockIdx.x * 2 * H;
      out[h] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
      out[H + h] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
    __syncthreads();
  }
}

extern "C" int32_t d2d_critic_dpre_blocks(int64_t B) {
  const int64_t g = (B + 2047) / 2048;
  return (int32_t)(g < 1 ? 1 : g > 1024 ? 1024 : g);
}

extern "C" int d2d_critic_dpre_split(int32_t H, int64_t B, const float* pre, const float* w2, const float* dv,
                                     uint16_t* dhm, float* partial, int32_t G, void* stream) {
  if (H < 1 || B < 0 || G != d2d_critic_dpre_blocks(B) || !pre || !w2 || !dv || !dhm || !partial) {
    d2d_set_error("d2d_critic_dpre_split: bad arguments (G must be d2d_critic_dpre_blocks(B))");
    return D2D_EINVAL;
  }
  const int64_t chunk = (B + G - 1) / G;
  hipLaunchKernelGGL(critic_dpre_kernel<2>, dim3((unsigned)G), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), H,
                     B, chunk, pre, w2, dv, dhm, partial);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}

extern "C" int d2d_critic_dpre_split3(int32_t H, int64_t B, const float* pre, const float* w2, const float* dv,
                                      uint16_t* dhm, float* partial, int32_t G, void* stream) {
  if (H < 1 || B < 0 || G != d2d_critic_dpre_blocks(B) || !pre || !w2 || !dv || !dhm || !partial) {
    d2d_set_error("d2d_critic_dpre_split3: bad arguments (G must be d2d_critic_dpre_blocks(B))");
    return D2D_EINVAL;
  }
  const int64_t chunk = (B + G - 1) / G;
  hipLaunchKernelGGL(critic_dpre_kernel<3>, dim3((unsigned)G), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), H,
                     B, chunk, pre, w2, dv, dhm, partial);
  D2D_CHECK_HIP(hipGetLastError());
  return D2D_OK;
}
