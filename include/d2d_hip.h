/* d2d_hip.h — C ABI of the MI355X (gfx950) D2D-PPO hot path.
 *
 * The reference (benrobaglia/D2D-PPO) is pure Python with no FFI; its
 * "plugin interface" is the duck-typed env/learner API.  These
 * entry points are what that API's hot methods bind to (ctypes, see
 * INTEGRATION.md); each cites the reference code it replaces.
 *
 * Conventions
 *   - every buffer is caller-allocated device memory (plain pointers);
 *   - the `stream` argument is a hipStream_t passed as void*;
 *   - calls are stream-ordered, never allocate, never synchronise the host,
 *     and are therefore graph-capturable;
 *   - return 0 (D2D_OK) or a negative code; d2d_last_error() describes it
 *     (thread-local string).
 *   - one stream per env batch; not re-entrant for the same state buffers.
 *
 * Env batch = E independent environments with identical parameters (one
 * rank's shard).  Device layouts, N agents, C channels,
 * D = max deadline, DW = d2d_buffer_words(D) (1,2,3,4 or 8 uint32 per row):
 *   buffers   uint32 [E][N][DW]  byte j of agent k's row = packets with j
 *                                slots to deadline (byte 0 expires next)
 *   channels  comb : mask [E][N] (uint8 if C<=8, uint16 if C<=16, uint32 if
 *                    C<=32); bit c = 1 <=> channel c is good for agent k
 *             chsel: uint32 [E], bit j = state of channel j (0..C)
 *             single: uint8 [E][N], 0/1 = agent k's channel state
 *   actions   comb : mask [E][N] (same width as channels), bit c = attempt on c
 *             chsel: uint8 [E][N], channel id 0..C (0 = idle)
 *             single: uint8 [E][N], 0/1 (transmit)
 *   obs       float [E][N][obs_dim], agent k's row is prefix-compact:
 *               comb  [B[k,:w_k], channel_row_k (pre-evolve), ack(C), 0 ...]
 *               chsel [B[k,:d_k], ack(C+1), 0 ...]
 *               single [B[j,:d_j] for j in nbr(k), H[j] for j in nbr(k), ack, 0 ...]
 *                      (post-evolve channel; ack in {1, 0, -1})
 *             (w_k = D when homogeneous_size else d_k)
 *   state     float [E][state_stride], the reference's np.concatenate(state)
 */
#ifndef D2D_HIP_H
#define D2D_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define D2D_ABI_VERSION 15  /* 4: GRU entry points; 5: compact obs record (obs_record, obs_format);
                              6: d2d_env_desc.poisson_cdf; 7: d2d_f32_to_bf16_exact, d2d_states_to_bf16_exact,
                              d2d_critic_dpre_split; 8: d2d_gae_scan_moments, d2d_normalize_pair;
                              9: d2d_gae_scan_moments without outputs, d2d_gae_scan_normalized;
                              10: d2d_states_to_bf16_padded, d2d_critic_dpre_split3;
                              11: D2D_OPT_CRITIC_GRAD_ROWS; 12: d2d_ppo_critic_grad_values, d2d_central_critic_*;
                              13: d2d_comb_policy_fused_step, D2D_OPT_FUSED_SLICE, d2d_env_out.state_bf16;
                              14: d2d_policy_gru_carry, d2d_gru_carry_floats, d2d_central_critic_dw1, single obs_record;
                              15: actions = NULL in forced mode (d2d_policy_mlp_step, d2d_policy_gru) */

enum { D2D_ENV_COMBINATORIAL = 0, D2D_ENV_CHANNEL_SELECTION = 1, D2D_ENV_SINGLE = 2 };
enum { D2D_ARRIVAL_POISSON = 0, D2D_ARRIVAL_SCHEDULED_BERNOULLI = 1, D2D_ARRIVAL_NONE = 2 };
enum { D2D_OK = 0, D2D_EINVAL = -1, D2D_EUNSUPPORTED = -2, D2D_EHIP = -3 };

/* Per-agent parameters, device table [N] (32 bytes each). */
typedef struct d2d_agent_entry {
    uint8_t deadline;      /* d_k  (deadlines[k], combinatorial_env.py:9) */
    uint8_t obs_width;     /* w_k  buffer columns in obs (D if homogeneous_size, :104-107) */
    uint8_t arrival_kind;  /* D2D_ARRIVAL_*  (traffic model split, :66-85) */
    uint8_t reserved;
    int32_t state_offset;  /* sum_{j<k} d_j  (all_buffers concat, :207) */
    double lam;            /* Poisson mean lbdas[k] */
    double pois_p0;        /* exp(-lam) */
    uint64_t arrival_thr;  /* Bernoulli(arrival_probs[k]) threshold floor(q * 2^32) */
} d2d_agent_entry;

typedef struct d2d_env_desc {
    int32_t env_kind;       /* D2D_ENV_* */
    int32_t n_agents;       /* N <= 1024 */
    int32_t n_channels;     /* C <= 32 (comb), C <= 31 (chsel) */
    int32_t max_deadline;   /* D <= 32 */
    int32_t obs_dim;        /* D + 2C (comb) / D + C + 1 (chsel) */
    int32_t state_dim;      /* sum d + C(N+1) (comb) / sum d + C + 1 (chsel) */
    int32_t state_stride;   /* >= state_dim, multiple of 4 */
    int32_t n_envs;         /* E, envs in this batch */
    uint64_t env_base;      /* global index of env 0 (Philox counter; rank shard offset) */
    uint64_t seed;          /* Philox key */
    const d2d_agent_entry* agents;  /* device [N] */
    const uint64_t* flip_thr;       /* device: comb [N][C], chsel [C+1]; floor(p * 2^32) */
    /* host-side arrival schedule (evaluated per call, numpy float semantics):
     * agent k draws at timestep t iff kind==POISSON or
     * (kind==SCHEDULED_BERNOULLI and fmod(t, period[k]) == offset[k]) */
    const uint8_t* arrival_kind_host;  /* host [N] */
    const double* period_host;         /* host [N] */
    const double* offset_host;         /* host [N] */
    /* D2D_ENV_SINGLE only: device int32 [N*obs_dim + state_dim] gather codes of the
     * neighbourhood obs rows then the state row, built on the host by
     * d2d_env_single_gather_map (envs/env.py neighbourhoods, :39-49, 91-98) */
    const int32_t* gather;
    /* optional device uint32 added to every call's rng_step when the kernel runs (NULL = 0):
     * a captured HIP graph of reset/step calls replays with fresh Philox counters by
     * updating this one word instead of the baked launch arguments */
    const uint32_t* rng_offset;
    /* device uint32 [N][256]: inverse-CDF thresholds of the Philox-mode Poisson arrival draw,
     * t[k][x] = min(ceil(F_k(x) * 2^32), 2^32) - 1 with F_k(x) the running double sum
     * exp(-lam), p = p * lam / x, F += p (x <= 254), t[k][255] = 2^32 - 1; the draw of word r is the
     * number of leading entries with r > t[k][x] -- bitwise the sequential inversion of the reference
     * oracle (oracle/philox.py poisson_inversion), without a double division per step.  Rows of
     * non-Poisson agents are never read.  Required (spec.py poisson_cdf_table builds it). */
    const uint32_t* poisson_cdf;
} d2d_env_desc;

typedef struct d2d_env_state {
    uint32_t* buffers;
    void* channels;
    uint32_t* received;     /* [E][N] packets received this episode (received_packets) */
    uint32_t* discarded;    /* [E][N] packets expired (discarded_packets) */
    uint32_t* sel_quality;  /* chsel [E] selected_channel_qualities; single [E] channel_errors; NULL for comb */
    uint32_t* sel_count;    /* chsel [E] number_selected_channel; single [E] n_collisions; NULL for comb */
} d2d_env_state;

typedef struct d2d_env_out {  /* any field may be NULL */
    float* obs;         /* [E][N][obs_dim] */
    float* state;       /* [E][state_stride] */
    int32_t* reward;    /* [E]  |successful users| (single: the ack); broadcast to all agents by the host */
    void* ack;          /* comb int8 [E][C] in {-1,0,1}; chsel double [E][C+1]; single int8 [E] */
    uint8_t* success;   /* [E][N] 1 if agent k delivered a packet this slot */
    /* comb and (ABI 14) single: the compact obs record [E][N][D2D_RECORD_BYTES(obs_dim)] (16-byte aligned),
     * the obs row above one byte per column: packet counts and channel bits as uint8, the acks (comb: columns
     * [w_k + C, w_k + 2C); single: the last-feedback column, gather code -1) as int8, then byte obs_dim = 1
     * (the networks' layer-1 bias input) and zeros.  Every obs value of these envs is an integer in those
     * ranges, so the record is exact; consumers take it with obs_format = D2D_OBS_U8.  single: the agents'
     * gather codes are staged in LDS (N * (record bytes + 4) * 4 bytes beside the rows; D2D_EUNSUPPORTED past
     * 160 KiB, e.g. full neighbourhoods of ~96 agents). */
    uint8_t* obs_record;
    /* comb only (ABI v13): the state row as bf16 -- exact, every state value is an integer in [-1, 255] -- for
     * the D2D central critic's operand: env e's row at state_bf16 + e * state_bf16_ld (elements; a multiple of
     * 8, >= state_dim rounded up to 8, 16-byte aligned base), columns [state_dim, round_up(state_dim, 8)) zero.
     * A caller passing the slot-t base of an env-major [E][T][ld] buffer with ld_env = T * ld gets the
     * learner's [E*T][ld] operand with no fp32 copy and no conversion pass. */
    uint16_t* state_bf16;
    int64_t state_bf16_ld;
} d2d_env_out;

/* Row bytes of the compact obs record: 32 per chunk of 32 network inputs (obs columns + the
 * layer-1 bias input), the chunking of the MLP / GRU kernels. */
#define D2D_RECORD_BYTES(obs_dim) (32 * (((obs_dim) + 32) / 32))
enum { D2D_OBS_F32 = 0, D2D_OBS_U8 = 1 };

typedef struct d2d_env_replay {  /* parity mode; both NULL = Philox production stream */
    const void* flips;        /* comb mask [E][N]; chsel uint32 [E] */
    const uint8_t* arrivals;  /* [E][N] arrival value for agents that draw at this call */
} d2d_env_replay;

/* Replaces CombinatorialEnv.reset (envs/combinatorial_env.py:61-114),
 * ChannelSelectionEnv.reset (envs/channel_selection_env.py:49-98) and
 * D2DEnv.reset (envs/env.py:51-99). */
int d2d_env_reset(const d2d_env_desc* desc, const d2d_env_state* st, const d2d_env_replay* replay,
                  const d2d_env_out* out, uint32_t rng_step, void* stream);

/* Replaces CombinatorialEnv.step (envs/combinatorial_env.py:127-242, with
 * evolve_channel 116-118 and evolve_buffer 120-124) and
 * ChannelSelectionEnv.step (envs/channel_selection_env.py:116-214) and
 * D2DEnv.step (envs/env.py:116-213, with decode_signal 101-103,
 * evolve_channel 105-107 and evolve_buffer 109-113).
 * `timestep` is the value after the increment (t = 1, 2, ...). */
int d2d_env_step(const d2d_env_desc* desc, const d2d_env_state* st, const void* actions,
                 const d2d_env_replay* replay, const d2d_env_out* out, int32_t timestep, uint32_t rng_step,
                 void* stream);

/* Synthetic actions (env-only benchmark; replaces the per-agent
 * np.random.binomial of baselines.CombinatorialRandomAccess.act,
 * algorithms/baselines.py:181-183): comb mask bit c ~ Bernoulli(thr/2^32);
 * chsel uniform channel id in 0..C; single 0/1 ~ Bernoulli(thr/2^32)
 * (GFAccess.act, algorithms/baselines.py:121-125). */
int d2d_sample_actions(const d2d_env_desc* desc, void* actions, uint64_t threshold, uint32_t rng_step,
                       void* stream);

/* Host-only: the D2DEnv gather table (envs/env.py:39-49 obs_length / state_length,
 * 91-98 obs / state concatenation).  Agent k observes agents
 * nbr_idx[nbr_ptr[k] .. nbr_ptr[k+1]) in that order.  Writes obs_dim*N + S codes
 * (S = sum d + N + 1): code >= 0 is j*64 + q (byte q of agent j's buffer row,
 * q < 32) or j*64 + 32 (agent j's channel state); -1 = the ack; -2 = zero padding.
 * obs_dim must be >= every obs length.  Returns the number of codes written. */
int d2d_env_single_gather_map(int32_t n_agents, const int32_t* deadlines, const int32_t* nbr_ptr,
                              const int32_t* nbr_idx, int32_t obs_dim, int32_t* out, int64_t out_len);

/* Bytes of one comb channel/action mask for C channels (1, 2 or 4). */
int d2d_mask_bytes(int32_t n_channels);

/* uint32 words per agent buffer row for max deadline D (D<=4:1, <=8:2, <=12:3, <=16:4, <=32:8). */
int d2d_buffer_words(int32_t max_deadline);

/* ---- GAE / discounted returns (algorithms/ippo.py:92-116 == d2d_ppo.py:100-124) ----
 * Sequence semantics: the batch is the reference's sequential rollout of the
 * E envs' episodes in env-major order, so row (t, e) of column c follows
 *   R = r + gamma * R' * (1 - done_t),  delta = r + gamma V' (1-done_t) - V,
 *   gae = delta + gamma*lam*(1-done_t)*gae,  adv = gae + V  (quirk Q1),
 * except the globally last element (e = E-1, t = T-1 on the last shard),
 * whose adv is r - V (ippo.py:94).
 *   rewards [T][E][reward_cols] (reward_cols 1 = broadcast over columns, or cols),
 *   values [T][E][cols], dones [T] (every env's sequence ends at t = T-1)
 *   adv, ret [T][E][cols] float (raw, un-normalised)                     */
int d2d_gae_scan(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards, const float* values,
                 const uint8_t* dones, double gamma, double lam, int32_t last_shard, float* adv, float* ret,
                 void* stream);

/* The same scan on the [T][cols][E] layout (values / adv / ret element (t, e, c) at
 * (t * cols + c) * E + e; rewards [T][E] when reward_cols == 1, else [T][cols][E]). */
int d2d_gae_scan_tce(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards,
                     const float* values, const uint8_t* dones, double gamma, double lam, int32_t last_shard,
                     float* adv, float* ret, void* stream);

/* Column sums over rows of x [rows][cols]: out[c] = sum_r (x[r][c] - center[c])^p,
 * p = 1 when center == NULL else 2.  Deterministic two-level reduction in
 * double; `partial` is a workspace of d2d_colstats_workspace(rows, cols) doubles. */
int64_t d2d_colstats_workspace(int64_t rows, int32_t cols);
int d2d_colstats(int64_t rows, int32_t cols, const float* x, const double* center, double* partial,
                 double* out, void* stream);

/* d2d_colstats over x [T][cols][E] (column c = the T*E elements (t, c, e)); same workspace. */
int d2d_colstats_tce(int32_t T, int32_t cols, int32_t E, const float* x, const double* center, double* partial,
                     double* out, void* stream);

/* The scan above with the normalisation statistics of BOTH outputs fused into it (ABI 8): one pass
 * writes adv / ret and accumulates, per column, n, sum and M2 = sum of squared deviations from the
 * column mean of the stored fp32 values (compute_gae's np.std / discount_rewards' torch std inputs,
 * ippo.py:99-101, 113-115), combined in double with Chan's pairwise formula in a fixed order (bitwise
 * reproducible, no atomics).  layout 0 = [T][E][cols] (d2d_gae_scan), 1 = [T][cols][E] (_tce).
 *   moments [2][3][cols] doubles out: [0] adv, [1] ret; [k][0] n, [k][1] sum, [k][2] M2
 *   workspace: d2d_gae_moments_workspace(E, cols, layout) doubles
 * Data-parallel shards combine their moments with two all-reduces of [cols] vectors (d2dhip/gae.py);
 * one rank passes sum / M2 straight to d2d_colstats_finalize. */
int64_t d2d_gae_moments_workspace(int32_t E, int32_t cols, int32_t layout);
int d2d_gae_scan_moments(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards,
                         const float* values, const uint8_t* dones, double gamma, double lam, int32_t last_shard,
                         int32_t layout, float* adv, float* ret, double* moments, double* workspace,
                         int64_t workspace_len, void* stream);
/* ABI 9: adv == ret == NULL computes the moments only (nothing written but moments): the first of the
 * two scans of a normalised GAE.  The second, d2d_gae_scan_normalized, recomputes the same recursion
 * and writes adv_k = gate_k ? (adv_k - mean_k) * scale_k : adv_k (and ret likewise; mean == NULL: raw)
 * -- bitwise the outputs of d2d_gae_scan_moments + d2d_normalize_pair, with 16 B of HBM traffic per
 * element instead of 28 (ippo.py:92-116: compute_gae + discount_rewards + their normalisation). */
int d2d_gae_scan_normalized(int32_t T, int32_t E, int32_t cols, int32_t reward_cols, const float* rewards,
                            const float* values, const uint8_t* dones, double gamma, double lam, int32_t last_shard,
                            int32_t layout, float* adv, const double* mean0, const double* scale0,
                            const int32_t* gate0, float* ret, const double* mean1, const double* scale1,
                            const int32_t* gate1, void* stream);

/* mean = sum / n ; when m2 != NULL: std = sqrt(m2 / (n - ddof)), scale = 1/std and
 * *gate = all columns std > 0 (ippo.py:100-101, 114-115); when m2 == NULL only mean. */
int d2d_colstats_finalize(int32_t cols, const double* sum, const double* m2, double n, int32_t ddof,
                          double* mean, double* scale, int32_t* gate, void* stream);

/* x = gate ? (x - mean) * scale : x  (per column) */
int d2d_normalize_columns(int64_t rows, int32_t cols, float* x, const double* mean, const double* scale,
                          const int32_t* gate, void* stream);
/* the same on x [T][cols][E] */
int d2d_normalize_columns_tce(int32_t T, int32_t cols, int32_t E, float* x, const double* mean, const double* scale,
                              const int32_t* gate, void* stream);

/* Both outputs of the scan normalised in one pass (ABI 8): x_k = gate_k ? (x_k - mean_k) * scale_k : x_k
 * per column, k = 0, 1; x1 (or x0) may be NULL; layout as d2d_gae_scan_moments; x 16-byte aligned. */
int d2d_normalize_pair(int32_t T, int32_t E, int32_t cols, int32_t layout, float* x0, const double* mean0,
                       const double* scale0, const int32_t* gate0, float* x1, const double* mean1,
                       const double* scale1, const int32_t* gate1, void* stream);

/* fp32 -> bf16 (the high 16 bits) of n floats in one pass, *inexact = 1 iff some x is not
 * bf16-exact (nonzero low 16 bits), else 0.  x 16-byte, out 8-byte aligned.  Replaces the
 * conversion + exactness check of the D2D central critic's bf16 GEMM operand (the states,
 * algorithms/d2d_ppo.py:95-98 Value.forward on the whole state batch; ABI v7). */
int d2d_f32_to_bf16_exact(int64_t n, const float* x, uint16_t* out, int32_t* inexact, void* stream);
/* The same from the rollout's slot-major state buffer x [T][E][ld] (its first S floats per row) into
 * the env-major bf16 operand out [E*T][S] (row e*T + t), no fp32 env-major copy first (ABI v7). */
int d2d_states_to_bf16_exact(int32_t T, int32_t E, int32_t S, int64_t ld, const float* x, uint16_t* out,
                             int32_t* inexact, void* stream);
/* The same into rows of out_ld >= S bf16 (columns [S, out_ld) written as zeros): the GEMM-aligned operand
 * [E*T][out_ld] of a state width that is not a multiple of 8 (configs[1]'s S = 117).  ABI v10. */
int d2d_states_to_bf16_padded(int32_t T, int32_t E, int32_t S, int64_t ld, const float* x, uint16_t* out,
                              int64_t out_ld, int32_t* inexact, void* stream);

/* D2D central critic backward glue (algorithms/d2d_ppo.py:208-216 value_loss.backward() through
 * Value = linear2(relu(linear1(state)))), pre [H][B] (the first layer's pre-activations), w2 [H]
 * (linear2.weight), dv [B] (dL/dV): dpre = pre > 0 ? w2[h] dv[b] : 0 written as the two-way RNE bf16
 * split dhm [2H][B] (rows h: RNE(dpre), rows H + h: RNE(dpre - RNE(dpre))), and per-block sums
 * partial [G][2H]: [g][h] = sum dpre (db1), [g][H + h] = sum relu(pre) dv (dW2) over block g's samples;
 * G = d2d_critic_dpre_blocks(B).  Deterministic (fixed-order sums, no atomics).  ABI v7. */
int32_t d2d_critic_dpre_blocks(int64_t B);
int d2d_critic_dpre_split(int32_t H, int64_t B, const float* pre, const float* w2, const float* dv, uint16_t* dhm,
                          float* partial, int32_t G, void* stream);
/* The same with a three-way RNE split, dhm [3H][B] (rows 2H + h: RNE(dpre - rows h - rows H + h)): the dW1
 * GEMM over the three parts is accurate to ~2^-24 per product term (torch fp32's level).  ABI v10. */
int d2d_critic_dpre_split3(int32_t H, int64_t B, const float* pre, const float* w2, const float* dv, uint16_t* dhm,
                           float* partial, int32_t G, void* stream);

/* D2D-PPO's sequential agent update chain (algorithms/d2d_ppo.py:405-433): for the agent
 * permutation perm[0..N), M[perm[j]][b] = adv[b] * prod_{l<j} exp(logp_new[perm[l]][b] -
 * logp_old(perm[l], b)), multiplied left to right in fp32.  b = t*E + e over T*E samples;
 * adv [T*E], logp_new [N][T*E], logp_old [T][N][E] (the rollout layout), M [N][T*E]; perm device int32. */
int d2d_happo_chain(int32_t n_agents, int32_t T, int32_t E, const float* adv, const float* logp_new,
                    const float* logp_old, const int32_t* perm, float* M, void* stream);

/* ---- fused behaviour-policy slot (MLP learners) ----
 * Replaces Policy/Value.forward + PPO.select_action for every agent of every env
 * (algorithms/ippo.py:54-90, 154-176; d2d_ppo.py:62-98, 159-181).  Weights are the
 * agent-stacked nn.Linear tensors:  w1 [N][H][F], b1 [N][H], w2 [N][A][H], b2 [N][A];
 * optional critic v1 [N][H][F], c1 [N][H], v2 [N][1][H], c2 [N][1] (NULL = no critic).
 * kind 0: softmax -> Bernoulli per output (combinatorial, A = C channels), actions =
 *         channel masks [E][N] (d2d_mask_bytes(A) bytes), logp = mean_c log_prob;
 * kind 1: softmax -> Categorical over A = C+1 ids, actions = uint8 [E][N].
 * obs [E][N][F] (the env kernel's layout); logp, value [N][E].  forced != NULL
 * evaluates the given actions instead of sampling; actions may then be NULL (ABI 15: only logp is written --
 * D2D-PPO's epoch-start log-prob pass).  deterministic = argmax / p > 0.5.
 * Sampling uses Philox stream 3 at (env_base + env, agent, rng_step).
 * Shapes: obs_dim <= 64, n_out <= 16, hidden <= 64, or hidden <= 128 when obs_dim + 1 <= 32 (the
 * learners' default hidden_size 128 on the reference envs; one wave per SIMD there), else D2D_EUNSUPPORTED;
 * the update kernels below take the same hidden limits with obs_dim + 1 <= 64. */
typedef struct d2d_mlp_desc {
    int32_t n_agents, n_envs, obs_dim, hidden, n_out, kind;
    const float *w1, *b1, *w2, *b2;
    const float *v1, *c1, *v2, *c2;
    uint64_t seed, env_base;
    const uint32_t* rng_offset;  /* optional device uint32 added to rng_step (graph replays), as in d2d_env_desc */
    /* obs_format D2D_OBS_F32: every `obs` argument below is float [..][N][obs_dim];
     * D2D_OBS_U8: it is the env kernel's compact record [..][N][D2D_RECORD_BYTES(obs_dim)] and
     * obs_signed (device uint32 [N][D2D_RECORD_BYTES(obs_dim) / 32]) marks agent k's int8 columns:
     * bit b of word c = column 32c + b is signed (the acks), every other byte is uint8. */
    int32_t obs_format, reserved;
    const uint32_t* obs_signed;
} d2d_mlp_desc;

int d2d_policy_mlp_step(const d2d_mlp_desc* desc, const void* obs, const void* forced, uint32_t rng_step,
                        int32_t deterministic, void* actions, float* logp, float* value, void* stream);

/* Fused env + policy rollout slot (the loop body of create_rollouts,
 * /root/reference/algorithms/ippo.py:293-330): d2d_env_step of slot t (actions -> out->obs_record = the
 * record of slot t + 1, env state, rewards; timestep / env_rng_step as d2d_env_step) followed by
 * d2d_policy_mlp_step of slot t + 1 on that record (policy_rng_step, deterministic; actions_out,
 * logp_out) in ONE launch: each workgroup steps a slice of envs and runs the policy of every agent on
 * the slice's records from LDS.  The results equal the two calls' bit for bit.  actions_out may alias
 * actions (a slice reads its own envs' actions before it writes them).  Prototype scope: the
 * combinatorial env with 64 agents and 8 channels, obs_dim < 32 (32-byte record), out without obs /
 * state rows; policy D2D_OBS_U8 on this env (same agents, envs, obs_dim, env_base), kind 0, n_out <= 8,
 * hidden <= 64, no critic, no forced actions -- else D2D_EUNSUPPORTED / D2D_EINVAL.
 * Measured against the two-launch slot in tools/gpu/fused_slot.py. */
int d2d_comb_policy_fused_step(const d2d_env_desc* desc, const d2d_env_state* st, const void* actions,
                               const d2d_env_out* out, int32_t timestep, uint32_t env_rng_step,
                               const d2d_mlp_desc* policy, uint32_t policy_rng_step, int32_t deterministic,
                               void* actions_out, float* logp_out, void* stream);

/* ---- fused PPO update: per-agent gradients of the MLP learners' losses ----
 * Replaces evaluate() + loss + backward() of PPO.train_step for every agent at once
 * (algorithms/ippo.py:178-217; d2d_ppo.py:183-216): the actor loss
 *   L_k = -mean_s min(r W, clamp(r, 1-clip, 1+clip) W) - beta * mean_s entropy,
 *   r = exp(logp(a_s) - logp_old_s),  W = advantage (iPPO) or M (D2D chain),
 * and the critic loss mean_s (V(x_s) - R_s)^2 (ippo.py:210-216).  "mean" is `scale` * sum over
 * the T * n_envs samples of this call (scale = 1/B; for data-parallel shards 1/B_local, the
 * caller averages across ranks).  Samples are the rollout slots t < T of envs e < n_envs:
 *   obs      [T][n_envs][N][F] fp32 (the rollout buffer the env kernel writes),
 *   actions  [T][n_envs][N] channel masks (kind 0) / uint8 ids (kind 1),
 *   logp_old, weight, returns: element (t, e, k) at t*s[0] + e*s[1] + k*s[2] (strides in floats).
 * Network: the d2d_mlp_desc weights (actor w1, b1, w2, b2; critic: its v1, c1, v2, c2 passed as
 * w1, b1, w2, b2 with n_out ignored).  Outputs (overwritten, agent-stacked like the weights):
 * gw1 [N][H][F], gb1 [N][H], gw2 [N][A][H], gb2 [N][A]; stats [N][2] = (sum_s min(...),
 * sum_s entropy) for the actor, (sum_s (V - R)^2, 0) for the critic (NULL = not wanted).
 * workspace: d2d_ppo_workspace(...) floats of device scratch.  Deterministic (fixed-order sums). */
int64_t d2d_ppo_workspace(int32_t n_agents, int32_t T, int32_t n_envs, int32_t obs_dim, int32_t hidden,
                          int32_t n_out);
int d2d_ppo_actor_grad(const d2d_mlp_desc* desc, int32_t T, const void* obs, const void* actions,
                       const float* logp_old, const int64_t* logp_strides, const float* weight,
                       const int64_t* weight_strides, float clip, float beta, float scale, float* gw1, float* gb1,
                       float* gw2, float* gb2, float* stats, float* workspace, int64_t workspace_floats,
                       void* stream);
int d2d_ppo_critic_grad(const d2d_mlp_desc* desc, int32_t T, const void* obs, const float* returns,
                        const int64_t* return_strides, float scale, float* gw1, float* gb1, float* gw2, float* gb2,
                        float* stats, float* workspace, int64_t workspace_floats, void* stream);
/* ABI 12: d2d_ppo_critic_grad that also writes the critic's value V(obs) of every sample, element (t, e, k) at
 * t * values_strides[0] + e * values_strides[1] + k * values_strides[2] (NULL values = d2d_ppo_critic_grad).
 * Replaces the per-slot critic forward of iPPO.create_rollouts (algorithms/ippo.py:308, the values GAE needs,
 * ippo.py:337): the critic's weights do not change between the rollout and the first epoch's critic gradient,
 * so the learners take the rollout's values from that pass instead of from every rollout slot. */
int d2d_ppo_critic_grad_values(const d2d_mlp_desc* desc, int32_t T, const void* obs, const float* returns,
                               const int64_t* return_strides, float scale, float* gw1, float* gb1, float* gw2,
                               float* gb2, float* stats, float* workspace, int64_t workspace_floats, float* values,
                               const int64_t* values_strides, void* stream);

/* ---- D2D-PPO central critic, forward + the backward's per-sample glue (ABI 12) -------------------------------
 * The Value network over the whole state (d2d_ppo.py:62-98: linear1 [H][S], relu, linear2 [1][H]) for every sample
 * b of xb [B][ldx] (the rollout's states as exact bf16 integers, columns [S, ldx) zero, ldx a multiple of 8,
 * 16-byte aligned; EVERY element of xb finite: the K loop reads whole 32-column chunks rounded up to its chunk
 * group, so past column ldx it reads the next row's leading columns against zero W1 image columns, and a
 * non-finite value there would turn 0 * x into NaN): values[b] = V(x_b); against ret [B] (the critic target, returns.mean(1), d2d_ppo.py:339) the
 * MSE loss's backward through linear2 / relu (d2d_ppo.py:440-446, value_loss.backward()): dpre_b = [pre_b > 0] w2
 * 2 (v_b - ret_b) / B as its three-way RNE bf16 split in dhm [B][3H] (parts h | m | l; dW1 = sum_b dpre_b x_b^T is
 * the caller's split-K GEMM), and per-workgroup sums partial [G][2H + 2] = db1 | dW2 | db2 | sum (v - ret)^2.
 * w1img: d2d_central_critic_image_bytes(H, S) bytes of device scratch (W1's split image, rebuilt by every call);
 * G = d2d_central_critic_blocks(H, B).  H a multiple of 4 in [4, 128]; else D2D_EUNSUPPORTED. */
int32_t d2d_central_critic_blocks(int32_t hidden, int64_t B);
int64_t d2d_central_critic_image_bytes(int32_t hidden, int32_t S);
int d2d_central_critic_fwd(int32_t hidden, int64_t B, int32_t S, int64_t ldx, const uint16_t* xb, const float* w1,
                           const float* b1, const float* w2, const float* b2, const float* ret, void* w1img,
                           float* values, uint16_t* dhm, float* partial, int32_t G, void* stream);

/* dW1 = sum_b dpre_b x_b^T of the same critic (d2d_ppo.py:440-446: value_loss.backward() into linear1.weight) from
 * d2d_central_critic_fwd's dhm [B][3H] (the three RNE parts of dpre, all accumulated: the result is dW1 itself) and
 * the operand xb [B][ldx] (as d2d_central_critic_fwd: bf16, columns [S, ldx) zero, every element finite, 16-byte
 * aligned), on bf16 MFMAs through LDS (critic_kernels.hip; ABI 14, replacing the hipBLASLt split-K bmm of rounds 4-5).
 * dw1: [H][S] fp32 (overwritten).  workspace: d2d_central_critic_dw1_workspace(H, B, S, ldx) floats of device scratch
 * (the per-K-range partials, summed in fixed order: deterministic).  H a multiple of 4 in [4, 128]. */
int64_t d2d_central_critic_dw1_workspace(int32_t hidden, int64_t B, int32_t S, int64_t ldx);
int d2d_central_critic_dw1(int32_t hidden, int64_t B, int32_t S, int64_t ldx, const uint16_t* xb, const uint16_t* dhm,
                           float* workspace, int64_t workspace_floats, float* dw1, void* stream);

/* ---- GRU window policies (the reference's RNN module, algorithms/ippo.py:14-51 == d2d_ppo.py:24-59) ----
 * Per agent: torch.nn.GRU(F, H) weights w_ih [N][3H][F], w_hh [N][3H][H], b_ih, b_hh [N][3H] (gate order
 * r, z, n) and the head layers.0 w1 [N][H][H], b1 [N][H], layers.2 w2 [N][n_out][H], b2 [N][n_out]
 * (agent-stacked).  kind 0: sigmoid head -> Bernoulli per channel (combinatorial actor), 1: softmax ->
 * Categorical (channel-selection / D2DEnv actor), 2: no activation, n_out 1 (iPPO value critic).
 * Windows are rebuilt in-kernel from the rollout buffer obs [T][n_envs][N][F] (T a multiple of
 * episode_length): for slot s at episode position p = s % episode_length the window is the last
 * S = min(p + 1, history_len) obs of the episode, unpadded (rollout / test, ippo.py:302-304, 362-364)
 * or front-zero-padded to history_len steps (training, preprocess_input_for_rnn ippo.py:390-403);
 * h0 = 0 for every window.  Sampling as d2d_policy_mlp_step (Philox stream 3, sample index
 * (s - slot0) * n_envs + e, i.e. the env index for one-slot launches). */
typedef struct d2d_gru_desc {
    int32_t n_agents, n_envs, obs_dim, hidden, n_out, kind;
    int32_t history_len, episode_length;
    const float *w_ih, *w_hh, *b_ih, *b_hh, *w1, *b1, *w2, *b2;
    uint64_t seed, env_base;
    const uint32_t* rng_offset;  /* optional device uint32 added to rng_step (graph replays) */
    int32_t obs_format, reserved;  /* as in d2d_mlp_desc: D2D_OBS_U8 = obs is the compact record */
    const uint32_t* obs_signed;
} d2d_gru_desc;

/* Behaviour policy / value over slots [slot0, slot0 + n_slots) of the buffer (ippo.py:154-191 per agent,
 * batch 1, replaced for all agents and envs): kinds 0/1 write actions [n_slots][n_envs][N] (masks / ids;
 * forced != NULL: evaluate these instead of sampling; deterministic: p > 0.5 / argmax) and log-probs
 * out [N][n_slots * n_envs]; kind 2 writes the values to out [N][n_slots * n_envs]. */
int d2d_policy_gru(const d2d_gru_desc* desc, int32_t T, const void* obs, int32_t slot0, int32_t n_slots,
                   int32_t padded, const void* forced, uint32_t rng_step, int32_t deterministic, void* actions,
                   float* out, void* stream);

/* d2d_policy_gru for ONE unpadded slot (rollout / test windows, ippo.py:302-304, 362-364) with a carried hidden state
 * (ABI 14).  While the slot's episode position p = slot % episode_length is below history_len, its window is the
 * previous slot's window plus obs[slot] (both start at the episode's first slot; h0 = 0), so a rollout that runs its
 * slots in order need not recompute the window: hcarry (d2d_gru_carry_floats(desc) floats of device scratch owned by
 * the caller, one per (policy, env batch)) holds h after the previous slot's window, carry_in != 0 says so, and the
 * launch runs the window's last step only.  Every launch whose next window extends its own (p + 1 < history_len)
 * writes h after its window to hcarry.  carry_in requires p in [1, history_len - 1] (else D2D_EINVAL) and the
 * previous launch on hcarry to have been slot - 1 of the same buffer, batch and weights (the caller's sequence).
 * Actions, log-probs and values are bitwise those of d2d_policy_gru (the same steps on the same h). */
int64_t d2d_gru_carry_floats(const d2d_gru_desc* desc);
int d2d_policy_gru_carry(const d2d_gru_desc* desc, int32_t T, const void* obs, int32_t slot, const void* forced,
                         uint32_t rng_step, int32_t deterministic, void* actions, float* out, float* hcarry,
                         int32_t carry_in, void* stream);

/* PPO.train_step's evaluate + loss + backward for GRU policies (ippo.py:178-217, d2d_ppo.py:183-216) and
 * the iPPO GRU critic's MSE (ippo.py:210-216) over every sample of the buffer (training windows, padded):
 * the gradients of all tensors above (overwritten) and stats [N][2] = (sum min-surrogate, sum entropy)
 * or (sum (V - R)^2, 0).  actions / logp_old / weight strides as d2d_ppo_actor_grad; weight = advantage
 * or M (kinds 0, 1), return target (kind 2).  obs_dim <= 31.  workspace: d2d_gru_grad_workspace floats. */
int64_t d2d_gru_grad_workspace(const d2d_gru_desc* desc, int32_t T);
int d2d_gru_grad(const d2d_gru_desc* desc, int32_t T, const void* obs, const void* actions, const float* logp_old,
                 const int64_t* logp_strides, const float* weight, const int64_t* weight_strides, float clip,
                 float beta, float scale, float* g_w_ih, float* g_w_hh, float* g_b_ih, float* g_b_hh, float* g_w1,
                 float* g_b1, float* g_w2, float* g_b2, float* stats, float* workspace, int64_t workspace_floats,
                 void* stream);

/* Process-wide tuning options (not part of the reference interface).
 * D2D_OPT_NT_STORES: 1 = write obs/state with non-temporal (streaming) stores.
 * D2D_OPT_POLICY_F32_MFMA: 1 = d2d_policy_mlp_step on v_mfma_f32_16x16x4_f32 instead of the
 *   default exact-split bf16 MFMA kernel (both fp32-accurate; for A/B timing and tests).
 * D2D_OPT_GRU_GRAD_HISTORY: 1 = d2d_gru_grad accumulates the weight gradients through the per-wave
 *   global row history also where the cooperative LDS path applies (ABI 9; A/B timing and tests).  It
 *   selects the workspace layout: set it before the d2d_gru_grad_workspace query that sizes the buffer
 *   (d2d_gru_grad re-checks the size against its own snapshot of the option and returns D2D_EINVAL
 *   for a buffer sized under the other setting).
 * D2D_OPT_POLICY_CRITIC_SPLIT: d2d_policy_mlp_step with a critic runs the actor and the critic value as two
 *   launches of the split kernel (1) or as one fused launch (0); the same arithmetic either way (bitwise
 *   identical actions, log-probs and values).  Default: policy_kernels.hip's D2D_POLICY_CRITIC_SPLIT.
 * D2D_OPT_CRITIC_GRAD_ROWS: 1 = d2d_ppo_critic_grad on the sample-on-rows kernel of rounds 2-4 (A/B; the same
 *   gradients within fp32 rounding); 0 (default) = the hidden-on-rows kernel (update_kernels.hip).
 * D2D_OPT_FUSED_SLICE: envs per workgroup of d2d_comb_policy_fused_step, 32 (0 = default) or 64 (A/B; the same
 *   results, bit for bit); other values D2D_EINVAL.
 * Options are process-wide words (relaxed atomics) read once per call. */
enum { D2D_OPT_NT_STORES = 1, D2D_OPT_POLICY_F32_MFMA = 2, D2D_OPT_GRU_GRAD_HISTORY = 3, D2D_OPT_POLICY_CRITIC_SPLIT = 4,
       D2D_OPT_CRITIC_GRAD_ROWS = 5, D2D_OPT_FUSED_SLICE = 6 };
int d2d_set_option(int32_t option, int32_t value);

const char* d2d_last_error(void);
int d2d_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* D2D_HIP_H */
