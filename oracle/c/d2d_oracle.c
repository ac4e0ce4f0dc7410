/* TEST INFRASTRUCTURE ONLY — CPU checker and CPU baseline; never linked by
 * the product library (d2d-ppo_amd/).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it.
 *
 * Plain-C restatement of the reference environments over a batch of E envs,
 * one env per loop iteration (OpenMP over envs), with the same production
 * random stream as the HIP kernels (Philox4x32-10, oracle/philox.py) or
 * recorded draws (replay).  Follows:
 *   /root/reference/envs/combinatorial_env.py   reset 61-114, step 127-242
 *   /root/reference/envs/channel_selection_env.py reset 49-98, step 116-214
 * and is pinned against the numpy oracle (itself pinned to the reference's
 * golden vectors) by tests/test_c_oracle.py.
 *
 * Layout (unpacked, the natural CPU layout):
 *   buf  uint8 [E][N][D]   packets by slots-to-deadline (column 0 expires next)
 *   chan uint8 [E][N][C]   comb channel state (1 good);  chsel: uint8 [E][C+1]
 *   recv/disc uint32 [E][N], selq/seln uint32 [E] (chsel counters)
 *   obs  float [E][N][F]  prefix-compact rows; state float [E][S]
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define STREAM_FLIP 0u
#define STREAM_ARRIVAL 1u
#define STREAM_ACTION 2u
#define PER_ENV 0xFFFFFFFFu

typedef struct {
    int kind; /* 0 combinatorial, 1 channel selection */
    int N, C, D, F, S;
    const int32_t *d, *w, *state_off, *arr_kind; /* arr_kind: 0 Poisson every slot, 1 Bernoulli on schedule, 2 none */
    const double *lam, *p0, *period, *offset;
    const uint64_t *q_thr, *flip_thr; /* comb flip_thr [N*C], chsel [C+1] */
    uint64_t seed, env_base;
} OSpec;

static void philox(uint32_t c[4], uint64_t seed) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    }
}

static uint32_t word(const OSpec* s, uint64_t env, uint32_t agent, uint32_t step, uint32_t stream, int idx) {
    uint32_t c[4] = {(uint32_t)env, agent, step, (stream << 24) | (uint32_t)(idx >> 2)};
    philox(c, s->seed);
    return c[idx & 3];
}

static int poisson_inv(uint32_t r, double lam, double p0) {
    double u = (double)r * (1.0 / 4294967296.0);
    double p = p0, F = p;
    int x = 0;
    while (u >= F && x < 255) {
        x += 1;
        p = (p * lam) / (double)x;
        F = F + p;
    }
    return x;
}

static int draws_at(const OSpec* s, int k, int t) {
    int kk = s->arr_kind[k];
    if (kk == 0) return 1;
    if (kk == 1) return fmod((double)t, s->period[k]) == s->offset[k];
    return 0;
}

static int arrival(const OSpec* s, uint64_t env, int k, uint32_t step, const uint8_t* replay) {
    if (replay) return replay[k];
    uint32_t r = word(s, env, (uint32_t)k, step, STREAM_ARRIVAL, 0);
    if (s->arr_kind[k] == 0) return poisson_inv(r, s->lam[k], s->p0[k]);
    return (uint64_t)r < s->q_thr[k];
}

static void emit(const OSpec* s, const uint8_t* b, const uint8_t* chan_obs, const double* ack, const uint8_t* chan_now,
                 float* obs, float* state) {
    const int N = s->N, C = s->C, D = s->D, F = s->F;
    if (obs) {
        for (int k = 0; k < N; ++k) {
            float* o = obs + (size_t)k * F;
            int j = 0;
            for (int i = 0; i < s->w[k]; ++i) o[j++] = (float)b[k * D + i];
            if (s->kind == 0) {
                for (int c = 0; c < C; ++c) o[j++] = (float)chan_obs[k * C + c];
                for (int c = 0; c < C; ++c) o[j++] = (float)ack[c];
            } else {
                for (int c = 0; c <= C; ++c) o[j++] = (float)ack[c];
            }
            for (; j < F; ++j) o[j] = 0.f;
        }
    }
    if (state) {
        int j = 0;
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < s->d[k]; ++i) state[j++] = (float)b[k * D + i];
        if (s->kind == 0) {
            for (int i = 0; i < N * C; ++i) state[j++] = (float)chan_now[i];
            for (int c = 0; c < C; ++c) state[j++] = (float)ack[c];
        } else {
            for (int c = 0; c <= C; ++c) state[j++] = (float)chan_now[c];
        }
    }
}

static int nthreads_set(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

int oracle_reset(const OSpec* s, int E, uint32_t rng_step, const uint8_t* arr_replay, uint8_t* buf, uint8_t* chan,
                 uint32_t* recv, uint32_t* disc, uint32_t* selq, uint32_t* seln, float* obs, float* state,
                 int nthreads) {
    nthreads_set(nthreads);
    const int N = s->N, C = s->C, D = s->D;
    const int nch = s->kind == 0 ? N * C : C + 1;
#pragma omp parallel for schedule(static)
    for (int e = 0; e < E; ++e) {
        uint8_t* b = buf + (size_t)e * N * D;
        uint8_t* h = chan + (size_t)e * nch;
        memset(b, 0, (size_t)N * D);
        for (int k = 0; k < N; ++k) {
            int a = draws_at(s, k, 0) ? arrival(s, s->env_base + e, k, rng_step, arr_replay ? arr_replay + (size_t)e * N : 0) : 0;
            b[k * D + s->d[k] - 1] = (uint8_t)a;
            recv[(size_t)e * N + k] = (uint32_t)a;
            disc[(size_t)e * N + k] = 0;
        }
        memset(h, 1, (size_t)nch);
        if (selq) { selq[e] = 0; seln[e] = 0; }
        double ack[64];
        uint8_t ones[32 * 1024];
        if (s->kind == 0) {
            for (int c = 0; c < C; ++c) ack[c] = 1.0;
            memset(ones, 1, (size_t)N * C);
            emit(s, b, ones, ack, h, obs ? obs + (size_t)e * N * s->F : 0, state ? state + (size_t)e * s->S : 0);
        } else {
            for (int c = 0; c <= C; ++c) ack[c] = 0.0;
            emit(s, b, 0, ack, h, obs ? obs + (size_t)e * N * s->F : 0, state ? state + (size_t)e * s->S : 0);
        }
    }
    return 0;
}

int oracle_step(const OSpec* s, int E, int t, uint32_t rng_step, const uint8_t* actions, const uint8_t* flips_replay,
                const uint8_t* arr_replay, uint8_t* buf, uint8_t* chan, uint32_t* recv, uint32_t* disc, uint32_t* selq,
                uint32_t* seln, float* obs, float* state, int32_t* reward, double* ack_out, uint8_t* success,
                int nthreads) {
    nthreads_set(nthreads);
    const int N = s->N, C = s->C, D = s->D;
    const int nch = s->kind == 0 ? N * C : C + 1;
    if (N > 1024 || C > 32) return -1;
#pragma omp parallel for schedule(static)
    for (int e = 0; e < E; ++e) {
        uint8_t* b = buf + (size_t)e * N * D;
        uint8_t* h = chan + (size_t)e * nch;
        const uint8_t* act = actions + (size_t)e * (s->kind == 0 ? N * C : N);
        uint8_t hobs[32 * 1024];
        uint8_t succ[1024];
        double ack[64];
        int nsucc = 0;
        memcpy(hobs, h, (size_t)nch); /* obs carries the pre-evolve channel (combinatorial_env.py:145) */
        memset(succ, 0, (size_t)N);
        if (s->kind == 0) {
            int n_c[32] = {0}, g_c[32] = {0};
            for (int k = 0; k < N; ++k) {
                int has = 0;
                for (int i = 0; i < D; ++i) has |= b[k * D + i];
                for (int c = 0; c < C; ++c) {
                    int a = (act[k * C + c] != 0) && has;
                    n_c[c] += a;
                    g_c[c] += a && h[k * C + c];
                }
            }
            for (int c = 0; c < C; ++c) ack[c] = n_c[c] == 0 ? 0.0 : ((n_c[c] == 1 && g_c[c] == 1) ? 1.0 : -1.0);
            for (int k = 0; k < N; ++k) {
                int has = 0;
                for (int i = 0; i < D; ++i) has |= b[k * D + i];
                for (int c = 0; c < C && has; ++c)
                    if (act[k * C + c] && h[k * C + c] && ack[c] == 1.0) { succ[k] = 1; break; }
            }
        } else {
            int n_j[33] = {0};
            int att[1024];
            for (int k = 0; k < N; ++k) {
                int has = 0;
                for (int i = 0; i < D; ++i) has |= b[k * D + i];
                att[k] = has ? act[k] : 0;
                if (att[k] > 0 && att[k] <= C) n_j[att[k]]++;
            }
            ack[0] = 0.0;
            for (int j = 1; j <= C; ++j) {
                if (n_j[j] == 0) { ack[j] = 0.0; continue; }
                seln[e] += 1;
                if (h[j]) { selq[e] += 1; ack[j] = 1.0 / (double)n_j[j]; }
                else ack[j] = -1.0;
            }
            for (int k = 0; k < N; ++k) {
                int j = att[k];
                if (j > 0 && j <= C && n_j[j] == 1 && h[j]) succ[k] = 1;
            }
        }
        for (int k = 0; k < N; ++k) {
            if (!succ[k]) continue;
            ++nsucc;
            for (int i = 0; i < D; ++i)
                if (b[k * D + i]) { b[k * D + i] -= 1; break; }
        }
        /* evolve_buffer: expire column 0, shift left (combinatorial_env.py:120-124) */
        for (int k = 0; k < N; ++k) {
            disc[(size_t)e * N + k] += b[k * D];
            memmove(b + k * D, b + k * D + 1, (size_t)D - 1);
            b[k * D + D - 1] = 0;
        }
        /* evolve_channel (116-118 / 104-107) */
        if (s->kind == 0) {
            for (int k = 0; k < N; ++k)
                for (int c = 0; c < C; ++c) {
                    int f = flips_replay ? flips_replay[((size_t)e * N + k) * C + c]
                                         : (uint64_t)word(s, s->env_base + e, (uint32_t)k, rng_step, STREAM_FLIP, c) <
                                               s->flip_thr[k * C + c];
                    h[k * C + c] ^= (uint8_t)(f != 0);
                }
        } else {
            for (int j = 0; j <= C; ++j) {
                int f = flips_replay ? flips_replay[(size_t)e * (C + 1) + j]
                                     : (uint64_t)word(s, s->env_base + e, PER_ENV, rng_step, STREAM_FLIP, j) < s->flip_thr[j];
                h[j] ^= (uint8_t)(f != 0);
            }
        }
        /* arrivals (178-196 / 159-177) */
        for (int k = 0; k < N; ++k) {
            if (!draws_at(s, k, t)) continue;
            int a = arrival(s, s->env_base + e, k, rng_step, arr_replay ? arr_replay + (size_t)e * N : 0);
            b[k * D + s->d[k] - 1] = (uint8_t)a;
            recv[(size_t)e * N + k] += (uint32_t)a;
        }
        if (reward) reward[e] = nsucc;
        if (success) memcpy(success + (size_t)e * N, succ, (size_t)N);
        if (ack_out) {
            int na = s->kind == 0 ? C : C + 1;
            memcpy(ack_out + (size_t)e * na, ack, sizeof(double) * (size_t)na);
        }
        emit(s, b, hobs, ack, h, obs ? obs + (size_t)e * N * s->F : 0, state ? state + (size_t)e * s->S : 0);
    }
    return 0;
}

/* synthetic actions for the env-only benchmark: Bernoulli(thr / 2^32) per
 * (agent, channel) for comb (uint8 0/1 [E][N][C]); uniform channel id for chsel */
int oracle_sample_actions(const OSpec* s, int E, uint32_t rng_step, uint64_t thr, uint8_t* actions, int nthreads) {
    nthreads_set(nthreads);
    const int N = s->N, C = s->C;
#pragma omp parallel for schedule(static)
    for (int e = 0; e < E; ++e)
        for (int k = 0; k < N; ++k) {
            if (s->kind == 0) {
                for (int c = 0; c < C; ++c)
                    actions[((size_t)e * N + k) * C + c] =
                        (uint64_t)word(s, s->env_base + e, (uint32_t)k, rng_step, STREAM_ACTION, c) < thr;
            } else {
                uint32_t r = word(s, s->env_base + e, (uint32_t)k, rng_step, STREAM_ACTION, 0);
                actions[(size_t)e * N + k] = (uint8_t)(((uint64_t)r * (uint64_t)(C + 1)) >> 32);
            }
        }
    return 0;
}

int oracle_max_threads(void) { return nthreads_set(0); }
