/*
 * oracle/nnue_cpu_simd.c — the CPU baseline: Stockfish 15.1 NNUE evaluation as
 * the engine itself runs it on an AVX2 host, restated with intrinsics.
 *
 *   TEST INFRASTRUCTURE (bench.py's cpu_baseline leg and tests/ only; the
 *   product never links it).  Same arithmetic as the scalar oracle
 *   (nnue_oracle.c), which the CPU tests hold it to bit for bit.
 *
 * What it mirrors from upstream (official-stockfish/Stockfish, SF 15.1):
 *   nnue_feature_transformer.h  update_accumulator / refresh: register tiles of
 *                               NumRegs = 16 ymm (256 int16 columns) per pass,
 *                               each weight row read once per tile; PSQT rows
 *                               as one 8 x int32 add; incremental updates
 *                               (acc_prev - removed rows + added rows) along
 *                               a game, refresh when the perspective's own
 *                               king moved;
 *                               transform: clamp / mullo / >> 7 / packus;
 *   layers/affine_transform.h   propagate with maddubs + madd (u8 x i8 -> i32;
 *                               inputs <= 126, so maddubs never saturates);
 *   layers/clipped_relu.h, sqr_clipped_relu.h, nnue_architecture.h tail.
 * Groups (include/fnnue.h FNNUE_GROUP_CHAIN / _STAR) carry accumulators
 * along a game (each ply from the previous one) or from a parent to each of
 * its 1-ply children, as the engine's StateInfo chain does.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "nnue_oracle.h"

#define S_MAX_HD 4096

typedef struct {
    int16_t acc[2][S_MAX_HD] __attribute__((aligned(32)));
    int32_t psq[2][O_PSQT_BUCKETS] __attribute__((aligned(32)));
    uint8_t board[64];
    int ksq[2];
    int ok;
} s_state;

/* ---- board ---- */
static void s_unpack(const uint8_t *p36, uint8_t *board, int *stm) {
    for (int s = 0; s < 64; ++s) board[s] = (p36[s >> 1] >> (4 * (s & 1))) & 15;
    *stm = p36[32];
}

/* piece count, or -1 for an invalid board (same rule as the scalar oracle) */
static int s_check(const uint8_t *board, int *wk, int *bk) {
    int n = 0, nwk = 0, nbk = 0;
    for (int s = 0; s < 64; ++s) {
        const int pc = board[s];
        if (!pc) continue;
        if (!((pc >= 1 && pc <= 6) || (pc >= 9 && pc <= 14))) return -1;
        ++n;
        if (pc == 6) { *wk = s; ++nwk; }
        if (pc == 14) { *bk = s; ++nbk; }
    }
    return (nwk != 1 || nbk != 1 || n > 32) ? -1 : n;
}

/* ---- feature transformer: register-tiled refresh / update ---- */
#define S_DEFINE_TILED(R)                                                                                  \
    static void s_rows_##R(const onet *n, const int16_t *start, const int *sub, int nsub, const int *add,  \
                           int nadd, int16_t *acc) {                                                       \
        const uint32_t hd = n->hd;                                                                         \
        for (uint32_t c = 0; c < hd; c += 16 * R) {                                                        \
            __m256i r[R];                                                                                  \
            for (int k = 0; k < R; ++k) r[k] = _mm256_loadu_si256((const __m256i *)(start + c + 16 * k)); \
            for (int i = 0; i < nsub; ++i) {                                                               \
                const int16_t *row = n->ft_w + (size_t)sub[i] * hd + c;                                    \
                for (int k = 0; k < R; ++k)                                                                \
                    r[k] = _mm256_sub_epi16(r[k], _mm256_loadu_si256((const __m256i *)(row + 16 * k)));    \
            }                                                                                              \
            for (int i = 0; i < nadd; ++i) {                                                               \
                const int16_t *row = n->ft_w + (size_t)add[i] * hd + c;                                    \
                for (int k = 0; k < R; ++k)                                                                \
                    r[k] = _mm256_add_epi16(r[k], _mm256_loadu_si256((const __m256i *)(row + 16 * k)));    \
            }                                                                                              \
            for (int k = 0; k < R; ++k) _mm256_storeu_si256((__m256i *)(acc + c + 16 * k), r[k]);         \
        }                                                                                                  \
    }
S_DEFINE_TILED(16)
S_DEFINE_TILED(8)
S_DEFINE_TILED(4)

/* The same with 512-bit registers (SF's x86-64-avx512 / -vnni512 builds, the
 * ones fishnet picks on an AVX-512 host: NumRegs = 16 zmm = 512 columns). */
#define S_AVX512 __attribute__((target("avx512f,avx512bw,avx512vnni,avx512dq,avx512vl")))
#define S_DEFINE_TILED512(R)                                                                                  \
    S_AVX512 static void s_rows512_##R(const onet *n, const int16_t *start, const int *sub, int nsub,        \
                                       const int *add, int nadd, int16_t *acc) {                             \
        const uint32_t hd = n->hd;                                                                            \
        for (uint32_t c = 0; c < hd; c += 32 * R) {                                                           \
            __m512i r[R];                                                                                     \
            for (int k = 0; k < R; ++k) r[k] = _mm512_loadu_si512((const void *)(start + c + 32 * k));      \
            for (int i = 0; i < nsub; ++i) {                                                                  \
                const int16_t *row = n->ft_w + (size_t)sub[i] * hd + c;                                       \
                for (int k = 0; k < R; ++k)                                                                   \
                    r[k] = _mm512_sub_epi16(r[k], _mm512_loadu_si512((const void *)(row + 32 * k)));         \
            }                                                                                                 \
            for (int i = 0; i < nadd; ++i) {                                                                  \
                const int16_t *row = n->ft_w + (size_t)add[i] * hd + c;                                       \
                for (int k = 0; k < R; ++k)                                                                   \
                    r[k] = _mm512_add_epi16(r[k], _mm512_loadu_si512((const void *)(row + 32 * k)));         \
            }                                                                                                 \
            for (int k = 0; k < R; ++k) _mm512_storeu_si512((void *)(acc + c + 32 * k), r[k]);              \
        }                                                                                                     \
    }
S_DEFINE_TILED512(16)
S_DEFINE_TILED512(8)

/* 1 = AVX-512 VNNI code paths (host supports them and FNNUE_CPU_ISA != "avx2"), 0 = AVX2 */
static int s_isa512 = -1;
static int s_use512(void) {
    if (s_isa512 < 0) {
        const char *e = getenv("FNNUE_CPU_ISA");
        __builtin_cpu_init();
        s_isa512 = !(e && strcmp(e, "avx2") == 0) && __builtin_cpu_supports("avx512bw") &&
                   __builtin_cpu_supports("avx512vnni");
    }
    return s_isa512;
}

/* acc = start - sum(rows sub) + sum(rows add) (int16 wrap); psq likewise (int32 wrap) */
static void s_apply(const onet *n, const int16_t *start, const int32_t *pstart, const int *sub, int nsub,
                    const int *add, int nadd, int16_t *acc, int32_t *psq) {
    if (s_isa512 && n->hd % 512 == 0) s_rows512_16(n, start, sub, nsub, add, nadd, acc);
    else if (s_isa512 && n->hd % 256 == 0) s_rows512_8(n, start, sub, nsub, add, nadd, acc);
    else if (n->hd % 256 == 0) s_rows_16(n, start, sub, nsub, add, nadd, acc);
    else if (n->hd % 128 == 0) s_rows_8(n, start, sub, nsub, add, nadd, acc);
    else s_rows_4(n, start, sub, nsub, add, nadd, acc);
    __m256i p = pstart ? _mm256_loadu_si256((const __m256i *)pstart) : _mm256_setzero_si256();
    for (int i = 0; i < nsub; ++i)
        p = _mm256_sub_epi32(p, _mm256_loadu_si256((const __m256i *)(n->psqt_w + (size_t)sub[i] * O_PSQT_BUCKETS)));
    for (int i = 0; i < nadd; ++i)
        p = _mm256_add_epi32(p, _mm256_loadu_si256((const __m256i *)(n->psqt_w + (size_t)add[i] * O_PSQT_BUCKETS)));
    _mm256_storeu_si256((__m256i *)psq, p);
}

static void s_refresh(const onet *n, const uint8_t *board, int persp, int ksq, int16_t *acc, int32_t *psq) {
    int f[32], nf = 0;
    for (int s = 0; s < 64; ++s)
        if (board[s]) f[nf++] = oracle_make_index(persp, s, board[s], ksq);
    s_apply(n, n->ft_bias, NULL, NULL, 0, f, nf, acc, psq);
}

/* ---- transform + layer stack ---- */
/* the 8 horizontal sums of v[0..7], in order */
static inline __m256i s_hsum8(const __m256i v[8]) {
    const __m256i t0 = _mm256_hadd_epi32(v[0], v[1]), t1 = _mm256_hadd_epi32(v[2], v[3]);
    const __m256i t2 = _mm256_hadd_epi32(v[4], v[5]), t3 = _mm256_hadd_epi32(v[6], v[7]);
    const __m256i u0 = _mm256_hadd_epi32(t0, t1), u1 = _mm256_hadd_epi32(t2, t3);
    return _mm256_add_epi32(_mm256_permute2x128_si256(u0, u1, 0x20), _mm256_permute2x128_si256(u0, u1, 0x31));
}

static inline int s_crelu(int32_t v) { const int x = v >> 6; return x < 0 ? 0 : (x > 127 ? 127 : x); }
static inline int s_sqr_crelu(int32_t v) {
    const long long q = (((long long)v * v) >> 12) / 128;
    return q > 127 ? 127 : (int)q;
}

/* transform + fc_0 with 512-bit registers: packus per 128-bit lane, then a
 * qword permute; fc_0 by VPDPBUSD (u8 x i8 dot products into int32, exact). */
S_AVX512 static void s_transform_fc0_512(const onet *n, const s_state *st, const int persp[2], const ostack *sk,
                                         uint8_t *x, int32_t *y) {
    const uint32_t hd = n->hd, half = hd / 2;
    const __m512i zero = _mm512_setzero_si512(), top = _mm512_set1_epi16(127);
    const __m512i fix = _mm512_set_epi64(7, 5, 3, 1, 6, 4, 2, 0);
    for (int p = 0; p < 2; ++p) {
        const int16_t *a = st->acc[persp[p]];
        for (uint32_t j = 0; j < half; j += 64) {
            __m512i s0a = _mm512_loadu_si512((const void *)(a + j));
            __m512i s0b = _mm512_loadu_si512((const void *)(a + j + 32));
            __m512i s1a = _mm512_loadu_si512((const void *)(a + half + j));
            __m512i s1b = _mm512_loadu_si512((const void *)(a + half + j + 32));
            s0a = _mm512_min_epi16(_mm512_max_epi16(s0a, zero), top);
            s0b = _mm512_min_epi16(_mm512_max_epi16(s0b, zero), top);
            s1a = _mm512_min_epi16(_mm512_max_epi16(s1a, zero), top);
            s1b = _mm512_min_epi16(_mm512_max_epi16(s1b, zero), top);
            const __m512i pa = _mm512_srli_epi16(_mm512_mullo_epi16(s0a, s1a), 7);
            const __m512i pb = _mm512_srli_epi16(_mm512_mullo_epi16(s0b, s1b), 7);
            _mm512_storeu_si512((void *)(x + p * half + j),
                                _mm512_permutexvar_epi64(fix, _mm512_packus_epi16(pa, pb)));
        }
    }
    for (int i = 0; i < O_L2; ++i) {
        __m512i sum = _mm512_setzero_si512();
        const int8_t *w = sk->w0 + (size_t)i * hd;
        for (uint32_t j = 0; j < hd; j += 64)
            sum = _mm512_dpbusd_epi32(sum, _mm512_loadu_si512((const void *)(x + j)),
                                      _mm512_loadu_si512((const void *)(w + j)));
        y[i] = sk->b0[i] + _mm512_reduce_add_epi32(sum);
    }
}

/* transform + fc_0 with 256-bit registers (SF's AVX2 paths) */
static void s_transform_fc0_256(const onet *n, const s_state *st, const int persp[2], const ostack *sk,
                                uint8_t *x, int32_t *y) {
    const uint32_t hd = n->hd, half = hd / 2;
    const __m256i ones = _mm256_set1_epi16(1);
    const __m256i zero = _mm256_setzero_si256(), top = _mm256_set1_epi16(127);
    for (int p = 0; p < 2; ++p) {
        const int16_t *a = st->acc[persp[p]];
        for (uint32_t j = 0; j < half; j += 32) {
            __m256i s0a = _mm256_loadu_si256((const __m256i *)(a + j));
            __m256i s0b = _mm256_loadu_si256((const __m256i *)(a + j + 16));
            __m256i s1a = _mm256_loadu_si256((const __m256i *)(a + half + j));
            __m256i s1b = _mm256_loadu_si256((const __m256i *)(a + half + j + 16));
            s0a = _mm256_min_epi16(_mm256_max_epi16(s0a, zero), top);
            s0b = _mm256_min_epi16(_mm256_max_epi16(s0b, zero), top);
            s1a = _mm256_min_epi16(_mm256_max_epi16(s1a, zero), top);
            s1b = _mm256_min_epi16(_mm256_max_epi16(s1b, zero), top);
            const __m256i pa = _mm256_srli_epi16(_mm256_mullo_epi16(s0a, s1a), 7);
            const __m256i pb = _mm256_srli_epi16(_mm256_mullo_epi16(s0b, s1b), 7);
            const __m256i packed = _mm256_permute4x64_epi64(_mm256_packus_epi16(pa, pb), 0xD8);
            _mm256_store_si256((__m256i *)(x + p * half + j), packed);
        }
    }
    for (int g = 0; g < O_L2; g += 8) {
        __m256i sums[8];
        for (int k = 0; k < 8; ++k) sums[k] = _mm256_setzero_si256();
        for (uint32_t j = 0; j < hd; j += 32) {
            const __m256i xv = _mm256_load_si256((const __m256i *)(x + j));
            for (int k = 0; k < 8; ++k) {
                const __m256i w = _mm256_loadu_si256((const __m256i *)(sk->w0 + (size_t)(g + k) * hd + j));
                sums[k] = _mm256_add_epi32(sums[k], _mm256_madd_epi16(_mm256_maddubs_epi16(xv, w), ones));
            }
        }
        _mm256_store_si256((__m256i *)(y + g),
                           _mm256_add_epi32(s_hsum8(sums), _mm256_loadu_si256((const __m256i *)(sk->b0 + g))));
    }
}

static void s_propagate(const onet *n, const s_state *st, int stm, int cnt, int32_t *psqt_out, int32_t *pos_out) {
    const uint32_t hd = n->hd;
    const int bucket = (cnt - 1) / 4;
    const int persp[2] = { stm, 1 - stm };
    *psqt_out = (int32_t)((uint32_t)st->psq[persp[0]][bucket] - (uint32_t)st->psq[persp[1]][bucket]) / 2;
    uint8_t x[S_MAX_HD] __attribute__((aligned(64)));
    const ostack *sk = &n->st[bucket];
    const __m256i ones = _mm256_set1_epi16(1);
    int32_t y[O_L2] __attribute__((aligned(32)));
    if (s_isa512 && hd % 128 == 0) s_transform_fc0_512(n, st, persp, sk, x, y);
    else s_transform_fc0_256(n, st, persp, sk, x, y);
    uint8_t x1[O_FC1_IN] __attribute__((aligned(32)));
    for (int i = 0; i < O_L2 - 1; ++i) { x1[i] = (uint8_t)s_sqr_crelu(y[i]); x1[15 + i] = (uint8_t)s_crelu(y[i]); }
    x1[30] = x1[31] = 0;
    const __m256i x1v = _mm256_load_si256((const __m256i *)x1);
    int32_t z[O_L3] __attribute__((aligned(32)));
    for (int g = 0; g < O_L3; g += 8) {
        __m256i m[8];
        for (int k = 0; k < 8; ++k) {
            const __m256i w = _mm256_loadu_si256((const __m256i *)(sk->w1 + (g + k) * O_FC1_IN));
            m[k] = _mm256_madd_epi16(_mm256_maddubs_epi16(x1v, w), ones);
        }
        _mm256_store_si256((__m256i *)(z + g),
                           _mm256_add_epi32(s_hsum8(m), _mm256_loadu_si256((const __m256i *)(sk->b1 + g))));
    }
    int32_t out = sk->b2;
    for (int j = 0; j < O_L3; ++j) out += (int32_t)sk->w2[j] * s_crelu(z[j]);
    *pos_out = out + (int32_t)(((int64_t)y[O_L2 - 1] * (600 * 16)) / (127 * 64));
}

/* ---- one position: from scratch, or incrementally from `base` ---- */
static int s_eval_from(const onet *n, const uint8_t *p36, const s_state *base, s_state *st, int32_t *ps, int32_t *po) {
    int stm, wk = -1, bk = -1;
    s_unpack(p36, st->board, &stm);
    const int cnt = s_check(st->board, &wk, &bk);
    st->ok = cnt >= 0 && (stm == 0 || stm == 1);
    if (!st->ok) { *ps = 0; *po = 0; return -1; }
    st->ksq[0] = wk;
    st->ksq[1] = bk;
    for (int c = 0; c < 2; ++c) {
        if (!base || !base->ok || base->ksq[c] != st->ksq[c]) {  /* own king moved: refresh */
            s_refresh(n, st->board, c, st->ksq[c], st->acc[c], st->psq[c]);
            continue;
        }
        int sub[64], add[64], ns = 0, na = 0;
        for (int s = 0; s < 64; ++s) {
            const int a = base->board[s], b = st->board[s];
            if (a == b) continue;
            if (a) sub[ns++] = oracle_make_index(c, s, a, st->ksq[c]);
            if (b) add[na++] = oracle_make_index(c, s, b, st->ksq[c]);
        }
        if (ns + na >= cnt) s_refresh(n, st->board, c, st->ksq[c], st->acc[c], st->psq[c]);
        else s_apply(n, base->acc[c], base->psq[c], sub, ns, add, na, st->acc[c], st->psq[c]);
    }
    s_propagate(n, st, stm, cnt, ps, po);
    return 0;
}

/* ---- threaded drivers ---- */
typedef struct {
    const onet *n;
    const uint8_t *packed;
    const uint32_t *off;  /* NULL: independent positions */
    int mode;
    size_t b, e;          /* positions, or groups when off != NULL */
    int32_t *ps, *po;
    int rc;
} s_job;

static void *s_worker(void *arg) {
    s_job *j = (s_job *)arg;
    s_state *st = (s_state *)aligned_alloc(64, (2 * sizeof(s_state) + 63) & ~(size_t)63);
    if (!st) { j->rc = -2; return NULL; }
    int bad = 0;
    if (!j->off) {
        for (size_t i = j->b; i < j->e; ++i)
            bad |= s_eval_from(j->n, j->packed + 36 * i, NULL, st, &j->ps[i], &j->po[i]) != 0;
    } else {
        for (size_t g = j->b; g < j->e; ++g) {
            const size_t lo = j->off[g], hi = j->off[g + 1];
            for (size_t i = lo; i < hi; ++i) {
                /* CHAIN: ply k from ply k-1 (st[] ping-pong); STAR: children from the parent in st[0] */
                const size_t k = i - lo;
                const s_state *base = k == 0 ? NULL : j->mode == 0 ? &st[(k - 1) & 1] : &st[0];
                s_state *dst = k == 0 ? &st[0] : j->mode == 0 ? &st[k & 1] : &st[1];
                bad |= s_eval_from(j->n, j->packed + 36 * i, base, dst, &j->ps[i], &j->po[i]) != 0;
            }
        }
    }
    free(st);
    j->rc = bad ? -1 : 0;
    return NULL;
}

static int s_run(const onet *n, const uint8_t *packed, const uint32_t *off, int mode, size_t count, int32_t *ps,
                 int32_t *po, int threads) {
    if (n->hd > S_MAX_HD || n->hd % 64) return -3;
    s_use512();
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    s_job jobs[256];
    const size_t per = (count + threads - 1) / threads;
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        const size_t b = (size_t)t * per, e = b + per > count ? count : b + per;
        if (b >= e) break;
        jobs[t] = (s_job){ n, packed, off, mode, b, e, ps, po, 0 };
        pthread_create(&tid[t], NULL, s_worker, &jobs[t]);
        ++started;
    }
    int rc = 0;
    for (int t = 0; t < started; ++t) {
        pthread_join(tid[t], NULL);
        if (jobs[t].rc) rc = rc ? rc : jobs[t].rc;
    }
    return rc;
}

/* Independent positions, accumulators from scratch (BASELINE config 2). */
int cpu_simd_eval_packed(const onet *n, const uint8_t *packed, size_t count, int32_t *psqt, int32_t *positional,
                         int threads) {
    return s_run(n, packed, NULL, 0, count, psqt, positional, threads);
}

/* Groups (mode 0 = CHAIN: each position from the previous one; 1 = STAR: each
 * from the group's first), threads split the groups (configs 3 and 4). */
int cpu_simd_eval_groups(const onet *n, const uint8_t *packed, const uint32_t *off, size_t ngroups, int mode,
                         int32_t *psqt, int32_t *positional, int threads) {
    if (mode != 0 && mode != 1) return -3;
    return s_run(n, packed, off, mode, ngroups, psqt, positional, threads);
}

/* ---- whole analysis batches: expansion + evaluation (bench.py --workload backend) ----
 * What the reference's host does per acquired batch, restated: parse the root
 * FEN, play the UCI moves one by one (IncomingBatch::from_acquired, [ref]
 * src/queue.rs:571-606; here the oracle's own minimal board code, without the
 * legality checks shakmaty makes, so the baseline is if anything flattered),
 * then evaluate every ply with accumulators carried along the game (the
 * engine's StateInfo chain).  Game g's FEN is text[fen_off[g] .. mv_off[g]),
 * its moves text[mv_off[g] .. fen_off[g + 1]); its results go to
 * ps/po[out_off[g] ..] (out_off[g + 1] - out_off[g] = plies).  Threads split
 * the games. */
typedef struct {
    const onet *n;
    const char *text;
    const uint32_t *fen_off, *mv_off, *out_off;
    size_t b, e;
    int32_t *ps, *po;
    int rc;
} s_games_job;

static void s_pack(const uint8_t *board, int stm, uint8_t *p36) {
    for (int i = 0; i < 32; ++i) p36[i] = (uint8_t)(board[2 * i] | (board[2 * i + 1] << 4));
    p36[32] = (uint8_t)stm;
    p36[33] = p36[34] = p36[35] = 0;
}

static void *s_games_worker(void *arg) {
    s_games_job *j = (s_games_job *)arg;
    s_state *st = (s_state *)aligned_alloc(64, (2 * sizeof(s_state) + 63) & ~(size_t)63);
    char *fen = (char *)malloc(256);
    if (!st || !fen) { free(st); free(fen); j->rc = -2; return NULL; }
    int bad = 0;
    for (size_t g = j->b; g < j->e && !bad; ++g) {
        const uint32_t f0 = j->fen_off[g], m0 = j->mv_off[g], end = j->fen_off[g + 1];
        const uint32_t flen = m0 - f0 < 255 ? m0 - f0 : 255;
        memcpy(fen, j->text + f0, flen);
        fen[flen] = 0;
        uint8_t board[64], p36[36];
        int stm, ep;
        if (oracle_board_from_fen(fen, board, &stm, &ep)) { bad = 1; break; }
        const uint32_t o = j->out_off[g], nply = j->out_off[g + 1] - o;
        uint32_t k = 0, p = m0;
        for (;;) {
            s_pack(board, stm, p36);
            const s_state *base = k == 0 ? NULL : &st[(k - 1) & 1];
            bad |= s_eval_from(j->n, p36, base, &st[k & 1], &j->ps[o + k], &j->po[o + k]) != 0;
            if (++k >= nply) break;
            while (p < end && j->text[p] == ' ') ++p;
            char tok[8];
            int len = 0;
            while (p < end && j->text[p] != ' ') {
                if (len < 7) tok[len++] = j->text[p];
                ++p;
            }
            tok[len] = 0;
            if (!len || oracle_apply_uci(board, &stm, &ep, tok)) { bad = 1; break; }
        }
    }
    free(fen);
    free(st);
    j->rc = bad ? -1 : 0;
    return NULL;
}

int cpu_simd_eval_games(const onet *n, const char *text, const uint32_t *fen_off, const uint32_t *mv_off,
                        size_t ngames, const uint32_t *out_off, int32_t *psqt, int32_t *positional, int threads) {
    if (n->hd > S_MAX_HD || n->hd % 64) return -3;
    s_use512();
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    s_games_job jobs[256];
    const size_t per = (ngames + threads - 1) / threads;
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        const size_t b = (size_t)t * per, e = b + per > ngames ? ngames : b + per;
        if (b >= e) break;
        jobs[t] = (s_games_job){ n, text, fen_off, mv_off, out_off, b, e, psqt, positional, 0 };
        pthread_create(&tid[t], NULL, s_games_worker, &jobs[t]);
        ++started;
    }
    int rc = 0;
    for (int t = 0; t < started; ++t) {
        pthread_join(tid[t], NULL);
        if (jobs[t].rc) rc = rc ? rc : jobs[t].rc;
    }
    return rc;
}

/* 1 if the AVX-512 VNNI paths are in use on this host (FNNUE_CPU_ISA=avx2 forces AVX2). */
int cpu_simd_isa512(void) { return s_use512(); }

/* Tests: select the AVX2 (0) or AVX-512 (1) paths; returns the ISA now in use
 * (AVX-512 only where the host has it).  Not thread-safe against running evals. */
int cpu_simd_set_isa(int isa512) {
    s_isa512 = -1;
    s_isa512 = isa512 && s_use512();
    return s_isa512;
}
