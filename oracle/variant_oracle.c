/*
 * oracle/variant_oracle.c — CPU restatement of Fairy-Stockfish's variant NNUE
 * (feature set "HalfKAv2 variants") for the 8x8 lichess variants, used ONLY
 * as the parity checker of the product's variant path.
 *
 *   TEST INFRASTRUCTURE (see nnue_oracle.c): only tests/ load this library.
 *
 * PARITY STATUS: "parity unpinned", twice over.  The reference drives every
 * variant with Fairy-Stockfish's classical eval (src/assets.rs:384-391
 * EngineFlavor::MultiVariant -> EvalFlavor::Hce; src/stockfish.rs:248-260
 * `Use NNUE false`), the Fairy-Stockfish/ submodule is empty and no variant
 * net is pinned.  This file restates the published
 * Fairy-Stockfish algorithm as recalled (src/nnue/features/
 * half_ka_v2_variants.{h,cpp}; the NNUE index tables built in variant.h
 * Variant::conclude):
 *
 *   nnueSquares = 64, nnuePockets = 2 * FILE_NB = 16 when the variant has
 *   pockets (crazyhouse) else 0, pieceTypes P N B R Q K (king last):
 *     pieceSquareIndex[c][own pt_i]   = 2i * 64,   [c][their pt_i] = (2i + 1) * 64,
 *     both kings: 2 * 5 * 64 = 640 (the king shares one plane),
 *     pieceHandIndex[c][own pt_i]     = 704 + 2i * 16,  their: 704 + (2i + 1) * 16,
 *     nnuePieceIndices K = 704 + 2 * 5 * 16 = 864 (pockets) or 704,
 *     kingSquareIndex[ksq] = ksq * K (all 64 squares are king squares).
 *   orient(perspective, s) = s for white, s ^ 56 (rank flip) for black; no
 *   horizontal mirroring (unlike HalfKAv2_hm).
 *   board feature  = orient(s) + pieceSquareIndex[persp][pc] + K * orient(ksq)
 *   hand feature k = k + pieceHandIndex[persp][pc] + K * orient(ksq), for the
 *                    k-th (0-based) piece of that type in that side's hand.
 *   The feature transformer hash is HalfKAv2's 0x5F234CB8 ^ (2 * HD); the
 *   layer stacks, transform, PSQT term and bucket (board pieces - 1) / 4 are
 *   the SF 15.1 ones of nnue_oracle.c (oracle_propagate).
 *
 * Packed variant position (include/fnnue.h fnnue_vpos, 48 bytes): 32 bytes of
 * board nibbles as fnnue_pos, stm, hand[10] = white P N B R Q, black P N B R Q.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "nnue_oracle.h"

#define OV_POS_BYTES 48
#define OV_BOARD_ROWS 704
#define OV_HAND_SLOTS 16

uint32_t oracle_variant_features(int variant) {
    if (variant == OV_CRAZYHOUSE) return 64 * (OV_BOARD_ROWS + 2 * 5 * OV_HAND_SLOTS);
    if (variant == OV_ATOMIC) return 64 * OV_BOARD_ROWS;
    return 0;
}

static int ov_rows(int variant) { return (int)oracle_variant_features(variant) / 64; }
static int ov_orient(int persp, int s) { return persp ? s ^ 56 : s; }

/* pieceSquareIndex[perspective][pc] / 64 */
static int ov_plane(int persp, int pc) {
    const int type = pc & 7, color = pc >> 3;
    if (type == 6) return 10;
    return 2 * (type - 1) + (color != persp);
}

int voracle_board_index(int variant, int persp, int s, int pc, int ksq) {
    return ov_orient(persp, s) + 64 * ov_plane(persp, pc) + ov_rows(variant) * ov_orient(persp, ksq);
}

/* color: owner of the hand piece (0 white, 1 black); pt: 1..5 (P..Q); k: 0-based ordinal */
int voracle_hand_index(int variant, int persp, int color, int pt, int k, int ksq) {
    return k + OV_BOARD_ROWS + (2 * (pt - 1) + (color != persp)) * OV_HAND_SLOTS + ov_rows(variant) * ov_orient(persp, ksq);
}

typedef struct { uint8_t board[64]; int stm; uint8_t hand[10]; int wk, bk, cnt; } ovpos;

/* Unpacks and validates; returns 0, -1 (invalid) or 1 (atomic game over: one
 * king exploded — no NNUE evaluation, the result is (0, 0); fishnet's atomic
 * games end with that position, [ref] src/queue.rs:586-600 sends every ply). */
static int ov_unpack(int variant, const uint8_t *p, ovpos *v) {
    int nwk = 0, nbk = 0, hand_total = 0;
    v->cnt = 0;
    for (int s = 0; s < 64; ++s) {
        const int pc = (p[s >> 1] >> (4 * (s & 1))) & 15;
        v->board[s] = (uint8_t)pc;
        if (!pc) continue;
        if (pc == 7 || pc == 8 || pc == 15) return -1;
        ++v->cnt;
        if (pc == 6) { v->wk = s; ++nwk; }
        if (pc == 14) { v->bk = s; ++nbk; }
    }
    v->stm = p[32];
    for (int i = 0; i < 10; ++i) {
        v->hand[i] = p[33 + i];
        if (v->hand[i] > OV_HAND_SLOTS) return -1;
        if (v->hand[i] && variant != OV_CRAZYHOUSE) return -1;
        hand_total += v->hand[i];
    }
    if (v->stm > 1 || v->cnt + hand_total > 32) return -1;
    if (variant == OV_ATOMIC && nwk + nbk == 1) return 1;
    if (nwk != 1 || nbk != 1) return -1;
    return 0;
}

/* Active features of one perspective (FeatureSet::append_active_indices). */
static int ov_features(int variant, const ovpos *v, int persp, int32_t *out) {
    const int ksq = persp ? v->bk : v->wk;
    int k = 0;
    for (int s = 0; s < 64; ++s)
        if (v->board[s]) out[k++] = voracle_board_index(variant, persp, s, v->board[s], ksq);
    for (int c = 0; c < 2; ++c)
        for (int pt = 1; pt <= 5; ++pt)
            for (int i = 0; i < v->hand[5 * c + pt - 1]; ++i)
                out[k++] = voracle_hand_index(variant, persp, c, pt, i, ksq);
    return k;
}

static void ov_refresh(const onet *n, const ovpos *v, int persp, int16_t *acc, int32_t *psq) {
    int32_t f[64];
    const int nf = ov_features(n->variant, v, persp, f);
    for (uint32_t j = 0; j < n->hd; ++j) acc[j] = n->ft_bias[j];
    for (int b = 0; b < O_PSQT_BUCKETS; ++b) psq[b] = 0;
    for (int i = 0; i < nf; ++i) {
        const int16_t *row = n->ft_w + (size_t)f[i] * n->hd;
        for (uint32_t j = 0; j < n->hd; ++j) acc[j] = (int16_t)(uint16_t)((uint16_t)acc[j] + (uint16_t)row[j]);
        for (int b = 0; b < O_PSQT_BUCKETS; ++b)
            psq[b] = (int32_t)((uint32_t)psq[b] + (uint32_t)n->psqt_w[(size_t)f[i] * O_PSQT_BUCKETS + b]);
    }
}

int voracle_eval(const onet *n, const uint8_t *p48, int32_t *psqt, int32_t *positional) {
    ovpos v;
    if (!n->variant) return -1;
    const int u = ov_unpack(n->variant, p48, &v);
    if (u) {
        *psqt = *positional = 0;
        return u > 0 ? 0 : -1;
    }
    int16_t acc[2][4096];
    int32_t psq[2][O_PSQT_BUCKETS];
    ov_refresh(n, &v, 0, acc[0], psq[0]);
    ov_refresh(n, &v, 1, acc[1], psq[1]);
    const int16_t *const a2[2] = { acc[0], acc[1] };
    const int32_t *const p2[2] = { psq[0], psq[1] };
    oracle_propagate(n, a2, p2, v.stm, (v.cnt - 1) / 4, psqt, positional);
    return 0;
}

/* Incremental accumulators along CHAIN (mode 0: previous position) / STAR
 * (mode 1: the group's first position) groups: for each perspective, add the
 * features present only in the new position and subtract those present only
 * in the base (feature-set difference, including pocket counts); refresh when
 * the perspective's king moved (HalfKAv2 variants requires_refresh) or there
 * is no valid base.  Mod 2^16 the result equals a refresh: the test of
 * incremental == refresh at the oracle level. */
static int cmp_i32(const void *a, const void *b) { int32_t x = *(const int32_t *)a, y = *(const int32_t *)b; return (x > y) - (x < y); }

int voracle_eval_groups(const onet *n, const uint8_t *packed, const uint32_t *off, size_t ngroups, int mode,
                        int32_t *psqt, int32_t *positional) {
    int16_t (*acc)[4096] = malloc(sizeof(int16_t) * 4 * 4096);  /* [persp][..] current, [2 + persp] base */
    int32_t psq[4][O_PSQT_BUCKETS];
    int bad = 0;
    for (size_t g = 0; g < ngroups; ++g) {
        ovpos base;
        int have = 0;
        for (uint32_t i = off[g]; i < off[g + 1]; ++i) {
            ovpos v;
            const int u = ov_unpack(n->variant, packed + (size_t)OV_POS_BYTES * i, &v);
            if (u) {
                psqt[i] = positional[i] = 0;
                if (u < 0) bad = 1;
                if (mode == 0 || i == off[g]) have = 0;
                continue;
            }
            for (int c = 0; c < 2; ++c) {
                const int ksq = c ? v.bk : v.wk, bksq = c ? base.bk : base.wk;
                if (!have || ksq != bksq) {
                    ov_refresh(n, &v, c, acc[c], psq[c]);
                    continue;
                }
                int32_t fa[64], fb[64];
                const int na = ov_features(n->variant, &v, c, fa), nb = ov_features(n->variant, &base, c, fb);
                qsort(fa, (size_t)na, 4, cmp_i32);
                qsort(fb, (size_t)nb, 4, cmp_i32);
                memcpy(acc[c], acc[2 + c], n->hd * sizeof(int16_t));
                memcpy(psq[c], psq[2 + c], sizeof psq[c]);
                int ia = 0, ib = 0;
                while (ia < na || ib < nb) {
                    int sign;
                    int32_t f;
                    if (ib >= nb || (ia < na && fa[ia] < fb[ib])) { f = fa[ia++]; sign = 1; }
                    else if (ia >= na || fb[ib] < fa[ia]) { f = fb[ib++]; sign = -1; }
                    else { ++ia; ++ib; continue; }
                    const int16_t *row = n->ft_w + (size_t)f * n->hd;
                    for (uint32_t j = 0; j < n->hd; ++j)
                        acc[c][j] = (int16_t)(uint16_t)((uint16_t)acc[c][j] + (uint16_t)(sign * row[j]));
                    for (int b = 0; b < O_PSQT_BUCKETS; ++b)
                        psq[c][b] = (int32_t)((uint32_t)psq[c][b] + (uint32_t)(sign * n->psqt_w[(size_t)f * O_PSQT_BUCKETS + b]));
                }
            }
            const int16_t *const a2[2] = { acc[0], acc[1] };
            const int32_t *const p2[2] = { psq[0], psq[1] };
            oracle_propagate(n, a2, p2, v.stm, (v.cnt - 1) / 4, &psqt[i], &positional[i]);
            if (mode == 0 || i == off[g]) {
                base = v;
                have = 1;
                memcpy(acc[2], acc[0], n->hd * sizeof(int16_t));
                memcpy(acc[3], acc[1], n->hd * sizeof(int16_t));
                memcpy(psq[2], psq[0], sizeof psq[0]);
                memcpy(psq[3], psq[1], sizeof psq[1]);
            }
        }
    }
    free(acc);
    return bad ? -1 : 0;
}

typedef struct { const onet *n; const uint8_t *p; size_t b, e; int32_t *ps, *po; int rc; } ov_job;
static void *ov_worker(void *arg) {
    ov_job *j = (ov_job *)arg;
    for (size_t i = j->b; i < j->e; ++i)
        if (voracle_eval(j->n, j->p + (size_t)OV_POS_BYTES * i, &j->ps[i], &j->po[i])) {
            j->ps[i] = j->po[i] = 0;
            j->rc = -1;
        }
    return NULL;
}

int voracle_eval_packed(const onet *n, const uint8_t *packed, size_t count, int32_t *psqt, int32_t *positional,
                        int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    ov_job jobs[256];
    const size_t per = (count + (size_t)threads - 1) / (size_t)threads;
    int started = 0, rc = 0;
    for (int t = 0; t < threads; ++t) {
        const size_t b = (size_t)t * per, e = b + per > count ? count : b + per;
        if (b >= e) break;
        jobs[t] = (ov_job){ n, packed, b, e, psqt, positional, 0 };
        pthread_create(&tid[t], NULL, ov_worker, &jobs[t]);
        ++started;
    }
    for (int t = 0; t < started; ++t) {
        pthread_join(tid[t], NULL);
        if (jobs[t].rc) rc = -1;
    }
    return rc;
}

/* Feature list of one perspective (tests: index known values, invariances). */
int voracle_features(int variant, const uint8_t *p48, int persp, int32_t *out) {
    ovpos v;
    if (ov_unpack(variant, p48, &v) != 0) return -1;
    return ov_features(variant, &v, persp, out);
}
