/*
 * oracle/nnue_oracle.c — CPU restatement of Stockfish 15.1 ("SFNNv5") NNUE
 * static evaluation, used ONLY as the parity checker.
 *
 *   TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's
 *   cpu_baseline leg may load this library.  The product (fishnet_amd/,
 *   libfnnue.so) never links, calls or falls back to it.
 *
 * PARITY STATUS: "parity unpinned".  The reference (schlawg/fishnet) drives
 * Stockfish over UCI (src/stockfish.rs:203-344) and the arithmetic lives in the
 * git submodule Stockfish/, which is EMPTY in /root/reference (.gitmodules:1-3).
 * The pinned net nn-ad9b42354671.nnue (build.rs:7) is absent as well, and the
 * reference has no tests or golden vectors.  This file is a
 * restatement of the published upstream algorithm (official-stockfish/
 * Stockfish, SF 15.1 tree) from the upstream file names cited per function.
 * What pins it instead: the .nnue header self-check (version + structure hash
 * chain, which a real net would have to match), color-flip / file-mirror
 * invariance, incremental == refresh, and perft on the product's board code.
 *
 * Scalar, portable C99; the only concession to speed is that the row-add loops
 * are written so gcc auto-vectorises them (the cpu_baseline leg times this
 * file with -O3 across host threads, kind "port").
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "nnue_oracle.h"


static uint32_t o_affine_hash(uint32_t prev, uint32_t out) {
    uint32_t h = O_AFFINE_HASH + out;
    h ^= prev >> 1;
    h ^= prev << 31;
    return h;
}

/* nnue_architecture.h Network::get_hash_value (fc_0, ac_0, fc_1, ac_1, fc_2) */
uint32_t oracle_net_hash(uint32_t hd) {
    uint32_t h = O_NET_HASH_BASE ^ (hd * 2);
    h = o_affine_hash(h, O_L2);
    h = O_CRELU_HASH + h;
    h = o_affine_hash(h, O_L3);
    h = O_CRELU_HASH + h;
    h = o_affine_hash(h, 1);
    return h;
}

/* nnue_feature_transformer.h: FeatureSet::HashValue ^ (OutputDimensions*2), OutputDimensions = HD */
uint32_t oracle_ft_hash(uint32_t hd) { return O_FT_HASH_BASE ^ (hd * 2); }
static uint32_t o_ft_hash_for(int variant, uint32_t hd) {
    return (variant ? O_FT_HASH_BASE_VARIANTS : O_FT_HASH_BASE) ^ (hd * 2);
}

/* ---- little-endian stream (nnue_common.h read_little_endian / read_leb_128) ---- */
typedef struct { const uint8_t *p; size_t n, off; int fail; } ostream;

static uint32_t rd_u32(ostream *s) {
    if (s->off + 4 > s->n) { s->fail = 1; return 0; }
    const uint8_t *q = s->p + s->off; s->off += 4;
    return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
}

/* Reads `count` signed integers of `bytes` width, either plain little-endian or
 * a COMPRESSED_LEB128 block (magic, u32 byte count, signed LEB128 values). */
static void rd_ints(ostream *s, int bytes, void *dst, size_t count) {
    const size_t ml = sizeof(O_LEB_MAGIC) - 1;
    if (s->off + ml <= s->n && memcmp(s->p + s->off, O_LEB_MAGIC, ml) == 0) {
        s->off += ml;
        uint32_t left = rd_u32(s);
        if (s->fail || s->off + left > s->n) { s->fail = 1; return; }
        const uint8_t *q = s->p + s->off;
        size_t pos = 0;
        for (size_t i = 0; i < count; ++i) {
            int64_t result = 0; unsigned shift = 0; uint8_t byte;
            do {
                if (pos >= left) { s->fail = 1; return; }
                byte = q[pos++];
                result |= (int64_t)(byte & 0x7f) << shift;
                shift += 7;
            } while ((byte & 0x80) && shift < (unsigned)bytes * 8 + 7);
            if (byte & 0x80) { s->fail = 1; return; }
            if (shift < 64 && (byte & 0x40)) result |= -((int64_t)1 << shift);
            if (bytes == 1) ((int8_t *)dst)[i] = (int8_t)result;
            else if (bytes == 2) ((int16_t *)dst)[i] = (int16_t)result;
            else ((int32_t *)dst)[i] = (int32_t)result;
        }
        if (pos != left) { s->fail = 1; return; }
        s->off += left;
        return;
    }
    if (s->off + (size_t)bytes * count > s->n) { s->fail = 1; return; }
    const uint8_t *q = s->p + s->off;
    for (size_t i = 0; i < count; ++i) {
        if (bytes == 1) ((int8_t *)dst)[i] = (int8_t)q[i];
        else if (bytes == 2) ((int16_t *)dst)[i] = (int16_t)(q[2 * i] | (q[2 * i + 1] << 8));
        else {
            uint32_t v = (uint32_t)q[4 * i] | ((uint32_t)q[4 * i + 1] << 8) |
                         ((uint32_t)q[4 * i + 2] << 16) | ((uint32_t)q[4 * i + 3] << 24);
            ((int32_t *)dst)[i] = (int32_t)v;
        }
    }
    s->off += (size_t)bytes * count;
}

void oracle_net_free(onet *n) {
    if (!n) return;
    free(n->desc); free(n->ft_bias); free(n->ft_w); free(n->psqt_w);
    for (int i = 0; i < O_STACKS; ++i) free(n->st[i].w0);
    free(n);
}

/* evaluate_nnue.cpp read_header + read_parameters; Detail::read_parameters
 * (per-component hash word); FeatureTransformer::read_parameters (biases,
 * weights, psqtWeights); AffineTransform::read_parameters (biases then
 * Output x PaddedInput weights); must end exactly at EOF.
 * Returns 0 on success, negative code on failure. */
int oracle_net_load_mem(const void *buf, size_t len, onet **out) {
    return oracle_net_load_variant_mem(buf, len, 0, out);
}

/* The same file format for Fairy-Stockfish variant nets: only the feature
 * set's hash and row count differ (variant 0 = chess HalfKAv2_hm). */
int oracle_net_load_variant_mem(const void *buf, size_t len, int variant, onet **out) {
    *out = NULL;
    const uint32_t nfeat = variant ? oracle_variant_features(variant) : O_FEATURES;
    if (!nfeat) return -1;
    ostream s = { (const uint8_t *)buf, len, 0, 0 };
    uint32_t version = rd_u32(&s), file_hash = rd_u32(&s), dlen = rd_u32(&s);
    if (s.fail || version != O_VERSION) return -2;
    if (s.off + dlen > len) return -3;
    onet *n = (onet *)calloc(1, sizeof(onet));
    n->desc = (char *)malloc(dlen + 1);
    memcpy(n->desc, s.p + s.off, dlen); n->desc[dlen] = 0; s.off += dlen;
    n->file_hash = file_hash;
    uint32_t fth = rd_u32(&s);
    uint32_t hd = (fth ^ (variant ? O_FT_HASH_BASE_VARIANTS : O_FT_HASH_BASE)) / 2;
    if (s.fail || hd == 0 || hd > 4096 || (hd % 128) != 0 || o_ft_hash_for(variant, hd) != fth) {
        oracle_net_free(n); return -4;
    }
    n->hd = hd;
    n->nfeat = nfeat;
    n->variant = variant;
    if ((o_ft_hash_for(variant, hd) ^ oracle_net_hash(hd)) != file_hash) { oracle_net_free(n); return -5; }
    n->ft_bias = (int16_t *)malloc(sizeof(int16_t) * hd);
    n->ft_w = (int16_t *)malloc(sizeof(int16_t) * (size_t)hd * nfeat);
    n->psqt_w = (int32_t *)malloc(sizeof(int32_t) * (size_t)O_PSQT_BUCKETS * nfeat);
    rd_ints(&s, 2, n->ft_bias, hd);
    rd_ints(&s, 2, n->ft_w, (size_t)hd * nfeat);
    rd_ints(&s, 4, n->psqt_w, (size_t)O_PSQT_BUCKETS * nfeat);
    if (s.fail) { oracle_net_free(n); return -6; }
    uint32_t nh = oracle_net_hash(hd);
    for (int b = 0; b < O_STACKS; ++b) {
        ostack *st = &n->st[b];
        if (rd_u32(&s) != nh || s.fail) { oracle_net_free(n); return -7; }
        st->w0 = (int8_t *)malloc((size_t)O_L2 * hd);
        rd_ints(&s, 4, st->b0, O_L2);
        rd_ints(&s, 1, st->w0, (size_t)O_L2 * hd);
        rd_ints(&s, 4, st->b1, O_L3);
        rd_ints(&s, 1, st->w1, O_L3 * O_FC1_IN);
        rd_ints(&s, 4, &st->b2, 1);
        rd_ints(&s, 1, st->w2, O_L3);
        if (s.fail) { oracle_net_free(n); return -8; }
    }
    if (s.off != len) { oracle_net_free(n); return -9; } /* stream.peek() == EOF */
    *out = n;
    return 0;
}

int oracle_net_load(const char *path, onet **out) {
    *out = NULL;
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END); long len = ftell(f); fseek(f, 0, SEEK_SET);
    if (len < 0) { fclose(f); return -1; }
    void *buf = malloc((size_t)len + 1);
    size_t got = fread(buf, 1, (size_t)len, f);
    fclose(f);
    if (got != (size_t)len) { free(buf); return -1; }
    int rc = oracle_net_load_mem(buf, (size_t)len, out);
    free(buf);
    return rc;
}

uint32_t oracle_net_hd(const onet *n) { return n->hd; }
uint32_t oracle_net_file_hash(const onet *n) { return n->file_hash; }
const char *oracle_net_desc(const onet *n) { return n->desc; }

/* ---- features/half_ka_v2_hm.{h,cpp} ----
 * Squares A1=0..H8=63; pieces W_PAWN=1..W_KING=6, B_PAWN=9..B_KING=14 (types.h). */
static const int O_KING_BUCKETS[64] = {
    -1, -1, -1, -1, 31, 30, 29, 28,
    -1, -1, -1, -1, 27, 26, 25, 24,
    -1, -1, -1, -1, 23, 22, 21, 20,
    -1, -1, -1, -1, 19, 18, 17, 16,
    -1, -1, -1, -1, 15, 14, 13, 12,
    -1, -1, -1, -1, 11, 10,  9,  8,
    -1, -1, -1, -1,  7,  6,  5,  4,
    -1, -1, -1, -1,  3,  2,  1,  0 };

/* PieceSquareIndex[perspective][piece] / 64: W=us, B=them; king shares plane 10. */
static int o_plane(int persp, int pc) {
    int type = pc & 7, color = pc >> 3;
    if (type == 6) return 10;
    return 2 * (type - 1) + (color != persp);
}

/* HalfKAv2_hm::orient: s ^ (persp * SQ_A8) ^ ((file_of(ksq) < FILE_E) * SQ_H1) */
static int o_orient(int persp, int s, int ksq) {
    return s ^ (persp ? 56 : 0) ^ (((ksq & 7) < 4) ? 7 : 0);
}

/* HalfKAv2_hm::make_index */
int oracle_make_index(int persp, int s, int pc, int ksq) {
    return o_orient(persp, s, ksq) + 64 * o_plane(persp, pc) + 704 * O_KING_BUCKETS[o_orient(persp, ksq, ksq)];
}

static int o_valid_piece(int pc) { return (pc >= 1 && pc <= 6) || (pc >= 9 && pc <= 14); }

/* Validates a 64-square board; returns piece count or -1. */
static int o_check_board(const uint8_t *board, int *wk, int *bk) {
    int n = 0, nwk = 0, nbk = 0;
    for (int s = 0; s < 64; ++s) {
        int pc = board[s];
        if (!pc) continue;
        if (!o_valid_piece(pc)) return -1;
        ++n;
        if (pc == 6) { *wk = s; ++nwk; }
        if (pc == 14) { *bk = s; ++nbk; }
    }
    if (nwk != 1 || nbk != 1 || n > 32) return -1;
    return n;
}

/* FeatureTransformer refresh (update_accumulator with no computed ancestor):
 * acc = biases + sum of weight rows (int16, wrapping); psqt = sum of psqt rows. */
static void o_refresh(const onet *n, const uint8_t *board, int persp, int ksq, int16_t *acc, int32_t *psqt) {
    const uint32_t hd = n->hd;
    for (uint32_t j = 0; j < hd; ++j) acc[j] = n->ft_bias[j];
    for (int b = 0; b < O_PSQT_BUCKETS; ++b) psqt[b] = 0;
    for (int s = 0; s < 64; ++s) {
        int pc = board[s];
        if (!pc) continue;
        size_t f = (size_t)oracle_make_index(persp, s, pc, ksq);
        const int16_t *row = n->ft_w + f * hd;
        for (uint32_t j = 0; j < hd; ++j) acc[j] = (int16_t)(uint16_t)((uint16_t)acc[j] + (uint16_t)row[j]);
        for (int b = 0; b < O_PSQT_BUCKETS; ++b)
            psqt[b] = (int32_t)((uint32_t)psqt[b] + (uint32_t)n->psqt_w[f * O_PSQT_BUCKETS + b]);
    }
}

/* layers/clipped_relu.h: clamp(v >> WeightScaleBits, 0, 127) */
static int o_crelu(int32_t v) { int x = v >> 6; return x < 0 ? 0 : (x > 127 ? 127 : x); }
/* layers/sqr_clipped_relu.h: min(127, ((long long)v*v >> (2*WeightScaleBits)) / 128) */
static int o_sqr_crelu(int32_t v) {
    long long q = (((long long)v * v) >> 12) / 128;
    return q > 127 ? 127 : (int)q;
}

/* Full static eval of one board: evaluate_nnue.cpp evaluate() up to (psqt, positional);
 * FeatureTransformer::transform; nnue_architecture.h Network::propagate.
 * Returns 0, or -1 for an invalid board. */
int oracle_eval_board(const onet *n, const uint8_t *board, int stm, int32_t *psqt_out, int32_t *pos_out) {
    int wk = -1, bk = -1;
    int cnt = o_check_board(board, &wk, &bk);
    if (cnt < 0 || (stm != 0 && stm != 1)) return -1;
    int16_t acc[2][4096];
    int32_t psq[2][O_PSQT_BUCKETS];
    if (n->variant) return -1;
    o_refresh(n, board, 0, wk, acc[0], psq[0]);
    o_refresh(n, board, 1, bk, acc[1], psq[1]);
    const int16_t *const a2[2] = { acc[0], acc[1] };
    const int32_t *const p2[2] = { psq[0], psq[1] };
    oracle_propagate(n, a2, p2, stm, (cnt - 1) / 4, psqt_out, pos_out);
    return 0;
}

void oracle_propagate(const onet *n, const int16_t *const acc[2], const int32_t *const psq[2], int stm, int bucket,
                      int32_t *psqt_out, int32_t *pos_out) {
    const uint32_t hd = n->hd;
    const int persp[2] = { stm, 1 - stm };
    /* transform(): psqt = (psqtAcc[stm][b] - psqtAcc[~stm][b]) / 2 (C truncation) */
    int32_t psqt = (int32_t)((uint32_t)psq[persp[0]][bucket] - (uint32_t)psq[persp[1]][bucket]) / 2;
    uint8_t x[4096];
    for (int p = 0; p < 2; ++p) {
        const int16_t *a = acc[persp[p]];
        for (uint32_t j = 0; j < hd / 2; ++j) {
            int s0 = a[j], s1 = a[j + hd / 2];
            s0 = s0 < 0 ? 0 : (s0 > 127 ? 127 : s0);
            s1 = s1 < 0 ? 0 : (s1 > 127 ? 127 : s1);
            x[p * (hd / 2) + j] = (uint8_t)(s0 * s1 / 128);
        }
    }
    const ostack *st = &n->st[bucket];
    int32_t y[O_L2];
    for (int i = 0; i < O_L2; ++i) {
        int32_t sum = st->b0[i];
        const int8_t *w = st->w0 + (size_t)i * hd;
        for (uint32_t j = 0; j < hd; ++j) sum += (int32_t)w[j] * (int32_t)x[j];
        y[i] = sum;
    }
    /* ac_sqr_0 -> [0,15), memcpy(ac_0 out) -> [15,30), [30,32) stay zero */
    uint8_t x1[O_FC1_IN];
    for (int i = 0; i < O_L2 - 1; ++i) { x1[i] = (uint8_t)o_sqr_crelu(y[i]); x1[15 + i] = (uint8_t)o_crelu(y[i]); }
    x1[30] = x1[31] = 0;
    uint8_t x2[O_L3];
    for (int i = 0; i < O_L3; ++i) {
        int32_t sum = st->b1[i];
        for (int j = 0; j < O_FC1_IN; ++j) sum += (int32_t)st->w1[i * O_FC1_IN + j] * (int32_t)x1[j];
        x2[i] = (uint8_t)o_crelu(sum);
    }
    int32_t out = st->b2;
    for (int j = 0; j < O_L3; ++j) out += (int32_t)st->w2[j] * (int32_t)x2[j];
    /* fwdOut = fc_0_out[15] * (600*OutputScale) / (127*(1<<WeightScaleBits)); 64-bit, see DESIGN.md */
    int32_t fwd = (int32_t)(((int64_t)y[O_L2 - 1] * (600 * 16)) / (127 * 64));
    *psqt_out = psqt;
    *pos_out = out + fwd;
}

/* ---- packed positions (include/fnnue.h fnnue_pos, 36 bytes) ---- */
static void o_unpack(const uint8_t *p36, uint8_t *board, int *stm) {
    for (int s = 0; s < 64; ++s) board[s] = (p36[s >> 1] >> (4 * (s & 1))) & 15;
    *stm = p36[32];
}

int oracle_eval_packed_range(const onet *n, const uint8_t *packed, size_t begin, size_t end,
                             int32_t *psqt, int32_t *positional) {
    int bad = 0;
    for (size_t i = begin; i < end; ++i) {
        uint8_t board[64]; int stm;
        o_unpack(packed + 36 * i, board, &stm);
        if (oracle_eval_board(n, board, stm, &psqt[i], &positional[i]) != 0) { psqt[i] = 0; positional[i] = 0; bad = 1; }
    }
    return bad ? -1 : 0;
}

typedef struct { const onet *n; const uint8_t *packed; size_t b, e; int32_t *ps, *po; int rc; } o_job;
static void *o_worker(void *arg) {
    o_job *j = (o_job *)arg;
    j->rc = oracle_eval_packed_range(j->n, j->packed, j->b, j->e, j->ps, j->po);
    return NULL;
}

/* Multi-threaded batch eval (cpu_baseline leg). */
int oracle_eval_packed(const onet *n, const uint8_t *packed, size_t count, int32_t *psqt, int32_t *positional, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256]; o_job jobs[256];
    size_t per = (count + threads - 1) / threads;
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        size_t b = (size_t)t * per, e = b + per > count ? count : b + per;
        if (b >= e) break;
        jobs[t] = (o_job){ n, packed, b, e, psqt, positional, 0 };
        pthread_create(&tid[t], NULL, o_worker, &jobs[t]);
        ++started;
    }
    int rc = 0;
    for (int t = 0; t < started; ++t) { pthread_join(tid[t], NULL); if (jobs[t].rc) rc = -1; }
    return rc;
}

/* ---- minimal board text handling (FEN placement + UCI move application) ----
 * Independent of the product's board code; no legality checks. Castling is
 * accepted both as king-two-squares (e1g1) and as king-takes-own-rook (Chess960
 * UCI, which fishnet sends: src/queue.rs:547, src/stockfish.rs:213). */
typedef struct { uint8_t board[64]; int stm; int ep; } oboard;

static int o_piece_from_char(char c) {
    const char *w = "PNBRQK", *b = "pnbrqk";
    for (int i = 0; i < 6; ++i) { if (c == w[i]) return i + 1; if (c == b[i]) return i + 9; }
    return 0;
}

int oracle_board_from_fen(const char *fen, uint8_t *board, int *stm, int *ep) {
    memset(board, 0, 64);
    int rank = 7, file = 0;
    const char *p = fen;
    for (; *p && *p != ' '; ++p) {
        if (*p == '/') { --rank; file = 0; continue; }
        if (*p >= '1' && *p <= '8') { file += *p - '0'; continue; }
        int pc = o_piece_from_char(*p);
        if (!pc || rank < 0 || file > 7) return -1;
        board[rank * 8 + file] = (uint8_t)pc; ++file;
    }
    while (*p == ' ') ++p;
    *stm = (*p == 'b') ? 1 : 0;
    if (*p) ++p;
    while (*p == ' ') ++p;
    while (*p && *p != ' ') ++p;     /* castling field: irrelevant to features */
    while (*p == ' ') ++p;
    *ep = -1;
    if (p[0] >= 'a' && p[0] <= 'h' && p[1] >= '1' && p[1] <= '8') *ep = (p[1] - '1') * 8 + (p[0] - 'a');
    return 0;
}

int oracle_apply_uci(uint8_t *board, int *stm, int *ep, const char *uci) {
    if (strlen(uci) < 4) return -1;
    int from = (uci[1] - '1') * 8 + (uci[0] - 'a');
    int to = (uci[3] - '1') * 8 + (uci[2] - 'a');
    if (from < 0 || from > 63 || to < 0 || to > 63) return -1;
    int pc = board[from];
    if (!pc || (pc >> 3) != *stm) return -1;
    int type = pc & 7, new_ep = -1;
    if (type == 6 && (board[to] == (uint8_t)((*stm << 3) | 4) ||
                      ((from >> 3) == (to >> 3) && ((from & 7) - (to & 7) == 2 || (to & 7) - (from & 7) == 2)))) {
        /* castling */
        int king_side;
        int rook_from;
        if (board[to] == (uint8_t)((*stm << 3) | 4)) { rook_from = to; king_side = (to & 7) > (from & 7); }
        else { king_side = (to & 7) > (from & 7); rook_from = (from & 56) | (king_side ? 7 : 0); }
        int rank = from & 56;
        int kto = rank | (king_side ? 6 : 2), rto = rank | (king_side ? 5 : 3);
        int rook = board[rook_from];
        board[from] = 0; board[rook_from] = 0;
        board[kto] = (uint8_t)pc; board[rto] = (uint8_t)rook;
    } else {
        if (type == 1 && to == *ep && board[to] == 0 && (from & 7) != (to & 7)) board[to + (*stm ? 8 : -8)] = 0;
        if (type == 1 && (from ^ to) == 16) new_ep = (from + to) / 2;
        board[from] = 0;
        if (type == 1 && uci[4]) {
            int pt = 0;
            switch (uci[4]) { case 'n': pt = 2; break; case 'b': pt = 3; break; case 'r': pt = 4; break; case 'q': pt = 5; break; default: return -1; }
            pc = (*stm << 3) | pt;
        }
        board[to] = (uint8_t)pc;
    }
    *ep = new_ep;
    *stm ^= 1;
    return 0;
}

/* Evaluate every position of a game: root FEN + space-separated UCI moves.
 * Writes n_moves+1 results; returns the count or a negative code. */
long oracle_eval_game(const onet *n, const char *fen, const char *moves, int32_t *psqt, int32_t *positional, long cap) {
    uint8_t board[64]; int stm, ep;
    if (oracle_board_from_fen(fen, board, &stm, &ep)) return -1;
    long k = 0;
    if (k >= cap || oracle_eval_board(n, board, stm, &psqt[k], &positional[k])) return -2;
    ++k;
    const char *p = moves;
    char tok[8];
    while (*p) {
        while (*p == ' ') ++p;
        if (!*p) break;
        int len = 0;
        while (p[len] && p[len] != ' ' && len < 7) { tok[len] = p[len]; ++len; }
        tok[len] = 0; p += len;
        while (*p && *p != ' ') ++p;
        if (oracle_apply_uci(board, &stm, &ep, tok)) return -3;
        if (k >= cap || oracle_eval_board(n, board, stm, &psqt[k], &positional[k])) return -4;
        ++k;
    }
    return k;
}

/* Debug/introspection helpers used by the tests. */
int oracle_features(const uint8_t *board, int persp, int32_t *out) {
    int wk = -1, bk = -1;
    if (o_check_board(board, &wk, &bk) < 0) return -1;
    int ksq = persp ? bk : wk, k = 0;
    for (int s = 0; s < 64; ++s) if (board[s]) out[k++] = oracle_make_index(persp, s, board[s], ksq);
    return k;
}

/* Returns the transformed feature vector (hd bytes) and L1 outputs for a board (for
 * clamp-regime coverage tests). */
int oracle_eval_trace(const onet *n, const uint8_t *board, int stm, uint8_t *x_out, int32_t *y_out, int16_t *acc_out) {
    int wk = -1, bk = -1;
    int cnt = o_check_board(board, &wk, &bk);
    if (cnt < 0) return -1;
    const uint32_t hd = n->hd;
    int16_t acc[2][4096]; int32_t psq[2][O_PSQT_BUCKETS];
    o_refresh(n, board, 0, wk, acc[0], psq[0]);
    o_refresh(n, board, 1, bk, acc[1], psq[1]);
    const int persp[2] = { stm, 1 - stm };
    for (int p = 0; p < 2; ++p) {
        const int16_t *a = acc[persp[p]];
        if (acc_out) memcpy(acc_out + p * hd, a, hd * sizeof(int16_t));
        for (uint32_t j = 0; j < hd / 2; ++j) {
            int s0 = a[j], s1 = a[j + hd / 2];
            s0 = s0 < 0 ? 0 : (s0 > 127 ? 127 : s0);
            s1 = s1 < 0 ? 0 : (s1 > 127 ? 127 : s1);
            x_out[p * (hd / 2) + j] = (uint8_t)(s0 * s1 / 128);
        }
    }
    const ostack *st = &n->st[(cnt - 1) / 4];
    for (int i = 0; i < O_L2; ++i) {
        int32_t sum = st->b0[i];
        for (uint32_t j = 0; j < hd; ++j) sum += (int32_t)st->w0[(size_t)i * hd + j] * (int32_t)x_out[j];
        y_out[i] = sum;
    }
    return (cnt - 1) / 4;
}
