/*
 * oracle/nnue_oracle.h — shared definitions of the CPU restatement (test
 * infrastructure only; see nnue_oracle.c): SF 15.1 constants and the parsed
 * net, used by the scalar oracle and by its vectorised twin nnue_cpu_simd.c.
 */
#ifndef FNNUE_ORACLE_H
#define FNNUE_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#define O_VERSION 0x7AF32F20u          /* nnue_common.h: Version                */
#define O_FT_HASH_BASE 0x7F234CB8u     /* half_ka_v2_hm.h: HashValue            */
#define O_NET_HASH_BASE 0xEC42E90Du    /* nnue_architecture.h: get_hash_value   */
#define O_AFFINE_HASH 0xCC03DAE4u      /* layers/affine_transform.h             */
#define O_CRELU_HASH 0x538D24C7u       /* layers/clipped_relu.h                 */
#define O_FEATURES 22528               /* half_ka_v2_hm.h: Dimensions = 64*11*64/2 */
#define O_PSQT_BUCKETS 8               /* nnue_architecture.h: PSQTBuckets      */
#define O_STACKS 8                     /* nnue_architecture.h: LayerStacks      */
#define O_L2 16                        /* FC_0_OUTPUTS + 1                      */
#define O_L3 32                        /* FC_1_OUTPUTS                          */
#define O_FC1_IN 32                    /* ceil_to_multiple(2*FC_0_OUTPUTS, 32)  */
#define O_LEB_MAGIC "COMPRESSED_LEB128" /* nnue_common.h: Leb128MagicString     */

typedef struct {
    int32_t b0[O_L2];
    int8_t *w0;                  /* [O_L2][hd]  row-major (file order)         */
    int32_t b1[O_L3];
    int8_t w1[O_L3 * O_FC1_IN];  /* [32][32]                                   */
    int32_t b2;
    int8_t w2[O_L3];
} ostack;

typedef struct {
    uint32_t hd;                 /* TransformedFeatureDimensions               */
    uint32_t nfeat;              /* feature rows: O_FEATURES, or a variant set  */
    int variant;                 /* 0 chess (HalfKAv2_hm), else OV_* below     */
    uint32_t file_hash;
    char *desc;
    int16_t *ft_bias;            /* [hd]                                       */
    int16_t *ft_w;               /* [nfeat][hd]                                */
    int32_t *psqt_w;             /* [nfeat][8]                                 */
    ostack st[O_STACKS];
} onet;

int oracle_make_index(int persp, int s, int pc, int ksq);
int oracle_eval_board(const onet *n, const uint8_t *board, int stm, int32_t *psqt_out, int32_t *pos_out);
int oracle_board_from_fen(const char *fen, uint8_t *board, int *stm, int *ep);
int oracle_apply_uci(uint8_t *board, int *stm, int *ep, const char *uci);

/* Shared by the chess and the variant restatements: FeatureTransformer::
 * transform + Network[bucket]::propagate from the two perspectives'
 * accumulators (acc[c] = perspective c's int16[hd], psq[c] its 8 PSQT sums). */
void oracle_propagate(const onet *n, const int16_t *const acc[2], const int32_t *const psq[2], int stm, int bucket,
                      int32_t *psqt_out, int32_t *pos_out);

/* ---- Fairy-Stockfish variant nets (variant_oracle.c) ---- */
#define OV_CRAZYHOUSE 1                /* HalfKAv2 variants, 8x8 + pockets: 64 x 864 */
#define OV_ATOMIC 2                    /* HalfKAv2 variants, 8x8, no pockets: 64 x 704 */
#define O_FT_HASH_BASE_VARIANTS 0x5F234CB8u /* HalfKAv2(Variants)::HashValue (recalled) */
uint32_t oracle_variant_features(int variant);
int oracle_net_load_variant_mem(const void *buf, size_t len, int variant, onet **out);

#endif
