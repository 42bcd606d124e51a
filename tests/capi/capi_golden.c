/* capi_golden.c — the C ABI (include/fnnue.h) driven from plain C, with no
 * Python or torch in the process: the shape of the Rust FFI consumer that
 * would sit beside StockfishActor ([ref] src/stockfish.rs:23-54).
 *
 * Reads a text fixture (written by tests/test_capi_c.py from
 * tests/golden/golden_evals.json):
 *   <nnets>
 *   per net: <seed> <hd> <flags> <file_hash> <npos>, then npos lines
 *            "<72 hex chars = fnnue_pos> <psqt> <positional>"
 * and for every net: synthesizes it (fnnue_net_synthesize), checks its file
 * hash, evaluates the positions on GPU 0 through fnnue_eval_positions (both
 * feature-transformer implementations), fnnue_eval_groups (CHAIN over the
 * whole list and STAR pairs) and fnnue_multi (ndev = 1, RCCL broadcast), and
 * compares every result bit-exactly with the fixture.  Exit 0 = all equal. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/fnnue.h"

#define CK(x)                                                               \
  do {                                                                      \
    int rc_ = (x);                                                          \
    if (rc_) {                                                              \
      fprintf(stderr, "%s -> %d: %s\n", #x, rc_, fnnue_last_error());       \
      return 3;                                                             \
    }                                                                       \
  } while (0)

static int hexval(int c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }

static int compare(const char *what, size_t n, const int32_t *ps, const int32_t *po, const int32_t *eps,
                   const int32_t *epo) {
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i)
    if (ps[i] != eps[i] || po[i] != epo[i]) {
      if (bad < 3) fprintf(stderr, "%s: position %zu gives (%d, %d), expected (%d, %d)\n", what, i, ps[i], po[i],
                           eps[i], epo[i]);
      ++bad;
    }
  return bad != 0;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <fixture.txt>\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[1], "r");
  if (!f) return 2;
  int nnets = 0, failed = 0;
  if (fscanf(f, "%d", &nnets) != 1) return 2;
  for (int k = 0; k < nnets; ++k) {
    unsigned long long seed;
    unsigned hd, flags, fhash;
    size_t n;
    if (fscanf(f, "%llu %u %u %u %zu", &seed, &hd, &flags, &fhash, &n) != 5) return 2;
    fnnue_pos *pos = calloc(2 * n, sizeof(fnnue_pos));
    int32_t *eps = calloc(2 * n, 4), *epo = calloc(2 * n, 4), *ps = calloc(2 * n, 4), *po = calloc(2 * n, 4);
    uint32_t *off = calloc(n + 1, 4);
    char hex[80];
    for (size_t i = 0; i < n; ++i) {
      if (fscanf(f, "%79s %d %d", hex, &eps[i], &epo[i]) != 3 || strlen(hex) != 72) return 2;
      uint8_t *b = (uint8_t *)&pos[i];
      for (int j = 0; j < 36; ++j) b[j] = (uint8_t)(hexval(hex[2 * j]) << 4 | hexval(hex[2 * j + 1]));
    }
    void *buf;
    size_t len;
    CK(fnnue_net_synthesize(seed, hd, flags, &buf, &len));
    fnnue_net *net;
    CK(fnnue_net_load_mem(buf, len, &net));
    uint32_t got_hd, got_hash;
    CK(fnnue_net_info(net, &got_hd, &got_hash, NULL));
    if (got_hd != hd || got_hash != fhash) {
      fprintf(stderr, "net %d: hd %u hash %08x, fixture says %u %08x\n", k, got_hd, got_hash, hd, fhash);
      return 1;
    }
    fnnue_ctx *ctx;
    CK(fnnue_ctx_create(net, 0, &ctx));
    char what[64];
    for (int impl = FNNUE_FT_SLICED; impl <= FNNUE_FT_GATHER; ++impl) {
      CK(fnnue_ctx_set_ft_impl(ctx, impl));
      CK(fnnue_eval_positions(ctx, pos, n, ps, po));
      snprintf(what, sizeof what, "net %d positions impl %d", k, impl);
      failed |= compare(what, n, ps, po, eps, epo);
      off[0] = 0;
      off[1] = (uint32_t)n;  /* CHAIN: the whole list as one group (deltas or refreshes) */
      CK(fnnue_eval_groups(ctx, pos, n, off, 1, FNNUE_GROUP_CHAIN, ps, po));
      snprintf(what, sizeof what, "net %d chain impl %d", k, impl);
      failed |= compare(what, n, ps, po, eps, epo);
    }
    CK(fnnue_ctx_set_ft_impl(ctx, FNNUE_FT_SLICED));
    /* STAR pairs: (p, p) per group, the second derived from the first */
    for (size_t i = 0; i < n; ++i) {
      pos[n + i] = pos[i];
      off[i] = (uint32_t)(2 * i);
    }
    off[n] = (uint32_t)(2 * n);
    fnnue_pos *pairs = calloc(2 * n, sizeof(fnnue_pos));
    for (size_t i = 0; i < n; ++i) pairs[2 * i] = pairs[2 * i + 1] = pos[i];
    CK(fnnue_eval_groups(ctx, pairs, 2 * n, off, n, FNNUE_GROUP_STAR, ps, po));
    for (size_t i = 0; i < n; ++i) {
      int32_t a = ps[2 * i + 1], b = po[2 * i + 1];
      ps[i] = a;
      po[i] = b;
    }
    snprintf(what, sizeof what, "net %d star pairs", k);
    failed |= compare(what, n, ps, po, eps, epo);
    fnnue_ctx_free(ctx);
    int dev0 = 0;
    fnnue_multi *m;
    CK(fnnue_multi_create(net, &dev0, 1, &m));
    CK(fnnue_multi_eval_positions(m, pos, n, ps, po));
    snprintf(what, sizeof what, "net %d multi", k);
    failed |= compare(what, n, ps, po, eps, epo);
    fnnue_multi_free(m);
    fnnue_net_free(net);
    fnnue_buffer_free(buf);
    free(pairs);
    free(pos);
    free(eps);
    free(epo);
    free(ps);
    free(po);
    free(off);
    if (!failed) printf("net %d (hd %u): %zu positions bit-exact on 6 paths\n", k, hd, n);
  }
  fclose(f);
  printf(failed ? "FAILED\n" : "ok\n");
  return failed;
}
