"""GPU diagnostic 2: determinism and batch-context dependence of variant evals."""
import sys
sys.path.insert(0, '.')
import numpy as np
import fishnet_amd as F
from oracle.oracle import VariantOracleNet

variant, hd = F.VARIANT_ATOMIC, 256
data = F.synthesize_variant_net(3, hd, variant)
ev = F.Evaluator(F.Net.from_bytes_variant(data, variant), 0)
on = VariantOracleNet(data, variant)
pos = F.random_vpositions(11 + hd, variant, 3000, 160)
a = ev.eval_vpositions(pos)
b = ev.eval_vpositions(pos)
print("deterministic", np.array_equal(a[0], b[0]), np.array_equal(a[1], b[1]))
ops, opo, rc = on.eval_packed(pos, threads=8)
bad = np.nonzero((a[0] != ops) | (a[1] != opo))[0]
print("bad", len(bad))
single = [ev.eval_vpositions(pos[i:i + 1]) for i in bad[:40]]
ok_single = sum(int(s[0][0] == ops[i] and s[1][0] == opo[i]) for s, i in zip(single, bad[:40]))
print("bad positions correct when evaluated alone:", ok_single, "of", min(40, len(bad)))
# same positions, different order
perm = np.random.default_rng(0).permutation(len(pos))
c = ev.eval_vpositions(pos[perm])
print("permuted batch bad", int(((c[0] != ops[perm]) | (c[1] != opo[perm])).sum()))
# only high-count positions
b8 = np.zeros((len(pos), 64), np.uint8); b8[:, 0::2] = pos[:, :32] & 15; b8[:, 1::2] = pos[:, :32] >> 4
cnt = (b8 != 0).sum(1)
for lo, hi in ((2, 8), (8, 16), (16, 33)):
    m = (cnt >= lo) & (cnt < hi)
    r = ev.eval_vpositions(pos[m])
    print(f"cnt [{lo},{hi}) alone: {m.sum()} positions, bad {int(((r[0] != ops[m]) | (r[1] != opo[m])).sum())}")
i = bad[0]
print("bad[0]", i, "cnt", cnt[i], "wk", int((b8[i] == 6).argmax()), "bk", int((b8[i] == 14).argmax()),
      "stm", pos[i][32], "gpu", a[0][i], a[1][i], "oracle", ops[i], opo[i], "alone", single[0][0][0], single[0][1][0])
print(b8[i].reshape(8, 8)[::-1])
