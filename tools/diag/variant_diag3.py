"""GPU diagnostic 3: is the failure tied to the atomic geometry or to low piece counts?"""
import sys
sys.path.insert(0, '.')
import numpy as np
import fishnet_amd as F
from oracle.oracle import VariantOracleNet

hd = 256
apos = F.random_vpositions(11 + hd, F.VARIANT_ATOMIC, 3000, 160)   # low counts, no hands
zpos = F.random_vpositions(11 + hd, F.VARIANT_CRAZYHOUSE, 3000, 160)
for variant, name in ((F.VARIANT_CRAZYHOUSE, "crazyhouse net"), (F.VARIANT_ATOMIC, "atomic net")):
    data = F.synthesize_variant_net(3, hd, variant)
    ev = F.Evaluator(F.Net.from_bytes_variant(data, variant), 0)
    on = VariantOracleNet(data, variant)
    for pname, pos in (("atomic walks", apos), ("crazyhouse walks, hands cleared", zpos)):
        pos = pos.copy()
        pos[:, 33:43] = 0
        b8 = np.zeros((len(pos), 64), np.uint8); b8[:, 0::2] = pos[:, :32] & 15; b8[:, 1::2] = pos[:, :32] >> 4
        ops, opo, rc = on.eval_packed(pos, threads=8)
        r = [ev.eval_vpositions(pos) for _ in range(2)]
        bad = (r[0][0] != ops) | (r[0][1] != opo)
        print(f"{name} on {pname}: rc {rc} psqt bad {(r[0][0] != ops).mean():.3f} pos bad {(r[0][1] != opo).mean():.3f} "
              f"repeat-equal {np.array_equal(r[0][1], r[1][1])} mean cnt {(b8 != 0).sum(1).mean():.1f}")
    ev.close()
