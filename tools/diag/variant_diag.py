"""GPU diagnostic for the variant path: mismatch statistics against the oracle."""
import sys
sys.path.insert(0, '.')
import numpy as np
import fishnet_amd as F
from oracle.oracle import VariantOracleNet

for variant in (F.VARIANT_ATOMIC, F.VARIANT_CRAZYHOUSE):
    for hd in (256, 512):
        data = F.synthesize_variant_net(3, hd, variant)
        ev = F.Evaluator(F.Net.from_bytes_variant(data, variant), 0)
        on = VariantOracleNet(data, variant)
        pos = F.random_vpositions(11 + hd, variant, 3000, 160)
        ps, po = ev.eval_vpositions(pos)
        ev.set_swar(False)
        ps2, po2 = ev.eval_vpositions(pos)
        ops, opo, rc = on.eval_packed(pos, threads=8)
        b = np.zeros((len(pos), 64), np.uint8)
        b[:, 0::2] = pos[:, :32] & 15
        b[:, 1::2] = pos[:, :32] >> 4
        cnt = (b != 0).sum(1)
        bad_ps, bad_po = ps != ops, po != opo
        print(f"variant {variant} hd {hd}: psqt bad {bad_ps.mean():.3f} positional bad {bad_po.mean():.3f} "
              f"swar==packed {np.array_equal(ps, ps2) and np.array_equal(po, po2)} rc {rc}")
        for c in sorted(set(cnt.tolist())):
            m = cnt == c
            print(f"  cnt {c:2d}: n {m.sum():5d} psqt bad {bad_ps[m].mean():.2f} pos bad {bad_po[m].mean():.2f}")
        i = np.nonzero(bad_ps | bad_po)[0][:3]
        print("  first bad", i, ps[i], ops[i], po[i], opo[i])
        wk = (b == 6).argmax(1)
        bk = (b == 14).argmax(1)
        print("  bad by white king sq:", {int(k): round(float((bad_po[wk == k]).mean()), 2) for k in sorted(set(wk.tolist()))})
        ev.close()
