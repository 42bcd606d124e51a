"""Generates tests/golden/golden_variant_evals.json: (psqt, positional) of the
variant CPU restatement (oracle/variant_oracle.c) on seeded synthetic
Fairy-Stockfish HalfKAv2-variants nets, for fixed FENs with crazyhouse
holdings and atomic positions, plus a SHA-256 over a larger set of random
variant walks.  A regression pin of the restatement and of the device path
against it — NOT Fairy-Stockfish outputs: no Fairy-Stockfish source or
variant net exists offline (parity unpinned).

Usage: python tests/golden/make_variant_fixtures.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import fishnet_amd as F  # noqa: E402
from oracle.oracle import VariantOracleNet  # noqa: E402

FENS = {
    F.VARIANT_CRAZYHOUSE: [
        "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR[] w KQkq - 0 1",
        "r1bqkb1r/ppp2ppp/2n2n2/4p3/4P3/5N2/PPP2PPP/RNBQKB1R[Pp] w KQkq - 0 1",
        "r1bqk2r/pppp1ppp/2n2n2/2b5/2B5/2N2N2/PPPP1PPP/R1BQK2R/Nb b KQkq - 0 1",
        "r2qk2r/ppp2ppp/2n1bn2/3p4/1b1P4/2N2N2/PP3PPP/R1BQKB1R[PBp] w KQkq - 0 1",
        "4k3/8/8/8/8/8/8/4K3[QQRRBBNNPPPPPPPqqrrbbnnppppppp] b - - 0 1",
        "r3k2r/8/8/3pP3/8/8/8/R3K2R[PPpp] w KQkq d6 0 1",
    ],
    F.VARIANT_ATOMIC: [
        "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
        "rnbqkb1r/pppp1ppp/5n2/4p3/4P3/5N2/PPPP1PPP/RNBQKB1R w KQkq - 0 1",
        "r1b1k2r/ppp2ppp/2n5/3p4/8/2N5/PPP2PPP/R3KB1R b KQkq - 0 1",
        "4k3/8/8/8/8/8/8/4K3 w - - 0 1",
        "8/2p5/3k4/8/8/4K3/5P2/8 w - - 0 1",
    ],
}
NETS = [(F.VARIANT_CRAZYHOUSE, 11, 256), (F.VARIANT_CRAZYHOUSE, 12, 512), (F.VARIANT_ATOMIC, 13, 256),
        (F.VARIANT_ATOMIC, 14, 512)]
WALKS = 4000


def main():
    out = {"note": "variant CPU restatement outputs on synthetic nets (regression pin; parity unpinned)", "nets": []}
    for variant, seed, hd in NETS:
        data = F.synthesize_variant_net(seed, hd, variant)
        on = VariantOracleNet(data, variant)
        pos = np.stack([F.vpos_from_fen(variant, f) for f in FENS[variant]])
        ps, po, rc = on.eval_packed(pos, threads=4)
        assert rc == 0
        walks = F.random_vpositions(seed, variant, WALKS, 160)
        wps, wpo, rc = on.eval_packed(walks, threads=8)
        assert rc == 0
        digest = hashlib.sha256(wps.astype("<i4").tobytes() + wpo.astype("<i4").tobytes()).hexdigest()
        out["nets"].append({"variant": int(variant), "seed": seed, "hd": hd, "fens": FENS[variant],
                            "psqt": ps.tolist(), "positional": po.tolist(), "walks_seed": seed,
                            "walks_count": WALKS, "walks_max_plies": 160, "walks_sha256": digest})
    with open(os.path.join(HERE, "golden_variant_evals.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(out["nets"]), "nets")


if __name__ == "__main__":
    main()
