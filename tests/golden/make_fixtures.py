"""Generates the committed fixtures under tests/golden/ (run in the build
container; inputs that only exist here are not needed at test time).

1. wcc_games.json — standard-start games from the World Championship PGN
   corpus shipped offline with networkx, SAN converted
   to UCI by the small resolver below.  Used as real-game inputs for the
   batch-expansion and incremental (CHAIN) parity tests, in the lichess wire
   shape {position, moves} of AcquireResponseBody ([ref] src/api.rs:293-309).
2. golden_evals.json — (psqt, positional) of the CPU oracle on seeded
   synthetic nets for fixed positions, plus a SHA-256 over a larger random
   playout set.  These freeze the oracle (regression pin); they are NOT
   Stockfish outputs — no Stockfish or real net exists here (parity unpinned).

Usage: python tests/golden/make_fixtures.py
"""
from __future__ import annotations

import bz2
import hashlib
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

PGN = "/opt/conda/share/doc/networkx-2.6.3/examples/drawing/chess_masters_WCC.pgn.bz2"
START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"

# ---- minimal SAN resolver (pseudo-legal generation + king-safety filter) ----
KN = [(1, 2), (2, 1), (2, -1), (1, -2), (-1, -2), (-2, -1), (-2, 1), (-1, 2)]
KG = [(a, b) for a in (-1, 0, 1) for b in (-1, 0, 1) if a or b]
RD = [(1, 0), (-1, 0), (0, 1), (0, -1)]
BD = [(1, 1), (1, -1), (-1, 1), (-1, -1)]


class Pos:
    def __init__(self):
        self.b = {}
        back = "RNBQKBNR"
        for f in range(8):
            self.b[(0, f)] = ("w", back[f])
            self.b[(1, f)] = ("w", "P")
            self.b[(6, f)] = ("b", "P")
            self.b[(7, f)] = ("b", back[f])
        self.stm = "w"
        self.ep = None
        self.castle = {"wK", "wQ", "bK", "bQ"}

    def attacks(self, sq, color):
        r, f = sq
        for dr, df in KN:
            if self.b.get((r + dr, f + df)) == (color, "N"):
                return True
        for dr, df in KG:
            if self.b.get((r + dr, f + df)) == (color, "K"):
                return True
        pr = -1 if color == "w" else 1
        for df in (-1, 1):
            if self.b.get((r + pr, f + df)) == (color, "P"):
                return True
        for dirs, kinds in ((RD, "RQ"), (BD, "BQ")):
            for dr, df in dirs:
                rr, ff = r + dr, f + df
                while 0 <= rr < 8 and 0 <= ff < 8:
                    p = self.b.get((rr, ff))
                    if p:
                        if p[0] == color and p[1] in kinds:
                            return True
                        break
                    rr += dr
                    ff += df
        return False

    def can_reach(self, frm, to, kind):
        (r0, f0), (r1, f1) = frm, to
        dr, df = r1 - r0, f1 - f0
        if kind == "N":
            return (dr, df) in KN
        if kind == "K":
            return (dr, df) in KG
        if kind in "RBQ":
            straight = dr == 0 or df == 0
            diag = abs(dr) == abs(df)
            if (kind == "R" and not straight) or (kind == "B" and not diag) or (kind == "Q" and not (straight or diag)):
                return False
            sr = (dr > 0) - (dr < 0)
            sf = (df > 0) - (df < 0)
            rr, ff = r0 + sr, f0 + sf
            while (rr, ff) != (r1, f1):
                if (rr, ff) in self.b:
                    return False
                rr += sr
                ff += sf
            return True
        return False

    def play(self, frm, to, promo=None):
        color, kind = self.b.pop(frm)
        if kind == "P" and to == self.ep and to not in self.b:
            self.b.pop((frm[0], to[1]), None)
        self.b[to] = (color, promo or kind)
        self.ep = ((frm[0] + to[0]) // 2, frm[1]) if kind == "P" and abs(to[0] - frm[0]) == 2 else None
        if kind == "K":
            self.castle -= {color + "K", color + "Q"}
        for sq, right in (((0, 0), "wQ"), ((0, 7), "wK"), ((7, 0), "bQ"), ((7, 7), "bK")):
            if frm == sq or to == sq:
                self.castle.discard(right)
        self.stm = "b" if self.stm == "w" else "w"

    def king(self, color):
        return next(s for s, p in self.b.items() if p == (color, "K"))

    def legal_after(self, frm, to, promo=None):
        saved = (dict(self.b), self.stm, self.ep, set(self.castle))
        color = self.stm
        self.play(frm, to, promo)
        ok = not self.attacks(self.king(color), "b" if color == "w" else "w")
        self.b, self.stm, self.ep, self.castle = saved
        return ok


def sq(name):
    return (int(name[1]) - 1, ord(name[0]) - 97)


def name(s):
    return chr(97 + s[1]) + str(s[0] + 1)


SAN = re.compile(r"^([NBRQK])?([a-h])?([1-8])?x?([a-h][1-8])(=?[NBRQ])?[+#]?$")


def san_to_uci(p: Pos, san: str) -> str:
    c = p.stm
    rank = 0 if c == "w" else 7
    s = san.rstrip("+#!?")
    if s in ("O-O", "O-O-O"):
        frm, to = (rank, 4), (rank, 6 if s == "O-O" else 2)
        p.play(frm, to)
        rf, rt = ((rank, 7), (rank, 5)) if s == "O-O" else ((rank, 0), (rank, 3))
        p.b[rt] = p.b.pop(rf)
        return name(frm) + name(to)
    m = SAN.match(s)
    if not m:
        raise ValueError(san)
    kind = m.group(1) or "P"
    to = sq(m.group(4))
    promo = m.group(5)[-1] if m.group(5) else None
    cands = []
    for frm, pc in list(p.b.items()):
        if pc != (c, kind):
            continue
        if m.group(2) and frm[1] != ord(m.group(2)) - 97:
            continue
        if m.group(3) and frm[0] != int(m.group(3)) - 1:
            continue
        if kind == "P":
            d = 1 if c == "w" else -1
            if frm[1] == to[1]:
                ok = to not in p.b and (to[0] - frm[0] == d or (
                    to[0] - frm[0] == 2 * d and frm[0] == (1 if c == "w" else 6) and (frm[0] + d, frm[1]) not in p.b))
            else:
                ok = abs(frm[1] - to[1]) == 1 and to[0] - frm[0] == d and (
                    (to in p.b and p.b[to][0] != c) or to == p.ep)
        else:
            ok = p.can_reach(frm, to, kind) and (to not in p.b or p.b[to][0] != c)
        if ok and p.legal_after(frm, to, promo):
            cands.append(frm)
    if len(cands) != 1:
        raise ValueError(f"ambiguous/illegal {san}: {cands}")
    frm = cands[0]
    p.play(frm, to, promo)
    return name(frm) + name(to) + (promo.lower() if promo else "")


def parse_pgn(text: str):
    games, headers, body = [], {}, []
    for line in text.splitlines() + [""]:
        if line.startswith("["):
            if body:
                games.append((headers, " ".join(body)))
                headers, body = {}, []
            k, v = line[1:-1].split(" ", 1)
            headers[k] = v.strip('"')
        elif line.strip():
            body.append(line.strip())
    if body:
        games.append((headers, " ".join(body)))
    return games


def convert_games(limit: int):
    text = bz2.open(PGN, "rt", errors="replace").read()
    out = []
    for headers, body in parse_pgn(text):
        if "FEN" in headers:
            continue
        body = re.sub(r"\{[^}]*\}", " ", body)
        body = re.sub(r"\d+\.(\.\.)?", " ", body)
        toks = [t for t in body.split() if t not in ("1-0", "0-1", "1/2-1/2", "*")]
        p = Pos()
        try:
            uci = [san_to_uci(p, t) for t in toks]
        except (ValueError, StopIteration, KeyError):
            continue
        if len(uci) < 10:
            continue
        out.append({"id": f"{headers.get('Event', '')} r{headers.get('Round', '')}", "position": START,
                    "moves": " ".join(uci)})
        if len(out) >= limit:
            break
    return out


def main():
    games = convert_games(60)
    with open(os.path.join(HERE, "wcc_games.json"), "w") as f:
        json.dump({"source": "networkx-2.6.3 examples chess_masters_WCC.pgn.bz2 (SAN->UCI by make_fixtures.py)",
                   "games": games}, f, indent=0)
    print(f"wrote {len(games)} games")

    import numpy as np
    import fishnet_amd as F
    from oracle.oracle import OracleNet
    from positions import FENS

    nets = [(1, 1024, 0), (7, 128, 0), (3, 1024, F._native.SYNTH_WRAP)]
    golden = {"note": "CPU-oracle outputs on synthetic nets (regression pin; parity unpinned vs Stockfish)",
              "nets": []}
    fen_pos = np.stack([F.pos_from_fen(x) for x in FENS])
    wcc = F.game_positions(games[0]["position"], games[0]["moves"])
    rnd = F.random_playouts(11, 64, threads=4)
    fixed = np.concatenate([fen_pos, wcc, rnd])
    big = F.random_playouts(1, 5000, threads=4)
    for seed, hd, flags in nets:
        on = OracleNet(F.synthesize_net(seed, hd, flags))
        ps, po, rc = on.eval_packed(fixed)
        assert rc == 0
        bps, bpo, rc = on.eval_packed(big, threads=4)
        assert rc == 0
        digest = hashlib.sha256(bps.astype("<i4").tobytes() + bpo.astype("<i4").tobytes()).hexdigest()
        golden["nets"].append({"seed": seed, "hd": hd, "flags": flags, "file_hash": on.file_hash,
                               "psqt": ps.tolist(), "positional": po.tolist(),
                               "playouts_seed": 1, "playouts_count": 5000, "playouts_sha256": digest})
    golden["positions_hex"] = [bytes(r).hex() for r in fixed]
    with open(os.path.join(HERE, "golden_evals.json"), "w") as f:
        json.dump(golden, f)
    print(f"wrote golden vectors for {len(fixed)} positions x {len(nets)} nets")


if __name__ == "__main__":
    main()
