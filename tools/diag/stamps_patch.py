"""Writes tools/exp/diag_replay_stamps.patch against the working tree: s_memtime
stamps of game 0's replay phases in the one-wave kernel (FEN, tokenising, board
chain, check + pack, tail, game-end flags) into a device array read by
fnnue_diag_replay_stamps (tools/diag/replay_stamps.py; run it with
FNNUE_REPLAY_PAIR_MAX=0 so that every call takes the one-wave kernel).
Diagnostic builds only (tools/exp_build.sh)."""
import difflib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rw = os.path.join(ROOT, "fishnet_amd", "csrc", "replay_wave.h")
bh = os.path.join(ROOT, "fishnet_amd", "csrc", "builder.hip")
orig_rw, orig_bh = open(rw).read(), open(bh).read()


def sub(s, a, b):
    assert a in s, a
    return s.replace(a, b, 1)


s = orig_rw
s = sub(s, "constexpr int kTokRing = 128;", "__device__ unsigned long long g_stamp[8];\nconstexpr int kTokRing = 128;")
s = sub(s, "  const uint32_t nmoves = nply - 1;\n",
        "  const uint32_t nmoves = nply - 1;\n#ifndef STAMP_GAME\n#define STAMP_GAME 0\n#endif\n"
        "  const bool diag = g == STAMP_GAME && lane == 0;\n"
        "  unsigned long long T0 = __builtin_amdgcn_s_memtime(), Tk = T0, acc[6] = {0, 0, 0, 0, 0, 0};\n"
        "#define STAMP(i) do { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); acc[i] += n_ - Tk; "
        "Tk = n_; } while (0)\n")
# (the one-wave kernel, the file's first; FNNUE_REPLAY_PAIR_MAX=0 runs it for every call)
s = sub(s, "  // windows of up to 64 moves: tokenise, chain, check", "  STAMP(0);\n  // windows of up to 64 moves: tokenise, chain, check")
s = sub(s, "    tokenise<R>(t, text, e, TXT, TK, 64, lane);\n", "    tokenise<R>(t, text, e, TXT, TK, 64, lane);\n    STAMP(1);\n")
s = sub(s, "    const uint32_t kplay = chain<R>(sc, sqv, myc, k, win, SNAP, lane, mvw, scw);\n",
        "    const uint32_t kplay = chain<R>(sc, sqv, myc, k, win, SNAP, lane, mvw, scw);\n    STAMP(2);\n")
s = sub(s, "o0 + done + 1);\n", "o0 + done + 1);\n    STAMP(3);\n")
s = sub(s, "  if (final) {\n    reinterpret_cast<uint8_t*>(SNAP[0])[lane] = (uint8_t)sqv;",
        "  STAMP(4);\n  if (final) {\n    reinterpret_cast<uint8_t*>(SNAP[0])[lane] = (uint8_t)sqv;")
s = sub(s, "    if (lane == 0) final[g] = f;\n  }\n}\n",
        "    if (lane == 0) final[g] = f;\n  }\n  STAMP(5);\n  if (diag) {\n    for (int i = 0; i < 6; ++i) g_stamp[i] = acc[i];\n"
        "    g_stamp[6] = __builtin_amdgcn_s_memtime() - T0;\n    g_stamp[7] = nmoves;\n  }\n}\n")
b = sub(orig_bh, "hipError_t perft_device(",
        'extern "C" int fnnue_diag_replay_stamps(unsigned long long* out) {\n'
        "  return hipMemcpyFromSymbol(out, HIP_SYMBOL(replay::g_stamp), 64) == hipSuccess ? 0 : -1;\n}\n\n"
        "hipError_t perft_device(")
d = ""
for path, old, new in ((rw, orig_rw, s), (bh, orig_bh, b)):
    rel = os.path.relpath(path, ROOT)
    d += "".join(difflib.unified_diff(old.splitlines(True), new.splitlines(True), "a/" + rel, "b/" + rel))
open(os.path.join(ROOT, "tools", "exp", "diag_replay_stamps.patch"), "w").write(d)
print("tools/exp/diag_replay_stamps.patch")
