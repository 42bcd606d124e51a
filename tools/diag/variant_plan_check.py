"""GPU diagnostic: fetch the variant plan and check it on the host."""
import sys, ctypes as C
sys.path.insert(0, '.')
import numpy as np
import fishnet_amd as F
from fishnet_amd import _native as N
from oracle.oracle import variant_features

lib = N.lib
lib.fnnue_debug_variant_plan.argtypes = [C.c_void_p] * 2 + [C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t] + [C.c_void_p] * 4
variant, hd = F.VARIANT_ATOMIC, 256
ev = F.Evaluator(F.Net.from_bytes_variant(F.synthesize_variant_net(3, hd, variant), variant), 0)
pos = F.random_vpositions(11 + hd, variant, 3000, 160)
n = len(pos)
VB = 64 * 33 + 9
ctr = np.zeros(3 * VB + 16, np.uint32)
units = np.zeros((200, 4), np.int32)
items = np.zeros(2 * n, np.uint32)
flist = np.zeros((2 * n, 32), np.uint16)
perm = np.zeros(n, np.uint32)
bucket = np.zeros(n, np.uint8)
rc = lib.fnnue_debug_variant_plan(ev.handle, N.ptr(pos), n, N.ptr(ctr), len(ctr), N.ptr(units), len(units), N.ptr(items),
                                  N.ptr(flist), N.ptr(perm), N.ptr(bucket))
print("rc", rc, "nunits", ctr[3 * VB])
nu = int(ctr[3 * VB])
U = units[:nu]
print("units", U[:8].tolist())
cover = np.zeros(2 * n, int)
for kb, b, e, _ in U:
    cover[b:e] += 1
print("items covered once:", (cover == 1).all(), "min/max", cover.min(), cover.max())
print("perm is a permutation:", np.array_equal(np.sort(perm), np.arange(n)))
# check each item's list and record
b8 = np.zeros((n, 64), np.uint8); b8[:, 0::2] = pos[:, :32] & 15; b8[:, 1::2] = pos[:, :32] >> 4
cnt = (b8 != 0).sum(1)
inv = np.argsort(perm)  # position -> slot
bad = 0
seen = np.zeros((n, 2), int)
for it in range(2 * n):
    rec = int(items[it]); nf = rec >> 24; bk = (rec >> 21) & 7; rowf = rec & 0x1FFFFF; slot, half = rowf >> 1, rowf & 1
    p = int(perm[slot]); stm = int(pos[p][32]); persp = stm if half == 0 else 1 - stm
    seen[p, persp] += 1
    kb = [u[0] for u in U if u[1] <= it < u[2]][0]
    ksq = int((b8[p] == (6 if persp == 0 else 14)).argmax())
    okb = ksq ^ 56 if persp else ksq
    want = sorted((f - 704 * okb) for f in variant_features(variant, pos[p], persp) if f - 704 * okb != 640 + okb)
    got = sorted(int(e) >> 4 for e in flist[it] if (int(e) >> 4) != 704)
    ok = kb == okb and got == want and nf == cnt[p] and bk == (cnt[p] - 1) // 4 and bucket[slot] == bk
    if not ok:
        bad += 1
        if bad <= 5:
            print("item", it, "slot", slot, "pos", p, "persp", persp, "kb", kb, okb, "nf", nf, cnt[p], "bk", bk, bucket[slot],
                  "lists equal", got == want, len(got), len(want))
print("bad items", bad, "every position twice:", (seen == 1).all())
# sortedness within units
srt = all(np.all(np.diff(items[b:e] >> 24) >= 0) for kb, b, e, _ in U)
print("n ascending within units:", srt)
