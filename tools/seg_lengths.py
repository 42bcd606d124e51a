import numpy as np, sys
sys.path.insert(0, '/root/repo')
import fishnet_amd as F
pos, off = F.random_playouts(1, 10000, 0, 160, mode=F.PLAYOUT_PLIES, threads=8)
b = np.zeros((len(pos), 64), np.uint8)
b[:, 0::2] = pos[:, :32] & 15
b[:, 1::2] = pos[:, :32] >> 4
wk = (b == 6).argmax(1); bk = (b == 14).argmax(1)
L = []
for c, ks in ((0, wk), (1, bk)):
    for g in range(len(off) - 1):
        a, e = off[g], off[g + 1]
        if e <= a: continue
        k = ks[a:e]
        starts = np.r_[0, np.nonzero(k[1:] != k[:-1])[0] + 1]
        ends = np.r_[starts[1:], e - a]
        L.extend((ends - starts).tolist())
L = np.array(L)
print("segments", len(L), "positions", L.sum(), "mean L", L.mean())
for t in (1, 2, 3, 4, 5, 8, 9, 16, 17, 32):
    print(t, (L == t).mean() if t < 9 else (L <= t).mean())
# executed position-steps: roots 1 + ceil((L-1)/8)*8 per item (waves of 8 items take the max in the pass; ignore)
steps = np.ceil((L - 1) / 8) * 8
print("useful delta positions", (L - 1).sum(), "executed (8-batches)", steps.sum(), "waste frac", 1 - (L - 1).sum() / steps.sum())
for bs in (1, 2, 4):
    st = np.ceil((L - 1) / bs) * bs
    print("batch", bs, "executed", st.sum(), "waste", 1 - (L - 1).sum() / st.sum())
