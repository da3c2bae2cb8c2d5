import numpy as np
def read(path):
    a = np.fromfile(path, dtype=np.float64)
    k, out = 0, {}
    while k < len(a):
        fid, r, c = int(a[k]), int(a[k + 1]), int(a[k + 2])
        ids = a[k + 3:k + 3 + c].astype(int)
        k += 3 + c
        M = a[k:k + r * (c + 1)].reshape(r, c + 1)
        k += r * (c + 1)
        out[fid] = (ids, M)
    return out
G, Ov = read("gpurun_out/g.bin"), read("gpurun_out/o.bin")
print(len(G), len(Ov))
worst=[]
for fid in sorted(G):
    ig, Mg = G[fid]; io, Mo = Ov[fid]
    ids = sorted(set(ig) | set(io)); pos = {v: k for k, v in enumerate(ids)}
    def lift(i, M):
        A = np.zeros((M.shape[0], len(ids) + 1))
        for j, v in enumerate(i): A[:, pos[v]] += M[:, j]
        A[:, -1] = M[:, -1]
        return A
    Ag, Ao = lift(ig, Mg), lift(io, Mo)
    Gg, Go = Ag.T @ Ag, Ao.T @ Ao
    d = np.abs(Gg - Go)
    cd = d.max(axis=0) / (np.abs(Go).max(axis=0) + 1e-300)
    worst.append((cd.max(), fid, [(ids[k] if k < len(ids) else "r", "%.1e" % cd[k]) for k in np.argsort(-cd)[:5]], Mg.shape, Mo.shape))
worst.sort(key=lambda z: -z[0])
for w in worst[:6]: print(w)
print("median", np.median([w[0] for w in worst]))
