import numpy as np
p = np.load("gpurun_out/pack.npz"); b = np.load("gpurun_out/base.npz")
def rep(name, x, y):
    d = np.abs(x - y); m = d.reshape(-1, 4).max(1) > 0
    print(f"{name}: px differ {m.sum()} max {d.max():.3g}  alpha(count) differs {(np.abs(x[...,3]-y[...,3])>0).sum()}")
    return m
rep("lit base vs pack", b["lit"], p["lit"])
rep("fast base vs lit base", b["fast"], b["lit"])
m = rep("fast pack vs fast base", p["fast"], b["fast"])
rep("fast pack vs lit", p["fast"], p["lit"])
idx = np.nonzero(m)[0][:8]
for i in idx:
    print(i, p["fast"].reshape(-1, 4)[i], b["fast"].reshape(-1, 4)[i])
d8 = np.abs(p["fast8"].astype(int) - p["lit8"].astype(int)).reshape(-1, 4).max(1)
print("rgba8 pack fast vs lit", (d8 > 0).sum(), d8.max())
