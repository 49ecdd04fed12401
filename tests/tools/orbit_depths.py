"""Test-infrastructure model (CPU oracle): per-tile depths of the bicycle stand-in's tile-centre rays and a
reprojected dispatch order scored against the round-4 orbit cost dumps (profiles/EXPERIMENTS.md round 6).
usage: python tests/tools/orbit_depths.py bicycle && python tests/tools/orbit_reproject_model.py bicycle"""
import os
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys, importlib, numpy as np
sys.path.insert(0,_ROOT); sys.path.insert(0,os.path.join(_ROOT,'oracle'))
gv=importlib.import_module("3dgvrt_lightfield_amd"); import oracle as O
from scipy.ndimage import maximum_filter
import heapq
SLOTS=4096
def makespan(costs):
    h=[0.0]*SLOTS
    for c in costs: heapq.heappush(h, heapq.heappop(h)+c)
    return max(h)
def rank(x):
    r=np.empty(len(x)); r[np.argsort(x,kind="stable")]=np.arange(len(x)); return r
def score(cost, proxy):
    proxy=proxy.reshape(-1); order=np.argsort(-proxy,kind="stable"); bound=max(cost.sum()/SLOTS,cost.max())
    return round(float(np.corrcoef(rank(proxy),rank(cost))[0,1]),3), round(makespan(cost[order])/bound,4)
cfg=sys.argv[1]
d=np.load(os.path.join(_ROOT,'profiles')+'/r04/orbit_costs_%s.npz'%cfg)
gen,W,H,_=gv.scene.CONFIGS[cfg]; s=gv.scene.make(**gen)
TX,TY=W//8,H//8
vi0,pi0=gv.scene.mipnerf_camera(W,H,azimuth_deg=30.0)
px=(np.arange(TX)*8+4); py=(np.arange(TY)*8+4)
PX,PY=np.meshgrid(px,py)
rays=(PY*W+PX).reshape(-1).astype(np.uint64)
e=O.enclose(s)
r=O.render(e,vi0,pi0,W,H,subset=rays,ray_dirs=True,proxy_mode=1)
dep=r['depth']; dirs=r['ray_dirs'][:,:3].astype(np.float64)
VI0=np.asarray(vi0,np.float64).reshape(4,4)
print('depth stats', np.percentile(dep,[5,50,95]), 'VI0 row/col?', VI0[3], VI0[:,3])
sc=O.Scene(e)
import time; t0=time.time()
zs=np.zeros(len(rays)); zmed=np.zeros(len(rays))
for i,ray in enumerate(rays):
    tr=sc.trace(vi0,pi0,W,H,int(ray))
    if len(tr)==0: zs[i]=np.nan; zmed[i]=np.nan; continue
    t=tr[:,1]; T=tr[:,4]; acc=tr[:,5]>0
    Tb=np.concatenate([[1.0],T[:-1]]); w=(Tb-T)
    zs[i]=(t*w).sum()/max(w.sum(),1e-6) if w.sum()>1e-4 else np.median(t)
    zmed[i]=np.median(t)
print('traced', time.time()-t0)
np.savez('/tmp/orbit_depth_%s.npz'%cfg, zs=zs, zmed=zmed, dirs=dirs)
