"""Test-infrastructure model (CPU oracle): per-tile depths of the bicycle stand-in's tile-centre rays and a
reprojected dispatch order scored against the round-4 orbit cost dumps (profiles/EXPERIMENTS.md round 6).
usage: python tests/tools/orbit_depths.py bicycle && python tests/tools/orbit_reproject_model.py bicycle"""
import os
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys, importlib, numpy as np, heapq
sys.path.insert(0,_ROOT)
gv=importlib.import_module("3dgvrt_lightfield_amd")
from scipy.ndimage import maximum_filter
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
z=np.load('/tmp/orbit_depth_%s.npz'%cfg)
gen,W,H,_=gv.scene.CONFIGS[cfg]
TX,TY=W//8,H//8
prev=d['static'].astype(np.float64)
vi0,pi0=gv.scene.mipnerf_camera(W,H,azimuth_deg=30.0)
M0=np.asarray(vi0,np.float64).reshape(4,4).T
o0=M0[:3,3]
dirs=z['dirs']
for key in ('zs','zmed'):
  zz=z[key].copy(); zz[~np.isfinite(zz)]=1e3
  P=o0[None,:]+dirs*zz[:,None]
  for D in (0.5,2):
    cost=np.exp2(d['moved_%g'%D]/4.0).reshape(-1)
    vi1,pi1=gv.scene.mipnerf_camera(W,H,azimuth_deg=30.0+D)
    V1=np.linalg.inv(np.asarray(vi1,np.float64).reshape(4,4).T); P1=np.linalg.inv(np.asarray(pi1,np.float64).reshape(4,4).T)
    # direction-only projection: view-space target.xyz ~ proj_inv * ndc; invert: ndc from view-space direction
    Pv=(V1@np.c_[P,np.ones(len(P))].T).T[:,:3]
    clip=(P1@np.c_[Pv/np.linalg.norm(Pv,axis=1,keepdims=True),np.ones(len(P))].T).T
    ndc=clip[:,:2]/clip[:,3:4]
    # check: pixel = (ndc+1)/2*size (pixel_offset 0 corner rays)
    pxy=(ndc+1)/2*np.array([W,H])
    tx=np.floor(pxy[:,0]/8).astype(int); ty=np.floor(pxy[:,1]/8).astype(int)
    ok=(tx>=0)&(tx<TX)&(ty>=0)&(ty<TY)
    g=np.zeros((TY,TX))-1
    w=prev.reshape(-1)
    np.maximum.at(g,(ty[ok],tx[ok]),w[ok])
    holes=g<0
    fill=maximum_filter(np.where(holes,-1,g),size=3)
    g2=np.where(holes,np.maximum(fill,0),g)
    for rad in (0,1):
        gg=maximum_filter(g2,size=2*rad+1) if rad else g2
        print(cfg,key,D,'reproj r%d'%rad,score(cost,np.exp2(gg/4.0)),'holes %.3f'%holes.mean())
    print(cfg,key,D,'previous',score(cost,np.exp2(prev/4.0)), 'dilated1', score(cost,np.exp2(maximum_filter(prev,size=3)/4.0)))
# sanity: reproject with D=0 must give identity
vi1,pi1=vi0,pi0
