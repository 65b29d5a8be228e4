"""Cell-run census of the C5 NMS workload (synth.nms_boxes seed 99, one 100k
image, iou 0.3): a numpy restatement of csrc/nms.hip's grid keys (log-extent
classes of width 1.01 * -ln(t) / kK, cells of 1.05 f x the largest extent of
classes c-kK..c+kK) — how many boxes share a (class, cell) run and how large
the (run, neighbour run) tiles of a cell-pair-tiled search would be.

  python3 tools/nms_grid_census.py
"""
import numpy as np, sys, collections
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'jabd-joint-attention-based-detector-for-small-face-detection_amd'))
from jabd_amd import synth
bx, sc = synth.nms_boxes(1, 100_000, seed=99)
b = bx[0].astype(np.float32)
thr=0.3; kK=2
wcls = 1.01*-np.log(thr); wcls=max(wcls,0.2)/kK; inv_w=np.float32(1/wcls)
f=1.05*max((1-thr)/(1+thr),0.05)
w=b[:,2]-b[:,0]; h=b[:,3]-b[:,1]
cw=np.floor(np.log(w)*inv_w).astype(int); ch=np.floor(np.log(h)*inv_w).astype(int)
print("width classes", np.unique(cw).size, "height classes", np.unique(ch).size)
def cellsize(c, e):
    ext={}
    for cc,ee in zip(c,e): ext[cc]=max(ext.get(cc,0),ee)
    return {cc: f*max(ext.get(cc+d,0) for d in range(-kK,kK+1)) for cc in ext}, ext
sxm, ew = cellsize(cw,w); sym, eh = cellsize(ch,h)
sx=np.array([sxm[c] for c in cw]); sy=np.array([sym[c] for c in ch])
X=np.floor((b[:,0]+b[:,2])*0.5/sx).astype(int); Y=np.floor((b[:,1]+b[:,3])*0.5/sy).astype(int)
keys=list(zip(cw,ch,Y,X))
cnt=collections.Counter(keys)
sizes=np.array(list(cnt.values()))
print("runs",len(cnt),"mean size",sizes.mean())
for lo,hi in [(1,1),(2,3),(4,7),(8,15),(16,31),(32,63),(64,10**9)]:
    m=(sizes>=lo)&(sizes<=hi); print(f"size {lo}-{hi}: runs {m.sum()}, boxes {sizes[m].sum()}")
# tile pairs (run R, neighbour run S) as grid_pairs enumerates (approx: window by class max)
tests=0; tiles=0; tiles_nonempty=0; probes=0
tile_sizes=[]
runs_by=collections.defaultdict(list)
for k,v in cnt.items(): pass
# per run: neighbour windows using the run's max box size (per-box windows differ); approximate using center cell +-1
nb=[(0,d) for d in range(0,kK+1)]+[(dw,dh) for dw in range(1,kK+1) for dh in range(-kK,kK+1)]
for (a,c,y,x),n1 in cnt.items():
    for (dw,dh) in nb:
        a2,c2=a+dw,c+dh
        if a2 not in ew or c2 not in eh: continue
        for yy in (y-1,y,y+1):
            for xx in (x-1,x,x+1):
                # cell coords of class2 differ in size: approximate
                probes+=1
                n2=cnt.get((a2,c2,yy,xx),0)
                if n2:
                    tiles+=1; tile_sizes.append((n1,n2)); tests+=n1*n2
print("probes(run-level)",probes,"nonempty tiles",tiles,"tests",tests)
ts=np.array(tile_sizes)
print("tile n1 mean",ts[:,0].mean(),"n2 mean",ts[:,1].mean(), "tests in tiles with n1*n2>=64:", (ts[:,0]*ts[:,1])[ts[:,0]*ts[:,1]>=64].sum())
