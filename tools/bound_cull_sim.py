"""Round-6 estimate ("fewer pairs"): how many (32-point tile, hypothesis) pairs of the
bound kernel a conservative per-tile geometric test could skip.  C4-like problem (2,000 matches in
640x480, 160 planted inliers, 5 px), points ordered by a 4-D kd split into 32-point tiles; per
(tile, hypothesis) the tile survives unless W keeps one sign over the source box and the interval of
+-(X - uW), +-(Y - vW) over the 8 (x, y, u) corners clears 5.05 |W|max.  Prints the survival per pair,
per 32- and 64-hypothesis group (what an MFMA column block could skip) and per lane.
    python tools/bound_cull_sim.py > profiles/r06x_bound_cull_sim.txt
"""
import numpy as np
rng=np.random.default_rng(1)
n=2000; ninl=160; W,Hh=640,480
src=np.c_[rng.uniform(0,W,n),rng.uniform(0,Hh,n)]
dst=np.c_[rng.uniform(0,W,n),rng.uniform(0,Hh,n)]
# true H: mild perspective
Ht=np.array([[0.9,0.1,30],[-0.05,1.1,20],[1e-4,-5e-5,1.0]])
p=np.c_[src[:ninl],np.ones(ninl)]@Ht.T; dst[:ninl]=p[:,:2]/p[:,2:]+rng.uniform(-.5,.5,(ninl,2))
perm=rng.permutation(n); src=src[perm]; dst=dst[perm]
P=np.c_[src,dst]
def kd(idx,depth):
    if len(idx)<=32: return [idx]
    X=P[idx]; d=np.argmax(X.max(0)-X.min(0)); o=idx[np.argsort(X[:,d])]; h=len(o)//2
    # keep halves multiple of 32 where possible
    h=max(32,(h//32)*32) if len(o)>64 else h
    return kd(o[:h],depth+1)+kd(o[h:],depth+1)
tiles=kd(np.arange(n),0)
print(len(tiles),[len(t) for t in tiles][:5])
def homog(s,d):
    A=[]
    for (x,y),(u,v) in zip(s,d):
        A.append([x,y,1,0,0,0,-u*x,-u*y,-u]);A.append([0,0,0,x,y,1,-v*x,-v*y,-v])
    _,_,Vt=np.linalg.svd(np.array(A)); return Vt[-1].reshape(3,3)
thr=5.0
nh=2000
surv=np.zeros((nh,len(tiles)),bool)
cnt=[]
for k in range(nh):
    s=rng.choice(n,4,replace=False); Hm=homog(src[s],dst[s]); Hm/=Hm[2,2]
    q=np.c_[src,np.ones(n)]@Hm.T
    e=np.hypot(q[:,0]/q[:,2]-dst[:,0],q[:,1]/q[:,2]-dst[:,1]); cnt.append((e<thr).sum())
    for t,ti in enumerate(tiles):
        X=P[ti]; x0,y0,u0,v0=X.min(0); x1,y1,u1,v1=X.max(0)
        cx=np.array([x0,x1,x0,x1]); cy=np.array([y0,y0,y1,y1])
        Wc=Hm[2,0]*cx+Hm[2,1]*cy+Hm[2,2]
        if Wc.min()*Wc.max()<=0: surv[k,t]=True; continue
        sg=np.sign(Wc[0]); Wmax=np.abs(Wc).max()
        ok=True
        for row,(a0,a1) in ((0,(u0,u1)),(1,(v0,v1))):
            Xc=Hm[row,0]*cx+Hm[row,1]*cy+Hm[row,2]
            vals=np.concatenate([Xc-a0*Wc,Xc-a1*Wc])*sg
            lo,hi=vals.min(),vals.max()
            r=thr*1.01*Wmax+1e-3
            if lo>r or hi<-r: ok=False
        surv[k,t]=ok
print("counts", np.percentile(cnt,[50,90,99]))
print("pair survival", surv.mean())
g=surv[:1984].reshape(-1,32,len(tiles)).any(1); print("32-group survival", g.mean())
g=surv[:1984].reshape(-1,64,len(tiles)).any(1); print("64-group survival", g.mean())
print("max per lane over 64 lanes", surv[:1984].reshape(-1,64,len(tiles)).sum(2).max(1).mean()/len(tiles))
