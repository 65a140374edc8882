"""numpy study behind the bounded exit's stage 0 (gic_bc7.hip k_fit6): how many
blocks of G1 / G0 a direct mode-6 fit (first-projection indices, least squares
for BC7's 4-bit weights, 7-bit codes + parity) brings within MSE 0.5, with and
without the joint parity choice and the refit.  (A study, not the model: the
bit-exact restatement is oracle/orc_bc7.c orc_bc7_fit6.)

    python tools/fit6_study.py
"""
import numpy as np, sys
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..'))
from gfx_imagecompress_amd import synth
W=np.array([0,4,9,13,17,21,26,30,34,38,43,47,51,55,60,64],dtype=np.int64)
def blocks(img, rows):
    H,Wd,_=img.shape
    return np.array([img[by*4:by*4+4, bx*4:bx*4+4].reshape(16,4) for by in rows for bx in range(Wd//4)]).astype(np.int64)
def firstproj(B):
    Bf=B.astype(np.float64); mean=Bf.mean(1,keepdims=True); C=Bf-mean
    cov=np.einsum('nki,nkj->nij',C,C); w,v=np.linalg.eigh(cov); d=v[:,:,-1]
    prj=np.einsum('nki,ni->nk',C,d); lo=prj.min(1,keepdims=True); hi=prj.max(1,keepdims=True)
    return np.rint((prj-lo)/np.where(hi>lo,hi-lo,1)*15).astype(np.int64)
def fit(X, idx):
    w=W[idx]; a00=((64-w)**2).sum(); a01=((64-w)*w).sum(); a11=(w*w).sum()
    r0=((64-w)[:,None]*X).sum(0); r1=(w[:,None]*X).sum(0)
    det=a00*a11-a01*a01
    if det==0: m=X.mean(0); return m,m
    return 64.0*(a11*r0-a01*r1)/det, 64.0*(a00*r1-a01*r0)/det
def quant(e, joint, X=None, e1=None):
    out=[]
    for ei in e:
        best=None
        for p in (0,1):
            c=np.clip(np.floor((ei-p)/2+0.5),0,127); q=2*c+p; err=((q-ei)**2).sum()
            if best is None or err<best[0]: best=(err,q)
        out.append(best[1].astype(np.int64))
    return out
def sse_of(X,q0,q1):
    pal=((64-W)[:,None]*q0[None,:]+W[:,None]*q1[None,:]+32)>>6
    dd=((X[:,None,:]-pal[None,:,:])**2).sum(2)
    return dd.min(1).sum(), dd.argmin(1)
def joint(X,e0,e1):
    best=None
    for p0 in (0,1):
        for p1 in (0,1):
            q0=2*np.clip(np.floor((e0-p0)/2+0.5),0,127).astype(np.int64)+p0
            q1=2*np.clip(np.floor((e1-p1)/2+0.5),0,127).astype(np.int64)+p1
            s,ix=sse_of(X,q0,q1)
            if best is None or s<best[0]: best=(s,ix)
    return best
def run(B, iters, jnt):
    idx0=firstproj(B); out=np.zeros(len(B))
    for b in range(len(B)):
        X=B[b]; idx=idx0[b]; best=1e18
        for it in range(iters):
            e0,e1=fit(X,idx)
            e0=np.clip(e0,0,255); e1=np.clip(e1,0,255)
            if jnt: s,ix=joint(X,e0,e1)
            else:
                q0,q1=quant([e0,e1],False); s,ix=sse_of(X,q0,q1)
            best=min(best,s); idx=ix
        out[b]=best
    return out
for name,img,rows in (("G1",synth.g1(8192,1024),range(0,256,8)),("G0",synth.g0(8192,1024),range(0,256,32))):
    B=blocks(img,rows)
    for iters,jnt in ((1,False),(1,True),(2,True),(3,True)):
        s=run(B,iters,jnt)
        print(name,len(B),"iters",iters,"joint",jnt,"pass",round((s<=32).mean(),4),"meanMSE",round((s/64).mean(),4),flush=True)
