"""CPU feasibility check (numpy, no GPU): can the ResNet residual join of
the streaming 1x1 kernel — out = sat(rne(((y - z3) s3 + (r - zr) sr) * fp32(1/so)))
over the 256 x 256 (y3, identity) byte pairs, in the kernel's fp32 op order —
be written exactly as one two-variable form rne(fma(y, a, fma(r, b, c)))?
Random realistic qparams (zr = 0, zo = 0: post-ReLU identity and output);
a crude search around (s3/so, sr/so, -(z3 s3 + zr sr)/so).  Round 4 result:
187 of 200 layers exact, the rest off by one pair (DESIGN §5 ResNet, next).

    python tools/join_affine_feasibility.py
"""
import numpy as np
F=np.float32
rng=np.random.default_rng(3)
y=np.arange(256,dtype=np.float32)[:,None]; r=np.arange(256,dtype=np.float32)[None,:]
def ref(s3,z3,sr,zr,so):
    inv=F(1)/F(so)
    sm=((y-F(z3))*F(s3) + (r-F(zr))*F(sr)).astype(F)
    sm=(sm*inv).astype(F)
    return np.clip(np.rint(sm),0,255)
def aff(a,b,c):
    v=(y.astype(np.float64)*np.float64(a) + (r.astype(np.float64)*np.float64(b)+np.float64(c)).astype(F).astype(np.float64)).astype(F)
    return np.clip(np.rint(v),0,255)
tot=0; ok=0; mism=[]
for t in range(200):
    s3=F(10**rng.uniform(-2.5,-1)); sr=F(s3*2**rng.uniform(-1.5,1.5)); so=F(max(s3,sr)*2**rng.uniform(0,1.5))
    z3=int(rng.integers(60,200)); zr=0
    g=ref(s3,z3,sr,zr,so)
    inv=1/np.float64(so)
    best=None
    for da in (0,1,-1,2,-2):
        for dc in np.linspace(-2e-4,2e-4,9):
            a=F(np.float64(s3)*inv*(1+da*1e-7)); b=F(np.float64(sr)*inv); c=F(-(z3*np.float64(s3)+zr*np.float64(sr))*inv+dc)
            m=int((aff(a,b,c)!=g).sum())
            if best is None or m<best: best=m
            if m==0: break
        if best==0: break
    tot+=1; ok+= best==0; mism.append(best)
print("exact forms found", ok, "of", tot, "; mismatch counts of the rest:", sorted(mism)[-10:])
