"""Debug aid (CPU): exact numpy emulation of the MFMA kernels' phase reduction
(r = fma(phase, 1/2pi_hi, -m) per 16-channel block, the per-pixel
phase_offset tail) with and without the k * phase_index tail correction,
accumulated in double, against the exact sum of the same f32 phases;
reference metric, one C = 256 (or argv[1]) -c subgrid.  DESIGN.md §3.1."""
import sys, numpy as np
import os
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in ("ska-sdp-idg-bench_amd", "oracle", "tests", "tools/debug"):
    sys.path.insert(0, os.path.join(REPO, _p))
import idg_amd, oracle as orc
from phase_reduction_emul import fma32, IH, TAIL, f32
o=orc.Oracle()
C=int(sys.argv[1]) if len(sys.argv)>1 else 256
a=idg_amd.generate(2,2,128,C,1024,32,nthreads=8)
S=32; G=1024; img=f32(0.01)
k=a["wavenumbers"]
for s in (0,1):
    m=a["metadata"][s]
    idx=((np.arange(S)+0.5-S/2)*np.float64(img)/S).astype(f32)
    l=np.broadcast_to(idx[None,:],(S,S)).astype(f32).ravel(); mm=np.broadcast_to(idx[:,None],(S,S)).astype(f32).ravel()
    scale=2*np.pi/np.float64(img)
    uo=f32((int(m["x"])+S//2-G//2)*scale); vo=f32((int(m["y"])+S//2-G//2)*scale)
    poff=fma32(uo,l,(vo*mm).astype(f32))
    T=128; rows=slice(int(m["time_offset"]),int(m["time_offset"])+T)
    uvw=a["uvw"].reshape(-1,3)[rows]; vis=a["visibilities"].reshape(-1,C,4,2)[rows]
    V=vis[...,0].astype(np.float64)+1j*vis[...,1]
    Pex=np.zeros((4,S*S),complex); Pem=np.zeros((4,S*S),complex); Pfix=np.zeros((4,S*S),complex)
    for t in range(T):
        pidx=fma32(uvw[t,0],l,(uvw[t,1]*mm).astype(f32))
        ph=fma32(-pidx[None,:],k[:,None],poff[None,:])  # [C][npix] f32
        ex=np.exp(1j*ph.astype(np.float64))
        # emulate: r = fma(ph, IH, -m) with m = rint(A*IH) per 16-ch block; phasor = exp(2pi i r) * exp(i poff kPhaseTail)
        A=ph[0::16]; 
        mblk=np.rint((A.astype(np.float64)*np.float64(IH)).astype(f32).astype(np.float64))
        mfull=np.repeat(mblk,16,axis=0)[:C]
        r=(ph.astype(np.float64)*np.float64(IH)-mfull).astype(f32).astype(np.float64)
        em=np.exp(2j*np.pi*r)*np.exp(1j*poff.astype(np.float64)*(1-2*np.pi*np.float64(IH)))[None,:]
        # corrected: add the k*pidx tail per block (k of block's first channel)
        kb=np.repeat(k[0::16],16)[:C].astype(np.float64)
        fix=np.exp(-1j*kb[:,None]*pidx[None,:].astype(np.float64)*(1-2*np.pi*np.float64(IH)))
        Pex+=V[t].T@ex; Pem+=V[t].T@em; Pfix+=V[t].T@(em*fix)
    def cz(P): 
        out=np.zeros((1,4,S,S,2),np.float32); out[0,...,0]=P.real.reshape(4,S,S); out[0,...,1]=P.imag.reshape(4,S,S); return out
    e=cz(Pex)
    print(f"C={C} s={s}: emul(tail poff only)-vs-exact {o.check_error(cz(Pem),e)[0]:.3e}  emul+k-tail-fix vs exact {o.check_error(cz(Pfix),e)[0]:.3e}")
