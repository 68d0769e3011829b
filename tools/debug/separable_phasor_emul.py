"""Debug aid (CPU): could the mirror gridder form its phasors separably?
For w = 0 the phase is linear in (l, m), so exp(i(phase_offset - k pidx))
= exp(i poff) exp(-i k u l) exp(-i k v m): 2 x 32 phasors per (t, c) and a
complex multiply per pixel instead of v_sin/v_cos of every (pixel, t, c).
That is the exact-math phase, not the reference's f32-rounded one
(poff - k * pidx rounded at |phase| ~ 1,600 rad: ulp 1.2e-4).  This
compares, within one numpy emulation (both sums in double, the reference's
own f32 phase_offset kept), the exact-math sum against the sum of the
reference's f32 phases in the reference metric:

    python tools/debug/separable_phasor_emul.py [C]

Measured: 1.7e-5 at C = 16, 4.5e-5 at C = 256 -- above the 1e-5 bar, so the
phase must keep the reference's rounding.  (The absolute
lines against oracle/_ref are printed too; this emulation's A-term
orientation differs from the oracle's, so only the self-consistent line is
meaningful.)"""
import os, sys
import numpy as np
REPO=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("ska-sdp-idg-bench_amd","oracle","tests","tools/debug"):
    sys.path.insert(0, os.path.join(REPO,p))
import idg_amd, oracle as orc
from mfma_accum_emul import f32, f64, fma32
C=int(sys.argv[1]) if len(sys.argv) > 1 else 16; T=128; S=32; G=1024
a=idg_amd.generate(2,2,T,C,G,S,nthreads=8)
ns=a["metadata"].size
o=orc.Oracle()
args=(ns,G,S,idg_amd.IMAGE_SIZE,idg_amd.W_STEP,C,2)
ins=(a["uvw"],a["wavenumbers"],a["visibilities"],a["spheroidal"],a["aterms"],a["metadata"])
ref=np.zeros((ns,4,S,S,2),np.float32); orc.Reference(portable=True).gridder(*args,*ins,ref)
ex=np.zeros(ref.shape,np.float64); o.gridder_exact(*args,*ins,ex,nthreads=8)
# exact-math phases: phase = poff - k*pidx in double from the same f32 inputs
img=f64(idg_amd.IMAGE_SIZE); k=a["wavenumbers"].astype(f64)
idx=((np.arange(S)+0.5-S/2)*img/S).astype(f32).astype(f64)
l=np.broadcast_to(idx[None,:],(S,S)).ravel(); m=np.broadcast_to(idx[:,None],(S,S)).ravel()
at=a["aterms"].reshape(-1,2,S,S,4,2); at=at[...,0].astype(f64)+1j*at[...,1]
sph=a["spheroidal"].reshape(S*S).astype(f64)
out=np.zeros(ref.shape,np.float64); out2=np.zeros(ref.shape,np.float64)
for s in range(ns):
    md=a["metadata"][s]; su=2*np.pi/img
    uo=f64(f32((int(md["x"])+S//2-G//2)*su)); vo=f64(f32((int(md["y"])+S//2-G//2)*su))
    poff=fma32(f32(uo),l.astype(f32),(f32(vo)*m.astype(f32)).astype(f32)).astype(f64)
    rows=slice(int(md["time_offset"]),int(md["time_offset"])+T)
    uvw=a["uvw"].reshape(-1,3)[rows].astype(f64)
    V=a["visibilities"].reshape(-1,C,4,2)[rows]; V=V[...,0].astype(f64)+1j*V[...,1]
    P=np.zeros((S*S,4),complex); P2=np.zeros((S*S,4),complex)
    for t in range(T):
        pidx=uvw[t,0]*l+uvw[t,1]*m
        ph=poff[None,:]-k[:,None]*pidx[None,:]
        P+=np.exp(1j*ph).T@V[t]
        pidx32=fma32(f32(uvw[t,0]),l.astype(f32),(f32(uvw[t,1])*m.astype(f32)).astype(f32))
        ph32=fma32(-pidx32[None,:],k.astype(f32)[:,None],poff.astype(f32)[None,:]).astype(f64)
        P2+=np.exp(1j*ph32).T@V[t]
    a1=at[int(md["aterm_index"]),int(md["station1"])].reshape(S*S,2,2)
    a2=at[int(md["aterm_index"]),int(md["station2"])].reshape(S*S,2,2)
    for dst,PP in ((out,P),(out2,P2)):
        Q=np.conj(np.transpose(a1,(0,2,1)))@PP.reshape(S*S,2,2)@a2
        Q=Q.reshape(S*S,4)*sph[:,None]
        dst[s,...,0]=Q.real.T.reshape(4,S,S); dst[s,...,1]=Q.imag.T.reshape(4,S,S)
o32=out.astype(np.float32); e32=ex.astype(np.float32)
print(f"C={C}: SELF-CONSISTENT exactmath_vs_refphases {o.check_error(out.astype(np.float32),out2.astype(np.float32))[0]:.3e} emul-refphases_vs_oracle_exact {o.check_error(out2.astype(np.float32),e32)[0]:.3e}");print(f"C={C}: exactmath_vs_ref {o.check_error(o32,ref)[0]:.3e}  exactmath_vs_exact(ref phases) {o.check_error(o32,e32)[0]:.3e}  ref_vs_exact {o.check_error(ref,e32)[0]:.3e}")
