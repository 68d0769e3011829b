"""Static instruction mix of the MFMA loop bodies of one kernel (ISA listing
from `make -C ska-sdp-idg-bench_amd isa`).  Usage:
  python tools/probes/isa_loops.py build/isa/gridder_mi355x.s ILi32ELi4ELi16ELi1E"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read()
pat = sys.argv[2]
for f in re.split(r'\n(?=_Z\w+:)', src):
    name = f.split(':')[0].strip()
    if pat not in name:
        continue
    for b in re.split(r'\n(?=\.LBB\d+_\d+:)', f):
        ins = [l.strip() for l in b.split('\n')[1:]
               if l.strip() and not l.strip().startswith(('.', ';', '//'))]
        nm = sum('v_mfma' in l for l in ins)
        if not nm:
            continue
        c = Counter(l.split()[0] for l in ins)
        trans = c['v_sin_f32_e32'] + c['v_cos_f32_e32']
        split = c['v_cvt_pk_f16_f32'] + c['v_fma_mixlo_f16'] + c['v_fma_mixhi_f16']
        valu = sum(v for k, v in c.items() if k.startswith('v_') and 'mfma' not in k)
        other = valu - trans - split - c['v_pk_fma_f32'] - c['v_pk_add_f32']
        print(b.split('\n')[0][:10], 'n', len(ins), 'mfma', nm, 'trans', trans,
              'split', split, 'pk', c['v_pk_fma_f32'] + c['v_pk_add_f32'],
              'other', other, 'nop', c['s_nop'],
              'est_cyc/phasor %.2f' % ((trans * 9.65 + (valu - trans) * 4.47) / (2 * nm)))
        if '-v' in sys.argv:
            print(sorted(((k, v) for k, v in c.items()), key=lambda x: -x[1]))
