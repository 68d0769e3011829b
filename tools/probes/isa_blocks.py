"""Per-block instruction counts of one kernel in an ISA listing (debug aid):
  python tools/probes/isa_blocks.py LISTING.s NAME_PATTERN [FIRST_LINE LAST_LINE]
prints each basic block's label, loop comment, #instructions, #VALU, #s_waitcnt."""
import re
import sys

src = open(sys.argv[1]).read()
f = [x for x in re.split(r'\n(?=_Z\w+:\s*\n)', src) if sys.argv[2] in x.split(':')[0]][0]
blocks = re.split(r'\n(?=\.LBB\d+_\d+:)', f)
for b in blocks:
    head = b.split('\n')[0]
    ins = [l.strip() for l in b.split('\n')[1:]
           if l.strip() and not l.strip().startswith(('.', ';', '//'))]
    valu = sum(1 for l in ins if l.startswith('v_'))
    wc = [l for l in ins if l.startswith('s_waitcnt')]
    flags = ' '.join(sorted({w.split()[0] for w in ins if w.startswith(('global_load_lds', 's_barrier', 'scratch_', 'v_mfma', 'ds_bpermute', 'ds_max'))}))
    print(head[:70].ljust(70), 'n', len(ins), 'valu', valu, 'wait', len(wc), flags)
