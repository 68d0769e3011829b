"""Static check of the gridder's L2-prefetch LDS-DMA in an ISA listing: no
s_waitcnt counting vmcnt between a global_load_lds_* and the next MFMA (a
compiler wait there would drain the prefetch and expose its latency), at
least one wait state between an SALU write of M0 and the LDS-DMA that reads
it as its LDS address (the gfx9 "M0 -> LDS DMA" hazard: hipcc pads it for
its own code but not inside an asm string), and where the kernels' scratch
(spill) accesses sit.
  python tools/probes/dma_drain_check.py LISTING.s"""
import re
import sys


def m0_hazards(ins, i):
    """1 if the instruction right before the LDS-DMA ins[i] writes M0 (no
    wait state between them), else 0."""
    j = i - 1
    while j >= 0 and ins[j].endswith(':'):
        j -= 1
    if j < 0:
        return 0
    return 1 if re.match(r's_\w+\s+m0\b', ins[j]) else 0


def check(text, with_m0=False):
    res = []
    for f in re.split(r'\n(?=_Z\w+:)', text):
        if 'global_load_lds' not in f:
            continue
        name = f.split(':')[0]
        # labels kept (as "LABEL:") so an unconditional s_branch can be
        # followed: the walk goes in execution order, not listing order
        ins = [l.strip() for l in f.split('\n')
               if l.strip() and (not l.strip().startswith(('.', ';'))
                                 or re.match(r'\.LBB\w+:', l.strip()))]
        where = {l[:-1]: k for k, l in enumerate(ins) if l.endswith(':')}
        drained = total = m0 = 0
        for i, l in enumerate(ins):
            if l.startswith('global_load_lds'):
                total += 1
                m0 += m0_hazards(ins, i)
                j, seen = i + 1, set()
                while j < len(ins) and j not in seen:
                    seen.add(j)
                    t = ins[j]
                    if 'v_mfma' in t:
                        break
                    if t.startswith('s_waitcnt') and 'vmcnt' in t:
                        drained += 1
                        break
                    if t.startswith('s_branch '):
                        j = where.get(t.split()[1], len(ins))
                        continue
                    j += 1
        scratch = sum(1 for l in ins if l.startswith('scratch_'))
        res.append((name, total, drained, scratch, m0) if with_m0 else
                   (name, total, drained, scratch))
    return res


if __name__ == '__main__':
    for name, total, drained, scratch, m0 in check(open(sys.argv[1]).read(),
                                                   with_m0=True):
        print(name[:80], 'dma', total, 'drained before MFMA', drained,
              'scratch ops', scratch, 'M0 write -> DMA with no wait state', m0)
