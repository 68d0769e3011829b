"""Static check of the gridder's L2-prefetch LDS-DMA in an ISA listing: no
s_waitcnt counting vmcnt between a global_load_lds_* and the next MFMA (a
compiler wait there would drain the prefetch and expose its latency), and
where the kernels' scratch (spill) accesses sit.
  python tests/probes/dma_drain_check.py LISTING.s"""
import re
import sys


def check(text):
    res = []
    for f in re.split(r'\n(?=_Z\w+:)', text):
        if 'global_load_lds' not in f:
            continue
        name = f.split(':')[0]
        ins = [l.strip() for l in f.split('\n')
               if l.strip() and not l.strip().startswith(('.', ';'))]
        drained = total = 0
        for i, l in enumerate(ins):
            if l.startswith('global_load_lds'):
                total += 1
                for j in range(i + 1, len(ins)):
                    if 'v_mfma' in ins[j]:
                        break
                    if ins[j].startswith('s_waitcnt') and 'vmcnt' in ins[j]:
                        drained += 1
                        break
        scratch = sum(1 for l in ins if l.startswith('scratch_'))
        res.append((name, total, drained, scratch))
    return res


if __name__ == '__main__':
    for name, total, drained, scratch in check(open(sys.argv[1]).read()):
        print(name[:80], 'dma', total, 'drained before MFMA', drained,
              'scratch ops', scratch)
