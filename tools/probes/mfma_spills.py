"""Scratch (spill) instructions inside basic blocks that issue an MFMA, per
kernel of an ISA listing (the hot loops; make -C ska-sdp-idg-bench_amd isa).
  python tools/probes/mfma_spills.py LISTING.s"""
import re
import sys


def per_kernel(text):
    out = {}
    for func in re.split(r"\n(?=_Z\w+:)", text):
        m = re.match(r"(_Z\w+):", func)
        if not m:
            continue
        hot = spills = 0
        for block in re.split(r"\n(?=\.LBB\d+_\d+:)", func):
            if "v_mfma" not in block:
                continue
            hot += 1
            spills += sum(1 for l in block.split("\n")
                          if re.match(r"\s*(scratch_|buffer_(load|store)_dword)",
                                      l))
        if hot:
            out[m.group(1)] = (hot, spills)
    return out


if __name__ == "__main__":
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    from resources import short
    for name, (hot, spills) in per_kernel(open(sys.argv[1]).read()).items():
        print(f"{short(name):38s} mfma blocks {hot:3d} spill ops in them {spills}")
