"""Per-kernel register / scratch / occupancy / LDS summary of a
-Rpass-analysis=kernel-resource-usage log (make -C ska-sdp-idg-bench_amd isa
writes build/isa/*.resources.txt).
  python tools/probes/resources.py ska-sdp-idg-bench_amd/build/isa/*.resources.txt"""
import re
import sys


def parse(text):
    out, cur = [], None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"),
                         ("sgpr", r"SGPRs: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                         ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    return out


def short(name):
    m = re.search(r"kernel_(\w+?)_mi355xI(.*?)EEv", name)
    if not m:
        return name[:60]
    args = re.findall(r"Li(-?\d+)E", m.group(2) + "E")
    return f"{m.group(1)}<{','.join(args)}>"


if __name__ == "__main__":
    for path in sys.argv[1:]:
        for k in parse(open(path).read()):
            print(f"{short(k['name']):38s} vgpr {k.get('vgpr', '?'):>4} "
                  f"agpr {k.get('agpr', '?'):>3} scratch {k.get('scratch', '?'):>4}"
                  f" occ {k.get('occ', '?')} lds {k.get('lds', '?')}")
