"""Median / min duration of the pipeline kernels in rocprofv3 kernel-trace
databases: python tools/debug/kt_pipeline.py gpurun_out/kt_*/run_results.db"""
import collections
import sqlite3
import sys

for db in sys.argv[1:]:
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    ni, si, ei = cols.index("name"), cols.index("start"), cols.index("end")
    d = collections.defaultdict(list)
    for r in con.execute("select * from kernels"):
        n = r[ni]
        if any(k in n for k in ("adder", "splitter", "home", "subgrid_fft")):
            d[n.split("(")[0].split("::")[-1][:40]].append((r[ei] - r[si]) / 1e6)
    for k, v in d.items():
        v.sort()
        print(f"{db.split('/')[-2]:10s} {k:40s} {len(v):3d} median {v[len(v)//2]:.4f} min {v[0]:.4f}")
