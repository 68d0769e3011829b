"""Per-launch HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of
tools/probes/summarize_profiles.py) of the gridder / degridder from the
rocprofv3 --pmc databases an A/B script wrote (tools/debug/r05_s64_ab.sh,
r05_nt_ab.sh): python tools/debug/ab_traffic.py DIR LIB [LIB ...]"""
import glob
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "probes"))
import summarize_profiles as sp  # noqa: E402

d = sys.argv[1]
for lib in sys.argv[2:]:
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        db = glob.glob(os.path.join(d, f"{lib}_{c}", "**", "*.db"),
                       recursive=True)[0]
        for key, cs in sp.counters(sp.read_rows(sp.to_csv(db, "counter"))).items():
            if isinstance(key, tuple):
                per.setdefault(key[0], {}).setdefault(c, 0.0)
                per[key[0]][c] += cs[c]
    for k in sorted(per):
        t = per[k]
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            gb = (2 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024 / 1e9
            print(f"{lib:10s} {k:28s} {gb:8.3f} GB per launch "
                  f"(fetch {t['FETCH_SIZE'] * 1024 / 1e9:.3f} x2, "
                  f"write {t['WRITE_SIZE'] * 1024 / 1e9:.3f})")
