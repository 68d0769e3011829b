"""Debug aid: bench.py's cpu_baseline (1 thread and N threads) on a small
batch, here on the CPU: python tests/debug/cpu_baseline_check.py [threads]."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
sys.path.insert(0, REPO)
os.environ.setdefault("IDG_CPU_BASELINE_THREADS",
                      sys.argv[1] if len(sys.argv) > 1 else "4")
import bench  # noqa: E402
import idg_amd  # noqa: E402

w = dict(bench.WORKLOADS["default"])
w["nr_timeslots"] = 1
a = idg_amd.generate(50, 1, 128, 16, 1024, 32, nthreads=8)
r = bench.cpu_baseline(w, a, int(os.environ.get("NSAMPLE", "16")))
print(r["value"], r["cores"], r["gridder_mvis_s"], r["degridder_mvis_s"],
      r.get("single_thread", {}).get("gridder_mvis_s"),
      r.get("single_thread", {}).get("degridder_mvis_s"))
