#!/bin/bash
# Round 4, first GPU call: the GPU suite on this tree (general-path pixel
# geometry in LDS: the combined gridder spill-free), the K-step probe with
# f32-MFMA fractions, the mirror gridder with channel
# quads on the f32 matrix core (IDG_GRID_F32MASK builds under ab/) against
# this tree and against HEAD (ab/head.so), the wterm workload A/B, and the
# gridder parity tests + accuracy on the 2/4 f32 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04kstep
mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iska-sdp-idg-bench_amd/csrc \
  -mllvm -amdgpu-sched-strategy=max-ilp tests/probes/kstep_probe.hip -o $out/kstep_probe || exit 1
bash tests/debug/session.sh $out/s suite || exit 1
for rep in 1 2; do
  timeout -k 10 120 $out/kstep_probe > $out/kstep.$rep.txt 2>&1 || { cat $out/kstep.$rep.txt; exit 1; }
  cat $out/kstep.$rep.txt
done
bash tests/debug/session.sh $out/ab ab=ab/head.so,ab/base.so,ab/f32m2.so,ab/f32m10.so,ab/f32m14.so || exit 1
BENCH_ARGS="--workload wterm" STEPS=10 bash tests/debug/session.sh $out/abw ab=ab/head.so,ab/base.so || exit 1
bash tests/debug/session.sh $out/f32 'suite@ab/f32m10.so=gridder and not fft and not pipeline' \
  accuracy@ab/f32m10.so accuracy@ab/base.so
