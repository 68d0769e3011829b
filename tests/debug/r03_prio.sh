#!/bin/bash
# Round 3: static issue priority for one half of the waves (IDG_PRIO=1:
# the second-dispatched half, 2: the first) against the shipped build.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
bash tests/debug/ab.sh ab/base.so ab/prio1.so ab/prio2.so
echo done
