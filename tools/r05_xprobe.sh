#!/bin/bash
# round 5: what bounds the expansion (pass 2) -- the default build against diagnostic builds of it
# (GSA_EXPAND_PROBE=1: one add per cell instead of the recurrence; =2: no interior stores), full batch
# field of the bench, alternated 3 times (tools/r05_ab_full.sh); the box's plain fill rate beside it
set -e
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
bash tools/r05_ab_full.sh gpuseqalign_amd/libgsa_xp1.so gpuseqalign_amd/libgsa_xp2.so
