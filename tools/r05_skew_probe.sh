#!/bin/bash
# NW from both ends: where the halves meet.  Lane taps on both sides (GSA_BIDI_GRAN=0) against the
# top half ending on a ticket boundary (its tap from the granules) with GSA_BIDI_SKEW extra rows.
# (profiles/r05_bidi_skew.txt also has a no-tap timing column from a probe knob since removed.)
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
n=${1:-50000}
timeout -k 10 400 python3 -u $ROOT/tools/r05_bidi_ab.py $n 7 NW-AG,NW-LG SCORE_BIDI=0 BIDI_GRAN=0 \
    BIDI_GRAN=1,BIDI_SKEW=0 BIDI_GRAN=1,BIDI_SKEW=1500 BIDI_GRAN=1,BIDI_SKEW=3000 BIDI_GRAN=1,BIDI_SKEW=4500 \
    BIDI_GRAN=1,BIDI_SKEW=6000 BIDI_GRAN=1
