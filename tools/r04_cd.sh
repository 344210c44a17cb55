#!/bin/bash
# Round 4, calls C + D in one: two-car REWARD lane-per-car exactness and A/B, then the
# self-play tests, the driver's bench command, 1,000 steady steps and the window trace.
set -u
bash tools/r04_d.sh || exit 1
bash tools/r04_c.sh || exit 1
echo R04CD_DONE
