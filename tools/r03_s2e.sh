#!/bin/bash
# Round 3, session 2, call 5: class-order search for the ray-wave dispatch
# (65,536 envs) and the RX_RAY_DISPATCH modes at 4,096 envs (configs[1] geometry).
set -u
export TMPDIR=/tmp
AB_SETS="tree||;disp3|disp3|;ordb|ordb|;ordc|ordc|;ordd|ordd|;orde|orde|;ordf|ordf|;ordg|ordg|" OUT_SUB=r03s2e bash tools/ab_args.sh || exit 1
AB_SETS="t4096||--envs-per-gpu 4096;d3_4096|disp3|--envs-per-gpu 4096;d1_4096|disp1|--envs-per-gpu 4096;d2_4096|disp2|--envs-per-gpu 4096" OUT_SUB=r03s2e bash tools/ab_args.sh || exit 1
echo S2E_DONE
