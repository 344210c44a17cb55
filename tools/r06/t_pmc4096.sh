#!/bin/bash
# r06 t: steady-state PMC of the env kernels at 4,096 envs (configs[1]'s env size: LPR 4, the latency-bound regime)
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pmc_steady.py $O/pmc_4096.json --envs 4096 --scratch gpurun_out/pmc4096 > $O/pmc.log 2>&1 \
  || { tail -30 $O/pmc.log; exit 1; }
