#!/bin/bash
# Mid-N single-agent step: one-kernel k_dyn1<4> + k_rays vs the split step (RX_DYN1_LPE=1: k_kin1 + k_step2)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do for n in ${NS:-2048 4096 8192}; do
  for cfg in "lpe4|RX_SEG_FILTER=1" "split|RX_DYN1_LPE=1" "split_lpe2|RX_DYN1_LPE=2"; do
    IFS='|' read -r label envs <<< "$cfg"
    echo -n "$label $n "; env $envs timeout -k 10 120 python tools/env_probe.py $n 1 400 | tail -1 || exit 1
  done
done; done
