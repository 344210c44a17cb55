#!/bin/bash
# Round 3, session 2, call 9: REWARD workgroups after the ray ones (librx_rlast,
# RX_REWARD_LAST=1) vs first (tree), and the spatial re-sort period (8 / 16 / 32).
set -u
export TMPDIR=/tmp
AB_SETS="tree||;rlast|rlast|;sort8||--sort-interval 8;sort32||--sort-interval 32;tree4k||--envs-per-gpu 4096;rlast4k|rlast|--envs-per-gpu 4096" OUT_SUB=r03s2i bash tools/ab_args.sh || exit 1
echo S2I_DONE
