#!/bin/bash
# Round 3 profiling evidence under profiles/r03 (profiling builds; the product library has no stamps):
#   k_ppo_grad phase stamps incl. the forward's sub-phases (tools/ppo_stamps.py; build it here first:
#   python tools/ppo_stamps.py build), persistent-rollout phases (every ray wave; the REWARD half's
#   own phases, tools/rollout_stamps.py), and a kernel trace of back-to-back fused minibatch steps
#   (tools/ppo_micro.py) for the graph's kernel-to-kernel gaps (tools/trace_gaps.py).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python tools/ppo_stamps.py 32768 fp32 > $OUT/ppo_grad_stamps_fp32.json 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
timeout -k 10 120 python tools/ppo_stamps.py 32768 bf16 > $OUT/ppo_grad_stamps_bf16.json 2>> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
timeout -k 10 120 python tools/rollout_stamps.py 16 512 > $OUT/rollout_stamps_16env.json 2>> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
timeout -k 10 120 python tools/rollout_stamps.py 16 512 dyn > $OUT/rollout_reward_phases_16env.json 2>> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ppoprof -o run -- \
  python tools/ppo_micro.py 32768 fp32 > $OUT/ppo_micro_prof.log 2>&1 || { tail -5 $OUT/ppo_micro_prof.log; exit 1; }
cp $(find /tmp/ppoprof -name '*kernel_stats.csv' | head -1) $OUT/ppo_micro_update_kernel_stats.csv
python tools/trace_gaps.py $(find /tmp/ppoprof -name '*kernel_trace.csv' | head -1) | grep -E "k_ppo|k_adam" > $OUT/ppo_micro_update_gaps.txt
echo PROFILES_DONE
