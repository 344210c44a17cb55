#!/bin/bash
# Round-2 final measurement: headline bench + rocprofv3 + steady-state PMC (tools/round2_measure.sh),
# then PPO throughput at the BASELINE configs and the two-car env probe.  Stops at the first failure.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/round2_measure.sh || exit 1
: > $OUT/ppo_final.jsonl
for a in "--mode single --envs 16 --steps 2048" "--mode single --envs 4096 --steps 128 --device-shuffle" \
         "--mode single --envs 4096 --steps 128 --device-shuffle --bf16" "--mode single --envs 65536 --steps 64 --device-shuffle" \
         "--mode selfplay --envs 8192 --steps 128 --device-shuffle" "--mode selfplay --envs 8192 --steps 128"; do
  timeout -k 10 300 python tools/bench_ppo.py $a > $OUT/ppo_one.log 2>&1 || { tail -20 $OUT/ppo_one.log; exit 1; }
  grep '^{' $OUT/ppo_one.log | tail -1 >> $OUT/ppo_final.jsonl
  tail -1 $OUT/ppo_final.jsonl | cut -c1-400
done
: > $OUT/env_probe_final.jsonl
for na in "65536 2" "8192 2" "4096 1" "16 1"; do
  timeout -k 10 120 python tools/env_probe.py $na 400 | tail -1 >> $OUT/env_probe_final.jsonl || exit 1
  tail -1 $OUT/env_probe_final.jsonl
done
echo FINAL_DONE
