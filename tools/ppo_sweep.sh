#!/bin/bash
# PPO throughput sweep (tools/bench_ppo.py); stops at the first failing run.
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
: > "$OUT/bench_ppo.log"
while IFS= read -r a; do
  [ -z "$a" ] && continue
  timeout -k 10 300 python tools/bench_ppo.py $a >> "$OUT/bench_ppo.log" 2> "$OUT/bench_ppo.err"; rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED ($rc): $a"; tail -20 "$OUT/bench_ppo.err"; exit $rc; fi
done <<< "${SWEEP:-"--mode single --envs 16 --steps 2048 --no-graph
--mode single --envs 16 --steps 2048
--mode single --envs 4096 --steps 128
--mode single --envs 4096 --steps 128 --bf16
--mode single --envs 65536 --steps 64
--mode selfplay --envs 8192 --steps 128"}"
cat "$OUT/bench_ppo.log"
