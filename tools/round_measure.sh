#!/bin/bash
# Round measurement: full GPU tests, smoke, headline bench, rocprof stats, PMC traffic / VALU,
# PPO throughput and PPO time-to-90% runs.  Stops at the first failing step.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-tests,smoke,bench,prof} bash tools/gpu_check.sh || exit $?
if [ -z "${NO_PMC:-}" ]; then
  PMC_BENCH_ARGS="--steps 20 --warmup 100 --no-cpu-baseline --async-probe-groups 0 --ppo-updates 0 --sample-every 1" \
    bash tools/pmc.sh > "$OUT/pmc.out" 2>&1 || { tail -20 "$OUT/pmc.out"; exit 1; }
fi
: > "$OUT/bench_ppo.jsonl"
for a in "--envs 16 --steps 2048" "--envs 4096 --steps 128" "--envs 4096 --steps 128 --device-shuffle" \
         "--envs 65536 --steps 64 --device-shuffle" "--mode selfplay --envs 8192 --steps 128"; do
  timeout -k 10 300 python tools/bench_ppo.py $a >> "$OUT/bench_ppo.jsonl" 2> "$OUT/bench_ppo.err" || { echo "bench_ppo failed: $a"; tail -20 "$OUT/bench_ppo.err"; exit 1; }
done
: > "$OUT/time_to_90.jsonl"
for a in "--num-envs 16 --num-steps 2048 --eval-every 1" \
         "--num-envs 4096 --num-steps 128 --eval-every 1" \
         "--num-envs 4096 --num-steps 128 --eval-every 1 --device-shuffle"; do
  timeout -k 10 600 python tools/time_to_success.py $a --max-minutes 5 > "$OUT/tts.tmp" 2> "$OUT/tts.err"; rc=$?
  [ $rc -eq 0 ] || { echo "time_to_success failed ($rc): $a"; tail -20 "$OUT/tts.err"; exit $rc; }
  tail -1 "$OUT/tts.tmp" >> "$OUT/time_to_90.jsonl"
done
python - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
for l in open(out + "/bench_ppo.jsonl"):
    d = json.loads(l)
    print("ppo", d["mode"], d["envs"], d["num_steps"], d["shuffle"], "rollout %.3g train %.3g update %.1f ms" % (
        d["rollout_env_steps_per_s"], d["train_env_steps_per_s"], 1e3 * d["update_s"]))
for l in open(out + "/time_to_90.jsonl"):
    d = json.loads(l)
    print("tts", d["config"]["num_envs"], d["config"]["num_steps"], d["config"].get("shuffle"), "->", d.get("value_s"), "s at step", d.get("reached_at_step"))
PY
echo ROUND_DONE
