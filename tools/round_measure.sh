#!/bin/bash
# Round measurement: full GPU tests, smoke, headline bench, rocprof stats, PPO time-to-90% runs.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=tests,smoke,bench,prof bash tools/gpu_check.sh || exit $?
for a in "--num-envs 16 --num-steps 2048 --eval-every 1" \
         "--num-envs 4096 --num-steps 128 --eval-every 1" \
         "--num-envs 4096 --num-steps 128 --eval-every 1 --device-shuffle"; do
  timeout -k 10 600 python tools/time_to_success.py $a --max-minutes 5 > "$OUT/tts.tmp" 2> "$OUT/tts.err"; rc=$?
  [ $rc -eq 0 ] || { echo "time_to_success failed ($rc): $a"; tail -20 "$OUT/tts.err"; exit $rc; }
  tail -1 "$OUT/tts.tmp" >> "$OUT/time_to_90.jsonl"
done
python - "$OUT/time_to_90.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["config"]["num_envs"], d["config"]["num_steps"], d["config"].get("shuffle"), "->", d.get("value_s"), "s at step", d.get("reached_at_step"))
PY
