#!/bin/bash
# Same-session A/B of librx variants on the configs[1] PPO update (k_ppo_grad time from rocprofv3):
#   LIBS="base wg512 wg128" bash tools/gpu_ppo_ab.sh
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
LIBDIR=$(pwd)/self-play-racing_amd/rx/lib
for rep in 1 2; do for lib in $LIBS; do
  p=""; [ "$lib" != base ] && p=$LIBDIR/librx_$lib.so
  RX_LIB_PATH=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ppoab_$lib -o run --output-format csv -- \
    python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 2 ${X:-} > $OUT/ppoab_$lib.log 2>&1 || { tail -20 $OUT/ppoab_$lib.log; exit 1; }
  python - $lib $OUT/ppoab_$lib <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = {r["Name"]: r for r in csv.DictReader(open(f))}
g = [r for n, r in rows.items() if "k_ppo_grad" in n][0]
log = [l for l in open(sys.argv[2] + ".log") if l.startswith("{")][-1]
d = json.loads(log)
print(sys.argv[1], "k_ppo_grad_us", round(float(g["AverageNs"]) / 1e3, 2), "update_ms", round(d["update_s"] * 1e3, 2),
      "train_Msteps", round(d["train_env_steps_per_s"] / 1e6, 2))
PY
done; done
