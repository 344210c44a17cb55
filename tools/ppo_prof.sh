set -u
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ppo_prof -o run --output-format csv -- python tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 2 > $OUT/ppo_prof.log 2>&1 || { tail -20 $OUT/ppo_prof.log; exit 1; }
tail -1 $OUT/ppo_prof.log
python - <<'PY'
import csv,glob,os
f=glob.glob(os.environ["GRAFT_REPO_ROOT"]+"/gpurun_out/ppo_prof/**/*kernel_stats.csv",recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:90], r["Calls"], r["AverageNs"], r["Percentage"])
PY
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
grep -c . $OUT/counters_list.txt
