#!/bin/bash
# Round 3, session 2, call 10: steady-state PMC counters of the production env kernels
# after the dispatch-order change (tools/pmc_steady.py, one counter group per pass).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03pmc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 tools/pmc_steady.py $OUT/pmc_steady.json --scratch /tmp/pmcs > $OUT/pmc.log 2>&1 || { tail -30 $OUT/pmc.log; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/pmc_steady.json'))
for k in ('k_step2','k_kin1'): print(k, {c:d[k].get(c) for c in ('FETCH_SIZE','WRITE_SIZE','hbm_bytes_per_launch','SQ_INSTS_VALU','SQ_ACTIVE_INST_VALU','GRBM_GUI_ACTIVE','SQ_WAVES','l2_hit_rate')})"

# where a configs[1] PPO iteration goes (fp32 and bf16, device shuffles): rocprofv3 kernel stats
for p in fp32 bf16; do
  extra=""; [ $p = bf16 ] && extra="--bf16"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ppoprof_$p -o run -- \
    python3 tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 3 $extra > $OUT/bench_ppo_prof_$p.jsonl 2> $OUT/bench_ppo_prof_$p.err || { tail -20 $OUT/bench_ppo_prof_$p.err; exit 1; }
  cp $(find /tmp/ppoprof_$p -name '*kernel_stats.csv' | head -1) $OUT/ppo_prof_${p}_kernel_stats.csv
  echo "== $p"; tail -1 $OUT/bench_ppo_prof_$p.jsonl; python3 tools/kstats.py $OUT/ppo_prof_${p}_kernel_stats.csv 14
done
echo PPOPROF_DONE
