#!/bin/bash
# Round 4, call AA: the timed region as one HIP graph replay of the --steps production steps
# (bench.py --graph on, default) against one rx_step call per step (--graph off): the driver's
# command twice each, interleaved, then 1,000 steady-state steps each way.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04aa; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for g in on off; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --graph $g --no-cpu-baseline --no-time-to-90 \
      --ppo-updates 0 --selfplay-updates 0 > $OUT/drv_$g$rep.jsonl 2> $OUT/drv_$g$rep.err || { tail -30 $OUT/drv_$g$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$g', 'driver20', round(d['value']/1e6,1), d['ms_per_step'], d['steady_state']['launch'])" $OUT/drv_$g$rep.jsonl
  done
done
for g in on off; do
  timeout -k 10 300 python -u bench.py --steps 1000 --warmup 5 --graph $g --no-cpu-baseline --no-time-to-90 --ppo-updates 0 \
    --selfplay-updates 0 > $OUT/steady_$g.jsonl 2> $OUT/steady_$g.err || { tail -30 $OUT/steady_$g.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$g', 'steady1000', round(d['value']/1e6,1), d['ms_per_step'])" $OUT/steady_$g.jsonl
done
echo R04AA_DONE
