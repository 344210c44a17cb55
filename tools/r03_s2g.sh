#!/bin/bash
# Round 3, session 2, call 7: raycast wave phase stamps (tools/ray_stamps.py) and the
# driver's command after the per-step host trims (one stream lookup per step).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python tools/ray_stamps.py 65536 > $OUT/ray_stamps_65536.json 2> $OUT/rs.err || { tail -20 $OUT/rs.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/ray_stamps_65536.json'))
r=d['runs'][-1]; print('span',r['span_us'],'all',r['all']); print('tail',r['tail_last_25pct']); print('corr',r['corr_wall_us_vs_box_tests'],r['corr_wall_us_vs_leaf_scans'])
for i,x in enumerate(r['by_dispatch_rank']): print(i,x)"
for rep in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-time-to-90 --no-cpu-baseline --ppo-updates 0 > $OUT/driver20_$rep.jsonl 2> $OUT/driver20.err || { tail -20 $OUT/driver20.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/driver20_$rep.jsonl').read().splitlines()[-1]);print('driver20',d['value'],d['ms_per_step'],d['kernels_ms'])"
done
echo S2G_DONE
