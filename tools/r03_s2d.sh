#!/bin/bash
# Round 3, session 2, call 4: k_step2 wave-fill profile with per-class costs
# (tools/wave_profile.py) and a same-session A/B of the ray-wave dispatch order
# (RX_RAY_DISPATCH builds: 0 tree default, 1 centre classes first, 2 class-major
# ascending, 3 edge classes first).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2d; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
summ() { python3 -c "
import json;d=json.load(open('$1'))
for l in d['launches'][:2]: print('$2', {k:v for k,v in l.items() if k not in ('active_waves_by_us','raw_start_us','raw_end_us')})"; }
timeout -k 10 200 python tools/wave_profile.py 65536 4 > $OUT/wave_profile_65536.json 2> $OUT/wp.err || { tail -20 $OUT/wp.err; exit 1; }
summ $OUT/wave_profile_65536.json tree
for m in 1 3; do
  RX_LIB_PATH=$LIB/librx_disp$m.so timeout -k 10 200 python tools/wave_profile.py 65536 4 > $OUT/wave_profile_65536_disp$m.json 2> $OUT/wp.err || { tail -20 $OUT/wp.err; exit 1; }
  summ $OUT/wave_profile_65536_disp$m.json disp$m
done
AB_SETS="tree||;disp1|disp1|;disp2|disp2|;disp3|disp3|" OUT_SUB=r03s2d bash tools/ab_args.sh || exit 1
echo S2D_DONE
