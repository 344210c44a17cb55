#!/bin/bash
# Round 4, call L: box tests LPR at a time for rays at 2 / 4 lanes per ray (RX_BOX_BATCH,
# A/B build librx_bb.so): bit-exact env tests on it, then env probes at the LPR 4 / 2 sizes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04l; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
RX_LIB_PATH=$LIB/librx_bb.so timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_env_gpu.py tests/test_fullsize_gpu.py > $OUT/pytest_bb.txt 2>&1 || { tail -60 $OUT/pytest_bb.txt; exit 1; }
tail -2 $OUT/pytest_bb.txt
for rep in 1 2 3; do
  for v in t bb; do
    p=""; [ $v != t ] && p=$LIB/librx_$v.so
    for cfg in "4096 1" "8192 1" "16384 1" "2048 2" "4096 2"; do
      RX_LIB_PATH=$p timeout -k 10 120 python -u tools/env_probe.py $cfg 400 | sed "s/^/$v $cfg /" | cut -c1-170 >> $OUT/probe_ab.txt || exit 1
    done
  done
done
python3 - $OUT/probe_ab.txt <<'PY'
import json, sys, collections
r = collections.defaultdict(list)
for l in open(sys.argv[1]):
    v, n, a, js = l.split(" ", 3)
    try:
        d = json.loads(js)
    except Exception:
        d = {"env_steps_per_s": float(js.split('"env_steps_per_s": ')[1].split(",")[0])}
    r[(int(n), int(a), v)].append(d["env_steps_per_s"] / 1e6)
for k in sorted(r):
    print(k, [round(x, 1) for x in sorted(r[k])])
PY
echo R04L_DONE
