#!/bin/bash
# Round 4, call Y: the re-sort period across env counts now that a re-sort is two launches
# (~13 us at 65,536 envs): tools/env_probe.py at sort_interval 4 / 8 / 16, two interleaved passes.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04y; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "4096 1" "16384 1" "65536 1" "8192 2" "65536 2"; do
    for si in 4 8 16; do
      PROBE_SORT=$si timeout -k 10 120 python -u tools/env_probe.py $cfg 600 | cut -c1-110 >> $OUT/probe_sort.txt \
        || { tail -5 $OUT/probe_sort.txt; exit 1; }
    done
  done
done
cat $OUT/probe_sort.txt
echo R04Y_DONE
