#!/bin/bash
# Round 4, call T: steady-state PMC counters of the final kernels (tools/pmc_steady.py, one
# counter group per rocprofv3 --pmc pass) -> the bench's traffic / compute-roofline source,
# then the driver's bench command reading them.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04t; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u tools/pmc_steady.py $OUT/pmc_steady.json --scratch /tmp/pmc_r04t > $OUT/pmc_steady.log 2>&1 \
  || { tail -30 $OUT/pmc_steady.log; exit 1; }
tail -3 $OUT/pmc_steady.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver20.jsonl 2> $OUT/bench_driver20.err \
  || { tail -30 $OUT/bench_driver20.err; exit 1; }
tail -c 300 $OUT/bench_driver20.jsonl; echo
echo R04T_DONE
