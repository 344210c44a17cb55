#!/bin/bash
# k_flow bring-up: the window parity tests on the task-graph path, then its throughput
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05e}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_window_gpu.py \
  -k "k_flow and (4096 or ragged)" > $OUT/pytest_flow_small.txt 2>&1 || { tail -40 $OUT/pytest_flow_small.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/pytest_flow_small.txt | tail -8
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -m gpu tests/test_window_gpu.py \
  > $OUT/pytest_window_all.txt 2>&1 || { tail -40 $OUT/pytest_window_all.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $OUT/pytest_window_all.txt | tail -16
timeout -k 10 200 python -u tools/window_probe.py --envs 65536 --steps 400 --reps 2 --mode 2 --label flow \
  > $OUT/probe_flow.jsonl 2> $OUT/probe_flow.err || { tail -20 $OUT/probe_flow.err; exit 1; }
cut -c1-1500 $OUT/probe_flow.jsonl
echo R05E_DONE
