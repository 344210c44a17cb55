#!/bin/bash
# Round 3, session 2, call 3: k_step2 templated per (REWARD lanes, ray lanes) schedule
# + REWARD late-address recompute (no spills at the 64-VGPR cap): full GPU suite,
# smoke, per-wave fill profile of k_step2 (tools/wave_profile.py), same-session A/B
# against the HEAD kernels (librx_k2old: HEAD's rx_kernels.hip behind this ABI).
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r03s2c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for n in 65536 4096; do
  timeout -k 10 200 python tools/wave_profile.py $n 4 > $OUT/wave_profile_$n.json 2> $OUT/wave_profile.err || { tail -20 $OUT/wave_profile.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/wave_profile_$n.json'))
for l in d['launches'][:2]: print($n, {k:v for k,v in l.items() if k!='active_waves_by_us'})"
done
AB_SETS="old|k2old|;new||" OUT_SUB=r03s2c bash tools/ab_args.sh || exit 1
echo S2C_DONE
