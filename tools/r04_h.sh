#!/bin/bash
# Round 4, call H: k_ppo_grad A/B, same session: HEAD, the tree (scalar loads of the
# uniform operands + epilogue index remat: zero scratch), the tree without the remat.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r04h; mkdir -p $OUT; export TMPDIR=/tmp
LIB=$(pwd)/self-play-racing_amd/rx/lib
for rep in 1 2 3; do
  for prec in fp32 bf16; do
    for v in head tree noremat; do
      p=""; [ $v != tree ] && p=$LIB/librx_$v.so
      RX_LIB_PATH=$p timeout -k 10 120 python -u tools/ppo_micro.py 32768 $prec $v >> $OUT/ppo_micro_ab.jsonl 2>> $OUT/ppo_micro.err || { tail -20 $OUT/ppo_micro.err; exit 1; }
    done
  done
done
python3 - $OUT/ppo_micro_ab.jsonl <<'PY'
import json, sys, collections
r = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r[(d["precision"], d["label"])].append((d["grad_us"], d["update_us"]))
for k, v in sorted(r.items()):
    print(k, "grad", sorted(x[0] for x in v), "update", sorted(x[1] for x in v))
PY
echo R04H_DONE
