#!/bin/bash
# bf16 k_ppo_grad: rows-per-workgroup variants (RX_PPO_MAXWG 128 / 256 / 512) in ppo_micro, then the
# closing PMC of the new kernel over the configs[1] training loop (counters only, two passes)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${RUN_DIR:-r05m}; mkdir -p $OUT; export TMPDIR=/tmp
for v in new bfw128 bfw512 new; do
  if [ $v = new ]; then unset RX_LIB_PATH; else export RX_LIB_PATH=$(pwd)/build/variants/$v.so; fi
  timeout -k 10 120 python -u tools/ppo_micro.py 32768 bf16 $v > $OUT/micro_$v.jsonl 2> $OUT/micro_$v.err || { tail -20 $OUT/micro_$v.err; exit 1; }
  cat $OUT/micro_$v.jsonl
done
unset RX_LIB_PATH
timeout -k 10 600 python tools/pmc_steady.py $OUT/pmc_ppo_bf16.json --last 64 --scratch /tmp/pmc_ppo \
  --cmd "tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 1 --bf16" \
  --passes "SQ_INSTS_VALU_MFMA_MOPS_BF16,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,GRBM_GUI_ACTIVE;SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU_TRANS_F32,SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,GRBM_GUI_ACTIVE" \
  > $OUT/pmc_ppo_bf16.log 2>&1 || { tail -30 $OUT/pmc_ppo_bf16.log; exit 1; }
python3 - $OUT/pmc_ppo_bf16.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if isinstance(v, dict) and 'ppo' in k:
        print(k, {c: round(x) if isinstance(x, float) else x for c, x in v.items()})
PY
echo R05M_DONE
