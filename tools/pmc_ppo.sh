#!/bin/bash
# PMC passes over the PPO training loop (tools/bench_ppo.py): MFMA / VALU / LDS / wait counters of
# k_ppo_grad, k_policy_act and the optimizer kernels, counters only.
set -u
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python tools/pmc_steady.py $OUT/pmc_ppo.json --last 64 --scratch $OUT/pmc_ppo \
  --cmd "tools/bench_ppo.py --envs 4096 --steps 128 --device-shuffle --updates 1" \
  --passes "SQ_INSTS_VALU_MFMA_MOPS_F32,SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,GRBM_GUI_ACTIVE;SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU_TRANS_F32,SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,GRBM_GUI_ACTIVE" \
  > $OUT/pmc_ppo.log 2>&1 || { tail -30 $OUT/pmc_ppo.log; exit 1; }
python - $OUT/pmc_ppo.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if isinstance(v, dict):
        print(k, {c: round(x) if isinstance(x, float) else x for c, x in v.items()})
PY
