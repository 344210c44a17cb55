#!/bin/bash
# r06 y: steady-state PMC of the production env kernels on the round-6 tree (bench.py's compute_roofline /
# traffic source), one counter group per rocprofv3 --pmc pass (tools/pmc_steady.py)
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/pmc_steady.py $O/pmc_steady.json > $O/pmc_steady.log 2>&1 \
  || { tail -30 $O/pmc_steady.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/pmc_steady.json'));k=[x for x in d if 'k_step2' in x];print({x: {c: d[x].get(c) for c in ('SQ_INSTS_VALU','FETCH_SIZE','WRITE_SIZE','SQ_WAVE_CYCLES')} for x in k})"
