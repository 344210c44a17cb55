set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ppo_fused_gpu.py tests/test_optim_gpu.py tests/test_ppo_golden.py tests/test_bf16_gpu.py tests/test_ppo_gpu.py > $OUT/ab1_pytest.log 2>&1; rc=$?
tail -3 $OUT/ab1_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="head tree" bash tools/gpu_ppo_ab.sh
