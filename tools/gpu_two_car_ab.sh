set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_env_gpu.py tests/test_fullsize_gpu.py > $OUT/t5.log 2>&1; rc=$?
tail -3 $OUT/t5.log; [ $rc -eq 0 ] || exit $rc
LIBS="pre base m8" bash tools/ab_probe2.sh
