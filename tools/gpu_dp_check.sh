set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ppo_fused_gpu.py tests/test_dist_gpu.py tests/test_optim_gpu.py -m gpu > $OUT/t2.log 2>&1; rc=$?; tail -25 $OUT/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --async-probe-groups 0 > $OUT/b2.log 2>&1; rc=$?; tail -1 $OUT/b2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ppo_train'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --async-probe-groups 0 > $OUT/b3.log 2>&1; rc=$?; tail -1 $OUT/b3.log; exit $rc
