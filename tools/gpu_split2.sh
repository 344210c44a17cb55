set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_env_gpu.py -m gpu -k "split or multi or two_car" > gpurun_out/t_split2.log 2>&1 || { tail -30 gpurun_out/t_split2.log; exit 1; }
tail -3 gpurun_out/t_split2.log
for n in 8192 65536; do for s in 0 1; do RX_SPLIT=$s timeout -k 10 120 python tools/env_probe.py $n 2 400; done; done
timeout -k 10 300 python tools/bench_ppo.py --mode selfplay --envs 8192 --steps 128
