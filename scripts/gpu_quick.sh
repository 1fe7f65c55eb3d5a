set -e
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generic_ops_gpu.py > gpurun_out/t0.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --steps 50 --warmup 10 > gpurun_out/b_rn.log 2>&1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_rn -o rn -- python /root/repo/bench.py --model resnet18 --dtype bf16 --steps 10 --warmup 3 --no-eval > /root/repo/gpurun_out/prof_rn.log 2>&1
