set -e
cd /root/repo
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/tall.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --steps 30 --warmup 10 > gpurun_out/b_rn32_fp32.log 2>&1
