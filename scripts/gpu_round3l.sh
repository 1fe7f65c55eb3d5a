#!/bin/bash
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_wino_gpu.py tests/test_native_mnist_gpu.py tests/test_mnist_bf16_gpu.py -q --timeout 120 --timeout-method thread" \
  "120 python bench.py --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --steps 20 --warmup 5" \
  "120 python bench.py --dtype bf16 --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --dtype bf16 --steps 20 --warmup 5" \
  "120 python scripts/wino_lab.py --phases --reps 200" \
  "200 bash scripts/gpu_mnist_prof16.sh"
