#!/bin/bash
cd /root/repo
bash scripts/gpu_session.sh \
  "120 MTA_BNB_CHECK=1 python scripts/bnb_model_check.py --hw 32 --batch 32" \
  "200 python -u -m pytest tests/test_wino_gpu.py tests/test_native_mnist_gpu.py tests/test_mnist_bf16_gpu.py -q --timeout 120 --timeout-method thread" \
  "120 python scripts/wino_lab.py --phases --reps 200" \
  "120 python bench.py --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --steps 20 --warmup 5" \
  "300 python -u -m pytest tests/test_accuracy_gpu.py -q -s -k 'native_full_run' --timeout 300 --timeout-method thread"
