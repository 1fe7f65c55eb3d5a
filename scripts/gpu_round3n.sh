#!/bin/bash
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_native_mnist_gpu.py tests/test_wino_gpu.py -q --timeout 120 --timeout-method thread" \
  "120 MTA_FC1_SGD=0 python bench.py --steps 1000 --warmup 100 --no-eval" \
  "120 MTA_FC1_SGD=1 python bench.py --steps 1000 --warmup 100 --no-eval" \
  "120 MTA_FC1_SGD=0 python bench.py --steps 20 --warmup 5" \
  "120 MTA_FC1_SGD=1 python bench.py --steps 20 --warmup 5" \
  "200 bash scripts/gpu_mnist_prof.sh"
