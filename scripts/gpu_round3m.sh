#!/bin/bash
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_wino_gpu.py tests/test_native_mnist_gpu.py tests/test_mnist_bf16_gpu.py -q --timeout 120 --timeout-method thread" \
  "200 bash scripts/gpu_mnist_prof.sh" \
  "200 bash scripts/gpu_mnist_prof16.sh"
