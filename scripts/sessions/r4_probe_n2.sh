#!/bin/bash
# Round 4: world > 1 fused SGD + the driver's N>1 entry points on ONE GPU
cd /root/repo
bash scripts/gpu_session.sh \
  "100 python bench.py --steps 20 --warmup 5" \
  "100 python bench.py --dtype bf16 --steps 20 --warmup 5" \
  "100 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval" \
  "400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wino_gpu.py tests/test_native_mnist_gpu.py tests/test_mnist_bf16_gpu.py tests/test_captured_sync_gpu.py tests/test_native_sync_gpu.py" \
  "400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_generic_ops_gpu.py" \
  "600 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_driver_n2_gpu.py"
