#!/bin/bash
# stem filter-gradient slice cap 256: numerics + ResNet fp32 / LeNet steps
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py tests/test_lenet_native_gpu.py -q --timeout 120 --timeout-method thread" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_GCAP=128 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval"
