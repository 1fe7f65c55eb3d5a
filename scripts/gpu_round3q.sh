#!/bin/bash
# fp32 tiled gather forward (ResNet stem): numerics, per-layer time, step
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "120 python scripts/conv_lab.py --dtype fp32 --layers 0,1 --reps 10" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10" \
  "150 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval"
