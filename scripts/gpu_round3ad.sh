#!/bin/bash
# fp32 filter-gradient slice cap 256: generic tests + step A/B vs 64 / 128
cd /root/repo
bash scripts/gpu_session.sh \
  "300 python -u -m pytest tests/test_generic_ops_gpu.py -q -x --timeout 240 --timeout-method thread" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_VCAP=128 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_VCAP=64 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_VCAP=128 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval"
