#!/bin/bash
# fp32 filter-gradient slice cap: step A/B (default 64 vs 128 vs 256)
cd /root/repo
bash scripts/gpu_session.sh \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_VCAP=128 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_VCAP=256 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_VCAP=128 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_VCAP=256 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval"
