#!/bin/bash
# fp32 BatchNorm forward statistics from the tiled forward: tests + A/B
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -q --timeout 120 --timeout-method thread" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_BN_FWD_F32=0 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_BN_FWD_F32=0 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval"
