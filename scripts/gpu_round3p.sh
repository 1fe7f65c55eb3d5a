#!/bin/bash
# fp32 tiled convs: loads two K tiles ahead (MTA_TILED_D2) A/B
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "200 env MTA_TILED_D2=0 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "200 env MTA_TILED_D2=1 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "150 env MTA_TILED_D2=0 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_D2=1 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_D2=0 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_D2=1 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model lenet5"
