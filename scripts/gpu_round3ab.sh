#!/bin/bash
# fp32 phase-decomposed dgrad with transposed weights (MTA_TILED_DGRAD_WT): tests + A/B
cd /root/repo
bash scripts/gpu_session.sh \
  "300 python -u -m pytest tests/test_generic_ops_gpu.py -q -x --timeout 240 --timeout-method thread" \
  "120 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops dgrad" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_DGRAD_WT=0 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_DGRAD_WT=0 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval"
