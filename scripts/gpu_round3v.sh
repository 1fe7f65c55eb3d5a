#!/bin/bash
# fp32 tiled convs: 64-column fwd / dgrad tiles experiment (MTA_TILED_N64), step A/B
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -q -x --timeout 120 --timeout-method thread -k 'conv_fwd_bwd or batchnorm or resnet'" \
  "120 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "120 env MTA_TILED_N64=1 python scripts/conv_lab.py --dtype fp32 --reps 10 --ops fwd,dgrad" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_N64=1 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "150 env MTA_TILED_N64=1 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval"
