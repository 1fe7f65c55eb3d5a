#!/bin/bash
# fp32 ResNet-18 conv survey: per-layer op times + step trace
cd /root/repo
R=/root/repo
O=$R/gpurun_out
bash scripts/gpu_session.sh \
  "200 python scripts/conv_lab.py --dtype fp32 --reps 10" \
  "150 python bench.py --model resnet18 --steps 30 --warmup 10 --no-eval" \
  "200 bash scripts/gpu_resnet_prof32.sh"
