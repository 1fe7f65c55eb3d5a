#!/bin/bash
# BN backward statistics epilogue: debug lab, GPU tests, ResNet-18 A/B + trace
cd /root/repo
RB="python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval"
bash scripts/gpu_session.sh \
  "60 python scripts/bnb_debug.py" \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "120 $RB" \
  "120 MTA_BN_BWD_EPILOGUE=0 $RB" \
  "120 $RB --batch-size 128" \
  "200 bash scripts/gpu_resnet_prof16.sh"
