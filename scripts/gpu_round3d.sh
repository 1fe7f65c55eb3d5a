#!/bin/bash
cd /root/repo
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -x -q -k 'bn_backward_epilogue or resnet18_bf16_trains or dgrad_epilogue' --timeout 120 --timeout-method thread" \
  "120 python scripts/wino_lab.py --phases --reps 200" \
  "120 python scripts/wino_lab.py --reps 200"
