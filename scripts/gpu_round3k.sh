#!/bin/bash
cd /root/repo
RB="python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval"
bash scripts/gpu_session.sh \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -q -x --timeout 120 --timeout-method thread" \
  "200 python scripts/conv_lab.py --ops fwd,dgrad --layers 1,3,6,9 --reps 20" \
  "120 $RB" \
  "120 MTA_BN_BWD_EPILOGUE=0 $RB" \
  "200 bash scripts/gpu_resnet_ab.sh"
