#!/bin/bash
cd /root/repo
T="python -u -m pytest tests/test_generic_ops_gpu.py -q --timeout 120 --timeout-method thread -k bn_backward_epilogue"
bash scripts/gpu_session.sh \
  "120 MTA_BNB_ROUTES=0,0 $T" \
  "120 MTA_BNB_ROUTES=1,1 $T" \
  "120 python -u -m pytest tests/test_wino_gpu.py tests/test_native_mnist_gpu.py -q --timeout 120 --timeout-method thread" \
  "120 python scripts/wino_lab.py --phases --reps 200" \
  "120 python bench.py --steps 1000 --warmup 100 --no-eval" \
  "120 python bench.py --steps 20 --warmup 5"
