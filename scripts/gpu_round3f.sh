#!/bin/bash
cd /root/repo
T="python -u -m pytest tests/test_generic_ops_gpu.py -q --timeout 120 --timeout-method thread"
bash scripts/gpu_session.sh \
  "120 MTA_BNB_CHECK=1 python scripts/bnb_model_check.py --hw 32 --batch 32" \
  "120 MTA_BNB_CHECK=1 MTA_BN_FWD_EPILOGUE=0 python scripts/bnb_model_check.py --hw 32 --batch 32" \
  "120 MTA_BN_FWD_EPILOGUE=0 $T -k bn_backward_epilogue" \
  "120 python scripts/wino_lab.py --phases --reps 200" \
  "120 python -u -m pytest tests/test_native_mnist_gpu.py tests/test_wino_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "120 python bench.py --steps 20 --warmup 5" \
  "120 python bench.py --steps 1000 --warmup 100 --no-eval"
