#!/bin/bash
cd /root/repo
T="python -u -m pytest tests/test_generic_ops_gpu.py -q --timeout 120 --timeout-method thread"
bash scripts/gpu_session.sh \
  "120 $T -k bn_backward_epilogue" \
  "120 MTA_BN_BWD_EPILOGUE=0 $T -k resnet18_bf16_trains" \
  "120 MTA_BN_BWD_EPILOGUE=1 MTA_BN_FWD_EPILOGUE=0 $T -k resnet18_bf16_trains" \
  "200 bash scripts/gpu_resnet_ab.sh"
