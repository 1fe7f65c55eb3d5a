#!/bin/bash
# diagnosis: NaN in the BN backward statistics route test
cd /root/repo
bash scripts/gpu_session.sh \
  "200 env MTA_BNB_CHECK=1 python -u -m pytest tests/test_generic_ops_gpu.py -q -x -s --timeout 120 --timeout-method thread" \
  "200 python -u -m pytest tests/test_generic_ops_gpu.py -q --timeout 120 --timeout-method thread -k 'dgrad_epilogue or bn_backward or batchnorm'"
