#!/bin/bash
# Round-3 diagnosis session: BN backward statistics lab, ResNet-18 A/B of the
# BN statistics epilogues + kernel trace, MNIST kernel lab, bf16 trace,
# accuracy prints.   gpurun -- 'bash scripts/gpu_round3b.sh'
cd /root/repo
O=gpurun_out
RB="python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10 --no-eval"
bash scripts/gpu_session.sh \
  "60 python scripts/bnb_debug.py" \
  "120 $RB" \
  "120 MTA_BN_BWD_EPILOGUE=0 $RB" \
  "120 MTA_BN_BWD_EPILOGUE=0 MTA_BN_FWD_EPILOGUE=0 $RB" \
  "120 python scripts/kernel_lab.py --reps 200" \
  "200 bash scripts/gpu_resnet_prof16.sh" \
  "200 bash scripts/gpu_mnist_prof16.sh" \
  "400 python -u -m pytest tests/test_accuracy_gpu.py -x -q -s --timeout 300 --timeout-method thread"
