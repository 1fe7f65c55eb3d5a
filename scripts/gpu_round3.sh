#!/bin/bash
# Round-3 checkpoint session: GPU tests, smoke, driver-window benches, and the
# MNIST / ResNet-18 kernel traces (gpurun -- 'bash scripts/gpu_round3.sh')
cd /root/repo
bash scripts/gpu_session.sh \
  "120 python -u -m pytest tests/test_generic_ops_gpu.py tests/test_mnist_bf16_gpu.py -x -q -k 'dgrad_epilogue or fused_conv12' --timeout 120 --timeout-method thread" \
  "700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "60 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "120 python bench.py --steps 20 --warmup 5" \
  "120 python bench.py --steps 20 --warmup 5 --dtype bf16" \
  "120 python bench.py --model resnet18 --dtype bf16 --steps 30 --warmup 10" \
  "200 bash scripts/gpu_mnist_prof.sh"
