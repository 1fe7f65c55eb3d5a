#!/bin/bash
# Round-3 closing: the two re-bounded GPU tests, then the kernel traces
cd /root/repo
bash scripts/gpu_session.sh \
  "300 python -u -m pytest tests/test_native_sync_gpu.py tests/test_accuracy_gpu.py -q --timeout 240 --timeout-method thread -k 'sharded_schedule_matches_buckets or resnet18_bf16_tracks'" \
  "200 bash scripts/gpu_mnist_prof.sh" \
  "200 bash scripts/gpu_mnist_prof16.sh" \
  "200 bash scripts/gpu_resnet_prof16.sh" \
  "200 bash scripts/gpu_resnet_prof32.sh" \
  "200 bash scripts/gpu_lenet_prof.sh"
