set -e
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generic_ops_gpu.py -k "bf16 or join or resnet" > gpurun_out/t0.log 2>&1
timeout -k 10 300 python scripts/conv_lab.py --batch 32 --dtype bf16 > gpurun_out/conv_lab.log 2>&1
timeout -k 10 300 python bench.py --model resnet18 --dtype bf16 --steps 50 --warmup 10 > gpurun_out/b_rn.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d /root/repo/gpurun_out/pmc1 -o p -- python /root/repo/scripts/conv_lab.py --layers 1,3,6 --ops fwd --reps 10 > /root/repo/gpurun_out/pmc1.log 2>&1
