set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc1 -o p -- python $R/scripts/conv_lab.py --layers 1,3,6 --ops fwd --reps 10 > $R/gpurun_out/pmc1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_VALU FETCH_SIZE -d $R/gpurun_out/pmc2 -o p -- python $R/scripts/conv_lab.py --layers 1,3,6 --ops fwd --reps 10 > $R/gpurun_out/pmc2.log 2>&1
