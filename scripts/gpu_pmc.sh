set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d $R/gpurun_out/pmc1 -o p -- python $R/scripts/conv_lab.py --batch 128 --layers 1,2 --ops fwd,dgrad --reps 5 > $R/gpurun_out/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU FETCH_SIZE -d $R/gpurun_out/pmc2 -o p -- python $R/scripts/conv_lab.py --batch 128 --layers 1,2 --ops fwd,dgrad --reps 5 > $R/gpurun_out/pmc2.log 2>&1
