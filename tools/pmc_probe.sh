#!/bin/bash
# SQ/TCC counter passes (one rocprofv3 run per counter group) over one probe kernel.
# usage: tools/pmc_probe.sh <tag> <kernel>
TAG=$1; K=$2
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
[ -f $OUT/counters.txt ] || timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
         ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G -d $OUT/g$i -o pmc --output-format csv -- \
     python3 tools/kernel_probe.py $K --reps 5 > $OUT/g$i.log 2>&1 || echo "group $i ($G) failed rc=$?" >> $OUT/errors.txt
done
echo done
