#!/bin/bash
# SQ/TCC counter passes (one rocprofv3 run per counter group) over an arbitrary python probe.
# usage: tools/pmc_cmd.sh <tag> <python args...>     (env is inherited: FS2_* switches apply)
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G -d $OUT/g$i -o pmc --output-format csv -- python3 "$@" > $OUT/g$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "group $i ($G) failed rc=$rc" >> $OUT/errors.txt; [ $rc -ge 124 ] && exit $rc; fi
done
echo done
