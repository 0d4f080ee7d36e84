#!/bin/bash
# PMC passes over eager forwards (tools/fwd_probe.py; its args after the tag), one rocprofv3 run per
# counter group, then the per-launch table (tools/pmc_fwd.py): HBM MB (2 x FETCH_SIZE + WRITE_SIZE),
# MFMA busy per SIMD, kernel cycles.    usage: tools/pmc_fwd.sh <tag> [fwd_probe args]
TAG=$1; shift
OUT=gpurun_out/pmcf_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for G in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $G -d $OUT/g$i -o pmc --output-format csv -- python3 tools/fwd_probe.py "$@" \
    > $OUT/g$i.log 2>&1 || { echo "pmc group $i ($G) failed rc=$?"; tail -5 $OUT/g$i.log; exit 1; }
done
python3 tools/pmc_fwd.py $OUT --json $OUT/table.json > $OUT/table.txt && cat $OUT/table.txt
