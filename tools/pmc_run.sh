#!/bin/bash
# usage: tools/pmc_run.sh OUTDIR KERNEL_SUBSTR [bench args]  -- one rocprofv3 --pmc pass per counter group
OUT=$1; KER=$2; shift 2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_ANY" "FETCH_SIZE GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY" "WRITE_SIZE SQ_INSTS_VALU_MFMA_MOPS_F32" \
         "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  n=$(echo $P | tr " " _)
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d $OUT/$n -o run -- python3 bench.py --no-cpu "$@" > $OUT/$n.log 2>&1 || { echo "FAIL $n"; tail -5 $OUT/$n.log; exit 1; }
done
python tools/pmc_summary.py "$KER" $OUT/*/
