#!/bin/bash
# GPU-box: SQ counter passes (<= 8 SQ counters each) over the bench, for k_chain
# and k_level: wait / issue ratios and LDS bank conflicts.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
P=gpurun_out/sq_${1:-r2}
mkdir -p $P
B="bench.py --steps 3 --warmup 2 --cpu-baseline 0 --hotspot 0 --e2e 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $P/a -o a -- python3 -u $B > $P/a.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS --output-format csv -d $P/b -o b -- python3 -u $B > $P/b.txt 2>&1 &&
python3 tools/pmc_sum.py $P/a $P/b -k k_chain > $P/sum.txt && python3 tools/pmc_sum.py $P/a $P/b -k k_level >> $P/sum.txt
rc=$?
cat $P/sum.txt
exit $rc
