#!/bin/bash
# k_pnet phase probe: timing per VTF_PNET_DEBUG phase-skip mask, then two SQ counter passes per
# mask, summarised on the box.  bash scripts/probe_pnet_pmc.sh TAG "masks"
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pp_$1
MASKS=${2:-"0 1 2 4 8 127"}
mkdir -p $O
timeout -k 10 400 python3 -u scripts/probe_pnet.py $MASKS > $O/masks.txt 2> $O/masks.err
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for m in $MASKS; do
    VTF_PNET_DEBUG=$m timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/p1_$m -o run --output-format csv -- python3 scripts/probe_pnet.py child > /dev/null 2>> $O/pmc.err
    VTF_PNET_DEBUG=$m timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/p2_$m -o run --output-format csv -- python3 scripts/probe_pnet.py child > /dev/null 2>> $O/pmc.err
    VTF_PNET_DEBUG=$m timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAVES -d $O/p3_$m -o run --output-format csv -- python3 scripts/probe_pnet.py child > /dev/null 2>> $O/pmc.err
done
KFILTER='true>' python3 scripts/probe_pnet_table.py $O $MASKS > $O/table_x.txt
python3 scripts/probe_pnet_table.py $O $MASKS > $O/table.txt
find $O -name '*.csv' -size +5M -delete
cat $O/masks.txt $O/table.txt $O/table_x.txt
