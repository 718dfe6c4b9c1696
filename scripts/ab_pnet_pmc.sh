#!/bin/bash
# k_pnet A/B of two builds on one box with counters: lib/libvtf_hip_base.so ("base") vs
# lib/libvtf_hip.so ("new").  Solo timing (interleaved, 3 rounds), phase clocks (VTF_PNET_DEBUG=256)
# and the three SQ counter passes of probe_pnet_pmc.sh per build; tables for both variants.
# bash scripts/ab_pnet_pmc.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/apm_${1:-a}
mkdir -p $O
L=$PWD/video-to-faces_amd/lib
for rep in 1 2 3; do
  for t in base new; do
    lib=$L/libvtf_hip_$t.so; [ $t = new ] && lib=$L/libvtf_hip.so
    VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/t.txt 2> $O/t.err
    echo "$t pnet $(tail -1 $O/t.txt)"
  done
done
for t in base new; do
  lib=$L/libvtf_hip_$t.so; [ $t = new ] && lib=$L/libvtf_hip.so
  VTF_HIP_LIB=$lib VTF_PNET_DEBUG=256 timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/clk_$t.txt 2> $O/clk_$t.err
  echo "$t $(grep -m1 'phase clocks' $O/clk_$t.err)"
done
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for t in base new; do
  lib=$L/libvtf_hip_$t.so; [ $t = new ] && lib=$L/libvtf_hip.so
  VTF_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $P1 -d $O/p1_$t -o run --output-format csv -- python3 scripts/probe_pnet.py child > /dev/null 2>> $O/pmc.err
  VTF_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $P2 -d $O/p2_$t -o run --output-format csv -- python3 scripts/probe_pnet.py child > /dev/null 2>> $O/pmc.err
  VTF_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAVES -d $O/p3_$t -o run --output-format csv -- python3 scripts/probe_pnet.py child > /dev/null 2>> $O/pmc.err
done
KFILTER='true>' python3 scripts/probe_pnet_table.py $O base new > $O/table_x.txt
KFILTER='false>' python3 scripts/probe_pnet_table.py $O base new > $O/table_g.txt
find $O -name '*.csv' -size +5M -delete
cat $O/table_x.txt $O/table_g.txt
