#!/bin/bash
# Kernel traces + PMC counters of the bench workloads (run on the GPU box through gpurun).
#   bash scripts/profile_r02.sh TAG [c2 c3 c4]
# Outputs under gpurun_out/prof_TAG/; summarise with scripts/kstats.py and scripts/pmc_table.py.
# Counter passes are separate runs (one block's slots each, MI355X_MICROARCH.md "PMC slots"):
#   sq:    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
#          SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE + GRBM_GUI_ACTIVE
#   fetch: FETCH_SIZE (x2 on gfx950 for wide streaming reads)     write: WRITE_SIZE
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
shift || true
CFGS=${@:-c2 c3 c4}
O=gpurun_out/prof_$TAG
mkdir -p $O
B="--no-cpu-baseline --no-extras --sustain-frames 0"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for c in $CFGS; do
  # default lanes under the tracer, then one lane (the kernels' own durations)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${c}_trace -o run -- python3 bench.py --config $c --steps 10 --warmup 3 $B > $O/${c}_trace.json 2> $O/${c}_trace.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${c}_trace1 -o run -- python3 bench.py --config $c --steps 10 --warmup 3 --lanes 1 $B > $O/${c}_trace1.json 2> $O/${c}_trace1.err
  timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/${c}_pmc_sq -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --lanes 1 $B > /dev/null 2> $O/${c}_pmc_sq.err
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${c}_pmc_fetch -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --lanes 1 $B > /dev/null 2> $O/${c}_pmc_fetch.err
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/${c}_pmc_write -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --lanes 1 $B > /dev/null 2> $O/${c}_pmc_write.err
  echo "$c done"
done
echo profile-done
