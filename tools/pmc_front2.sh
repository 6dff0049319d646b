# SQ counters of the front-end kernels (tools/bench_front.py), three passes; summarised per kernel by
# tools/pmc_front2_summarize.py.
# usage: tools/pmc_front2.sh [tag]  (tag names the output dirs; MARLMAZE_FRONT_BWD / MARLMAZE_FRONT_FWD pick
# the backward / forward kernels, default valu / row1)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${1:-}
export MARLMAZE_FRONT_BWD=${MARLMAZE_FRONT_BWD:-valu}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P3="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_COUNT"
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmc_front2${T}_p$i -o f --output-format csv -- python3 tools/bench_front.py > gpurun_out/pmc_front2${T}_p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo "pmc_front2 rc=0"
