# SQ counters of one GEMM (tools/gemm_one.py), k_bres and k_x3nt, two passes each (8 SQ counters per pass).
# Summaries per kernel: tools/pmc_gemm_summarize.py gpurun_out/pmc_gemm_*.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for algo in 1 0; do
  i=1
  for P in "$P1" "$P2"; do
    MARLMAZE_GEMM_BRES=$algo ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_gemm_b${algo}_p$i -o g --output-format csv -- python3 tools/gemm_one.py > gpurun_out/pmc_gemm_b${algo}_p$i.log 2>&1 || { echo "pass b$algo p$i failed"; exit 1; }
    i=$((i+1))
  done
done
echo "pmc_gemm rc=0"
