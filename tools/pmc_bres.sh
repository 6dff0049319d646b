# SQ counters of k_bres on one shape (tools/gemm_one.py), three passes (8 SQ counters each at most).
# Summary: python tools/pmc_gemm_summarize.py "gpurun_out/pmc_bres_p*"
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
i=1
for P in "$P1" "$P2" "$P3"; do
  ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_bres_p$i -o g --output-format csv -- python3 tools/gemm_one.py > gpurun_out/pmc_bres_p$i.log 2>&1 || { echo "pass p$i failed"; exit 1; }
  i=$((i+1))
done
echo "pmc_bres rc=0"
