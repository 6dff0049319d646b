# SQ counters of the front-end kernels (tools/bench_front.py), one pass per backward algorithm.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
for algo in mfma valu; do
  MARLMAZE_FRONT_BWD=$algo timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU -d gpurun_out/pmc_front_$algo -o front --output-format csv -- python3 tools/bench_front.py > gpurun_out/pmc_front_$algo.log 2>&1 || exit 1
done
echo "pmc_front rc=0"
