# MFMA utilisation of the bench's kernels: one rocprofv3 --pmc pass (SQ + GRBM
# counters only) over a short bench run, summarised per kernel by
# tools/pmc_mfma_summarize.py -> gpurun_out/pmc_mfma_bench.json.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma${1:+_$1} -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${1:+--dtype $1} > gpurun_out/pmc_mfma.log 2>&1 \
 && python3 tools/pmc_mfma_summarize.py gpurun_out/pmc_mfma${1:+_$1}/bench_counter_collection.csv gpurun_out/pmc_mfma_bench${1:+_$1}.json
echo "pmc_mfma rc=$?"
