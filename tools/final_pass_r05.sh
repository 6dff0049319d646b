set -o pipefail
cd /root/repo && export TMPDIR=/tmp
mkdir -p gpurun_out/r05
R=gpurun_out/r05
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $R/pytest_gpu_final1.log 2>&1 || { tail -30 $R/pytest_gpu_final1.log; exit 1; }
tail -2 $R/pytest_gpu_final1.log
timeout -k 10 400 python -u bench.py > $R/bench_final1.log 2>&1 || { tail -20 $R/bench_final1.log; exit 1; }
tail -1 $R/bench_final1.log | cut -c1-300
timeout -k 10 300 python -u bench.py --mazes 4096 --horizon 32 --no-cpu-baseline > $R/bench_config1.log 2>&1 || { tail -20 $R/bench_config1.log; exit 1; }
tail -1 $R/bench_config1.log | cut -c1-200
bash tools/prof_bench.sh
python tools/trace_kstep.py gpurun_out/prof/bench_kernel_trace.csv --warmup 1 --steps 2 --horizon 16 --out $R/kstep_trace_final1.json > /dev/null 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma_f16 -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dtype f16 --mazes 32768 > $R/pmc_mfma_f16.log 2>&1 && python3 tools/pmc_mfma_summarize.py gpurun_out/pmc_mfma_f16/bench_counter_collection.csv $R/pmc_mfma_bench_f16.json
echo done
