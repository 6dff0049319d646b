# HBM traffic of the bench's env-step kernel: FETCH_SIZE and WRITE_SIZE in two
# separate --pmc passes over the same bench command (MI355X_MICROARCH.md: the
# two TCC counters do not fit one pass), then the per-launch summary JSON.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_bench_fetch -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_bench_fetch.log 2>&1 \
 && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_bench_write -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_bench_write.log 2>&1 \
 && python3 tools/pmc_summarize.py gpurun_out/pmc_bench_fetch/bench_counter_collection.csv gpurun_out/pmc_bench_write/bench_counter_collection.csv gpurun_out/pmc_env_step_65536x10.json
echo "pmc_bench rc=$?"
