# rocprofv3 of the env-step microbench (65,536 10x10 mazes): kernel trace +
# stats, then HBM traffic counters in separate passes (FETCH_SIZE, WRITE_SIZE).
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_env -o env --output-format csv -- python3 tools/bench_env.py --steps 200 --warmup 50 > gpurun_out/prof_env.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o env --output-format csv -- python3 tools/bench_env.py --steps 20 --warmup 5 > gpurun_out/pmc_fetch.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o env --output-format csv -- python3 tools/bench_env.py --steps 20 --warmup 5 > gpurun_out/pmc_write.log 2>&1
echo "prof_env rc=$?"
