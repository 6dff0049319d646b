# rocprofv3 kernel trace + stats of a short bench run (no cpu baseline)
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"
