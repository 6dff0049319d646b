# Round-5 closing record at HEAD: headline line (with the CPU baseline), its kernel trace + k_step timed
# summary, the configs[1] and f16 lines.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
R=gpurun_out/r05
mkdir -p $R
timeout -k 10 400 python -u bench.py > $R/bench_final4.log 2>&1 || { tail -20 $R/bench_final4.log; exit 1; }
tail -1 $R/bench_final4.log | cut -c1-160
bash tools/prof_bench.sh
python tools/trace_kstep.py gpurun_out/prof/bench_kernel_trace.csv --warmup 1 --steps 2 --horizon 16 --out $R/kstep_trace_final4.json > /dev/null 2>&1
timeout -k 10 300 python -u bench.py --mazes 4096 --horizon 32 --no-cpu-baseline > $R/bench_config1_final4.log 2>&1 || { tail -20 $R/bench_config1_final4.log; exit 1; }
timeout -k 10 300 python -u bench.py --dtype f16 --mazes 32768 --no-cpu-baseline > $R/bench_f16_final4.log 2>&1 || { tail -20 $R/bench_f16_final4.log; exit 1; }
echo done
