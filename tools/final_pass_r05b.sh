# Round-5 final pass at the fused-trunk code: GPU tests, headline / configs[1] / fp16 configs[4]-share bench
# lines, the headline's kernel trace + k_step timed summary, the configs[1] kernel stats.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
R=gpurun_out/r05
mkdir -p $R gpurun_out/prof_c1
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $R/pytest_gpu_final2.log 2>&1 || { tail -30 $R/pytest_gpu_final2.log; exit 1; }
tail -2 $R/pytest_gpu_final2.log
timeout -k 10 400 python -u bench.py > $R/bench_final2.log 2>&1 || { tail -20 $R/bench_final2.log; exit 1; }
tail -1 $R/bench_final2.log | cut -c1-200
timeout -k 10 300 python -u bench.py --mazes 4096 --horizon 32 --no-cpu-baseline > $R/bench_config1_final2.log 2>&1 || { tail -20 $R/bench_config1_final2.log; exit 1; }
tail -1 $R/bench_config1_final2.log | cut -c1-200
timeout -k 10 300 python -u bench.py --dtype f16 --mazes 32768 --no-cpu-baseline > $R/bench_f16_final2.log 2>&1 || { tail -20 $R/bench_f16_final2.log; exit 1; }
tail -1 $R/bench_f16_final2.log | cut -c1-200
bash tools/prof_bench.sh
python tools/trace_kstep.py gpurun_out/prof/bench_kernel_trace.csv --warmup 1 --steps 2 --horizon 16 --out $R/kstep_trace_final2.json > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o c1 --output-format csv -- python3 bench.py --mazes 4096 --horizon 32 --steps 3 --warmup 1 --no-cpu-baseline > $R/prof_c1.log 2>&1
echo "prof c1 rc=$?"
echo done
