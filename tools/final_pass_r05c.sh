# Round-5 last pass at the final code: every GPU test, the three bench lines, the headline's kernel trace +
# k_step timed summary, the f16 line's kernel stats, the trunk + heads against the unfused step at large M.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
R=gpurun_out/r05
mkdir -p $R gpurun_out/prof_f16
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $R/pytest_gpu_final3.log 2>&1 || { tail -30 $R/pytest_gpu_final3.log; exit 1; }
tail -2 $R/pytest_gpu_final3.log
timeout -k 10 400 python -u bench.py > $R/bench_final3.log 2>&1 || { tail -20 $R/bench_final3.log; exit 1; }
tail -1 $R/bench_final3.log | cut -c1-200
timeout -k 10 300 python -u bench.py --mazes 4096 --horizon 32 --no-cpu-baseline > $R/bench_config1_final3.log 2>&1 || { tail -20 $R/bench_config1_final3.log; exit 1; }
tail -1 $R/bench_config1_final3.log | cut -c1-200
timeout -k 10 300 python -u bench.py --dtype f16 --mazes 32768 --no-cpu-baseline > $R/bench_f16_final3.log 2>&1 || { tail -20 $R/bench_f16_final3.log; exit 1; }
tail -1 $R/bench_f16_final3.log | cut -c1-200
bash tools/prof_bench.sh
python tools/trace_kstep.py gpurun_out/prof/bench_kernel_trace.csv --warmup 1 --steps 2 --horizon 16 --out $R/kstep_trace_final3.json > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f16 -o f16 --output-format csv -- python3 bench.py --dtype f16 --mazes 32768 --steps 2 --warmup 1 --no-cpu-baseline > $R/prof_f16.log 2>&1
echo "prof f16 rc=$?"
timeout -k 10 120 python -u tools/bench_trunk.py 8192 65536 131072 --heads > $R/bench_trunk_heads.log 2>&1 && cat $R/bench_trunk_heads.log
echo done
