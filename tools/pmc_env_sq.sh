# SQ instruction / cycle counters of the env-step microbench (one pass).
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_sq -o env --output-format csv -- python3 tools/bench_env.py --steps 20 --warmup 5 > gpurun_out/pmc_sq.log 2>&1
echo "pmc_sq rc=$?"
