# Re-tune the GEMMs of the bench workload (TunableOp) on an MI355X; the results
# land in gpurun_out/tunableop0.csv -> copy to marl-maze_amd/marlmaze/tuned/gemm_gfx950.csv
cd /root/repo && mkdir -p gpurun_out
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop.csv \
  timeout -k 10 900 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-tuned-gemms > gpurun_out/tune_gemms.log 2>&1
echo "tune rc=$?"
