# HBM traffic of one GEMM launch shape (tools/gemm_one.py): FETCH_SIZE and WRITE_SIZE in two separate --pmc
# passes, summarised per launch against the algorithmic bytes (A read once + C written once + the bit mask).
#   PREC=x2 FORM=fwd SHAPE=264x264 bash tools/pmc_gemm_traffic.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-gemm}
SHAPE=${SHAPE:-264x264}; M=${M:-419430}
N=${SHAPE%x*}; K=${SHAPE#*x}
if [ "${FORM:-fwd}" = wgrad ]; then  # dY and X read once (the partials' bytes are small)
  ALG=$(python3 -c "M=$M; N=$N; K=$K; print(4 * M * K + 4 * M * N)")
else
  ALG=$(python3 -c "M=$M; N=$N; K=$K; print(4 * M * K + 4 * M * N + (M + 255) // 256 * 256 // 16 * 64 * 12)")
fi
for C in FETCH_SIZE WRITE_SIZE; do
  ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/pmc_${TAG}_$C -o g --output-format csv -- python3 tools/gemm_one.py > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "pass $C failed"; exit 1; }
done
python3 tools/pmc_traffic_summarize.py "${KERN:-k_bres}" gpurun_out/pmc_${TAG}_FETCH_SIZE/g_counter_collection.csv gpurun_out/pmc_${TAG}_WRITE_SIZE/g_counter_collection.csv gpurun_out/pmc_${TAG}.json "$ALG" "PREC=${PREC:-x3} FORM=${FORM:-fwd} SHAPE=$SHAPE M=$M"
