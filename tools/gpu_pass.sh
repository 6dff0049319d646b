# One parameterised GPU pass (replaces the per-round final_pass_r05*.sh copies).
#
#   bash tools/gpu_pass.sh TAG STEP [STEP ...]
#
# Every step writes under gpurun_out/TAG/ and runs under its own time limit; the first failing step ends the
# pass (no GPU step runs after a failure, a fault or a time limit).  Steps:
#   tests            every GPU test                       tests=EXPR  the GPU tests matching -k EXPR
#   bench            the headline line (configs[2]: 65,536 10x10 mazes, CPU baseline included)
#   config1          configs[1]: 4,096 mazes, horizon 32   config3  configs[3]'s per-GPU share: 8,192 20x20 mazes
#   f16              configs[4]'s per-GPU share: 32,768 mazes, fp16 actor/critic
#   prof             rocprofv3 kernel trace + stats of a short headline run, the k_step timed summary and the
#                    k_step rows of the trace (profiles/ keeps both)
#   prof1            the same kernel stats for configs[1]     proff16  the same for the f16 share
#   pmc              k_step HBM traffic: FETCH_SIZE and WRITE_SIZE in two separate --pmc passes
#   mfma16           MFMA busy / clock per kernel of the f16 share (one --pmc pass)
#   wgdma            the x2 trunk weight gradients, LDS-DMA staging against register staging (A/B in one process)
#   dp               two gloo ranks on the one GPU through bench.py's multi-process path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
TAG=$1
shift
R=gpurun_out/$TAG
mkdir -p "$R"
fail() { echo "STEP $1 FAILED rc=$2"; tail -30 "$3"; exit 1; }
for s in "$@"; do
  case $s in
    tests)
      timeout -k 10 1100 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu \
        > $R/pytest_gpu.log 2>&1 || fail "$s" $? $R/pytest_gpu.log
      tail -2 $R/pytest_gpu.log ;;
    tests=*)
      timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -s \
        -k "${s#tests=}" > $R/pytest_sel.log 2>&1 || fail "$s" $? $R/pytest_sel.log
      grep -E "PASSED|FAILED|^trunk3|^f16|passed|failed" $R/pytest_sel.log | tail -60 ;;
    bench)
      timeout -k 10 400 python -u bench.py > $R/bench.log 2>&1 || fail "$s" $? $R/bench.log
      tail -1 $R/bench.log > $R/bench_line.json; cut -c1-300 $R/bench_line.json ;;
    config1)
      timeout -k 10 300 python -u bench.py --mazes 4096 --horizon 32 --no-cpu-baseline > $R/bench_config1.log 2>&1 \
        || fail "$s" $? $R/bench_config1.log
      tail -1 $R/bench_config1.log > $R/bench_line_config1_4096.json; cut -c1-300 $R/bench_line_config1_4096.json ;;
    config3)
      timeout -k 10 300 python -u bench.py --mazes 8192 --size 20 --no-cpu-baseline > $R/bench_config3.log 2>&1 \
        || fail "$s" $? $R/bench_config3.log
      tail -1 $R/bench_config3.log > $R/bench_line_config3_share_8192x20.json
      cut -c1-300 $R/bench_line_config3_share_8192x20.json ;;
    f16)
      timeout -k 10 300 python -u bench.py --dtype f16 --mazes 32768 --no-cpu-baseline > $R/bench_f16.log 2>&1 \
        || fail "$s" $? $R/bench_f16.log
      tail -1 $R/bench_f16.log > $R/bench_line_f16.json; cut -c1-300 $R/bench_line_f16.json ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/prof -o bench --output-format csv -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/prof_bench.log 2>&1 || fail "$s" $? $R/prof_bench.log
      python3 tools/trace_kstep.py $R/prof/bench_kernel_trace.csv --warmup 1 --steps 2 --horizon 16 \
        --out $R/kstep_trace_summary.json --rows $R/kstep_trace_rows.csv > /dev/null || fail "$s" $? $R/prof_bench.log
      echo "prof ok" ;;
    prof1)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/prof1 -o c1 --output-format csv -- \
        python3 bench.py --mazes 4096 --horizon 32 --steps 2 --warmup 1 --no-cpu-baseline > $R/prof1.log 2>&1 \
        || fail "$s" $? $R/prof1.log
      echo "prof1 ok" ;;
    proff16)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/prof_f16 -o f16 --output-format csv -- \
        python3 bench.py --dtype f16 --mazes 32768 --steps 2 --warmup 1 --no-cpu-baseline > $R/prof_f16.log 2>&1 \
        || fail "$s" $? $R/prof_f16.log
      echo "proff16 ok" ;;
    pmc)
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/pmc_fetch -o bench --output-format csv -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/pmc_fetch.log 2>&1 || fail "$s" $? $R/pmc_fetch.log
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/pmc_write -o bench --output-format csv -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/pmc_write.log 2>&1 || fail "$s" $? $R/pmc_write.log
      python3 tools/pmc_summarize.py $R/pmc_fetch/bench_counter_collection.csv \
        $R/pmc_write/bench_counter_collection.csv $R/pmc_env_step_65536x10.json || fail "$s" $? $R/pmc_write.log
      cat $R/pmc_env_step_65536x10.json | cut -c1-400 ;;
    mfma16)
      timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        -d $R/pmc_mfma_f16 -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        --dtype f16 --mazes 32768 > $R/pmc_mfma_f16.log 2>&1 || fail "$s" $? $R/pmc_mfma_f16.log
      python3 tools/pmc_mfma_summarize.py $R/pmc_mfma_f16/bench_counter_collection.csv $R/pmc_mfma_bench_f16.json ;;
    wgdma)
      timeout -k 10 300 python -u tools/bench_wgrad_dma.py > $R/bench_wgrad_dma.jsonl 2>&1 || fail "$s" $? $R/bench_wgrad_dma.jsonl
      cat $R/bench_wgrad_dma.jsonl ;;
    dp)
      MARLMAZE_DP_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --mazes 8192 --steps 2 --warmup 1 \
        > $R/dp_rehearsal.log 2>&1 || fail "$s" $? $R/dp_rehearsal.log
      tail -1 $R/dp_rehearsal.log | cut -c1-300 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "pass $TAG done"
