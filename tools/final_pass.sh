#!/bin/bash
# Round-end measurement pass (one gpurun call): GPU tests, the bench lines of every BASELINE config this build
# reports, and rocprofv3 kernel statistics / MFMA counters of the fp32-class and fp16 benches.
#   bash tools/final_pass.sh TAG
T=${1:-final}
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "${T}_tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "${T}_bench:400:python bench.py" \
  "${T}_c1:200:python bench.py --mazes 4096 --horizon 32 --no-cpu-baseline" \
  "${T}_f16:200:python bench.py --dtype f16 --no-cpu-baseline" \
  "${T}_c3:200:python bench.py --size 20 --mazes 8192 --horizon 32 --no-cpu-baseline" \
  "${T}_prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "${T}_proff16:300:rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_proff16 -o bench --output-format csv -- python3 bench.py --dtype f16 --steps 5 --warmup 2 --no-cpu-baseline" \
  "${T}_pmcf16:300:rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${T}_pmcf16 -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --dtype f16"
