# Diagnostic builds of csrc/x3mlp.hip with parts of the kernel switched off, each
# timed by tools/bench_x3nt.py (their numbers are NOT valid results: the
# outputs are wrong by construction).  Run on the GPU box from the repo root.
set -e
mkdir -p tools/_var gpurun_out
SRC=marl-maze_amd/csrc
for v in BASE NO_DMA NO_ALOAD NO_DMA_NO_ALOAD; do
  defs=""
  case $v in
    NO_EPI) defs="-DX3_NO_EPI";;
    NO_DMA) defs="-DX3_NO_DMA";;
    NO_ALOAD) defs="-DX3_NO_ALOAD";;
    NO_DMA_NO_ALOAD) defs="-DX3_NO_DMA -DX3_NO_ALOAD";;
  esac
  if true; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off $defs -I include -I $SRC \
      -o tools/_var/x3_$v.so $SRC/*.hip
  fi
done
