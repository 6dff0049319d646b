# Diagnostic builds of k_bres (csrc/x3mlp.hip), timings only (outputs of ROW0 / NOSPLIT wrong):
#   ROW0: every unit reads the same 32 A rows (L2-resident: no HBM latency on the A loads);
#   NOSPLIT: no A split (raw bits as fragments: the split's VALU removed);
#   NOSLP: the normal kernel built with -fno-slp-vectorize (no packed f32 VALU beside the MFMAs).
#   MARLMAZE_LIB=tools/_var/bres_NOSPLIT.so python tools/bench_gemm_ab.py
set -e
mkdir -p tools/_var
SRC=marl-maze_amd/csrc
for v in ROW0 NOSPLIT NOSLP; do
  case $v in
    ROW0) defs="-DBRES_ROW0";;
    NOSPLIT) defs="-DBRES_NO_SPLIT";;
    NOSLP) defs="-fno-slp-vectorize";;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off $defs -I include -I $SRC \
    -o tools/_var/bres_$v.so $SRC/*.hip &
done
wait
