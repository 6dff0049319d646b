# Diagnostic / tuning builds of k_bres (csrc/x3mlp.hip), for tools/bench_gemm_ab.py through MARLMAZE_LIB:
#   ROW0: every unit reads the same 32 A rows (L2-resident: no HBM latency on the A loads; outputs wrong);
#   NOSPLIT: no A split (raw bits as fragments; outputs wrong);
#   NOBREAD: no B fragment LDS reads (A registers reused as B; outputs wrong);
# (tools/ab_build.py NAME -D... builds any combination; tools/ab_libs.py times builds in one process)
#   W<n>_P<b>: <n> waves per workgroup, B fragments of the next column read ahead (b = 1) or not.
set -e
mkdir -p tools/_var
SRC=marl-maze_amd/csrc
for v in ${VARIANTS:-ROW0 NOSPLIT W16_P1 W12_P1 W8_P1 W12_P0}; do
  case $v in
    ROW0) defs="-DBRES_ROW0";;
    NOSPLIT) defs="-DBRES_NO_SPLIT";;
    W*_P*) w=${v#W}; w=${w%_P*}; b=${v#*_P}; defs="-DBRES_WAVES=$w -DBRES_BPREF=$b";;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off $defs -I include -I $SRC \
    -o tools/_var/bres_$v.so $SRC/*.hip &
done
wait
