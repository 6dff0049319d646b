# Diagnostic builds of the weight-gradient kernel (csrc/x3mlp.hip k_wgrad) with
# parts switched off, timed by tools/bench_wgrad.py through MARLMAZE_LIB (their
# outputs are wrong by construction; only the times mean something).  Build
# here (CPU), run the timing on the GPU box:
#   for v in BASE NO_MFMA NO_GLOAD; do MARLMAZE_LIB=tools/_var/wg_$v.so python tools/bench_wgrad.py; done
set -e
mkdir -p tools/_var
SRC=marl-maze_amd/csrc
for v in BASE NO_MFMA NO_GLOAD NO_BOTH GENERIC CONV_LATE; do
  defs=""
  case $v in
    NO_MFMA) defs="-DWG_NO_MFMA";;
    NO_GLOAD) defs="-DWG_NO_GLOAD";;
    NO_BOTH) defs="-DWG_NO_MFMA -DWG_NO_GLOAD";;
    GENERIC) defs="-DWG_GENERIC";;
    CONV_LATE) defs="-DWG_CONV_LATE";;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off $defs -I include -I $SRC \
    -o tools/_var/wg_$v.so $SRC/*.hip &
done
wait
