# Build the X3_STAMPS diagnostic library (phase clocks of k_x3nt; outputs unchanged,
# one extra store per phase) for tools/x3_stamps.py.  Build here (CPU); on the GPU box:
#   MARLMAZE_LIB=tools/_var/x3_STAMPS.so python tools/x3_stamps.py
set -e
mkdir -p tools/_var
SRC=marl-maze_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -DX3_STAMPS -I include -I $SRC \
  -o tools/_var/x3_STAMPS.so $SRC/*.hip
