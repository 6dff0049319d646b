# Builds libmarlmaze variants that differ only in actor_front.hip's build knobs (FRONT_P3_UNROLL,
# FRONT_EF_UNROLL, FRONT_EF_ROWS) into tools/_var/, for A/B timing with MARLMAZE_LIB=... python
# tools/bench_front.py.
# usage: tools/front_variants.sh "P3 EF ROWS" ...   e.g. tools/front_variants.sh "4 2 4" "4 2 2"
set -e
cd "$(dirname "$0")/.." && mkdir -p tools/_var
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I include -I marl-maze_amd/csrc"
for s in env_kernels rl_kernels x3mlp; do
  [ tools/_var/$s.o -nt marl-maze_amd/csrc/$s.hip ] || /opt/rocm/bin/hipcc $F -c marl-maze_amd/csrc/$s.hip -o tools/_var/$s.o
done
for v in "$@"; do
  set -- $v
  /opt/rocm/bin/hipcc $F -DFRONT_P3_UNROLL=$1 -DFRONT_EF_UNROLL=$2 -DFRONT_EF_ROWS=$3 -c marl-maze_amd/csrc/actor_front.hip -o tools/_var/af_$1_$2_$3.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_var/lib_$1_$2_$3.so tools/_var/af_$1_$2_$3.o tools/_var/env_kernels.o tools/_var/rl_kernels.o tools/_var/x3mlp.o
  echo tools/_var/lib_$1_$2_$3.so
done
