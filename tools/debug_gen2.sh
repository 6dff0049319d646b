set -x
timeout -k 10 60 ./tools/debug_obs
timeout -k 10 120 python tools/debug_gen.py 2>&1 | grep "obs diff"
cp marl-maze_amd/libmarlmaze.so /tmp/keep.so && cp marl-maze_amd/libmarlmaze_O1.so marl-maze_amd/libmarlmaze.so && timeout -k 10 120 python tools/debug_gen.py 2>&1 | grep "obs diff"; cp /tmp/keep.so marl-maze_amd/libmarlmaze.so
