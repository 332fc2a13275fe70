#!/bin/bash
# Build diagnostic variants of libhrl.so with conv3x3_block_bwd2_kernel's phases removed (BB2_VARIANT bits,
# csrc/hrl_conv.hip): tools/micro/libhrl_bb2_v<N>.so.  Run on the GPU box:
#   for v in 1 2 4 6; do HRL_LIB_PATH=tools/micro/libhrl_bb2_v$v.so python tools/block_bench.py; done
set -e
cd "$(dirname "$0")/.."
python -c "from handyrl_amd import build; build.build(verbose=False)"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I include"
OBJS=$(ls build/obj/*.o | grep -v hrl_conv)
for v in "$@"; do
  hipcc $FLAGS -DBB2_VARIANT=$v -c handyrl_amd/csrc/hrl_conv.hip -o /tmp/bb2_conv_v$v.o &
done
wait
for v in "$@"; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o tools/micro/libhrl_bb2_v$v.so $OBJS /tmp/bb2_conv_v$v.o
done
ls -la tools/micro/libhrl_bb2_v*.so
