#!/bin/bash
# Build diagnostic variants of libhrl.so with conv3x3_fwd_ls_kernel's stores reduced or its LDS writes re-addressed (FW5_VARIANT bits,
# csrc/hrl_conv.hip) into tools/variants/libhrl_fw5_v<N>.so (not gpurun-ignored, so they travel; delete them after
# the run).  On the GPU box:
#   for v in 1 2 4; do HRL_LIB_PATH=tools/variants/libhrl_fw5_v$v.so python tools/fwd_bench.py --forms 3; done
set -e
cd "$(dirname "$0")/.."
python -c "from handyrl_amd import build; build.build(verbose=False)"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I include"
OBJS=$(ls build/obj/*.o | grep -v hrl_conv)
mkdir -p tools/variants
for v in "$@"; do
  hipcc $FLAGS -DFW5_VARIANT=$v -c handyrl_amd/csrc/hrl_conv.hip -o /tmp/fw5_conv_v$v.o &
done
wait
for v in "$@"; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/libhrl_fw5_v$v.so $OBJS /tmp/fw5_conv_v$v.o
done
ls -la tools/variants/
